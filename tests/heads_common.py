"""Shared fixture for the feature-level head tests (tests/golden/heads.npz)."""
import numpy as np
import torch

from clipmi import synth

LN100 = float(np.log(100.0))


def fixture():
    """The same tables tools/gen_goldens.py heads_fixture() fed the reference."""
    E, n_desc, n_img = 512, 5, 24
    desc = synth.normal((7 * n_desc, E), 7, "heads_desc")
    img = synth.normal((n_img, E), 8, "heads_img")
    labels = np.random.default_rng(9).integers(0, 7, n_img).astype(np.int64)
    return desc, img, labels


def weights(g, which, nm):
    return [torch.from_numpy(g[f"{which}/{nm}/{k}"]) for k in ("fc1.weight", "fc1.bias", "fc2.weight", "fc2.bias")]

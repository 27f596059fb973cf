"""CPU oracle for the resize of the input step: CLIPImageProcessor's shortest-edge resize.

TEST INFRASTRUCTURE ONLY (same rule as oracle/clip_ref.py: only tests/ may import it, as the
checker; the product path is vlm-clip_amd/csrc/data.hip clipmi_resize_u8).

The reference gets pixel_values from CLIPProcessor.from_pretrained(...) (model_m.py:30,
dataset.py:152-164); without torchvision, transformers 5.15 runs CLIPImageProcessorPil, whose
resize is PIL's Image.resize((w, h), BICUBIC) (transformers image_transforms.resize) to the
shortest edge = image size (get_resize_output_image_size: new_long = int(size * long / short)).
PIL (Pillow 12.2, third-party, not under /root/reference) restated from its published algorithm
(libImaging/Resample.c):
  * per output coordinate x: scale = in / out, filterscale = max(scale, 1), support = 2 *
    filterscale (bicubic, a = -0.5), center = (x + 0.5) * scale, taps j in [xmin, xmax) with
    xmin = max(int(center - support + 0.5), 0), xmax = min(int(center + support + 0.5), in),
    w_j = bicubic((j - center + 0.5) / filterscale), normalised to sum 1 (fp64), then fixed point
    k_j = int(w_j * 2^22 +- 0.5) (PRECISION_BITS = 22, rounded away from zero);
  * horizontal pass first into an 8-bit image, then the vertical pass: out = clip8((2^21 +
    sum_j k_j * in_j) >> 22), clipped to [0, 255].
Pinned against PIL itself (tests/test_oracle_golden.py::test_resize_oracle_matches_pil) and the
processor goldens (tests/golden/image_processor_resize.npz, tools/gen_goldens.py).
"""
from __future__ import annotations

import numpy as np

PRECISION_BITS = 22


def bicubic(x):
    a = -0.5
    x = abs(x)
    if x < 1.0:
        return ((a + 2.0) * x - (a + 3.0)) * x * x + 1.0
    if x < 2.0:
        return (((x - 5.0) * x + 8.0) * x - 4.0) * a
    return 0.0


def coeffs(in_size, out_size):
    """-> (xmin [out], xmax [out] (tap counts), k [out, ksize] int64 fixed point)."""
    scale = in_size / out_size
    filterscale = max(scale, 1.0)
    support = 2.0 * filterscale
    ksize = int(np.ceil(support)) * 2 + 1
    xmins = np.zeros(out_size, np.int64)
    xcnt = np.zeros(out_size, np.int64)
    kk = np.zeros((out_size, ksize), np.int64)
    ss = 1.0 / filterscale
    for xx in range(out_size):
        center = (xx + 0.5) * scale
        xmin = int(center - support + 0.5)
        if xmin < 0:
            xmin = 0
        xmax = int(center + support + 0.5)
        if xmax > in_size:
            xmax = in_size
        xmax -= xmin
        w = [bicubic((x + xmin - center + 0.5) * ss) for x in range(xmax)]
        ww = sum(w)
        for x in range(xmax):
            v = w[x] / ww if ww != 0.0 else w[x]
            kk[xx, x] = int(-0.5 + v * (1 << PRECISION_BITS)) if v < 0 else int(0.5 + v * (1 << PRECISION_BITS))
        xmins[xx], xcnt[xx] = xmin, xmax
    return xmins, xcnt, kk


def _pass(img, axis, out_size):
    """One 8-bit pass along axis (1 = width, 0 = height) of img [H, W, C] uint8."""
    xmin, xcnt, kk = coeffs(img.shape[axis], out_size)
    src = np.moveaxis(img.astype(np.int64), axis, 0)  # [in, other, C]
    out = np.empty((out_size,) + src.shape[1:], np.int64)
    for xx in range(out_size):
        n = xcnt[xx]
        acc = np.full(src.shape[1:], 1 << (PRECISION_BITS - 1), np.int64)
        acc += np.tensordot(kk[xx, :n], src[xmin[xx]:xmin[xx] + n], axes=(0, 0))
        out[xx] = acc
    out = np.clip(out >> PRECISION_BITS, 0, 255).astype(np.uint8)
    return np.moveaxis(out, 0, axis)


def resize_bicubic(img, out_h, out_w):
    """PIL Image.resize((out_w, out_h), BICUBIC) of an RGB uint8 image [H, W, 3]: horizontal then
    vertical pass (a pass whose size does not change is skipped, as PIL does)."""
    x = img
    if out_w != img.shape[1]:
        x = _pass(x, 1, out_w)
    if out_h != img.shape[0]:
        x = _pass(x, 0, out_h)
    return x


def shortest_edge_size(h, w, size):
    """transformers get_resize_output_image_size(default_to_square=False): short edge -> size,
    long edge -> int(size * long / short)."""
    if w <= h:
        return int(size * h / w), size
    return size, int(size * w / h)

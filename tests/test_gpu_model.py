"""End-to-end parity of clipmi.CLIPWithAdapters / CLIPAdapterTrainer on the GPU against
goldens produced by running the reference (tests/golden, tools/gen_goldens.py) and the
CPU oracle.  Tolerances: fp32 parity mode -> logits within 1e-3 absolute (north_star);
bf16 MFMA mode -> logits within 0.07 absolute at logit scale 100 (bf16 GEMM operands over
12-24 layers, fp32 residual stream; SURVEY §6 measured 0.058-0.146 for bf16 variants of the reference itself)."""
import hashlib

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from clipmi import CLIPWithAdapters, CLIPAdapterTrainer, synth  # noqa: E402
from clipmi import config as C  # noqa: E402

# bf16x3: fp32 activations, tower GEMMs as bf16x3 split products -- held to the fp32 tolerances
# bf16 (fp32 residual stream, trained and frozen towers since round 6): measured 0.019-0.033 on the full-size
# fixtures (B/32, B/16, L/14, L/14@336; round 5 with the bf16 stream on frozen towers 0.042-0.12), bound ~2x that
LOGIT_TOL = {"fp32": 1e-3, "bf16x3": 1e-3, "bf16": 0.07}
# the tiny 2-layer fixture has 64-dim features: bf16 rounding of LN'd activations is ~1 %
# per element there, so its bf16 logits get a looser bound than the full-size models (measured 0.122)
BF16_TINY_LOGIT_TOL = 0.25


def batch(cfg, B, g=None, seed=1234):
    b = synth.synthetic_batch(cfg, B, seed=seed)
    if g is not None:
        h = hashlib.sha256()
        for k in ("pixel_values", "input_ids", "attention_mask"):
            h.update(np.ascontiguousarray(b[k]).tobytes())
        assert h.hexdigest()[:16] == str(g["input_digest"])
    return {k: torch.from_numpy(v).cuda() for k, v in b.items()}


def make(preset, adapters, precision, freeze=True):
    return CLIPWithAdapters(preset, use_text_adapter=adapters, use_vision_adapter=adapters, use_shared_adapters=False,
                            freeze_clip=freeze, device="cuda", precision=precision)


@pytest.mark.parametrize("precision", ["fp32", "bf16x3", "bf16"])
@pytest.mark.parametrize("tag,preset,B,adapters", [("tiny", "tiny", 4, True), ("b32", "B/32", 8, True),
                                                   ("b32_noadapter", "B/32", 8, False),
                                                   ("b16", "B/16", 4, False),
                                                   # config 4's model: P=14 (patch K 588 -> 640), N=257
                                                   ("l14", "L/14", 2, True),
                                                   # config 5's model at 336 px: N = 577 (streamed attention)
                                                   ("l14_336", "L/14@336", 2, True)])
def test_forward_matches_reference(golden, precision, tag, preset, B, adapters):
    g = golden(f"forward_{tag}.npz")
    m = make(preset, adapters, precision)
    with torch.no_grad():
        out = m(**batch(m.config, B, g))
    torch.cuda.synchronize()
    lt = out["logits_per_text"].cpu().numpy()
    err = np.abs(lt - g["logits_per_text"]).max()
    print(f"\n[{tag} {precision}] max|dlogit|={err:.4g}")
    tol = BF16_TINY_LOGIT_TOL if (precision == "bf16" and preset == "tiny") else LOGIT_TOL[precision]
    assert err < tol, err
    assert np.abs(out["loss"].item() - g["loss"]) < tol
    assert np.allclose(out["logits_per_image"].cpu().numpy(), lt.T)
    fe = 1e-4 if precision != "bf16" else 3e-2
    assert np.abs(out["text_features"].cpu().numpy() - g["text_features"]).max() < fe
    assert np.abs(out["image_features"].cpu().numpy() - g["image_features"]).max() < fe


@pytest.mark.parametrize("tag,preset,B,adapters", [("b32", "B/32", 8, True), ("l14", "L/14", 2, True)])
def test_frozen_towers_fp32_residual_forward(golden, tag, preset, B, adapters):
    """residual_fp32=True given explicitly on frozen towers (the default since round 6; round 5 kept the bf16 stream
    there): the bf16 mode with the fp32 residual stream against the reference goldens."""
    g = golden(f"forward_{tag}.npz")
    m = CLIPWithAdapters(preset, use_text_adapter=adapters, use_vision_adapter=adapters, use_shared_adapters=False,
                         freeze_clip=True, device="cuda", precision="bf16", residual_fp32=True)
    assert m._rt.resid32
    with torch.no_grad():
        out = m(**batch(m.config, B, g))
    torch.cuda.synchronize()
    err = np.abs(out["logits_per_text"].cpu().numpy() - g["logits_per_text"]).max()
    print(f"\n[{tag} bf16 fp32-residual] max|dlogit|={err:.4g}")
    assert err < 0.10, err


def test_eos_pooling_fp32(golden):
    g = golden("forward_b32_noadapter.npz")
    m = CLIPWithAdapters("B/32", use_text_adapter=False, use_vision_adapter=False, use_shared_adapters=False,
                         device="cuda", precision="fp32", pooling="eos")
    b = batch(m.config, 8, g)
    with torch.no_grad():
        tf = m.get_text_features(b["input_ids"], b["attention_mask"])
    assert np.abs(tf.cpu().numpy() - g["text_eos_projected"]).max() < 2e-4


@pytest.mark.parametrize("precision", ["fp32", "bf16x3", "bf16"])
@pytest.mark.parametrize("tag,preset,B,adapters,freeze", [("tiny_adapter_grads", "tiny", 4, True, True),
                                                          ("tiny_full_grads", "tiny", 4, False, False),
                                                          ("l14", "L/14", 2, True, True)])
def test_gradients_match_reference(golden, precision, tag, preset, B, adapters, freeze):
    if preset != "tiny" and precision == "bf16":
        # B=2 with near-saturated softmax: d loss/d logit = p - y is a small difference of
        # O(1) terms, so bf16's ~0.12 logit error (checked by test_forward_matches_reference)
        # moves it by tens of percent whatever the kernels do; the bf16 backward arithmetic
        # is pinned by the tiny cases, the L/14 shapes by the fp32 case
        pytest.skip("ill-conditioned at B=2 in bf16; see comment")
    g = golden(f"forward_{tag}.npz")
    m = make(preset, adapters, precision, freeze=freeze)
    out = m(**batch(m.config, B, g))
    out["loss"].backward()
    torch.cuda.synchronize()
    # bf16x3: each product carries ~2^-16 relative error (the bf16 hi/lo split keeps 16 of fp32's 24
    # significant bits) -- measured 1.0e-5 on this loss of 2.09, at the fp32 bound; the logits (north_star's
    # 1e-3) and the gradients below are held to the fp32 tolerances
    ltol = {"fp32": 1e-5, "bf16x3": 3e-5}.get(precision, 2e-2)
    assert abs(out["loss"].item() - float(g["loss"])) < ltol
    params = dict(m.named_parameters())
    names = [k[5:] for k in g.files if k.startswith("grad/")]
    assert names
    # Some true gradients are identically zero (k_proj biases: softmax shift invariance; text
    # q/k under first-token pooling, quirk Q1: token 0 attends only to itself), so errors are
    # measured against max(|ref| of the tensor, 5 % of the largest gradient of its group).
    gmax = max(float(np.abs(g["grad/" + n]).max()) for n in names)
    worst = (0.0, "")
    for n in names:
        p = params[n]
        assert p.grad is not None, n
        ref = g["grad/" + n]
        scale = max(float(np.abs(ref).max()), 0.05 * gmax, 1e-6)
        e = float(np.abs(p.grad.cpu().numpy() - ref).max()) / scale
        worst = max(worst, (e, n))
    print(f"\n[{tag} {precision}] worst grad err {worst[0]:.3e} at {worst[1]}")
    # bf16 mode stores activation gradients in bf16 (pooled-row gradient cast, LN backward
    # cancellation): measured worst 0.14 on the adapter biases
    # L/14 (24 layers, fp32): the features carry ~1e-5 relative summation-order error, which
    # the logit scale (100) turns into ~4e-4 on the adapter gradients: bound 1e-3 there
    assert worst[0] < ((2e-4 if preset == "tiny" else 1e-3) if precision != "bf16" else 0.2), worst


def test_trainer_three_steps_match_reference(golden, tmp_path):
    """trainer.py:16-124 on the tiny model: 3 AdamW steps (lr 1e-3, warmup 1) vs the reference run."""
    g = golden("trainer_tiny.npz")
    m = make("tiny", True, "fp32")
    b_np = synth.synthetic_batch(m.config, 12, seed=99)
    loader = [{k: torch.from_numpy(v[i:i + 4]) for k, v in b_np.items()} for i in range(0, 12, 4)]
    tr = CLIPAdapterTrainer(m, loader, learning_rate=1e-3, weight_decay=0.01, warmup_steps=1, max_grad_norm=1.0,
                            output_dir=str(tmp_path))
    tr.train(num_epochs=1, save_every=1)
    params = dict(m.named_parameters())
    for k in g.files:
        if k.startswith("param/"):
            n = k[6:]
            np.testing.assert_allclose(params[n].detach().cpu().numpy(), g[k], atol=2e-5, rtol=1e-4, err_msg=n)
    # the checkpoint written by train() reloads through the reference's format
    m.load_adapter_weights(str(tmp_path / "final_adapter.pt"))


def test_training_reduces_loss_bf16():
    # EOS pooling: with the reference's first-token pooling every caption has the same
    # feature (quirk Q1) and the loss is floored at ln(B)
    m = CLIPWithAdapters("tiny", use_text_adapter=False, use_vision_adapter=False, use_shared_adapters=False,
                         freeze_clip=False, device="cuda", precision="bf16", pooling="eos")
    b = batch(m.config, 16)
    tr = CLIPAdapterTrainer(m, [b], learning_rate=1e-3, output_dir="/tmp/clipmi_ck", trainable="requires_grad")
    losses = [tr.train_step(b, i, 20).item() for i in range(20)]
    assert losses[-1] < losses[0] * 0.8, losses


@pytest.mark.parametrize("precision", ["fp32", "bf16x3", "bf16"])
def test_uint8_images_match_processor_path(precision):
    """uint8 channels-last images through the GPU input step (shortest-edge resize, center crop,
    rescale, normalize) give the logits of the reference's path (CLIPImageProcessor
    pixel_values; oracle resize_ref + image_processor, pinned by tests/golden/image_processor*.npz)
    on the same model and captions."""
    from oracle import clip_ref as R
    from oracle import resize_ref as RR
    from clipmi import towers as T
    m = make("tiny", False, precision, freeze=True)
    cfg = m.config
    rng = np.random.default_rng(5)
    imgs = rng.integers(0, 256, (2, 72, 80, 3), dtype=np.uint8)
    S = cfg.vision_config.image_size
    oh, ow = RR.shortest_edge_size(72, 80, S)
    pv = R.image_processor(np.stack([RR.resize_bicubic(im, oh, ow) for im in imgs]), S, T.IMAGE_MEAN, T.IMAGE_STD)
    b = batch(cfg, 2)
    with torch.no_grad():
        a = m(input_ids=b["input_ids"], attention_mask=b["attention_mask"], pixel_values=torch.from_numpy(pv).cuda())
        u = m(input_ids=b["input_ids"], attention_mask=b["attention_mask"], pixel_values=torch.from_numpy(imgs).cuda())
    torch.cuda.synchronize()
    # bf16x3: the two input paths' last-bit pixel differences move operands across bf16 hi/lo rounding
    # boundaries (~2^-16 relative per product): measured 1.3e-5 on logits of ~1.8
    tol = {"fp32": 1e-5, "bf16x3": 5e-5}.get(precision, 2e-2)
    assert (a["logits_per_text"] - u["logits_per_text"]).abs().max().item() < tol


@pytest.mark.parametrize("precision", ["fp32", "bf16x3", "bf16"])
def test_shared_adapters_match_reference(golden, precision):
    """SharedMHSAttentionAdapter x2 (adapter/clip_adapter.py:69-128, model_m.py:95-100) with the
    batch broadcast: features and gradients vs the reference run caption by caption (it only
    runs at batch 1, quirk Q3), eval mode."""
    g = golden("shared_adapters.npz")
    m = CLIPWithAdapters("B/32", use_shared_adapters=True, freeze_clip=True, device="cuda", precision=precision)
    m.eval()  # the reference ran in eval mode (no dropout)
    b = batch(m.config, 4, g)
    tf = m.get_text_features(b["input_ids"], b["attention_mask"])
    ref = g["text_features_raw"]
    err = float(np.abs(tf.detach().cpu().numpy() - ref).max() / np.abs(ref).max())
    G = torch.from_numpy(synth.normal((4, m.config.projection_dim), 11, "shared_G")).cuda()
    (tf * G).sum().backward()
    torch.cuda.synchronize()
    params = dict(m.named_parameters())
    worst = (0.0, "")
    for k in g.files:
        if not k.startswith("grad/"):
            continue
        n = k[5:]
        r = g[k]
        got = params[n].grad
        assert got is not None, n
        got = got.cpu().numpy()
        got = got if got.ndim == 1 else got[:8]
        worst = max(worst, (float(np.abs(got - r).max() / max(np.abs(r).max(), 1e-8)), n))
    print(f"\n[shared {precision}] features rel err {err:.3e}; worst grad rel err {worst[0]:.3e} at {worst[1]}")
    assert err < (1e-4 if precision != "bf16" else 5e-2)
    assert worst[0] < (1e-3 if precision != "bf16" else 0.2), worst
    sd_path = "/tmp/clipmi_shared_ckpt.pt"
    m.save_adapter_weights(sd_path)
    sd = torch.load(sd_path, weights_only=True)
    assert "shared_adapters" in sd and "0.cross_attn.in_proj_weight" in sd["shared_adapters"]
    m.load_adapter_weights(sd_path)


def _sampled(g):
    out = {}
    for k in g.files:
        if k.startswith("grad/"):
            out[k[5:]] = ("full", g[k], None)
        elif k.startswith("grad_head/"):
            out[k[10:]] = ("head", g[k], None)
        elif k.startswith("grad_rows/"):
            out[k[10:]] = ("rows", g[k], g["grad_rows_idx/" + k[10:]])
    return out


def _take(kind, t, idx):
    t = t.detach().float().cpu()
    if kind == "full":
        return t.numpy()
    if kind == "head":
        return t.reshape(t.shape[0], -1)[:8].numpy()
    return t[torch.as_tensor(idx)].numpy()


def test_b16_full_finetune_gradients_fp32(golden):
    """BASELINE config 3's workload (ViT-B/16 full fine-tune, adapters off, logit_scale trainable)
    at B=2 in the fp32 parity mode: every parameter's gradient (sampled rows) vs the reference's
    loss backward, relative to the tensor's scale (floored at 5 % of the largest gradient:
    k-projection biases and text q/k are exactly zero in the reference, quirk Q1), within a bound derived
    from the fixture's measured conditioning (below).  Measured 7.9e-4 (r03) on the vision embeddings and
    logit_scale, 1.30e-3 with attention.hip built without SLP packing (r05), against a fixed 1e-3 bound that
    flagged rounding-order changes rather than kernel errors.  That is this fixture's conditioning, not
    a kernel error (numbers: test_oracle_golden.test_b16_contrastive_b2_is_ill_conditioned): the two
    text rows are identical (Q1), the logits [[5.20, 5.24]] x 2, and a 1e-6 relative perturbation of
    the reference's own features moves the image-feature gradient by ~5e-4 of its scale in fp64
    (1.6e-3 at 3e-6); the GPU's fp32 features differ from the CPU's by that order (summation order
    over 12 layers), the oracle's (same torch ops as the reference) do not, hence its 8e-5.  The
    backward itself is pinned at 1.8e-5 on the well-conditioned fixture
    (test_b16_feature_gradients_fp32, bound 2e-4)."""
    g = golden("forward_b16_full_grads.npz")
    m = make("B/16", False, "fp32", freeze=False)
    out = m(**batch(m.config, 2, g))
    out["loss"].backward()
    torch.cuda.synchronize()
    assert abs(out["loss"].item() - float(g["loss"])) < 1e-5
    params = dict(m.named_parameters())
    s = _sampled(g)
    assert len(s) == sum(1 for p in params.values() if p.requires_grad) - 2  # post_layernorm unused (Q2)
    gmax = max(float(np.abs(r).max()) for _, r, _ in s.values())
    errs = []
    for n, (kind, ref, idx) in s.items():
        got = _take(kind, params["clip." + n].grad, idx)
        scale = max(float(np.abs(ref).max()), 0.05 * gmax, 1e-8)
        errs.append((float(np.abs(got - ref).max()) / scale, n))
    errs.sort(reverse=True)
    worst = errs[0]
    # The bound is derived from this fixture's conditioning, measured on this run against exact arithmetic (the
    # oracle, oracle/clip_ref.py, pinned to the reference, run in fp64 on the same weights and batch).  Under
    # quirk Q1 the two captions are identical and the loss sits at ln 2, so the two samples' loss gradients
    # (w.r.t. each caption's and each image's features, model_m.py:146-163) are nearly opposite, and every
    # parameter gradient is the small sum of two large per-sample contributions: per-sample errors are amplified
    # by kappa = max_b |g_b| / |sum_b g_b| (fp64, max over both modalities).  The fp32 backward's per-sample error is
    # pinned by the well-conditioned fixture (test_b16_feature_gradients_fp32: 1.8e-5, rounded up to 2e-5), so the
    # bound is twice the error model: 2 * kappa * 2e-5.  The reference's own fp32 run (the golden) is measured the
    # same way, beside this run.
    e_gpu, e_ref, kappa = _fp64_oracle_errors(m, g, s, gmax)
    bound = 2 * kappa * 2e-5
    print(f"\n[b16 full fp32] vs the reference's fp32 run: largest grad errs {[(round(e, 6), n) for e, n in errs[:4]]}\n"
          f"  vs the fp64 oracle: this run {e_gpu}, the reference's fp32 run {e_ref}; per-sample cancellation "
          f"kappa {kappa:.1f}; bound {bound:.3e} (headroom {bound / e_gpu[0][0]:.2f}x)")
    assert e_gpu[0][0] < bound, (e_gpu, kappa)


def _fp64_oracle_errors(m, g, s, gmax):
    """Against the oracle in fp64 on the GPU: (3 worst errors of this run's sampled gradients, 3 worst of the
    golden's) with the test's scale convention, and kappa = the per-sample cancellation of the contrastive loss's
    feature gradients, max over modalities of max_b |g_b| / |sum_b g_b| (max-abs norms)."""
    from oracle import clip_ref as R
    p = {n[5:]: t.detach().double().clone().requires_grad_(True) for n, t in m.named_parameters()}
    b = {k: v.to(torch.float64) if v.is_floating_point() else v for k, v in batch(m.config, 2, g).items()}
    with torch.device("cuda"):
        tf = R.text_features(b["input_ids"], b["attention_mask"], p, m.config)
        imf = R.image_features(b["pixel_values"], p, m.config)
        tf.retain_grad()
        imf.retain_grad()
        loss = R.contrastive(tf, imf, p["logit_scale"])["loss"]
    loss.backward()
    kappa = max(float(f.grad.abs().max() / f.grad.sum(0).abs().max()) for f in (tf, imf))
    params = dict(m.named_parameters())
    e_gpu, e_ref = [], []
    for n, (kind, ref, idx) in s.items():
        exact = _take(kind, p[n].grad, idx).astype(np.float64)
        got = _take(kind, params["clip." + n].grad, idx)
        scale = max(float(np.abs(exact).max()), 0.05 * gmax, 1e-8)
        e_gpu.append((float(np.abs(got - exact).max()) / scale, n))
        e_ref.append((float(np.abs(ref - exact).max()) / scale, n))
    return sorted(e_gpu, reverse=True)[:3], sorted(e_ref, reverse=True)[:3], kappa


def test_b16_feature_gradients_fp32(golden):
    """Config 3's backward in a well-conditioned form (tools/gen_goldens.gen_b16_feature_grads):
    ViT-B/16 full fine-tune, B = 4, L = <text_features, Gt> + <image_features, Gi> with fixed random
    G through the reference's own feature paths (no contrastive softmax).  Every sampled parameter
    gradient of the fp32 parity path within 2e-4 of the tensor's scale (floored at 1e-4 of the
    largest gradient: k-projection biases and the text q/k weights are exactly zero, quirk Q1); the
    CPU oracle meets 2e-5 on the same fixture (test_oracle_golden.test_b16_feature_gradients)."""
    g = golden("forward_b16_feature_grads.npz")
    m = make("B/16", False, "fp32", freeze=False)
    b = batch(m.config, 4, g)
    tf = m.get_text_features(b["input_ids"], b["attention_mask"])
    imf = m.get_image_features(b["pixel_values"])
    Gt = torch.from_numpy(synth.normal(tuple(tf.shape), 31, "featgrad_Gt")).cuda()
    Gi = torch.from_numpy(synth.normal(tuple(imf.shape), 31, "featgrad_Gi")).cuda()
    ((tf * Gt).sum() + (imf * Gi).sum()).backward()
    torch.cuda.synchronize()
    assert np.abs(tf.detach().cpu().numpy() - g["text_features"]).max() < 2e-5
    assert np.abs(imf.detach().cpu().numpy() - g["image_features"]).max() < 2e-5
    params = dict(m.named_parameters())
    s = _sampled(g)
    gmax = max(float(np.abs(r).max()) for _, r, _ in s.values())
    errs = []
    for n, (kind, ref, idx) in s.items():
        gr = params["clip." + n].grad
        if gr is None:
            assert float(np.abs(ref).max()) == 0.0, n
            continue
        got = _take(kind, gr, idx)
        scale = max(float(np.abs(ref).max()), 1e-4 * gmax)
        errs.append((float(np.abs(got - ref).max()) / scale, n))
    errs.sort(reverse=True)
    print(f"\n[b16 feature grads fp32] largest errs {[(round(e, 7), n) for e, n in errs[:8]]}")
    assert len(errs) >= 390
    assert errs[0][0] < 2e-4, errs[0]


def test_b16_full_finetune_bf16_gradients_cosine():
    """The bf16 MFMA path's full backward at config 3's shapes against the fp32 path on the same
    weights and batch.  The upstream gradient is a fixed G on both feature vectors (EOS pooling so
    every text parameter gets a gradient), which keeps the comparison about the backward kernels'
    bf16 arithmetic rather than the contrastive softmax's conditioning: per-tensor cosine
    similarity >= 0.999 for every tensor with a non-negligible gradient (k-projection biases are
    identically zero by softmax shift invariance)."""
    grads = {}
    for precision in ("fp32", "bf16x3", "bf16"):
        m = CLIPWithAdapters("B/16", use_text_adapter=False, use_vision_adapter=False, use_shared_adapters=False,
                             freeze_clip=False, device="cuda", precision=precision, pooling="eos")
        b = batch(m.config, 8)
        tf = m.get_text_features(b["input_ids"], b["attention_mask"])
        imf = m.get_image_features(b["pixel_values"])
        Gt = torch.from_numpy(synth.normal(tuple(tf.shape), 21, "cos_Gt")).cuda()
        Gi = torch.from_numpy(synth.normal(tuple(imf.shape), 21, "cos_Gi")).cuda()
        ((tf * Gt).sum() + (imf * Gi).sum()).backward()
        torch.cuda.synchronize()
        grads[precision] = {n: p.grad.detach().double().cpu().flatten() for n, p in m.named_parameters()
                            if p.grad is not None}
        del m
    g32, g16 = grads["fp32"], grads["bf16"]
    nmax = max(float(v.norm()) for v in g32.values())
    worst = (1.0, "")
    checked = 0
    for n, a in g32.items():
        if "k_proj.bias" in n or float(a.norm()) < 1e-4 * nmax:
            continue
        b = g16[n]
        cos = float(a @ b / (a.norm() * b.norm() + 1e-30))
        worst = min(worst, (cos, n))
        checked += 1
    print(f"\n[b16 bf16 vs fp32] {checked} tensors, worst cosine {worst[0]:.6f} at {worst[1]}")
    assert checked > 150
    assert worst[0] >= 0.999, worst


@pytest.mark.parametrize("precision", ["fp32", "bf16x3", "bf16"])
def test_b32_adapter_b256_matches_reference(golden, precision):
    """BASELINE config 2's batch: ViT-B/32 + text/vision adapters, frozen towers, B=256: logits,
    loss and the adapter gradients (the trainable set) vs the reference run."""
    g = golden("forward_b32_adapter_b256.npz")
    m = make("B/32", True, precision)
    out = m(**batch(m.config, 256, g))
    out["loss"].backward()
    torch.cuda.synchronize()
    err = float(np.abs(out["logits_per_text"].detach().cpu().numpy() - g["logits_per_text"]).max())
    print(f"\n[b32 B=256 {precision}] max|dlogit| {err:.4g}")
    assert err < LOGIT_TOL[precision], err
    assert abs(out["loss"].item() - float(g["loss"])) < (1e-4 if precision != "bf16" else 2e-2)
    params = dict(m.named_parameters())
    names = [k[5:] for k in g.files if k.startswith("grad/")]
    assert len(names) == 12
    worst, worst_cos, worst_rel = (0.0, ""), (1.0, ""), (0.0, "")
    for n in names:
        ref = g["grad/" + n].astype(np.float64).ravel()
        got = params[n].grad.detach().double().cpu().numpy().ravel()
        worst = max(worst, (float(np.abs(got - ref).max()) / max(float(np.abs(ref).max()), 1e-8), n))
        worst_cos = min(worst_cos, (float(got @ ref / (np.linalg.norm(got) * np.linalg.norm(ref) + 1e-30)), n))
        worst_rel = max(worst_rel, (float(np.linalg.norm(got - ref) / max(np.linalg.norm(ref), 1e-30)), n))
    print(f"[b32 B=256 {precision}] worst adapter grad err {worst[0]:.3e} at {worst[1]}; "
          f"worst cosine {worst_cos[0]:.6f} at {worst_cos[1]}; worst rel-L2 {worst_rel[0]:.4f} at {worst_rel[1]}")
    if precision != "bf16":
        assert worst[0] < 1e-3, worst
    else:
        # bf16 logits (within 0.15 at scale 100) move individual softmax weights by a few percent,
        # so elementwise bounds measure the softmax's conditioning; the gradient's direction is
        # what the bf16 arithmetic must preserve
        assert worst_cos[0] > 0.993, worst_cos  # measured 0.9951 (r03)


def test_shared_adapters_unfrozen_position_embedding_grad(golden):
    """with the CLIP parameters unfrozen, the shared adapters' keys/values (the vision
    position embedding, model_m.py:96-100) must carry their gradient into that parameter."""
    g = golden("shared_adapters_unfrozen.npz")
    m = CLIPWithAdapters("B/32", use_shared_adapters=True, freeze_clip=False, device="cuda", precision="fp32")
    m.eval()
    b = batch(m.config, 4, g)
    tf = m.get_text_features(b["input_ids"], b["attention_mask"])
    G = torch.from_numpy(synth.normal((4, m.config.projection_dim), 11, "shared_G")).cuda()
    (tf * G).sum().backward()
    torch.cuda.synchronize()
    params = dict(m.named_parameters())
    for n in ("vision_model.embeddings.position_embedding.weight", "text_projection.weight",
              "shared_adapters.0.image_proj.weight", "shared_adapters.1.norm1.weight"):
        key = n if n.startswith("shared") else "clip." + n
        ref = g["grad/" + n]
        got = params[key].grad.detach().cpu().numpy()
        e = float(np.abs(got - ref).max()) / float(np.abs(ref).max())
        print(f"\n[shared unfrozen] {n}: rel err {e:.3e}")
        assert e < 1e-3, (n, e)


def test_projection_width_mismatch_raises():
    """a pooled row whose width does not match the projection raises F.linear's error
    (L/14 with shared adapters: 512-wide rows into the 768x768 text_projection)."""
    from clipmi import towers as T
    m = make("tiny", False, "fp32")
    h = torch.zeros(2, 3, m.config.text_config.hidden_size + 64, device="cuda")
    with pytest.raises(RuntimeError, match="cannot be multiplied"):
        T.PoolProjFn.apply(h, m.clip.text_projection.weight, m._rt, "text_projection.weight", None)


def test_shared_adapters_training_dropout_matches_oracle_with_same_masks():
    """SharedMHSAttentionAdapter in training mode (dropout 0.1 on the attention probabilities and
    after mlp.2, adapter/clip_adapter.py:84,96): features and adapter gradients vs the oracle fed the
    masks the adapters drew (replayed from their seed/offset), fp32; and eval mode is unchanged."""
    from oracle import clip_ref as R
    from clipmi import towers as T
    cfg = C.resolve("B/32")
    m = CLIPWithAdapters("B/32", use_shared_adapters=True, freeze_clip=True, device="cuda", precision="fp32")
    m.train()
    b = batch(cfg, 4)
    t, v = cfg.text_config, cfg.vision_config
    nh, Hd, Nv, Rr = 8, 512, v.num_positions, 4
    masks = []
    for sa in m.shared_adapters:  # each layer draws [nh * R * Nv] then [R * H]
        off = sa.drop_offset
        kp = torch.empty(nh * Rr * Nv, dtype=torch.uint8, device="cuda")
        km = torch.empty(Rr * Hd, dtype=torch.uint8, device="cuda")
        T.call("clipmi_dropout_mask", T.K.stream(), kp.data_ptr(), kp.numel(), sa.p, sa.drop_seed, off)
        T.call("clipmi_dropout_mask", T.K.stream(), km.data_ptr(), km.numel(), sa.p, sa.drop_seed, off + kp.numel())
        masks.append((kp.view(nh, Rr, Nv).cpu(), km.view(Rr, Hd).cpu()))
    tf = m.get_text_features(b["input_ids"], b["attention_mask"])
    G = torch.from_numpy(synth.normal((4, cfg.projection_dim), 11, "shared_G")).cuda()
    (tf * G).sum().backward()
    torch.cuda.synchronize()
    p = R.to_torch(synth.clip_state_dict(cfg, seed=0))
    ta = R.to_torch(synth.adapter_state_dict(t.hidden_size, 256, 0, "text_adapter"))
    sh = [R.to_torch(synth.shared_adapter_state_dict(t.hidden_size, v.hidden_size, 0, f"shared_adapters.{i}"),
                     requires_grad=True) for i in range(2)]
    bc = {k: x.cpu() for k, x in b.items()}
    h = R.adapter(R.text_tower(bc["input_ids"], bc["attention_mask"], p, cfg), ta)[:, :1]
    for s_, (kp, km) in zip(sh, masks):
        h = R.shared_adapter(h, p["vision_model.embeddings.position_embedding.weight"], s_, keep_p=kp, keep_m=km)
    ref = R.linear(h[:, 0], p["text_projection.weight"])
    (ref * G.cpu()).sum().backward()
    err = (tf.detach().cpu() - ref.detach()).abs().max().item() / ref.abs().max().item()
    assert err < 1e-4, err
    params = dict(m.named_parameters())
    for i in range(2):
        for k, r in sh[i].items():
            got = params[f"shared_adapters.{i}.{k}"].grad.cpu()
            e = (got - r.grad).abs().max().item() / max(r.grad.abs().max().item(), 1e-8)
            assert e < 1e-3, (i, k, e)
    m.eval()
    with torch.no_grad():
        a1 = m.get_text_features(b["input_ids"], b["attention_mask"])
        a2 = m.get_text_features(b["input_ids"], b["attention_mask"])
    assert torch.equal(a1, a2)  # no dropout in eval mode


# MXFP8 towers (BASELINE config 5).  Stated tolerance: every GEMM input is rounded to e4m3 (3
# mantissa bits, one power-of-two scale per 32 inputs), i.e. ~2-3 % per element, over 24 + 12
# layers; the logits (100 x cosine) are bounded by FP8_LOGIT_TOL and the features' direction by a
# cosine similarity with the reference's.
# Bounds ~2x the measured error (r03: L/14@336 B=2 0.234, B/32 B=8 0.243; bf16 on the same
# fixtures 0.10 / 0.07).
FP8_LOGIT_TOL = {"l14_336": 0.5, "b32": 0.5}
FP8_FEATURE_COS = 0.99


@pytest.mark.parametrize("tag,preset,B", [("l14_336", "L/14@336", 2), ("b32", "B/32", 8)])
def test_fp8_towers_match_reference(golden, tag, preset, B):
    g = golden(f"forward_{tag}.npz")
    m = make(preset, True, "fp8")
    with torch.no_grad():
        out = m(**batch(m.config, B, g))
        fb = make(preset, True, "bf16")(**batch(m.config, B, g))
    torch.cuda.synchronize()
    lt = out["logits_per_text"].cpu().numpy()
    err = float(np.abs(lt - g["logits_per_text"]).max())
    err16 = float(np.abs(fb["logits_per_text"].cpu().numpy() - g["logits_per_text"]).max())

    def cos(a, b):
        a, b = a.astype(np.float64), b.astype(np.float64)
        return float(((a * b).sum(-1) / (np.linalg.norm(a, axis=-1) * np.linalg.norm(b, axis=-1))).min())
    ci = cos(out["image_features"].cpu().numpy(), g["image_features"])
    ct = cos(out["text_features"].cpu().numpy(), g["text_features"])
    print(f"\n[{tag} fp8] max|dlogit| {err:.4f} (bf16 {err16:.4f}); min feature cosine image {ci:.5f} text {ct:.5f}")
    assert err < FP8_LOGIT_TOL[tag], err
    assert ci > FP8_FEATURE_COS and ct > FP8_FEATURE_COS, (ci, ct)


# Per-depth fp8 error growth at L/14@336: the same synthetic weights truncated to the first d
# layers of both towers (weights are drawn per parameter name, so depth d is a prefix of the full
# model), fp8 features against this library's fp32 parity path (itself pinned to the reference by
# forward_l14_336.npz at 1e-5).  Minimum per-sample feature cosine at every depth >= 0.99.
FP8_DEPTH_COS = 0.99


def test_fp8_feature_cosine_per_depth():
    import dataclasses
    base = C.resolve("L/14@336")
    B = 2
    rows = []
    for d in (1, 2, 6, 12, 24):
        cfg = dataclasses.replace(
            base, name=f"l14_336_depth{d}",
            vision_config=dataclasses.replace(base.vision_config, num_hidden_layers=d),
            text_config=dataclasses.replace(base.text_config, num_hidden_layers=min(d, base.text_config.num_hidden_layers)))
        feats = {}
        for prec in ("fp32", "fp8"):
            m = CLIPWithAdapters(cfg, use_text_adapter=False, use_vision_adapter=False, use_shared_adapters=False,
                                 freeze_clip=True, device="cuda", precision=prec)
            with torch.no_grad():
                out = m(**batch(m.config, B))
            feats[prec] = (out["image_features"].double(), out["text_features"].double())
            del m, out
        torch.cuda.empty_cache()

        def cos(a, b):
            return float(torch.nn.functional.cosine_similarity(a, b, dim=-1).min())
        ci = cos(feats["fp8"][0], feats["fp32"][0])
        ct = cos(feats["fp8"][1], feats["fp32"][1])
        rows.append((d, ci, ct))
        print(f"\n[fp8 depth {d:2d}] min feature cosine vs fp32: image {ci:.5f} text {ct:.5f}")
    for d, ci, ct in rows:
        assert ci > FP8_DEPTH_COS and ct > FP8_DEPTH_COS, (d, ci, ct)


def test_fp8_rejects_training_towers():
    with pytest.raises(ValueError, match="frozen"):
        CLIPWithAdapters("tiny", freeze_clip=False, device="cuda", precision="fp8")


# Tensors whose gradient is summed with fp32 atomics (order varies between runs, so equal only to
# rounding): the token-embedding scatter (wave-aggregated atomics per id chunk).  (The Linear bias
# gradients fused into split-K weight-gradient GEMMs are summed in split order: bitwise.)
_ATOMIC_GRADS = ("token_embedding.weight",)


def test_bf16x3_long_sequence_backward_matches_fp32():
    """bf16x3 with more than 288 vision tokens (N = 325: past the x3 attention kernels' LDS limit), so the engine
    takes its fallback branches -- the exact-f32 attention and the split passes over O and d_qkv -- beside the fused
    image producers (fc1 / fc2's input gradient, LayerNorm backwards): loss, logits and every gradient against the
    exact-f32 mode on the same weights and batch (the x3 error model: ~2^-16 per product)."""
    cfg = C.CLIPConfig(C._text(128, 256, 2, 2, vocab_size=1000, eos_token_id=999, bos_token_id=998),
                       C._vision(128, 256, 2, 2, 8, image=144), 64, name="long")
    res = {}
    for precision in ("fp32", "bf16x3"):
        m = CLIPWithAdapters(cfg, use_text_adapter=False, use_vision_adapter=False, use_shared_adapters=False,
                             freeze_clip=False, device="cuda", precision=precision)
        assert m.config.vision_config.num_positions > 288
        out = m(**batch(m.config, 8), return_loss=True)
        out["loss"].backward()
        torch.cuda.synchronize()
        res[precision] = (out["loss"].item(), out["logits_per_text"].detach().float().clone(),
                          {n: p.grad.detach().double().clone() for n, p in m.named_parameters() if p.grad is not None})
        del m, out
    (l0, z0, g0), (l1, z1, g1) = res["fp32"], res["bf16x3"]
    gmax = max(float(v.abs().max()) for v in g0.values())
    worst = max((float((g1[n] - v).abs().max()) / max(float(v.abs().max()), 0.05 * gmax, 1e-6), n)
                for n, v in g0.items())
    dz = float((z1 - z0).abs().max())
    print(f"\n[bf16x3 N=325 vs fp32] |dloss| {abs(l1 - l0):.2e}, max|dlogit| {dz:.2e}, worst grad err {worst[0]:.2e} "
          f"at {worst[1]}")
    # measured: |dloss| 1e-6, max|dlogit| 1.2e-4, worst gradient 1.6e-4 (layer 0's fc2 weight); bounds with >= 3x
    # headroom: the logits at north_star's 1e-3, the gradients at 5e-4 of the tensor's (or 5 % of the largest) scale
    assert abs(l1 - l0) < 3e-5 and dz < 1e-3
    assert g0.keys() == g1.keys() and worst[0] < 5e-4, worst


@pytest.mark.parametrize("freeze,precision", [(True, "bf16"), (False, "bf16"), (False, "bf16x3")])
def test_deterministic_replay(freeze, precision):
    """SURVEY §5 race check: the same step twice on the same inputs.  Logits and loss must be
    bitwise equal, and so must every gradient but the token embedding's (summed by fp32 atomics:
    within rounding); a racy kernel shows up as a bitwise difference here.  bf16x3: the producers that
    write split images and bias-gradient column partials (GEMM epilogues, attention and LayerNorm backwards)."""
    runs = []
    for _ in range(2):
        m = CLIPWithAdapters("B/32", freeze_clip=freeze, use_shared_adapters=False, device="cuda",
                             precision=precision, init_seed=3)
        b = batch(m.config, 64)
        out = m(**b, return_loss=True)
        out["loss"].backward()
        torch.cuda.synchronize()
        runs.append((out["logits_per_image"].detach().clone(), out["loss"].detach().clone(),
                     {n: p.grad.detach().clone() for n, p in m.named_parameters() if p.grad is not None}))
        del m, out
    (l0, s0, g0), (l1, s1, g1) = runs
    assert torch.equal(l0, l1) and torch.equal(s0, s1)
    assert g0.keys() == g1.keys() and len(g0) > 0
    racy = []
    for n in g0:
        if torch.equal(g0[n], g1[n]):
            continue
        d = (g0[n] - g1[n]).abs().max().item() / max(g0[n].abs().max().item(), 1e-30)
        if any(k in n for k in _ATOMIC_GRADS) and d < 1e-5:
            continue
        racy.append((n, d))
    print(f"\n[replay freeze={freeze} {precision}] {len(g0)} gradients, not bitwise equal beyond atomics: {racy[:8]}")
    assert not racy, racy


@pytest.mark.parametrize("precision,tol", [("fp32", 1e-3), ("bf16", 0.15)])
def test_load_reference_checkpoint(golden, tmp_path, precision, tol):
    """The reference's test_checkpoints/test_adapter.pt (tensors in tests/golden, written back here
    in its {"text_adapter": sd, "vision_adapter": sd} format) through load_adapter_weights; the
    forward must match the reference model that loaded the original file."""
    g = golden("checkpoint_test_adapter.npz")
    ck = {top: {k.split("/", 1)[1]: torch.from_numpy(g[k].copy()) for k in g.files if k.startswith(top + "/")}
          for top in ("text_adapter", "vision_adapter")}
    path = tmp_path / "test_adapter.pt"
    torch.save(ck, path)
    m = CLIPWithAdapters("B/32", use_shared_adapters=False, device="cuda", precision=precision)
    m.load_adapter_weights(str(path))
    for top, mod in (("text_adapter", m.text_adapter), ("vision_adapter", m.vision_adapter)):
        sd = mod.state_dict()
        for k, v in ck[top].items():
            assert torch.equal(sd[k].float().cpu(), v), (top, k)
    with torch.no_grad():
        out = m(**batch(m.config, 2, g), return_loss=True)
    got = out["logits_per_text"].float().cpu().numpy()
    err = float(np.abs(got - g["logits_per_text"]).max())
    print(f"\n[reference checkpoint {precision}] max|dlogit| {err:.3g}")
    assert err < tol


def test_enhanced_adapter_main_checkpoint_roundtrip(tmp_path):
    """main.py:186-193's EnhancedCLIPAdapter checkpoint schema: save -> load into a fresh head."""
    from clipmi.heads import EnhancedCLIPAdapter
    a = EnhancedCLIPAdapter("tiny", device="cuda", seed=1)
    b = EnhancedCLIPAdapter(a.model, device="cuda", seed=2)
    path = tmp_path / "enhanced_adapters_weights.pth"
    a.save_adapter_weights(str(path))
    sd = torch.load(path, weights_only=True)
    assert set(sd) == {"visual_adapter_state_dict", "text_adapter_state_dict", "context_adapter_state_dict"}
    assert set(sd["visual_adapter_state_dict"]) == {"fc1.weight", "fc1.bias", "fc2.weight", "fc2.bias"}
    b.load_adapter_weights(str(path))
    for name in ("visual_adapter", "text_adapter", "context_adapter"):
        for k, v in getattr(a, name).state_dict().items():
            assert torch.equal(getattr(b, name).state_dict()[k], v)
    with pytest.raises(FileNotFoundError):
        b.load_adapter_weights(str(tmp_path / "missing.pth"))


@pytest.mark.parametrize("tag", ["pair", "land"])
def test_uint8_images_match_processor_b32(golden, tag):
    """B/32 (224 px) on raw uint8 images vs the reference processor's own pixel_values
    (CLIPImageProcessor with resize, tests/golden/image_processor_resize.npz)."""
    g = golden("image_processor_resize.npz")
    m = CLIPWithAdapters("B/32", use_shared_adapters=False, device="cuda", precision="fp32")
    n = g[f"{tag}_images"].shape[0]
    b = batch(m.config, n)
    with torch.no_grad():
        a = m.get_image_features(torch.from_numpy(g[f"{tag}_pixel_values"]).cuda())
        u = m.get_image_features(torch.from_numpy(g[f"{tag}_images"]).cuda())
    torch.cuda.synchronize()
    assert (a - u).abs().max().item() < 1e-4 * max(1.0, a.abs().max().item())


def test_config3_full_size_overlap_is_bitwise_serial(monkeypatch):
    """Config 3 at its full size (B/16 full fine-tune, B = 1024, bf16): running the text tower
    on its own stream beside the vision tower (the benchmarked schedule) must not change a bit of
    the loss or of any non-atomic gradient versus the serial schedule; a race between the two
    streams' kernels or workspaces would show here and not at test sizes.  Likewise the deferred
    reductions (split-K and LayerNorm affine sums run by the next persistent GEMM, CLIPMI_DEFER=0: each
    on its own launch) must give the standalone kernels' bits."""
    res = {}
    for ov, df in (("0", "1"), ("1", "1"), ("1", "0")):
        monkeypatch.setenv("CLIPMI_OVERLAP", ov)
        monkeypatch.setenv("CLIPMI_DEFER", df)
        m = CLIPWithAdapters("B/16", use_text_adapter=False, use_vision_adapter=False, use_shared_adapters=False,
                             freeze_clip=False, device="cuda", precision="bf16", fast_init=True)
        b = batch(m.config, 1024)
        out = m(**b, return_loss=True)
        out["loss"].backward()
        torch.cuda.synchronize()
        assert torch.isfinite(out["loss"]).item()
        res[ov + df] = (out["loss"].detach().clone(),
                        {n: p.grad.detach().clone() for n, p in m.named_parameters() if p.grad is not None})
        del m, out, b
        torch.cuda.empty_cache()
    l0, g0 = res["01"]
    for key in ("11", "10"):
        l1, g1 = res[key]
        assert torch.equal(l0, l1), key
        racy = [n for n in g0 if not torch.equal(g0[n], g1[n]) and not any(k in n for k in _ATOMIC_GRADS)]
        print(f"\n[config 3 full size, overlap/defer {key} vs 01] loss {l0.item():.5f}; {len(g0)} gradients, "
              f"differing beyond atomics: {racy[:6]}")
        assert not racy, key


@pytest.mark.parametrize("B", [64])
def test_b16_full_bf16_forward_batch64_matches_oracle(B):
    """Config 3's model (ViT-B/16, full fine-tune setup, bf16 MFMA path) at a wider batch than the
    B <= 8 goldens: the [B, B] contrastive logits and loss against the CPU oracle (oracle/clip_ref.py,
    pinned to the reference by forward_b16.npz) in fp32 on the same synthetic weights and batch.
    Stated bf16 bound as for the goldens: 0.15 at logit scale 100."""
    from oracle import clip_ref as R
    torch.set_num_threads(16)
    m = make("B/16", False, "bf16", freeze=False)
    b = batch(m.config, B, seed=777)
    with torch.no_grad():
        out = m(**b)
    torch.cuda.synchronize()
    p = R.to_torch(synth.clip_state_dict(m.config, seed=0))
    with torch.no_grad():
        ref = R.clip_with_adapters_forward({k: x.cpu() for k, x in b.items()}, p, m.config)
    err = float((out["logits_per_text"].float().cpu() - ref["logits_per_text"]).abs().max())
    lerr = abs(out["loss"].item() - ref["loss"].item())
    print(f"\n[b16 bf16 B={B}] max|dlogit| {err:.4f}, |dloss| {lerr:.2e}")
    assert err < LOGIT_TOL["bf16"], err
    assert lerr < 0.02, lerr


def test_config3_full_size_matches_torch_oracle():
    """Config 3 at its full benchmarked size (ViT-B/16 full fine-tune, B = 1024, the reference's
    contrastive loss) against the oracle (oracle/clip_ref.py, pinned to the reference by the goldens)
    run by PyTorch on the same GPU, weights and batch: (1) clipmi fp32 vs the oracle in fp32 --
    loss, logits and every parameter gradient (relative L2 of the difference); (2) clipmi bf16 vs the
    same fp32 oracle, measured against PyTorch's mixed-precision run of the oracle (torch.autocast
    bf16: bf16 GEMM operands with fp32 accumulation, fp32 LayerNorm / softmax / loss, fp32 residual
    stream and master weights): clipmi's max |dlogit| and every tensor's gradient error at most 1.5x
    the mixed-precision run's, and max |dlogit| <= 0.10 at logit scale 100 (the fp32 residual stream;
    profiles/r05_config3_full_size_parity.log: 0.065 vs AMP's 0.083); (3) clipmi bf16x3 (fp32 activations,
    split-product GEMMs) within north_star's 1e-3 logits and the fp32 mode's gradient bounds.  PyTorch's
    all-bf16 run is printed beside them.  Tensors with a negligible gradient (k-projection biases: zero by softmax
    shift invariance) are skipped."""
    from oracle import clip_ref as R
    res, params = {}, None
    for precision in ("fp32", "bf16x3", "bf16"):
        m = CLIPWithAdapters("B/16", use_text_adapter=False, use_vision_adapter=False, use_shared_adapters=False,
                             freeze_clip=False, device="cuda", precision=precision, fast_init=True)
        b = batch(m.config, 1024)
        out = m(**b, return_loss=True)
        out["loss"].backward()
        torch.cuda.synchronize()
        cfg = m.config
        res[precision] = (out["loss"].item(), out["logits_per_text"].detach().float().clone(),
                          {n[5:]: p.grad.detach().float().clone() for n, p in m.named_parameters() if p.grad is not None})
        if params is None:
            params = {n[5:]: p.detach().clone() for n, p in m.named_parameters()}
        del m, out
        torch.cuda.empty_cache()
    for dt, tag, amp in ((torch.float32, "torch32", False), (torch.float32, "torchamp", True),
                         (torch.bfloat16, "torch16", False)):
        p = {k: v.to(dt).clone().requires_grad_(True) for k, v in params.items()}
        with torch.device("cuda"), torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
            out = R.clip_with_adapters_forward(b, p, cfg)
        out["loss"].backward()
        torch.cuda.synchronize()
        res[tag] = (out["loss"].item(), out["logits_per_text"].detach().float().clone(),
                    {k: v.grad.float() for k, v in p.items() if v.grad is not None})
        del p, out
        torch.cuda.empty_cache()
    lref, zref, gref = res["torch32"]
    nmax = max(float(v.norm()) for v in gref.values())
    names = [n for n, a in gref.items() if "k_proj.bias" not in n and float(a.norm()) >= 1e-4 * nmax]
    kinds = ("fp32", "bf16x3", "bf16", "torchamp", "torch16")
    rel = {k: {n: float((res[k][2][n] - gref[n]).norm() / gref[n].norm()) for n in names} for k in kinds}
    dz = {k: float((res[k][1] - zref).abs().max()) for k in kinds}
    dl = {k: abs(res[k][0] - lref) for k in kinds}
    ratio = sorted(((rel["bf16"][n] / max(rel["torchamp"][n], 1e-6), n) for n in names), reverse=True)
    r32 = sorted(((v, n) for n, v in rel["fp32"].items()), reverse=True)
    w32 = r32[0]
    rx3 = sorted(((v, n) for n, v in rel["bf16x3"].items()), reverse=True)
    print(f"\n[config 3 B=1024 vs torch fp32 oracle] {len(names)} tensors; |dloss| {dl}; max|dlogit| {dz}\n"
          f"  clipmi fp32: worst grad rel-L2 {r32[:3]}; median {r32[len(r32) // 2]}\n"
          f"  clipmi bf16x3: worst grad rel-L2 {rx3[:3]}; median {rx3[len(rx3) // 2]}\n"
          f"  clipmi bf16: worst rel-L2 {max((v, n) for n, v in rel['bf16'].items())}; "
          f"torch amp worst {max((v, n) for n, v in rel['torchamp'].items())}; "
          f"torch all-bf16 worst {max((v, n) for n, v in rel['torch16'].items())}\n"
          f"  worst bf16 ratio clipmi/amp {ratio[:4]}; median {ratio[len(ratio) // 2]}")
    assert len(names) > 150
    assert dl["fp32"] < 1e-4 and dz["fp32"] < 1e-3, (dl, dz)
    # fp32: summation order over R = 201,728 rows (bias / weight gradients are sums over every token,
    # with heavy cancellation) -- measured worst 5.1e-3 (last layer's v-projection bias)
    assert w32[0] < 1e-2, w32
    assert r32[len(r32) // 2][0] < 2e-3, r32[len(r32) // 2]  # measured median 7.4e-4
    # bf16x3 (fp32 activations, split-product GEMMs) meets north_star's fp32 logit bound
    assert dl["bf16x3"] < 1e-4 and dz["bf16x3"] < 1e-3, (dl, dz)
    assert rx3[0][0] < 2e-2 and rx3[len(rx3) // 2][0] < 4e-3, rx3[:3]
    # bf16 (fp32 residual stream since round 5) against PyTorch's mixed precision
    assert dl["bf16"] < 0.02, dl
    assert dz["bf16"] <= 0.10 and dz["bf16"] <= 1.5 * dz["torchamp"], dz
    assert ratio[0][0] <= 1.5, ratio[:4]


def test_config4_model_frozen_towers_matches_torch_amp():
    """BASELINE config 4's model and per-GPU batch (ViT-L/14 adapter fine-tune, frozen towers, B = 1024) against
    the oracle run by PyTorch on the same GPU, weights and batch: clipmi bf16 (the default fp32 residual stream)
    vs the fp32 oracle, measured against PyTorch's mixed-precision run of the oracle (torch.autocast bf16).
    clipmi's max |dlogit| and each adapter tensor's gradient error (relative L2) at most 1.5x the mixed-precision
    run's, and max |dlogit| <= 0.15 at logit scale 100 (the forward goldens' bf16 bound).  Measured
    (profiles/r06_config4_frozen_vs_amp.log): 0.061 vs AMP's 0.066; the bf16 residual stream (residual_fp32=False,
    round 5's frozen-tower default) 0.236."""
    residual_fp32 = None
    from oracle import clip_ref as R
    B = 1024
    m = CLIPWithAdapters("L/14", use_text_adapter=True, use_vision_adapter=True, use_shared_adapters=False,
                         freeze_clip=True, device="cuda", precision="bf16", fast_init=True, residual_fp32=residual_fp32)
    cfg = m.config
    b = batch(cfg, B)
    out = m(**b, return_loss=True)
    out["loss"].backward()
    torch.cuda.synchronize()
    res = {"clipmi": (out["loss"].item(), out["logits_per_text"].detach().float().clone(),
                      {f"{t}.{k}": v.grad.detach().float().clone() for t, a in
                       (("text", m.text_adapter), ("vision", m.vision_adapter)) for k, v in a.named_parameters()})}
    params = {n[5:]: p.detach().clone() for n, p in m.named_parameters() if n.startswith("clip.")}
    ads = {t: {k: v.detach().clone() for k, v in a.state_dict().items()}
           for t, a in (("text", m.text_adapter), ("vision", m.vision_adapter))}
    resid32 = m._rt.resid32
    del m, out
    torch.cuda.empty_cache()
    for tag, amp in (("torch32", False), ("torchamp", True)):
        a = {t: {k: v.clone().requires_grad_(True) for k, v in sd.items()} for t, sd in ads.items()}
        with torch.device("cuda"), torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
            o = R.clip_with_adapters_forward(b, params, cfg, text_adapter=a["text"], vision_adapter=a["vision"])
        o["loss"].backward()
        torch.cuda.synchronize()
        res[tag] = (o["loss"].item(), o["logits_per_text"].detach().float().clone(),
                    {f"{t}.{k}": v.grad.float() for t, sd in a.items() for k, v in sd.items()})
        del a, o
        torch.cuda.empty_cache()
    lref, zref, gref = res["torch32"]
    names = sorted(gref)
    rel = {k: {n: float((res[k][2][n] - gref[n]).norm() / gref[n].norm().clamp_min(1e-30)) for n in names}
           for k in ("clipmi", "torchamp")}
    dz = {k: float((res[k][1] - zref).abs().max()) for k in ("clipmi", "torchamp")}
    dl = {k: abs(res[k][0] - lref) for k in ("clipmi", "torchamp")}
    ratio = sorted(((rel["clipmi"][n] / max(rel["torchamp"][n], 1e-6), n) for n in names), reverse=True)
    print(f"\n[config 4 L/14 frozen B={B} resid32={resid32}] |dloss| {dl}; max|dlogit| {dz}\n"
          f"  grad rel-L2 clipmi {sorted(((v, n) for n, v in rel['clipmi'].items()), reverse=True)[:3]}\n"
          f"  torch amp {sorted(((v, n) for n, v in rel['torchamp'].items()), reverse=True)[:3]}\n"
          f"  worst ratio clipmi/amp {ratio[:4]}")
    assert len(names) == 12
    assert dz["clipmi"] <= 0.15 and dz["clipmi"] <= 1.5 * dz["torchamp"], dz
    assert ratio[0][0] <= 1.5, ratio[:4]

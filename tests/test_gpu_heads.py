"""Feature-level adapter heads (clipmi.heads over csrc/heads.hip) on the GPU against the
reference-pinned oracle (oracle/heads_ref.py, tests/golden/heads.npz).  All fp32: head
outputs within 1e-5 of the reference, trained weights within 1e-4 after 6 Adam steps (lr 3e-4;
Adam's m/sqrt(v) amplifies summation-order noise on near-zero gradient entries)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from clipmi import heads as HD  # noqa: E402
from oracle import heads_ref as H  # noqa: E402
from heads_common import fixture, weights, LN100  # noqa: E402

EMOS = ["angry", "disgust", "fear", "happy", "neutral", "sad", "surprise"]  # reference constants.EMOTIONS


class StubBackbone:
    """Frozen-backbone stand-in serving the fixture's feature tables (the tower features are
    pinned by test_gpu_model); same role as the stub in tools/gen_goldens.py gen_heads."""
    projection_dim = 512

    def __init__(self, desc, img):
        self.desc, self.img = torch.from_numpy(desc).cuda(), torch.from_numpy(img).cuda()
        self.logit_scale = torch.tensor(LN100, device="cuda")

    def get_text_features(self, input_ids, attention_mask=None):
        return self.desc[input_ids[:, 0]]

    def get_image_features(self, pixel_values):
        return self.img[pixel_values.long()]


def make(g):
    desc, img, labels = fixture()
    descs = {e: (torch.arange(i * 5, i * 5 + 5, device="cuda").view(5, 1), None) for i, e in enumerate(EMOS)}
    ca = HD.CLIPAdapter(StubBackbone(desc, img), alpha=0.2, beta=0.2, bottleneck_dim=64, descriptions=descs)
    for nm, ad in (("visual", ca.visual_adapter), ("text", ca.text_adapter)):
        ad.load_state_dict_(dict(zip(("fc1.weight", "fc1.bias", "fc2.weight", "fc2.bias"), weights(g, "init", nm))))
    return ca, desc, img, labels, descs


def test_clip_adapter_matches_reference(golden):
    g = golden("heads.npz")
    ca, desc, img, labels, _ = make(g)
    np.testing.assert_allclose(ca.emotion_embedding_tensor.cpu().numpy(), g["emotion_embedding_tensor"], atol=1e-6)
    idx = torch.arange(24, device="cuda")
    np.testing.assert_allclose(ca.predict(idx).cpu().numpy(), g["predict_untrained"], atol=1e-5)
    lab = torch.from_numpy(labels).cuda()
    loader = [(idx[i:i + 8], lab[i:i + 8], None) for i in range(0, 24, 8)]
    hist = ca.train(loader, num_epochs=2, learning_rate=3e-4)
    assert len(hist) == 2 and all(np.isfinite(hist))
    for nm, ad in (("visual", ca.visual_adapter), ("text", ca.text_adapter)):
        got = ad.state_dict_()
        for k, ref in zip(("fc1.weight", "fc1.bias", "fc2.weight", "fc2.bias"), weights(g, "final", nm)):
            err = (got[k] - ref).abs().max().item()
            assert err < 1e-4, (nm, k, err)
    np.testing.assert_allclose(ca.adapted_emotion_embedding_tensor.cpu().numpy(),
                               g["adapted_emotion_embedding_tensor"], atol=1e-5)
    np.testing.assert_allclose(ca.predict(idx).cpu().numpy(), g["predict"], atol=1e-4)
    np.testing.assert_allclose(ca.predict_with_all_descriptions(idx).cpu().numpy(), g["predict_all"], atol=1e-4)


def test_zero_shot_matches_reference(golden):
    g = golden("heads.npz")
    desc, img, _ = fixture()
    descs = {e: (torch.arange(i * 5, i * 5 + 5, device="cuda").view(5, 1), None) for i, e in enumerate(EMOS)}
    zs = HD.ZeroShotEmotionRecognition(StubBackbone(desc, img), descriptions=descs)
    idx = torch.arange(24, device="cuda")
    np.testing.assert_allclose(zs.predict(idx).cpu().numpy(), g["zs_predict"], atol=1e-5)
    np.testing.assert_allclose(zs.predict_with_all_descriptions(idx).cpu().numpy(), g["zs_predict_all"], atol=1e-5)


@pytest.mark.parametrize("B,E,A,norm_in", [(5, 512, 64, True), (300, 768, 256, False), (3, 1024, 17, True)])
def test_feature_adapter_fwd_bwd_matches_torch(B, E, A, norm_in):
    torch.manual_seed(B)
    ad = HD.FeatureAdapter(E, A, "cuda", seed=B)
    x = torch.randn(B, E, device="cuda")
    out, saved = ad.blend(x, 0.3, norm_in)
    w = [t.detach().clone().requires_grad_(True) for t in (ad.fc1.weight, ad.fc1.bias, ad.fc2.weight, ad.fc2.bias)]
    ref = H.blend(x, w, 0.3, norm_in)
    assert (out - ref).abs().max().item() < 1e-5
    dout = torch.randn(B, E, device="cuda")
    ref.backward(dout)
    ad.grad.zero_()
    ad.backward_(dout, saved)
    ad.backward_(dout, saved)  # accumulates
    got = [ad.grad[:A * E].view(A, E), ad.grad[A * E:A * E + A], ad.grad[A * E + A:2 * A * E + A].view(E, A),
           ad.grad[2 * A * E + A:]]
    for gg, rr in zip(got, w):
        scale = rr.grad.abs().max().item() + 1e-12
        assert ((gg - 2 * rr.grad).abs().max().item()) / scale < 1e-4
    raw = ad(x)
    assert (raw - H.adapter(x, *w)).abs().max().item() < 1e-4


def test_class_scores_and_ce_match_torch():
    torch.manual_seed(3)
    B, E, C = 40, 512, 9
    img = torch.nn.functional.normalize(torch.randn(B, E, device="cuda"), dim=1).requires_grad_(True)
    P = torch.nn.functional.normalize(torch.randn(C, E, device="cuda"), dim=1).requires_grad_(True)
    labels = torch.randint(0, C, (B,), device="cuda")
    off = torch.arange(C + 1, dtype=torch.int32, device="cuda")
    scores, probs, loss_rows, dscore, bad = HD.class_scores(img.detach(), P.detach(), off, 50.0, labels)
    logits = 50.0 * img @ P.T
    assert (scores - logits).abs().max().item() < 1e-4
    assert (probs - logits.softmax(1)).abs().max().item() < 1e-5
    loss = torch.nn.functional.cross_entropy(logits, labels)
    assert abs(loss_rows.mean().item() - loss.item()) < 1e-5 and bad.item() == 0
    loss.backward()
    dimg, dP = torch.empty_like(img), torch.empty_like(P)
    HD.call("clipmi_class_ce_bwd", HD.T.K.stream(), dscore.data_ptr(), img.data_ptr(), P.data_ptr(), B, C, E, 50.0,
            None, dimg.data_ptr(), dP.data_ptr())
    assert (dimg - img.grad).abs().max().item() < 1e-5
    assert (dP - P.grad).abs().max().item() < 1e-5
    # segments: max over each class's descriptions
    D = torch.randn(3 * C, E, device="cuda")
    off3 = torch.arange(0, 3 * C + 1, 3, dtype=torch.int32, device="cuda")
    s3 = HD.class_scores(img.detach(), D, off3, 100.0)[0]
    ref3 = (100.0 * img.detach() @ D.T).view(B, C, 3).amax(2)
    assert (s3 - ref3).abs().max().item() < 1e-3
    bad_lab = labels.clone()
    bad_lab[0] = C
    assert HD.class_scores(img.detach(), P.detach(), off, 50.0, bad_lab)[4].item() == 1


@pytest.mark.parametrize("precision,tol", [("fp32", 1e-4), ("bf16", 5e-2)])
def test_backbone_hf_feature_semantics(golden, precision, tol):
    """The heads' backbone: EOS-pooled text features and CLS + post_layernorm image features
    ([HF] get_text_features / get_image_features, what model_t.py calls) on the native towers."""
    import hashlib
    from clipmi import synth
    g = golden("forward_b32.npz")
    bb = HD._Backbone("B/32", "cuda", precision)
    b = synth.synthetic_batch(bb.m.config, 8, seed=1234)
    h = hashlib.sha256()
    for k in ("pixel_values", "input_ids", "attention_mask"):
        h.update(np.ascontiguousarray(b[k]).tobytes())
    assert h.hexdigest()[:16] == str(g["input_digest"])
    b = {k: torch.from_numpy(v).cuda() for k, v in b.items()}
    fi = bb.get_image_features(b["pixel_values"]).cpu().numpy()
    ft = bb.get_text_features(b["input_ids"], b["attention_mask"]).cpu().numpy()
    ri, rt = g["hf_image_features"], g["text_eos_projected"]
    assert np.abs(fi - ri).max() / np.abs(ri).max() < tol
    assert np.abs(ft - rt).max() / np.abs(rt).max() < tol


def _enhanced(g, ctx_dim=512):
    """EnhancedCLIPAdapter over the fixture's feature tables, adapters initialised from the
    heads.npz init weights (visual, text) and a seeded context adapter."""
    desc, img, labels = fixture()
    descs = {e: (torch.arange(i * 5, i * 5 + 5, device="cuda").view(5, 1), None) for i, e in enumerate(EMOS)}
    m = HD.EnhancedCLIPAdapter(StubBackbone(desc, img), alpha=0.2, beta=0.2, gamma=0.3, bottleneck_dim=64,
                               descriptions=descs, seed=3)
    for nm, ad in (("visual", m.visual_adapter), ("text", m.text_adapter)):
        ad.load_state_dict_(dict(zip(("fc1.weight", "fc1.bias", "fc2.weight", "fc2.bias"), weights(g, "init", nm))))
    ctx = torch.from_numpy(np.random.default_rng(4).standard_normal((24, ctx_dim)).astype(np.float32)).cuda()
    return m, desc, img, labels, ctx


def _w(ad):
    sd = ad.state_dict_()
    return [sd[k].clone() for k in ("fc1.weight", "fc1.bias", "fc2.weight", "fc2.bias")]


def test_enhanced_clip_adapter_eval_matches_oracle(golden):
    """model_v.EnhancedCLIPAdapter eval path (model_v.py:260-353): logits and predict_probs with and
    without context features vs oracle/heads_ref.enhanced_logits (no dropout in eval)."""
    g = golden("heads.npz")
    m, desc, img, labels, ctx = _enhanced(g)
    m.eval()
    m.encode_emotion_descriptions()
    idx = torch.arange(24, device="cuda")
    protos = torch.from_numpy(H.encode(torch.from_numpy(desc), 5)[1].numpy())
    wv, wt, wc = _w(m.visual_adapter), _w(m.text_adapter), _w(m.context_adapter)
    T = float(np.exp(LN100))
    for c in (None, ctx):
        got = m(idx, c).cpu()
        ref = H.enhanced_logits(torch.from_numpy(img), None if c is None else c.cpu(), protos, wv, wt, wc, 0.2, 0.2,
                                0.3, T)
        np.testing.assert_allclose(got.numpy(), ref.numpy(), atol=2e-3, rtol=1e-5)
        pr = m.predict_probs(idx, c).cpu()
        np.testing.assert_allclose(pr.numpy(), torch.softmax(ref, 1).numpy(), atol=1e-5)
    # a context of the wrong width is skipped with a warning, as in the reference (:294-300)
    bad = torch.zeros(24, 7, device="cuda")
    np.testing.assert_allclose(m(idx, bad).cpu().numpy(), m(idx, None).cpu().numpy(), atol=1e-6)


def test_enhanced_clip_adapter_training_matches_oracle_with_same_masks(golden):
    """main.py:55-100 train loop (CE + Adam over visual/text/context adapters, dropout 0.1 in training
    mode): 3 steps with context features; the oracle replays the same dropout masks (the seeded
    counter generator makes them reproducible)."""
    g = golden("heads.npz")
    m, desc, img, labels, ctx = _enhanced(g)
    m.eval()
    m.encode_emotion_descriptions()
    m.train()
    protos = torch.from_numpy(H.encode(torch.from_numpy(desc), 5)[1].numpy())
    params = [p.clone().requires_grad_(True) for p in _w(m.visual_adapter) + _w(m.context_adapter) + _w(m.text_adapter)]
    opt = torch.optim.Adam(params, lr=3e-4)
    T = float(np.exp(LN100))
    lab = torch.from_numpy(labels)
    for step in range(3):
        sl = slice(8 * step, 8 * step + 8)
        # the masks the three adapters will draw this step: visual [8, A], context [8, A], text [7, A]
        keeps = []
        for ad, n in ((m.visual_adapter, 8), (m.context_adapter, 8), (m.text_adapter, 7)):
            d = HD.Dropout(ad.dropout.p, ad.dropout.seed)
            d.offset = ad.dropout.offset
            keeps.append(d.mask(n * ad.A, "cuda").view(n, ad.A).cpu())
        loss = m.train_step(torch.arange(8 * step, 8 * step + 8, device="cuda"), lab[sl].cuda(), ctx[sl],
                            learning_rate=3e-4)
        ref = H.enhanced_train_step(params, torch.from_numpy(img[sl]), ctx[sl].cpu(), protos, lab[sl], 0.2, 0.2, 0.3,
                                    T, opt, keeps)
        assert abs(loss.item() - ref.item()) < 1e-4, (step, loss.item(), ref.item())
    for ad, ref in ((m.visual_adapter, params[:4]), (m.context_adapter, params[4:8]), (m.text_adapter, params[8:])):
        for got, r in zip(_w(ad), ref):
            assert (got - r.detach()).abs().max().item() < 1e-4


def test_dropout_masks_statistics_and_replay():
    """Dropout(0.1) masks: ~10 % dropped, the kept values scaled by 1/0.9 keep the mean, and the same
    (seed, offset) replays the same mask."""
    d = HD.Dropout(0.1, 1234)
    k1 = d.mask(1 << 20, "cuda").float()
    frac = 1.0 - k1.mean().item()
    assert abs(frac - 0.1) < 0.003, frac
    x = torch.rand(1 << 20, device="cuda")
    y = torch.empty_like(x)
    HD.call("clipmi_dropout_apply", HD.T.K.stream(), x.data_ptr(), d.mask(1 << 20, "cuda").data_ptr(), x.numel(),
            d.scale, None, y.data_ptr())
    assert abs(y.mean().item() / x.mean().item() - 1.0) < 0.01
    d2 = HD.Dropout(0.1, 1234)
    assert torch.equal(d2.mask(1 << 20, "cuda").float(), k1)
    assert not torch.equal(d2.mask(1 << 20, "cuda").float(), k1)  # the next draw differs

"""Per-kernel parity of libclipmi against plain PyTorch fp32 references of the same op:
LayerNorm (+ fused vision embedding add), attention fwd/bwd (causal + key padding and
bidirectional), embeddings, column sums, contrastive CE, AdamW and grad-norm."""
import math

import numpy as np

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from clipmi import towers as T  # noqa: E402
from clipmi import kernels as kern  # noqa: E402
from clipmi._lib import BF16, F32  # noqa: E402

DT = {torch.bfloat16: BF16, torch.float32: F32}
TOL = {torch.bfloat16: 3e-2, torch.float32: 2e-5}


def rnd(shape, seed, dtype=torch.float32, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to("cuda", dtype)


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-6)).item()


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("D", [128, 512, 768, 1024, 96, 320, 1000, 2050])  # the last four: the any-width kernels
def test_layernorm_fwd_bwd(dtype, D):
    R = 333
    x = rnd((R, D), 1, dtype)
    w = rnd((D,), 2, dtype, 0.2) + 1
    b = rnd((D,), 3, dtype, 0.2)
    y = torch.empty_like(x)
    st = torch.empty(2, R, device="cuda")
    s = kern.stream()
    T.call("clipmi_layernorm_fwd", s, DT[dtype], x.data_ptr(), D, y.data_ptr(), D, w.data_ptr(), b.data_ptr(),
           st[0].data_ptr(), st[1].data_ptr(), R, D, 1e-5, None, None, 0)
    xr = x.float().requires_grad_(True)
    wr = w.float().requires_grad_(True)
    br = b.float().requires_grad_(True)
    yr = F.layer_norm(xr, (D,), wr, br, 1e-5)
    assert rel(y, yr) < TOL[dtype]
    dy = rnd((R, D), 4, dtype)
    dres = rnd((R, D), 5, dtype)
    yr.backward(dy.float())
    dx = torch.empty_like(x)
    dw = torch.zeros(D, device="cuda")
    db = torch.zeros(D, device="cuda")
    ws = torch.empty(int(T._lib.lib().clipmi_layernorm_bwd_ws(R, D)), dtype=torch.uint8, device="cuda")
    T.call("clipmi_layernorm_bwd", s, DT[dtype], dy.data_ptr(), D, x.data_ptr(), D, st[0].data_ptr(),
           st[1].data_ptr(), w.data_ptr(), dx.data_ptr(), D, dres.data_ptr(), D, dw.data_ptr(), db.data_ptr(), 1,
           ws.data_ptr(), ws.numel(), R, D)
    assert rel(dx, xr.grad + dres.float()) < TOL[dtype] * 2
    assert rel(dw, wr.grad) < TOL[dtype] * 2
    assert rel(db, br.grad) < TOL[dtype] * 2


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_layernorm_vision_embed_fused(dtype):
    B, N, D = 3, 50, 768
    h0 = rnd((B * N, D), 6, dtype)
    pos = rnd((N, D), 7, dtype)
    cls = rnd((D,), 8, dtype)
    w = rnd((D,), 9, dtype, 0.1) + 1
    b = rnd((D,), 10, dtype, 0.1)
    ref_in = h0.float().view(B, N, D) + pos.float()[None]
    ref_in[:, 0] += cls.float()
    y = torch.empty_like(h0)
    st = torch.empty(2, B * N, device="cuda")
    T.call("clipmi_layernorm_fwd", kern.stream(), DT[dtype], h0.data_ptr(), D, y.data_ptr(), D, w.data_ptr(),
           b.data_ptr(), st[0].data_ptr(), st[1].data_ptr(), B * N, D, 1e-5, pos.data_ptr(), cls.data_ptr(), N)
    assert rel(h0.view(B, N, D), ref_in) < TOL[dtype]
    assert rel(y.view(B, N, D), F.layer_norm(ref_in, (D,), w.float(), b.float(), 1e-5)) < TOL[dtype]


def attn_ref(qkv, B, N, H, mask, causal):
    D = H * 64
    q, k, v = qkv.float().view(B, N, 3, H, 64).permute(2, 0, 3, 1, 4)
    s = q @ k.transpose(-1, -2) / 8.0
    blocked = torch.zeros(B, 1, N, N, dtype=torch.bool, device=qkv.device)
    if causal:
        blocked |= torch.triu(torch.ones(N, N, dtype=torch.bool, device=qkv.device), 1)
    if mask is not None:
        blocked |= (mask == 0)[:, None, None, :]
    s = s.masked_fill(blocked, float("-inf"))
    p = torch.softmax(s, -1)
    o = (p @ v).transpose(1, 2).reshape(B * N, D)
    return o, torch.logsumexp(s, -1).reshape(-1)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("B,N,H,causal", [(3, 17, 2, False), (2, 50, 12, False), (2, 197, 12, False),
                                           (3, 77, 8, True), (2, 256, 2, False), (3, 150, 2, True),
                                           # ViT-L/14 at 224 (N = 257) and the N <= 288 limit
                                           (2, 257, 16, False), (3, 288, 2, False), (40, 257, 16, False),
                                           # more (batch, head) items than the persistent grid
                                           (90, 197, 12, False), (130, 77, 8, True),
                                           # ViT-L/14@336 (N = 577): K/V-streaming kernels
                                           (2, 577, 4, False), (2, 400, 3, False), (3, 400, 2, True)])
@pytest.mark.parametrize("fa", [False, True])
def test_attention(dtype, B, N, H, causal, fa, monkeypatch):
    """fa: the K/V-streaming flash forward (attn_fwd_fa) for every N (it is the only bf16 forward
    for N > 288); otherwise the whole-K/V kernel where N allows."""
    if fa and dtype == torch.float32:
        pytest.skip("kernel choice applies to the bf16 path")
    monkeypatch.setenv("CLIPMI_ATTN_FA", "1" if fa else "0")
    D = H * 64
    qkv = rnd((B * N, 3 * D), 11, dtype)
    mask = None
    if causal:
        g = torch.Generator().manual_seed(12)
        lens = torch.randint(5, N + 1, (B,), generator=g)
        mask = (torch.arange(N)[None] < lens[:, None]).to(torch.int64).cuda()
    o = torch.empty(B * N, D, dtype=dtype, device="cuda")
    lse = torch.empty(B * H * N, device="cuda")
    s = kern.stream()
    T.call("clipmi_attention_fwd", s, DT[dtype], qkv.data_ptr(), o.data_ptr(), lse.data_ptr(),
           mask.data_ptr() if mask is not None else None, int(causal), B, H, N, D)
    qr = qkv.float().requires_grad_(True)
    oref, lref = attn_ref(qr, B, N, H, mask, causal)
    assert rel(o, oref) < TOL[dtype], "O"
    assert (lse - lref).abs().max().item() < (2e-2 if dtype == torch.bfloat16 else 1e-4), "lse"
    do = rnd((B * N, D), 13, dtype)
    oref.backward(do.float())
    dqkv = torch.empty_like(qkv)
    T.call("clipmi_attention_bwd", s, DT[dtype], qkv.data_ptr(), o.data_ptr(), lse.data_ptr(), do.data_ptr(),
           dqkv.data_ptr(), mask.data_ptr() if mask is not None else None, int(causal), B, H, N, D)
    g = qr.grad
    for i, nm in enumerate("qkv"):
        sl = slice(i * D, (i + 1) * D)
        assert rel(dqkv[:, sl], g[:, sl]) < TOL[dtype] * 2, nm


@pytest.mark.parametrize("B,N,H,causal", [(3, 17, 2, False), (2, 50, 12, False), (2, 197, 12, False),
                                           (3, 77, 8, True), (3, 150, 2, True), (2, 257, 16, False),
                                           (3, 288, 2, False), (90, 197, 12, False), (130, 77, 8, True),
                                           # N > 288: the exact-f32 kernels
                                           (2, 400, 3, False)])
def test_attention_x3(B, N, H, causal):
    """The bf16x3 mode's attention (attention_x3.hip: every product as three bf16 MFMA products of the hi / lo
    splits) against an fp64 reference: ~2^-16 relative per product, held to 1e-4 (O, lse) and 3e-4 (dq, dk,
    dv) -- the bf16 kernels' bound is 3e-2."""
    D = H * 64
    qkv = rnd((B * N, 3 * D), 11, torch.float32)
    mask = None
    if causal:
        g = torch.Generator().manual_seed(12)
        lens = torch.randint(5, N + 1, (B,), generator=g)
        mask = (torch.arange(N)[None] < lens[:, None]).to(torch.int64).cuda()
    o = torch.empty(B * N, D, device="cuda")
    lse = torch.empty(B * H * N, device="cuda")
    s = kern.stream()
    T.call("clipmi_attention_fwd_x3", s, qkv.data_ptr(), o.data_ptr(), lse.data_ptr(),
           mask.data_ptr() if mask is not None else None, int(causal), B, H, N, D)
    qr = qkv.double().requires_grad_(True)
    oref, lref = attn_ref64(qr, B, N, H, mask, causal)
    e_o, e_l = rel(o, oref), (lse.double() - lref).abs().max().item()
    do = rnd((B * N, D), 13, torch.float32)
    oref.backward(do.double())
    dqkv = torch.empty_like(qkv)
    T.call("clipmi_attention_bwd_x3", s, qkv.data_ptr(), o.data_ptr(), lse.data_ptr(), do.data_ptr(),
           dqkv.data_ptr(), mask.data_ptr() if mask is not None else None, int(causal), B, H, N, D)
    g = qr.grad
    e_g = [rel(dqkv[:, i * D:(i + 1) * D], g[:, i * D:(i + 1) * D]) for i in range(3)]
    print(f"\n[x3 attention B={B} N={N} H={H} causal={causal}] O {e_o:.2e} lse {e_l:.2e} dq/dk/dv {e_g}")
    assert e_o < 1e-4 and e_l < 1e-4, (e_o, e_l)
    assert max(e_g) < 3e-4, e_g


@pytest.mark.parametrize("B,N,H,causal", [(3, 17, 2, False), (2, 197, 12, False), (5, 77, 8, True),
                                           (3, 288, 2, False), (40, 197, 12, False)])
def test_attention_bwd_x3img_matches_fp32_then_split(B, N, H, causal):
    """clipmi_attention_bwd_x3img (the bf16x3 engine's attention backward since round 6): d_qkv written as its
    pattern-1 split image and its column sums (the qkv bias gradient) added onto colsum -- bit for bit the image
    clipmi_split3_colsum makes of clipmi_attention_bwd_x3's fp32 d_qkv, the sums against fp64."""
    D = H * 64
    qkv = rnd((B * N, 3 * D), 41, torch.float32)
    mask = None
    if causal:
        g = torch.Generator().manual_seed(42)
        lens = torch.randint(5, N + 1, (B,), generator=g)
        mask = (torch.arange(N)[None] < lens[:, None]).to(torch.int64).cuda()
    mp = mask.data_ptr() if mask is not None else None
    o = torch.empty(B * N, D, device="cuda")
    lse = torch.empty(B * H * N, device="cuda")
    s = kern.stream()
    T.call("clipmi_attention_fwd_x3", s, qkv.data_ptr(), o.data_ptr(), lse.data_ptr(), mp, int(causal), B, H, N, D)
    do = rnd((B * N, D), 43, torch.float32)
    dqkv = torch.empty_like(qkv)
    T.call("clipmi_attention_bwd_x3", s, qkv.data_ptr(), o.data_ptr(), lse.data_ptr(), do.data_ptr(),
           dqkv.data_ptr(), mp, int(causal), B, H, N, D)
    img = torch.full((B * N, 9 * D), float("nan"), dtype=torch.bfloat16, device="cuda")
    cs0 = rnd((3 * D,), 44, torch.float32)
    cs = cs0.clone()
    ws = T._ws(T._lib.lib().clipmi_attention_bwd_x3img_ws(B, D), "cuda")
    T.call("clipmi_attention_bwd_x3img", s, qkv.data_ptr(), o.data_ptr(), lse.data_ptr(), do.data_ptr(),
           img.data_ptr(), cs.data_ptr(), 1, ws.data_ptr(), ws.numel(), mp, int(causal), B, H, N, D)
    assert torch.equal(img, _split_ref(dqkv, 1))
    assert rel(cs - cs0, dqkv.double().sum(0)) < 1e-5
    # the forward's image form: O and lse unchanged, O's pattern-0 image beside them
    o2, lse2 = torch.empty_like(o), torch.empty_like(lse)
    oimg = torch.full((B * N, 3 * D), float("nan"), dtype=torch.bfloat16, device="cuda")
    T.call("clipmi_attention_fwd_x3img", s, qkv.data_ptr(), o2.data_ptr(), oimg.data_ptr(), lse2.data_ptr(), mp,
           int(causal), B, H, N, D)
    assert torch.equal(o2, o) and torch.equal(lse2, lse) and torch.equal(oimg, _split_ref(o, 0))
    with pytest.raises(ValueError, match="N <= 288"):
        T.call("clipmi_attention_bwd_x3img", s, qkv.data_ptr(), o.data_ptr(), lse.data_ptr(), do.data_ptr(),
               img.data_ptr(), cs.data_ptr(), 1, ws.data_ptr(), ws.numel(), mp, int(causal), 1, H, 300, D)


def attn_ref64(qkv, B, N, H, mask, causal):
    D = H * 64
    q, k, v = qkv.view(B, N, 3, H, 64).permute(2, 0, 3, 1, 4)
    s = q @ k.transpose(-1, -2) / 8.0
    blocked = torch.zeros(B, 1, N, N, dtype=torch.bool, device=qkv.device)
    if causal:
        blocked |= torch.triu(torch.ones(N, N, dtype=torch.bool, device=qkv.device), 1)
    if mask is not None:
        blocked |= (mask == 0)[:, None, None, :]
    s = s.masked_fill(blocked, float("-inf"))
    p = torch.softmax(s, -1)
    o = (p @ v).transpose(1, 2).reshape(B * N, D)
    return o, torch.logsumexp(s, -1).reshape(-1)


@pytest.mark.parametrize("B,N,H,causal", [(2, 197, 12, False), (90, 197, 12, False), (3, 150, 2, True),
                                           (2, 224, 3, False), (2, 129, 2, False)])
def test_attention_bwd_single_pass(B, N, H, causal, monkeypatch):
    """The opt-in single-pass backward (attn_bwd_sp, CLIPMI_ATTN_BWD_SP=1: dQ from the dS^T image
    instead of a second, recomputing phase) against the torch fp32 reference, like test_attention."""
    monkeypatch.setenv("CLIPMI_ATTN_FA", "0")
    monkeypatch.setenv("CLIPMI_ATTN_BWD_SP", "1")
    dtype = torch.bfloat16
    D = H * 64
    qkv = rnd((B * N, 3 * D), 31, dtype)
    mask = None
    if causal:
        g = torch.Generator().manual_seed(32)
        lens = torch.randint(5, N + 1, (B,), generator=g)
        mask = (torch.arange(N)[None] < lens[:, None]).to(torch.int64).cuda()
    mp = mask.data_ptr() if mask is not None else None
    o = torch.empty(B * N, D, dtype=dtype, device="cuda")
    lse = torch.empty(B * H * N, device="cuda")
    s = kern.stream()
    T.call("clipmi_attention_fwd", s, DT[dtype], qkv.data_ptr(), o.data_ptr(), lse.data_ptr(), mp, int(causal), B, H, N, D)
    qr = qkv.float().requires_grad_(True)
    oref, _ = attn_ref(qr, B, N, H, mask, causal)
    do = rnd((B * N, D), 33, dtype)
    oref.backward(do.float())
    dqkv = torch.empty_like(qkv)
    T.call("clipmi_attention_bwd", s, DT[dtype], qkv.data_ptr(), o.data_ptr(), lse.data_ptr(), do.data_ptr(),
           dqkv.data_ptr(), mp, int(causal), B, H, N, D)
    for i, nm in enumerate("qkv"):
        sl = slice(i * D, (i + 1) * D)
        assert rel(dqkv[:, sl], qr.grad[:, sl]) < TOL[dtype] * 2, nm


@pytest.mark.parametrize("qpw", ["2", "4"])
@pytest.mark.parametrize("B,N,H,causal", [(2, 577, 4, False), (3, 400, 2, True), (2, 197, 12, False)])
def test_attention_flash_chunk_switch(qpw, B, N, H, causal, monkeypatch):
    """CLIPMI_FA_QPW (the flash forward's query blocks per wave, i.e. 128- or 256-query chunks) keeps
    the forward within the bf16 tolerance of the torch fp32 reference."""
    monkeypatch.setenv("CLIPMI_ATTN_FA", "1")
    monkeypatch.setenv("CLIPMI_FA_QPW", qpw)
    dtype = torch.bfloat16
    D = H * 64
    qkv = rnd((B * N, 3 * D), 41, dtype)
    mask = None
    if causal:
        g = torch.Generator().manual_seed(42)
        lens = torch.randint(5, N + 1, (B,), generator=g)
        mask = (torch.arange(N)[None] < lens[:, None]).to(torch.int64).cuda()
    o = torch.empty(B * N, D, dtype=dtype, device="cuda")
    lse = torch.empty(B * H * N, device="cuda")
    T.call("clipmi_attention_fwd", kern.stream(), DT[dtype], qkv.data_ptr(), o.data_ptr(), lse.data_ptr(),
           mask.data_ptr() if mask is not None else None, int(causal), B, H, N, D)
    oref, lref = attn_ref(qkv.float(), B, N, H, mask, causal)
    assert rel(o, oref) < TOL[dtype]
    assert (lse - lref).abs().max().item() < 2e-2


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_text_embedding_fwd_bwd(dtype):
    B, S, D, V = 6, 77, 512, 1000
    g = torch.Generator().manual_seed(14)
    ids = torch.randint(0, V, (B, S), generator=g)
    ids[:, 40:] = V - 1  # heavy repetition, like EOS padding
    ids = ids.cuda()
    tok = rnd((V, D), 15, dtype)
    pos = rnd((S, D), 16, dtype)
    x0 = torch.empty(B * S, D, dtype=dtype, device="cuda")
    bad = torch.zeros(1, dtype=torch.int32, device="cuda")
    s = kern.stream()
    T.call("clipmi_text_embed", s, DT[dtype], ids.data_ptr(), tok.data_ptr(), pos.data_ptr(), x0.data_ptr(),
           B * S, S, D, V, bad.data_ptr())
    ref = tok.float()[ids] + pos.float()[None]
    assert rel(x0.view(B, S, D), ref) < TOL[dtype]
    assert bad.item() == 0
    dx = rnd((B * S, D), 17, dtype)
    gtok = torch.zeros(V, D, device="cuda")
    ws = torch.empty(int(T._lib.lib().clipmi_text_embed_bwd_ws(B * S, V)), dtype=torch.uint8, device="cuda")
    T.call("clipmi_text_embed_bwd", s, DT[dtype], ids.data_ptr(), dx.data_ptr(), B * S, D, V, gtok.data_ptr(), 1,
           ws.data_ptr(), ws.numel())
    gref = torch.zeros(V, D, device="cuda").index_add_(0, ids.view(-1), dx.float())
    assert rel(gtok, gref) < 1e-5
    gpos = torch.zeros(S, D, device="cuda")
    T.call("clipmi_period_sum", s, DT[dtype], dx.data_ptr(), D, B, S, S, D, gpos.data_ptr(), 1)
    assert rel(gpos, dx.float().view(B, S, D).sum(0)) < 1e-5
    ids_bad = ids.clone()
    ids_bad[0, 3] = V + 5
    T.call("clipmi_text_embed", s, DT[dtype], ids_bad.data_ptr(), tok.data_ptr(), pos.data_ptr(), x0.data_ptr(),
           B * S, S, D, V, bad.data_ptr())
    assert bad.item() == 1


@pytest.mark.parametrize("B,N,H,causal", [(4, 197, 12, False), (3, 150, 2, True), (2, 224, 3, False),
                                           (2, 129, 2, False), (2, 255, 2, False)])
def test_attention_wave_count_invariant(B, N, H, causal, monkeypatch):
    """The 16-wave whole-K/V kernels (one query / key block per wave) compute every block with the
    same instruction sequence as the 8-wave ones (two blocks per wave): identical outputs.  (The
    4-wave backward, four blocks per wave, is compiled only into the experiments build; there
    CLIPMI_ATTN_BWD_NW=4 selects it, in the product library the 8-wave kernel.)"""
    D = H * 64
    qkv = rnd((B * N, 3 * D), 21, torch.bfloat16)
    do = rnd((B * N, D), 22, torch.bfloat16)
    mask = None
    if causal:
        g = torch.Generator().manual_seed(23)
        lens = torch.randint(5, N + 1, (B,), generator=g)
        mask = (torch.arange(N)[None] < lens[:, None]).to(torch.int64).cuda()
    mp = mask.data_ptr() if mask is not None else None
    s = kern.stream()
    monkeypatch.setenv("CLIPMI_ATTN_FA", "0")
    outs = []
    for nw in ("8", "16", "4"):
        monkeypatch.setenv("CLIPMI_ATTN_FWD_NW", nw)
        monkeypatch.setenv("CLIPMI_ATTN_BWD_NW", nw)
        o = torch.empty(B * N, D, dtype=torch.bfloat16, device="cuda")
        lse = torch.empty(B * H * N, device="cuda")
        dqkv = torch.empty_like(qkv)
        T.call("clipmi_attention_fwd", s, DT[torch.bfloat16], qkv.data_ptr(), o.data_ptr(), lse.data_ptr(), mp,
               int(causal), B, H, N, D)
        T.call("clipmi_attention_bwd", s, DT[torch.bfloat16], qkv.data_ptr(), o.data_ptr(), lse.data_ptr(),
               do.data_ptr(), dqkv.data_ptr(), mp, int(causal), B, H, N, D)
        torch.cuda.synchronize()
        outs.append((o, lse, dqkv))
    for other in outs[1:]:
        for a, b, nm in zip(outs[0], other, ("O", "lse", "dqkv")):
            assert torch.equal(a, b), nm


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("H,P", [(64, 16), (56, 14)])  # P=14 (ViT-L/14): K = 588 padded to 640
def test_im2col_matches_conv(dtype, H, P):
    B, D = 2, 128
    px = rnd((B, 3, H, H), 18)
    W = rnd((D, 3, P, P), 19, scale=0.05)
    G = H // P
    Kc = 3 * P * P
    Kp = (Kc + 63) // 64 * 64 if Kc % 8 else Kc
    X = torch.empty(B * (G * G + 1), Kp, dtype=dtype, device="cuda")
    X.fill_(7.0)  # every element must be written (pad columns and the class-token rows as zeros)
    T.call("clipmi_im2col", kern.stream(), DT[dtype], px.data_ptr(), X.data_ptr(), B, 3, H, P, Kp)
    assert X[:, Kc:].abs().max().item() == 0 if Kp > Kc else True
    # element for element: torch's unfold of the same pixels (a zero row per image for the class token)
    ref_x = F.unfold(px, P, stride=P).transpose(1, 2).to(dtype)  # [B, G*G, 3*P*P]
    Xv = X.view(B, G * G + 1, Kp)
    assert torch.equal(Xv[:, 1:, :Kc], ref_x) and Xv[:, 0].abs().max().item() == 0
    out = torch.empty(B * (G * G + 1), D, dtype=torch.float32, device="cuda")
    Wd = F.pad(W.to(dtype).view(D, Kc), (0, Kp - Kc)).contiguous()
    kern.gemm(B * (G * G + 1), D, Kp, X, Kp, True, Wd, Kp, True, out, D)
    ref = F.conv2d(px, W, stride=P).flatten(2).transpose(1, 2)
    out = out.view(B, G * G + 1, D)
    assert out[:, 0].abs().max().item() == 0.0
    assert rel(out[:, 1:], ref) < TOL[dtype]


def test_colsum():
    R, N = 5000, 3072
    x = rnd((R, N), 20, torch.bfloat16)
    out = rnd((N,), 21)
    o0 = out.clone()
    ws = torch.empty(int(T._lib.lib().clipmi_colsum_ws(R, N)), dtype=torch.uint8, device="cuda")
    T.call("clipmi_colsum", kern.stream(), BF16, x.data_ptr(), N, R, N, out.data_ptr(), 1, ws.data_ptr(), ws.numel())
    assert rel(out, o0 + x.float().sum(0)) < 1e-5


@pytest.mark.parametrize("B,E", [(8, 64), (256, 512), (1000, 512)])
def test_contrastive_fn_matches_torch(B, E):
    t = rnd((B, E), 22).requires_grad_(True)
    i = rnd((B, E), 23).requires_grad_(True)
    ls = torch.tensor(math.log(100.0), device="cuda", requires_grad=True)

    class _A:  # minimal arena stand-in for the logit_scale gradient
        def __init__(self):
            self.grad = torch.zeros(64, device="cuda")

        def prepare_grads(self):
            pass

        def ptr(self, name, buf):
            return buf.data_ptr()

    ar = _A()
    loss, th, ih, lt, li = T.ContrastiveFn.apply(t, i, ls, None, True, ar)
    loss.backward()
    tr = t.detach().clone().requires_grad_(True)
    ir = i.detach().clone().requires_grad_(True)
    lr_ = ls.detach().clone().requires_grad_(True)
    tn, inn = tr / tr.norm(dim=-1, keepdim=True), ir / ir.norm(dim=-1, keepdim=True)
    L = tn @ inn.t() * lr_.exp()
    lab = torch.arange(B, device="cuda")
    lref = (F.cross_entropy(L, lab) + F.cross_entropy(L.t(), lab)) / 2
    lref.backward()
    assert abs(loss.item() - lref.item()) < 1e-5
    assert rel(lt, L) < 1e-5
    assert rel(li, L.t()) < 1e-5
    assert rel(t.grad, tr.grad) < 1e-4
    assert rel(i.grad, ir.grad) < 1e-4
    assert abs(ar.grad[0].item() - lr_.grad.item()) < 1e-4 * max(1, abs(lr_.grad.item()))


@pytest.mark.parametrize("B,E,chunk", [(1000, 512, 256), (1000, 512, 333), (4096, 768, 1024), (64, 64, 1),
                                        # config 5's global batch on one GPU: Bg = 32768 columns in
                                        # [32768, 8192] chunks vs the materialised 4.3 GB logits
                                        (32768, 768, 8192)])
def test_contrastive_streamed_matches_materialised(B, E, chunk, monkeypatch):
    """Column-streamed InfoNCE (Bg > CLIPMI_CE_CHUNK: online log-sum-exp over column chunks,
    chunk recompute in backward, [B, Bg] never materialised) against the plain path."""

    class _A:
        def __init__(self):
            self.grad = torch.zeros(64, device="cuda")

        def prepare_grads(self):
            pass

        def ptr(self, name, buf):
            return buf.data_ptr()

    res = []
    for ch in (None, chunk):
        if ch is None:
            monkeypatch.delenv("CLIPMI_CE_CHUNK", raising=False)
        else:
            monkeypatch.setenv("CLIPMI_CE_CHUNK", str(ch))
        t = rnd((B, E), 26).requires_grad_(True)
        i = rnd((B, E), 27).requires_grad_(True)
        ls = torch.tensor(math.log(100.0), device="cuda", requires_grad=True)
        ar = _A()
        loss, th, ih, lt, li = T.ContrastiveFn.apply(t, i, ls, None, True, ar)
        assert (lt is None) == (ch is not None)
        (loss + (th * th.detach()).sum() * 1e-3).backward()  # a feature-output gradient too
        res.append((loss.item(), t.grad, i.grad, ar.grad[0].item()))
    (l0, t0, i0, s0), (l1, t1, i1, s1) = res
    assert abs(l1 - l0) < 1e-5 * max(1.0, abs(l0))
    assert rel(t1, t0) < 1e-5
    assert rel(i1, i0) < 1e-5
    assert abs(s1 - s0) < 1e-5 * max(1.0, abs(s0))


def test_adamw_and_clip_match_torch():
    n = 100_003
    p = rnd((n,), 24)
    g = rnd((n,), 25, scale=3.0)
    p_ref = p.clone().requires_grad_(True)
    opt = torch.optim.AdamW([p_ref], lr=1e-3, weight_decay=0.01)
    m = torch.zeros(n, device="cuda")
    v = torch.zeros(n, device="cuda")
    shadow = torch.empty(n, dtype=torch.bfloat16, device="cuda")
    norm = torch.zeros(2, device="cuda")
    gp = (T.c_vp * 1)(g.data_ptr())
    gn = (T.c_i64 * 1)(n)
    ws = torch.empty(int(T._lib.lib().clipmi_grad_norm_multi_ws(1)), dtype=torch.uint8, device="cuda")
    for step in range(1, 4):
        T.call("clipmi_grad_norm_multi", kern.stream(), gp, gn, 1, 1.0, norm.data_ptr(), ws.data_ptr(), ws.numel())
        T.call("clipmi_adamw", kern.stream(), p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(),
               shadow.data_ptr(), n, 1e-3, 0.9, 0.999, 1e-8, 0.01, step, norm.data_ptr())
        p_ref.grad = g.clone()
        tn = torch.nn.utils.clip_grad_norm_([p_ref], 1.0)
        opt.step()
        assert abs(norm[0].item() - tn.item()) < 1e-3 * tn.item()
    assert rel(p, p_ref.detach()) < 1e-5
    assert rel(shadow, p_ref.detach()) < 1e-2


@pytest.mark.parametrize("n", [50_001, 9_000_011])  # the second spans both 4-parameter groups of a lane
def test_adamw_vector_path_matches_scalar_path(n):
    """16-B-aligned arenas take the 4-per-lane AdamW kernel, a 4-B offset the scalar one: the same
    update to the last bit or two (the compiler may contract a mul+add into an fma differently in
    the packed body; each path is itself deterministic).  n = 9,000,011 > 2 x 4096 x 256 x 4 runs the
    second parameter group of every lane and the clamped tail of the grid-stride loop."""
    outs = []
    for off in (0, 1):  # element offset 0: aligned (vector body + tail); 1: misaligned (scalar)
        bufs = [torch.zeros(n + 4, device="cuda") for _ in range(4)]
        for i, b in enumerate(bufs):
            b[off:off + n] = rnd((n,), 40 + i)
        p, g, m, v = (b[off:off + n] for b in bufs)
        v.abs_()
        sh = torch.empty(n + 4, dtype=torch.bfloat16, device="cuda")[off:off + n]
        T.call("clipmi_adamw", kern.stream(), p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(),
               sh.data_ptr(), n, 1e-3, 0.9, 0.999, 1e-8, 0.01, 3, None)
        torch.cuda.synchronize()
        outs.append([p.clone(), m.clone(), v.clone(), sh.clone()])
    for a, b in zip(*outs):
        assert torch.allclose(a.float(), b.float(), rtol=2e-6, atol=1e-9) if a.dtype == torch.float32 else \
            (a.float() - b.float()).abs().max().item() <= 2 ** -7 * b.float().abs().max().item()


@pytest.mark.parametrize("tag", ["sq", "crop"])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("P", [16, 14])
def test_im2col_uint8_matches_processor(golden, tag, dtype, P):
    """Fused input step (uint8 NHWC -> crop + rescale + normalise + im2col) vs im2col of the
    reference processor's pixel_values (tests/golden/image_processor.npz)."""
    g = golden("image_processor.npz")
    imgs = torch.from_numpy(g[f"{tag}_images"]).cuda()
    pv = torch.from_numpy(g[f"{tag}_pixel_values"]).cuda()
    B, S = imgs.shape[0], 224
    Kc = 3 * P * P
    Kp = (Kc + 63) // 64 * 64 if Kc % 8 else Kc  # P=14 (ViT-L/14): 588 padded to 640, pad columns zeroed
    R = B * ((S // P) ** 2 + 1)
    X = torch.full((R, Kp), 7.0, device="cuda", dtype=dtype)
    T.im2col_uint8(imgs, X, S, P)
    Xr = torch.empty(R, Kp, device="cuda", dtype=dtype)
    T.call("clipmi_im2col", kern.stream(), DT[dtype], pv.data_ptr(), Xr.data_ptr(), B, 3, S, P, Kp)
    torch.cuda.synchronize()
    tol = 2e-6 if dtype == torch.float32 else 2e-2
    assert (X.float() - Xr.float()).abs().max().item() < tol


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
@pytest.mark.parametrize("tag,D,ln", [("text", 512, True), ("vision", 768, True), ("textual", 512, False)])
def test_adapter_fn_all_tokens_matches_reference(golden, precision, tag, D, ln):
    """towers.AdapterFn on every token of [2, 5, D] (TextAdapter / VisionAdapter, and with ln=False
    peclip.TextualAdapter, adapter/peclip.py:13-18) through libclipmi's one-call entry points
    clipmi_adapter_fwd / clipmi_adapter_bwd: output, input gradient and parameter gradients vs the
    reference modules' run (tests/golden/adapters.npz)."""
    import types
    import numpy as np
    from clipmi import synth
    from clipmi import towers as T
    from clipmi.modules import AdapterParams
    g = golden("adapters.npz")
    names = ("down_project", "up_project") if ln else ("down_proj", "up_proj")
    mod = AdapterParams(D, 256, "cuda", ln=ln, shadow=precision == "bf16", names=names)
    sd = synth.adapter_state_dict(D, 256, 7, f"{tag}_adapter", ln=ln)
    if not ln:
        sd = {k.replace("down_project", "down_proj").replace("up_project", "up_proj"): v for k, v in sd.items()}
    mod.load_numpy(sd)
    dtype = torch.bfloat16 if precision == "bf16" else torch.float32
    rt = types.SimpleNamespace(dtype=dtype)
    x = torch.from_numpy(synth.normal((2, 5, D), 7, f"{tag}/x")).cuda().requires_grad_(True)
    gy = torch.from_numpy(synth.normal((2, 5, D), 7, f"{tag}/gy")).cuda()
    anchor = next(iter(mod.parameters()))
    y = T.AdapterFn.apply(x, anchor, rt, mod, True)
    y.float().backward(gy)
    torch.cuda.synchronize()
    tol = 1e-4 if precision == "fp32" else 5e-2

    def rel(a, b):
        return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-6))
    assert rel(y.detach().float().cpu().numpy(), g[f"{tag}_y"]) < tol
    assert rel(x.grad.float().cpu().numpy(), g[f"{tag}_gx"]) < tol
    for k, p in mod.named_parameters():
        assert rel(p.grad.cpu().numpy(), g[f"{tag}_g/{k}"]) < (tol if precision == "fp32" else 0.1), k


def _adapter_torch(x, sd, ln):
    """fp32 PyTorch restatement of TextAdapter.forward (adapter/clip_adapter.py:17-23)."""
    import torch.nn.functional as F
    h = F.gelu(F.linear(x, sd["down.weight"], sd["down.bias"]))
    z = F.linear(h, sd["up.weight"], sd["up.bias"]) + x
    return F.layer_norm(z, (x.shape[-1],), sd["ln.weight"], sd["ln.bias"], 1e-5) if ln else z


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("R,D,A,ln", [(1024, 768, 256, True), (1000, 1024, 256, True), (77, 512, 64, False),
                                      (1, 512, 256, True),
                                      # bottleneck / hidden widths that are not multiples of 8 (nn.Linear takes
                                      # any): fp32 runs them, bf16 (16-byte MFMA rows) refuses with ValueError
                                      (64, 768, 100, True), (33, 512, 99, True), (16, 100, 37, False)])
def test_adapter_fused_pooled_rows_matches_torch(dtype, R, D, A, ln):
    """clipmi_adapter_fwd / clipmi_adapter_bwd at the pooled-row sizes of the bench configs (R = the
    per-GPU batch, ragged R = 1000, a single row) vs an fp32 PyTorch autograd run of the same
    adapter on the same (storage-dtype-rounded) inputs; parameter gradients accumulate onto
    non-zero grads; a replay is bitwise equal (fixed-order sums, no split-K atomics).  Tolerance: max-relative 2e-5
    fp32, 3e-2 bf16 (storage rounding of pre / act / z)."""
    g = torch.Generator().manual_seed(R + D + A)
    mk = lambda *s, sc=1.0: (torch.randn(*s, generator=g) * sc).cuda().to(dtype)
    sd = {"down.weight": mk(A, D, sc=D ** -0.5), "down.bias": mk(A, sc=0.1), "up.weight": mk(D, A, sc=A ** -0.5),
          "up.bias": mk(D, sc=0.1), "ln.weight": mk(D, sc=0.2) + 1, "ln.bias": mk(D, sc=0.1)}
    x, dy = mk(R, D), mk(R, D)
    names = ["down.weight", "down.bias", "up.weight", "up.bias", "ln.weight", "ln.bias"]
    grads0 = {k: torch.randn(v.shape, generator=g).cuda() for k, v in sd.items()}
    dc, s = DT[dtype], kern.stream()

    def run():
        y = torch.empty(R, D, dtype=dtype, device="cuda")
        pre, act = (torch.empty(R, A, dtype=dtype, device="cuda") for _ in range(2))
        z = torch.empty(R, D, dtype=dtype, device="cuda")
        st = torch.empty(2, R, device="cuda")
        T.call("clipmi_adapter_fwd", s, dc, R, D, A, x.data_ptr(), D, *(sd[k].data_ptr() for k in names), 1e-5,
               int(ln), y.data_ptr(), D, pre.data_ptr(), act.data_ptr(), z.data_ptr(), st[0].data_ptr(),
               st[1].data_ptr())
        gr = {k: v.clone() for k, v in grads0.items()}
        dx = torch.empty(R, D, dtype=dtype, device="cuda")
        ws = T._ws(T._lib.lib().clipmi_adapter_bwd_ws(R, D, A), "cuda")
        T.call("clipmi_adapter_bwd", s, dc, R, D, A, dy.data_ptr(), D, x.data_ptr(), D, pre.data_ptr(),
               act.data_ptr(), z.data_ptr(), st[0].data_ptr(), st[1].data_ptr(), sd["down.weight"].data_ptr(),
               sd["up.weight"].data_ptr(), sd["ln.weight"].data_ptr(), int(ln), dx.data_ptr(), D,
               *(gr[k].data_ptr() for k in names), ws.data_ptr(), ws.numel())
        torch.cuda.synchronize()
        return y, dx, gr

    if dtype == torch.bfloat16 and (D % 8 or A % 8):
        with pytest.raises(ValueError, match="multiples of 8"):
            run()
        return
    y, dx, gr = run()
    y2, dx2, gr2 = run()
    assert torch.equal(y, y2) and torch.equal(dx, dx2) and all(torch.equal(gr[k], gr2[k]) for k in names)
    ref = {k: v.float().clone().requires_grad_(True) for k, v in sd.items()}
    xr = x.float().clone().requires_grad_(True)
    yr = _adapter_torch(xr, ref, ln)
    yr.backward(dy.float())
    tol = 2e-5 if dtype == torch.float32 else 3e-2
    assert rel(y, yr) < tol, "y"
    assert rel(dx, xr.grad) < tol, "dx"
    for k in names:
        if not ln and k.startswith("ln."):
            assert torch.equal(gr[k], grads0[k]), k  # untouched without the LayerNorm
            continue
        assert rel(gr[k] - grads0[k], ref[k].grad) < (tol if dtype == torch.float32 else 5e-2), k


@pytest.mark.parametrize("R,D,A", [(1024, 768, 256), (1000, 1024, 256), (33, 512, 512), (1, 512, 64), (300, 768, 128)])
def test_adapter_fwd_fused_kernel_matches_sequence(R, D, A, monkeypatch):
    """The bf16 adapter forward as one kernel (adapter_fused.hip: down GEMM + gelu, up GEMM + residual and the
    LayerNorm's row statistics as wavefront reductions in one workgroup) against the launch sequence it replaces
    (CLIPMI_ADAPTER_FUSED=0: down GEMM, up GEMM, LayerNorm): the same MFMA k-order, epilogue arithmetic and
    LayerNorm summation order, so pre / act / z / y / mean / rstd agree bit for bit (y and the statistics up to a
    last-bit difference in the odd element)."""
    g = torch.Generator().manual_seed(R + D + A + 7)
    mk = lambda *sh, sc=1.0: (torch.randn(*sh, generator=g) * sc).cuda().to(torch.bfloat16)
    names = ["down.weight", "down.bias", "up.weight", "up.bias", "ln.weight", "ln.bias"]
    sd = {"down.weight": mk(A, D, sc=D ** -0.5), "down.bias": mk(A, sc=0.1), "up.weight": mk(D, A, sc=A ** -0.5),
          "up.bias": mk(D, sc=0.1), "ln.weight": mk(D, sc=0.2) + 1, "ln.bias": mk(D, sc=0.1)}
    x = mk(R, D)
    s = kern.stream()
    outs = {}
    for fused in ("1", "0"):
        monkeypatch.setenv("CLIPMI_ADAPTER_FUSED", fused)
        y = torch.empty(R, D, dtype=torch.bfloat16, device="cuda")
        pre, act = (torch.empty(R, A, dtype=torch.bfloat16, device="cuda") for _ in range(2))
        z = torch.empty(R, D, dtype=torch.bfloat16, device="cuda")
        st = torch.empty(2, R, device="cuda")
        T.call("clipmi_adapter_fwd", s, BF16, R, D, A, x.data_ptr(), D, *(sd[k].data_ptr() for k in names), 1e-5, 1,
               y.data_ptr(), D, pre.data_ptr(), act.data_ptr(), z.data_ptr(), st[0].data_ptr(), st[1].data_ptr())
        torch.cuda.synchronize()
        outs[fused] = (pre, act, z, y, st)
    (p1, a1, z1, y1, s1), (p0, a0, z0, y0, s0) = outs["1"], outs["0"]
    neq = {k: int((u != v).sum()) for k, (u, v) in {"pre": (p1, p0), "act": (a1, a0), "z": (z1, z0), "y": (y1, y0),
                                                     "stats": (s1, s0)}.items()}
    print(f"\n[adapter fused vs sequence R={R} D={D} A={A}] differing elements {neq}")
    assert torch.equal(p1, p0) and torch.equal(a1, a0) and torch.equal(z1, z0)
    assert rel(y1, y0) < 1e-3 and rel(s1, s0) < 1e-6
    assert neq["y"] <= max(1, y1.numel() // 1000)


@pytest.mark.parametrize("B,N,H,causal", [(2, 577, 4, False), (3, 300, 2, True), (1, 1000, 2, False)])
def test_attention_fwd_mxfp8_output(B, N, H, causal):
    """clipmi_attention_fwd_mxfp8 (config 5's out-projection operand straight from the streaming
    forward) vs the same forward's bf16 output: the same lse bit for bit, every block's E8M0 scale by
    clipmi_quant_mxfp8's rule (a block max on a power-of-two boundary may land either side after the
    bf16 rounding of the comparison output) and every element within two e4m3 steps."""
    from clipmi import kernels as K
    D = H * 64
    qkv = rnd((B * N, 3 * D), 61, torch.bfloat16)
    mask = None
    if causal:
        g = torch.Generator().manual_seed(62)
        lens = torch.randint(5, N + 1, (B,), generator=g)
        mask = (torch.arange(N)[None] < lens[:, None]).to(torch.int64).cuda()
    mp = mask.data_ptr() if mask is not None else None
    s = kern.stream()
    o = torch.empty(B * N, D, dtype=torch.bfloat16, device="cuda")
    lse = torch.empty(B * H * N, device="cuda")
    q8 = torch.empty(B * N, D, dtype=torch.uint8, device="cuda")
    s8 = torch.empty(B * N, D // 32, dtype=torch.uint8, device="cuda")
    lse8 = torch.empty(B * H * N, device="cuda")
    import os
    old = os.environ.get("CLIPMI_ATTN_FA")
    os.environ["CLIPMI_ATTN_FA"] = "1"  # the same (streaming) kernel for the bf16 comparison
    try:
        T.call("clipmi_attention_fwd", s, DT[torch.bfloat16], qkv.data_ptr(), o.data_ptr(), lse.data_ptr(), mp,
               int(causal), B, H, N, D)
    finally:
        if old is None:
            del os.environ["CLIPMI_ATTN_FA"]
        else:
            os.environ["CLIPMI_ATTN_FA"] = old
    T.call("clipmi_attention_fwd_mxfp8", s, qkv.data_ptr(), q8.data_ptr(), s8.data_ptr(), lse8.data_ptr(), mp,
           int(causal), B, H, N, D)
    torch.cuda.synchronize()
    assert torch.equal(lse, lse8)
    ref = o.float()
    R = B * N
    amax = ref.abs().view(R, D // 32, 32).amax(-1)
    e = torch.ceil(torch.log2(amax / 448.0)).clamp(-127, 127)
    same = (s8.to(torch.int32) - 127 == e.to(torch.int32)).float().mean().item()
    assert same >= 0.99, same
    d = K.MX8(q8, s8).dequant()
    step = torch.pow(2.0, (s8.to(torch.float32) - 127) - 9).repeat_interleave(32, 1)
    err = (d - ref).abs() - (ref.abs() * (2.0 ** -3 + 2.0 ** -7) + 2 * step)
    assert (err <= 0).all(), err.max().item()


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_attention_online_softmax_rescale(dtype, monkeypatch):
    """cdna_hip_programming.md rule 26: force the deferred-max rescale branch of the streaming
    forward.  Key 400 (tile 6 of 64) gets a score ~40 log2-units above the others for every
    query, key 10 (tile 0) a moderate one; N = 577 runs the streamed kernels in both dtypes."""
    monkeypatch.setenv("CLIPMI_ATTN_FA", "1")
    B, N, H = 1, 577, 2
    D = H * 64
    qkv = rnd((B * N, 3 * D), 21, torch.float32)
    q = qkv[:, :D].view(N, H, 64)
    k = qkv[:, D:2 * D].view(N, H, 64)
    u = rnd((H, 64), 22, torch.float32)
    u = u / u.norm(dim=-1, keepdim=True)
    q += 3.0 * u          # every query shares a component along u
    k[400] = 30.0 * u     # scores ~ (3 + N(0,1)) * 3.75: ~15 log2 units above the rest
    k[10] = 10.0 * u      # a smaller bump in the first tile
    qkv = qkv.to(dtype).contiguous()
    o = torch.empty(B * N, D, dtype=dtype, device="cuda")
    lse = torch.empty(B * H * N, device="cuda")
    T.call("clipmi_attention_fwd", kern.stream(), DT[dtype], qkv.data_ptr(), o.data_ptr(), lse.data_ptr(), None, 0,
           B, H, N, D)
    oref, lref = attn_ref(qkv.float(), B, N, H, None, False)
    assert rel(o, oref) < TOL[dtype], "O"
    assert (lse - lref).abs().max().item() < (5e-2 if dtype == torch.bfloat16 else 1e-4), "lse"


@pytest.mark.parametrize("tag", ["land", "port", "pair", "up", "wide"])
def test_resize_u8_matches_processor(golden, tag):
    """clipmi_resize_u8 = CLIPImageProcessor's (PIL bicubic) shortest-edge resize, bit-exact."""
    from clipmi import towers as T
    g = golden("image_processor_resize.npz")
    imgs = torch.from_numpy(g[f"{tag}_images"]).cuda()
    oh, ow = T.shortest_edge_size(imgs.shape[1], imgs.shape[2], 224)
    out = T.resize_uint8(imgs, oh, ow)
    torch.cuda.synchronize()
    assert torch.equal(out.cpu(), torch.from_numpy(g[f"{tag}_resized"]))


def test_resize_u8_matches_oracle_random_sizes():
    """Odd sizes in both directions, batch of 3, against the PIL restatement."""
    from clipmi import towers as T
    from oracle import resize_ref as RR
    rng = np.random.default_rng(12)
    for h, w, oh, ow in [(64, 80, 64, 71), (33, 47, 224, 300), (500, 40, 17, 230), (9, 9, 5, 3), (77, 77, 77, 50)]:
        img = rng.integers(0, 256, (3, h, w, 3), dtype=np.uint8)
        out = T.resize_uint8(torch.from_numpy(img).cuda(), oh, ow).cpu().numpy()
        ref = np.stack([RR.resize_bicubic(im, oh, ow) for im in img])
        assert np.array_equal(out, ref), (h, w, oh, ow)


def test_gemm_batched_beyond_grid_z_limit():
    """clipmi_gemm_batched with nb1 * nb2 > 65535 (e.g. peclip's general head width at B = 8192 x 8 heads): the
    wrapper splits the batch over several launches (grid z is capped at 65535); every product vs torch."""
    nb1, nb2, M, N, K = 8500, 8, 5, 6, 7
    g = torch.Generator().manual_seed(3)
    A = torch.randn(nb1, nb2, M, K, generator=g).cuda()
    B = torch.randn(nb1, nb2, N, K, generator=g).cuda()
    C = torch.full((nb1, nb2, M, N), float("nan"), device="cuda")
    kern.gemm_batched(M, N, K, A, K, True, B, K, True, C, N, nb1, nb2, (nb2 * M * K, M * K), (nb2 * N * K, N * K),
                      (nb2 * M * N, M * N))
    ref = A @ B.transpose(-1, -2)
    assert rel(C, ref) < 2e-5


def test_layernorm_bwd_any_width_lds_grows():
    """ln_bwd_any_kernel's dynamic LDS (32 * D bytes with affine gradients) is opted in by the largest size asked
    so far: a small-D call first, then D = 4000 (125 KiB), both against torch."""
    for D in (96, 4000):
        R = 40
        x = rnd((R, D), D, torch.float32)
        w = rnd((D,), D + 1, torch.float32) * 0.2 + 1
        b = rnd((D,), D + 2, torch.float32) * 0.1
        dy = rnd((R, D), D + 3, torch.float32)
        y = torch.empty_like(x)
        st = torch.empty(2, R, device="cuda")
        s = kern.stream()
        T.call("clipmi_layernorm_fwd", s, F32, x.data_ptr(), D, y.data_ptr(), D, w.data_ptr(), b.data_ptr(),
               st[0].data_ptr(), st[1].data_ptr(), R, D, 1e-5, None, None, 0)
        dx = torch.empty_like(x)
        dw, db = torch.zeros(D, device="cuda"), torch.zeros(D, device="cuda")
        ws = T._ws(T._lib.lib().clipmi_layernorm_bwd_ws(R, D), "cuda")
        T.call("clipmi_layernorm_bwd", s, F32, dy.data_ptr(), D, x.data_ptr(), D, st[0].data_ptr(), st[1].data_ptr(),
               w.data_ptr(), dx.data_ptr(), D, None, 0, dw.data_ptr(), db.data_ptr(), 0, ws.data_ptr(), ws.numel(),
               R, D)
        xr, wr, br = (t.clone().requires_grad_(True) for t in (x, w, b))
        F.layer_norm(xr, (D,), wr, br, 1e-5).backward(dy)
        assert rel(dx, xr.grad) < 1e-4 and rel(dw, wr.grad) < 1e-4 and rel(db, br.grad) < 1e-4, D


@pytest.mark.parametrize("R,D", [(1000, 768), (77, 512), (5000, 768), (3, 1024)])
def test_layernorm_bwd_x3_writes_dx_image_and_colsum(R, D):
    """clipmi_layernorm_bwd_x3 (the bf16x3 engine's LayerNorm backwards since round 6): the fp32 backward with the
    residual gradient, plus dx's pattern-1 split image (bit for bit clipmi_split3_colsum's image of the fp32 dx) and
    dx's column sums added onto colsum (a Linear's bias gradient); dgamma / dbeta as the plain backward."""
    x = rnd((R, D), 51, torch.float32)
    w = rnd((D,), 52, torch.float32) * 0.2 + 1
    b = rnd((D,), 53, torch.float32) * 0.1
    dy = rnd((R, D), 54, torch.float32)
    dres = rnd((R, D), 55, torch.float32)
    y = torch.empty_like(x)
    st = torch.empty(2, R, device="cuda")
    s = kern.stream()
    T.call("clipmi_layernorm_fwd", s, F32, x.data_ptr(), D, y.data_ptr(), D, w.data_ptr(), b.data_ptr(),
           st[0].data_ptr(), st[1].data_ptr(), R, D, 1e-5, None, None, 0)
    dx = torch.empty_like(x)
    dw, db = torch.zeros(D, device="cuda"), torch.zeros(D, device="cuda")
    ws = T._ws(T._lib.lib().clipmi_layernorm_bwd_ws(R, D), "cuda")
    T.call("clipmi_layernorm_bwd", s, F32, dy.data_ptr(), D, x.data_ptr(), D, st[0].data_ptr(), st[1].data_ptr(),
           w.data_ptr(), dx.data_ptr(), D, dres.data_ptr(), D, dw.data_ptr(), db.data_ptr(), 0, ws.data_ptr(),
           ws.numel(), R, D)
    dx3 = torch.empty_like(x)
    dw3, db3 = torch.full((D,), 2.0, device="cuda"), torch.full((D,), 3.0, device="cuda")
    img = torch.full((R, 3 * D), float("nan"), dtype=torch.bfloat16, device="cuda")
    cs0 = rnd((D,), 56, torch.float32)
    cs = cs0.clone()
    ws3 = T._ws(T._lib.lib().clipmi_layernorm_bwd_x3_ws(R, D), "cuda")
    T.call("clipmi_layernorm_bwd_x3", s, dy.data_ptr(), D, x.data_ptr(), D, st[0].data_ptr(), st[1].data_ptr(),
           w.data_ptr(), dx3.data_ptr(), D, dres.data_ptr(), D, dw3.data_ptr(), db3.data_ptr(), 1, img.data_ptr(),
           cs.data_ptr(), 1, ws3.data_ptr(), ws3.numel(), R, D)
    assert torch.equal(dx3, dx)
    assert torch.equal(img, _split_ref(dx, 1))
    assert rel(dw3 - 2.0, dw) < 1e-6 and rel(db3 - 3.0, db) < 1e-6
    assert rel(cs - cs0, dx.double().sum(0)) < 1e-5


def _split_ref(x, pattern):
    """bf16x3 image of fp32 x [R, N]: [R, 3N] bf16, segments (h, h, l) (pattern 0) or (h, l, h) (pattern 1)."""
    h = x.to(torch.bfloat16)
    lo = (x - h.float()).to(torch.bfloat16)
    return torch.cat([h, h, lo] if pattern == 0 else [h, lo, h], dim=1)


@pytest.mark.parametrize("R,N", [(1000, 768), (77, 512), (5, 2304), (3, 3072)])
@pytest.mark.parametrize("pattern", [0, 1])
def test_split3_colsum_and_layernorm_x3(R, N, pattern):
    """The bf16x3 mode's producers: clipmi_split3_colsum writes the split image bit for bit (h = bf16(x),
    l = bf16(x - h)) and adds the column sums (the bias gradient) onto colsum; clipmi_layernorm_fwd_x3 writes the
    image of the fp32 LayerNorm output (== clipmi_layernorm_fwd's fp32 output, split)."""
    x = rnd((R, N), 7, torch.float32)
    out = torch.empty(R, 3 * N, dtype=torch.bfloat16, device="cuda")
    cs0 = rnd((N,), 8, torch.float32)
    cs = cs0.clone()
    ws = T._ws(T._lib.lib().clipmi_split3_colsum_ws(R, N), "cuda")
    s = kern.stream()
    T.call("clipmi_split3_colsum", s, x.data_ptr(), N, R, N, out.data_ptr(), pattern, cs.data_ptr(), 1,
           ws.data_ptr(), ws.numel())
    assert torch.equal(out, _split_ref(x, pattern))
    assert rel(cs - cs0, x.double().sum(0)) < 1e-5
    if N % 64 == 0 and N // 64 in (1, 2, 3, 4, 6, 8, 12, 16):
        w = rnd((N,), 9, torch.float32) * 0.2 + 1
        b = rnd((N,), 10, torch.float32) * 0.1
        y = torch.empty(R, N, device="cuda")
        st = torch.empty(2, R, device="cuda")
        T.call("clipmi_layernorm_fwd", s, F32, x.data_ptr(), N, y.data_ptr(), N, w.data_ptr(), b.data_ptr(),
               st[0].data_ptr(), st[1].data_ptr(), R, N, 1e-5, None, None, 0)
        y3 = torch.empty(R, 3 * N, dtype=torch.bfloat16, device="cuda")
        st3 = torch.empty(2, R, device="cuda")
        T.call("clipmi_layernorm_fwd_x3", s, x.data_ptr(), N, y3.data_ptr(), pattern, w.data_ptr(), b.data_ptr(),
               st3[0].data_ptr(), st3[1].data_ptr(), R, N, 1e-5)
        assert torch.equal(y3, _split_ref(y, pattern)) and torch.equal(st, st3)


@pytest.mark.parametrize("R,K,w4", [(600, 256, "1"), (520, 256, "1"), (777, 256, "1"), (777, 512, "1"),
                                    (777, 512, "0")])
def test_gemm_x3out_writes_the_split_image(R, K, w4, monkeypatch):
    """clipmi_gemm_x3out (the bf16x3 mode's fc1 forward and fc2 input gradient since round 6): the epilogue writes the
    split image of its fp32 result instead of the result -- equal to the fp32-output product split afterwards
    (clipmi_split3_colsum's rounding), with fc1's fp32 derivative beside it and the pattern-1 product's column sums
    (the bias gradient) added onto colsum.  R = 520 / 777: partial 256-row tiles, one with a wave wholly past M.
    Kernels: K' = 3K = 768 runs fc1 on the 8-wave kernel and fc2's input gradient on the persistent 4-wave one,
    K' = 1536 both on the 4-wave kernel, or both on the 8-wave one with CLIPMI_GEMM_X3_W4=0."""
    from clipmi import _lib
    monkeypatch.setenv("CLIPMI_GEMM_X3_W4", w4)
    N = 384
    s = kern.stream()
    x = rnd((R, K), 31, torch.float32)
    w = rnd((N, K), 32, torch.float32) * 0.05
    b = rnd((N,), 33, torch.float32) * 0.1
    x3 = torch.empty(R, 3 * K, dtype=torch.bfloat16, device="cuda")
    T.call("clipmi_split3", s, x.data_ptr(), K, R, K, 1, x3.data_ptr(), 0)
    w3 = torch.empty(N, 3 * K, dtype=torch.bfloat16, device="cuda")
    T.call("clipmi_split3", s, w.data_ptr(), K, N, K, 1, w3.data_ptr(), 1)
    fl = _lib.EPI_BIAS | _lib.EPI_QGELU | _lib.EPI_STORE_DACT
    assert T._lib.lib().clipmi_gemm_x3out_ok(R, N, 3 * K, 1, 1, fl)
    y = torch.empty(R, N, device="cuda")
    dact = torch.empty(R, N, device="cuda")
    kern.gemm(R, N, 3 * K, x3, 3 * K, True, w3, 3 * K, True, y, N, bias=b, aux=dact, ldaux=N, flags=fl)
    img = torch.full((R, 3 * N), float("nan"), dtype=torch.bfloat16, device="cuda")
    dact2 = torch.empty(R, N, device="cuda")
    kern.gemm_x3out(R, N, 3 * K, x3, 3 * K, w3, 3 * K, True, img, 0, bias=b, aux=dact2, ldaux=N, flags=fl)
    ref = _split_ref(y, 0)
    assert torch.equal(img[:, :N], img[:, N:2 * N])
    hl = img[:, :N].float() + img[:, 2 * N:].float()
    # h + l keeps ~16 of fp32's 24 bits (2^-17 relative); the image is bit for bit the split of the fp32 product
    mh = (img[:, :N] != ref[:, :N]).float().mean().item()
    ml = (img[:, 2 * N:] != ref[:, 2 * N:]).float().mean().item()
    print(f"\n[x3out fc1 R={R} K={K} w4={w4}] h mismatch {mh:.2e}, l mismatch {ml:.2e}, rel(h + l, y) {rel(hl, y):.2e}")
    assert rel(hl, y) < 2e-5 and torch.equal(img, ref)
    assert rel(dact2, dact) < 1e-6
    # fc2's input gradient: d_pre = (dy W2) * dact, pattern 1, bias gradient of fc1 from its column sums
    dy = rnd((R, K), 34, torch.float32)
    dy3 = torch.empty(R, 3 * K, dtype=torch.bfloat16, device="cuda")
    T.call("clipmi_split3", s, dy.data_ptr(), K, R, K, 1, dy3.data_ptr(), 1)
    w2 = rnd((K, N), 35, torch.float32) * 0.05  # fc2 weight [out K][in N]
    ld8 = (N + 7) // 8 * 8
    w23 = torch.zeros(3 * K, ld8, dtype=torch.bfloat16, device="cuda")
    T.call("clipmi_split3", s, w2.data_ptr(), N, N, K, 0, w23.data_ptr(), 0)
    g = torch.empty(R, N, device="cuda")
    kern.gemm(R, N, 3 * K, dy3, 3 * K, True, w23, ld8, False, g, N, aux=dact, ldaux=N, flags=_lib.EPI_MUL_AUX)
    assert rel(g, (dy.double() @ w2.double()) * dact.double()) < 1e-4
    gimg = torch.full((R, 3 * N), float("nan"), dtype=torch.bfloat16, device="cuda")
    cs0 = rnd((N,), 36, torch.float32)
    cs = cs0.clone()
    kern.gemm_x3out(R, N, 3 * K, dy3, 3 * K, w23, ld8, False, gimg, 1, aux=dact, ldaux=N, flags=_lib.EPI_MUL_AUX,
                    colsum=cs)
    assert torch.equal(gimg[:, :N], gimg[:, 2 * N:])
    hl = gimg[:, :N].float() + gimg[:, N:2 * N].float()
    gref = _split_ref(g, 1)
    mh = (gimg[:, :N] != gref[:, :N]).float().mean().item()
    ml = (gimg[:, N:2 * N] != gref[:, N:2 * N]).float().mean().item()
    print(f"[x3out fc2 dgrad R={R} K={K} w4={w4}] h mismatch {mh:.2e}, l mismatch {ml:.2e}, rel(h + l, g) {rel(hl, g):.2e}")
    assert rel(hl, g) < 2e-5 and torch.equal(gimg, gref)
    assert rel(cs - cs0, g.double().sum(0)) < 1e-5
    cs1 = torch.zeros(N, device="cuda")
    kern.gemm_x3out(R, N, 3 * K, dy3, 3 * K, w23, ld8, False, gimg, 1, aux=dact, ldaux=N, flags=_lib.EPI_MUL_AUX,
                    colsum=cs1, beta=False)
    assert rel(cs1, g.double().sum(0)) < 1e-5
    # shapes / flags without the fused form are refused (the engine checks clipmi_gemm_x3out_ok first)
    assert not T._lib.lib().clipmi_gemm_x3out_ok(200, N, 3 * K, 1, 1, fl)
    assert not T._lib.lib().clipmi_gemm_x3out_ok(R, N, 3 * K, 1, 1, _lib.EPI_BIAS)
    with pytest.raises(ValueError, match="x3out"):
        kern.gemm_x3out(200, N, 3 * K, x3, 3 * K, w3, 3 * K, True, img, 0, bias=b, aux=dact2, ldaux=N, flags=fl)


def test_gemm_over_split_images_matches_split3_flag():
    """A bf16 GEMM over pre-split images (the engine's bf16x3 path since round 6) -- forward (k-major images,
    reduction 3K) and weight gradient (images read as [3R][K], reduction over 3R interleaved rows) -- against
    the CLIPMI_GEMM_SPLIT3 flag's split-per-call product and fp64."""
    from clipmi import _lib
    R, K, N = 600, 256, 384
    x = rnd((R, K), 21, torch.float32)
    w = rnd((N, K), 22, torch.float32) * 0.05
    s = kern.stream()
    x3 = torch.empty(R, 3 * K, dtype=torch.bfloat16, device="cuda")
    T.call("clipmi_split3", s, x.data_ptr(), K, R, K, 1, x3.data_ptr(), 0)
    assert torch.equal(x3, _split_ref(x, 0))
    w3 = torch.empty(N, 3 * K, dtype=torch.bfloat16, device="cuda")
    T.call("clipmi_split3", s, w.data_ptr(), K, N, K, 1, w3.data_ptr(), 1)
    y = torch.empty(R, N, device="cuda")
    kern.gemm(R, N, 3 * K, x3, 3 * K, True, w3, 3 * K, True, y, N)
    y_flag = torch.empty(R, N, device="cuda")
    kern.gemm(R, N, K, x, K, True, w, K, True, y_flag, N, split3=True)
    ref = x.double() @ w.double().T
    assert rel(y, ref) < 1e-4 and rel(y, y_flag) < 1e-5
    # weight gradient: gW[N][K] = sum_r dy[r][n] x[r][k] from a pattern-1 image of dy and the pattern-0 image of x
    dy = rnd((R, N), 23, torch.float32)
    dy3 = _split_ref(dy, 1).contiguous()
    gw = torch.zeros(N, K, device="cuda")
    kern.gemm(N, K, 3 * R, dy3, N, False, x3, K, False, gw, K, flags=_lib.EPI_BETA)
    assert rel(gw, dy.double().T @ x.double()) < 1e-4

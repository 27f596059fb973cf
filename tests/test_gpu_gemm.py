"""GEMM parity: libclipmi MFMA/f32 GEMM vs a plain PyTorch fp32 matmul (all 4 operand
layouts, tails, every epilogue flag, split-K)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

from clipmi import _lib  # noqa: E402
from clipmi import kernels as kern  # noqa: E402


def _mk(shape, dtype, seed):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return torch.randn(*shape, generator=g).to("cuda", dtype)


def _ref_epi(acc, flags, bias=None, aux=None, res=None, cold=None, alpha=1.0):
    v = acc * alpha
    if flags & _lib.EPI_BIAS:
        v = v + bias.float()
    pre = v.clone()
    if flags & _lib.EPI_STORE_DACT:  # the activation's derivative at the pre-activation -> aux
        if flags & _lib.EPI_QGELU:
            sg = torch.sigmoid(1.702 * v)
            pre = sg + 1.702 * v * sg * (1 - sg)
        else:
            pre = 0.5 * (1 + torch.erf(v / 2 ** 0.5)) + v * torch.exp(-0.5 * v * v) / (2 * torch.pi) ** 0.5
    if flags & _lib.EPI_QGELU:
        v = v * torch.sigmoid(1.702 * v)
    if flags & _lib.EPI_GELU:
        v = torch.nn.functional.gelu(v)
    if flags & _lib.EPI_DQGELU:
        a = aux.float()
        s = torch.sigmoid(1.702 * a)
        v = v * (s + 1.702 * a * s * (1 - s))
    if flags & _lib.EPI_MUL_AUX:
        v = v * aux.float()
    if flags & _lib.EPI_RESID:
        v = v + res.float()
    if flags & _lib.EPI_BETA:
        v = v + cold.float()
    return v, pre


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("akm,bkm", [(True, True), (True, False), (False, True), (False, False)])
# production schedule, 128 tile, single-group 256, half-tile pipeline
@pytest.mark.parametrize("small", [0, 1, 4, 11])
@pytest.mark.parametrize("M,N,K", [(256, 256, 128), (200, 136, 72), (77, 64, 768), (1000, 512, 200),
                                   (1000, 776, 768), (600, 264, 1000), (512, 256, 64), (520, 384, 96),
                                   (768, 256, 4160)])
def test_gemm_layouts(dtype, akm, bkm, M, N, K, small):
    if dtype == torch.float32 and small:
        pytest.skip("tile choice only applies to the bf16 path")
    if dtype == torch.bfloat16 and (not akm) and M % 8:
        pytest.skip("row-major A needs M % 8 == 0")
    if dtype == torch.bfloat16 and (akm or bkm) and K % 8:
        pytest.skip("k-major needs K % 8 == 0")
    A = _mk((M, K) if akm else (K, M), dtype, 1)
    B = _mk((N, K) if bkm else (K, N), dtype, 2)
    C = torch.empty(M, N, device="cuda", dtype=torch.float32)
    if dtype == torch.bfloat16 and (not bkm) and N % 8:
        pytest.skip("row-major B needs N % 8 == 0")
    kern.gemm(M, N, K, A, A.stride(0), akm, B, B.stride(0), bkm, C, N, small_tile=small)
    Af = (A if akm else A.t()).float()
    Bf = (B if bkm else B.t()).float()
    ref = Af @ Bf.t()
    torch.cuda.synchronize()
    tol = 1e-3 if dtype == torch.float32 else 2e-2
    err = (C - ref).abs().max().item() / max(1.0, ref.abs().max().item())
    assert err < tol, err


@pytest.mark.parametrize("flags", [
    _lib.EPI_BIAS, _lib.EPI_BIAS | _lib.EPI_QGELU | _lib.EPI_STORE_PRE, _lib.EPI_BIAS | _lib.EPI_GELU,
    _lib.EPI_BIAS | _lib.EPI_RESID, _lib.EPI_DQGELU, _lib.EPI_BETA,
    _lib.EPI_BIAS | _lib.EPI_QGELU | _lib.EPI_STORE_DACT, _lib.EPI_BIAS | _lib.EPI_GELU | _lib.EPI_STORE_DACT,
    _lib.EPI_MUL_AUX])
@pytest.mark.parametrize("cdtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("small", [0, 11])
def test_gemm_epilogues(flags, cdtype, small):
    M, N, Kd = 300, 192, 256
    A = _mk((M, Kd), torch.bfloat16, 3)
    B = _mk((N, Kd), torch.bfloat16, 4)
    bias = _mk((N,), torch.float32, 5)
    aux = _mk((M, N), cdtype, 6)
    res = _mk((M, N), cdtype, 7)
    C = _mk((M, N), cdtype, 8)
    cold = C.clone()
    aux_in = aux.clone()
    kern.gemm(M, N, Kd, A, Kd, True, B, Kd, True, C, N, bias=bias, residual=res, ldr=N, aux=aux, ldaux=N,
              alpha=0.5, flags=flags, small_tile=small)
    acc = A.float() @ B.float().t()
    ref, pre = _ref_epi(acc, flags, bias, aux_in, res, cold, alpha=0.5)
    torch.cuda.synchronize()
    tol = 3e-2 if cdtype == torch.bfloat16 else 1e-2
    assert (C.float() - ref).abs().max().item() / max(1.0, ref.abs().max().item()) < tol
    if flags & (_lib.EPI_STORE_PRE | _lib.EPI_STORE_DACT):
        assert (aux.float() - pre).abs().max().item() / max(1.0, pre.abs().max().item()) < tol


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_gemm_splitk_wgrad(dtype):
    # dW[n_out][k_in] = sum_tokens dY[t][n_out] X[t][k_in]: both operands row-major in k
    T, Nout, Kin = 3000, 256, 192
    dY = _mk((T, Nout), dtype, 9)
    X = _mk((T, Kin), dtype, 10)
    C = _mk((Nout, Kin), torch.float32, 11)
    c0 = C.clone()
    ws = torch.empty(8 * Nout * Kin, device="cuda", dtype=torch.float32)
    kern.gemm(Nout, Kin, T, dY, Nout, False, X, Kin, False, C, Kin, flags=_lib.EPI_BETA, split_k=8, workspace=ws)
    ref = c0 + dY.float().t() @ X.float()
    torch.cuda.synchronize()
    assert (C - ref).abs().max().item() / ref.abs().max().item() < (1e-4 if dtype == torch.float32 else 1e-2)


@pytest.mark.parametrize("T,Nout,Kin,split", [(3000, 256, 192, 8), (50000, 768, 3072, 12), (77, 64, 128, 1),
                                              (20000, 2304, 768, 4), (300, 768, 768, 3), (4100, 512, 256, 2)])
def test_wgrad_fused_bias_grad(T, Nout, Kin, split):
    """256 wgrad kernel with the fused bias gradient (sum over tokens of dY); split-K bias partials
    are summed in split order, so a second run gives bitwise the same bias gradient."""
    dY = _mk((T, Nout), torch.bfloat16, 12)
    X = _mk((T, Kin), torch.bfloat16, 13)
    C = _mk((Nout, Kin), torch.float32, 14)
    db = _mk((Nout,), torch.float32, 15)
    c0, db0 = C.clone(), db.clone()
    ws = torch.empty(max(1, split) * Nout * (Kin + 1), device="cuda", dtype=torch.float32)  # + bias partials
    kern.gemm(Nout, Kin, T, dY, Nout, False, X, Kin, False, C, Kin, flags=_lib.EPI_BETA, split_k=split,
              workspace=ws, bias_grad=db)
    ref = c0 + dY.float().t() @ X.float()
    dref = db0 + dY.float().sum(0)
    db2 = db0.clone()
    kern.gemm(Nout, Kin, T, dY, Nout, False, X, Kin, False, C.clone(), Kin, flags=_lib.EPI_BETA, split_k=split,
              workspace=ws, bias_grad=db2)
    torch.cuda.synchronize()
    assert torch.equal(db2, db)
    torch.cuda.synchronize()
    assert (C - ref).abs().max().item() / ref.abs().max().item() < 1e-2
    assert (db - dref).abs().max().item() / dref.abs().max().item() < 1e-3


# ------------------------------------------------------------------ MXFP8 (config 5)
def _mx8_exact(R, K, seed):
    """Small integers (exact in e4m3) with random E8M0 block scales 2^-2 .. 2^3."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    v = torch.randint(-8, 9, (R, K), generator=g).float()
    s = torch.randint(125, 131, (R, K // 32), generator=g).to(torch.uint8)
    q = v.to(torch.float8_e4m3fn).view(torch.uint8)
    return kern.MX8(q.cuda(), s.cuda())


@pytest.mark.parametrize("M,N,K", [(256, 256, 128), (300, 520, 256), (1024, 768, 1024), (77, 64, 640),
                                   (256, 256, 384), (2304, 1280, 4096), (1000, 1100, 768), (4096, 512, 2048)])
@pytest.mark.parametrize("variant", [0, 40, 41])
def test_gemm_fp8_block_scaled_exact(M, N, K, variant):
    """v_mfma_scale_f32_32x32x64_f8f6f4 GEMMs (0: production dispatch; 40: the 8-wave kernel everywhere;
    41: the persistent 4-wave kernel wherever K % 256 == 0 and M, N >= 256): integer operands and power-of-two
    block scales make every product and sum exact in fp32, so the result must equal the dequantised
    product exactly (checks the fp8 fragment map and which lanes' scale bytes apply to which k-blocks)."""
    A, B = _mx8_exact(M, K, 1), _mx8_exact(N, K, 2)
    C = torch.empty(M, N, device="cuda", dtype=torch.float32)
    kern.gemm_fp8(M, N, K, A, B, C, N, variant=variant)
    ref = A.dequant() @ B.dequant().t()
    torch.cuda.synchronize()
    assert torch.equal(C, ref), (C - ref).abs().max().item()


@pytest.mark.parametrize("flags", [0, _lib.EPI_BIAS, _lib.EPI_BIAS | _lib.EPI_RESID, _lib.EPI_BIAS | _lib.EPI_QGELU])
@pytest.mark.parametrize("variant", [0, 40, 41])
def test_gemm_fp8_epilogues(flags, variant):
    M, N, K = 600, 384, 512
    x = _mk((M, K), torch.bfloat16, 21)
    w = _mk((N, K), torch.bfloat16, 22) * 0.05
    A, B = kern.quant_mxfp8(x), kern.quant_mxfp8(w.contiguous())
    bias = _mk((N,), torch.bfloat16, 23)
    res = _mk((M, N), torch.bfloat16, 24)
    C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    kern.gemm_fp8(M, N, K, A, B, C, N, bias=bias, residual=res, ldr=N, flags=flags, variant=variant)
    acc = A.dequant() @ B.dequant().t()
    ref, _ = _ref_epi(acc, flags, bias, None, res)
    torch.cuda.synchronize()
    assert (C.float() - ref).abs().max().item() / max(1.0, ref.abs().max().item()) < 2e-2


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_quant_mxfp8_roundtrip(dtype):
    """Per 32-element block: scale = the smallest power of two bringing max|x| to <= 448; every
    element within e4m3's rounding (2^-4 relative, or the block's subnormal step)."""
    R, K = 97, 1024
    g = torch.Generator(device="cpu").manual_seed(5)
    x = (torch.randn(R, K, generator=g) * torch.exp(torch.randn(R, K // 32, generator=g) * 3).repeat_interleave(32, 1))
    x = x.to(dtype).cuda()
    m = kern.quant_mxfp8(x)
    d = m.dequant()
    xf = x.float()
    amax = xf.abs().view(R, K // 32, 32).amax(-1)
    e = torch.ceil(torch.log2(amax / 448.0))
    assert torch.equal(m.s.to(torch.int32) - 127, e.to(torch.int32))
    step = torch.pow(2.0, e - 9).repeat_interleave(32, 1)
    assert ((d - xf).abs() <= xf.abs() * 2.0 ** -4 + step).all()


def _mx_close(m, ref, frac=0.99):
    """MXFP8 m vs the fp32 values ref it should encode: the block scales equal ref's exact rule
    (ceil(log2(amax / 448))) for nearly every block (an amax on a power-of-two boundary may round
    either way after a different fp32 summation order) and every element within two e4m3 steps."""
    R, K = ref.shape
    amax = ref.abs().view(R, K // 32, 32).amax(-1)
    e = torch.ceil(torch.log2(amax / 448.0)).clamp(-127, 127)
    same = (m.s.to(torch.int32) - 127 == e.to(torch.int32)).float().mean().item()
    assert same >= frac, same
    d = m.dequant()
    step = torch.pow(2.0, e - 9).repeat_interleave(32, 1)
    err = (d - ref).abs() - (ref.abs() * 2.0 ** -3 + 2 * step)
    assert (err <= 0).all(), err.max().item()


@pytest.mark.parametrize("variant", [0, 40, 41])
def test_gemm_fp8_mxfp8_output(variant):
    """fc1's fused epilogue in the fp8 towers: bias + quick_gelu, written as MXFP8 [M, N] + scales."""
    M, N, K = 600, 512, 512
    x = _mk((M, K), torch.bfloat16, 31)
    w = _mk((N, K), torch.bfloat16, 32) * 0.05
    A, B = kern.quant_mxfp8(x), kern.quant_mxfp8(w.contiguous())
    bias = _mk((N,), torch.bfloat16, 33)
    C = kern.MX8(torch.empty(M, N, dtype=torch.uint8, device="cuda"),
                 torch.empty(M, N // 32, dtype=torch.uint8, device="cuda"))
    flags = _lib.EPI_BIAS | _lib.EPI_QGELU
    kern.gemm_fp8(M, N, K, A, B, C, N, bias=bias, flags=flags, variant=variant)
    acc = A.dequant() @ B.dequant().t()
    ref, _ = _ref_epi(acc, flags, bias, None, None)
    torch.cuda.synchronize()
    _mx_close(C, ref)


def test_gemm_fp8_mxfp8_output_rejects_residual():
    M, N, K = 256, 256, 128
    A, B = _mx8_exact(M, K, 1), _mx8_exact(N, K, 2)
    C = kern.MX8(torch.empty(M, N, dtype=torch.uint8, device="cuda"),
                 torch.empty(M, N // 32, dtype=torch.uint8, device="cuda"))
    res = torch.zeros(M, N, dtype=torch.bfloat16, device="cuda")
    with pytest.raises(ValueError):
        kern.gemm_fp8(M, N, K, A, B, C, N, residual=res, ldr=N, flags=_lib.EPI_RESID)


@pytest.mark.parametrize("R,D", [(1000, 1024), (77, 768), (4, 512)])
def test_layernorm_mxfp8(R, D):
    """clipmi_layernorm_fwd_mxfp8 = LayerNorm in fp32, quantised like clipmi_quant_mxfp8."""
    x = _mk((R, D), torch.bfloat16, 41) * 3
    w = (1 + 0.1 * _mk((D,), torch.bfloat16, 42)).to(torch.bfloat16)
    b = (0.1 * _mk((D,), torch.bfloat16, 43)).to(torch.bfloat16)
    m, mean, rstd = kern.layernorm_mxfp8(x, w, b, 1e-5)
    ref = torch.nn.functional.layer_norm(x.float(), (D,), w.float(), b.float(), 1e-5)
    torch.cuda.synchronize()
    _mx_close(m, ref)
    assert torch.allclose(mean, x.float().mean(1), atol=1e-4)


@pytest.mark.parametrize("var", [28, 32])
@pytest.mark.parametrize("bkm,flags", [
    (True, _lib.EPI_BIAS), (True, _lib.EPI_BIAS | _lib.EPI_RESID),
    (True, _lib.EPI_BIAS | _lib.EPI_QGELU | _lib.EPI_STORE_PRE), (True, _lib.EPI_BIAS | _lib.EPI_QGELU), (True, 0),
    (False, 0), (False, _lib.EPI_DQGELU),
    (True, _lib.EPI_BIAS | _lib.EPI_QGELU | _lib.EPI_STORE_DACT), (False, _lib.EPI_MUL_AUX)])
@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (1000, 776, 768), (520, 384, 128), (300, 264, 192),
                                   (2048, 512, 3072)])
def test_gemm_4wave_matches_pingpong(var, bkm, flags, M, N, K):
    """Persistent 4-wave 256x256 kernel (gemm4.hip, 128x128 per wave; 31: counted item-start wait)
    against the 8-wave ping-pong kernel forced for every shape (variant 9: production would send the
    K >= 1536 and MUL_AUX rows to the 4-wave kernel itself): the same k order of MFMA accumulation,
    so bitwise-equal outputs (and pre-activations / derivatives); also within bf16 rounding of a
    torch fp32 reference."""
    A = _mk((M, K), torch.bfloat16, 11)
    B = _mk((N, K) if bkm else (K, N), torch.bfloat16, 12)
    bias = _mk((N,), torch.bfloat16, 13)
    res = _mk((M, N), torch.bfloat16, 14)
    aux0 = _mk((M, N), torch.bfloat16, 15)
    outs = []
    for v in (9, var):
        C = torch.zeros(M, N, device="cuda", dtype=torch.bfloat16)
        aux = aux0.clone()
        kern.gemm(M, N, K, A, K, True, B, B.stride(0), bkm, C, N, bias=bias, residual=res, ldr=N, aux=aux, ldaux=N,
                  flags=flags, small_tile=v)
        outs.append((C, aux))
    torch.cuda.synchronize()
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1])
    acc = A.float() @ (B.float().t() if bkm else B.float())
    ref, _ = _ref_epi(acc, flags, bias, aux0, res)
    assert (outs[1][0].float() - ref).abs().max().item() / max(1.0, ref.abs().max().item()) < 3e-2


@pytest.mark.parametrize("T,Nout,Kin,split", [(3000, 256, 192, 8), (50000, 768, 3072, 12), (77, 64, 128, 1),
                                              (20000, 2304, 768, 4), (300, 768, 768, 3), (4100, 520, 264, 2),
                                              (9000, 768, 768, 1)])
@pytest.mark.parametrize("bias", [False, True])
@pytest.mark.parametrize("var", [28])
def test_wgrad_4wave_matches_8wave(T, Nout, Kin, split, bias, var):
    """Weight gradient on the persistent 4-wave kernel (gemm4.hip, variant 28) vs the 8-wave wgrad
    kernel (variant 4): the same k order of MFMA accumulation per output element, so bitwise-equal
    slabs / beta outputs and bias gradients; and within bf16-product rounding of torch fp32."""
    dY = _mk((T, Nout), torch.bfloat16, 21)
    X = _mk((T, Kin), torch.bfloat16, 22)
    C0 = _mk((Nout, Kin), torch.float32, 23)
    db0 = _mk((Nout,), torch.float32, 24)
    outs = []
    for v in (4, var):
        C, db = C0.clone(), db0.clone()
        ws = torch.empty(max(1, split) * Nout * (Kin + 1), device="cuda", dtype=torch.float32)
        kern.gemm(Nout, Kin, T, dY, Nout, False, X, Kin, False, C, Kin, flags=_lib.EPI_BETA, split_k=split,
                  workspace=ws if split > 1 else None, bias_grad=db if bias else None, small_tile=v)
        outs.append((C, db))
    torch.cuda.synchronize()
    assert torch.equal(outs[0][0], outs[1][0])
    if bias:
        assert torch.equal(outs[0][1], outs[1][1])
    ref = C0 + dY.float().t() @ X.float()
    assert (outs[1][0] - ref).abs().max().item() / ref.abs().max().item() < 1e-2


@pytest.mark.parametrize("raster", ["0", "4", "8"])
@pytest.mark.parametrize("var", [9, 28])
def test_gemm_raster_groups_bitwise(raster, var, monkeypatch):
    """CLIPMI_RASTER (tile-rows per rasterisation group) only reorders the tiles: every output
    element keeps its k order, so the result is bitwise equal to row-major order (both the 8-wave
    and the persistent 4-wave kernel; 3000 rows = 12 ragged tile-rows)."""
    M, N, K = 3000, 776, 768
    A = _mk((M, K), torch.bfloat16, 51)
    B = _mk((N, K), torch.bfloat16, 52)
    bias = _mk((N,), torch.bfloat16, 53)
    outs = []
    for r in ("0", raster):
        monkeypatch.setenv("CLIPMI_RASTER", r)
        C = torch.zeros(M, N, device="cuda", dtype=torch.bfloat16)
        kern.gemm(M, N, K, A, K, True, B, K, True, C, N, bias=bias, flags=_lib.EPI_BIAS, small_tile=var)
        outs.append(C)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])


# ---- bf16x3 split-operand fp32 GEMM (CLIPMI_GEMM_SPLIT3, precision "bf16x3")
@pytest.mark.parametrize("akm,bkm,flags,split", [
    (True, True, 0, 1), (True, True, _lib.EPI_BIAS, 1), (True, True, _lib.EPI_BIAS | _lib.EPI_RESID, 1),
    (True, True, _lib.EPI_BIAS | _lib.EPI_QGELU | _lib.EPI_STORE_DACT, 1), (True, True, _lib.EPI_BIAS | _lib.EPI_QGELU, 1),
    (True, False, 0, 1), (True, False, _lib.EPI_MUL_AUX, 1),
    (False, False, _lib.EPI_BETA, 1), (False, False, _lib.EPI_BETA, 5), (False, True, 0, 1)])
@pytest.mark.parametrize("M,N,K", [(1000, 776, 768), (520, 384, 3072), (77, 64, 128), (2048, 256, 512)])
def test_gemm_split3_fp32_accuracy(akm, bkm, flags, split, M, N, K):
    """fp32 operands through the bf16x3 split product: against an fp64 reference the error is ~2^-16
    relative per product (the dropped lo x lo term plus fp32 accumulation), 30x+ below a plain bf16
    product of the same operands, on every layout / epilogue the bf16x3 mode issues."""
    if not akm and M % 8:
        pytest.skip("row-major A needs M % 8 == 0")
    A = _mk((M, K) if akm else (K, M), torch.float32, 1)
    B = _mk((N, K) if bkm else (K, N), torch.float32, 2)
    Ad = (A if akm else A.t()).double()
    Bd = (B if bkm else B.t()).double()
    acc = Ad @ Bd.t()
    bias, res, aux = _mk((N,), torch.float32, 3), _mk((M, N), torch.float32, 4), None
    cold = _mk((M, N), torch.float32, 5)
    if flags & _lib.EPI_MUL_AUX:
        aux = _mk((M, N), torch.float32, 6)
    elif flags & _lib.EPI_STORE_DACT:
        aux = torch.zeros(M, N, device="cuda")
    C = cold.clone() if flags & _lib.EPI_BETA else torch.empty(M, N, device="cuda")
    kern.gemm(M, N, K, A, K if akm else M, akm, B, K if bkm else N, bkm, C, N, bias=bias if flags & _lib.EPI_BIAS else None,
              residual=res if flags & _lib.EPI_RESID else None, ldr=N if flags & _lib.EPI_RESID else 0,
              aux=aux, ldaux=N if aux is not None else 0, flags=flags, split_k=split, split3=True)
    ref, pre = _ref_epi(acc, flags, bias.double(), None if aux is None else aux.double(), res.double(),
                        cold.double())
    scale = acc.abs().max().item()
    err = (C.double() - ref).abs().max().item() / scale
    # the same product with bf16-rounded operands: the precision bf16x3 buys back
    e16 = (((A.bfloat16().double() if akm else A.t().bfloat16().double()) @
            (B.bfloat16().double() if bkm else B.t().bfloat16().double()).t()) - acc).abs().max().item() / scale
    assert err < 2e-5 and err * 30 < e16, (err, e16)
    if flags & _lib.EPI_STORE_DACT:
        # quick_gelu'(v) at the computed pre-activation: v carries err * scale absolute error (scale ~ 130
        # here) and |quick_gelu''| < 1, plus the kernel's fast exp: measured 3.8e-4
        assert ((aux.double() - pre).abs().max().item()) < 2e-3


def test_gemm_split3_rejects_bad_workspace_and_bias_grad():
    A, B = _mk((256, 256), torch.float32, 1), _mk((256, 256), torch.float32, 2)
    C = torch.empty(256, 256, device="cuda")
    with pytest.raises(ValueError, match="split3"):
        kern.gemm(256, 256, 256, A, 256, False, B, 256, False, C, 256, flags=_lib.EPI_BETA,
                  bias_grad=torch.zeros(256, device="cuda"), split3=True)
    with pytest.raises(ValueError, match="workspace"):
        kern.gemm(256, 256, 256, A, 256, True, B, 256, True, C, 256, flags=_lib.GEMM_SPLIT3,
                  workspace=torch.empty(1024, dtype=torch.uint8, device="cuda"))


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
    if flags & _lib.EPI_QGELU:
        v = v * torch.sigmoid(1.702 * v)
    if flags & _lib.EPI_GELU:
        v = torch.nn.functional.gelu(v)
    if flags & _lib.EPI_DQGELU:
        a = aux.float()
        s = torch.sigmoid(1.702 * a)
        v = v * (s + 1.702 * a * s * (1 - s))
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
    _lib.EPI_BIAS | _lib.EPI_RESID, _lib.EPI_DQGELU, _lib.EPI_BETA])
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
    if flags & _lib.EPI_STORE_PRE:
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
    """256 wgrad kernel with the fused bias gradient (sum over tokens of dY)."""
    dY = _mk((T, Nout), torch.bfloat16, 12)
    X = _mk((T, Kin), torch.bfloat16, 13)
    C = _mk((Nout, Kin), torch.float32, 14)
    db = _mk((Nout,), torch.float32, 15)
    c0, db0 = C.clone(), db.clone()
    ws = torch.empty(max(1, split) * Nout * Kin, device="cuda", dtype=torch.float32)
    kern.gemm(Nout, Kin, T, dY, Nout, False, X, Kin, False, C, Kin, flags=_lib.EPI_BETA, split_k=split,
              workspace=ws, bias_grad=db)
    ref = c0 + dY.float().t() @ X.float()
    dref = db0 + dY.float().sum(0)
    torch.cuda.synchronize()
    assert (C - ref).abs().max().item() / ref.abs().max().item() < 1e-2
    assert (db - dref).abs().max().item() / dref.abs().max().item() < 1e-3

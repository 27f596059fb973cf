"""Thin tensor-level wrappers over the libclipmi C ABI.

Every function enqueues on torch's current HIP stream and never synchronises.  Shapes
are validated here and again in C; tensors must live on the GPU (the product path has
no CPU fallback)."""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from ._lib import BF16, F32, FP8, GemmDesc

_DT = {torch.float32: F32, torch.bfloat16: BF16}


def dt(t: torch.Tensor) -> int:
    try:
        return _DT[t.dtype]
    except KeyError:
        raise ValueError(f"unsupported dtype {t.dtype}") from None


def ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _on_gpu(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise ValueError("libclipmi ops need GPU tensors (no CPU fallback)")


def gemm(M, N, K, A, lda, a_kmajor, B, ldb, b_kmajor, C, ldc, *, bias=None, residual=None, ldr=0,
         aux=None, ldaux=0, alpha=1.0, flags=0, split_k=1, workspace=None, bias_grad=None, small_tile=False,
         split3=False):
    """C[m,n] = epi(alpha * sum_k A(m,k) B(n,k)); see include/clipmi.h clipmi_gemm.  split3: fp32 operands
    and output computed as a bf16x3 split product on the bf16 MFMA kernels (CLIPMI_GEMM_SPLIT3; its
    split images and any split-K slabs in a scratch allocated here, `workspace` is not used)."""
    _on_gpu(A, B, C, bias, residual, aux, workspace)
    if A.dtype != B.dtype:
        raise ValueError("A and B must share a dtype")
    if split3:
        flags |= _lib.GEMM_SPLIT3
        nb = int(_lib.lib().clipmi_gemm_split3_ws(M, N, K, int(a_kmajor), int(b_kmajor), split_k))
        workspace = torch.empty(max(nb, 16), dtype=torch.uint8, device=C.device)
    d = GemmDesc()
    d.M, d.N, d.K = M, N, K
    d.A, d.lda, d.a_kmajor = A.data_ptr(), lda, int(a_kmajor)
    d.B, d.ldb, d.b_kmajor = B.data_ptr(), ldb, int(b_kmajor)
    d.C, d.ldc = C.data_ptr(), ldc
    d.bias = bias.data_ptr() if bias is not None else None
    d.residual, d.ldr = (residual.data_ptr() if residual is not None else None), ldr
    d.aux, d.ldaux = (aux.data_ptr() if aux is not None else None), ldaux
    d.alpha, d.flags = alpha, flags
    d.ab_dtype, d.c_dtype = dt(A), dt(C)
    d.bias_dtype = dt(bias) if bias is not None else F32
    d.split_k = split_k
    d.bias_grad = bias_grad.data_ptr() if bias_grad is not None else None
    d.force_small_tile = int(small_tile)
    if workspace is not None:
        d.workspace, d.workspace_bytes = workspace.data_ptr(), workspace.numel() * workspace.element_size()
    _lib.check(_lib.lib().clipmi_gemm(stream(), ctypes.byref(d)), "clipmi_gemm")
    return C


def gemm_x3out(M, N, K, A, lda, B, ldb, b_kmajor, C3, pattern, *, bias=None, aux=None, ldaux=0, flags=0,
               colsum=None, beta=True):
    """The bf16x3 mode's image-output product (include/clipmi.h clipmi_gemm_x3out): bf16 k-major A, the fp32
    epilogue's result written as the split image C3 bf16 [M][3N] (pattern 0: h, h, l; 1: h, l, h); colsum (fp32
    [N]): the result's column sums added (beta) or stored."""
    _on_gpu(A, B, C3, bias, aux, colsum)
    if A.dtype != torch.bfloat16 or B.dtype != torch.bfloat16 or C3.dtype != torch.bfloat16:
        raise ValueError("gemm_x3out: bf16 operands and image")
    d = GemmDesc()
    d.M, d.N, d.K = M, N, K
    d.A, d.lda, d.a_kmajor = A.data_ptr(), lda, 1
    d.B, d.ldb, d.b_kmajor = B.data_ptr(), ldb, int(b_kmajor)
    d.C, d.ldc = C3.data_ptr(), 3 * N
    d.bias = bias.data_ptr() if bias is not None else None
    d.aux, d.ldaux = (aux.data_ptr() if aux is not None else None), ldaux
    d.alpha, d.flags = 1.0, flags
    d.ab_dtype, d.c_dtype = BF16, F32
    d.bias_dtype = dt(bias) if bias is not None else F32
    d.split_k = 1
    ws = None
    if colsum is not None:
        ws = torch.empty(int(_lib.lib().clipmi_gemm_x3out_ws(M, N)), dtype=torch.uint8, device=C3.device)
    _lib.check(_lib.lib().clipmi_gemm_x3out(stream(), ctypes.byref(d), pattern,
                                            colsum.data_ptr() if colsum is not None else None, int(beta),
                                            ws.data_ptr() if ws is not None else None,
                                            ws.numel() if ws is not None else 0), "clipmi_gemm_x3out")
    return C3


def gemm_batched(M, N, K, A, lda, a_kmajor, B, ldb, b_kmajor, C, ldc, nb1, nb2, sa, sb, sc, *, alpha=1.0,
                 beta=False):
    """nb1 x nb2 fp32 products in one launch: product (i1, i2) reads A + i1 sa[0] + i2 sa[1], B + ...,
    writes C + i1 sc[0] + i2 sc[1] (element strides); see include/clipmi.h clipmi_gemm_batched."""
    _on_gpu(A, B, C)
    if not (A.dtype == B.dtype == C.dtype == torch.float32):
        raise ValueError("gemm_batched: fp32 operands and output")
    d = GemmDesc()
    d.M, d.N, d.K = M, N, K
    d.A, d.lda, d.a_kmajor = A.data_ptr(), lda, int(a_kmajor)
    d.B, d.ldb, d.b_kmajor = B.data_ptr(), ldb, int(b_kmajor)
    d.C, d.ldc = C.data_ptr(), ldc
    d.alpha, d.flags = alpha, (_lib.EPI_BETA if beta else 0)
    d.ab_dtype = d.c_dtype = d.bias_dtype = F32
    d.split_k = 1
    _lib.check(_lib.lib().clipmi_gemm_batched(stream(), ctypes.byref(d), nb1, nb2, sa[0], sa[1], sb[0], sb[1],
                                               sc[0], sc[1]), "clipmi_gemm_batched")
    return C


def linear(x, w, bias=None, *, act=None, residual=None, out=None, pre_out=None):
    """y = act(x @ w.T + bias) (+ residual): nn.Linear forward on the MFMA GEMM."""
    x2 = x.reshape(-1, x.shape[-1])
    M, K = x2.shape
    N = w.shape[0]
    if out is None:
        out = torch.empty(M, N, device=x.device, dtype=x.dtype)
    flags = 0
    if bias is not None:
        flags |= _lib.EPI_BIAS
    if act == "quick_gelu":
        flags |= _lib.EPI_QGELU
    elif act == "gelu":
        flags |= _lib.EPI_GELU
    if residual is not None:
        flags |= _lib.EPI_RESID
    if pre_out is not None:
        flags |= _lib.EPI_STORE_PRE
    gemm(M, N, K, x2, x2.stride(0), True, w, w.stride(0), True, out, out.stride(0), bias=bias,
         residual=residual.reshape(-1, N) if residual is not None else None, ldr=N,
         aux=pre_out, ldaux=N, flags=flags)
    return out.view(*x.shape[:-1], N)


_lib.declare("clipmi_quant_mxfp8", [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64,
                                    ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p])
_lib.declare("clipmi_layernorm_fwd_mxfp8", [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int64,
                                            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                            ctypes.c_float])


class MX8:
    """An MXFP8 matrix: OCP e4m3 bytes q [R, K] + E8M0 block scales s [R, K/32] (uint8)."""

    def __init__(self, q, s):
        self.q, self.s = q, s

    @property
    def shape(self):
        return tuple(self.q.shape)

    def dequant(self):
        """fp32 values (for tests): fp8 * 2^(scale - 127)."""
        v = self.q.view(torch.float8_e4m3fn).float()
        e = self.s.to(torch.int32) - 127
        return v * torch.pow(2.0, e.float()).repeat_interleave(32, dim=1)


def quant_mxfp8(x, out=None):
    """x [R, K] bf16/fp32 (K % 32 == 0) -> MX8 (clipmi_quant_mxfp8)."""
    _on_gpu(x)
    R, Kd = x.shape
    if out is None:
        out = MX8(torch.empty(R, Kd, dtype=torch.uint8, device=x.device),
                  torch.empty(R, Kd // 32, dtype=torch.uint8, device=x.device))
    _lib.check(_lib.lib().clipmi_quant_mxfp8(stream(), dt(x), x.data_ptr(), x.stride(0), R, Kd, out.q.data_ptr(),
                                             out.s.data_ptr()), "clipmi_quant_mxfp8")
    return out


def layernorm_mxfp8(x, w, b, eps=1e-5):
    """LayerNorm of x [R, D] (bf16) written as MXFP8 (clipmi_layernorm_fwd_mxfp8) -> (MX8, mean, rstd)."""
    _on_gpu(x, w, b)
    R, D = x.shape
    out = MX8(torch.empty(R, D, dtype=torch.uint8, device=x.device),
              torch.empty(R, D // 32, dtype=torch.uint8, device=x.device))
    mean = torch.empty(R, dtype=torch.float32, device=x.device)
    rstd = torch.empty(R, dtype=torch.float32, device=x.device)
    _lib.check(_lib.lib().clipmi_layernorm_fwd_mxfp8(stream(), dt(x), x.data_ptr(), x.stride(0), out.q.data_ptr(),
                                                     out.s.data_ptr(), w.data_ptr(), b.data_ptr(), mean.data_ptr(),
                                                     rstd.data_ptr(), R, D, eps), "clipmi_layernorm_fwd_mxfp8")
    return out, mean, rstd


def gemm_fp8(M, N, K, A, B, C, ldc, *, bias=None, residual=None, ldr=0, alpha=1.0, flags=0, variant=0):
    """C[m,n] = epi(alpha * sum_k A(m,k) B(n,k)) with A [M, K], B [N, K] MXFP8 (MX8).  C is a
    tensor (bf16 / fp32) or an MX8 [M, N] (MXFP8 output: flags bias / activation only)."""
    q8o = isinstance(C, MX8)
    _on_gpu(A.q, B.q, C.q if q8o else C, bias, residual)
    d = GemmDesc()
    d.M, d.N, d.K = M, N, K
    d.A, d.lda, d.a_kmajor = A.q.data_ptr(), A.q.stride(0), 1
    d.B, d.ldb, d.b_kmajor = B.q.data_ptr(), B.q.stride(0), 1
    d.a_scale, d.b_scale = A.s.data_ptr(), B.s.data_ptr()
    d.C, d.ldc = (C.q if q8o else C).data_ptr(), ldc
    d.c_scale = C.s.data_ptr() if q8o else None
    d.bias = bias.data_ptr() if bias is not None else None
    d.residual, d.ldr = (residual.data_ptr() if residual is not None else None), ldr
    d.alpha, d.flags = alpha, flags
    d.ab_dtype, d.c_dtype = FP8, (FP8 if q8o else dt(C))
    d.bias_dtype = dt(bias) if bias is not None else F32
    d.split_k = 1
    d.force_small_tile = int(variant)  # 40: the 8-wave fp8 kernel instead of the persistent 4-wave one
    _lib.check(_lib.lib().clipmi_gemm(stream(), ctypes.byref(d)), "clipmi_gemm")
    return C

"""adapter/peclip.py's three modules on libclipmi, with the reference's class names, constructor
arguments and state-dict keys (checkpoints load either way).

    TextualAdapter(input_dim, hidden_dim)   up_proj(GELU(down_proj(x))) + x          (peclip.py:6-18)
    ContextAdapter(input_dim, num_heads)    layer_norm(mhsa(x, x, x) + x)            (peclip.py:21-34)
    SharedAdapter(input_dim, num_heads)     the same computation, its own class      (peclip.py:37-48)

``mhsa`` is nn.MultiheadAttention(batch_first=True, dropout 0, bias on): one fused in-projection
GEMM [B*N, 3D] (q | k | v, head h at h*head_dim -- the layout clipmi_attention reads), softmax
attention with scale head_dim^-0.5 and no mask, the out-projection GEMM with its bias and the
residual x fused into the epilogue, then the LayerNorm kernel (eps 1e-5).  head_dim 64 and
N <= 4096 run the flash attention kernels (clipmi_attention_fwd/bwd); other head widths run the
scores, softmax and context of every (sample, head) as strided-batched exact-fp32 GEMMs
(clipmi_gemm_batched) and row-softmax kernels over all rows: three launches forward, five backward,
whatever B * H is.  Every op is a libclipmi GPU kernel; there is no CPU path (construction works
anywhere, forward needs CUDA tensors).

``precision`` is the compute precision, as in CLIPWithAdapters: "fp32" (parity) or "bf16" (MFMA
operands from the bf16 shadow of the fp32 master weights, fp32 accumulation and gradients).  The
general-head-width path above computes in fp32 under either setting (``attention_precision`` says
which one a module runs: "bf16" only with head_dim 64).
Initialisation draws from torch's default generator in nn.Linear / nn.MultiheadAttention's order,
so under the same torch.manual_seed the parameters equal the reference module's.
"""
from __future__ import annotations

import math
import types

import torch
import torch.nn as nn

from . import _lib
from . import kernels as K
from . import towers as T
from .modules import ArenaModule, AdapterParams

P_, call, F32 = T.P_, T.call, T.F32
_lib.declare("clipmi_softmax_rows", [T.c_vp, T.c_vp, T.c_vp, T.c_int, T.c_int, T.c_float])
_lib.declare("clipmi_softmax_rows_bwd", [T.c_vp, T.c_vp, T.c_vp, T.c_vp, T.c_int, T.c_int, T.c_float])
EPS = 1e-5


def _init_linear(w, b):
    """nn.Linear.reset_parameters (weight kaiming_uniform a=sqrt(5), then bias U(+-1/sqrt(fan_in)))."""
    cw = torch.empty(w.shape)
    nn.init.kaiming_uniform_(cw, a=math.sqrt(5))
    bound = 1.0 / math.sqrt(w.shape[1]) if w.shape[1] > 0 else 0.0
    cb = torch.empty(b.shape).uniform_(-bound, bound)
    return cw, cb


def _check_precision(precision):
    if precision not in ("fp32", "bf16"):
        raise ValueError("precision must be 'fp32' or 'bf16'")
    return torch.float32 if precision == "fp32" else torch.bfloat16


class TextualAdapter(AdapterParams):
    """peclip.TextualAdapter (peclip.py:6-18): the bottleneck adapter with no LayerNorm, on
    towers.AdapterFn (down GEMM + bias + GELU(erf), up GEMM + bias + residual)."""

    def __init__(self, input_dim, hidden_dim, *, device=None, precision="fp32"):
        dtype = _check_precision(precision)
        if device is None:
            device = "cuda" if torch.cuda.is_available() else "cpu"
        super().__init__(input_dim, hidden_dim, device, ln=False, shadow=dtype == torch.bfloat16,
                         names=("down_proj", "up_proj"))
        self._rt = types.SimpleNamespace(dtype=dtype)
        with torch.no_grad():  # construction order of the reference: down_proj, then up_proj
            for n in ("down_proj", "up_proj"):
                w, b = _init_linear(self.arena.view(f"{n}.weight"), self.arena.view(f"{n}.bias"))
                self.arena.view(f"{n}.weight").copy_(w)
                self.arena.view(f"{n}.bias").copy_(b)

    def forward(self, x):
        if x.shape[-1] != self.hidden:  # nn.Linear's error in down_proj
            rows = x.numel() // max(1, x.shape[-1])
            raise RuntimeError(f"mat1 and mat2 shapes cannot be multiplied ({rows}x{x.shape[-1]} and "
                               f"{self.hidden}x{self.bottleneck})")
        anchor = next(self.parameters())
        need = torch.is_grad_enabled() and (x.requires_grad or self.arena.any_requires_grad())
        y = T.AdapterFn.apply(x, anchor, self._rt, self, need)
        return y.to(x.dtype)


def _mhsa_specs(D):
    return [("mhsa.in_proj_weight", (3 * D, D)), ("mhsa.in_proj_bias", (3 * D,)),
            ("mhsa.out_proj.weight", (D, D)), ("mhsa.out_proj.bias", (D,)),
            ("layer_norm.weight", (D,)), ("layer_norm.bias", (D,))]


class _MHSAResidualLN(ArenaModule):
    """layer_norm(mhsa(x, x, x) + x): ContextAdapter / SharedAdapter (peclip.py:21-48)."""

    def __init__(self, input_dim, num_heads, *, device=None, precision="fp32"):
        dtype = _check_precision(precision)
        # nn.MultiheadAttention's own argument checks
        if input_dim % num_heads:
            raise AssertionError("embed_dim must be divisible by num_heads")
        if device is None:
            device = "cuda" if torch.cuda.is_available() else "cpu"
        super().__init__(_mhsa_specs(input_dim), device, shadow=dtype == torch.bfloat16)
        self.embed_dim, self.num_heads, self.head_dim = input_dim, num_heads, input_dim // num_heads
        self.dtype = dtype
        # the compute precision of the whole block: the head_dim-64 flash path follows ``precision``,
        # other head widths run exact fp32 (module docstring)
        self.attention_precision = ("bf16" if dtype == torch.bfloat16 else "fp32") if self.head_dim == 64 else "fp32"
        D = input_dim
        with torch.no_grad():
            # nn.MultiheadAttention.__init__: out_proj (an nn.Linear: kaiming weight, uniform bias) is
            # built first, then _reset_parameters: xavier_uniform_(in_proj_weight), both biases zeroed;
            # nn.LayerNorm: ones / zeros
            wo, _ = _init_linear(self.arena.view("mhsa.out_proj.weight"), self.arena.view("mhsa.out_proj.bias"))
            win = torch.empty(3 * D, D)
            nn.init.xavier_uniform_(win)
            self.arena.view("mhsa.out_proj.weight").copy_(wo)
            self.arena.view("mhsa.in_proj_weight").copy_(win)
            self.arena.view("layer_norm.weight").fill_(1.0)

    def forward(self, x):
        D = self.embed_dim
        if x.dim() not in (2, 3):
            raise AssertionError(f"query should be unbatched 2D or batched 3D tensor but received {x.dim()}-D "
                                 "query tensor")
        if x.shape[-1] != D:
            raise AssertionError(f"was expecting embedding dimension of {D}, but got {x.shape[-1]}")
        if D > 4096:  # clipmi_layernorm_fwd's widest row
            raise ValueError(f"clipmi ContextAdapter/SharedAdapter need input_dim <= 4096 (got {D})")
        anchor = next(self.parameters())
        need = torch.is_grad_enabled() and (x.requires_grad or self.arena.any_requires_grad())
        xb = x if x.dim() == 3 else x.unsqueeze(0)
        y = MHSAResidualLNFn.apply(xb, anchor, self, need)
        return (y if x.dim() == 3 else y.squeeze(0)).to(x.dtype)


class ContextAdapter(_MHSAResidualLN):
    """peclip.ContextAdapter (peclip.py:21-34): spatial context over image patch tokens."""


class SharedAdapter(_MHSAResidualLN):
    """peclip.SharedAdapter (peclip.py:37-48): the same self-attention + LayerNorm residual."""


def _fast_attention(mod, N):
    return mod.head_dim == 64 and N <= 4096


class MHSAResidualLNFn(torch.autograd.Function):
    """y = LN(out_proj(softmax(q k^T / sqrt(hd)) v) + x) with [q|k|v] = in_proj(x), per head."""

    @staticmethod
    def forward(ctx, x, anchor, mod, need):
        a = mod.arena
        B, N, D = x.shape
        H, hd = mod.num_heads, mod.head_dim
        fast = _fast_attention(mod, N)
        dtype = mod.dtype if fast else torch.float32  # the general head width runs in fp32
        dc = T.dcode(dtype)
        wbuf = T._wbuf(a, dtype)
        R = B * N
        dev = x.device
        K._on_gpu(x, a.data)
        s = K.stream()
        x2 = x.to(dtype).reshape(R, D).contiguous()
        e = lambda *sh: torch.empty(*sh, dtype=dtype, device=dev)  # noqa: E731
        qkv, o, z, y = e(R, 3 * D), e(R, D), e(R, D), e(R, D)
        W = lambda n: a.view(n, wbuf)  # noqa: E731
        K.gemm(R, 3 * D, D, x2, D, True, W("mhsa.in_proj_weight"), D, True, qkv, 3 * D,
               bias=W("mhsa.in_proj_bias"), flags=_lib.EPI_BIAS)
        lse = P = None
        if fast:
            lse = torch.empty(B * H * N, dtype=torch.float32, device=dev)
            call("clipmi_attention_fwd", s, dc, P_(qkv), P_(o), P_(lse), None, 0, B, H, N, D)
        else:  # three launches for every (sample, head): scores, row softmax, context
            P = torch.empty(B, H, N, N, dtype=torch.float32, device=dev)
            scale = hd ** -0.5
            sq, sp = (N * 3 * D, hd), (H * N * N, N * N)
            K.gemm_batched(N, N, hd, qkv, 3 * D, True, qkv[:, D:], 3 * D, True, P, N, B, H, sq, sq, sp)
            call("clipmi_softmax_rows", s, P_(P), P_(P), B * H * N, N, scale)
            K.gemm_batched(N, hd, N, P, N, True, qkv[:, 2 * D:], 3 * D, False, o, D, B, H, sp, sq, (N * D, hd))
        K.gemm(R, D, D, o, D, True, W("mhsa.out_proj.weight"), D, True, z, D, bias=W("mhsa.out_proj.bias"),
               residual=x2, ldr=D, flags=_lib.EPI_BIAS | _lib.EPI_RESID)
        stats = torch.empty(2, R, dtype=torch.float32, device=dev)
        call("clipmi_layernorm_fwd", s, dc, P_(z), D, P_(y), D, a.ptr("layer_norm.weight", wbuf),
             a.ptr("layer_norm.bias", wbuf), P_(stats[0]), P_(stats[1]), R, D, EPS, None, None, 0)
        if need:
            ctx.save = (x2, qkv, o, z, stats, lse, P)
            ctx.mod, ctx.fast, ctx.dtype, ctx.shape = mod, fast, dtype, x.shape
        return y.view(B, N, D)

    @staticmethod
    def backward(ctx, dy):
        mod, fast, dtype = ctx.mod, ctx.fast, ctx.dtype
        x2, qkv, o, z, stats, lse, P = ctx.save
        a = mod.arena
        B, N, D = ctx.shape
        H, hd = mod.num_heads, mod.head_dim
        R = B * N
        dev = dy.device
        s = K.stream()
        dc = T.dcode(dtype)
        wbuf = T._wbuf(a, dtype)
        W = lambda n: a.view(n, wbuf)  # noqa: E731
        train = a.any_requires_grad()
        if train:
            a.prepare_grads()
        g = a.grad
        G = lambda n: a.view(n, g)  # noqa: E731
        gp = lambda n: a.ptr(n, g) if train else None  # noqa: E731
        bf = dtype == torch.bfloat16
        e = lambda *sh: torch.empty(*sh, dtype=dtype, device=dev)  # noqa: E731
        dy2 = dy.to(dtype).reshape(R, D).contiguous()
        # LayerNorm backward (its affine gradients accumulate into the arena)
        dz = e(R, D)
        lws = T._ws(_lib.lib().clipmi_layernorm_bwd_ws(R, D), dev)
        call("clipmi_layernorm_bwd", s, dc, P_(dy2), D, P_(z), D, P_(stats[0]), P_(stats[1]),
             a.ptr("layer_norm.weight", wbuf), P_(dz), D, None, 0, gp("layer_norm.weight"), gp("layer_norm.bias"),
             1, P_(lws), lws.numel(), R, D)
        cws = T._ws(_lib.lib().clipmi_colsum_ws(R, 3 * D), dev)

        def colsum(t, n, name):
            call("clipmi_colsum", s, dc, P_(t), n, R, n, gp(name), 1, P_(cws), cws.numel())

        # out-projection: z = o Wo^T + bo + x
        if train:
            K.gemm(D, D, R, dz, D, False, o, D, False, G("mhsa.out_proj.weight"), D, flags=_lib.EPI_BETA,
                   bias_grad=G("mhsa.out_proj.bias") if bf else None)
            if not bf:
                colsum(dz, D, "mhsa.out_proj.bias")
        do = e(R, D)
        K.gemm(R, D, D, dz, D, True, W("mhsa.out_proj.weight"), D, False, do, D)
        # attention
        dqkv = e(R, 3 * D)
        if fast:
            call("clipmi_attention_bwd", s, dc, P_(qkv), P_(o), P_(lse), P_(do), P_(dqkv), None, 0, B, H, N, D)
        else:  # five launches for every (sample, head)
            dS = torch.empty(B, H, N, N, dtype=torch.float32, device=dev)
            scale = hd ** -0.5
            sq, sp, so = (N * 3 * D, hd), (H * N * N, N * N), (N * D, hd)
            K.gemm_batched(N, N, hd, do, D, True, qkv[:, 2 * D:], 3 * D, True, dS, N, B, H, so, sq, sp)  # dP
            call("clipmi_softmax_rows_bwd", s, P_(P), P_(dS), P_(dS), B * H * N, N, scale)          # dS
            K.gemm_batched(N, hd, N, dS, N, True, qkv[:, D:], 3 * D, False, dqkv, 3 * D, B, H, sp, sq, sq)  # dQ
            K.gemm_batched(N, hd, N, dS, N, False, qkv, 3 * D, False, dqkv[:, D:], 3 * D, B, H, sp, sq, sq)  # dK
            K.gemm_batched(N, hd, N, P, N, False, do, D, False, dqkv[:, 2 * D:], 3 * D, B, H, sp, so, sq)   # dV
        # in-projection: qkv = x Win^T + bin
        if train:
            K.gemm(3 * D, D, R, dqkv, 3 * D, False, x2, D, False, G("mhsa.in_proj_weight"), D, flags=_lib.EPI_BETA,
                   bias_grad=G("mhsa.in_proj_bias") if bf else None)
            if not bf:
                colsum(dqkv, 3 * D, "mhsa.in_proj_bias")
        dx = e(R, D)
        K.gemm(R, D, 3 * D, dqkv, 3 * D, True, W("mhsa.in_proj_weight"), D, False, dx, D, residual=dz, ldr=D,
               flags=_lib.EPI_RESID)
        ctx.save = None
        return dx.view(B, N, D), None, None, None

"""SharedMHSAttentionAdapter (adapter/clip_adapter.py:69-128) on libclipmi, with the batch
broadcast that the reference lacks (its keys are the vision position
embedding [1, N_v, D_v] (model_m.py:95-100), so nn.MultiheadAttention fails for batch > 1;
here the image tokens are shared by every caption, which is what batch 1 computes).

    t  = text_proj(x)                        k/v input = norm1(image_proj(pos_emb))
    t2 = norm2(t) + out_proj(MHA(norm2(t), k, v))         (8 heads of 64, softmax fp32)
    y  = t2 + mlp.2(GELU(mlp.0(norm3(t2))))

Every text token is processed independently (queries only attend to the image tokens), and
only the pooled token reaches the features (model_m.py:102), so the adapter runs on that row
alone.  fp32 throughout (a few MFLOP per caption): the clipmi fp32 GEMM with fused
bias / GELU / residual epilogues, native LayerNorm, row softmax and column-sum kernels.
Dropout (p = 0.1, adapter/clip_adapter.py:84,96) runs in training mode (nn.Module.train()) on
the attention probabilities (nn.MultiheadAttention's dropout) and on mlp.2's output, with masks
from libclipmi's seeded counter generator (clipmi_dropout_mask; a seed replays its masks); in
eval mode the outputs equal the reference's, which is what the parity tests pin.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from . import kernels as K
from . import synth
from . import towers as T
from .modules import ArenaModule

P_, call, F32 = T.P_, T.call, T.F32
_lib.declare("clipmi_softmax_rows", [T.c_vp, T.c_vp, T.c_vp, T.c_int, T.c_int, T.c_float])
_lib.declare("clipmi_softmax_rows_bwd", [T.c_vp, T.c_vp, T.c_vp, T.c_vp, T.c_int, T.c_int, T.c_float])
_lib.declare("clipmi_dropout_mask", [T.c_vp, T.c_vp, T.c_i64, T.c_float, ctypes.c_uint64, ctypes.c_uint64])
_lib.declare("clipmi_dropout_apply", [T.c_vp, T.c_vp, T.c_vp, T.c_i64, T.c_float, T.c_vp, T.c_vp])

HEAD = 64


def shared_specs(text_in, image_in, hidden=512):
    H = hidden
    return [("text_proj.weight", (H, text_in)), ("text_proj.bias", (H,)),
            ("image_proj.weight", (H, image_in)), ("image_proj.bias", (H,)),
            ("cross_attn.in_proj_weight", (3 * H, H)), ("cross_attn.in_proj_bias", (3 * H,)),
            ("cross_attn.out_proj.weight", (H, H)), ("cross_attn.out_proj.bias", (H,)),
            ("norm1.weight", (H,)), ("norm1.bias", (H,)), ("norm2.weight", (H,)), ("norm2.bias", (H,)),
            ("norm3.weight", (H,)), ("norm3.bias", (H,)),
            ("mlp.0.weight", (4 * H, H)), ("mlp.0.bias", (4 * H,)),
            ("mlp.2.weight", (H, 4 * H)), ("mlp.2.bias", (H,))]


class SharedAdapterParams(ArenaModule):
    """Parameters with SharedMHSAttentionAdapter's state-dict names, in one fp32 arena."""

    def __init__(self, text_in, image_in, device, hidden=512, seed=0, prefix="shared_adapters.0", dropout=0.1):
        super().__init__(shared_specs(text_in, image_in, hidden), device, shadow=False)
        self.text_in, self.image_in, self.hidden = text_in, image_in, hidden
        if hidden % HEAD:
            raise ValueError("hidden_size must be a multiple of 64 (8 heads of 64 in the reference)")
        self.load_numpy(synth.shared_adapter_state_dict(text_in, image_in, seed, prefix, hidden))
        self.p = float(dropout)
        self.drop_seed = (seed * 1000003 + sum(map(ord, prefix))) & (2 ** 63 - 1)
        self.drop_offset = 0

    def dropout_mask(self, n, device):
        """Counter-based keep mask for the next n elements.  Replay: a mask is a pure function of
        (drop_seed, rank, drop_offset, n); the offset advances by n on every training-mode call,
        so re-running the same calls from the same drop_offset reproduces the masks.  In a
        data-parallel group the rank is mixed into the seed, so ranks draw different masks for
        their different samples (as independent torch RNG streams would)."""
        keep = torch.empty(n, dtype=torch.uint8, device=device)
        seed = self.drop_seed
        if torch.distributed.is_available() and torch.distributed.is_initialized():
            r = torch.distributed.get_rank()
            if r:
                seed = (seed ^ ((r * 0x9E3779B97F4A7C15) & (2 ** 64 - 1))) & (2 ** 63 - 1)
        call("clipmi_dropout_mask", K.stream(), P_(keep), n, self.p, seed, self.drop_offset)
        self.drop_offset += n
        return keep


def _ln(x, w, b, R, D):
    y = torch.empty_like(x)
    st = torch.empty(2, R, dtype=torch.float32, device=x.device)
    call("clipmi_layernorm_fwd", K.stream(), F32, P_(x), D, P_(y), D, w, b, P_(st[0]), P_(st[1]), R, D, 1e-5,
         None, None, 0)
    return y, st


def _ln_bwd(dy, x, st, w, gw, gb, R, D, dres=None):
    dx = torch.empty_like(x)
    ws = T._ws(_lib.lib().clipmi_layernorm_bwd_ws(R, D), x.device)
    call("clipmi_layernorm_bwd", K.stream(), F32, P_(dy), D, P_(x), D, P_(st[0]), P_(st[1]), w, P_(dx), D,
         P_(dres), D if dres is not None else 0, gw, gb, 1, P_(ws), ws.numel(), R, D)
    return dx


def _colsum(x, R, N, out_ptr):
    ws = T._ws(_lib.lib().clipmi_colsum_ws(R, N), x.device)
    call("clipmi_colsum", K.stream(), F32, P_(x), N, R, N, out_ptr, 1, P_(ws), ws.numel())


class SharedAdapterFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, anchor, mod, image_tokens, need):
        a = mod.arena
        W = lambda n: a.view(n)  # noqa: E731  (fp32 master weights)
        shp, dt = x.shape, x.dtype
        if shp[-1] != mod.text_in:  # nn.Linear's error in text_proj (adapter/clip_adapter.py:101)
            rows = x.numel() // max(1, shp[-1])
            raise RuntimeError(f"mat1 and mat2 shapes cannot be multiplied ({rows}x{shp[-1]} and "
                               f"{mod.text_in}x{mod.hidden})")
        x32 = x.reshape(-1, mod.text_in).to(torch.float32).contiguous()
        img = image_tokens.to(torch.float32).contiguous()
        R, Nv, H, nh = x32.shape[0], img.shape[0], mod.hidden, mod.hidden // HEAD
        dev = x.device
        E_B, E_R = _lib.EPI_BIAS, _lib.EPI_RESID
        f = lambda *s: torch.empty(*s, dtype=torch.float32, device=dev)  # noqa: E731
        t, u = f(R, H), f(Nv, H)
        K.gemm(R, H, mod.text_in, x32, mod.text_in, True, W("text_proj.weight"), mod.text_in, True, t, H,
               bias=W("text_proj.bias"), flags=E_B)
        K.gemm(Nv, H, mod.image_in, img, mod.image_in, True, W("image_proj.weight"), mod.image_in, True, u, H,
               bias=W("image_proj.bias"), flags=E_B)
        ln1, st1 = _ln(u, a.ptr("norm1.weight", a.data), a.ptr("norm1.bias", a.data), Nv, H)
        ln2, st2 = _ln(t, a.ptr("norm2.weight", a.data), a.ptr("norm2.bias", a.data), R, H)
        Win, bin_ = W("cross_attn.in_proj_weight"), W("cross_attn.in_proj_bias")
        q, k, v = f(R, H), f(Nv, H), f(Nv, H)
        K.gemm(R, H, H, ln2, H, True, Win[:H], H, True, q, H, bias=bin_[:H], flags=E_B)
        K.gemm(Nv, H, H, ln1, H, True, Win[H:2 * H], H, True, k, H, bias=bin_[H:2 * H], flags=E_B)
        K.gemm(Nv, H, H, ln1, H, True, Win[2 * H:], H, True, v, H, bias=bin_[2 * H:], flags=E_B)
        P, o = f(nh, R, Nv), f(R, H)
        scale = HEAD ** -0.5
        drop = mod.training and mod.p > 0
        ds = 1.0 / (1.0 - mod.p) if drop else 1.0
        keep_p = mod.dropout_mask(nh * R * Nv, dev).view(nh, R, Nv) if drop else None
        Pd = f(nh, R, Nv) if drop else P  # dropped probabilities (nn.MultiheadAttention dropout)
        for h in range(nh):
            c = slice(h * HEAD, (h + 1) * HEAD)
            K.gemm(R, Nv, HEAD, q[:, c], H, True, k[:, c], H, True, P[h], Nv)
            call("clipmi_softmax_rows", K.stream(), P_(P[h]), P_(P[h]), R, Nv, scale)
            if drop:
                call("clipmi_dropout_apply", K.stream(), P_(P[h]), P_(keep_p[h]), R * Nv, ds, None, P_(Pd[h]))
            K.gemm(R, HEAD, Nv, Pd[h], Nv, True, v[:, c], H, False, o[:, c], H)
        t2 = f(R, H)
        K.gemm(R, H, H, o, H, True, W("cross_attn.out_proj.weight"), H, True, t2, H,
               bias=W("cross_attn.out_proj.bias"), residual=ln2, ldr=H, flags=E_B | E_R)
        ln3, st3 = _ln(t2, a.ptr("norm3.weight", a.data), a.ptr("norm3.bias", a.data), R, H)
        pre, act, y = f(R, 4 * H), f(R, 4 * H), f(R, H)
        K.gemm(R, 4 * H, H, ln3, H, True, W("mlp.0.weight"), H, True, act, 4 * H, bias=W("mlp.0.bias"), aux=pre,
               ldaux=4 * H, flags=E_B | _lib.EPI_GELU | _lib.EPI_STORE_PRE)
        keep_m = None
        if drop:  # mlp = Sequential(Linear, GELU, Linear, Dropout): y = t2 + dropout(mlp.2(.))
            z = f(R, H)
            K.gemm(R, H, 4 * H, act, 4 * H, True, W("mlp.2.weight"), 4 * H, True, z, H, bias=W("mlp.2.bias"),
                   flags=E_B)
            keep_m = mod.dropout_mask(R * H, dev)
            call("clipmi_dropout_apply", K.stream(), P_(z), P_(keep_m), R * H, ds, P_(t2), P_(y))
        else:
            K.gemm(R, H, 4 * H, act, 4 * H, True, W("mlp.2.weight"), 4 * H, True, y, H, bias=W("mlp.2.bias"),
                   residual=t2, ldr=H, flags=E_B | E_R)
        if need:
            ctx.save = (x32, img, t, u, ln1, st1, ln2, st2, q, k, v, P, Pd, o, t2, ln3, st3, pre, act, keep_p, keep_m, ds)
            ctx.mod, ctx.shape, ctx.dt = mod, shp, dt
        return y.view(*shp[:-1], H).to(dt)

    @staticmethod
    def backward(ctx, dy):
        mod = ctx.mod
        x32, img, t, u, ln1, st1, ln2, st2, q, k, v, P, Pd, o, t2, ln3, st3, pre, act, keep_p, keep_m, ds = ctx.save
        a = mod.arena
        R, Nv, H, nh = x32.shape[0], img.shape[0], mod.hidden, mod.hidden // HEAD
        Dt, Dv = mod.text_in, mod.image_in
        dev = dy.device
        f = lambda *s: torch.empty(*s, dtype=torch.float32, device=dev)  # noqa: E731
        W = lambda n: a.view(n)  # noqa: E731
        train = a.any_requires_grad()
        if train:
            a.prepare_grads()
        G = lambda n: a.view(n, a.grad)  # noqa: E731
        gp = lambda n: a.ptr(n, a.grad) if train else None  # noqa: E731
        BETA = _lib.EPI_BETA
        d = dy.reshape(R, H).to(torch.float32).contiguous()
        dm = d  # gradient reaching mlp.2's output (through its dropout)
        if keep_m is not None:
            dm = f(R, H)
            call("clipmi_dropout_apply", K.stream(), P_(d), P_(keep_m), R * H, ds, None, P_(dm))
        # MLP
        if train:
            K.gemm(H, 4 * H, R, dm, H, False, act, 4 * H, False, G("mlp.2.weight"), 4 * H, flags=BETA)
            _colsum(dm, R, H, gp("mlp.2.bias"))
        dpre = f(R, 4 * H)
        K.gemm(R, 4 * H, H, dm, H, True, W("mlp.2.weight"), 4 * H, False, dpre, 4 * H, aux=pre, ldaux=4 * H,
               flags=_lib.EPI_DGELU)
        if train:
            K.gemm(4 * H, H, R, dpre, 4 * H, False, ln3, H, False, G("mlp.0.weight"), H, flags=BETA)
            _colsum(dpre, R, 4 * H, gp("mlp.0.bias"))
        dln3 = f(R, H)
        K.gemm(R, H, 4 * H, dpre, 4 * H, True, W("mlp.0.weight"), H, False, dln3, H)
        dt2 = _ln_bwd(dln3, t2, st3, a.ptr("norm3.weight", a.data), gp("norm3.weight"), gp("norm3.bias"), R, H,
                      dres=d)
        # attention output projection (t2 = ln2 + out_proj(o))
        if train:
            K.gemm(H, H, R, dt2, H, False, o, H, False, G("cross_attn.out_proj.weight"), H, flags=BETA)
            _colsum(dt2, R, H, gp("cross_attn.out_proj.bias"))
        do = f(R, H)
        K.gemm(R, H, H, dt2, H, True, W("cross_attn.out_proj.weight"), H, False, do, H)
        dq, dk, dv, dP = f(R, H), f(Nv, H), f(Nv, H), f(R, Nv)
        scale = HEAD ** -0.5
        for h in range(nh):
            c = slice(h * HEAD, (h + 1) * HEAD)
            K.gemm(R, Nv, HEAD, do[:, c], H, True, v[:, c], H, True, dP, Nv)
            if keep_p is not None:  # through the probabilities' dropout
                call("clipmi_dropout_apply", K.stream(), P_(dP), P_(keep_p[h]), R * Nv, ds, None, P_(dP))
            call("clipmi_softmax_rows_bwd", K.stream(), P_(P[h]), P_(dP), P_(dP), R, Nv, scale)  # dP -> dS
            K.gemm(R, HEAD, Nv, dP, Nv, True, k[:, c], H, False, dq[:, c], H)
            K.gemm(Nv, HEAD, R, dP, Nv, False, q[:, c], H, False, dk[:, c], H)
            K.gemm(Nv, HEAD, R, Pd[h], Nv, False, do[:, c], H, False, dv[:, c], H)
        Win = W("cross_attn.in_proj_weight")
        if train:
            gWin = G("cross_attn.in_proj_weight")
            gb0 = gp("cross_attn.in_proj_bias")
            K.gemm(H, H, R, dq, H, False, ln2, H, False, gWin[:H], H, flags=BETA)
            K.gemm(H, H, Nv, dk, H, False, ln1, H, False, gWin[H:2 * H], H, flags=BETA)
            K.gemm(H, H, Nv, dv, H, False, ln1, H, False, gWin[2 * H:], H, flags=BETA)
            _colsum(dq, R, H, gb0)
            _colsum(dk, Nv, H, gb0 + 4 * H)
            _colsum(dv, Nv, H, gb0 + 8 * H)
        dln2, dln1 = f(R, H), f(Nv, H)
        K.gemm(R, H, H, dq, H, True, Win[:H], H, False, dln2, H, residual=dt2, ldr=H, flags=_lib.EPI_RESID)
        K.gemm(Nv, H, H, dk, H, True, Win[H:2 * H], H, False, dln1, H)
        K.gemm(Nv, H, H, dv, H, True, Win[2 * H:], H, False, dln1, H, flags=BETA)
        dt = _ln_bwd(dln2, t, st2, a.ptr("norm2.weight", a.data), gp("norm2.weight"), gp("norm2.bias"), R, H)
        need_img = ctx.needs_input_grad[3]  # the vision position embedding trains (CLIP unfrozen)
        dimg = None
        if train or need_img:
            du = _ln_bwd(dln1, u, st1, a.ptr("norm1.weight", a.data), gp("norm1.weight"), gp("norm1.bias"), Nv, H)
        if train:
            K.gemm(H, Dt, R, dt, H, False, x32, Dt, False, G("text_proj.weight"), Dt, flags=BETA)
            _colsum(dt, R, H, gp("text_proj.bias"))
            K.gemm(H, Dv, Nv, du, H, False, img, Dv, False, G("image_proj.weight"), Dv, flags=BETA)
            _colsum(du, Nv, H, gp("image_proj.bias"))
        if need_img:  # d image_tokens = du @ image_proj.weight (model_m.py:96-100 backpropagates into it)
            dimg = f(Nv, Dv)
            K.gemm(Nv, Dv, H, du, H, True, W("image_proj.weight"), Dv, False, dimg, Dv)
        dx = f(R, Dt)
        K.gemm(R, Dt, H, dt, H, True, W("text_proj.weight"), Dt, False, dx, Dt)
        ctx.save = None
        return dx.view(ctx.shape).to(ctx.dt), None, None, dimg, None

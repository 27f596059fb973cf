"""Autograd functions that run the CLIP path on libclipmi.

Each Function's forward/backward is a short sequence of C-ABI calls (the encoder stack
is ONE call per direction, sequenced natively in csrc/engine.cpp).  Parameter
gradients are written straight into the fp32 gradient arena (``Arena.grad``) and exposed
as ``p.grad`` views (AccumulateGrad semantics emulated by ``Arena.prepare_grads``), so
autograd only carries activation gradients between the Functions.

Reference mapping:
  VisionTowerFn  <- CLIPVisionModel.forward ([HF] modeling_clip.py:638-651), last_hidden_state
                    without post_layernorm (model_m.py:116, quirk Q2)
  TextTowerFn    <- CLIPTextModel.forward ([HF] :513-559), last_hidden_state after final LN
  AdapterFn      <- TextAdapter/VisionAdapter.forward (adapter/clip_adapter.py:17-23, 144-150),
                    peclip.TextualAdapter (adapter/peclip.py:13-18) with ln=False
  PoolProjFn     <- [:, 0, :] + text_projection / visual_projection (model_m.py:102-103, 122-123)
  ContrastiveFn  <- model_m.py:146-171 (+ the SURVEY §8e data-parallel all-gather form)
"""
from __future__ import annotations

import ctypes
import os

import torch
import torch.distributed as dist

from . import _lib
from . import comm as CM
from . import kernels as K
from ._lib import BF16, F32

c_vp, c_i64, c_int, c_float = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_float

W_FIELDS = ["ln1_w", "ln1_b", "qkv_w", "qkv_b", "out_w", "out_b", "ln2_w", "ln2_b", "fc1_w", "fc1_b", "fc2_w", "fc2_b"]
A_FIELDS = ["x_in", "ln1", "qkv", "o", "h", "ln2", "pre", "act", "mean1", "rstd1", "lse", "mean2", "rstd2"]


class LayerW(ctypes.Structure):
    _fields_ = [(n, c_vp) for n in W_FIELDS]


class LayerG(ctypes.Structure):
    _fields_ = [(n, c_vp) for n in W_FIELDS]


class LayerAct(ctypes.Structure):
    _fields_ = [(n, c_vp) for n in A_FIELDS]


W8_FIELDS = ["qkv_w", "qkv_s", "out_w", "out_s", "fc1_w", "fc1_s", "fc2_w", "fc2_s"]


class LayerW8(ctypes.Structure):
    _fields_ = [(n, c_vp) for n in W8_FIELDS]


class EncoderDesc(ctypes.Structure):
    _fields_ = [("dtype", c_int), ("B", c_int), ("N", c_int), ("D", c_int), ("F", c_int), ("H", c_int),
                ("L", c_int), ("eps", c_float), ("causal", c_int), ("attention_mask", c_vp),
                ("layers", ctypes.POINTER(LayerW)), ("grads", ctypes.POINTER(LayerG)),
                ("act", ctypes.POINTER(LayerAct)), ("x_out", c_vp), ("workspace", c_vp),
                ("workspace_bytes", c_i64), ("layers8", ctypes.POINTER(LayerW8)), ("q8", c_vp), ("s8", c_vp),
                ("resid_f32", c_int), ("gemm_x3", c_int), ("x3_ws", c_vp), ("x3_ws_bytes", c_i64)]


P = ctypes.POINTER
_lib.declare("clipmi_encoder_fwd", [c_vp, P(EncoderDesc)])
_lib.declare("clipmi_encoder_bwd", [c_vp, P(EncoderDesc), c_vp])
_lib.declare("clipmi_encoder_bwd_ws", [P(EncoderDesc)], c_i64)
_lib.declare("clipmi_encoder_x3_ws", [P(EncoderDesc)], c_i64)
_lib.declare("clipmi_encoder_bwd_layers", [c_vp, P(EncoderDesc), c_vp, c_int, c_int])
_lib.declare("clipmi_layernorm_fwd", [c_vp, c_int, c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_int, c_int,
                                      c_float, c_vp, c_vp, c_int])
_lib.declare("clipmi_layernorm_fwd2", [c_vp, c_int, c_int, c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_int,
                                       c_int, c_float, c_vp, c_vp, c_int])
_lib.declare("clipmi_layernorm_bwd2", [c_vp, c_int, c_int, c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_i64,
                                       c_vp, c_i64, c_vp, c_vp, c_int, c_vp, c_i64, c_int, c_int])
_lib.declare("clipmi_layernorm_bwd3", [c_vp, c_int, c_int, c_int, c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp,
                                       c_i64, c_vp, c_i64, c_vp, c_vp, c_int, c_vp, c_i64, c_int, c_int])
_lib.declare("clipmi_layernorm_bwd_ws", [c_int, c_int], c_i64)
_lib.declare("clipmi_layernorm_bwd_x3_ws", [c_int, c_int], c_i64)
_lib.declare("clipmi_layernorm_bwd_x3", [c_vp, c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_i64,
                                         c_vp, c_vp, c_int, c_vp, c_vp, c_int, c_vp, c_i64, c_int, c_int])
_lib.declare("clipmi_layernorm_bwd", [c_vp, c_int, c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp,
                                      c_i64, c_vp, c_vp, c_int, c_vp, c_i64, c_int, c_int])
_lib.declare("clipmi_colsum_ws", [c_int, c_int], c_i64)
_lib.declare("clipmi_colsum", [c_vp, c_int, c_vp, c_i64, c_int, c_int, c_vp, c_int, c_vp, c_i64])
_lib.declare("clipmi_period_sum", [c_vp, c_int, c_vp, c_i64, c_int, c_int, c_int, c_int, c_vp, c_int])
_lib.declare("clipmi_text_embed", [c_vp, c_int, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_vp])
_lib.declare("clipmi_text_embed_bwd_ws", [c_int, c_int], c_i64)
_lib.declare("clipmi_text_embed_bwd", [c_vp, c_int, c_vp, c_vp, c_int, c_int, c_int, c_vp, c_int, c_vp, c_i64])
_lib.declare("clipmi_im2col", [c_vp, c_int, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int])
_lib.declare("clipmi_im2col_u8", [c_vp, c_int, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int,
                                  ctypes.POINTER(c_float), ctypes.POINTER(c_float)])

# CLIPImageProcessor defaults (OpenAI CLIP, [HF] utils/constants.py: OPENAI_CLIP_MEAN / _STD)
IMAGE_MEAN = (0.48145466, 0.4578275, 0.40821073)
IMAGE_STD = (0.26862954, 0.26130258, 0.27577711)


def im2col_uint8(images, X, image_size, patch, mean=IMAGE_MEAN, std=IMAGE_STD):
    """uint8 images [B, H, W, 3] (channels last, H, W >= image_size: resized by resize_uint8
    first) -> normalised im2col rows in X [B*(G*G+1), 3*P*P]: CLIPImageProcessor's center_crop +
    rescale + normalize fused into patch-embed's im2col (one kernel, 1 B read per pixel value
    instead of 4)."""
    B, H, W, C = images.shape
    m = (c_float * 3)(*mean)
    sd = (c_float * 3)(*std)
    call("clipmi_im2col_u8", K.stream(), dcode(X.dtype), P_(images), P_(X), B, H, W, image_size, patch,
         X.shape[1], m, sd)
_lib.declare("clipmi_resize_u8_ws", [c_int, c_int, c_int, c_int, c_int], c_i64)
_lib.declare("clipmi_resize_u8", [c_vp, c_vp, c_int, c_int, c_int, c_vp, c_int, c_int, c_vp, c_i64])


def shortest_edge_size(h, w, size):
    """CLIPImageProcessor's output size (transformers get_resize_output_image_size,
    default_to_square=False): short edge -> size, long edge -> int(size * long / short)."""
    if w <= h:
        return int(size * h / w), size
    return size, int(size * w / h)


def resize_uint8(images, out_h, out_w):
    """CLIPImageProcessor's resize of uint8 [B, H, W, 3] (PIL bicubic, bit-exact) on the GPU
    (clipmi_resize_u8)."""
    B, H, W, C = images.shape
    out = torch.empty(B, out_h, out_w, C, dtype=torch.uint8, device=images.device)
    nb = int(_lib.lib().clipmi_resize_u8_ws(B, H, W, out_h, out_w))
    ws = torch.empty(max(nb, 16), dtype=torch.uint8, device=images.device)
    call("clipmi_resize_u8", K.stream(), P_(images), B, H, W, P_(out), out_h, out_w, P_(ws), nb)
    return out


_lib.declare("clipmi_adapter_fwd", [c_vp, c_int, c_int, c_int, c_int, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                    c_float, c_int, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp])
_lib.declare("clipmi_adapter_bwd_ws", [c_int, c_int, c_int], c_i64)
_lib.declare("clipmi_adapter_bwd", [c_vp, c_int, c_int, c_int, c_int, c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp,
                                    c_vp, c_vp, c_vp, c_vp, c_int, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                    c_i64])
_lib.declare("clipmi_pool_index", [c_vp, c_vp, c_int, c_int, c_i64, c_int, c_vp])
_lib.declare("clipmi_gather_rows", [c_vp, c_int, c_vp, c_vp, c_int, c_int, c_int, c_vp])
_lib.declare("clipmi_scatter_rows", [c_vp, c_int, c_vp, c_vp, c_int, c_int, c_int, c_vp, c_int])
_lib.declare("clipmi_attention_fwd", [c_vp, c_int, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int])
_lib.declare("clipmi_attention_bwd", [c_vp, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int,
                                      c_int])
_lib.declare("clipmi_split3_elems", [c_int, c_int, c_int], c_i64)
_lib.declare("clipmi_split3", [c_vp, c_vp, c_i64, c_int, c_int, c_int, c_vp, c_int])
_lib.declare("clipmi_split3_colsum_ws", [c_int, c_int], c_i64)
_lib.declare("clipmi_split3_colsum", [c_vp, c_vp, c_i64, c_int, c_int, c_vp, c_int, c_vp, c_int, c_vp, c_i64])
_lib.declare("clipmi_layernorm_fwd_x3", [c_vp, c_vp, c_i64, c_vp, c_int, c_vp, c_vp, c_vp, c_vp, c_int, c_int,
                                         ctypes.c_float])
_lib.declare("clipmi_attention_fwd_x3", [c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int])
_lib.declare("clipmi_attention_bwd_x3", [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int])
_lib.declare("clipmi_attention_fwd_x3img", [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int])
_lib.declare("clipmi_attention_bwd_x3img_ws", [c_int, c_int], c_i64)
_lib.declare("clipmi_attention_bwd_x3img", [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_vp, c_i64, c_vp, c_int,
                                            c_int, c_int, c_int, c_int])
_lib.declare("clipmi_attention_fwd_mxfp8", [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int])
_lib.declare("clipmi_l2norm_fwd", [c_vp, c_vp, c_vp, c_vp, c_int, c_int])
_lib.declare("clipmi_l2norm_bwd", [c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int])
_lib.declare("clipmi_contrastive_ce_fwd", [c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_vp, c_vp])
_lib.declare("clipmi_contrastive_ce_bwd", [c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_float, c_vp, c_vp])
_lib.declare("clipmi_sum2", [c_vp, c_vp, c_vp, c_int, c_float, c_vp, c_int])
_lib.declare("clipmi_contrastive_ce_fwd_chunk", [c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_vp, c_vp])
_lib.declare("clipmi_contrastive_ce_finish", [c_vp, c_vp, c_vp, c_int, c_vp, c_vp])
_lib.declare("clipmi_contrastive_ce_bwd_chunk", [c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int,
                                                 c_float, c_vp, c_vp, c_int])
_lib.declare("clipmi_cast_f32_bf16", [c_vp, c_vp, c_vp, c_i64])
_lib.declare("clipmi_grad_norm_ws", [], c_i64)
_lib.declare("clipmi_grad_norm", [c_vp, c_vp, c_i64, c_float, c_vp, c_vp, c_i64])
_lib.declare("clipmi_grad_scale", [c_vp, c_vp, c_i64, c_vp])
_lib.declare("clipmi_grad_norm_multi_ws", [c_int], c_i64)
_lib.declare("clipmi_grad_norm_multi", [c_vp, P(c_vp), P(c_i64), c_int, c_float, c_vp, c_vp, c_i64])
_lib.declare("clipmi_adamw", [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, ctypes.c_double, ctypes.c_double,
                              ctypes.c_double, ctypes.c_double, ctypes.c_double, c_int, c_vp])


def call(name, *args):
    _lib.check(getattr(_lib.lib(), name)(*args), name)


def P_(t):
    return None if t is None else t.data_ptr()


def dcode(dtype):
    return BF16 if dtype == torch.bfloat16 else F32


def _ws(nbytes, device):
    return torch.empty(max(int(nbytes), 16), dtype=torch.uint8, device=device)


def _gemm_f32(M, N, Kd, A, lda, akm, B, ldb, bkm, C, ldc, flags=0):
    """fp32 GEMM (the contrastive similarities and their gradients) split over K when its
    64x64 tiles would not fill two rounds of the CUs: at one GPU (B = Bg = 1024) the backward
    products have 128 tiles for 256 CUs."""
    tiles = ((M + 63) // 64) * ((N + 63) // 64)
    split = 1
    while split < 8 and tiles * split * 2 <= 512 and Kd // (split * 2) >= 128:
        split *= 2
    ws = torch.empty(split * M * N, dtype=torch.float32, device=C.device) if split > 1 else None
    K.gemm(M, N, Kd, A, lda, akm, B, ldb, bkm, C, ldc, flags=flags, split_k=split, workspace=ws)


# ------------------------------------------------------------------------------ encoder
class Encoder:
    """Binds one tower's encoder layers (an arena prefix) to the native engine."""

    def __init__(self, arena, prefix, tcfg, causal):
        self.arena, self.prefix, self.t, self.causal = arena, prefix, tcfg, causal
        self._wcache = {}

    def names(self, i):
        p = f"{self.prefix}.encoder.layers.{i}"
        return {"ln1_w": f"{p}.layer_norm1.weight", "ln1_b": f"{p}.layer_norm1.bias",
                "qkv_w": f"{p}.self_attn.q_proj.weight", "qkv_b": f"{p}.self_attn.q_proj.bias",
                "out_w": f"{p}.self_attn.out_proj.weight", "out_b": f"{p}.self_attn.out_proj.bias",
                "ln2_w": f"{p}.layer_norm2.weight", "ln2_b": f"{p}.layer_norm2.bias",
                "fc1_w": f"{p}.mlp.fc1.weight", "fc1_b": f"{p}.mlp.fc1.bias",
                "fc2_w": f"{p}.mlp.fc2.weight", "fc2_b": f"{p}.mlp.fc2.bias"}

    def _table(self, cls, buf):
        key = (cls.__name__, buf.data_ptr(), buf.dtype)
        tab = self._wcache.get(key)
        if tab is None:
            L = self.t.num_hidden_layers
            tab = (cls * L)()
            for i in range(L):
                for f, n in self.names(i).items():
                    setattr(tab[i], f, self.arena.ptr(n, buf))
            self._wcache[key] = tab
        return tab

    def weights(self, wbuf):
        return self._table(LayerW, wbuf)

    def grads(self):
        return self._table(LayerG, self.arena.grad)

    def alloc(self, B, N, dtype, device, train, resid32=False, x3=False):
        """Activation storage: per-layer for training, one shared set for inference.  resid32: the
        residual stream (x_in, h) in fp32 (the bf16 mode's fp32 residual stream).  x3 (the bf16x3 mode, fp32):
        ln1 / ln2 / act as bf16 split images [R, 3K] and o followed by its image (include/clipmi.h gemm_x3)."""
        t = self.t
        R, D, F, H, L = B * N, t.hidden_size, t.intermediate_size, t.num_attention_heads, t.num_hidden_layers
        es = 2 if dtype == torch.bfloat16 else 4
        xs = 4 if resid32 else es
        al = lambda n: (n + 255) // 256 * 256  # noqa: E731
        x3 = x3 and dtype == torch.float32
        ln_b = R * 3 * D * 2 if x3 else R * D * es
        o_b = al(R * D * 4) + R * 3 * D * 2 if x3 else R * D * es
        act_b = R * 3 * F * 2 if x3 else R * F * es
        parts = [("x_in", R * D * xs), ("ln1", ln_b), ("qkv", R * 3 * D * es), ("o", o_b),
                 ("h", R * D * xs), ("ln2", ln_b), ("act", act_b),
                 ("mean1", R * 4), ("rstd1", R * 4), ("lse", B * H * N * 4), ("mean2", R * 4), ("rstd2", R * 4)]
        if train:
            parts.append(("pre", R * F * es))
        per = sum(al(n) for _, n in parts)
        nsets = L if train else 1
        buf = torch.empty(per * nsets + 256, dtype=torch.uint8, device=device)
        acts = (LayerAct * L)()
        base = (buf.data_ptr() + 255) // 256 * 256
        for i in range(L):
            off = base + per * (i if train else 0)
            for name, n in parts:
                setattr(acts[i], name, off)
                off += al(n)
            if not train:
                acts[i].pre = None
        return buf, acts

    def weights8(self):
        """MXFP8 copies of the four GEMM weights of every layer (BASELINE config 5), quantised from
        the fp32 masters (clipmi_quant_mxfp8: e4m3 + one E8M0 scale per 32 inputs of an output row),
        rebuilt when the masters change."""
        a = self.arena
        key = ("w8", a.data.data_ptr(), a.data._version)
        hit = self._wcache.get("w8")
        if hit is not None and hit[0] == key:
            return hit[1]
        L = self.t.num_hidden_layers
        tab = (LayerW8 * L)()
        keep = []
        for i in range(L):
            n = self.names(i)
            D = self.t.hidden_size
            q0 = a.offsets[n["qkv_w"]][0]  # q/k/v weights are adjacent: the fused [3D, D] matrix
            for f, src in (("qkv", a.data[q0:q0 + 3 * D * D].view(3 * D, D)),
                           ("out", a.view(n["out_w"])), ("fc1", a.view(n["fc1_w"])), ("fc2", a.view(n["fc2_w"]))):
                m = K.quant_mxfp8(src.contiguous())
                keep.append(m)
                setattr(tab[i], f + "_w", m.q.data_ptr())
                setattr(tab[i], f + "_s", m.s.data_ptr())
        self._wcache["w8"] = (key, tab, keep)
        return tab

    def desc(self, dtype, B, N, wbuf, acts, x_out, mask, grads=None, ws=None, fp8=False, resid32=False, x3=False):
        """x3: the bf16x3 mode (fp32 encoder, every GEMM a split-operand bf16 product); its split-image
        scratch is allocated here and lives as long as the returned descriptor (d.x3_keep)."""
        t = self.t
        d = EncoderDesc()
        d.dtype, d.B, d.N, d.D, d.F = dcode(dtype), B, N, t.hidden_size, t.intermediate_size
        d.resid_f32 = int(resid32 and not fp8)
        if fp8:  # bf16 activations, MXFP8 GEMMs (forward only)
            d.dtype = _lib.FP8
            d.layers8 = self.weights8()
            R, Dh, F = B * N, t.hidden_size, t.intermediate_size
            q8 = torch.empty(R * (Dh + F) + 512, dtype=torch.uint8, device=self.arena.device)
            s8 = torch.empty(R * (Dh + F) // 32 + 512, dtype=torch.uint8, device=self.arena.device)
            self._scratch8 = (q8, s8)  # alive until the next call; stream order covers reuse
            d.q8, d.s8 = q8.data_ptr(), s8.data_ptr()
        d.H, d.L, d.eps, d.causal = t.num_attention_heads, t.num_hidden_layers, t.layer_norm_eps, int(self.causal)
        d.attention_mask = P_(mask)
        d.layers = self.weights(wbuf)
        d.grads = grads
        d.act = acts
        d.x_out = x_out
        if ws is not None:
            d.workspace, d.workspace_bytes = ws.data_ptr(), ws.numel()
        if x3 and dtype == torch.float32:
            d.gemm_x3 = 1
            d.x3_keep = _ws(_lib.lib().clipmi_encoder_x3_ws(ctypes.byref(d)), self.arena.device)
            d.x3_ws, d.x3_ws_bytes = d.x3_keep.data_ptr(), d.x3_keep.numel()
        return d


    def layer_range(self, lo, hi):
        """(offset, numel) of layers lo..hi-1 in the arena: each layer's parameters are one
        contiguous block (modules.layer_specs), consecutive layers adjacent."""
        a = self.arena
        start = a.offsets[f"{self.prefix}.encoder.layers.{lo}.layer_norm1.weight"][0]
        off, _, n = a.offsets[f"{self.prefix}.encoder.layers.{hi - 1}.mlp.fc2.bias"]
        return start, off + n - start

    def backward(self, s, d, dx, hook):
        """Encoder backward (layers L-1 .. 0).  With a gradient-ready hook (data-parallel runs)
        it runs in chunks of layers and reports each chunk's gradient slice as soon as its
        kernels are queued, so the all-reduce of the upper layers overlaps the lower layers'
        backward; without one it is a single native call."""
        L = self.t.num_hidden_layers
        if hook is None:
            _lib.check(_lib.lib().clipmi_encoder_bwd(s, ctypes.byref(d), dx), "clipmi_encoder_bwd")
            return
        step = max(1, (L + 3) // 4)
        hi = L
        while hi > 0:
            lo = max(0, hi - step)
            _lib.check(_lib.lib().clipmi_encoder_bwd_layers(s, ctypes.byref(d), dx, hi, lo), "clipmi_encoder_bwd_layers")
            off, n = self.layer_range(lo, hi)
            hook(self.arena, off, n)
            hi = lo


def _grad_hook(rt):
    """The data-parallel gradient-ready hook (trainer.GradBucketReducer.ready) when one is active."""
    return getattr(rt, "grad_hook", None)


def _wbuf(arena, dtype):
    if dtype == torch.bfloat16:
        arena.sync_shadow()
        return arena.shadow
    return arena.data


# ------------------------------------------------------------------------------ vision
class VisionTowerFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pixel_values, anchor, runtime):
        rt = runtime
        arena, v, dtype = rt.arena, rt.cfg.vision_config, rt.dtype
        B = pixel_values.shape[0]
        raw = pixel_values.dtype == torch.uint8  # decoded images, channels last: fused input step
        if raw:
            if pixel_values.dim() != 4 or pixel_values.shape[3] != v.num_channels:
                raise ValueError(f"uint8 images must be [B, H, W, {v.num_channels}] (channels last)")
            H, W = pixel_values.shape[1], pixel_values.shape[2]
        else:
            if pixel_values.dim() != 4 or pixel_values.shape[1] != v.num_channels:
                raise ValueError(f"pixel_values must be [B, {v.num_channels}, H, W]")
            H, W = pixel_values.shape[2], pixel_values.shape[3]
            if H != v.image_size or W != v.image_size:
                raise ValueError(f"Input image size ({H}*{W}) doesn't match model ({v.image_size}*{v.image_size}).")
        dev = pixel_values.device
        px = pixel_values.contiguous() if raw else pixel_values.to(torch.float32).contiguous()
        if raw:  # CLIPImageProcessor: resize the shortest edge to the image size, then center-crop
            oh, ow = shortest_edge_size(H, W, v.image_size)
            if (oh, ow) != (H, W):
                px = resize_uint8(px, oh, ow)
                H, W = oh, ow
        N, D, Pp = v.num_positions, v.hidden_size, v.patch_size
        Kc = v.num_channels * Pp * Pp
        # patch K padded to a multiple of 64 (ViT-L/14: 588 -> 640) so both GEMM operands are
        # 16-B aligned k-major rows the 256x256 LDS-DMA kernel takes; the pad columns are zero
        # in the im2col rows and in the weight copy, so they add nothing
        Kp = (Kc + 63) // 64 * 64 if Kc % 8 else Kc
        R = B * N
        train = rt.train_tower
        s = K.stream()
        wbuf = _wbuf(arena, dtype)
        dc = dcode(dtype)
        X = torch.empty(R, Kp, dtype=dtype, device=dev)
        if raw:
            im2col_uint8(px, X, v.image_size, Pp)
        else:
            call("clipmi_im2col", s, dc, P_(px), P_(X), B, v.num_channels, H, Pp, Kp)
        # the fp32 residual stream (bf16 mode): the patch product, the embedding sum and pre_layrnorm in
        # fp32 (fp32 master position / class / LN parameters), so layer 0's input is fp32 like every
        # later layer's; the patch GEMM's operands stay bf16
        fp8 = rt.fp8 and not train
        r32 = getattr(rt, "resid32", False) and not fp8
        xdtype = torch.float32 if r32 else dtype
        ebuf = arena.data if r32 else wbuf
        h0 = torch.empty(R, D, dtype=xdtype, device=dev)
        Wp = arena.view("vision_model.embeddings.patch_embedding.weight", wbuf).view(D, Kc)
        if Kp != Kc:
            Wp = torch.nn.functional.pad(Wp, (0, Kp - Kc))
        x3 = getattr(rt, "x3", False)  # bf16x3 mode: the patch product split too
        K.gemm(R, D, Kp, X, Kp, True, Wp, Kp, True, h0, D, split3=x3)
        buf, acts = rt.venc.alloc(B, N, dtype, dev, train, resid32=r32, x3=x3)
        stats0 = torch.empty(2, R, dtype=torch.float32, device=dev)
        call("clipmi_layernorm_fwd", s, dcode(xdtype), P_(h0), D, acts[0].x_in, D,
             arena.ptr("vision_model.pre_layrnorm.weight", ebuf), arena.ptr("vision_model.pre_layrnorm.bias", ebuf),
             P_(stats0[0]), P_(stats0[1]), R, D, v.layer_norm_eps,
             arena.ptr("vision_model.embeddings.position_embedding.weight", ebuf),
             arena.ptr("vision_model.embeddings.class_embedding", ebuf), N)
        out = torch.empty(B, N, D, dtype=xdtype, device=dev)
        d = rt.venc.desc(dtype, B, N, wbuf, acts, out.data_ptr(), None, fp8=fp8, resid32=r32, x3=x3)
        _lib.check(_lib.lib().clipmi_encoder_fwd(s, ctypes.byref(d)), "clipmi_encoder_fwd")
        del d
        if train:
            ctx.rt, ctx.B, ctx.buf, ctx.acts, ctx.X, ctx.h0, ctx.stats0 = rt, B, buf, acts, X, h0, stats0
            ctx.r32 = r32
        else:
            del buf
        return out

    @staticmethod
    def backward(ctx, dout):
        rt = ctx.rt
        arena, v, dtype = rt.arena, rt.cfg.vision_config, rt.dtype
        B, N, D = ctx.B, v.num_positions, v.hidden_size
        R = B * N
        dev = dout.device
        s = K.stream()
        dc = dcode(dtype)
        arena.prepare_grads()
        wbuf = _wbuf(arena, dtype)
        dx = dout.to(dtype).contiguous().clone()
        x3 = getattr(rt, "x3", False)
        d = rt.venc.desc(dtype, B, N, wbuf, ctx.acts, None, None, grads=rt.venc.grads(), resid32=ctx.r32, x3=x3)
        ws = _ws(_lib.lib().clipmi_encoder_bwd_ws(ctypes.byref(d)), dev)
        d.workspace, d.workspace_bytes = ws.data_ptr(), ws.numel()
        hook = _grad_hook(rt)
        rt.venc.backward(s, d, dx.data_ptr(), hook)
        del d, ws  # the workspaces return to the stream-ordered pool
        # pre_layrnorm backward -> gradient of the embedding sum h0 (h0 fp32 with the fp32 residual stream;
        # the gradients stay in the activation dtype)
        dh0 = torch.empty(R, D, dtype=dtype, device=dev)
        lws = _ws(_lib.lib().clipmi_layernorm_bwd_ws(R, D), dev)
        g = arena.grad
        # the forward's gamma: the fp32 master with the fp32 residual stream, else the shadow
        wdc = dcode(torch.float32) if ctx.r32 else dc
        gamma = arena.ptr("vision_model.pre_layrnorm.weight", arena.data if ctx.r32 else wbuf)
        call("clipmi_layernorm_bwd3", s, dcode(ctx.h0.dtype), dc, wdc, P_(dx), D, P_(ctx.h0), D, P_(ctx.stats0[0]),
             P_(ctx.stats0[1]), gamma, P_(dh0), D, None, 0,
             arena.ptr("vision_model.pre_layrnorm.weight", g), arena.ptr("vision_model.pre_layrnorm.bias", g), 1,
             P_(lws), lws.numel(), R, D)
        Kp, Kc = ctx.X.shape[1], v.num_channels * v.patch_size ** 2
        gW = arena.view("vision_model.embeddings.patch_embedding.weight", g).view(D, Kc)
        if Kp != Kc:  # padded patch K: accumulate the [D, Kp] product's first Kc columns
            gW_arena, gW = gW, torch.zeros(D, Kp, dtype=gW.dtype, device=dev)
        if x3:  # the bf16 256-tile kernel over 3R: about one round of workgroups
            splits = max(1, min(64, 256 // max(1, ((D + 255) // 256) * ((Kp + 255) // 256))))
            while splits > 1 and 3 * R // splits < 512:
                splits -= 1
        else:
            splits = max(1, min(32, 1024 // max(1, ((D + 127) // 128) * ((Kp + 127) // 128))))
            while splits > 1 and R // splits < 512:
                splits -= 1
        wsp = _ws(splits * D * Kp * 4, dev) if splits > 1 and not x3 else None
        K.gemm(D, Kp, R, dh0, D, False, ctx.X, Kp, False, gW, Kp, flags=_lib.EPI_BETA, split_k=splits,
               workspace=wsp, split3=x3)
        if Kp != Kc:
            gW_arena.add_(gW[:, :Kc])
        call("clipmi_period_sum", s, dc, P_(dh0), D, B, N, N, D,
             arena.ptr("vision_model.embeddings.position_embedding.weight", g), 1)
        call("clipmi_period_sum", s, dc, P_(dh0), D, B, N, 1, D, arena.ptr("vision_model.embeddings.class_embedding", g), 1)
        # class / patch / position embeddings + pre_layrnorm: one contiguous block.  Not final when
        # a shared adapter still has to add its position-embedding gradient (its backward runs
        # after this one): the reducer's finish() then takes the block
        if hook is not None and not getattr(rt, "shared_pos_grad", False):
            lo = arena.offsets["vision_model.embeddings.class_embedding"][0]
            hi = arena.offsets["vision_model.encoder.layers.0.layer_norm1.weight"][0]
            hook(arena, lo, hi - lo)
        # activations are released with backward, not with the graph object (a caller holding
        # last step's loss would otherwise keep them alive into the next forward: 2x memory and
        # fresh device mallocs mid-step); stream-ordered reuse keeps the queued kernels safe
        ctx.buf = ctx.acts = ctx.X = ctx.h0 = ctx.stats0 = None
        return None, None, None


# ------------------------------------------------------------------------------ text
class TextTowerFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, input_ids, attention_mask, anchor, runtime):
        rt = runtime
        arena, t, dtype = rt.arena, rt.cfg.text_config, rt.dtype
        B, S = input_ids.shape
        if S > t.max_position_embeddings:
            raise ValueError(f"Sequence length must be less than max_position_embeddings (got `sequence length`: "
                             f"{S} and max_position_embeddings: {t.max_position_embeddings}")
        dev = input_ids.device
        ids = input_ids.to(torch.int64).contiguous()
        mask = attention_mask.to(device=dev, dtype=torch.int64).contiguous() if attention_mask is not None else None
        D = t.hidden_size
        R = B * S
        train = rt.train_tower
        s = K.stream()
        dc = dcode(dtype)
        wbuf = _wbuf(arena, dtype)
        fp8 = rt.fp8 and not train
        r32 = getattr(rt, "resid32", False) and not fp8  # the fp32 residual stream (bf16 mode)
        xdtype = torch.float32 if r32 else dtype
        buf, acts = rt.tenc.alloc(B, S, dtype, dev, train, resid32=r32, x3=getattr(rt, "x3", False))
        bad = rt.bad_flag
        ebuf = arena.data if r32 else wbuf  # fp32 token / position embeddings into the fp32 stream
        call("clipmi_text_embed", s, dcode(xdtype), P_(ids), arena.ptr("text_model.embeddings.token_embedding.weight", ebuf),
             arena.ptr("text_model.embeddings.position_embedding.weight", ebuf), acts[0].x_in, R, S, D, t.vocab_size,
             P_(bad))
        xL = torch.empty(R, D, dtype=xdtype, device=dev)
        d = rt.tenc.desc(dtype, B, S, wbuf, acts, xL.data_ptr(), mask, fp8=fp8, resid32=r32,
                         x3=getattr(rt, "x3", False))
        _lib.check(_lib.lib().clipmi_encoder_fwd(s, ctypes.byref(d)), "clipmi_encoder_fwd")
        del d
        out = torch.empty(B, S, D, dtype=dtype, device=dev)
        stats = torch.empty(2, R, dtype=torch.float32, device=dev)
        call("clipmi_layernorm_fwd2", s, dcode(xdtype), dc, P_(xL), D, P_(out), D,
             arena.ptr("text_model.final_layer_norm.weight", wbuf), arena.ptr("text_model.final_layer_norm.bias", wbuf),
             P_(stats[0]), P_(stats[1]), R, D, t.layer_norm_eps, None, None, 0)
        if train:
            ctx.rt, ctx.B, ctx.S, ctx.buf, ctx.acts = rt, B, S, buf, acts
            ctx.ids, ctx.mask, ctx.xL, ctx.stats, ctx.r32 = ids, mask, xL, stats, r32
        return out

    @staticmethod
    def backward(ctx, dout):
        rt = ctx.rt
        arena, t, dtype = rt.arena, rt.cfg.text_config, rt.dtype
        B, S, D = ctx.B, ctx.S, t.hidden_size
        R = B * S
        dev = dout.device
        s = K.stream()
        dc = dcode(dtype)
        arena.prepare_grads()
        wbuf = _wbuf(arena, dtype)
        g = arena.grad
        dy = dout.to(dtype).contiguous()
        dx = torch.empty(R, D, dtype=dtype, device=dev)
        lws = _ws(_lib.lib().clipmi_layernorm_bwd_ws(R, D), dev)
        call("clipmi_layernorm_bwd2", s, dcode(ctx.xL.dtype), dc, P_(dy), D, P_(ctx.xL), D, P_(ctx.stats[0]),
             P_(ctx.stats[1]), arena.ptr("text_model.final_layer_norm.weight", wbuf), P_(dx), D, None, 0,
             arena.ptr("text_model.final_layer_norm.weight", g), arena.ptr("text_model.final_layer_norm.bias", g), 1,
             P_(lws), lws.numel(), R, D)
        d = rt.tenc.desc(dtype, B, S, wbuf, ctx.acts, None, ctx.mask, grads=rt.tenc.grads(), resid32=ctx.r32,
                         x3=getattr(rt, "x3", False))
        ws = _ws(_lib.lib().clipmi_encoder_bwd_ws(ctypes.byref(d)), dev)
        d.workspace, d.workspace_bytes = ws.data_ptr(), ws.numel()
        hook = _grad_hook(rt)
        rt.tenc.backward(s, d, dx.data_ptr(), hook)
        del d, ws
        V = t.vocab_size
        ews = _ws(_lib.lib().clipmi_text_embed_bwd_ws(R, V), dev)
        call("clipmi_text_embed_bwd", s, dc, P_(ctx.ids), P_(dx), R, D, V,
             arena.ptr("text_model.embeddings.token_embedding.weight", g), 1, P_(ews), ews.numel())
        call("clipmi_period_sum", s, dc, P_(dx), D, B, S, S, D,
             arena.ptr("text_model.embeddings.position_embedding.weight", g), 1)
        if hook is not None:  # token + position embeddings: the arena's first block
            hook(arena, 0, arena.offsets["text_model.encoder.layers.0.layer_norm1.weight"][0])
        ctx.buf = ctx.acts = ctx.xL = ctx.stats = None  # released with backward (see VisionTowerFn)
        return None, None, None, None


# ------------------------------------------------------------------------------ adapter
class AdapterFn(torch.autograd.Function):
    """y = LN(up(gelu(down(x))) + x)  (ln=False: up(gelu(down(x))) + x).

    One C-ABI call per direction (csrc/adapter.cpp): clipmi_adapter_fwd runs the down GEMM (+ bias +
    gelu_erf, pre-activation saved), the up GEMM (+ bias + residual) and the LayerNorm kernel;
    clipmi_adapter_bwd runs LN' and the four GEMMs (fused bias gradients in bf16).  The same entry
    points are the FFI binding of INTEGRATION.md, so the Python mirror and an FFI caller run one path."""

    @staticmethod
    def forward(ctx, x, anchor, runtime, mod, need):
        arena, dtype = mod.arena, runtime.dtype
        shp = x.shape
        Dh, A = mod.hidden, mod.bottleneck
        x2 = x.to(dtype).reshape(-1, Dh).contiguous()
        R = x2.shape[0]
        dev = x.device
        s = K.stream()
        dc = dcode(dtype)
        wbuf = _wbuf(arena, dtype)
        dn, up = mod.names
        pre = torch.empty(R, A, dtype=dtype, device=dev) if need else None
        act = torch.empty(R, A, dtype=dtype, device=dev)
        y = torch.empty(R, Dh, dtype=dtype, device=dev)
        z = torch.empty(R, Dh, dtype=dtype, device=dev) if mod.has_ln else None
        stats = torch.empty(2, R, dtype=torch.float32, device=dev) if mod.has_ln else None
        ln_ptr = (lambda n: arena.ptr(n, wbuf)) if mod.has_ln else (lambda n: None)
        call("clipmi_adapter_fwd", s, dc, R, Dh, A, P_(x2), Dh, arena.ptr(f"{dn}.weight", wbuf),
             arena.ptr(f"{dn}.bias", wbuf), arena.ptr(f"{up}.weight", wbuf), arena.ptr(f"{up}.bias", wbuf),
             ln_ptr("layer_norm.weight"), ln_ptr("layer_norm.bias"), 1e-5, int(mod.has_ln), P_(y), Dh, P_(pre),
             P_(act), P_(z), P_(stats[0]) if stats is not None else None,
             P_(stats[1]) if stats is not None else None)
        if need:
            ctx.save = (x2, pre, act, z, stats)
            ctx.mod, ctx.rt, ctx.shape = mod, runtime, shp
        return y.view(shp)

    @staticmethod
    def backward(ctx, dy):
        mod, rt = ctx.mod, ctx.rt
        x2, pre, act, z, stats = ctx.save
        arena, dtype = mod.arena, rt.dtype
        Dh, A = mod.hidden, mod.bottleneck
        R = x2.shape[0]
        dev = dy.device
        s = K.stream()
        dc = dcode(dtype)
        train_params = arena.any_requires_grad()
        if train_params:
            arena.prepare_grads()
        g = arena.grad
        wbuf = _wbuf(arena, dtype)
        dn, up = mod.names
        dy2 = dy.to(dtype).reshape(R, Dh).contiguous()
        dx = torch.empty(R, Dh, dtype=dtype, device=dev)
        gp = (lambda n: arena.ptr(n, g)) if train_params else (lambda n: None)
        lnp = gp if mod.has_ln else (lambda n: None)
        ws = _ws(_lib.lib().clipmi_adapter_bwd_ws(R, Dh, A), dev)
        call("clipmi_adapter_bwd", s, dc, R, Dh, A, P_(dy2), Dh, P_(x2), Dh, P_(pre), P_(act), P_(z),
             P_(stats[0]) if stats is not None else None, P_(stats[1]) if stats is not None else None,
             arena.ptr(f"{dn}.weight", wbuf), arena.ptr(f"{up}.weight", wbuf),
             arena.ptr("layer_norm.weight", wbuf) if mod.has_ln else None, int(mod.has_ln), P_(dx), Dh,
             gp(f"{dn}.weight"), gp(f"{dn}.bias"), gp(f"{up}.weight"), gp(f"{up}.bias"),
             lnp("layer_norm.weight"), lnp("layer_norm.bias"), P_(ws), ws.numel())
        ctx.save = None  # released with backward (see VisionTowerFn)
        return dx.view(ctx.shape), None, None, None, None


# ------------------------------------------------------------------------------ pool + projection
class PoolProjFn(torch.autograd.Function):
    """features[b] = W @ h[b, idx[b]]  (fp32 out).  idx None -> token 0 (model_m.py:102,122)."""

    @staticmethod
    def forward(ctx, h, anchor, runtime, wname, idx):
        arena, dtype = runtime.arena, runtime.dtype
        B, S, D = h.shape
        dev = h.device
        s = K.stream()
        dc = dcode(dtype)
        wbuf = _wbuf(arena, dtype)
        W = arena.view(wname, wbuf)
        E = W.shape[0]
        if W.shape[1] != D:  # F.linear's error for the reference's text_projection(x) (model_m.py:103)
            raise RuntimeError(f"mat1 and mat2 shapes cannot be multiplied ({B}x{D} and {W.shape[1]}x{E})")
        # gather the pooled rows in h's own dtype (the vision tower's fp32 residual stream), then cast
        # the B rows (not the whole [B, S, D] tensor) to the GEMM operand dtype
        hd = h.dtype if h.dtype in (torch.float32, torch.bfloat16) else dtype
        hc = h.to(hd).contiguous()
        pooled = torch.empty(B, D, dtype=hd, device=dev)
        call("clipmi_gather_rows", s, dcode(hd), P_(hc), P_(idx), B, S, D, P_(pooled))
        pooled = pooled.to(dtype)
        out = torch.empty(B, E, dtype=torch.float32, device=dev)
        K.gemm(B, E, D, pooled, D, True, W, D, True, out, E)
        ctx.save = (pooled, idx)
        ctx.rt, ctx.wname, ctx.shape, ctx.hdtype = runtime, wname, (B, S, D), hd
        return out

    @staticmethod
    def backward(ctx, dout):
        rt = ctx.rt
        arena, dtype = rt.arena, rt.dtype
        pooled, idx = ctx.save
        B, S, D = ctx.shape
        dev = dout.device
        s = K.stream()
        dc = dcode(dtype)
        wbuf = _wbuf(arena, dtype)
        W = arena.view(ctx.wname, wbuf)
        E = W.shape[0]
        d = dout.to(torch.float32).contiguous()
        if dtype == torch.bfloat16:
            d16 = torch.empty(B, E, dtype=dtype, device=dev)
            call("clipmi_cast_f32_bf16", s, P_(d), P_(d16), B * E)
            d = d16
        if arena.params[ctx.wname].requires_grad:
            arena.prepare_grads()
            K.gemm(E, D, B, d, E, False, pooled, D, False, arena.view(ctx.wname, arena.grad), D, flags=_lib.EPI_BETA)
        dpooled = torch.empty(B, D, dtype=dtype, device=dev)
        K.gemm(B, D, E, d, E, True, W, D, False, dpooled, D)
        # the gradient in h's dtype (autograd would otherwise cast the whole [B, S, D] tensor)
        dpooled = dpooled.to(ctx.hdtype)
        dh = torch.zeros(B, S, D, dtype=ctx.hdtype, device=dev)
        call("clipmi_scatter_rows", s, dcode(ctx.hdtype), P_(dpooled), P_(idx), B, S, D, P_(dh), 0)
        ctx.save = None
        return dh, None, None, None, None


class PoolRowsFn(torch.autograd.Function):
    """[B, S, D] -> [B, 1, D]: the pooled token of each sequence (idx None -> token 0), gathered
    by clipmi_gather_rows; backward scatters the row gradients into zeros (clipmi_scatter_rows).
    Lets the row-wise adapters run on the pooled rows only (model_m.py:102,122)."""

    @staticmethod
    def forward(ctx, h, runtime, idx):
        dtype = runtime.dtype
        B, S, D = h.shape
        hd = h.dtype if h.dtype in (torch.float32, torch.bfloat16) else dtype  # gathered in h's own dtype
        hc = h.to(hd).contiguous()
        out = torch.empty(B, 1, D, dtype=hd, device=h.device)
        call("clipmi_gather_rows", K.stream(), dcode(hd), P_(hc), P_(idx), B, S, D, P_(out))
        ctx.rt, ctx.idx, ctx.shape, ctx.hdtype = runtime, idx, (B, S, D), hd
        return out.to(dtype)

    @staticmethod
    def backward(ctx, dout):
        hd = ctx.hdtype
        B, S, D = ctx.shape
        d = dout.to(hd).contiguous()
        dh = torch.zeros(B, S, D, dtype=hd, device=dout.device)
        call("clipmi_scatter_rows", K.stream(), dcode(hd), P_(d), P_(ctx.idx), B, S, D, P_(dh), 0)
        return dh, None, None


# ------------------------------------------------------------------------------ contrastive
def _rccl(group):
    return dist.get_backend(group) == "nccl"


# The data-parallel group is a torch.distributed group (RCCL through torch, or gloo) or a clipmi.comm.Communicator
# (RCCL issued by libclipmi: clipmi_allgather_embed / clipmi_reducescatter_grad / clipmi_allreduce on the caller's
# stream).


def force_collectives():
    """CLIPMI_DP_FORCE_COLLECTIVES=1 (tests only): a one-rank group still takes the collective branches
    (all-gather, reduce-scatter, bucketed all-reduce), each then the identity, so a one-GPU box runs
    the RCCL code paths (tests/test_gpu_dp.py)."""
    return os.environ.get("CLIPMI_DP_FORCE_COLLECTIVES") == "1"


def _gather(x, group, world):
    """All-gather rows over the group (RCCL all_gather_into_tensor; list form for gloo)."""
    if world == 1 and not (group is not None and force_collectives()):
        return x
    x = x.contiguous()
    if CM.is_lib(group):
        return group.all_gather(x)
    if _rccl(group):
        out = torch.empty(world * x.shape[0], *x.shape[1:], dtype=x.dtype, device=x.device)
        dist.all_gather_into_tensor(out, x, group=group)
        return out
    parts = [torch.empty_like(x) for _ in range(world)]
    dist.all_gather(parts, x, group=group)
    return torch.cat(parts)


def _reduce_scatter(x, group, world):
    """Sum over the group, keep this rank's row block (RCCL reduce_scatter_tensor; gloo:
    all_reduce + slice, which gloo supports for device tensors)."""
    if world == 1 and not (group is not None and force_collectives()):
        return x
    x = x.contiguous()
    n = x.shape[0] // world
    if CM.is_lib(group):
        return group.reduce_scatter(x)
    if _rccl(group):
        out = torch.empty(n, *x.shape[1:], dtype=x.dtype, device=x.device)
        dist.reduce_scatter_tensor(out, x, group=group)
        return out
    y = x.clone()
    dist.all_reduce(y, group=group)
    r = dist.get_rank(group)
    return y[r * n:(r + 1) * n].contiguous()


def contrastive_chunk(world=2):
    """Columns per chunk of the column-streamed contrastive (CLIPMI_CE_CHUNK, default 8192): a
    data-parallel global batch wider than this is never materialised as [B, Bg] blocks (BASELINE
    config 5: Bg = 32768 at B = 4096 per GPU would be four 512 MiB fp32 blocks); at config 3
    (Bg <= 8192) the whole block is one chunk and the plain path runs.  On one device the logits
    are always materialised unless CLIPMI_CE_CHUNK is set explicitly: the reference's forward
    returns logits_per_text / logits_per_image (model_m.py:165-176), and callers index them."""
    env = os.environ.get("CLIPMI_CE_CHUNK")
    if env is None and world == 1:
        return 1 << 62
    return max(1, int(env or "8192"))


def _ce_streamed_fwd(s, x_local, y_all, ls, lab0, C, lse, ce):
    """Row-wise CE of logits = exp(ls) * x_local y_all^T over column chunks of width C."""
    B, E = x_local.shape
    Bg = y_all.shape[0]
    dev = x_local.device
    sbuf = torch.empty(B * min(C, Bg), dtype=torch.float32, device=dev)
    run = torch.empty(B, 2, dtype=torch.float32, device=dev)
    lab = torch.empty(B, dtype=torch.float32, device=dev)
    for c0 in range(0, Bg, C):
        cw = min(C, Bg - c0)
        _gemm_f32(B, cw, E, x_local, E, True, y_all[c0:], E, True, sbuf, cw)
        call("clipmi_contrastive_ce_fwd_chunk", s, P_(sbuf), P_(ls), B, cw, c0, Bg, lab0, P_(run), P_(lab))
    call("clipmi_contrastive_ce_finish", s, P_(run), P_(lab), B, P_(lse), P_(ce))


def _ce_streamed_bwd(s, x_local, y_all, ls, gl, lse, lab0, norm, C, dls, dy_all, dx_local):
    """Gradients of the streamed CE: dy_all[j] = sum_i dS[i, j] x_local[i] (column direction,
    every chunk writes its own rows) and dx_local = sum_j dS[:, j] y_all[j] (row direction,
    accumulated over the chunks), recomputing each chunk's cosines."""
    B, E = x_local.shape
    Bg = y_all.shape[0]
    dev = x_local.device
    sbuf = torch.empty(B * min(C, Bg), dtype=torch.float32, device=dev)
    dbuf = torch.empty_like(sbuf)
    for n, c0 in enumerate(range(0, Bg, C)):
        cw = min(C, Bg - c0)
        _gemm_f32(B, cw, E, x_local, E, True, y_all[c0:], E, True, sbuf, cw)
        call("clipmi_contrastive_ce_bwd_chunk", s, P_(sbuf), P_(lse), P_(ls), P_(gl), B, cw, c0, Bg, lab0, norm,
             P_(dbuf), P_(dls), 1 if n else 0)
        _gemm_f32(cw, E, B, dbuf, cw, False, x_local, E, False, dy_all[c0:], E)
        _gemm_f32(B, E, cw, dbuf, cw, True, y_all[c0:], E, False, dx_local, E, flags=_lib.EPI_BETA if n else 0)


class ContrastiveFn(torch.autograd.Function):
    """Symmetric InfoNCE.  Single device: exactly model_m.py:146-171.  With a process group
    of W ranks: all-gather the normalised features, each rank scores its B rows
    against all Bg = W*B columns with label offset rank*B, loss normalised by 2*Bg (so the
    all-reduced sum is the global loss), feature gradients reduce-scattered back.  When Bg
    exceeds contrastive_chunk() the score blocks are streamed by column chunks (online
    log-sum-exp forward, chunk recompute backward) and the logits outputs are None."""

    @staticmethod
    def forward(ctx, tf, imf, logit_scale, group, global_loss, arena):
        world, rank = CM.world_rank(group)
        B, E = tf.shape
        dev = tf.device
        s = K.stream()
        t = tf.to(torch.float32).contiguous()
        i = imf.to(torch.float32).contiguous()
        th, ih = torch.empty_like(t), torch.empty_like(i)
        tn = torch.empty(B, dtype=torch.float32, device=dev)
        inn = torch.empty(B, dtype=torch.float32, device=dev)
        call("clipmi_l2norm_fwd", s, P_(t), P_(th), P_(tn), B, E)
        call("clipmi_l2norm_fwd", s, P_(i), P_(ih), P_(inn), B, E)
        tg, ig = _gather(th, group, world), _gather(ih, group, world)
        Bg = tg.shape[0]
        C = contrastive_chunk(world)
        ls = logit_scale.detach().reshape(1)
        lab0 = rank * B
        if Bg > C:
            lse = torch.empty(2, B, dtype=torch.float32, device=dev)
            ce = torch.empty(2, B, dtype=torch.float32, device=dev)
            _ce_streamed_fwd(s, th, ig, ls, lab0, C, lse[0], ce[0])
            _ce_streamed_fwd(s, ih, tg, ls, lab0, C, lse[1], ce[1])
            loss = torch.empty((), dtype=torch.float32, device=dev)
            call("clipmi_sum2", s, P_(ce[0]), P_(ce[1]), B, 1.0 / (2 * Bg), P_(loss), 0)
            loss_out = loss
            if world > 1 and global_loss:
                loss_out = CM.all_reduce_(loss.clone(), group)
            ctx.save_for_backward(th, ih, tn, inn, tg, ig, lse, ls)
            ctx.group, ctx.world, ctx.B, ctx.Bg, ctx.lab0, ctx.chunk = group, world, B, Bg, lab0, C
            ctx.ls_param, ctx.arena = logit_scale, arena
            return loss_out, th, ih, None, None
        ctx.chunk = None
        lt = torch.empty(B, Bg, dtype=torch.float32, device=dev)
        li = torch.empty(B, Bg, dtype=torch.float32, device=dev)
        _gemm_f32(B, Bg, E, th, E, True, ig, E, True, lt, Bg)   # cos(t_local, i_all)
        _gemm_f32(B, Bg, E, ih, E, True, tg, E, True, li, Bg)   # cos(i_local, t_all)
        lse = torch.empty(2, B, dtype=torch.float32, device=dev)
        ce = torch.empty(2, B, dtype=torch.float32, device=dev)
        call("clipmi_contrastive_ce_fwd", s, P_(lt), P_(lt), P_(ls), B, Bg, lab0, P_(lse[0]), P_(ce[0]))
        call("clipmi_contrastive_ce_fwd", s, P_(li), P_(li), P_(ls), B, Bg, lab0, P_(lse[1]), P_(ce[1]))
        loss = torch.empty((), dtype=torch.float32, device=dev)
        call("clipmi_sum2", s, P_(ce[0]), P_(ce[1]), B, 1.0 / (2 * Bg), P_(loss), 0)
        if world > 1 and global_loss:
            loss_out = CM.all_reduce_(loss.clone(), group)
        else:
            loss_out = loss
        # outputs (th, ih, lt, li) must go through save_for_backward: keeping them as plain ctx
        # attributes forms node -> ctx -> output -> grad_fn -> node, a cycle that leaks the graph
        ctx.save_for_backward(th, ih, tn, inn, tg, ig, lt, li, lse, ls)
        ctx.group, ctx.world, ctx.B, ctx.Bg, ctx.lab0 = group, world, B, Bg, lab0
        ctx.ls_param, ctx.arena = logit_scale, arena
        ctx.mark_non_differentiable(lt, li)
        return loss_out, th, ih, lt, li

    @staticmethod
    def backward(ctx, gloss, gth, gih, glt, gli):
        if ctx.chunk is not None:
            return ContrastiveFn._backward_streamed(ctx, gloss, gth, gih)
        th, ih, tn, inn, tg, ig, lt, li, lse, ls = ctx.saved_tensors
        B, Bg, E, world = ctx.B, ctx.Bg, th.shape[1], ctx.world
        dev = th.device
        s = K.stream()
        gl = gloss.to(torch.float32).contiguous().reshape(1) if gloss is not None else None
        dSt = torch.empty(B, Bg, dtype=torch.float32, device=dev)
        dSi = torch.empty(B, Bg, dtype=torch.float32, device=dev)
        dls = torch.empty(2, B, dtype=torch.float32, device=dev)
        norm = 1.0 / (2 * Bg)
        call("clipmi_contrastive_ce_bwd", s, P_(lt), P_(lse[0]), P_(ls), P_(gl), B, Bg, ctx.lab0, norm, P_(dSt), P_(dls[0]))
        call("clipmi_contrastive_ce_bwd", s, P_(li), P_(lse[1]), P_(ls), P_(gl), B, Bg, ctx.lab0, norm, P_(dSi), P_(dls[1]))
        # dt^ = dSt i_all + (dSi^T i_local)[rank rows] ; di^ = dSi t_all + (dSt^T t_local)[rank rows]
        # column-direction terms first (reduce-scattered to their owners), then the row terms
        # accumulate on top through the GEMM's beta epilogue
        dTg = torch.empty(Bg, E, dtype=torch.float32, device=dev)
        dIg = torch.empty(Bg, E, dtype=torch.float32, device=dev)
        _gemm_f32(Bg, E, B, dSi, Bg, False, ih, E, False, dTg, E)
        _gemm_f32(Bg, E, B, dSt, Bg, False, th, E, False, dIg, E)
        dth = _reduce_scatter(dTg, ctx.group, world)
        dih = _reduce_scatter(dIg, ctx.group, world)
        _gemm_f32(B, E, Bg, dSt, Bg, True, ig, E, False, dth, E, flags=_lib.EPI_BETA)
        _gemm_f32(B, E, Bg, dSi, Bg, True, tg, E, False, dih, E, flags=_lib.EPI_BETA)
        return ContrastiveFn._finish_backward(ctx, s, dth, dih, gth, gih, dls, th, ih, tn, inn)

    @staticmethod
    def _backward_streamed(ctx, gloss, gth, gih):
        th, ih, tn, inn, tg, ig, lse, ls = ctx.saved_tensors
        B, Bg, E, world, C = ctx.B, ctx.Bg, th.shape[1], ctx.world, ctx.chunk
        dev = th.device
        s = K.stream()
        gl = gloss.to(torch.float32).contiguous().reshape(1) if gloss is not None else None
        dls = torch.empty(2, B, dtype=torch.float32, device=dev)
        norm = 1.0 / (2 * Bg)
        # logits_t = s t^_local i^_all^T feeds dt^ (rows) and di^_all (columns); logits_i the converse
        dTg = torch.empty(Bg, E, dtype=torch.float32, device=dev)
        dIg = torch.empty(Bg, E, dtype=torch.float32, device=dev)
        dth_row = torch.empty(B, E, dtype=torch.float32, device=dev)
        dih_row = torch.empty(B, E, dtype=torch.float32, device=dev)
        _ce_streamed_bwd(s, th, ig, ls, gl, lse[0], ctx.lab0, norm, C, dls[0], dIg, dth_row)
        _ce_streamed_bwd(s, ih, tg, ls, gl, lse[1], ctx.lab0, norm, C, dls[1], dTg, dih_row)
        dth = _reduce_scatter(dTg, ctx.group, world)
        dih = _reduce_scatter(dIg, ctx.group, world)
        dth += dth_row
        dih += dih_row
        return ContrastiveFn._finish_backward(ctx, s, dth, dih, gth, gih, dls, th, ih, tn, inn)

    @staticmethod
    def _finish_backward(ctx, s, dth, dih, gth, gih, dls, th, ih, tn, inn):
        B, E = th.shape
        dev = th.device
        if gth is not None:
            dth += gth
        if gih is not None:
            dih += gih
        p = ctx.ls_param
        if p.requires_grad:
            # d logit_scale accumulates straight into the grad arena; all ranks' shares are
            # summed by the data-parallel gradient all-reduce
            ctx.arena.prepare_grads()
            call("clipmi_sum2", s, P_(dls[0]), P_(dls[1]), B, 1.0, ctx.arena.ptr("logit_scale", ctx.arena.grad), 1)
        dt = torch.empty(B, E, dtype=torch.float32, device=dev)
        di = torch.empty(B, E, dtype=torch.float32, device=dev)
        call("clipmi_l2norm_bwd", s, P_(dth), P_(th), P_(tn), P_(dt), B, E)
        call("clipmi_l2norm_bwd", s, P_(dih), P_(ih), P_(inn), P_(di), B, E)
        return dt, di, None, None, None, None

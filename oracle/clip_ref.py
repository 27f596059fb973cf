"""CPU oracle for the CLIP dual-encoder + adapter contrastive step.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import this module, and only as the checker /
CPU baseline.  The product path (``vlm-clip_amd/clipmi``) never imports it.

This is a plain PyTorch-CPU restatement (fp32 by default, fp64 on request) of the math
the reference runs through HF transformers + its own modules.  Every function cites the
reference line it follows.  HF transformers is a third-party dependency of the reference
(pinned 4.51.3 at ``uv.lock:1540-1541``; not vendored under /root/reference); its CLIP
math is restated here from the published source (``[HF] models/clip/modeling_clip.py``,
installed copy 5.15.0).

Pinning: ``tests/golden/*.npz`` were produced by importing the reference's own
``model_m.CLIPWithAdapters`` / ``adapter.clip_adapter`` in the build container
(``tools/gen_goldens.py``); ``tests/test_oracle_golden.py`` checks this restatement
against them.  The reference ships no numeric fixtures of its own.
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F


def layer_norm(x, w, b, eps):
    # nn.LayerNorm(eps=config.layer_norm_eps)  [HF] modeling_clip.py:357,359
    return F.layer_norm(x, (x.shape[-1],), w, b, eps)


def quick_gelu(x):
    # [HF] activations.py:117-123: x * sigmoid(1.702 x)
    return x * torch.sigmoid(1.702 * x)


def gelu_erf(x):
    # nn.GELU() default (approximate='none'), adapter/clip_adapter.py:13,140
    return 0.5 * x * (1.0 + torch.erf(x / math.sqrt(2.0)))


def linear(x, w, b=None):
    y = x @ w.t()
    return y if b is None else y + b


def attention(x, p, prefix, heads, mask):
    """CLIPAttention.forward + eager_attention_forward, [HF] modeling_clip.py:259-335."""
    B, N, D = x.shape
    hd = D // heads
    q = linear(x, p[f"{prefix}.q_proj.weight"], p[f"{prefix}.q_proj.bias"])
    k = linear(x, p[f"{prefix}.k_proj.weight"], p[f"{prefix}.k_proj.bias"])
    v = linear(x, p[f"{prefix}.v_proj.weight"], p[f"{prefix}.v_proj.bias"])
    q, k, v = (t.view(B, N, heads, hd).transpose(1, 2) for t in (q, k, v))
    s = (q @ k.transpose(-1, -2)) * hd ** -0.5            # :268
    if mask is not None:
        s = s + mask                                         # :269-270
    pr = torch.softmax(s, dim=-1)                            # :271 (fp32 softmax)
    o = (pr @ v).transpose(1, 2).reshape(B, N, D)           # :274-275, :331
    return linear(o, p[f"{prefix}.out_proj.weight"], p[f"{prefix}.out_proj.bias"])


def encoder_layer(x, p, prefix, heads, eps, mask):
    """CLIPEncoderLayer.forward, [HF] modeling_clip.py:362-383 (pre-LN, two residuals)."""
    h = layer_norm(x, p[f"{prefix}.layer_norm1.weight"], p[f"{prefix}.layer_norm1.bias"], eps)
    x = x + attention(h, p, f"{prefix}.self_attn", heads, mask)
    h = layer_norm(x, p[f"{prefix}.layer_norm2.weight"], p[f"{prefix}.layer_norm2.bias"], eps)
    h = linear(h, p[f"{prefix}.mlp.fc1.weight"], p[f"{prefix}.mlp.fc1.bias"])   # :346-350
    h = quick_gelu(h)
    h = linear(h, p[f"{prefix}.mlp.fc2.weight"], p[f"{prefix}.mlp.fc2.bias"])
    return x + h


def causal_padding_mask(attention_mask, dtype):
    """Additive [B,1,N,N] mask: causal + key padding ([HF] modeling_clip.py:543-548)."""
    B, N = attention_mask.shape
    neg = torch.finfo(dtype).min
    causal = torch.triu(torch.ones(N, N, dtype=torch.bool), diagonal=1)
    keypad = attention_mask[:, None, None, :] == 0
    blocked = causal[None, None] | keypad
    return torch.zeros(B, 1, N, N, dtype=dtype).masked_fill(blocked, neg)


def text_tower(input_ids, attention_mask, p, cfg):
    """CLIPTextModel.forward → last_hidden_state (after final_layer_norm), [HF] :513-559."""
    t = cfg.text_config
    if input_ids.shape[-1] > t.max_position_embeddings:
        raise ValueError("Sequence length must be less than max_position_embeddings")
    pre = "text_model"
    dt = p[f"{pre}.embeddings.token_embedding.weight"].dtype
    x = p[f"{pre}.embeddings.token_embedding.weight"][input_ids]                   # :252
    x = x + p[f"{pre}.embeddings.position_embedding.weight"][: input_ids.shape[1]]  # :254-255
    mask = causal_padding_mask(attention_mask, dt)
    for i in range(t.num_hidden_layers):
        x = encoder_layer(x, p, f"{pre}.encoder.layers.{i}", t.num_attention_heads, t.layer_norm_eps, mask)
    return layer_norm(x, p[f"{pre}.final_layer_norm.weight"], p[f"{pre}.final_layer_norm.bias"], t.layer_norm_eps)


def image_processor(images, image_size, mean, std):
    """The input step of the reference (CLIPProcessor.from_pretrained(...) -> CLIPImageProcessor,
    model_m.py:30, dataset.py:152-164) without resize: [HF] image_processing_clip.py
    center_crop (top = (h - crop) // 2, left = (w - crop) // 2), rescale (x / 255), normalize
    ((x - mean) / std), channels first.  uint8 [B, H, W, 3] numpy -> float32 [B, 3, S, S]."""
    B, H, W, C = images.shape
    top, left = (H - image_size) // 2, (W - image_size) // 2
    x = images[:, top:top + image_size, left:left + image_size, :].astype(np.float32)
    x = x * np.float32(1.0 / 255.0)
    x = (x - np.asarray(mean, dtype=np.float32)) / np.asarray(std, dtype=np.float32)
    return np.ascontiguousarray(x.transpose(0, 3, 1, 2)).astype(np.float32)


def patch_embed(pixel_values, p, cfg):
    """CLIPVisionEmbeddings.forward, [HF] :202-218: conv(k=s=P, no bias), CLS, +pos."""
    v = cfg.vision_config
    B, C, H, W = pixel_values.shape
    if H != v.image_size or W != v.image_size:
        raise ValueError(f"Input image size ({H}*{W}) doesn't match model ({v.image_size}*{v.image_size}).")
    pre = "vision_model.embeddings"
    w = p[f"{pre}.patch_embedding.weight"]
    x = F.conv2d(pixel_values.to(w.dtype), w, stride=v.patch_size)      # :211
    x = x.flatten(2).transpose(1, 2)                                        # :212
    cls = p[f"{pre}.class_embedding"].expand(B, 1, -1)                     # :214
    x = torch.cat([cls, x], dim=1)
    return x + p[f"{pre}.position_embedding.weight"][None]                # :219


def vision_tower(pixel_values, p, cfg):
    """CLIPVisionModel.forward → last_hidden_state (NO post_layernorm), [HF] :638-651."""
    v = cfg.vision_config
    x = patch_embed(pixel_values, p, cfg)
    x = layer_norm(x, p["vision_model.pre_layrnorm.weight"], p["vision_model.pre_layrnorm.bias"], v.layer_norm_eps)
    for i in range(v.num_hidden_layers):
        x = encoder_layer(x, p, f"vision_model.encoder.layers.{i}", v.num_attention_heads, v.layer_norm_eps, None)
    return x


def adapter(x, a, layer_norm_on=True, eps=1e-5):
    """TextAdapter/VisionAdapter.forward (adapter/clip_adapter.py:17-23, 144-150):
    LN(up(GELU(down(x))) + x).  With ``layer_norm_on=False`` this is peclip.TextualAdapter
    (adapter/peclip.py:13-18): up(GELU(down(x))) + x."""
    h = linear(x, a["down_project.weight"], a["down_project.bias"])
    h = gelu_erf(h)
    h = linear(h, a["up_project.weight"], a["up_project.bias"])
    h = h + x
    if layer_norm_on:
        h = layer_norm(h, a["layer_norm.weight"], a["layer_norm.bias"], eps)
    return h


def mhsa_residual_ln(x, s, heads, eps=1e-5):
    """peclip.ContextAdapter / SharedAdapter.forward (adapter/peclip.py:31-34, 45-48):
    layer_norm(mhsa(x, x, x) + x), nn.MultiheadAttention(batch_first=True) restated: [q|k|v] =
    in_proj(x), per head softmax(q k^T / sqrt(D / heads)) v, out_proj.  x [B, N, D] or [N, D]."""
    unb = x.dim() == 2
    if unb:
        x = x[None]
    B, N, D = x.shape
    hd = D // heads
    qkv = linear(x, s["mhsa.in_proj_weight"], s["mhsa.in_proj_bias"])
    q, k, v = (t.reshape(B, N, heads, hd).transpose(1, 2) for t in qkv.split(D, dim=-1))
    pr = torch.softmax((q @ k.transpose(-1, -2)) * hd ** -0.5, dim=-1)
    o = (pr @ v).transpose(1, 2).reshape(B, N, D)
    y = layer_norm(linear(o, s["mhsa.out_proj.weight"], s["mhsa.out_proj.bias"]) + x,
                   s["layer_norm.weight"], s["layer_norm.bias"], eps)
    return y[0] if unb else y


def shared_adapter(x, img, s, heads=8, keep_p=None, keep_m=None, p=0.1):
    """SharedMHSAttentionAdapter.forward, adapter/clip_adapter.py:100-128, with the image tokens
    img [N_v, D_v] broadcast over the batch (quirk Q3; the reference runs at B=1).
    nn.MultiheadAttention core restated: q,k,v = in_proj; softmax(q k^T / sqrt(64)) v; out_proj.
    Training-mode dropout (p on the attention probabilities and on mlp.2's output, :84,96) when
    masks are given: keep_p [heads, B*T, N_v], keep_m [B*T, hidden] (0/1)."""
    t = linear(x, s["text_proj.weight"], s["text_proj.bias"])
    u = linear(img, s["image_proj.weight"], s["image_proj.bias"])
    kv = layer_norm(u, s["norm1.weight"], s["norm1.bias"], 1e-5)
    hs = layer_norm(t, s["norm2.weight"], s["norm2.bias"], 1e-5)
    W, b = s["cross_attn.in_proj_weight"], s["cross_attn.in_proj_bias"]
    H = W.shape[1]
    q = linear(hs, W[:H], b[:H])
    k = linear(kv, W[H:2 * H], b[H:2 * H])
    v = linear(kv, W[2 * H:], b[2 * H:])
    B, T = q.shape[0], q.shape[1]
    hd = H // heads
    qh = q.view(B, T, heads, hd).transpose(1, 2)
    kh = k.view(-1, heads, hd).transpose(0, 1)
    vh = v.view(-1, heads, hd).transpose(0, 1)
    pr = torch.softmax((qh @ kh.transpose(-1, -2)) * hd ** -0.5, dim=-1)
    if keep_p is not None:  # [heads, B*T, Nv] -> [B, heads, T, Nv]
        kp = keep_p.to(pr.dtype).view(heads, B, T, -1).transpose(0, 1)
        pr = pr * kp / (1.0 - p)
    a = pr @ vh
    a = a.transpose(1, 2).reshape(B, T, H)
    hs = hs + linear(a, s["cross_attn.out_proj.weight"], s["cross_attn.out_proj.bias"])
    m = gelu_erf(linear(layer_norm(hs, s["norm3.weight"], s["norm3.bias"], 1e-5), s["mlp.0.weight"], s["mlp.0.bias"]))
    z = linear(m, s["mlp.2.weight"], s["mlp.2.bias"])
    if keep_m is not None:
        z = z * keep_m.to(z.dtype).view(B, T, -1) / (1.0 - p)
    return hs + z


def text_features(input_ids, attention_mask, p, cfg, text_adapter=None, pooling="first", shared_adapters=None):
    """CLIPWithAdapters.get_text_features, model_m.py:77-105.

    pooling="first" reproduces ``text_features[:, 0, :]`` (model_m.py:102, quirk Q1);
    pooling="eos" is HF CLIPTextModel's pooler ([HF] :561-581).  shared_adapters: list of
    SharedMHSAttentionAdapter state dicts applied after the text adapter (model_m.py:95-100)."""
    h = text_tower(input_ids, attention_mask, p, cfg)
    if text_adapter is not None:
        h = adapter(h, text_adapter)                                          # :88-90
    for s in shared_adapters or []:
        h = shared_adapter(h, p["vision_model.embeddings.position_embedding.weight"], s)  # :95-100
    if pooling == "first":
        pooled = h[:, 0, :]
    else:
        eos = cfg.text_config.eos_token_id
        if eos == 2:
            idx = input_ids.to(torch.int).argmax(dim=-1)
        else:
            idx = (input_ids.to(torch.int) == eos).int().argmax(dim=-1)
        pooled = h[torch.arange(h.shape[0]), idx]
    return linear(pooled, p["text_projection.weight"])                      # :103


def image_features(pixel_values, p, cfg, vision_adapter=None):
    """CLIPWithAdapters.get_image_features, model_m.py:107-125 (quirk Q2: no post-LN)."""
    h = vision_tower(pixel_values, p, cfg)
    if vision_adapter is not None:
        h = adapter(h, vision_adapter)                                        # :117-118
    return linear(h[:, 0, :], p["visual_projection.weight"])                # :122-123


def contrastive(text_feat, image_feat, logit_scale):
    """CLIPWithAdapters.forward contrastive branch, model_m.py:146-171."""
    t = text_feat / text_feat.norm(dim=-1, keepdim=True)                     # :148
    i = image_feat / image_feat.norm(dim=-1, keepdim=True)                   # :149
    lpt = (t @ i.t()) * logit_scale.exp()                                    # :152-155
    lpi = lpt.t()                                                            # :156
    labels = torch.arange(t.shape[0])
    loss = (F.cross_entropy(lpt, labels) + F.cross_entropy(lpi, labels)) / 2  # :159-163
    return {"loss": loss, "text_features": t, "image_features": i,
            "logits_per_text": lpt, "logits_per_image": lpi}


def clip_with_adapters_forward(batch, p, cfg, text_adapter=None, vision_adapter=None,
                               return_loss=True, pooling="first"):
    """CLIPWithAdapters.forward, model_m.py:127-176 (shared adapters off, quirk Q3)."""
    tf = text_features(batch["input_ids"], batch["attention_mask"], p, cfg, text_adapter, pooling)
    imf = image_features(batch["pixel_values"], p, cfg, vision_adapter)
    if return_loss:
        return contrastive(tf, imf, p["logit_scale"])
    return {"text_features": tf, "image_features": imf}


def to_torch(sd, dtype=torch.float32, requires_grad=False):
    out = {}
    for k, v in sd.items():
        t = torch.as_tensor(v).to(dtype).clone()
        t.requires_grad_(requires_grad)
        out[k] = t
    return out


def adamw_reference(params, grads, m, v, step, lr, beta1=0.9, beta2=0.999, eps=1e-8, wd=0.01):
    """torch.optim.AdamW single step restated (decoupled weight decay), trainer.py:46-48,98."""
    out = []
    for p, g, mm, vv in zip(params, grads, m, v):
        p = p * (1 - lr * wd)
        mm = beta1 * mm + (1 - beta1) * g
        vv = beta2 * vv + (1 - beta2) * g * g
        mhat = mm / (1 - beta1 ** step)
        vhat = vv / (1 - beta2 ** step)
        p = p - lr * mhat / (vhat.sqrt() + eps)
        out.append((p, mm, vv))
    return out


def linear_warmup_lambda(step, warmup, total):
    """[HF] optimization.py:101-104 get_linear_schedule_with_warmup lr multiplier."""
    if step < warmup:
        return float(step) / float(max(1, warmup))
    return max(0.0, float(total - step) / float(max(1, total - warmup)))

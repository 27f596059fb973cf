"""Deterministic synthetic weights and batches.

No pretrained checkpoints or datasets exist offline, so every parity fixture and every
benchmark runs on weights and batches produced here.  The generator is counter based
(splitmix64 of ``seed ⊕ hash(name)`` and the element index, Box-Muller in float64,
rounded to float32) so it is platform independent and needs no library RNG state: the
same call gives the same bits in this container and on the GPU box.

Init scales follow HF ``CLIPPreTrainedModel._init_weights`` (``[HF] modeling_clip.py:404-452``).
LayerNorm affines and Linear biases, which HF initialises to 1/0, are perturbed here so
that parity tests exercise them.
"""
from __future__ import annotations

import hashlib
import math
from collections import OrderedDict

import numpy as np

from .config import CLIPConfig, LN100

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)
_C1 = np.uint64(0x9E3779B97F4A7C15)
_C2 = np.uint64(0xBF58476D1CE4E5B9)
_C3 = np.uint64(0x94D049BB133111EB)


def _stream_key(seed: int, name: str) -> np.uint64:
    h = hashlib.sha256(f"{seed}:{name}".encode()).digest()
    return np.uint64(int.from_bytes(h[:8], "little"))


def _splitmix(idx: np.ndarray, key: np.uint64) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = idx * _C1 + key
        z = (z ^ (z >> np.uint64(30))) * _C2
        z = (z ^ (z >> np.uint64(27))) * _C3
        z = z ^ (z >> np.uint64(31))
    return z


def uniform(n: int, seed: int, name: str) -> np.ndarray:
    """U[0,1) float64, element i = splitmix64(i; key)."""
    key = _stream_key(seed, name)
    out = np.empty(n, dtype=np.float64)
    chunk = 1 << 22
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        z = _splitmix(np.arange(s, e, dtype=np.uint64), key)
        out[s:e] = (z >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)
    return out


def normal(shape, seed: int, name: str, std: float = 1.0, mean: float = 0.0) -> np.ndarray:
    n = int(np.prod(shape)) if len(shape) else 1
    m = (n + 1) // 2
    u = uniform(2 * m, seed, name)
    u1 = np.maximum(u[0::2], 1e-300)
    u2 = u[1::2]
    r = np.sqrt(-2.0 * np.log(u1))
    z = np.concatenate([r * np.cos(2 * math.pi * u2), r * np.sin(2 * math.pi * u2)])[:n]
    return (mean + std * z).astype(np.float32).reshape(shape)


def _tower_layer_shapes(prefix, t, layers_std):
    d, f = t.hidden_size, t.intermediate_size
    in_std, out_std, fc_std, fc2_std = layers_std
    out = []
    for i in range(t.num_hidden_layers):
        p = f"{prefix}.encoder.layers.{i}"
        for nm in ("k_proj", "v_proj", "q_proj"):
            out.append((f"{p}.self_attn.{nm}.weight", (d, d), in_std, 0.0))
            out.append((f"{p}.self_attn.{nm}.bias", (d,), 0.02, 0.0))
        out.append((f"{p}.self_attn.out_proj.weight", (d, d), out_std, 0.0))
        out.append((f"{p}.self_attn.out_proj.bias", (d,), 0.02, 0.0))
        out.append((f"{p}.layer_norm1.weight", (d,), 0.1, 1.0))
        out.append((f"{p}.layer_norm1.bias", (d,), 0.1, 0.0))
        out.append((f"{p}.mlp.fc1.weight", (f, d), fc_std, 0.0))
        out.append((f"{p}.mlp.fc1.bias", (f,), 0.02, 0.0))
        out.append((f"{p}.mlp.fc2.weight", (d, f), fc2_std, 0.0))
        out.append((f"{p}.mlp.fc2.bias", (d,), 0.02, 0.0))
        out.append((f"{p}.layer_norm2.weight", (d,), 0.1, 1.0))
        out.append((f"{p}.layer_norm2.bias", (d,), 0.1, 0.0))
    return out


def clip_param_specs(cfg: CLIPConfig):
    """(name, shape, std, mean) for every CLIPModel parameter, HF state-dict names."""
    fac = cfg.initializer_factor
    specs = []
    t, v = cfg.text_config, cfg.vision_config

    def stds(tc):
        d, L = tc.hidden_size, tc.num_hidden_layers
        in_std = d ** -0.5 * (2 * L) ** -0.5 * fac
        return in_std, d ** -0.5 * fac, (2 * d) ** -0.5 * fac, in_std

    specs.append(("text_model.embeddings.token_embedding.weight", (t.vocab_size, t.hidden_size), 0.02 * fac, 0.0))
    specs.append(("text_model.embeddings.position_embedding.weight",
                  (t.max_position_embeddings, t.hidden_size), 0.01 * fac, 0.0))
    specs += _tower_layer_shapes("text_model", t, stds(t))
    specs.append(("text_model.final_layer_norm.weight", (t.hidden_size,), 0.1, 1.0))
    specs.append(("text_model.final_layer_norm.bias", (t.hidden_size,), 0.1, 0.0))
    specs.append(("vision_model.embeddings.class_embedding", (v.hidden_size,), v.hidden_size ** -0.5 * fac, 0.0))
    specs.append(("vision_model.embeddings.patch_embedding.weight",
                  (v.hidden_size, v.num_channels, v.patch_size, v.patch_size), cfg.initializer_range * fac, 0.0))
    specs.append(("vision_model.embeddings.position_embedding.weight",
                  (v.num_positions, v.hidden_size), cfg.initializer_range * fac, 0.0))
    specs.append(("vision_model.pre_layrnorm.weight", (v.hidden_size,), 0.1, 1.0))
    specs.append(("vision_model.pre_layrnorm.bias", (v.hidden_size,), 0.1, 0.0))
    specs += _tower_layer_shapes("vision_model", v, stds(v))
    specs.append(("vision_model.post_layernorm.weight", (v.hidden_size,), 0.1, 1.0))
    specs.append(("vision_model.post_layernorm.bias", (v.hidden_size,), 0.1, 0.0))
    specs.append(("visual_projection.weight", (cfg.projection_dim, v.hidden_size), v.hidden_size ** -0.5 * fac, 0.0))
    specs.append(("text_projection.weight", (cfg.projection_dim, t.hidden_size), t.hidden_size ** -0.5 * fac, 0.0))
    return specs


def clip_state_dict(cfg: CLIPConfig, seed: int = 0, logit_scale: float = LN100) -> "OrderedDict[str, np.ndarray]":
    sd = OrderedDict()
    for name, shape, std, mean in clip_param_specs(cfg):
        sd[name] = normal(shape, seed, name, std, mean)
    sd["logit_scale"] = np.array(logit_scale, dtype=np.float32)
    return sd


def adapter_param_specs(hidden: int, bottleneck: int, ln: bool = True):
    """TextAdapter / VisionAdapter (``adapter/clip_adapter.py:10-15, 137-142``) state dict."""
    specs = [("down_project.weight", (bottleneck, hidden), hidden ** -0.5, 0.0),
             ("down_project.bias", (bottleneck,), 0.05, 0.0),
             ("up_project.weight", (hidden, bottleneck), bottleneck ** -0.5, 0.0),
             ("up_project.bias", (hidden,), 0.05, 0.0)]
    if ln:
        specs += [("layer_norm.weight", (hidden,), 0.1, 1.0), ("layer_norm.bias", (hidden,), 0.1, 0.0)]
    return specs


def adapter_state_dict(hidden: int, bottleneck: int, seed: int, prefix: str, ln: bool = True):
    sd = OrderedDict()
    for name, shape, std, mean in adapter_param_specs(hidden, bottleneck, ln):
        sd[name] = normal(shape, seed, f"{prefix}.{name}", std, mean)
    return sd


def shared_adapter_state_dict(text_in: int, image_in: int, seed: int, prefix: str, hidden: int = 512):
    """SharedMHSAttentionAdapter (adapter/clip_adapter.py:69-128) weights: linear weights
    N(0, 1/fan_in), LayerNorm weights 1 + N(0, 0.1), biases N(0, 0.02)."""
    H = hidden
    shapes = [("text_proj.weight", (H, text_in)), ("text_proj.bias", (H,)),
              ("image_proj.weight", (H, image_in)), ("image_proj.bias", (H,)),
              ("cross_attn.in_proj_weight", (3 * H, H)), ("cross_attn.in_proj_bias", (3 * H,)),
              ("cross_attn.out_proj.weight", (H, H)), ("cross_attn.out_proj.bias", (H,)),
              ("norm1.weight", (H,)), ("norm1.bias", (H,)), ("norm2.weight", (H,)), ("norm2.bias", (H,)),
              ("norm3.weight", (H,)), ("norm3.bias", (H,)),
              ("mlp.0.weight", (4 * H, H)), ("mlp.0.bias", (4 * H,)),
              ("mlp.2.weight", (H, 4 * H)), ("mlp.2.bias", (H,))]
    sd = OrderedDict()
    for name, shape in shapes:
        if len(shape) == 2:
            sd[name] = normal(shape, seed, f"{prefix}.{name}", 1.0 / math.sqrt(shape[1]))
        elif name.startswith("norm") and name.endswith("weight"):
            sd[name] = normal(shape, seed, f"{prefix}.{name}", 0.1, 1.0)
        else:
            sd[name] = normal(shape, seed, f"{prefix}.{name}", 0.02)
    return sd


def mhsa_adapter_state_dict(D: int, seed: int, prefix: str):
    """peclip.ContextAdapter / SharedAdapter (adapter/peclip.py:21-48) weights: every tensor
    N(0, 1/D), except the LayerNorm affine: weight 1 + N(0, 0.1), bias N(0, 0.1)."""
    shapes = [("mhsa.in_proj_weight", (3 * D, D)), ("mhsa.in_proj_bias", (3 * D,)),
              ("mhsa.out_proj.weight", (D, D)), ("mhsa.out_proj.bias", (D,)),
              ("layer_norm.weight", (D,)), ("layer_norm.bias", (D,))]
    sd = OrderedDict()
    for name, shape in shapes:
        ln = name.startswith("layer_norm")
        sd[name] = normal(shape, seed, f"{prefix}/{name}", 0.1 if ln else 1.0 / math.sqrt(D),
                          1.0 if name == "layer_norm.weight" else 0.0)
    return sd


CLIP_MEAN = np.array([0.48145466, 0.4578275, 0.40821073], dtype=np.float64)
CLIP_STD = np.array([0.26862954, 0.26130258, 0.27577711], dtype=np.float64)


def synthetic_batch(cfg: CLIPConfig, batch: int, seed: int = 1234, start: int = 0, full_length: bool = False):
    """Rows [start, start+batch) of the global synthetic batch.

    pixel_values: CLIP-normalised U[0,1) fp32 NCHW.  input_ids: BOS, random ids, EOS,
    then EOS padding (CLIP tokenizer pads with <|endoftext|>, ``dataset.py:156-158``);
    attention_mask 1 on the first L_i positions, L_i ~ U{5..77}.
    Row r depends only on (seed, r), so shards of one global batch concatenate exactly."""
    v, t = cfg.vision_config, cfg.text_config
    S, H = t.max_position_embeddings, v.image_size
    rows = np.arange(start, start + batch)
    px = np.empty((batch, 3, H, H), dtype=np.float32)
    ids = np.empty((batch, S), dtype=np.int64)
    mask = np.zeros((batch, S), dtype=np.int64)
    bos, eos = t.bos_token_id, t.eos_token_id
    nvocab = min(t.vocab_size, eos + 1)
    for i, r in enumerate(rows):
        u = uniform(3 * H * H, seed, f"pixels/{r}").reshape(3, H, H)
        px[i] = ((u - CLIP_MEAN[:, None, None]) / CLIP_STD[:, None, None]).astype(np.float32)
        ur = uniform(S + 1, seed, f"ids/{r}")
        L = S if full_length else 5 + int(ur[0] * (S - 4))
        L = min(L, S)
        body = (ur[1:S + 1] * max(1, nvocab - 2)).astype(np.int64)
        ids[i, :] = eos if eos < t.vocab_size else t.vocab_size - 1
        ids[i, 0] = bos if bos < t.vocab_size else 0
        ids[i, 1:L - 1] = body[1:L - 1]
        ids[i, L - 1] = eos if eos < t.vocab_size else t.vocab_size - 1
        mask[i, :L] = 1
    return {"input_ids": ids, "attention_mask": mask, "pixel_values": px}

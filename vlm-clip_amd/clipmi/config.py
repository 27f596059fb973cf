"""Model shapes for the CLIP dual encoder on the hot path.

Field names follow HF ``CLIPTextConfig`` / ``CLIPVisionConfig`` / ``CLIPConfig``
(``[HF] models/clip/configuration_clip.py:47-64, 97-109, 160-162``) so that a config
dict written by ``CLIPModel.save_pretrained`` can be read back here.  The reference
loads these by hub name (``model_m.py:29``); offline we accept a local directory
holding ``config.json`` (+ ``model.safetensors``) or one of the presets below.
"""
from __future__ import annotations

import json
import math
import os
from dataclasses import asdict, dataclass, field, replace


@dataclass(frozen=True)
class TowerConfig:
    hidden_size: int
    intermediate_size: int
    num_hidden_layers: int
    num_attention_heads: int
    layer_norm_eps: float = 1e-5
    hidden_act: str = "quick_gelu"
    # text only
    vocab_size: int = 49408
    max_position_embeddings: int = 77
    eos_token_id: int = 49407
    bos_token_id: int = 49406
    pad_token_id: int = 1
    # vision only
    image_size: int = 224
    patch_size: int = 32
    num_channels: int = 3

    @property
    def head_dim(self) -> int:
        return self.hidden_size // self.num_attention_heads

    @property
    def num_patches(self) -> int:
        return (self.image_size // self.patch_size) ** 2

    @property
    def num_positions(self) -> int:  # vision tokens incl. CLS
        return self.num_patches + 1


@dataclass(frozen=True)
class CLIPConfig:
    text_config: TowerConfig
    vision_config: TowerConfig
    projection_dim: int = 512
    logit_scale_init_value: float = 2.6592
    initializer_factor: float = 1.0
    initializer_range: float = 0.02
    name: str = "custom"

    def to_hf_dict(self) -> dict:
        t = asdict(self.text_config)
        v = asdict(self.vision_config)
        for k in ("image_size", "patch_size", "num_channels"):
            t.pop(k)
        for k in ("vocab_size", "max_position_embeddings", "eos_token_id", "bos_token_id", "pad_token_id"):
            v.pop(k)
        return {
            "text_config": t,
            "vision_config": v,
            "projection_dim": self.projection_dim,
            "logit_scale_init_value": self.logit_scale_init_value,
            "initializer_factor": self.initializer_factor,
        }


def _text(d, mlp, layers, heads, **kw):
    return TowerConfig(hidden_size=d, intermediate_size=mlp, num_hidden_layers=layers,
                       num_attention_heads=heads, **kw)


def _vision(d, mlp, layers, heads, patch, image=224):
    return TowerConfig(hidden_size=d, intermediate_size=mlp, num_hidden_layers=layers,
                       num_attention_heads=heads, patch_size=patch, image_size=image)


# SURVEY.md §8 model-shape table.
PRESETS = {
    "openai/clip-vit-base-patch32": CLIPConfig(_text(512, 2048, 12, 8), _vision(768, 3072, 12, 12, 32),
                                               512, name="ViT-B/32"),
    "openai/clip-vit-base-patch16": CLIPConfig(_text(512, 2048, 12, 8), _vision(768, 3072, 12, 12, 16),
                                               512, name="ViT-B/16"),
    "openai/clip-vit-large-patch14": CLIPConfig(_text(768, 3072, 12, 12), _vision(1024, 4096, 24, 16, 14),
                                                768, name="ViT-L/14"),
    "openai/clip-vit-large-patch14-336": CLIPConfig(_text(768, 3072, 12, 12),
                                                    _vision(1024, 4096, 24, 16, 14, image=336),
                                                    768, name="ViT-L/14@336"),
    # test-sized CLIP: head_dim 64 like the real models, 2 layers, 17 vision tokens
    "tiny": CLIPConfig(_text(128, 256, 2, 2, vocab_size=1000, eos_token_id=999, bos_token_id=998), _vision(128, 256, 2, 2, 16, image=64),
                       64, name="tiny"),
}
ALIASES = {"B/32": "openai/clip-vit-base-patch32", "B/16": "openai/clip-vit-base-patch16",
           "L/14": "openai/clip-vit-large-patch14", "L/14@336": "openai/clip-vit-large-patch14-336"}


def from_hf_dict(d: dict, name: str = "custom") -> CLIPConfig:
    def tower(src, is_text):
        keys = TowerConfig.__dataclass_fields__.keys()
        kw = {k: src[k] for k in keys if k in src and src[k] is not None}
        if isinstance(kw.get("eos_token_id"), list):
            kw["eos_token_id"] = kw["eos_token_id"][0]
        return TowerConfig(**kw)
    return CLIPConfig(tower(d["text_config"], True), tower(d["vision_config"], False),
                      d.get("projection_dim", 512), d.get("logit_scale_init_value", 2.6592),
                      d.get("initializer_factor", 1.0), name=name)


def resolve(name_or_path) -> CLIPConfig:
    """Map a reference ``clip_model_name`` (``model_m.py:17``) to a config.

    Accepts a preset/hub name, an alias ("B/16"), a ``CLIPConfig`` or a local directory
    containing ``config.json``.  Hub downloads are never attempted (offline build)."""
    if isinstance(name_or_path, CLIPConfig):
        return name_or_path
    if name_or_path in ALIASES:
        name_or_path = ALIASES[name_or_path]
    if name_or_path in PRESETS:
        return PRESETS[name_or_path]
    cfg_file = os.path.join(str(name_or_path), "config.json")
    if os.path.isfile(cfg_file):
        with open(cfg_file) as f:
            return from_hf_dict(json.load(f), name=str(name_or_path))
    raise OSError(f"{name_or_path!r} is neither a known CLIP preset nor a local directory with config.json "
                  "(hub downloads are not available in this build)")


def forward_flops_per_pair(cfg: CLIPConfig) -> float:
    """Algorithmic forward FLOPs per image-text pair (SURVEY.md §8d formula)."""
    def enc(t: TowerConfig, n: int) -> float:
        d = t.hidden_size
        return t.num_hidden_layers * (2 * n * (4 * d * d + 2 * d * t.intermediate_size) + 4 * n * n * d)
    v, t = cfg.vision_config, cfg.text_config
    nv = v.num_positions
    patch = 2 * (nv - 1) * 3 * v.patch_size ** 2 * v.hidden_size
    proj = 2 * (v.hidden_size + t.hidden_size) * cfg.projection_dim
    return enc(v, nv) + enc(t, t.max_position_embeddings) + patch + proj


LN100 = math.log(100.0)

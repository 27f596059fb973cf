"""Parameter containers with HF ``CLIPModel`` / adapter state-dict names, backed by arenas.

The module tree reproduces the names of ``transformers.CLIPModel`` ([HF]
modeling_clip.py:660-676 and the towers above it) and of the reference adapters
(``adapter/clip_adapter.py:10-15, 137-142``) so checkpoints and ``state_dict()`` keys
are interchangeable with the reference.  The containers hold parameters only; compute
goes through ``clipmi.towers`` (the libclipmi kernels)."""
from __future__ import annotations

import torch
import torch.nn as nn

from .arena import Arena
from .config import CLIPConfig, TowerConfig


def layer_specs(prefix: str, t: TowerConfig):
    D, F = t.hidden_size, t.intermediate_size
    specs = []
    for i in range(t.num_hidden_layers):
        p = f"{prefix}.encoder.layers.{i}"
        specs += [(f"{p}.layer_norm1.weight", (D,)), (f"{p}.layer_norm1.bias", (D,)),
                  (f"{p}.self_attn.q_proj.weight", (D, D)), (f"{p}.self_attn.k_proj.weight", (D, D)),
                  (f"{p}.self_attn.v_proj.weight", (D, D)),
                  (f"{p}.self_attn.q_proj.bias", (D,)), (f"{p}.self_attn.k_proj.bias", (D,)),
                  (f"{p}.self_attn.v_proj.bias", (D,)),
                  (f"{p}.self_attn.out_proj.weight", (D, D)), (f"{p}.self_attn.out_proj.bias", (D,)),
                  (f"{p}.layer_norm2.weight", (D,)), (f"{p}.layer_norm2.bias", (D,)),
                  (f"{p}.mlp.fc1.weight", (F, D)), (f"{p}.mlp.fc1.bias", (F,)),
                  (f"{p}.mlp.fc2.weight", (D, F)), (f"{p}.mlp.fc2.bias", (D,))]
    return specs


def clip_specs(cfg: CLIPConfig):
    t, v = cfg.text_config, cfg.vision_config
    specs = [("text_model.embeddings.token_embedding.weight", (t.vocab_size, t.hidden_size)),
             ("text_model.embeddings.position_embedding.weight", (t.max_position_embeddings, t.hidden_size))]
    specs += layer_specs("text_model", t)
    specs += [("text_model.final_layer_norm.weight", (t.hidden_size,)),
              ("text_model.final_layer_norm.bias", (t.hidden_size,)),
              ("vision_model.embeddings.class_embedding", (v.hidden_size,)),
              ("vision_model.embeddings.patch_embedding.weight",
               (v.hidden_size, v.num_channels, v.patch_size, v.patch_size)),
              ("vision_model.embeddings.position_embedding.weight", (v.num_positions, v.hidden_size)),
              ("vision_model.pre_layrnorm.weight", (v.hidden_size,)),
              ("vision_model.pre_layrnorm.bias", (v.hidden_size,))]
    specs += layer_specs("vision_model", v)
    specs += [("vision_model.post_layernorm.weight", (v.hidden_size,)),
              ("vision_model.post_layernorm.bias", (v.hidden_size,)),
              ("visual_projection.weight", (cfg.projection_dim, v.hidden_size)),
              ("text_projection.weight", (cfg.projection_dim, t.hidden_size)),
              ("logit_scale", ())]
    return specs


def adapter_specs(hidden: int, bottleneck: int, ln: bool = True, names=("down_project", "up_project")):
    d, u = names
    specs = [(f"{d}.weight", (bottleneck, hidden)), (f"{d}.bias", (bottleneck,)),
             (f"{u}.weight", (hidden, bottleneck)), (f"{u}.bias", (hidden,))]
    if ln:
        specs += [("layer_norm.weight", (hidden,)), ("layer_norm.bias", (hidden,))]
    return specs


def _attach(root: nn.Module, name: str, param: nn.Parameter):
    parts = name.split(".")
    mod = root
    for i, part in enumerate(parts[:-1]):
        nxt_is_idx = parts[i + 1].isdigit()
        if isinstance(mod, nn.ModuleList):
            idx = int(part)
            while idx >= len(mod):  # parameter-free slots (e.g. nn.Sequential's GELU at mlp.1) stay empty
                mod.append(nn.ModuleList() if nxt_is_idx else nn.Module())
            mod = mod[idx]
        else:
            child = mod._modules.get(part)
            if child is None:
                child = nn.ModuleList() if nxt_is_idx else nn.Module()
                mod.add_module(part, child)
            mod = child
    mod.register_parameter(parts[-1], param)


class ArenaModule(nn.Module):
    """A module whose parameters are views into one Arena."""

    def __init__(self, specs, device, shadow=True):
        super().__init__()
        self.__dict__["arena"] = Arena(specs, device, dtype_shadow=shadow)
        for name, _ in specs:
            p = nn.Parameter(self.arena.view(name))
            self.arena.params[name] = p
            _attach(self, name, p)

    def _apply(self, fn, recurse=True):
        # move the arena once and re-create every parameter view (instead of per-param copies)
        if self.arena.apply_(fn):
            for name, old in list(self.arena.params.items()):
                p = nn.Parameter(self.arena.view(name), requires_grad=old.requires_grad)
                self.arena.params[name] = p
                parent = self
                *path, leaf = name.split(".")
                for part in path:
                    parent = parent[int(part)] if isinstance(parent, nn.ModuleList) else getattr(parent, part)
                parent._parameters[leaf] = p
        return self

    def load_numpy(self, sd: dict, strict=True):
        with torch.no_grad():
            for name, p in self.arena.params.items():
                if name in sd:
                    p.copy_(torch.as_tensor(sd[name]).to(p.dtype).reshape(p.shape))
                elif strict:
                    raise KeyError(f"missing {name}")


class CLIPParams(ArenaModule):
    """HF-named parameters of CLIPModel: .text_model, .vision_model, .text_projection,
    .visual_projection, .logit_scale."""

    def __init__(self, cfg: CLIPConfig, device, shadow=True):
        super().__init__(clip_specs(cfg), device, shadow)
        self.config = cfg
        t, v = cfg.text_config, cfg.vision_config
        for prefix, tc in (("text_model", t), ("vision_model", v)):
            for i in range(tc.num_hidden_layers):
                p = f"{prefix}.encoder.layers.{i}.self_attn"
                self.arena.check_adjacent([f"{p}.q_proj.weight", f"{p}.k_proj.weight", f"{p}.v_proj.weight"])
                self.arena.check_adjacent([f"{p}.q_proj.bias", f"{p}.k_proj.bias", f"{p}.v_proj.bias"])


class AdapterParams(ArenaModule):
    """TextAdapter / VisionAdapter parameters (adapter/clip_adapter.py:10-15, 137-142);
    with ln=False, peclip.TextualAdapter (adapter/peclip.py:7-11, names down_proj/up_proj)."""

    def __init__(self, hidden, bottleneck, device, ln=True, shadow=True, names=("down_project", "up_project")):
        super().__init__(adapter_specs(hidden, bottleneck, ln, names), device, shadow)
        self.hidden, self.bottleneck, self.has_ln, self.names = hidden, bottleneck, ln, names

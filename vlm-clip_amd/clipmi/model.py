"""Drop-in ``CLIPWithAdapters`` (model_m.py:10-248) on the MI355X-native kernels.

Same constructor arguments, forward signature, return dicts, feature methods, adapter
checkpoint format and error types as the reference; the compute runs on libclipmi
(``clipmi.towers``).  Extensions, all keyword-only:

  device       where the fp32 parameter arenas live (default: cuda if available)
  precision    "bf16" (MFMA path, default), "fp32" (exact-f32 parity mode),
               "bf16x3" (fp32 activations with the towers' GEMMs as bf16x3 split products on the MFMA
               kernels: north_star's 1e-3 logits at several times the fp32 mode's speed) or "fp8" (frozen
               towers with MXFP8 GEMMs, BASELINE config 5; adapters and the loss stay bf16 / fp32)
  residual_fp32  bf16 mode: keep the towers' residual stream (each layer's input, the attention-branch sum)
               in fp32 (default; False keeps it in bf16, ~7 % faster on the frozen-tower adapter configs)
  pooling      "first" (model_m.py:102 — quirk Q1, the reference behaviour) or "eos"
               (HF CLIPTextModel pooler, [HF] modeling_clip.py:561-581)
  init_seed    seed of the deterministic random init used when no weights file exists
  process_group data-parallel group of the contrastive loss: a torch.distributed group (RCCL
               through torch, or gloo) or a clipmi.comm.Communicator (RCCL issued by libclipmi)
"""
from __future__ import annotations

import os
import warnings

import torch
import torch.nn as nn

from . import comm as CM
from . import config as C
from . import synth
from . import towers as T
from .modules import AdapterParams, CLIPParams


class _Runtime:
    def __init__(self, clip: CLIPParams, dtype):
        self.arena = clip.arena
        self.cfg = clip.config
        self.dtype = dtype
        self.venc = T.Encoder(self.arena, "vision_model", self.cfg.vision_config, causal=False)
        self.tenc = T.Encoder(self.arena, "text_model", self.cfg.text_config, causal=True)
        self.train_tower = False
        self.bad_flag = torch.zeros(1, dtype=torch.int32, device=self.arena.device)
        self.grad_hook = None  # data-parallel gradient-ready hook (CLIPWithAdapters.set_grad_hook)
        self.shared_pos_grad = False  # a shared adapter adds into the vision position-embedding grad
        self.fp8 = False  # precision="fp8": the frozen towers' GEMMs in MXFP8 (BASELINE config 5)


def _anchor(module: nn.Module):
    for p in module.parameters():
        if p.requires_grad:
            return p
    return next(module.parameters())


class _JoinOnBackward(torch.autograd.Function):
    """Identity on the text tower's output.  Its backward runs on the side stream (autograd runs a
    node on its forward's stream) ahead of the rest of the text tower's backward, and queues a
    final callback that makes the stream backward() was called on wait for the side stream, so
    the optimizer sees the text tower's gradients (written straight into the grad arena)."""

    @staticmethod
    def forward(ctx, x, main, side):
        ctx.side = side
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        side = ctx.side
        dev = side.device

        def join():
            torch.cuda.current_stream(dev).wait_stream(side)

        torch.autograd.Variable._execution_engine.queue_callback(join)
        return g, None, None


class CLIPWithAdapters(nn.Module):
    """CLIP model with text and vision adapters (model_m.py:10-248)."""

    def __init__(self, clip_model_name="openai/clip-vit-base-patch32", text_adapter_size=256,
                 vision_adapter_size=256, shared_adapter_layers=2, freeze_clip=True, use_text_adapter=True,
                 use_vision_adapter=True, use_shared_adapters=True, *, device=None, precision="bf16",
                 pooling="first", init_seed=0, process_group=None, fast_init=False, residual_fp32=None):
        super().__init__()
        if device is None:
            device = "cuda" if torch.cuda.is_available() else "cpu"
        if precision not in ("bf16", "fp32", "bf16x3", "fp8"):
            raise ValueError("precision must be 'bf16', 'fp32', 'bf16x3' or 'fp8'")
        if precision == "fp8" and not freeze_clip:
            raise ValueError("precision='fp8' runs the frozen towers only (MXFP8 forward GEMMs); use freeze_clip=True")
        if pooling not in ("first", "eos"):
            raise ValueError("pooling must be 'first' or 'eos'")
        cfg = C.resolve(clip_model_name)
        self.config = cfg
        self.precision = precision
        self.pooling = pooling
        self.process_group = process_group
        exact = precision in ("fp32", "bf16x3")  # fp32 activations and weights (no bf16 shadow)
        dtype = torch.float32 if exact else torch.bfloat16
        shadow = not exact
        # model_m.py:29-30 — CLIPModel.from_pretrained / CLIPProcessor.from_pretrained
        self.clip = CLIPParams(cfg, device, shadow)
        self.clip.text_model.config = cfg.text_config
        self.clip.vision_model.config = cfg.vision_config
        self.processor = None  # tokenizer/image transform are host I/O, out of scope
        self._load_clip_weights(clip_model_name, init_seed, fast_init)
        text_hidden = cfg.text_config.hidden_size
        vision_hidden = cfg.vision_config.hidden_size
        self.use_text_adapter = use_text_adapter
        self.use_vision_adapter = use_vision_adapter
        self.use_shared_adapters = use_shared_adapters
        self.text_adapter = None
        self.vision_adapter = None
        self.shared_adapters = None
        if use_text_adapter:
            self.text_adapter = AdapterParams(text_hidden, text_adapter_size, device, shadow=shadow)
            self.text_adapter.load_numpy(synth.adapter_state_dict(text_hidden, text_adapter_size, init_seed,
                                                                  "text_adapter"))
        if use_vision_adapter:
            self.vision_adapter = AdapterParams(vision_hidden, vision_adapter_size, device, shadow=shadow)
            self.vision_adapter.load_numpy(synth.adapter_state_dict(vision_hidden, vision_adapter_size, init_seed,
                                                                    "vision_adapter"))
        if use_shared_adapters:
            # model_m.py:54-61: SharedMHSAttentionAdapter(text_hidden, vision_hidden) x layers;
            # hidden 512, so text_projection only fits text_hidden == 512 (B/* models), as in the reference
            from .shared_adapter import SharedAdapterParams
            self.shared_adapters = nn.ModuleList([SharedAdapterParams(text_hidden, vision_hidden, device,
                                                                      seed=init_seed, prefix=f"shared_adapters.{i}")
                                                  for i in range(shared_adapter_layers)])
        self._rt = _Runtime(self.clip, dtype)
        self._rt.fp8 = precision == "fp8"
        # bf16 mode: the towers' residual stream in fp32 (engine resid_f32; profiles/r05_bf16_error_sources.log),
        # trained or frozen: at config 4's model and batch (L/14, B = 1024) the bf16 stream measured max |dlogit|
        # 0.236 against PyTorch autocast's 0.066 (profiles/r06_config4_frozen_vs_amp.log); its 12 extra bytes per
        # element and layer cost ~7 % of the frozen-tower step
        if residual_fp32 is None:
            residual_fp32 = True
        self._rt.resid32 = precision == "bf16" and bool(residual_fp32)
        # bf16x3: the towers' GEMMs (patch embedding, every encoder GEMM) as split-operand bf16 products
        self._rt.x3 = precision == "bf16x3"
        if freeze_clip:
            self._freeze_clip_parameters()

    # ------------------------------------------------------------------ weights
    def _load_clip_weights(self, name, seed, fast_init=False):
        path = os.path.join(str(name), "model.safetensors")
        if fast_init and not os.path.isfile(path):
            # benchmark init: same per-tensor HF init scales, drawn on the device by torch's
            # generator (not bit-identical to clipmi.synth, which the parity tests use)
            g = torch.Generator(device=self.clip.arena.device).manual_seed(seed)
            with torch.no_grad():
                for pname, shape, std, mean in synth.clip_param_specs(self.config):
                    p = self.clip.arena.params[pname]
                    p.normal_(mean, std, generator=g)
                self.clip.logit_scale.fill_(C.LN100)
            return
        if os.path.isfile(path):
            from safetensors.torch import load_file
            sd = load_file(path, device="cpu")
            sd = {k: v for k, v in sd.items() if not k.endswith("position_ids")}
            missing = [k for k in self.clip.arena.params if k not in sd]
            if missing:
                raise ValueError(f"checkpoint {path} misses {missing[:4]}...")
            self.clip.load_numpy(sd)
        else:
            self.clip.load_numpy(synth.clip_state_dict(self.config, seed=seed))

    def _freeze_clip_parameters(self):
        """model_m.py:67-70."""
        for param in self.clip.parameters():
            param.requires_grad = False

    def _unfreeze_clip_parameters(self):
        """model_m.py:72-75 (also makes logit_scale trainable: SURVEY quirk Q4)."""
        for param in self.clip.parameters():
            param.requires_grad = True

    def set_grad_hook(self, fn):
        """fn(arena, offset, numel) is called when a contiguous slice of a gradient arena is
        final for this backward (trainer.GradBucketReducer.ready); None disables it."""
        self._rt.grad_hook = fn

    @property
    def dtype(self):
        return self._rt.dtype

    def arenas(self):
        out = [self.clip.arena]
        for a in (self.text_adapter, self.vision_adapter):
            if a is not None:
                out.append(a.arena)
        for a in (self.shared_adapters or []):
            out.append(a.arena)
        return out

    # ------------------------------------------------------------------ features
    def _tower_training(self):
        train = torch.is_grad_enabled() and self.clip.arena.any_requires_grad()
        if train and self._rt.fp8:
            raise NotImplementedError("precision='fp8' towers are forward-only; freeze the CLIP parameters")
        return train

    def _adapter_needs_grad(self, mod, x):
        return torch.is_grad_enabled() and (mod.arena.any_requires_grad() or x.requires_grad)

    def _check_device(self, t):
        if t.device != self.clip.arena.device:
            t = t.to(self.clip.arena.device, non_blocking=True)
        return t

    def text_hidden_states(self, input_ids, attention_mask=None):
        self._rt.train_tower = self._tower_training()
        ids = self._check_device(input_ids)
        mask = self._check_device(attention_mask) if attention_mask is not None else None
        h = T.TextTowerFn.apply(ids, mask, _anchor(self.clip), self._rt)
        if self.use_text_adapter:
            h = T.AdapterFn.apply(h, _anchor(self.text_adapter), self._rt, self.text_adapter,
                                  self._adapter_needs_grad(self.text_adapter, h))
        return h

    def get_text_features(self, input_ids, attention_mask):
        """model_m.py:77-105: text tower -> adapter -> token 0 -> text_projection."""
        self._rt.train_tower = self._tower_training()
        ids = self._check_device(input_ids)
        mask = self._check_device(attention_mask) if attention_mask is not None else None
        h = T.TextTowerFn.apply(ids, mask, _anchor(self.clip), self._rt)
        idx = None
        if self.pooling == "eos":
            t = self.config.text_config
            ids = ids.to(torch.int64).contiguous()
            idx = torch.empty(ids.shape[0], dtype=torch.int32, device=ids.device)
            mode = 2 if t.eos_token_id == 2 else 1
            T.call("clipmi_pool_index", T.K.stream(), T.P_(ids), ids.shape[0], ids.shape[1], t.eos_token_id, mode,
                   T.P_(idx))
        if self.use_text_adapter or self.use_shared_adapters:
            h = T.PoolRowsFn.apply(h, self._rt, idx)
            idx = None
        if self.use_text_adapter:
            # the adapter is row-wise (down/GELU/up/residual/LN per token) and only the pooled
            # row reaches the features (model_m.py:102), so it runs on that row alone: the same
            # values as adapting all 77 tokens and then pooling, at 1/77 of the work
            h = T.AdapterFn.apply(h, _anchor(self.text_adapter), self._rt, self.text_adapter,
                                  self._adapter_needs_grad(self.text_adapter, h))
        if self.use_shared_adapters:
            # model_m.py:95-100: image tokens = the vision position embedding, shared by the batch
            from .shared_adapter import SharedAdapterFn
            # the Parameter itself, so an unfrozen CLIP gets this path's position-embedding gradient
            pos = self.clip.vision_model.embeddings.position_embedding.weight
            # the shared adapters' position-embedding gradient lands after the vision tower's
            # backward: the tower must then leave its embedding block to the reducer's finish()
            self._rt.shared_pos_grad = torch.is_grad_enabled() and pos.requires_grad
            for sa in self.shared_adapters:
                need = self._adapter_needs_grad(sa, h) or (torch.is_grad_enabled() and pos.requires_grad)
                h = SharedAdapterFn.apply(h, _anchor(sa), sa, pos, need)
        return T.PoolProjFn.apply(h, self.clip.text_projection.weight, self._rt, "text_projection.weight", idx)


    def vision_hidden_states(self, pixel_values):
        self._rt.train_tower = self._tower_training()
        px = self._check_device(pixel_values)
        h = T.VisionTowerFn.apply(px, _anchor(self.clip), self._rt)
        if self.use_vision_adapter:
            h = T.AdapterFn.apply(h, _anchor(self.vision_adapter), self._rt, self.vision_adapter,
                                  self._adapter_needs_grad(self.vision_adapter, h))
        return h

    def get_image_features(self, pixel_values):
        """model_m.py:107-125: vision tower (no post-LN, quirk Q2) -> adapter -> CLS -> visual_projection."""
        self._rt.train_tower = self._tower_training()
        h = T.VisionTowerFn.apply(self._check_device(pixel_values), _anchor(self.clip), self._rt)
        if self.use_vision_adapter:  # CLS row only (model_m.py:122), as in get_text_features
            h = T.PoolRowsFn.apply(h, self._rt, None)
            h = T.AdapterFn.apply(h, _anchor(self.vision_adapter), self._rt, self.vision_adapter,
                                  self._adapter_needs_grad(self.vision_adapter, h))
        return T.PoolProjFn.apply(h, self.clip.visual_projection.weight, self._rt, "visual_projection.weight", None)

    # ------------------------------------------------------------------ forward
    def _overlap_ok(self, input_ids, attention_mask, pixel_values):
        """Run the text tower on a second HIP stream beside the vision tower (forward and, through
        autograd's per-node streams, backward): the two towers' kernels fill each other's tail
        rounds.  Safe when the towers share no gradient state that backward initialises on one
        stream: the clip arena's grads are attached by ContrastiveFn (on the caller's stream)
        before either tower's backward when logit_scale trains, and adapters have one arena each."""
        if os.environ.get("CLIPMI_OVERLAP", "1") == "0" or input_ids is None or attention_mask is None:
            return False
        if pixel_values is None or not isinstance(pixel_values, torch.Tensor) or not pixel_values.is_cuda:
            return False
        if self.clip.arena.device.type != "cuda":
            return False
        if not torch.is_grad_enabled() or not self.clip.arena.any_requires_grad():
            return True
        if self.use_shared_adapters:  # the text branch then also writes a vision parameter's gradient
            return False
        return self.clip.logit_scale.requires_grad

    def _side_stream(self):
        dev = self.clip.arena.device
        st = getattr(self, "_side", None)
        if st is None or st.device != dev:
            st = torch.cuda.Stream(device=dev)
            self._side = st
        return st

    def forward(self, input_ids=None, attention_mask=None, pixel_values=None, return_loss=True):
        """model_m.py:127-176."""
        if self._overlap_ok(input_ids, attention_mask, pixel_values):
            text_features, image_features = self._both_towers_overlapped(input_ids, attention_mask, pixel_values)
        else:
            if input_ids is not None and attention_mask is not None:
                text_features = self.get_text_features(input_ids, attention_mask)
            else:
                text_features = None
            image_features = self.get_image_features(pixel_values) if pixel_values is not None else None
        if return_loss and text_features is not None and image_features is not None:
            group = self.process_group
            loss, t, i, lpt, lpi = T.ContrastiveFn.apply(text_features, image_features, self.clip.logit_scale,
                                                         group, True, self.clip.arena)
            world = CM.world_rank(group)[0]
            return {"loss": loss, "text_features": t, "image_features": i, "logits_per_text": lpt,
                    "logits_per_image": lpt.t() if world == 1 and lpt is not None else lpi}
        return {"text_features": text_features, "image_features": image_features}

    def _both_towers_overlapped(self, input_ids, attention_mask, pixel_values):
        main = torch.cuda.current_stream(self.clip.arena.device)
        side = self._side_stream()
        for a in self.arenas():  # bf16 shadows refreshed on the caller's stream, before the fork
            a.sync_shadow()
        side.wait_stream(main)
        with torch.cuda.stream(side):
            for t in (input_ids, attention_mask):
                if isinstance(t, torch.Tensor) and t.is_cuda:
                    t.record_stream(side)
            text_features = _JoinOnBackward.apply(self.get_text_features(input_ids, attention_mask), main, side)
        image_features = self.get_image_features(pixel_values)
        main.wait_stream(side)
        text_features.record_stream(main)
        return text_features, image_features

    # ------------------------------------------------------------------ checkpoints
    def save_adapter_weights(self, save_path):
        """model_m.py:178-203 — {"text_adapter": sd, "vision_adapter": sd} via torch.save."""
        adapter_state_dict = {}
        if self.use_text_adapter:
            adapter_state_dict["text_adapter"] = {k: v.detach().clone() for k, v in self.text_adapter.state_dict().items()}
        if self.use_vision_adapter:
            adapter_state_dict["vision_adapter"] = {k: v.detach().clone()
                                                    for k, v in self.vision_adapter.state_dict().items()}
        if self.use_shared_adapters:
            adapter_state_dict["shared_adapters"] = {k: v.detach().clone()
                                                     for k, v in self.shared_adapters.state_dict().items()}
        if not adapter_state_dict:
            raise ValueError("No adapters enabled to save")
        d = os.path.dirname(save_path)
        if d:  # the reference calls os.makedirs("") for bare file names and crashes
            os.makedirs(d, exist_ok=True)
        torch.save(adapter_state_dict, save_path)
        print(f"Adapter weights saved to {save_path}")
        print(f"Saved adapters: {list(adapter_state_dict.keys())}")

    def load_adapter_weights(self, load_path):
        """model_m.py:205-248 (same validation and error types; safe loader only)."""
        if not os.path.exists(load_path):
            raise FileNotFoundError(f"No adapter weights found at {load_path}")
        adapter_state_dict = torch.load(load_path, map_location=self.clip.arena.device, weights_only=True)
        if "text_adapter" in adapter_state_dict:
            if not self.use_text_adapter:
                raise ValueError("Text adapter weights found but text adapter is not enabled")
            self.text_adapter.load_state_dict(adapter_state_dict["text_adapter"])
        elif self.use_text_adapter:
            raise ValueError("Text adapter is enabled but no weights found in checkpoint")
        if "vision_adapter" in adapter_state_dict:
            if not self.use_vision_adapter:
                raise ValueError("Vision adapter weights found but vision adapter is not enabled")
            self.vision_adapter.load_state_dict(adapter_state_dict["vision_adapter"])
        elif self.use_vision_adapter:
            raise ValueError("Vision adapter is enabled but no weights found in checkpoint")
        if "shared_adapters" in adapter_state_dict:
            if not self.use_shared_adapters:
                raise ValueError("Shared adapter weights found but shared adapters are not enabled")
            self.shared_adapters.load_state_dict(adapter_state_dict["shared_adapters"])
        elif self.use_shared_adapters:
            raise ValueError("Shared adapters are enabled but no weights found in checkpoint")
        print(f"Adapter weights loaded from {load_path}")
        print(f"Loaded adapters: {list(adapter_state_dict.keys())}")

    def input_error(self) -> bool:
        """True if any token id seen so far was outside the vocabulary (checked lazily, on device)."""
        return bool(self._rt.bad_flag.item())

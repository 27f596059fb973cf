"""Feature-level adapter heads over the native towers.

Drop-in for model_t.py's ``CLIPAdapter`` (:35-298) and ``ZeroShotEmotionRecognition``
(:300-404): the frozen backbone's features come from the clipmi towers (HF
``get_text_features`` / ``get_image_features`` semantics: EOS pooling and post-LN, which
model_t uses, unlike model_m's first-token pooling), and every head operation runs in
``libclipmi`` (csrc/heads.hip): the fused adapter + residual blend + renormalisation, the
prototype / all-description class scores, the CE loss and its backward, and Adam
(clipmi_adamw with weight decay 0 == torch.optim.Adam).

Differences from the reference, all forced by the offline image: the backbone is built from a
local config/weights path (never a hub name) and the class descriptions arrive pre-tokenised
(``{emotion: (input_ids [n, 77], attention_mask [n, 77])}``), since the CLIP BPE files are hub
downloads.  ``constants.EMOTIONS`` order is kept by the dict's order.
"""
from __future__ import annotations

import ctypes
import math
import os

import torch
from torch import nn

from . import _lib
from . import towers as T

c_vp, c_int, c_float, c_i64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_int64
_lib.declare("clipmi_feature_adapter_fwd", [c_vp, c_vp, c_int, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_float, c_int,
                                            c_vp, c_vp, c_vp, c_vp, c_vp, c_float])
_lib.declare("clipmi_feature_adapter_bwd_ws", [c_int, c_int, c_int])
_lib.declare("clipmi_feature_adapter_bwd", [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_vp, c_float,
                                            c_vp, c_vp, c_i64, c_float])
_lib.declare("clipmi_dropout_mask", [c_vp, c_vp, c_i64, c_float, ctypes.c_uint64, ctypes.c_uint64])
_lib.declare("clipmi_dropout_apply", [c_vp, c_vp, c_vp, c_i64, c_float, c_vp, c_vp])
_lib.declare("clipmi_fuse_avg", [c_vp, c_vp, c_vp, c_int, c_int, c_vp, c_vp])
_lib.declare("clipmi_fuse_avg_bwd", [c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_vp])
_lib.declare("clipmi_class_scores", [c_vp, c_vp, c_int, c_int, c_vp, c_vp, c_int, c_float, c_vp, c_vp, c_vp, c_vp,
                                     c_vp, c_vp])
_lib.declare("clipmi_row_mean", [c_vp, c_vp, c_int, c_vp])
_lib.declare("clipmi_class_ce_bwd", [c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_float, c_vp, c_vp, c_vp])

P_, call = T.P_, T.call


class _Linear:
    """nn.Linear's parameters as views of the adapter's flat fp32 buffer (weight [out, in])."""

    def __init__(self, weight, bias):
        self.weight, self.bias = weight, bias


class Dropout:
    """nn.Dropout(p) masks from libclipmi's counter-based generator: each draw takes the next
    `n` counters of (seed, offset), so a seed reproduces the whole sequence of masks."""

    def __init__(self, p, seed):
        self.p, self.seed, self.offset = float(p), int(seed) & (2 ** 63 - 1), 0

    def mask(self, n, device):
        keep = torch.empty(n, dtype=torch.uint8, device=device)
        call("clipmi_dropout_mask", T.K.stream(), P_(keep), n, self.p, self.seed, self.offset)
        self.offset += n
        return keep

    @property
    def scale(self):
        return 1.0 / (1.0 - self.p)


class FeatureAdapter(nn.Module):
    """model_t.VisualAdapter / TextAdapter (:13-33): fc2(relu(fc1(x))), parameters in one flat
    fp32 buffer [fc1.weight | fc1.bias | fc2.weight | fc2.bias] so the gradient and the Adam
    state are flat buffers too.  Initialised like nn.Linear (seeded), or from a state dict.
    dropout > 0 is model_v.BaseAdapter (:18-27): fc2(dropout(relu(fc1(x)))), active in
    training mode (nn.Module.train / eval)."""

    def __init__(self, input_dim, bottleneck_dim, device="cuda", seed=0, dropout=0.0):
        super().__init__()
        E, A = input_dim, bottleneck_dim
        self.E, self.A = E, A
        self.dropout = Dropout(dropout, seed * 7919 + 17) if dropout > 0 else None
        n = 2 * A * E + A + E
        self.flat = torch.zeros(n, dtype=torch.float32, device=device)
        self.grad = torch.zeros_like(self.flat)
        self.exp_avg = torch.zeros_like(self.flat)
        self.exp_avg_sq = torch.zeros_like(self.flat)
        self.step_count = 0
        o = [0, A * E, A * E + A, 2 * A * E + A, n]
        self.fc1 = _Linear(self.flat[o[0]:o[1]].view(A, E), self.flat[o[1]:o[2]])
        self.fc2 = _Linear(self.flat[o[2]:o[3]].view(E, A), self.flat[o[3]:o[4]])
        g = torch.Generator().manual_seed(seed)
        ref1, ref2 = nn.Linear(E, A), nn.Linear(A, E)
        for lin in (ref1, ref2):  # nn.Linear.reset_parameters' bounds, seeded
            bound = 1.0 / math.sqrt(lin.in_features)
            with torch.no_grad():
                lin.weight.uniform_(-bound, bound, generator=g)
                lin.bias.uniform_(-bound, bound, generator=g)
        self.load_state_dict_(
            {"fc1.weight": ref1.weight, "fc1.bias": ref1.bias, "fc2.weight": ref2.weight, "fc2.bias": ref2.bias})

    def state_dict_(self):
        return {"fc1.weight": self.fc1.weight.detach().cpu().clone(), "fc1.bias": self.fc1.bias.detach().cpu().clone(),
                "fc2.weight": self.fc2.weight.detach().cpu().clone(), "fc2.bias": self.fc2.bias.detach().cpu().clone()}

    def load_state_dict_(self, sd):
        with torch.no_grad():
            for k, dst in (("fc1.weight", self.fc1.weight), ("fc1.bias", self.fc1.bias),
                           ("fc2.weight", self.fc2.weight), ("fc2.bias", self.fc2.bias)):
                src = torch.as_tensor(sd[k], dtype=torch.float32)
                if tuple(src.shape) != tuple(dst.shape):
                    raise ValueError(f"{k}: shape {tuple(src.shape)} != {tuple(dst.shape)}")
                dst.copy_(src)

    def state_dict(self, *args, **kwargs):
        """nn.Linear key names of model_t / model_v adapters (fc1.weight, fc1.bias, fc2.weight, fc2.bias)."""
        return self.state_dict_()

    def load_state_dict(self, state_dict, strict=True):
        if strict and set(state_dict) != {"fc1.weight", "fc1.bias", "fc2.weight", "fc2.bias"}:
            raise RuntimeError(f"Error(s) in loading state_dict for {type(self).__name__}: keys {sorted(state_dict)}")
        self.load_state_dict_(state_dict)

    def parameters(self, recurse=True):  # model_t passes these to optim.Adam
        return iter([self.fc1.weight, self.fc1.bias, self.fc2.weight, self.fc2.bias])

    def blend(self, x, alpha, norm_in):
        """out = normalise(alpha * adapter(xn) + (1 - alpha) * xn), xn = x/|x| if norm_in else x.
        Returns (out, saved) where saved feeds backward."""
        x = x.to(device=self.flat.device, dtype=torch.float32).contiguous()
        B = x.shape[0]
        if x.dim() != 2 or x.shape[1] != self.E:
            raise ValueError(f"features must be [B, {self.E}], got {tuple(x.shape)}")
        xn, out = torch.empty_like(x), torch.empty_like(x)
        h = torch.empty(B, self.A, dtype=torch.float32, device=x.device)
        rz = torch.empty(B, dtype=torch.float32, device=x.device)
        keep, ks = None, 1.0
        if self.dropout is not None and self.training:
            keep, ks = self.dropout.mask(B * self.A, x.device), self.dropout.scale
        call("clipmi_feature_adapter_fwd", T.K.stream(), P_(x), B, self.E, self.A, P_(self.fc1.weight),
             P_(self.fc1.bias), P_(self.fc2.weight), P_(self.fc2.bias), float(alpha), int(norm_in), P_(xn), P_(h),
             P_(out), P_(rz), P_(keep), ks)
        return out, (out, rz, xn, h, float(alpha), ks)

    def backward_(self, dout, saved):
        """grad += d loss / d params given dout = d loss / d out (accumulates, like autograd)."""
        out, rz, xn, h, alpha, ks = saved
        B = out.shape[0]
        ws = T._ws(_lib.lib().clipmi_feature_adapter_bwd_ws(B, self.E, self.A), out.device)
        call("clipmi_feature_adapter_bwd", T.K.stream(), P_(dout.contiguous()), P_(out), P_(rz), P_(xn), P_(h), B,
             self.E, self.A, P_(self.fc2.weight), alpha, P_(self.grad), P_(ws), ws.numel(), ks)

    def forward(self, x):
        """fc2(relu(fc1(x))) (model_t.py:22-23): the fused kernel at alpha = 1, no input
        normalisation, with its output normalisation undone (out / rz = z)."""
        out, saved = self.blend(x, 1.0, False)
        return out / saved[1][:, None]

    def adam_step(self, lr, betas=(0.9, 0.999), eps=1e-8):
        self.step_count += 1
        call("clipmi_adamw", T.K.stream(), P_(self.flat), P_(self.grad), P_(self.exp_avg), P_(self.exp_avg_sq), None,
             self.flat.numel(), float(lr), float(betas[0]), float(betas[1]), float(eps), 0.0, self.step_count, None)


VisualAdapter = FeatureAdapter
TextAdapter = FeatureAdapter


def class_scores(img, desc, offsets, scale, labels=None):
    """-> (scores [B, C], probs [B, C], loss_rows, dscore); per class the max over its
    descriptions (offsets int32 [C+1]); CE outputs only when labels are given."""
    B, E = img.shape
    C = offsets.numel() - 1
    dev = img.device
    scores = torch.empty(B, C, dtype=torch.float32, device=dev)
    probs = torch.empty_like(scores)
    loss_rows = dscore = bad = None
    if labels is not None:
        labels = labels.to(device=dev, dtype=torch.int64).contiguous()
        loss_rows = torch.empty(B, dtype=torch.float32, device=dev)
        dscore = torch.empty_like(scores)
        bad = torch.zeros(1, dtype=torch.int32, device=dev)
    call("clipmi_class_scores", T.K.stream(), P_(img.contiguous()), B, E, P_(desc.contiguous()), P_(offsets), C,
         float(scale), P_(scores), P_(probs), P_(labels), P_(loss_rows), P_(dscore), P_(bad))
    return scores, probs, loss_rows, dscore, bad


class _Backbone:
    """Frozen HF-semantics features from the clipmi towers: text = EOS-pooled + projection
    ([HF] get_text_features), image = CLS + post_layernorm + projection ([HF] get_image_features)."""

    def __init__(self, model_name, device, precision):
        from .model import CLIPWithAdapters
        self.m = CLIPWithAdapters(model_name, use_text_adapter=False, use_vision_adapter=False,
                                  use_shared_adapters=False, freeze_clip=True, device=device, precision=precision,
                                  pooling="eos")
        self.logit_scale = self.m.clip.logit_scale

    @torch.no_grad()
    def get_text_features(self, input_ids, attention_mask=None):
        return self.m.get_text_features(input_ids, attention_mask).float()

    @torch.no_grad()
    def get_image_features(self, pixel_values):
        m, rt = self.m, self.m._rt
        rt.train_tower = False
        h = T.VisionTowerFn.apply(m._check_device(pixel_values), None, rt)
        cls = T.PoolRowsFn.apply(h, rt, None).reshape(h.shape[0], -1).contiguous()
        v = m.config.vision_config
        arena = m.clip.arena
        wbuf = T._wbuf(arena, rt.dtype)
        R, D = cls.shape
        y = torch.empty_like(cls)
        stats = torch.empty(2, R, dtype=torch.float32, device=cls.device)
        call("clipmi_layernorm_fwd", T.K.stream(), T.dcode(rt.dtype), P_(cls), D, P_(y), D,
             arena.ptr("vision_model.post_layernorm.weight", wbuf), arena.ptr("vision_model.post_layernorm.bias", wbuf),
             P_(stats[0]), P_(stats[1]), R, D, v.layer_norm_eps, None, None, 0)
        return T.PoolProjFn.apply(y.view(R, 1, D), None, rt, "visual_projection.weight", None).float()


def _normalise(x):
    y = torch.empty_like(x)
    n = torch.empty(x.shape[0], dtype=torch.float32, device=x.device)
    call("clipmi_l2norm_fwd", T.K.stream(), P_(x), P_(y), P_(n), x.shape[0], x.shape[1])
    return y


class _DescriptionBank:
    """Per-description normalised text features, their per-class means (model_t.py:71-98)."""

    def encode(self, model, descriptions):
        feats, off = [], [0]
        self.emotions = list(descriptions.keys())
        for emo in self.emotions:
            ids, mask = descriptions[emo]
            f = model.get_text_features(ids, mask)
            feats.append(_normalise(f.float().contiguous()))
            off.append(off[-1] + f.shape[0])
        self.desc = torch.cat(feats, 0).contiguous()
        dev = self.desc.device
        self.offsets = torch.tensor(off, dtype=torch.int32, device=dev)
        self.protos_offsets = torch.arange(len(self.emotions) + 1, dtype=torch.int32, device=dev)
        self.protos = torch.stack([x.mean(0) for x in feats]).contiguous()  # .mean(dim=0) per class


class CLIPAdapter:
    """model_t.CLIPAdapter (:35-298) on libclipmi.  ``model`` is a model name / local weights
    path (a clipmi backbone is built) or any object with ``get_text_features``,
    ``get_image_features`` and ``logit_scale`` (HF CLIPModel semantics)."""

    def __init__(self, model_name, alpha=0.2, beta=0.2, bottleneck_dim=64, descriptions=None, device="cuda",
                 precision="fp32", seed=0):
        self.model = _Backbone(model_name, device, precision) if isinstance(model_name, str) else model_name
        self.processor = None  # tokenisation happens before this path (BPE files are hub downloads)
        dim = int(self.model.m.config.projection_dim if isinstance(self.model, _Backbone)
                  else self.model.projection_dim)
        self.image_feature_dim = self.text_feature_dim = dim
        self.visual_adapter = VisualAdapter(dim, bottleneck_dim, device, seed=seed)
        self.text_adapter = TextAdapter(dim, bottleneck_dim, device, seed=seed + 1)
        self.alpha, self.beta = alpha, beta
        if descriptions is None:
            raise ValueError("descriptions {emotion: (input_ids, attention_mask)} are required (no tokenizer offline)")
        self.emotion_descriptions = descriptions
        self.encode_emotion_descriptions()

    def encode_emotion_descriptions(self):
        self._bank = _DescriptionBank()
        self._bank.encode(self.model, self.emotion_descriptions)
        self.emotion_embedding_tensor = self._bank.protos

    def update_emotion_embeddings(self):
        """model_t.py:100-121."""
        self.adapted_emotion_embedding_tensor, _ = self.text_adapter.blend(self.emotion_embedding_tensor, self.beta,
                                                                           False)

    def train_step(self, pixel_values, labels, learning_rate, temperature):
        """One iteration of model_t.py:165-218 (features -> adapters -> logits -> CE -> Adam).
        Labels are validated on the host first: torch's CrossEntropyLoss raises before
        optimizer.step(), so a bad batch must leave both adapters untouched."""
        lab = torch.as_tensor(labels).detach().to("cpu", torch.int64)
        C = self.emotion_embedding_tensor.shape[0]
        bad_lab = lab[(lab < 0) | (lab >= C)]
        if bad_lab.numel():
            raise IndexError(f"Target {int(bad_lab[0])} is out of bounds.")
        f = self.model.get_image_features(pixel_values)
        img, s_img = self.visual_adapter.blend(f, self.alpha, True)
        txt, s_txt = self.text_adapter.blend(self.emotion_embedding_tensor, self.beta, False)
        bank = self._bank
        _, _, loss_rows, dscore, bad = class_scores(img, txt, bank.protos_offsets, temperature, labels)
        loss = torch.empty(1, dtype=torch.float32, device=img.device)
        B, C, E = img.shape[0], txt.shape[0], img.shape[1]
        call("clipmi_row_mean", T.K.stream(), P_(loss_rows), B, P_(loss))
        dimg, dtxt = torch.empty_like(img), torch.empty_like(txt)
        call("clipmi_class_ce_bwd", T.K.stream(), P_(dscore), P_(img), P_(txt), B, C, E, float(temperature), None,
             P_(dimg), P_(dtxt))
        for ad, d, sv in ((self.visual_adapter, dimg, s_img), (self.text_adapter, dtxt, s_txt)):
            ad.grad.zero_()  # optimizer.zero_grad()
            ad.backward_(d, sv)
        self.visual_adapter.adam_step(learning_rate)
        self.text_adapter.adam_step(learning_rate)
        return loss, bad

    def train(self, train_loader, num_epochs=50, learning_rate=3e-4):
        """model_t.py:123-229; returns the per-epoch mean losses."""
        temperature = float(self.model.logit_scale.detach().float().exp().item())
        history = []
        for _ in range(num_epochs):
            losses = []
            for pixel_values, labels, _ in train_loader:
                loss, bad = self.train_step(pixel_values, labels, learning_rate, temperature)
                losses.append(loss)
                if int(bad.item()):
                    raise IndexError("Target out of bounds")  # torch CrossEntropyLoss's error
            history.append(float(torch.cat(losses).mean().item()))
            self.update_emotion_embeddings()
        self.update_emotion_embeddings()
        return history

    def _image(self, pixel_values):
        f = self.model.get_image_features(pixel_values)
        img, _ = self.visual_adapter.blend(f, self.alpha, True)
        return img

    def predict(self, pixel_values):
        """model_t.py:231-250."""
        img = self._image(pixel_values)
        protos = getattr(self, "adapted_emotion_embedding_tensor", None)
        if protos is None:
            protos = self.emotion_embedding_tensor
        return class_scores(img, protos, self._bank.protos_offsets, 100.0)[1]

    def predict_with_all_descriptions(self, pixel_values):
        """model_t.py:252-298: every description through the text adapter, max per class."""
        img = self._image(pixel_values)
        desc, _ = self.text_adapter.blend(self._bank.desc, self.beta, False)
        return class_scores(img, desc, self._bank.offsets, 100.0)[1]


class ZeroShotEmotionRecognition:
    """model_t.ZeroShotEmotionRecognition (:300-404) on libclipmi."""

    def __init__(self, model_name, descriptions=None, device="cuda", precision="fp32"):
        self.model = _Backbone(model_name, device, precision) if isinstance(model_name, str) else model_name
        self.processor = None
        if descriptions is None:
            raise ValueError("descriptions {emotion: (input_ids, attention_mask)} are required (no tokenizer offline)")
        self.emotion_descriptions = descriptions
        self.encode_emotion_descriptions()

    def encode_emotion_descriptions(self):
        self._bank = _DescriptionBank()
        self._bank.encode(self.model, self.emotion_descriptions)
        self.emotion_embedding_tensor = self._bank.protos

    def _image(self, pixel_values):
        return _normalise(self.model.get_image_features(pixel_values).float().contiguous())

    def predict(self, pixel_values):
        return class_scores(self._image(pixel_values), self.emotion_embedding_tensor, self._bank.protos_offsets,
                            100.0)[1]

    def predict_with_all_descriptions(self, pixel_values):
        return class_scores(self._image(pixel_values), self._bank.desc, self._bank.offsets, 100.0)[1]


class ContextAdapter(FeatureAdapter):
    """model_v.ContextAdapter (:30-31): the BaseAdapter bottleneck on VLM context features."""


class EnhancedCLIPAdapter(nn.Module):
    """model_v.EnhancedCLIPAdapter (:146-360) on libclipmi: visual / text / context BaseAdapters
    (fc1 -> ReLU -> Dropout(0.1) -> fc2), alpha / beta / gamma residual blends with
    renormalisation, average fusion of image and context features, logits = exp(logit_scale) *
    fused . text^T, predict_probs = softmax; training (main.py:55-100) = CrossEntropy + Adam over
    the three adapters, emotion embeddings refreshed after every epoch.

    Every head operation runs in csrc/heads.hip (the fused adapter with its dropout mask, the
    fusion, the class scores and CE, Adam).  The VLM context extractor (Qwen2.5-VL generation,
    model_v.py:43-142) is outside this path: context features are passed to forward(), as the
    reference's training loop does (main.py:68-77).  Descriptions arrive pre-tokenised
    ({emotion: (input_ids, attention_mask)}; model_v uses one per emotion, "A person expressing
    {emotion}", :204-206)."""

    def __init__(self, clip_model_name, alpha=0.2, beta=0.2, gamma=0.3, bottleneck_dim=192, device="cuda",
                 vlm_context_extractor=None, *, descriptions=None, precision="fp32", seed=0):
        super().__init__()
        self.device = device
        self.model = _Backbone(clip_model_name, device, precision) if isinstance(clip_model_name, str) \
            else clip_model_name
        self.processor = None
        dim = int(self.model.m.config.projection_dim if isinstance(self.model, _Backbone)
                  else self.model.projection_dim)
        self.image_feature_dim = self.text_feature_dim = dim
        self.visual_adapter = FeatureAdapter(dim, bottleneck_dim, device, seed=seed, dropout=0.1)
        self.text_adapter = FeatureAdapter(dim, bottleneck_dim, device, seed=seed + 1, dropout=0.1)
        self.context_adapter = ContextAdapter(dim, bottleneck_dim, device, seed=seed + 2, dropout=0.1)
        self.alpha, self.beta, self.gamma = alpha, beta, gamma
        self.vlm_context_extractor = vlm_context_extractor
        self.emotion_descriptions = descriptions
        self.adapted_emotion_embedding_tensor = None
        self.emotion_embedding_tensor = None

    def _adapters(self):
        return (self.visual_adapter, self.text_adapter, self.context_adapter)

    _CKPT_KEYS = (("visual_adapter_state_dict", "visual_adapter"), ("text_adapter_state_dict", "text_adapter"),
                  ("context_adapter_state_dict", "context_adapter"))

    def save_adapter_weights(self, path):
        """main.py:186-193's checkpoint: {visual,text,context}_adapter_state_dict -> nn.Linear state dicts."""
        torch.save({k: getattr(self, a).state_dict() for k, a in self._CKPT_KEYS}, path)

    def load_adapter_weights(self, path):
        """Reads main.py:186-193's checkpoint (safe loader); a missing file raises FileNotFoundError and a
        missing adapter key KeyError, as indexing the reference's dict would."""
        if not os.path.exists(path):
            raise FileNotFoundError(f"No adapter weights found at {path}")
        sd = torch.load(path, map_location="cpu", weights_only=True)
        for k, a in self._CKPT_KEYS:
            getattr(self, a).load_state_dict(sd[k])

    def encode_emotion_descriptions(self, emotions=None):
        """model_v.py:198-240: per emotion the mean of its normalised description features, then
        update_emotion_embeddings()."""
        if self.emotion_descriptions is None:
            raise ValueError("descriptions {emotion: (input_ids, attention_mask)} are required (no tokenizer offline)")
        descs = self.emotion_descriptions
        if emotions is not None:
            descs = {e: descs[e] for e in emotions}
        self._bank = _DescriptionBank()
        self._bank.encode(self.model, descs)
        self.emotion_embedding_tensor = self._bank.protos
        self.update_emotion_embeddings()

    def update_emotion_embeddings(self):
        """model_v.py:242-258 (in the module's current mode: dropout applies in training mode)."""
        if self.emotion_embedding_tensor is None:
            print("Warning: Original emotion embeddings not encoded. Call encode_emotion_descriptions first.")
            return
        self.adapted_emotion_embedding_tensor, _ = self.text_adapter.blend(self.emotion_embedding_tensor, self.beta,
                                                                           False)

    def _forward(self, pixel_values, context_features):
        """(logits, state for backward); model_v.py:260-343."""
        img_raw = self.model.get_image_features(pixel_values).float().contiguous()
        img, s_img = self.visual_adapter.blend(img_raw, self.alpha, True)
        combined, s_ctx, s_fuse = img, None, None
        if context_features is not None and context_features.nelement() > 0:
            if context_features.shape[-1] != self.text_feature_dim:
                print(f"Warning: Context feature dimension mismatch. Expected {self.text_feature_dim}, "
                      f"got {context_features.shape[-1]}. Skipping context.")
            else:
                ctx = context_features.to(device=img.device, dtype=torch.float32).contiguous()
                ctx_f, s_ctx = self.context_adapter.blend(ctx, self.gamma, False)
                combined = torch.empty_like(img)
                ru = torch.empty(img.shape[0], dtype=torch.float32, device=img.device)
                call("clipmi_fuse_avg", T.K.stream(), P_(img), P_(ctx_f), img.shape[0], img.shape[1], P_(combined),
                     P_(ru))
                s_fuse = (combined, ru)
        s_txt = None
        if self.training or self.adapted_emotion_embedding_tensor is None:
            txt, s_txt = self.text_adapter.blend(self.emotion_embedding_tensor, self.beta, False)
        else:
            txt = self.adapted_emotion_embedding_tensor
        temperature = float(self.model.logit_scale.detach().float().exp().item())
        return combined, txt, temperature, (s_img, s_ctx, s_fuse, s_txt)

    def forward(self, pixel_values, context_features=None, use_adapters_for_training=True):
        combined, txt, temperature, _ = self._forward(pixel_values, context_features)
        return class_scores(combined, txt, self._bank.protos_offsets, temperature)[0]

    def predict_probs(self, pixel_values, context_features=None):
        """model_v.py:345-353."""
        self.eval()
        combined, txt, temperature, _ = self._forward(pixel_values, context_features)
        return class_scores(combined, txt, self._bank.protos_offsets, temperature)[1]

    def get_trainable_parameters(self):
        params = []
        for ad in self._adapters():
            params.extend(list(ad.parameters()))
        return params

    def train_step(self, pixel_values, labels, context_features, learning_rate):
        """One iteration of main.py:66-86: logits -> CrossEntropy -> backward -> Adam (all three
        adapters).  Labels are validated on the host first (no update on a bad batch)."""
        lab = torch.as_tensor(labels).detach().to("cpu", torch.int64)
        C = self.emotion_embedding_tensor.shape[0]
        bad_lab = lab[(lab < 0) | (lab >= C)]
        if bad_lab.numel():
            raise IndexError(f"Target {int(bad_lab[0])} is out of bounds.")
        combined, txt, temperature, (s_img, s_ctx, s_fuse, s_txt) = self._forward(pixel_values, context_features)
        _, _, loss_rows, dscore, _ = class_scores(combined, txt, self._bank.protos_offsets, temperature, labels)
        B, E = combined.shape
        loss = torch.empty(1, dtype=torch.float32, device=combined.device)
        call("clipmi_row_mean", T.K.stream(), P_(loss_rows), B, P_(loss))
        dcomb, dtxt = torch.empty_like(combined), torch.empty_like(txt)
        call("clipmi_class_ce_bwd", T.K.stream(), P_(dscore), P_(combined), P_(txt), B, C, E, float(temperature), None,
             P_(dcomb), P_(dtxt))
        for ad in self._adapters():
            ad.grad.zero_()  # optimizer.zero_grad()
        if s_fuse is not None:
            dab = torch.empty_like(dcomb)
            call("clipmi_fuse_avg_bwd", T.K.stream(), P_(dcomb), P_(s_fuse[0]), P_(s_fuse[1]), B, E, P_(dab))
            self.visual_adapter.backward_(dab, s_img)
            self.context_adapter.backward_(dab, s_ctx)
        else:
            self.visual_adapter.backward_(dcomb, s_img)
        if s_txt is not None:
            self.text_adapter.backward_(dtxt, s_txt)
        for ad in self._adapters():
            ad.adam_step(learning_rate)
        return loss

    def train_adapters(self, train_loader, num_epochs, learning_rate):
        """main.py:55-100 (train_model): Adam over the adapters, CE on the logits, the emotion
        embeddings refreshed after each epoch; returns the per-epoch mean losses."""
        self.train()
        history = []
        for _ in range(num_epochs):
            losses = []
            for pixel_values, labels, _, context_features in train_loader:
                losses.append(self.train_step(pixel_values, labels, context_features, learning_rate))
            history.append(float(torch.cat(losses).mean().item()))
            self.update_emotion_embeddings()
        self.eval()
        return history

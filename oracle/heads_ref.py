"""CPU oracle for the feature-level adapter heads (model_t.py CLIPAdapter / ZeroShotEmotionRecognition).

TEST INFRASTRUCTURE ONLY (same rule as oracle/clip_ref.py: only tests/ may import it, as the
checker; the product path is vlm-clip_amd/clipmi/heads.py over csrc/heads.hip).

Plain PyTorch-CPU fp32 restatement, each function citing the reference lines it follows.
Pinned by tests/golden/heads.npz, produced by running the reference's own model_t.CLIPAdapter
.train/.predict/.predict_with_all_descriptions and ZeroShotEmotionRecognition with the CLIP
backbone replaced by a feature lookup (tools/gen_goldens.py gen_heads).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def adapter(x, W1, b1, W2, b2):
    """VisualAdapter/TextAdapter.forward, model_t.py:22-23, 32-33: fc2(relu(fc1(x)))."""
    return F.linear(torch.relu(F.linear(x, W1, b1)), W2, b2)


def blend(x, w, alpha, norm_in):
    """model_t.py:182-197 (visual: normalise, adapt, blend, renormalise) and :196-203 / :113-119
    (text prototypes: adapt, blend, renormalise; the input is the un-renormalised mean)."""
    if norm_in:
        x = x / x.norm(dim=-1, keepdim=True)
    z = alpha * adapter(x, *w) + (1 - alpha) * x
    return z / z.norm(dim=-1, keepdim=True)


def encode(desc, n_per_class):
    """encode_emotion_descriptions, model_t.py:71-98: normalise each description's features,
    class prototype = their mean (not renormalised)."""
    d = desc / desc.norm(dim=-1, keepdim=True)
    return d, d.view(-1, n_per_class, d.shape[1]).mean(1)


def train(img_feats, protos, labels, wv, wt, alpha, beta, temperature, batches, epochs, lr):
    """CLIPAdapter.train, model_t.py:123-229: per batch, CE(temperature * img . txt^T, labels),
    Adam (lr, betas .9/.999, eps 1e-8, no weight decay) over both adapters."""
    params = [p.clone().requires_grad_(True) for p in list(wv) + list(wt)]
    opt = torch.optim.Adam(params, lr=lr)
    for _ in range(epochs):
        for idx in batches:
            img = blend(img_feats[idx], params[:4], alpha, True)
            txt = blend(protos, params[4:], beta, False)
            loss = F.cross_entropy(temperature * img @ txt.T, labels[idx])
            opt.zero_grad()
            loss.backward()
            opt.step()
    return [p.detach() for p in params[:4]], [p.detach() for p in params[4:]]


def predict(img_feats, protos_adapted, wv, alpha):
    """model_t.py:231-250."""
    img = blend(img_feats, wv, alpha, True)
    return torch.softmax(100 * img @ protos_adapted.T, dim=1)


def predict_all(img_feats, desc_n, n_per_class, wv, wt, alpha, beta):
    """model_t.py:252-298: each description through the text adapter, max per class, softmax."""
    img = blend(img_feats, wv, alpha, True)
    d = blend(desc_n, wt, beta, False)
    s = (100 * img @ d.T).view(img.shape[0], -1, n_per_class).amax(2)
    return torch.softmax(s, dim=1)


def zero_shot(img_feats, desc_n, protos, n_per_class):
    """ZeroShotEmotionRecognition.predict / predict_with_all_descriptions, model_t.py:358-404."""
    img = img_feats / img_feats.norm(dim=-1, keepdim=True)
    p = torch.softmax(100 * img @ protos.T, dim=1)
    s = (100 * img @ desc_n.T).view(img.shape[0], -1, n_per_class).amax(2)
    return p, torch.softmax(s, dim=1)


# ---------------------------------------------------------------- model_v.EnhancedCLIPAdapter
# model_v.py cannot be imported in the build container (qwen_vl_utils / bitsandbytes absent,
# SURVEY §8c), so these functions restate it from source; their building blocks (adapter,
# blend, class scores, Adam) are the model_t ones pinned above by tests/golden/heads.npz.  The
# composition (context path, average fusion) is PARITY UNPINNED against a reference run.

def adapter_dropout(x, W1, b1, W2, b2, keep=None, p=0.1):
    """BaseAdapter.forward, model_v.py:25-26: fc2(dropout(relu(fc1(x)))); keep: the 0/1 mask."""
    h = torch.relu(F.linear(x, W1, b1))
    if keep is not None:
        h = h * keep.to(h.dtype) / (1.0 - p)
    return F.linear(h, W2, b2)


def blend_v(x, w, alpha, norm_in, keep=None):
    """model_v.py:269-285 (image: normalise first), :294-302 (context), :325-335 (text)."""
    if norm_in:
        x = x / x.norm(dim=-1, keepdim=True)
    z = alpha * adapter_dropout(x, *w, keep=keep) + (1 - alpha) * x
    return z / z.norm(dim=-1, keepdim=True)


def enhanced_logits(img_feats, ctx, protos, wv, wt, wc, alpha, beta, gamma, temperature, keeps=(None, None, None)):
    """EnhancedCLIPAdapter.forward, model_v.py:260-343 (training-mode text path: the text adapter
    on the prototypes each call); keeps = (visual, context, text) dropout masks or None."""
    img = blend_v(img_feats, wv, alpha, True, keeps[0])
    comb = img
    if ctx is not None and ctx.numel() > 0 and ctx.shape[-1] == img.shape[-1]:
        c = blend_v(ctx, wc, gamma, False, keeps[1])
        comb = (img + c) / 2.0                                  # :310-312
        comb = comb / comb.norm(dim=-1, keepdim=True)            # :313-315
    txt = blend_v(protos, wt, beta, False, keeps[2])
    return temperature * comb @ txt.T                           # :340-342


def enhanced_train_step(params, img_feats, ctx, protos, labels, alpha, beta, gamma, temperature, opt, keeps):
    """main.py:66-86: CE(logits, labels) -> backward -> Adam over the three adapters."""
    wv, wc, wt = params[:4], params[4:8], params[8:]
    loss = F.cross_entropy(enhanced_logits(img_feats, ctx, protos, wv, wt, wc, alpha, beta, gamma, temperature, keeps),
                           labels)
    opt.zero_grad()
    loss.backward()
    opt.step()
    return loss.detach()

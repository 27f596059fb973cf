"""Is a bf16x3 split-operand GEMM accurate enough for north_star's 1e-3 logits?  (GPU diagnostic.)

Config 3's weights and batch (ViT-B/16, B = 1024) through the oracle with every nn.Linear (and the
patch-embed conv) replaced by the split product a.b ~ ah.bh + ah.bl + al.bh (ah = bf16(a),
al = bf16(a - ah); exact bf16 products accumulated in fp32, as the MFMA does), everything else fp32:
  x3     split GEMMs, fp32 activations
  x3s    split GEMMs + every stored activation rounded to hi + lo (16 significant bits)
  x3sa   x3s with the attention products (QK^T, PV) split too
Prints max |dlogit| / |dloss| against the fp32 oracle, and the same for the library's fp32 mode."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vlm-clip_amd")]
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from clipmi import CLIPWithAdapters, synth  # noqa: E402
from oracle import clip_ref as R  # noqa: E402

B = int(os.environ.get("B", "1024"))
dev = os.environ.get("DEV", "cuda")  # DEV=cpu PRESET=tiny: a dry run of the emulation code on the host
PRESET = os.environ.get("PRESET", "B/16")


def rb(x):
    return x.to(torch.bfloat16).float()


def split(x):
    h = rb(x)
    return h, rb(x - h)


def mm3(a, b):  # a @ b with both operands split
    ah, al = split(a)
    bh, bl = split(b)
    return ah @ bh + (ah @ bl + al @ bh)


class X3:
    def __init__(self, store=False, attn=False):
        self.store, self.attn = store, attn

    def st(self, x):
        if not self.store:
            return x
        h, l = split(x)
        return h + l

    def lin(self, x, w, b=None):
        y = mm3(x, w.t())
        return y if b is None else y + b

    def attention(self, x, p, pre, heads, mask):
        Bq, N, D = x.shape
        hd = D // heads
        q = self.st(self.lin(x, p[f"{pre}.q_proj.weight"], p[f"{pre}.q_proj.bias"]))
        k = self.st(self.lin(x, p[f"{pre}.k_proj.weight"], p[f"{pre}.k_proj.bias"]))
        v = self.st(self.lin(x, p[f"{pre}.v_proj.weight"], p[f"{pre}.v_proj.bias"]))
        q, k, v = (t.view(Bq, N, heads, hd).transpose(1, 2) for t in (q, k, v))
        s = (mm3(q, k.transpose(-1, -2)) if self.attn else q @ k.transpose(-1, -2)) * hd ** -0.5
        if mask is not None:
            s = s + mask
        pr = torch.softmax(s, dim=-1)
        o = (mm3(pr, v) if self.attn else pr @ v).transpose(1, 2).reshape(Bq, N, D)
        return self.st(o)

    def layer(self, x, p, pre, heads, eps, mask):
        h = self.st(R.layer_norm(x, p[f"{pre}.layer_norm1.weight"], p[f"{pre}.layer_norm1.bias"], eps))
        o = self.attention(h, p, f"{pre}.self_attn", heads, mask)
        x = self.st(x + self.lin(o, p[f"{pre}.self_attn.out_proj.weight"], p[f"{pre}.self_attn.out_proj.bias"]))
        h = self.st(R.layer_norm(x, p[f"{pre}.layer_norm2.weight"], p[f"{pre}.layer_norm2.bias"], eps))
        a = self.st(R.quick_gelu(self.lin(h, p[f"{pre}.mlp.fc1.weight"], p[f"{pre}.mlp.fc1.bias"])))
        return self.st(x + self.lin(a, p[f"{pre}.mlp.fc2.weight"], p[f"{pre}.mlp.fc2.bias"]))

    def forward(self, b, p, cfg):
        t = cfg.text_config
        x = p["text_model.embeddings.token_embedding.weight"][b["input_ids"]] + \
            p["text_model.embeddings.position_embedding.weight"][: b["input_ids"].shape[1]]
        x = self.st(x)
        mask = R.causal_padding_mask(b["attention_mask"], torch.float32)
        for i in range(t.num_hidden_layers):
            x = self.layer(x, p, f"text_model.encoder.layers.{i}", t.num_attention_heads, t.layer_norm_eps, mask)
        x = self.st(R.layer_norm(x, p["text_model.final_layer_norm.weight"], p["text_model.final_layer_norm.bias"],
                                 t.layer_norm_eps))
        tf = self.lin(x[:, 0, :], p["text_projection.weight"])
        v = cfg.vision_config
        pv = b["pixel_values"]
        w = p["vision_model.embeddings.patch_embedding.weight"]
        P = v.patch_size
        cols = F.unfold(pv, P, stride=P).transpose(1, 2)  # [B, G*G, 3P^2], k = c*P*P + ky*P + kx
        xe = self.lin(cols, w.reshape(w.shape[0], -1))
        xe = torch.cat([p["vision_model.embeddings.class_embedding"].expand(pv.shape[0], 1, -1), xe], dim=1)
        xe = self.st(xe + p["vision_model.embeddings.position_embedding.weight"][None])
        x = self.st(R.layer_norm(xe, p["vision_model.pre_layrnorm.weight"], p["vision_model.pre_layrnorm.bias"],
                                 v.layer_norm_eps))
        for i in range(v.num_hidden_layers):
            x = self.layer(x, p, f"vision_model.encoder.layers.{i}", v.num_attention_heads, v.layer_norm_eps, None)
        imf = self.lin(x[:, 0, :], p["visual_projection.weight"])
        return R.contrastive(tf, imf, p["logit_scale"])


from clipmi import config as C  # noqa: E402
with torch.no_grad():
    if dev == "cuda":
        m = CLIPWithAdapters(PRESET, use_text_adapter=False, use_vision_adapter=False, use_shared_adapters=False,
                             freeze_clip=False, device=dev, precision="fp32", fast_init=True)
        cfg = m.config
        b = {k: torch.from_numpy(v).to(dev) for k, v in synth.synthetic_batch(cfg, B, seed=1234).items()}
        out = m(**b, return_loss=True)
        res = {"clipmi32": (out["loss"].item(), out["logits_per_text"].float())}
        params = {n[5:]: p.detach().float().clone() for n, p in m.named_parameters()}
        del m, out
        torch.cuda.empty_cache()
    else:
        cfg = C.resolve(PRESET)
        b = {k: torch.from_numpy(v) for k, v in synth.synthetic_batch(cfg, B, seed=1234).items()}
        params, res = R.to_torch(synth.clip_state_dict(cfg, seed=0)), {}
    torch.backends.cuda.matmul.allow_tf32 = False
    with torch.device(dev):
        o = R.clip_with_adapters_forward(b, params, cfg)
    res["fp32"] = (o["loss"].item(), o["logits_per_text"].float())
    for name, e in (("x3", X3()), ("x3s", X3(store=True)), ("x3sa", X3(store=True, attn=True))):
        with torch.device(dev):
            o = e.forward(b, params, cfg)
        res[name] = (o["loss"].item(), o["logits_per_text"].float())
        if dev == 'cuda':
            torch.cuda.empty_cache()
l0, z0 = res["fp32"]
for k, (l, z) in res.items():
    d = (z - z0).abs()
    print(f"{k:8s} |dloss| {abs(l - l0):.3e}  max|dlogit| {d.max().item():.3e}  rms {d.pow(2).mean().sqrt().item():.3e}",
          flush=True)

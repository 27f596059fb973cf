"""Where does clipmi bf16's logit error at config 3 come from?  (GPU diagnostic, forward only.)

Config 3's weights and batch (ViT-B/16, B = 1024, the test's fast_init weights and seed) through:
  fp32      the oracle (oracle/clip_ref.py) in fp32                       -- the reference
  amp       the same under torch.autocast(bf16) (PyTorch mixed precision: bf16 GEMMs with fp32
            accumulation, fp32 LayerNorm / softmax / loss, fp32 residual stream)
  emu       a restatement of clipmi's bf16 mode: GEMM operands bf16, fp32 accumulation, every stored
            activation rounded to bf16 (LN outputs, qkv, attention O, fc1 activation, the residual
            stream x / h), fp32 scores and softmax, P rounded to bf16 for PV, fp32 projections
  emu_r32   emu with the residual stream (x, h) kept in fp32
  emu_p32   emu with the residual stream in fp32 and the attention output / fc1 activation too
  clipmi    the library's bf16 mode itself
Prints max |dlogit| and |dloss| of each against fp32."""
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


class Emu:
    def __init__(self, resid32=False, act32=False):
        self.resid32, self.act32 = resid32, act32

    def lin(self, x, w, b=None, out_round=True):
        y = rb(x) @ rb(w).t()
        if b is not None:
            y = y + rb(b)
        return rb(y) if out_round else y

    def res(self, x):
        return x if self.resid32 else rb(x)

    def ln(self, x, w, b, eps):
        return rb(F.layer_norm(x, (x.shape[-1],), rb(w), rb(b), eps))

    def attention(self, x, p, pre, heads, mask):
        Bq, N, D = x.shape
        hd = D // heads
        q = self.lin(x, p[f"{pre}.q_proj.weight"], p[f"{pre}.q_proj.bias"])
        k = self.lin(x, p[f"{pre}.k_proj.weight"], p[f"{pre}.k_proj.bias"])
        v = self.lin(x, p[f"{pre}.v_proj.weight"], p[f"{pre}.v_proj.bias"])
        q, k, v = (t.view(Bq, N, heads, hd).transpose(1, 2) for t in (q, k, v))
        s = (q @ k.transpose(-1, -2)) * hd ** -0.5
        if mask is not None:
            s = s + mask
        pr = torch.softmax(s, dim=-1)
        o = (rb(pr) @ v).transpose(1, 2).reshape(Bq, N, D)
        o = o if self.act32 else rb(o)
        return o

    def layer(self, x, p, pre, heads, eps, mask):
        h = self.ln(x, p[f"{pre}.layer_norm1.weight"], p[f"{pre}.layer_norm1.bias"], eps)
        o = self.attention(h, p, f"{pre}.self_attn", heads, mask)
        x = self.res(x + self.lin(o, p[f"{pre}.self_attn.out_proj.weight"], p[f"{pre}.self_attn.out_proj.bias"],
                                  out_round=False))
        h = self.ln(x, p[f"{pre}.layer_norm2.weight"], p[f"{pre}.layer_norm2.bias"], eps)
        a = self.lin(h, p[f"{pre}.mlp.fc1.weight"], p[f"{pre}.mlp.fc1.bias"], out_round=False)
        a = R.quick_gelu(a)
        a = a if self.act32 else rb(a)
        return self.res(x + self.lin(a, p[f"{pre}.mlp.fc2.weight"], p[f"{pre}.mlp.fc2.bias"], out_round=False))

    def forward(self, b, p, cfg):
        t = cfg.text_config
        x = self.res(p["text_model.embeddings.token_embedding.weight"][b["input_ids"]] +
                     p["text_model.embeddings.position_embedding.weight"][: b["input_ids"].shape[1]])
        mask = R.causal_padding_mask(b["attention_mask"], torch.float32)
        for i in range(t.num_hidden_layers):
            x = self.layer(x, p, f"text_model.encoder.layers.{i}", t.num_attention_heads, t.layer_norm_eps, mask)
        x = self.ln(x, p["text_model.final_layer_norm.weight"], p["text_model.final_layer_norm.bias"], t.layer_norm_eps)
        tf = rb(x[:, 0, :]) @ rb(p["text_projection.weight"]).t()
        v = cfg.vision_config
        pv = b["pixel_values"]
        w = p["vision_model.embeddings.patch_embedding.weight"]
        xe = F.conv2d(rb(pv), rb(w), stride=v.patch_size).flatten(2).transpose(1, 2)
        xe = torch.cat([p["vision_model.embeddings.class_embedding"].expand(pv.shape[0], 1, -1), rb(xe)], dim=1)
        xe = xe + p["vision_model.embeddings.position_embedding.weight"][None]
        x = self.ln(xe, p["vision_model.pre_layrnorm.weight"], p["vision_model.pre_layrnorm.bias"], v.layer_norm_eps)
        for i in range(v.num_hidden_layers):
            x = self.layer(x, p, f"vision_model.encoder.layers.{i}", v.num_attention_heads, v.layer_norm_eps, None)
        imf = rb(x[:, 0, :]) @ rb(p["visual_projection.weight"]).t()
        return R.contrastive(tf, imf, p["logit_scale"])


from clipmi import config as C  # noqa: E402
with torch.no_grad():
    if dev == "cuda":
        m = CLIPWithAdapters(PRESET, use_text_adapter=False, use_vision_adapter=False, use_shared_adapters=False,
                             freeze_clip=False, device=dev, precision="bf16", fast_init=True)
        cfg = m.config
        b = {k: torch.from_numpy(v).to(dev) for k, v in synth.synthetic_batch(cfg, B, seed=1234).items()}
        out = m(**b, return_loss=True)
        res = {"clipmi": (out["loss"].item(), out["logits_per_text"].float())}
        params = {n[5:]: p.detach().float().clone() for n, p in m.named_parameters()}
        del m, out
        torch.cuda.empty_cache()
    else:
        cfg = C.resolve(PRESET)
        b = {k: torch.from_numpy(v) for k, v in synth.synthetic_batch(cfg, B, seed=1234).items()}
        params, res = R.to_torch(synth.clip_state_dict(cfg, seed=0)), {}
    with torch.device(dev):
        o = R.clip_with_adapters_forward(b, params, cfg)
    res["fp32"] = (o["loss"].item(), o["logits_per_text"].float())
    with torch.device(dev), torch.autocast("cuda", dtype=torch.bfloat16):
        o = R.clip_with_adapters_forward(b, params, cfg)
    res["amp"] = (o["loss"].item(), o["logits_per_text"].float())
    for name, e in (("emu", Emu()), ("emu_r32", Emu(resid32=True)), ("emu_p32", Emu(resid32=True, act32=True))):
        with torch.device(dev):
            o = e.forward(b, params, cfg)
        res[name] = (o["loss"].item(), o["logits_per_text"].float())
l0, z0 = res["fp32"]
for k, (l, z) in res.items():
    d = (z - z0).abs()
    print(f"{k:8s} |dloss| {abs(l - l0):.3e}  max|dlogit| {d.max().item():.4f}  rms {d.pow(2).mean().sqrt().item():.4f}",
          flush=True)

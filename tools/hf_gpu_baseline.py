"""The reference's own framework on the same GPU: Hugging Face transformers' CLIPModel (what model_m.py wraps,
model_m.py:29) running config 3's step -- ViT-B/16 full fine-tune, B = 1024, first-token text pooling and CLS image
pooling without post-LN (model_m.py:77-125, quirks Q1/Q2), the symmetric InfoNCE of model_m.py:146-163, backward,
clip_grad_norm_(1.0) and AdamW (trainer.py:91-99) -- timed in fp32 (the reference's arithmetic) and under
torch.autocast(bfloat16) (PyTorch's mixed precision).  Random-init weights (no checkpoints offline), the synthetic
batch of bench.py.  A point of comparison for bench.py's headline (bf16) and parity_mode (bf16x3, fp32-accurate)
numbers; it does not use the oracle or libclipmi.

    python tools/hf_gpu_baseline.py [--batch 1024] [--steps 5] [--warmup 2] [--precision fp32|amp|both]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vlm-clip_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--precision", default="both", choices=["fp32", "amp", "both"])
    ap.add_argument("--attn", default="sdpa", choices=["sdpa", "eager"])
    args = ap.parse_args()
    from transformers import CLIPConfig, CLIPModel
    from clipmi import config as C
    import bench
    cfg = C.resolve("B/16")
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    hc = CLIPConfig(**cfg.to_hf_dict())
    hc._attn_implementation = args.attn
    for sub in (hc.text_config, hc.vision_config):
        sub._attn_implementation = args.attn
    model = CLIPModel(hc).to(dev).train()
    with torch.no_grad():
        model.logit_scale.fill_(C.LN100)
    opt = torch.optim.AdamW(model.parameters(), lr=5e-5, weight_decay=0.01)
    batch = bench.synthetic_batch(cfg, args.batch, 0, dev)
    lab = torch.arange(args.batch, device=dev)

    def step(amp):
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
            t = model.text_model(input_ids=batch["input_ids"], attention_mask=batch["attention_mask"]).last_hidden_state
            t = model.text_projection(t[:, 0, :])                                      # model_m.py:102-103
            v = model.vision_model(pixel_values=batch["pixel_values"]).last_hidden_state
            v = model.visual_projection(v[:, 0, :])                                    # model_m.py:122-123
            t = t / t.norm(dim=-1, keepdim=True)
            v = v / v.norm(dim=-1, keepdim=True)
            lpt = model.logit_scale.exp() * t @ v.t()                                  # model_m.py:152-155
            loss = (F.cross_entropy(lpt, lab) + F.cross_entropy(lpt.t(), lab)) / 2     # model_m.py:159-163
        opt.zero_grad()
        loss.backward()
        torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
        opt.step()
        return loss

    out = {"workload": "HF transformers CLIPModel ViT-B/16, config 3's step (full fine-tune, B=%d)" % args.batch,
           "torch": torch.__version__, "attn_implementation": args.attn}
    for name, amp in (("fp32", False), ("amp_bf16", True)):
        if args.precision != "both" and name[:3] != args.precision[:3]:
            continue
        for _ in range(args.warmup):
            step(amp)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            loss = step(amp)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        out[name] = {"pairs_per_s": round(args.batch * args.steps / el, 1), "ms_per_step": round(el / args.steps * 1e3, 1),
                     "loss": round(float(loss.item()), 4), "steps": args.steps,
                     "peak_mem_gib": round(torch.cuda.max_memory_allocated(dev) / 2 ** 30, 1)}
        print(f"[hf baseline] {name}: {out[name]}", file=sys.stderr, flush=True)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

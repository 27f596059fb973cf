#!/usr/bin/env python3
"""Benchmark: image-text pairs/s of the ViT-B/16 contrastive training step (BASELINE.json
config 3: full fine-tune, adapters off, B=1024 per GPU, bf16 MFMA path), weak-scaled over
N GPUs (one process per GPU, RCCL).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

A step = forward of both towers + symmetric InfoNCE (all-gathered over ranks) + backward
through everything + data-parallel gradient all-reduce + global-norm clip + AdamW, i.e.
trainer.py:81-99 with all CLIP parameters (and logit_scale) trainable.  Inputs are
synthetic (CLIP-normalised U[0,1) pixels, BOS/ids/EOS captions padded with EOS) generated
once on the device; weights are random-init ViT-B/16 (no checkpoints offline).

Rank 0 prints ONE JSON line.  `roofline` is measured live: the dominant kernel's launches
inside the timed steps are bracketed by HIP events on their stream (clipmi_prof_*), and
achieved = its algorithmic FLOPs per launch / average launch duration.  `cpu_baseline` is
the CPU oracle (oracle/clip_ref.py, a restatement of the reference path) timed on this
host's cores on a bounded sample.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import math
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "vlm-clip_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from clipmi import config as C  # noqa: E402

METRIC = "image-text pairs/sec, ViT-B/16 contrastive step, 1/2/4/8 GPUs; MFMA % peak"
PEAK_BF16_TFLOPS = 2516.6  # 256 CU x 2.4 GHz x 4096 FLOP/CU/clk (dense bf16, MI355X_MICROARCH.md)


def log(msg):
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=1024, help="pairs per GPU")
    ap.add_argument("--model", default="B/16")
    ap.add_argument("--mode", default="full", choices=["full", "adapter"])
    ap.add_argument("--roofline-kernel", default=None,
                    help="kernel family timed live (default: gemm256_wgrad_splitk for --mode full, "
                         "gemm256_fwd_bias_qgelu = the frozen vision tower's fc1 for --mode adapter)")
    ap.add_argument("--cpu-sample", type=int, default=8, help="pairs per CPU-baseline step (0 = skip)")
    ap.add_argument("--cpu-steps", type=int, default=3)
    return ap.parse_args()


def synthetic_batch(cfg, B, rank, device, seed=1234):
    """SURVEY §8d synthetic batch, generated on the device (rank-dependent shard)."""
    v, t = cfg.vision_config, cfg.text_config
    g = torch.Generator(device=device).manual_seed(seed * 1000 + rank)
    mean = torch.tensor([0.48145466, 0.4578275, 0.40821073], device=device).view(1, 3, 1, 1)
    std = torch.tensor([0.26862954, 0.26130258, 0.27577711], device=device).view(1, 3, 1, 1)
    px = (torch.rand(B, 3, v.image_size, v.image_size, generator=g, device=device) - mean) / std
    S = t.max_position_embeddings
    L = torch.randint(5, S + 1, (B, 1), generator=g, device=device)
    pos = torch.arange(S, device=device).view(1, S)
    body = torch.randint(0, t.eos_token_id - 1, (B, S), generator=g, device=device)
    ids = torch.where(pos < L - 1, body, torch.full_like(body, t.eos_token_id))
    ids[:, 0] = t.bos_token_id
    mask = (pos < L).to(torch.int64)
    return {"input_ids": ids, "attention_mask": mask, "pixel_values": px.contiguous()}


def wgrad_algorithmic_bytes(cfg, B):
    """Mean compulsory HBM bytes of one gemm256_wgrad_splitk launch the live roofline times:
    both bf16 operands read once (tokens x (M + N) x 2 B) + the fp32 gradient written once
    (M x N x 4 B), over the vision tower's 49 wgrad launches per step (4 per encoder layer +
    the patch embedding; the text tower's run on the second stream and are not timed)."""
    v = cfg.vision_config
    shapes = []
    for tc, R in ((v, B * ((v.image_size // v.patch_size) ** 2 + 1)),):
        D, F = tc.hidden_size, tc.intermediate_size
        shapes += [(R, D, F), (R, F, D), (R, D, D), (R, 3 * D, D)] * tc.num_hidden_layers
    shapes.append((B * ((v.image_size // v.patch_size) ** 2 + 1), v.hidden_size, 3 * v.patch_size ** 2))
    tot = sum(R * (M + N) * 2 + M * N * 4 for R, M, N in shapes)
    return round(tot / len(shapes))


def fc1_algorithmic_bytes(cfg, B):
    """Compulsory HBM bytes of one frozen-tower vision fc1 launch (gemm256_fwd_bias_qgelu, the
    adapter-mode roofline kernel): LN'd activations [R, D] and weight [F, D] read once, the
    activated [R, F] output written once, bf16, plus the bias."""
    v = cfg.vision_config
    R, D, F = B * ((v.image_size // v.patch_size) ** 2 + 1), v.hidden_size, v.intermediate_size
    return 2 * (R * D + F * D + R * F + F)


def cpu_baseline(cfg, B, steps):
    """Oracle (oracle/clip_ref.py) full fine-tune step on the host: fwd + bwd + AdamW."""
    from clipmi import synth
    from oracle import clip_ref as R
    # the GPU box exposes every host CPU in the affinity mask but grants a share of them
    # (OMP_NUM_THREADS is set to that share there); never oversubscribe it
    threads = len(os.sched_getaffinity(0))
    if os.environ.get("OMP_NUM_THREADS", "").isdigit():
        threads = min(threads, int(os.environ["OMP_NUM_THREADS"]))
    torch.set_num_threads(threads)
    gen = torch.Generator().manual_seed(0)
    p = {}
    for name, shape, std, mean in synth.clip_param_specs(cfg):
        p[name] = (torch.randn(*shape, generator=gen) * std + mean).requires_grad_(True)
    p["logit_scale"] = torch.tensor(C.LN100, requires_grad=True)
    b = {k: torch.from_numpy(x) for k, x in synth.synthetic_batch(cfg, B, seed=1234).items()}
    params = list(p.values())
    m = [torch.zeros_like(x) for x in params]
    v = [torch.zeros_like(x) for x in params]
    times = []
    for it in range(steps + 1):
        t0 = time.perf_counter()
        for x in params:
            x.grad = None
        out = R.clip_with_adapters_forward(b, p, cfg)
        out["loss"].backward()
        with torch.no_grad():
            grads = [x.grad if x.grad is not None else torch.zeros_like(x) for x in params]  # post-LN unused (Q2)
            gn = torch.sqrt(sum((g.double() ** 2).sum() for g in grads))
            coef = min(1.0, 1.0 / (gn.item() + 1e-6))
            upd = R.adamw_reference(params, [g * coef for g in grads], m, v, it + 1, 5e-5)
            for x, (np_, nm, nv), i in zip(params, upd, range(len(params))):
                x.copy_(np_)
                m[i], v[i] = nm, nv
        if it > 0:
            times.append(time.perf_counter() - t0)
        log(f"cpu baseline step {it}: {time.perf_counter() - t0:.2f} s")
    times.sort()
    med = times[len(times) // 2]
    return {"value": round(B / med, 3), "unit": "pairs/s", "cores": threads, "kind": "port",
            "sample": f"oracle/clip_ref.py {cfg.name} full fine-tune step (fwd+bwd+AdamW) fp32, B={B}, "
                      f"median of {steps} steps after 1 warm-up, torch CPU threads={threads}"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"[bench] note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE", file=sys.stderr)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    group = None
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=dev)
        group = dist.group.WORLD

    from clipmi import CLIPWithAdapters
    from clipmi import _lib
    from clipmi.trainer import FusedAdamW, linear_schedule_with_warmup

    cfg = C.resolve(args.model)
    adapters = args.mode == "adapter"
    if args.roofline_kernel is None:
        args.roofline_kernel = "gemm256_fwd_bias_qgelu" if adapters else "gemm256_wgrad_splitk"
    model = CLIPWithAdapters(args.model, use_text_adapter=adapters, use_vision_adapter=adapters,
                             use_shared_adapters=False, freeze_clip=adapters, device=dev, precision="bf16",
                             fast_init=True, process_group=group)
    params = [p for n, p in model.named_parameters() if p.requires_grad]
    opt = FusedAdamW(params, lr=5e-5, weight_decay=0.01, arenas=model.arenas())
    batch = synthetic_batch(cfg, args.batch, rank, dev)
    total = args.warmup + args.steps

    def step(i):
        out = model(**batch)
        loss = out["loss"]
        opt.zero_grad()
        loss.backward()
        if world > 1:
            opt.grads_all_reduce(group)
        opt.clip_grad_norm(1.0)
        opt.step(lr=5e-5 * linear_schedule_with_warmup(i, 0, total))
        return loss

    for i in range(args.warmup):
        t_w = time.perf_counter()
        step(i)
        torch.cuda.synchronize()
        ms_ = torch.cuda.memory_stats(dev)
        log(f"warmup step {i} done in {time.perf_counter() - t_w:.3f} s (allocator retries "
            f"{ms_.get('num_alloc_retries')}, device mallocs {ms_.get('num_device_alloc')})")
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    L = _lib.lib()
    L.clipmi_prof_arm.argtypes = [ctypes.c_char_p, ctypes.c_int]
    L.clipmi_prof_read.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_double)]
    cap = 4096
    _lib.check(L.clipmi_prof_arm(args.roofline_kernel.encode(), cap), "prof_arm")
    # only the caller's stream: the text tower's launches run on a second stream beside the
    # vision tower's kernels (model.py), so their event spans include the other tower's work
    L.clipmi_prof_stream.argtypes = [ctypes.c_void_p]
    _lib.check(L.clipmi_prof_stream(ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)), "prof_stream")
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    t0 = time.perf_counter()
    evs[0].record()
    for i in range(args.warmup, total):
        loss = step(i)
        evs[i - args.warmup + 1].record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    log(f"timed {args.steps} steps: {elapsed:.3f} s; per-step GPU ms: "
        + " ".join(f"{evs[k].elapsed_time(evs[k + 1]):.1f}" for k in range(args.steps)))
    ms_ = torch.cuda.memory_stats(dev)
    log(f"allocator: retries {ms_.get('num_alloc_retries')} device-mallocs {ms_.get('num_device_alloc')} "
        f"frees {ms_.get('num_device_free')} reserved peak {ms_.get('reserved_bytes.all.peak', 0) / 2**30:.1f} GiB "
        f"allocated peak {ms_.get('allocated_bytes.all.peak', 0) / 2**30:.1f} GiB")
    L.clipmi_prof_disarm()
    ms = (ctypes.c_float * cap)()
    fl = (ctypes.c_double * cap)()
    n = L.clipmi_prof_read(cap, ms, fl)
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    pairs = args.batch * world * args.steps
    value = pairs / elapsed
    fwd = C.forward_flops_per_pair(cfg)
    step_flops_pair = 3 * fwd if not adapters else fwd
    roof = None
    traffic, traffic_src = None, None
    # HBM bytes per launch of the same kernel family from the committed PMC passes
    # (tools/traffic_pmc.sh -> profiles/*_traffic.json; newest file wins)
    import glob
    tfiles = sorted(glob.glob(os.path.join(REPO, "profiles", "*_traffic.json")), key=os.path.getmtime)
    for tf in reversed(tfiles):
        try:
            tj = json.load(open(tf))
        except (OSError, ValueError):
            continue
        if tj.get("kernel") == args.roofline_kernel:
            traffic, traffic_src = tj["bytes_per_launch"], os.path.relpath(tf, REPO)
            break
    if n > 0:
        avg_ms = sum(ms[i] for i in range(n)) / n
        avg_fl = sum(fl[i] for i in range(n)) / n
        ach = avg_fl / (avg_ms * 1e-3) / 1e12
        roof = {"bound": "mfma", "kernel": args.roofline_kernel, "launches": n,
                "avg_launch_ms": round(avg_ms, 4), "flops_per_launch": avg_fl,
                "achieved": round(ach, 1), "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
                "frac": round(ach / PEAK_BF16_TFLOPS, 4), "traffic": traffic,
                "traffic_unit": "bytes/launch (HBM, PMC)", "traffic_source": traffic_src,
                "algorithmic_bytes": (fc1_algorithmic_bytes(cfg, args.batch) if adapters
                                      else wgrad_algorithmic_bytes(cfg, args.batch))}
    result = {
        "metric": METRIC, "value": round(value, 2), "unit": "pairs/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 2),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
        "data": f"synthetic: CLIP-normalised U[0,1) {cfg.vision_config.image_size}px pixels + BOS/random-id/EOS captions (77 tok, EOS pad), "
                "random-init weights",
        "config": {"workload": f"{cfg.name} {'full fine-tune (adapters off)' if not adapters else 'adapter fine-tune'}"
                               f" contrastive step: fwd+bwd+all-reduce+clip+AdamW",
                   "per_gpu_batch": args.batch, "global_batch": args.batch * world,
                   "image_size": cfg.vision_config.image_size,
                   "text_len": 77, "parallelism": f"dp{world}"},
        "mfma_frac_step": round(value * step_flops_pair / (world * PEAK_BF16_TFLOPS * 1e12), 4),
        "step_tflops_per_gpu": round(value * step_flops_pair / world / 1e12, 1),
        "loss": round(float(loss.item()), 4),
        "roofline": roof,
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and args.cpu_sample > 0:
        result["cpu_baseline"] = cpu_baseline(cfg, args.cpu_sample, args.cpu_steps)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

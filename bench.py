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
PEAK_FP8_TFLOPS = 5033.2   # block-scaled f8f6f4 MFMA: 2x the bf16 rate (dense)
PEAK_FP32_TFLOPS = 157.3   # f32 MFMA (= the f32 vector rate, 1/16 of bf16; MI355X_MICROARCH.md)
PEAK_HBM_GBS = 8000.0      # HBM3E peak (MI355X_MICROARCH.md: 8 TB/s spec, ~6.3 achievable)


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
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp8", "fp32", "bf16x3"],
                    help="fp8: the frozen towers' GEMMs in MXFP8 (BASELINE config 5; needs --mode adapter); "
                         "fp32: the parity mode (f32 operands end to end), priced against the f32 MFMA peak")
    ap.add_argument("--roofline-family", default=None, choices=list(FAMILIES) + list(FAMILIES_FP32),
                    help="family reported as `roofline` (default: the one with the most measured time)")
    ap.add_argument("--cpu-sample", type=int, default=32,
                    help="pairs per CPU-baseline step (SURVEY 8d: B = 32; 0 = skip)")
    ap.add_argument("--cpu-steps", type=int, default=3)
    ap.add_argument("--comm", default="torch", choices=["torch", "clipmi"],
                    help="N > 1: the data-parallel exchanges through torch.distributed's RCCL (default) or RCCL issued "
                         "by libclipmi (clipmi.comm.Communicator bootstrapped over the same store)")
    ap.add_argument("--grad-bucket-dtype", default="fp32", choices=["fp32", "bf16"],
                    help="N > 1: dtype the gradient buckets are all-reduced in (bf16: half the bytes per ring)")
    ap.add_argument("--parity-steps", type=int, default=5,
                    help="N=1, bf16 full fine-tune: also time this many steps of the bf16x3 mode (the mode that meets "
                         "north_star's 1e-3 logits) in the same run, reported under `parity_mode` (0 = skip)")
    ap.add_argument("--parity-warmup", type=int, default=2)
    ap.add_argument("--launch-check", action="store_true",
                    help="test hook: each rank prints its rank/world and exits before touching the GPU")
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


# Kernel families timed live (labels returned by libclipmi's dispatch, csrc/gemm.hip, attention.hip)
FAMILIES = {
    "gemm256_fwd_dgrad": ["gemm256_fwd_bias", "gemm256_fwd_bias_resid", "gemm256_fwd_bias_qgelu_pre",
                          "gemm256_fwd_bias_qgelu_dact", "gemm256_fwd_bias_qgelu", "gemm256_fwd", "gemm256_dgrad",
                          "gemm256_dgrad_dqgelu", "gemm256_dgrad_mulaux",
                          # fp32 residual stream: out-projection / fc2 write the fp32 sum (round 5)
                          "gemm256_fwd_bias_resid_f32", "gemm256_fwd_bias_f32", "gemm256_fwd_f32",
                          # --precision bf16x3: the split products' fp32-output instances
                          "gemm256_fwd_bias_qgelu_dact_f32", "gemm256_fwd_bias_qgelu_f32", "gemm256_dgrad_f32",
                          "gemm256_dgrad_mulaux_f32"],
    "gemm256_wgrad": ["gemm256_wgrad_splitk", "gemm256_wgrad"],
    "attention": ["attn_fwd", "attn_bwd"],
    "gemm_fp8": ["gemm_fp8_fwd_bias", "gemm_fp8_fwd_bias_resid", "gemm_fp8_fwd_bias_qgelu",
                 "gemm_fp8_fwd_bias_qgelu_q8", "gemm_fp8", "gemm_fp8_generic"],
}
FAMILIES_FP32 = {"gemm_f32": ["gemm_f32"]}  # --precision fp32: every GEMM is the f32 kernel
PEAKS = {"gemm_fp8": PEAK_FP8_TFLOPS, "gemm_f32": PEAK_FP32_TFLOPS}
# HBM traffic per launch of each family, from rocprofv3 --pmc passes (tools/traffic_pmc.sh); named
# explicitly so the file read is the one committed for this build, not the newest on disk
TRAFFIC_FILES = {"gemm256_fwd_dgrad": "profiles/r06_traffic_fwd_dgrad.json",
                 "gemm256_wgrad": "profiles/r06_traffic_wgrad.json",
                 "attention": "profiles/r05_traffic_attention.json"}


def vision_gemm_shapes(cfg, B, train, resid32=False):
    """(M, N, K, extra_bytes) of the vision tower's 256-kernel launches on the caller's stream,
    per step, in the families above; extra = epilogue operands/outputs beyond A, B and C once
    (counted at 2 bytes per element).  resid32: the bf16 mode's fp32 residual stream (round 5) --
    the patch embedding, out-projection and fc2 write fp32 (+2 B per output element) and the
    latter two read the fp32 residual (4 B per element)."""
    v = cfg.vision_config
    R = B * ((v.image_size // v.patch_size) ** 2 + 1)
    D, F = v.hidden_size, v.intermediate_size
    Kp = 3 * v.patch_size ** 2
    Kp = (Kp + 63) // 64 * 64 if Kp % 8 else Kp
    rx = R * D * 6 if resid32 else R * D * 2  # residual read (+ the wider sum written)
    fwd = [(R, D, Kp, R * D * 2 if resid32 else 0)]
    for _ in range(v.num_hidden_layers):
        fwd += [(R, 3 * D, D, 0), (R, D, D, rx), (R, F, D, R * F * 2 if train else 0), (R, D, F, rx)]
    dgrad, wgrad = [], []
    if train:
        for _ in range(v.num_hidden_layers):
            dgrad += [(R, F, D, R * F * 2), (R, D, F, 0), (R, D, D, 0), (R, D, 3 * D, 0)]
            wgrad += [(D, F, R), (F, D, R), (D, D, R), (3 * D, D, R)]
        wgrad.append((D, Kp, R))
    return fwd + dgrad, wgrad


def algorithmic_bytes(cfg, B, train, resid32=False):
    """Mean compulsory HBM bytes per launch of each GEMM family (bf16 operands read once, output
    written once: bf16 for forward/dgrad, fp32 gradient for wgrad), vision tower launches."""
    fd, wg = vision_gemm_shapes(cfg, B, train, resid32)
    out = {"gemm256_fwd_dgrad": sum((M * K + N * K + M * N) * 2 + x for M, N, K, x in fd) / len(fd)}
    if wg:
        out["gemm256_wgrad"] = sum(K * (M + N) * 2 + M * N * 4 for M, N, K in wg) / len(wg)
    # attention (vision tower, one launch per layer and direction): forward reads Q, K, V and writes O
    # (+ the fp32 row LSE); backward reads Q, K, V, O, dO and the LSE and writes dQ, dK, dV
    v = cfg.vision_config
    N = (v.image_size // v.patch_size) ** 2 + 1
    T, D, H = B * N, v.hidden_size, v.num_attention_heads
    fwd = T * 4 * D * 2 + B * H * N * 4
    bwd = T * 8 * D * 2 + B * H * N * 4
    out["attention"] = (fwd + bwd) / 2 if train else fwd
    return {k: round(v) for k, v in out.items()}


def _cpu_model():
    """The host CPU's model string (/proc/cpuinfo), for the cpu_baseline record."""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline_adapter(cfg, B, steps, threads):
    """Oracle adapter fine-tune step (frozen towers, configs 2/4/5) on the host: the towers' forward,
    the adapters on the pooled rows (model_m.py:77-125), the contrastive loss and its backward into
    the adapters (AdamW over ~1 M adapter parameters is negligible and left out)."""
    from clipmi import synth
    from oracle import clip_ref as R
    torch.set_num_threads(threads)
    p = {name: torch.randn(*shape) * std + mean for name, shape, std, mean in synth.clip_param_specs(cfg)}
    p["logit_scale"] = torch.tensor(C.LN100)
    t, v = cfg.text_config, cfg.vision_config
    ta = R.to_torch(synth.adapter_state_dict(t.hidden_size, 256, 0, "text_adapter"), requires_grad=True)
    va = R.to_torch(synth.adapter_state_dict(v.hidden_size, 256, 0, "vision_adapter"), requires_grad=True)
    b = {k: torch.from_numpy(x) for k, x in synth.synthetic_batch(cfg, B, seed=1234).items()}
    times = []
    for it in range(steps + 1):
        t0 = time.perf_counter()
        with torch.no_grad():
            ht = R.text_tower(b["input_ids"], b["attention_mask"], p, cfg)[:, :1]
            hv = R.vision_tower(b["pixel_values"], p, cfg)[:, :1]
        tf = R.linear(R.adapter(ht, ta)[:, 0], p["text_projection.weight"])
        imf = R.linear(R.adapter(hv, va)[:, 0], p["visual_projection.weight"])
        R.contrastive(tf, imf, p["logit_scale"])["loss"].backward()
        if it > 0:
            times.append(time.perf_counter() - t0)
        log(f"cpu baseline step {it}: {time.perf_counter() - t0:.2f} s")
    times.sort()
    med = times[len(times) // 2]
    return {"value": round(B / med, 3), "unit": "pairs/s", "cores": threads, "kind": "port", "cpu": _cpu_model(),
            "sample": f"oracle/clip_ref.py {cfg.name} adapter fine-tune step (frozen towers fwd + adapters fwd/bwd + "
                      f"InfoNCE) fp32, B={B}, median of {steps} steps after 1 warm-up, torch CPU threads={threads}"}


def cpu_baseline(cfg, B, steps, adapters=False):
    """Oracle (oracle/clip_ref.py) full fine-tune step on the host: fwd + bwd + AdamW."""
    from clipmi import synth
    from oracle import clip_ref as R
    # the GPU box exposes every host CPU in the affinity mask but grants a share of them
    # (OMP_NUM_THREADS is set to that share there); never oversubscribe it
    threads = len(os.sched_getaffinity(0))
    if os.environ.get("OMP_NUM_THREADS", "").isdigit():
        threads = min(threads, int(os.environ["OMP_NUM_THREADS"]))
    if adapters:
        return cpu_baseline_adapter(cfg, B, steps, threads)
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
    return {"value": round(B / med, 3), "unit": "pairs/s", "cores": threads, "kind": "port", "cpu": _cpu_model(),
            "sample": f"oracle/clip_ref.py {cfg.name} full fine-tune step (fwd+bwd+AdamW) fp32, B={B}, "
                      f"median of {steps} steps after 1 warm-up, torch CPU threads={threads}"}


def self_launch(args):
    """`--gpus N` without a torch.distributed environment: start N ranks (one per GPU) through
    torch.distributed.run from this process, which has not touched the GPU, and exit with its
    code.  Rank 0 prints the JSON line."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    log(f"launching {args.gpus} ranks: {' '.join(cmd[1:])}")
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.run(cmd, env=env).returncode


def family_roofline(name, launches, cfg, B, train, resid32=False, x3=False):
    """launches: [(ms, flops)] of one family on the caller's stream inside the timed steps."""
    if not launches:
        return None
    tot_ms = sum(m for m, _ in launches)
    tot_fl = sum(f for _, f in launches)
    ach = tot_fl / (tot_ms * 1e-3) / 1e12
    peak = PEAKS.get(name, PEAK_BF16_TFLOPS)
    # bf16x3: the launches are the split products (3K bf16 reduction, fp32 C); their flops are the MFMA
    # work issued (3x the fp32 product's) and the bf16-operand byte model does not apply
    alg = None if x3 else algorithmic_bytes(cfg, B, train, resid32).get(name)
    res = {"bound": "mfma", "kernel": name, "labels": {**FAMILIES, **FAMILIES_FP32}[name], "launches": len(launches),
           "avg_launch_ms": round(tot_ms / len(launches), 4), "flops_per_launch": tot_fl / len(launches),
           "achieved": round(ach, 1), "peak": peak, "unit": "TFLOP/s",
           "frac": round(ach / peak, 4), "ms_per_step_caller_stream": None,
           "traffic": None, "traffic_unit": "bytes/launch (HBM, PMC)", "traffic_source": None,
           "algorithmic_bytes": alg}
    if name == "attention" and alg:
        # at CLIP's sequence lengths attention moves more bytes per FLOP than the chip's balance
        # point (per token and head 4*N*64 FLOP against 4*64*2 B of Q, K, V, O: N/2 FLOP/B, 99 at
        # N = 197, 289 at N = 577, vs 2.5 PF / 8 TB/s = 315), so its roofline is HBM: algorithmic
        # bytes / mean launch time
        gbs = alg / (tot_ms / len(launches) * 1e-3) / 1e9
        res.update({"bound": "hbm", "achieved": round(gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                    "frac": round(gbs / PEAK_HBM_GBS, 4), "mfma_tflops": round(ach, 1),
                    "mfma_frac": round(ach / PEAK_BF16_TFLOPS, 4)})
    tf = TRAFFIC_FILES.get(name)
    if tf and os.path.isfile(os.path.join(REPO, tf)):
        try:
            tj = json.load(open(os.path.join(REPO, tf)))
            if tj.get("kernel") == name and tj.get("workload") == f"{cfg.name}/{B}/{int(train)}":
                res["traffic"], res["traffic_source"] = tj["bytes_per_launch"], tf
        except (OSError, ValueError, KeyError):
            pass
    return res


def parity_mode_run(args, cfg, dev, batch):
    """The bf16x3 mode (fp32 activations, every tower GEMM a bf16x3 split product: max |dlogit| 1.1e-4 against
    the fp32 reference at this config, profiles/r05_config3_full_size_parity.log; test bound 1e-3) timed on the
    same workload and batch as the headline, after it, with the same step (fwd + bwd + clip + AdamW)."""
    from clipmi import CLIPWithAdapters
    from clipmi.trainer import FusedAdamW, linear_schedule_with_warmup
    model = CLIPWithAdapters(args.model, use_text_adapter=False, use_vision_adapter=False, use_shared_adapters=False,
                             freeze_clip=False, device=dev, precision="bf16x3", fast_init=True)
    params = [p for n, p in model.named_parameters() if p.requires_grad]
    opt = FusedAdamW(params, lr=5e-5, weight_decay=0.01, arenas=model.arenas())
    total = args.parity_warmup + args.parity_steps

    def step(i):
        out = model(**batch)
        opt.zero_grad()
        opt.armed_backward(out["loss"])
        opt.clip_grad_norm(1.0)
        opt.step(lr=5e-5 * linear_schedule_with_warmup(i, 0, total))
        return out["loss"]

    for i in range(args.parity_warmup):
        step(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.parity_warmup, total):
        loss = step(i)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    value = args.batch * args.parity_steps / el
    step_flops_pair = 3 * C.forward_flops_per_pair(cfg)
    log(f"parity mode (bf16x3): {args.parity_steps} steps in {el:.3f} s = {value:.1f} pairs/s")
    res = {"precision": "bf16x3", "value": round(value, 2), "unit": "pairs/s",
           "ms_per_step": round(el / args.parity_steps * 1e3, 2), "steps": args.parity_steps,
           "warmup": args.parity_warmup, "loss": round(float(loss.item()), 4), "max_dlogit_bound": 1e-3,
           "dtype": "fp32 (tower GEMMs and attention products as bf16x3 split products, fp32 accumulation)",
           # three bf16 MFMA products per fp32 one: priced against a third of the bf16 peak
           "mfma_frac_step": round(value * step_flops_pair / (PEAK_BF16_TFLOPS / 3 * 1e12), 4)}
    del model, opt, params
    torch.cuda.empty_cache()
    return res


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(self_launch(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.launch_check:
        print(json.dumps({"rank": rank, "world": world}), flush=True)
        return
    if world != args.gpus and rank == 0:
        print(f"[bench] note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE", file=sys.stderr)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    group = None
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=dev)
        group = dist.group.WORLD
        if args.comm == "clipmi":
            from clipmi.comm import Communicator
            group = Communicator.from_process_group(dist.group.WORLD)

    from clipmi import CLIPWithAdapters
    from clipmi import _lib
    from clipmi.trainer import FusedAdamW, linear_schedule_with_warmup

    cfg = C.resolve(args.model)
    adapters = args.mode == "adapter"
    if args.precision == "fp8" and not adapters:
        raise SystemExit("--precision fp8 runs frozen towers: use --mode adapter")
    model = CLIPWithAdapters(args.model, use_text_adapter=adapters, use_vision_adapter=adapters,
                             use_shared_adapters=False, freeze_clip=adapters, device=dev, precision=args.precision,
                             fast_init=True, process_group=group)
    params = [p for n, p in model.named_parameters() if p.requires_grad]
    opt = FusedAdamW(params, lr=5e-5, weight_decay=0.01, arenas=model.arenas(), process_group=group,
                     grad_bucket_dtype=torch.bfloat16 if args.grad_bucket_dtype == "bf16" else torch.float32)
    opt.overlap_with(model)  # world > 1: gradient buckets all-reduced under the backward (armed_backward)
    batch = synthetic_batch(cfg, args.batch, rank, dev)
    total = args.warmup + args.steps

    def step(i):
        out = model(**batch)
        loss = out["loss"]
        opt.zero_grad()
        opt.armed_backward(loss)
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
    L.clipmi_prof_read_labels.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
    cap = 16384
    fams = FAMILIES_FP32 if args.precision == "fp32" else FAMILIES
    labels = [lab for fam in fams.values() for lab in fam]
    _lib.check(L.clipmi_prof_arm(",".join(labels).encode(), cap), "prof_arm")
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
    wh = (ctypes.c_int * cap)()
    n = L.clipmi_prof_read(cap, ms, fl)
    L.clipmi_prof_read_labels(cap, wh)
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    pairs = args.batch * world * args.steps
    value = pairs / elapsed
    fwd = C.forward_flops_per_pair(cfg)
    step_flops_pair = 3 * fwd if not adapters else fwd
    per_fam = {name: [] for name in fams}
    for i in range(n):
        lab = labels[wh[i]]
        for name, labs in fams.items():
            if lab in labs:
                per_fam[name].append((ms[i], fl[i]))
    roofs = {}
    for name in fams:
        r = family_roofline(name, per_fam[name], cfg, args.batch, not adapters,
                            resid32=bool(getattr(model._rt, "resid32", False)), x3=args.precision == "bf16x3")
        if r is not None:
            r["ms_per_step_caller_stream"] = round(sum(m for m, _ in per_fam[name]) / args.steps, 2)
            roofs[name] = r
    if args.roofline_family and args.roofline_family in roofs:
        main_fam = args.roofline_family
    else:  # the dominant GEMM family by measured time
        gem = {k: v for k, v in roofs.items() if k.startswith("gemm")}
        main_fam = max(gem, key=lambda k: gem[k]["ms_per_step_caller_stream"]) if gem else None
    result = {
        "metric": METRIC, "value": round(value, 2), "unit": "pairs/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 2),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": {"fp8": "fp8 (MXFP8 e4m3 tower GEMMs; bf16 elsewhere)", "fp32": "fp32",
                  "bf16x3": "fp32 (tower GEMMs as bf16x3 split products, fp32 accumulation)"}.get(args.precision, "bf16"),
        "data": f"synthetic: CLIP-normalised U[0,1) {cfg.vision_config.image_size}px pixels + BOS/random-id/EOS captions (77 tok, EOS pad), "
                "random-init weights",
        "config": {"workload": f"{cfg.name} {'full fine-tune (adapters off)' if not adapters else 'adapter fine-tune'}"
                               f" contrastive step: fwd+bwd+all-reduce+clip+AdamW",
                   "per_gpu_batch": args.batch, "global_batch": args.batch * world,
                   "image_size": cfg.vision_config.image_size,
                   "text_len": 77, "parallelism": f"dp{world}",
                   "comm": f"{'libclipmi' if args.comm == 'clipmi' else 'torch.distributed'} RCCL, "
                           f"{args.grad_bucket_dtype} gradient buckets" if world > 1 else None},
        # bf16x3: the model's flops against a third of the bf16 peak (three bf16 products per fp32 one)
        "mfma_frac_step": round(value * step_flops_pair / (world * {"fp8": PEAK_FP8_TFLOPS, "fp32": PEAK_FP32_TFLOPS,
                                                                    "bf16x3": PEAK_BF16_TFLOPS / 3}
                                                           .get(args.precision, PEAK_BF16_TFLOPS) * 1e12), 4),
        "step_tflops_per_gpu": round(value * step_flops_pair / world / 1e12, 1),
        "loss": round(float(loss.item()), 4),
        "roofline": roofs.get(main_fam) if main_fam else None,
        "rooflines": {k: v for k, v in roofs.items() if k != main_fam},
        "cpu_baseline": None,
    }
    if (world == 1 and args.parity_steps > 0 and args.precision == "bf16" and not adapters):
        del model, opt, params
        torch.cuda.empty_cache()
        result["parity_mode"] = parity_mode_run(args, cfg, dev, batch)
    if rank == 0 and world == 1 and args.cpu_sample > 0:
        result["cpu_baseline"] = cpu_baseline(cfg, args.cpu_sample, args.cpu_steps, adapters)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

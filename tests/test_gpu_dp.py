"""Data-parallel path with the real kernels: 2 ranks share cuda:0 over a gloo group, and, where
two GPUs are visible, 2 ranks over RCCL (one GPU each; skipped on a one-GPU box).  The sum of
the ranks' losses and the all-reduced gradients must equal the single-device result on
the same global batch, fp32 parity mode."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _worker(rank, world, port, q, overlap=False, chunk=None, shared=False, backend="gloo", bucket=None):
    try:
        _worker_body(rank, world, port, q, overlap, chunk, shared, backend, bucket)
    except BaseException:  # report instead of leaving the parent waiting on the queue
        import traceback
        q.put((rank, None, traceback.format_exc()))
        raise


def _worker_body(rank, world, port, q, overlap, chunk, shared, backend="gloo", bucket=None):
    import sys
    if chunk is not None:  # column-streamed contrastive: Bg = 8 in chunks of 3, 3, 2
        os.environ["CLIPMI_CE_CHUNK"] = str(chunk)
    if world == 1:  # one-rank group: take the collective branches anyway (each is the identity)
        os.environ["CLIPMI_DP_FORCE_COLLECTIVES"] = "1"
    sys.path.insert(0, os.path.join(REPO, "vlm-clip_amd"))
    import torch.distributed as dist
    from clipmi import CLIPWithAdapters, synth
    from clipmi.trainer import FusedAdamW
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    # gloo: both ranks on cuda:0; nccl (= RCCL through torch) and clipmi (RCCL issued by libclipmi, a
    # clipmi.comm.Communicator bootstrapped over a gloo group's store): one GPU per rank
    dev = f"cuda:{rank}" if backend in ("nccl", "clipmi") else "cuda:0"
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo" if backend == "clipmi" else backend, rank=rank, world_size=world)
    group = dist.group.WORLD
    if backend == "clipmi":
        from clipmi.comm import Communicator
        group = Communicator.from_process_group(dist.group.WORLD)
    # shared adapters need text hidden 512 (their text_projection, model_m.py:54-61): B/32
    m = CLIPWithAdapters("B/32" if shared else "tiny", use_text_adapter=True, use_vision_adapter=True,
                         use_shared_adapters=shared,
                         freeze_clip=False, device=dev, precision="fp32", pooling="eos",
                         process_group=group)
    if shared:
        m.eval()  # shared-adapter dropout off: the ranks must reproduce the single-device gradients
    B = 4
    b = {k: torch.from_numpy(v).to(dev) for k, v in synth.synthetic_batch(m.config, B, seed=5, start=rank * B).items()}
    if overlap:  # gradient buckets all-reduced from the towers' chunked backward (GradBucketReducer)
        opt = FusedAdamW([p for p in m.parameters() if p.requires_grad], lr=1e-3, arenas=m.arenas(),
                         process_group=group,
                         grad_bucket_dtype=torch.bfloat16 if bucket == "bf16" else torch.float32).overlap_with(m)
    else:
        opt = FusedAdamW([p for p in m.parameters() if p.requires_grad], lr=1e-3, arenas=m.arenas())
    opt.zero_grad()
    out = m(**b)
    opt.armed_backward(out["loss"])
    opt.grads_all_reduce(group)
    torch.cuda.synchronize()
    g = {n: p.grad.detach().cpu().numpy().copy() for n, p in m.named_parameters() if p.grad is not None}
    q.put((rank, out["loss"].item(), g))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("overlap,chunk,shared,backend", [(False, None, False, "gloo"), (True, None, False, "gloo"),
                                                          (False, 3, False, "gloo"), (True, None, True, "gloo"),
                                                          # RCCL, one GPU per rank: the comm-stream ordering the
                                                          # overlapped reducer relies on
                                                          (True, None, False, "nccl"), (False, 3, False, "nccl"),
                                                          # RCCL issued by libclipmi (clipmi.comm.Communicator)
                                                          (True, None, False, "clipmi"), (False, 3, False, "clipmi")])
def test_two_rank_data_parallel_matches_single_device(overlap, chunk, shared, backend):
    """shared=True: shared adapters on an unfrozen CLIP add a position-embedding gradient after the
    vision tower's backward, so the overlapped reducer must leave that block to finish().
    backend nccl needs two visible GPUs (skipped on a one-GPU box)."""
    if backend in ("nccl", "clipmi") and torch.cuda.device_count() < 2:
        pytest.skip("RCCL ranks need one GPU each")
    import torch.multiprocessing as mp
    from clipmi import CLIPWithAdapters, synth
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29700 + os.getpid() % 500
    port += 37 * int(overlap) + 71 * int(chunk is not None) + 113 * int(shared) + 157 * int(backend == "nccl")
    port += 211 * int(backend == "clipmi")
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, overlap, chunk, shared, backend)) for r in range(2)]
    for p in procs:
        p.start()
    res = []
    for _ in procs:
        r = q.get(timeout=200)
        if r[1] is None:  # a rank failed: its partner may be stuck in a collective
            for p in procs:
                p.kill()
            raise AssertionError(f"rank {r[0]} failed:\n{r[2]}")
        res.append(r)
    res.sort(key=lambda x: x[0])
    for p in procs:
        p.join(120)
    m = CLIPWithAdapters("B/32" if shared else "tiny", use_shared_adapters=shared, freeze_clip=False, device="cuda:0",
                         precision="fp32", pooling="eos")
    if shared:
        m.eval()
    b = {k: torch.from_numpy(v).cuda() for k, v in synth.synthetic_batch(m.config, 8, seed=5).items()}
    out = m(**b)
    out["loss"].backward()
    torch.cuda.synchronize()
    ref = {n: p.grad.detach().cpu().numpy() for n, p in m.named_parameters() if p.grad is not None}
    gmax = max(float(np.abs(r).max()) for r in ref.values())
    for rank, loss, g in res:
        assert abs(loss - out["loss"].item()) < 1e-5, (rank, loss, out["loss"].item())
        worst = (0.0, "")
        for n, r in ref.items():
            # floor at 1 % of the largest gradient: some true gradients are ~0 (k biases)
            scale = max(float(np.abs(r).max()), 1e-2 * gmax)
            worst = max(worst, (float(np.abs(g[n] - r).max()) / scale, n))
        assert worst[0] < 1e-4, worst


@pytest.mark.parametrize("overlap,chunk,backend,bucket", [(True, None, "nccl", None), (False, 3, "nccl", None),
                                                          (True, None, "clipmi", None), (False, 3, "clipmi", None),
                                                          (True, None, "clipmi", "bf16")])
def test_one_rank_rccl_group_matches_single_device(overlap, chunk, backend, bucket):
    """The RCCL branches of the data-parallel path -- the embedding all-gather and gradient reduce-scatter
    around the contrastive loss, the bucketed all-reduce from the comm stream (overlap) or after the backward
    -- executed where only one GPU is visible: a one-rank group with CLIPMI_DP_FORCE_COLLECTIVES=1 takes every
    collective branch, each then the identity, so the result must equal the group-free run on the same 4
    samples.  backend nccl: torch.distributed's RCCL; clipmi: a clipmi.comm.Communicator, so the exchanges run
    as clipmi_allgather_embed / clipmi_reducescatter_grad / clipmi_allreduce.  bucket bf16: the gradient buckets
    reduced in bf16 -- at one rank each gradient comes back rounded to bf16, within 2^-8 of its scale."""
    import torch.multiprocessing as mp
    from clipmi import CLIPWithAdapters, synth
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 30300 + os.getpid() % 500 + 37 * int(overlap) + 71 * int(backend == "clipmi") + 113 * int(bucket is not None)
    p = ctx.Process(target=_worker, args=(0, 1, port, q, overlap, chunk, False, backend, bucket))
    p.start()
    r = q.get(timeout=200)
    if r[1] is None:
        p.kill()
        raise AssertionError(f"rank 0 failed:\n{r[2]}")
    p.join(120)
    m = CLIPWithAdapters("tiny", use_shared_adapters=False, freeze_clip=False, device="cuda:0", precision="fp32",
                         pooling="eos")
    b = {k: torch.from_numpy(v).cuda() for k, v in synth.synthetic_batch(m.config, 4, seed=5).items()}
    out = m(**b)
    out["loss"].backward()
    torch.cuda.synchronize()
    ref = {n: q_.grad.detach().cpu().numpy() for n, q_ in m.named_parameters() if q_.grad is not None}
    gmax = max(float(np.abs(v).max()) for v in ref.values())
    _, loss, g = r
    assert abs(loss - out["loss"].item()) < 1e-5, (loss, out["loss"].item())
    worst = (0.0, "")
    for n, v in ref.items():
        scale = max(float(np.abs(v).max()), 1e-2 * gmax)
        worst = max(worst, (float(np.abs(g[n] - v).max()) / scale, n))
    assert worst[0] < (2 ** -8 if bucket == "bf16" else 1e-4), worst

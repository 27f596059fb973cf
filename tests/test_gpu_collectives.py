"""The C-ABI collectives (clipmi_allgather_embed / clipmi_reducescatter_grad / clipmi_allreduce_grads over RCCL,
SURVEY §8b) through clipmi.comm: a one-rank communicator on the test GPU (the exchanges reduce to copies and
identities, exactly), and, where two GPUs are visible, two ranks in two processes (skipped on a one-GPU box)."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_single_rank_collectives_exact(dtype):
    from clipmi import comm
    c = comm.Communicator(comm.unique_id(), 1, 0)
    try:
        x = torch.randn(1024, 512, device="cuda").to(dtype)
        assert torch.equal(c.all_gather(x), x)
        assert torch.equal(c.reduce_scatter(x), x)
        g = torch.randn(3 * 2 ** 20 + 7, device="cuda")
        g0 = g.clone()
        c.all_reduce_(g)
        torch.cuda.synchronize()
        assert torch.equal(g, g0)
        gb = g.to(torch.bfloat16)  # the bf16 gradient buckets (clipmi_allreduce with CLIPMI_BF16)
        gb0 = gb.clone()
        c.all_reduce_(gb)
        torch.cuda.synchronize()
        assert torch.equal(gb, gb0)
        with pytest.raises(ValueError):
            c.all_reduce_(x.to(torch.float16))
    finally:
        c.close()


def _rank(rank, uid, q):
    try:
        import sys
        sys.path.insert(0, os.path.join(REPO, "vlm-clip_amd"))
        torch.cuda.set_device(rank)
        from clipmi import comm
        c = comm.Communicator(uid, 2, rank)
        x = torch.full((4, 8), float(rank + 1), device="cuda")
        ag = c.all_gather(x).cpu()
        rs = c.reduce_scatter(torch.arange(16, dtype=torch.float32, device="cuda").view(8, 2) * (rank + 1)).cpu()
        g = torch.full((1000,), float(rank + 1), device="cuda")
        ar = c.all_reduce_(g).cpu()
        torch.cuda.synchronize()
        c.close()
        q.put((rank, ag, rs, ar, None))
    except BaseException:
        import traceback
        q.put((rank, None, None, None, traceback.format_exc()))


def test_two_rank_collectives():
    if torch.cuda.device_count() < 2:
        pytest.skip("two GPUs needed (one rank per GPU)")
    import torch.multiprocessing as mp
    from clipmi import comm
    uid = comm.unique_id()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_rank, args=(r, uid, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = {}
    for _ in range(2):
        r, ag, rs, ar, err = q.get(timeout=240)
        assert err is None, err
        out[r] = (ag, rs, ar)
    for p in ps:
        p.join(timeout=60)
    full = torch.arange(16, dtype=torch.float32).view(8, 2) * 3  # rank 0 x1 + rank 1 x2
    for r in range(2):
        ag, rs, ar = out[r]
        assert torch.equal(ag[:4], torch.full((4, 8), 1.0)) and torch.equal(ag[4:], torch.full((4, 8), 2.0))
        assert torch.equal(rs, full[4 * r:4 * r + 4])
        assert torch.equal(ar, torch.full((1000,), 3.0))

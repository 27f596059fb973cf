"""Attention kernel throughput on the CLIP shapes (GPU): forward with the whole-K/V kernel (pf)
and the K/V-streaming flash kernel (fa), backward; algorithmic FLOPs as the live profiler counts
them (4*B*H*N*Npad*64 forward, 10*... backward, Npad = N rounded to 32)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "vlm-clip_amd"))
import torch
from clipmi import kernels as K, towers as T

SHAPES = [("vision_b16", 1024, 197, 12, False), ("text", 1024, 77, 8, True), ("vision_l14", 512, 257, 16, False),
          ("vision_l14_336", 256, 577, 16, False)]
only = sys.argv[1:] or None
NWS = os.environ.get("ATTN_NWS", "8").split(",")  # whole-K/V kernels: waves per workgroup (8 = production; A/B in one process)


def timeit(f, n=10):
    f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


for name, B, N, H, causal in SHAPES:
    if only and name not in only:
        continue
    D = H * 64
    qkv = (torch.randn(B * N, 3 * D, device="cuda") * 1.0).to(torch.bfloat16)
    mask = None
    if causal:
        lens = torch.randint(5, N + 1, (B,), device="cuda")
        mask = (torch.arange(N, device="cuda")[None] < lens[:, None]).to(torch.int64)
    o = torch.empty(B * N, D, dtype=torch.bfloat16, device="cuda")
    lse = torch.empty(B * H * N, device="cuda")
    do = torch.randn(B * N, D, device="cuda").to(torch.bfloat16)
    dqkv = torch.empty_like(qkv)
    s = K.stream()
    npad = (N + 31) // 32 * 32
    mp = mask.data_ptr() if mask is not None else None
    fwd = lambda: T.call("clipmi_attention_fwd", s, 1, qkv.data_ptr(), o.data_ptr(), lse.data_ptr(), mp, int(causal),
                         B, H, N, D)
    bwd = lambda: T.call("clipmi_attention_bwd", s, 1, qkv.data_ptr(), o.data_ptr(), lse.data_ptr(), do.data_ptr(),
                         dqkv.data_ptr(), mp, int(causal), B, H, N, D)
    for rep in range(2):
        for nw in NWS:
            os.environ["CLIPMI_ATTN_FWD_NW"] = os.environ["CLIPMI_ATTN_BWD_NW"] = nw
            for kern in ("pf", "fa"):
                if kern == "pf" and N > 288:
                    continue
                os.environ["CLIPMI_ATTN_FA"] = "1" if kern == "fa" else "0"
                ms = timeit(fwd)
                fl = 4.0 * B * H * N * npad * 64
                print(f"{name:16s} nw{nw:>2s} fwd {kern}: {ms * 1e3:8.1f} us {fl / ms / 1e9:7.1f} TF/s", flush=True)
            os.environ["CLIPMI_ATTN_FA"] = "0"
            for sp in os.environ.get("ATTN_BWD_SP", "0").split(","):  # 0: production two-phase; 1: single-pass (A/B)
                os.environ["CLIPMI_ATTN_BWD_SP"] = sp
                ms = timeit(bwd)
                fl = 10.0 * B * H * N * npad * 64
                print(f"{name:16s} nw{nw:>2s} bwd sp{sp}: {ms * 1e3:8.1f} us {fl / ms / 1e9:7.1f} TF/s", flush=True)

"""bf16x3 attention (csrc/attention_x3.hip) on the CLIP shapes: forward / backward time for the block-per-wave
variants (CLIPMI_ATTN_X3_NB, CLIPMI_ATTN_X3_NBA) in one process, A/B/A/B, plus their agreement with the production
form.  MFMA work counted as issued: three products per fp32 product."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "vlm-clip_amd"))
import torch
from clipmi import kernels as K, towers as T

SHAPES = [("vision_b16", 1024, 197, 12, False), ("text", 1024, 77, 8, True)]
VARIANTS = [v.split(":") for v in os.environ.get("X3_VARIANTS", "1:1,2:1,2:2").split(",")]  # NB:NBA
only = sys.argv[1:] or None


def timeit(f, n=5):
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
    torch.manual_seed(0)
    qkv = torch.randn(B * N, 3 * D, device="cuda")
    mask = None
    if causal:
        lens = torch.randint(5, N + 1, (B,), device="cuda")
        mask = (torch.arange(N, device="cuda")[None] < lens[:, None]).to(torch.int64)
    o = torch.empty(B * N, D, device="cuda")
    lse = torch.empty(B * H * N, device="cuda")
    do = torch.randn(B * N, D, device="cuda")
    dqkv = torch.empty_like(qkv)
    s = K.stream()
    npad = (N + 31) // 32 * 32
    mp = mask.data_ptr() if mask is not None else None
    fwd = lambda: T.call("clipmi_attention_fwd_x3", s, qkv.data_ptr(), o.data_ptr(), lse.data_ptr(), mp, int(causal),
                         B, H, N, D)
    bwd = lambda: T.call("clipmi_attention_bwd_x3", s, qkv.data_ptr(), o.data_ptr(), lse.data_ptr(), do.data_ptr(),
                         dqkv.data_ptr(), mp, int(causal), B, H, N, D)
    ref = None
    for rep in range(2):
        for nb, nba in VARIANTS:
            os.environ["CLIPMI_ATTN_X3_NB"], os.environ["CLIPMI_ATTN_X3_NBA"] = nb, nba
            mf = timeit(fwd)
            mb = timeit(bwd)
            fwd()
            bwd()
            torch.cuda.synchronize()
            out = (o.clone(), lse.clone(), dqkv.clone())
            if ref is None:
                ref = out
            dif = max(float((a - b).abs().max() / (b.abs().max() + 1e-30)) for a, b in zip(out, ref))
            ff, fb = 3 * 4.0 * B * H * N * npad * 64, 3 * 10.0 * B * H * N * npad * 64
            print(f"{name:12s} nb{nb} nba{nba}: fwd {mf * 1e3:8.1f} us {ff / mf / 1e9:6.0f} TF/s  bwd {mb * 1e3:8.1f} us "
                  f"{fb / mb / 1e9:6.0f} TF/s  max rel diff vs first {dif:.1e}", flush=True)

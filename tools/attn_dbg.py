import os, sys
sys.path.insert(0, "vlm-clip_amd"); sys.path.insert(0, "tests")
import torch
from clipmi import kernels as kern, towers as T
from test_gpu_kernels import attn_ref, rnd
os.environ["CLIPMI_ATTN_FA"] = "1"
for (B, N, H, causal, usemask) in [(130, 77, 8, True, True), (130, 77, 8, True, False), (130, 77, 8, False, True), (3, 77, 8, True, True), (40, 77, 8, True, True)]:
    D = H * 64
    qkv = rnd((B * N, 3 * D), 11, torch.bfloat16)
    mask = None
    if usemask:
        g = torch.Generator().manual_seed(12)
        lens = torch.randint(5, N + 1, (B,), generator=g)
        mask = (torch.arange(N)[None] < lens[:, None]).to(torch.int64).cuda()
    o = torch.empty(B * N, D, dtype=torch.bfloat16, device="cuda")
    lse = torch.empty(B * H * N, device="cuda")
    T.call("clipmi_attention_fwd", kern.stream(), 1, qkv.data_ptr(), o.data_ptr(), lse.data_ptr(),
           mask.data_ptr() if mask is not None else None, int(causal), B, H, N, D)
    oref, lref = attn_ref(qkv.float(), B, N, H, mask, causal)
    torch.cuda.synchronize()
    err = (o.float() - oref).abs().view(B, N, H, 64).amax(-1)  # [B, N, H]
    bad = (err > 0.05).nonzero()
    print(B, N, H, causal, usemask, "max err", err.max().item(), "bad rows", bad.shape[0], bad[:8].tolist(), flush=True)
    if usemask and bad.shape[0]:
        print(" lens of bad b:", sorted(set(lens[bad[:, 0].cpu()].tolist()))[:10])

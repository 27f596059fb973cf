"""Per-shape GEMM throughput of libclipmi on the ViT-B/16 B=1024 training shapes (GPU).

GEMM_VARIANTS=0,10 (force_small_tile values; 0 = production schedule) picks the schedules;
every variant's output is checked against variant 0's on the same inputs (max rel diff);
GEMM_TORCH=1 adds torch.matmul (hipBLASLt, plain product) for reference."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "vlm-clip_amd"))
import torch
from clipmi import kernels as K, _lib

R = 1024 * 197
RT = 1024 * 77
if os.environ.get("GEMM_ROWS"):  # GEMM_ROWS=vision,text: other batches (config 2, B/32 B=256: 12800,19712)
    R, RT = (int(x) for x in os.environ["GEMM_ROWS"].split(","))
SHAPES = [  # name, M, N, K, a_kmajor, b_kmajor, out dtype, flags, split
    ("fc1_fwd", R, 3072, 768, True, True, torch.bfloat16, _lib.EPI_BIAS | _lib.EPI_QGELU | _lib.EPI_STORE_PRE, 1),
    ("fc2_fwd", R, 768, 3072, True, True, torch.bfloat16, _lib.EPI_BIAS | _lib.EPI_RESID, 1),
    ("qkv_fwd", R, 2304, 768, True, True, torch.bfloat16, _lib.EPI_BIAS, 1),
    ("out_fwd", R, 768, 768, True, True, torch.bfloat16, _lib.EPI_BIAS | _lib.EPI_RESID, 1),
    ("fc2_dgrad", R, 3072, 768, True, False, torch.bfloat16, _lib.EPI_DQGELU, 1),
    # the training path's forms since r03: fc1 stores quick_gelu'(pre), fc2's dgrad multiplies by it
    ("fc1_fwd_dact", R, 3072, 768, True, True, torch.bfloat16, _lib.EPI_BIAS | _lib.EPI_QGELU | _lib.EPI_STORE_DACT, 1),
    ("fc2_dgrad_ma", R, 3072, 768, True, False, torch.bfloat16, _lib.EPI_MUL_AUX, 1),
    ("t_fc1_fwd_dact", RT, 2048, 512, True, True, torch.bfloat16, _lib.EPI_BIAS | _lib.EPI_QGELU | _lib.EPI_STORE_DACT, 1),
    ("t_fc2_dgrad_ma", RT, 2048, 512, True, False, torch.bfloat16, _lib.EPI_MUL_AUX, 1),
    ("fc1_dgrad", R, 768, 3072, True, False, torch.bfloat16, 0, 1),
    ("qkv_dgrad", R, 768, 2304, True, False, torch.bfloat16, 0, 1),
    ("out_dgrad", R, 768, 768, True, False, torch.bfloat16, 0, 1),
    ("fc1_wgrad", 3072, 768, R, False, False, torch.float32, _lib.EPI_BETA, 2),
    ("fc2_wgrad", 768, 3072, R, False, False, torch.float32, _lib.EPI_BETA, 2),
    ("qkv_wgrad", 2304, 768, R, False, False, torch.float32, _lib.EPI_BETA, 2),
    ("out_wgrad", 768, 768, R, False, False, torch.float32, _lib.EPI_BETA, 2),
    ("t_fc1_fwd", RT, 2048, 512, True, True, torch.bfloat16, _lib.EPI_BIAS | _lib.EPI_QGELU | _lib.EPI_STORE_PRE, 1),
    ("t_fc2_fwd", RT, 512, 2048, True, True, torch.bfloat16, _lib.EPI_BIAS | _lib.EPI_RESID, 1),
    ("t_qkv_fwd", RT, 1536, 512, True, True, torch.bfloat16, _lib.EPI_BIAS, 1),
    ("t_fc2_dgrad", RT, 2048, 512, True, False, torch.bfloat16, _lib.EPI_DQGELU, 1),
    ("t_fc1_dgrad", RT, 512, 2048, True, False, torch.bfloat16, 0, 1),
    ("t_qkv_dgrad", RT, 512, 1536, True, False, torch.bfloat16, 0, 1),
    # the bf16 mode's fp32 residual stream (round 5): out-projection and fc2 write the fp32 sum
    ("fc2_fwd_r32", R, 768, 3072, True, True, torch.float32, _lib.EPI_BIAS | _lib.EPI_RESID, 1),
    ("out_fwd_r32", R, 768, 768, True, True, torch.float32, _lib.EPI_BIAS | _lib.EPI_RESID, 1),
    ("t_fc2_fwd_r32", RT, 512, 2048, True, True, torch.float32, _lib.EPI_BIAS | _lib.EPI_RESID, 1),
    ("t_out_fwd_r32", RT, 512, 512, True, True, torch.float32, _lib.EPI_BIAS | _lib.EPI_RESID, 1),
    ("t_out_dgrad", RT, 512, 512, True, False, torch.bfloat16, 0, 1),
    ("t_fc1_wgrad", 2048, 512, RT, False, False, torch.float32, _lib.EPI_BETA, 2),
    ("t_fc2_wgrad", 512, 2048, RT, False, False, torch.float32, _lib.EPI_BETA, 2),
    ("t_qkv_wgrad", 1536, 512, RT, False, False, torch.float32, _lib.EPI_BETA, 2),
    ("t_out_wgrad", 512, 512, RT, False, False, torch.float32, _lib.EPI_BETA, 2),
    # the same shapes with K = 64: prologue + epilogue cost per tile
    ("fc1_k64", R, 3072, 64, True, True, torch.bfloat16, _lib.EPI_BIAS | _lib.EPI_QGELU | _lib.EPI_STORE_PRE, 1),
    ("qkv_k64", R, 2304, 64, True, True, torch.bfloat16, _lib.EPI_BIAS, 1),
    ("fc2d_k64", R, 3072, 64, True, False, torch.bfloat16, _lib.EPI_DQGELU, 1),
    # K sweep of the qkv forward (per-tile fixed cost vs per-k-step cost) and the same with no epilogue flags
    ("qkv_k192", R, 2304, 192, True, True, torch.bfloat16, _lib.EPI_BIAS, 1),
    ("qkv_k384", R, 2304, 384, True, True, torch.bfloat16, _lib.EPI_BIAS, 1),
    ("qkv_k1536", R, 2304, 1536, True, True, torch.bfloat16, _lib.EPI_BIAS, 1),
    ("qkv_fwd_noepi", R, 2304, 768, True, True, torch.bfloat16, 0, 1),
    ("fc1_fwd_bias", R, 3072, 768, True, True, torch.bfloat16, _lib.EPI_BIAS, 1),
    ("fc1_fwd_qgelu", R, 3072, 768, True, True, torch.bfloat16, _lib.EPI_BIAS | _lib.EPI_QGELU, 1),
    # reference points (not on the CLIP path): square, operands resident in MALL
    ("sq4k", 4096, 4096, 4096, True, True, torch.bfloat16, 0, 1),
    ("sq8k", 8192, 8192, 8192, True, True, torch.bfloat16, 0, 1),
]
if os.environ.get("GEMM_SPLITS"):  # GEMM_SPLITS=7,9,28: each wgrad shape once per explicit split (+ reduce)
    SHAPES = [sh[:-1] + (sp,) if sh[-1] == 2 else sh
              for sh in SHAPES for sp in ([int(x) for x in os.environ["GEMM_SPLITS"].split(",")] if sh[-1] == 2 else [0])]
VARIANTS = [int(v) for v in os.environ.get("GEMM_VARIANTS", "0,10").split(",")]
REPS = int(os.environ.get("GEMM_REPS", "10"))
only = sys.argv[1:] if len(sys.argv) > 1 else None


def timeit(f, n=REPS):
    for _ in range(2):
        f()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(n):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


torch.manual_seed(0)
# clock warm-up: ~1 s of bf16 GEMMs so the first measured shape does not pay the DVFS ramp
_w = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
_e = torch.cuda.Event(enable_timing=True)
_t0 = torch.cuda.Event(enable_timing=True)
_t0.record()
for _ in range(1000):
    _w2 = _w @ _w
    if _ % 50 == 49:
        _e.record()
        _e.synchronize()
        if _t0.elapsed_time(_e) > 1000:
            break
del _w, _w2
for name, M, N, Kd, akm, bkm, odt, flags, split in SHAPES:
    if (only and name not in only) or (not only and (name in ("sq4k", "sq8k") or "_k" in name or name.endswith(
            ("_noepi", "_fwd_bias", "_fwd_qgelu")))):
        continue
    A = (torch.rand(M * Kd, device="cuda") * 2 - 1).to(torch.bfloat16)
    B = (torch.rand(N * Kd, device="cuda") * 2 - 1).to(torch.bfloat16)
    lda = Kd if akm else M
    ldb = Kd if bkm else N
    C = torch.zeros(M, N, device="cuda", dtype=odt)
    bias = torch.randn(N, device="cuda").to(torch.bfloat16)
    aux = (torch.randn(M, N, device="cuda").to(odt)
           if flags & (_lib.EPI_DQGELU | _lib.EPI_STORE_PRE | _lib.EPI_STORE_DACT | _lib.EPI_MUL_AUX) else None)
    res = torch.randn(M, N, device="cuda").to(odt) if flags & _lib.EPI_RESID else None
    if split == 2:  # engine.cpp wgrad_splits: round efficiency minus the slabs' cost
        tiles = ((M + 255) // 256) * ((N + 255) // 256)
        compute = 2.0 * M * N * Kd / (4.1e12 * 256)
        split, best = 1, -1e30
        for sp in range(1, 65):
            if sp > 1 and Kd // sp < 512:
                break
            wg = tiles * sp
            eff = wg / (256 * ((wg + 255) // 256))
            score = eff - (2.0 * sp * M * N * 4 / 4.0e12 if sp > 1 else 0.0) / compute
            if score > best + 0.005:
                split, best = sp, score
    if split == 0:
        continue
    ws = torch.empty(split * M * (N + 1), device="cuda") if split > 1 else None  # slabs + bias partials
    bg = torch.zeros(M, device="cuda") if (odt == torch.float32 and not akm and not bkm) else None  # wgrad only
    kw = dict(bias=bias if flags & _lib.EPI_BIAS else None, residual=res, ldr=N, aux=aux, ldaux=N, flags=flags,
              split_k=split, workspace=ws, bias_grad=bg)
    if os.environ.get("GEMM_TORCH"):  # hipBLASLt via torch.matmul, plain product, for comparison
        a2 = A.view(M, Kd) if akm else A.view(Kd, M).t()
        b2 = B.view(N, Kd).t() if bkm else B.view(Kd, N)
        ms = timeit(lambda: torch.matmul(a2, b2))
        print(f"{name:10s} torch M={M} N={N} K={Kd}: {ms * 1e3:8.1f} us {2 * M * N * Kd / ms / 1e9:7.1f} TF/s",
              flush=True)
    ref = None
    for v in VARIANTS:  # 0 = production schedule, 1 = 128 tile, >= 2: 256-kernel schedule
        kw2 = dict(kw, bias_grad=None) if (v == 1 and bg is not None) else kw
        f = lambda: K.gemm(M, N, Kd, A, lda, akm, B, ldb, bkm, C, N, small_tile=v, **kw2)
        C.zero_()
        f()
        torch.cuda.synchronize()
        out = C.float().clone()
        if ref is None:
            ref, err = out, 0.0
        else:
            err = ((out - ref).abs().max() / ref.abs().max().clamp_min(1e-6)).item()
        del out
        ms = timeit(f)
        print(f"{name:10s} v{v} M={M} N={N} K={Kd} split={split}: {ms * 1e3:8.1f} us "
              f"{2 * M * N * Kd / ms / 1e9:7.1f} TF/s  maxrel-vs-v{VARIANTS[0]} {err:.2e}", flush=True)
    del A, B, C, aux, res, ws, ref
    torch.cuda.empty_cache()

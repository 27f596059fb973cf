"""Per-launch HBM bytes of bench.py's GEMM families (wgrad, forward+dgrad) from rocprofv3
FETCH_SIZE / WRITE_SIZE passes (counter_collection.csv, values in KiB), over the launches
bench.py's live roofline times: the vision tower's (the caller's stream; the text tower runs on
a second stream).  gfx950 FETCH_SIZE counts 128-B requests as 64 B (MI355X_MICROARCH.md §HBM),
so fetched bytes = 2 x FETCH_SIZE; WRITE_SIZE is exact for 16-B-per-lane stores.
Usage: traffic_summary.py FETCH_DIR WRITE_DIR OUT_PREFIX"""
import csv, glob, json, os, sys

FAMILIES = {
    # wgrad: split-K weight-gradient kernels (r02: gemm256_kernel; since r03 the persistent 4-wave
    # gemm_w4p_kernel<false, false, float, ...>, demangled or mangled); with CLIPMI_OVERLAP=0 each
    # step's 97 launches come in program order, the vision backward's 48 encoder wgrads + the patch
    # embedding first
    "gemm256_wgrad": ("gemm256_kernel<false, false, float, 0,", "gemm_w4p_kernel<false, false, float",
                      "gemm_w4p_kernelILb0ELb0Ef"),
    # forward + dgrad: every gemm_pp_kernel instantiation; the vision tower's launches are the ones
    # whose grid is a multiple of its M tiles (B=1024: 201,728 rows = 788 tiles of 256)
    "gemm256_fwd_dgrad": ("gemm_pp_kernel", "gemm_w4p_kernel<true", "gemm_w4p_kernelILb1"),  # demangled or mangled
}
# r03 forward + dgrad launches per step in program order (CLIPMI_OVERLAP=0): text forward 48, the
# patch embedding + vision forward 48, a 12-tile projection product, vision backward 48, an 8-tile
# one, text backward 48 -- the vision tower's are positions 48 .. 145
# r05 (fp32 residual stream: the patch embedding and the projections' forward are fp32-output launches of
# their own): text forward 48, text projection, patch embedding, vision forward 48, visual projection,
# a projection input gradient, vision backward 48, the text projection's, text backward 48 = 197; the
# vision tower's are positions 49 .. 147 (patch embedding .. vision backward, as r03's 48 .. 145)
FD_PER_STEP, FD_VISION = 197, (49, 148)
# r03: 99 wgrad launches per step -- a projection's (grid 6), the vision tower's 48 encoder wgrads +
# the patch embedding, the text projection's (grid 4), the text tower's 48 (r02: 97, vision first)
PER_STEP, VISION0, VISION, M_TILES = 99, 1, 49, 788
WORKLOAD = "ViT-B/16/1024/1"  # bench.py's default run (config name / per-GPU batch / training), matched by bench.py


def per_dispatch(d, counter, kernel):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    out, grid = {}, {}
    for r in csv.DictReader(open(f)):
        pats = kernel if isinstance(kernel, tuple) else (kernel,)
        if any(k in r["Kernel_Name"] for k in pats) and r["Counter_Name"] == counter:
            out[r["Dispatch_Id"]] = out.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
            grid[r["Dispatch_Id"]] = int(r["Grid_Size"]) // max(1, int(r["Workgroup_Size"]))
    ids = sorted(out, key=int)
    return [out[i] for i in ids], [grid[i] for i in ids]


def vision_only(family, vals, grids):
    if family == "gemm256_wgrad":
        assert len(vals) % PER_STEP == 0, f"{len(vals)} wgrad launches is not a whole number of steps"
        return [v for i, v in enumerate(vals) if VISION0 <= i % PER_STEP < VISION0 + VISION]
    assert len(vals) % FD_PER_STEP == 0, f"{len(vals)} forward/dgrad launches is not a whole number of steps"
    return [v for i, v in enumerate(vals) if FD_VISION[0] <= i % FD_PER_STEP < FD_VISION[1]]


def summarize(family, fetch_dir, write_dir):
    k = FAMILIES[family]
    fetch = vision_only(family, *per_dispatch(fetch_dir, "FETCH_SIZE", k))
    write = vision_only(family, *per_dispatch(write_dir, "WRITE_SIZE", k))
    rd = 2.0 * 1024 * sum(fetch) / len(fetch)
    wr = 1024.0 * sum(write) / len(write)
    return {"kernel": family, "workload": WORKLOAD, "launches": [len(fetch), len(write)], "read_bytes_per_launch": rd,
            "write_bytes_per_launch": wr, "bytes_per_launch": rd + wr,
            "subset": "vision tower launches (the ones bench.py's live roofline times on the caller's stream)",
            "method": "rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE in separate passes over CLIPMI_OVERLAP=0 bench.py "
                      "--steps 2 --warmup 1; FETCH_SIZE x2 (gfx950 tallies 128-B requests as 64 B; the guide's "
                      "calibration is for 16-B-per-lane streaming reads, which these LDS-DMA pieces are), KiB -> bytes"}


if __name__ == "__main__":
    # traffic_summary.py FETCH_DIR WRITE_DIR OUT_PREFIX  ->  OUT_PREFIX_wgrad.json, OUT_PREFIX_fwd_dgrad.json
    for fam, suffix in (("gemm256_wgrad", "wgrad"), ("gemm256_fwd_dgrad", "fwd_dgrad")):
        try:
            res = summarize(fam, sys.argv[1], sys.argv[2])
        except (ZeroDivisionError, AssertionError) as e:  # r03: the K >= 1536 forward/dgrad launches are
            print(fam, "not summarised:", e)               # persistent (grid 256), not matched by M tiles
            continue
        json.dump(res, open(f"{sys.argv[3]}_{suffix}.json", "w"), indent=1)
        print(fam, json.dumps(res))

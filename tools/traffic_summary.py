"""Per-launch HBM bytes of the roofline kernel family from rocprofv3 FETCH_SIZE / WRITE_SIZE
passes (counter_collection.csv, values in KiB), over the launches bench.py's live roofline
times: the vision tower's (the caller's stream; the text tower runs on a second stream).  The
passes run with CLIPMI_OVERLAP=0, so each step's 97 wgrad launches come in program order: the
vision backward's 48 encoder wgrads + the patch embedding, then the text tower's 48.  gfx950 FETCH_SIZE counts 128-B requests as
64 B (MI355X_MICROARCH.md §HBM): the wgrad kernel's LDS-DMA pieces are whole 128-B lines
(4 k-rows x 256 B), so fetched bytes = 2 x FETCH_SIZE.  WRITE_SIZE is exact for its 16-B
per-lane slab stores.  Usage: traffic_summary.py FETCH_DIR WRITE_DIR OUT.json"""
import csv, glob, json, os, sys

KERNEL = "gemm256_kernel<false, false, float, 0,"  # "gemm256_wgrad_splitk" in libclipmi's labels
LABEL = "gemm256_wgrad_splitk"


def per_dispatch(d, counter):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    out = {}
    for r in csv.DictReader(open(f)):
        if KERNEL in r["Kernel_Name"] and r["Counter_Name"] == counter:
            out[r["Dispatch_Id"]] = out.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return list(out.values())


PER_STEP, VISION = 97, 49


def vision_only(vals):
    assert len(vals) % PER_STEP == 0, f"{len(vals)} wgrad launches is not a whole number of steps"
    return [v for i, v in enumerate(vals) if i % PER_STEP < VISION]


fetch = vision_only(per_dispatch(sys.argv[1], "FETCH_SIZE"))
write = vision_only(per_dispatch(sys.argv[2], "WRITE_SIZE"))
rd = 2.0 * 1024 * sum(fetch) / len(fetch)
wr = 1024.0 * sum(write) / len(write)
res = {"kernel": LABEL, "launches": [len(fetch), len(write)], "read_bytes_per_launch": rd,
       "write_bytes_per_launch": wr, "bytes_per_launch": rd + wr,
       "subset": "vision tower launches (first 49 of each step's 97)",
       "method": "rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE in separate passes over CLIPMI_OVERLAP=0 bench.py "
                 "--steps 2 --warmup 1; FETCH_SIZE x2 (gfx950 reports 128-B requests as 64 B), KiB -> bytes"}
json.dump(res, open(sys.argv[3], "w"), indent=1)

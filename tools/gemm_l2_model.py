"""Model of the L2 fetch of the 256x256-tile GEMMs per tile order (CPU only; pins the PMC FETCH_SIZE).

Items are (k-slab, tile) pairs; the persistent kernels hand XCD x a contiguous run of ~32 item
indices per round (common.h xcd_remap, one workgroup per CU, 32 CUs per XCD), and the 8-wave
kernel's remapped grid gives each XCD a contiguous range of tiles that it walks ~32 at a time.
An item reads 256-row panels of A and B, one 64-k slice (32 KiB) per k-step, all of an XCD's
items in lockstep over k.

  wgrad   one round per launch: each XCD fetches every distinct (slab, panel) its items touch once.
          python3 tools/gemm_l2_model.py wgrad
  fwd     many rounds per launch: an LRU of 128 slices (the XCD's 4 MiB L2) per XCD, k-slices
          touched in item order; "snake" reverses k every other round (not built).
          python3 tools/gemm_l2_model.py fwd [max_rounds]

Checked against rocprofv3 FETCH_SIZE (x2, bytes) of gemm_bench launches (profiles/r05_wgrad_order_ab.log):
wgrad fc1 1.25x, fc2 1.66x row-major / 1.25x column-major, qkv 1.21x, out 1.125x -- model and counter
agree to the third digit.  Forward / input-gradient products (fwd): the weight panels leave L2 between
windows and are re-fetched (from the Infinity Cache) by every window: qkv / fc1 forward 3.7x / 5.7x of
their compulsory operand bytes, the N = 768 products 1.34x; the launch-mean model (1.27 GB + the
residual / aux reads) matches the measured 1.66 GB per vision launch (profiles/r05_traffic_fwd_dgrad.json)."""
import sys
from collections import OrderedDict

R = 1024 * 197  # ViT-B/16 tokens at B = 1024


def xcd_of_items(nwg):
    q, r = nwg >> 3, nwg & 7
    m = {}
    for bid in range(nwg):
        x = bid & 7
        m[(x * (q + 1) if x < r else r * (q + 1) + (x - r) * q) + (bid >> 3)] = x
    return m


def rowm(t, a, b):
    return t // b, t % b


def colm(t, a, b):
    return t % a, t // a


def rast(g):  # csrc/gemm_common.h tile_coords with p.raster = g
    def f(t, a, b):
        grp = t // (g * b)
        rem = t - grp * g * b
        rows = min(g, a - grp * g)
        tn = rem // rows
        return grp * g + rem - tn * rows, tn
    return f


def wgrad_ratio(M, N, K, splits, order):
    tm_, tn_ = (M + 255) // 256, (N + 255) // 256
    items = [(s, t) for s in range(splits) for t in range(tm_ * tn_)]
    x = xcd_of_items(min(len(items), 256))
    per = {}
    for i, (s, t) in enumerate(items):
        tm, tn = order(t, tm_, tn_)
        per.setdefault(x[i], set()).update({("A", s, tm), ("B", s, tn)})
    return sum(len(v) for v in per.values()) / (splits * (tm_ + tn_))


def fwd_fetch(M, N, K, order, rounds_max=None, snake=False, cap=128):
    """fetched bytes, compulsory operand bytes"""
    tm_, tn_ = (M + 255) // 256, (N + 255) // 256
    nt, ns = tm_ * tn_, K // 64
    nrounds = (nt + 255) // 256
    if rounds_max:
        nrounds = min(nrounds, rounds_max)
    miss, comp = 0, set()
    for x in range(8):
        lru = OrderedDict()
        for r in range(nrounds):
            tiles = [order(i, tm_, tn_) for i in (r * 256 + 32 * x + j for j in range(32)) if i < nt]
            for k in (range(ns - 1, -1, -1) if snake and r % 2 else range(ns)):
                for tm, tn in tiles:
                    for key in (("A", tm, k), ("B", tn, k)):
                        comp.add(key)
                        if key in lru:
                            lru.move_to_end(key)
                        else:
                            miss += 1
                            lru[key] = 1
                            if len(lru) > cap:
                                lru.popitem(last=False)
    return miss * 32768, len(comp) * 32768


WGRAD = {"fc1": (3072, 768, R, 7), "fc2": (768, 3072, R, 7), "qkv": (2304, 768, R, 9), "out": (768, 768, R, 28),
         "t_fc1": (2048, 512, 1024 * 77, 16), "t_fc2": (512, 2048, 1024 * 77, 16), "t_qkv": (1536, 512, 1024 * 77, 21),
         "t_out": (512, 512, 1024 * 77, 63)}
FWD = {"qkv_fwd": (R, 2304, 768), "out_fwd": (R, 768, 768), "fc1_fwd": (R, 3072, 768), "fc2_fwd": (R, 768, 3072),
       "qkv_dgrad": (R, 768, 2304), "out_dgrad": (R, 768, 768), "fc1_dgrad": (R, 768, 3072), "fc2_dgrad": (R, 3072, 768)}

if __name__ == "__main__":
    what = sys.argv[1] if len(sys.argv) > 1 else "wgrad"
    if what == "wgrad":
        for n, sh in WGRAD.items():
            print(f"{n:6s} row {wgrad_ratio(*sh, rowm):.3f}  col {wgrad_ratio(*sh, colm):.3f}  " +
                  "  ".join(f"r{g} {wgrad_ratio(*sh, rast(g)):.3f}" for g in (2, 3, 4, 8)))
    else:
        rm = int(sys.argv[2]) if len(sys.argv) > 2 else None
        tot = {False: [0, 0], True: [0, 0]}
        for n, (M, N, K) in FWD.items():
            line = []
            for sn in (False, True):
                f, c = fwd_fetch(M, N, K, rowm, rm, sn)
                tot[sn][0] += f
                tot[sn][1] += c
                line.append(f"{'snake' if sn else 'row'} {f / 1e9:.3f} GB ({f / c:.2f}x)")
            print(f"{n:10s} " + "  ".join(line), flush=True)
        for sn in (False, True):
            print(f"{'snake' if sn else 'row'}: launch mean {tot[sn][0] / len(FWD) / 1e9:.3f} GB fetched, "
                  f"{tot[sn][1] / len(FWD) / 1e9:.3f} GB compulsory")

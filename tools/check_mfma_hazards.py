"""Static check of the 4-wave GEMM's inline-asm MFMAs (csrc/gemm4.hip) for operand hazards the
compiler cannot see: a VALU instruction writing a VGPR/AGPR that the next MFMA (within 2
instructions) reads as a source.  hipcc pads hazards only around its own MFMAs, not around asm.

  python tools/check_mfma_hazards.py path/to/gemm4-hip-amdgcn-amd-amdhsa-gfx950.s
(produce the .s with: hipcc ... -c csrc/gemm4.hip --save-temps)"""
import re
import sys


def regs(tok):
    m = re.match(r"([va])\[(\d+):(\d+)\]", tok)
    if m:
        return {f"{m.group(1)}{i}" for i in range(int(m.group(2)), int(m.group(3)) + 1)}
    m = re.match(r"([va])(\d+)$", tok)
    return {tok} if m else set()


def main(path):
    lines = [l.strip() for l in open(path)]
    ins = [l for l in lines if l and not l.startswith((";", ".")) and not l.endswith(":")]
    bad = 0
    for i, l in enumerate(ins):
        if not l.startswith("v_mfma"):
            continue
        ops = [o.strip().split()[0] for o in l.split(None, 1)[1].split(",")]
        srcs = set().union(*(regs(o) for o in ops[1:]))  # A, B, C and (v_mfma_scale) the two scale operands
        for back in (1, 2):
            p = ins[i - back] if i >= back else ""
            if p.startswith("s_nop"):
                break
            if p.startswith(("v_", )) and not p.startswith("v_mfma"):
                dst = regs(p.split(None, 1)[1].split(",")[0].strip()) if " " in p else set()
                if dst & srcs:
                    bad += 1
                    print(f"hazard: '{p}' -> '{l}'")
    print(f"{bad} VALU-write -> MFMA-source hazards")
    return bad


if __name__ == "__main__":
    sys.exit(1 if main(sys.argv[1]) else 0)

#!/usr/bin/env python3
"""Static VALU issue-cost estimate of an asm line range, with the per-class
costs measured by tools/valu_cost.hip on MI355X (memtime cycles per
instruction per SIMD at 4 waves/SIMD): simple VOP1/VOP2 f32 ops 1.7, other
VALU 2.75, transcendentals / permlanes 5.0.
Usage: python tools/asm_cost.py file.s [first last] ..."""
import re
import sys

A_OPS = {"v_add_f32", "v_sub_f32", "v_subrev_f32", "v_mul_f32", "v_fmac_f32", "v_fma_f32", "v_mov_b32",
         "v_xor_b32", "v_add_u32", "v_sub_u32", "v_subrev_u32", "v_and_b32", "v_or_b32", "v_max_f32", "v_min_f32"}
C_PFX = ("v_exp_", "v_log_", "v_rcp_", "v_sqrt_", "v_rsq_", "v_sin_", "v_cos_", "v_permlane")


def cost(line):
    t = line.split()
    if not t or not t[0].startswith("v_"):
        return None
    op = t[0]
    base = re.sub(r"_(e32|e64|sdwa|dpp)$", "", op)
    if op.startswith(C_PFX):
        return "C"
    if base in A_OPS and not op.endswith(("_e64", "_sdwa", "_dpp")):
        ops = " ".join(t[1:])
        if re.search(r"\bs\d+|s\[", ops):
            return "B"
        return "A"
    return "B"


W = {"A": 1.7, "B": 2.75, "C": 5.0}


def region(lines, a, b):
    n = {"A": 0, "B": 0, "C": 0}
    for ln in lines[a - 1:b]:
        c = cost(ln.strip())
        if c:
            n[c] += 1
    return n, sum(W[k] * v for k, v in n.items())


if __name__ == "__main__":
    lines = open(sys.argv[1]).read().splitlines()
    args = sys.argv[2:]
    for i in range(0, len(args), 3):
        name, a, b = args[i], int(args[i + 1]), int(args[i + 2])
        n, c = region(lines, a, b)
        print(f"{name:10s} A {n['A']:4d}  B {n['B']:4d}  C {n['C']:3d}   cost {c:7.1f}")

#!/usr/bin/env python3
"""Per-tile issue-cycle model of a kernel's main loop (tools/isa.py --dump output on stdin).

Costs per wave64 instruction on one SIMD, measured on MI355X (profiles/r02/ubench_valu_cost.txt,
MFMA-calibrated): fp32 add/mul/fma/fmac/mov/sub and int add/and ("fast") 2.5 cycles; max/max3/
cvt/perm/DPP/v_pk_* and any VOP3 reading an SGPR ("slow") 4.3; exp/rcp/permlane*_swap 8;
32x32 MFMA (f16 x16, i8 x32) 32.  MFMA and VALU cycles ADD on a SIMD
(profiles/r02/ubench_mfma_split*.txt), so the sum is the loop's issue-time floor.
    python tools/isa.py <lib.o> <kernel> --dump | python tools/cycle_model.py <mfma per tile>
"""
import collections
import re
import sys

FAST = {"v_fma_f32", "v_fmac_f32_e32", "v_add_f32_e32", "v_mul_f32_e32", "v_sub_f32_e32", "v_mov_b32_e32",
        "v_fmaak_f32", "v_fmamk_f32", "v_add_u32_e32", "v_subrev_f32_e32", "v_and_b32_e32", "v_or_b32_e32",
        "v_lshlrev_b32_e32", "v_add_f32_e64", "v_mul_f32_e64", "v_sub_f32_e64", "v_fma_f32_e64",
        "v_cndmask_b32_e32", "v_cndmask_b32_e64", "v_sub_u32_e32", "v_subrev_u32_e32"}
EIGHT = {"v_exp_f32_e32", "v_rcp_f32_e32", "v_permlane32_swap_b32_e32", "v_permlane16_swap_b32_e32",
         "v_exp_f32_e64", "v_rcp_f32_e64"}


def main():
    per_tile_mfma = float(sys.argv[1]) if len(sys.argv) > 1 else 6.0
    body = [l for l in sys.stdin.read().split("\n") if l and not l.startswith((" ", "_Z"))]
    cost, n_mfma = collections.Counter(), 0
    for l in body:
        op = l.split()[0]
        if not op.startswith("v_"):
            continue
        if "mfma" in op:
            c = 32.0
            n_mfma += 1
        elif op in EIGHT:
            c = 8.0
        elif op in FAST:
            ops = l.split(None, 1)[1] if " " in l else ""
            c = 4.3 if re.search(r"\bs\d+|s\[", ops) else 2.5
        else:
            c = 4.3
        cost[op] += c
    tiles = n_mfma / per_tile_mfma
    print(f"tiles in loop {tiles:g}; modeled issue cycles per tile {sum(cost.values()) / tiles:.1f} "
          f"(MFMA {32 * per_tile_mfma:.0f})")
    for op, c in cost.most_common(20):
        print(f"  {c / tiles:7.1f} {op}")


if __name__ == "__main__":
    main()

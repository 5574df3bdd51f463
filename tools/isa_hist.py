#!/usr/bin/env python3
"""Static instruction histogram of one kernel in a gfx950 .s dump
(hipcc --cuda-device-only -S). Usage: isa_hist.py file.s symbol-substring.
Weights: measured issue cost per wave64 instruction (tools/micro/valu_rates.hip,
profiles/r02_valu_rates.txt): full-rate ~1.37, half-rate ~2.37, carry ops
and v_mad_u64_u32 ~2.58 cycles per SIMD."""
import re
import sys
from collections import Counter

FULL = {"v_xor_b32", "v_add_u32", "v_sub_u32", "v_lshrrev_b32", "v_lshlrev_b32", "v_bitop3_b32", "v_mov_b32",
        "v_and_b32", "v_or_b32", "v_subrev_u32", "v_ashrrev_i32", "v_not_b32"}
CARRY = {"v_add_co_u32", "v_addc_co_u32", "v_sub_co_u32", "v_subb_co_u32", "v_subrev_co_u32", "v_subbrev_co_u32",
         "v_mad_u64_u32"}


def kernel_lines(path, sym):
    out, on = [], False
    for ln in open(path):
        if re.match(r"^_Z\S*:", ln):
            on = sym in ln.split(":")[0]
            continue
        if on:
            if ln.startswith("\t.end_amdhsa_kernel") or ln.startswith(".Lfunc_end"):
                break
            out.append(ln)
    return out


def main():
    path, sym = sys.argv[1], sys.argv[2]
    c = Counter()
    for ln in kernel_lines(path, sym):
        m = re.match(r"\s+([sv]_\w+|ds_\w+|global_\w+|buffer_\w+|flat_\w+)", ln)
        if m:
            op = re.sub(r"_e(32|64)$", "", m.group(1))
            c[op] += 1
    valu = {k: v for k, v in c.items() if k.startswith("v_")}
    cost = sum(v * (1.37 if k in FULL else 2.58 if k in CARRY else 2.37) for k, v in valu.items())
    print(f"VALU instrs {sum(valu.values())}  weighted cycles {cost:.0f}  SALU {sum(v for k, v in c.items() if k.startswith('s_'))}"
          f"  LDS {sum(v for k, v in c.items() if k.startswith('ds_'))}  VMEM {sum(v for k, v in c.items() if k.startswith(('global', 'buffer', 'flat')))}")
    for k, v in c.most_common(40):
        print(f"  {v:6d} {k}")


if __name__ == "__main__":
    main()

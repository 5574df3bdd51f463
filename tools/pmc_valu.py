#!/usr/bin/env python3
"""Per-kernel VALU issue summary from one rocprofv3 --pmc pass
(SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU
SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE).

valu_ms = SQ_INSTS_VALU * 2 cycles / (1024 SIMDs * 2.4 GHz): the time the
kernel's VALU instructions need if every SIMD issued one wave64 instruction
per 2 cycles (MI355X_MICROARCH.md: 32 lanes/cycle, 2.4 GHz max clock);
valu_frac = valu_ms / kernel duration. Half-rate instructions (v_alignbit,
v_add3, v_mad_u64_u32, carry ops: tools/micro/valu_rates.hip) keep a saturated
kernel below 1.0.
"""
import csv
import re
import sys
from collections import defaultdict


def short(n):
    m = re.search(r"sezkp::(k_[A-Za-z0-9_]+)(<[^(]*>)?", n)
    return (m.group(1) + (m.group(2) or "")) if m else n.split("(")[0]


def main(path):
    per = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(dict)
    for r in csv.DictReader(open(path)):
        k = short(r["Kernel_Name"])
        per[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        dur[k][r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    rows = []
    for k, c in per.items():
        avg = {n: sum(v) / len(v) for n, v in c.items()}
        d = sorted(dur[k].values())
        ms = d[len(d) // 2]
        valu_ms = avg.get("SQ_INSTS_VALU", 0) * 2 / (1024 * 2.4e9) * 1e3
        rows.append((ms * len(d), k, len(d), ms, valu_ms, avg))
    rows.sort(reverse=True)
    print(f"{'kernel':44s} {'n':>4s} {'ms':>8s} {'valu_ms':>8s} {'frac':>5s} {'waves':>8s} {'valu/wave':>9s} {'lds/wave':>8s}")
    for _, k, n, ms, vms, a in rows:
        w = max(a.get("SQ_WAVES", 1), 1)
        print(f"{k[:44]:44s} {n:4d} {ms:8.4f} {vms:8.4f} {vms / ms if ms else 0:5.2f} {w:8.0f} "
              f"{a.get('SQ_INSTS_VALU', 0) / w:9.0f} {a.get('SQ_INSTS_LDS', 0) / w:8.0f}")


if __name__ == "__main__":
    main(sys.argv[1])

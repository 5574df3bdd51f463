#!/usr/bin/env python3
"""Kernel timeline of the last proof in a rocprofv3 kernel trace: one line per
kernel (start offset, duration, gap since the previous kernel on any stream,
stream id), plus busy/idle totals. Usage: tools/timeline.py run_kernel_trace.csv [first_kernel_name]"""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    first = sys.argv[2] if len(sys.argv) > 2 else "k_expand"
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("sezkp::", "")
           .replace("void ", ""), r["Stream_Id"], r["Grid_Size_X"], r["Workgroup_Size_X"]) for r in rows]
    ks.sort()
    starts = [i for i, k in enumerate(ks) if first in k[2]]
    a = starts[-1]
    b = len(ks)
    sel = ks[a:b]
    t0 = sel[0][0]
    end = t0
    busy = 0
    for s, e, name, sid, gx, wx in sel:
        gap = (s - end) / 1e3
        print(f"{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:8.1f} gap {gap:7.1f}  s{sid} grid {int(gx) // max(1, int(wx)):>7} {name[:60]}")
        busy += max(0, e - max(s, end))
        end = max(end, e)
    print(f"span {(end - t0) / 1e3:.1f} us, union busy {busy / 1e3:.1f} us, idle {(end - t0 - busy) / 1e3:.1f} us")


if __name__ == "__main__":
    main()

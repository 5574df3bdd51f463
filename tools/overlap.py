#!/usr/bin/env python3
"""Kernel-concurrency profile of an in-flight bench run from a rocprofv3
--kernel-trace CSV: fraction of the window with k kernels running, and per
kernel the time it ran alone (nothing to overlap with).

    python3 tools/overlap.py run_kernel_trace.csv T0_MS T1_MS NPROOFS
(T0/T1 in ms from the first dispatch of the trace)."""
import csv
import re
import sys
from collections import defaultdict


def short(n):
    m = re.search(r"sezkp::(k_[A-Za-z0-9_]+)(<[^(]*>)?", n)
    return (m.group(1) + (m.group(2) or "")) if m else n.split("(")[0][:30]


def main(path, a_ms, b_ms, nproofs):
    rows = list(csv.DictReader(open(path)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])) for r in rows)
    t0 = ev[0][0]
    start, end = t0 + int(a_ms * 1e6), t0 + int(b_ms * 1e6)
    pts = []
    sums = defaultdict(float)
    for s, e, n in ev:
        if e <= start or s >= end:
            continue
        s, e = max(s, start), min(e, end)
        sums[n] += e - s
        pts += [(s, 1, n), (e, -1, n)]
    pts.sort()
    active = defaultdict(int)
    last = start
    conc = defaultdict(float)
    alone = defaultdict(float)
    for t, d, n in pts:
        dt = t - last
        k = sum(active.values())
        conc[k] += dt
        if k == 1:
            for nn, c in active.items():
                if c:
                    alone[nn] += dt
        last = t
        active[n] += d
    conc[0] += end - last
    tot = end - start
    print(f"window {tot / 1e6:.3f} ms, {tot / 1e6 / nproofs:.3f} ms per proof")
    for k in sorted(conc):
        print(f"  {k} kernels running: {conc[k] / tot:.3f}")
    print("kernel: busy ms/proof (sum of its intervals) | ran alone ms/proof")
    for n, v in sorted(sums.items(), key=lambda x: -x[1])[:25]:
        print(f"  {n[:44]:44s} {v / 1e6 / nproofs:7.4f} | {alone[n] / 1e6 / nproofs:7.4f}")


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]), float(sys.argv[3]), int(sys.argv[4]))

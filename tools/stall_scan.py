#!/usr/bin/env python3
"""Scan a rocprofv3 kernel trace (run_kernel_trace.csv) of the default bench
for stalls: summed kernel time per 2 ms window (3 proofs in flight keep it
near 3), the longest contiguous busy run (warmup + timed pipeline), and every
window inside it whose summed kernel time falls below a threshold."""
import collections
import csv
import sys


def main(path, win_ms=2.0, low=1.5):
    rows = list(csv.DictReader(open(path)))
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows)
    t0, W = iv[0][0], int(win_ms * 1e6)
    busy = collections.Counter()
    for s, e in iv:
        a = s
        while a < e:
            w = (a - t0) // W
            b = min(e, t0 + (w + 1) * W)
            busy[w] += b - a
            a = b
    runs, cur = [], []
    for w in range(min(busy), max(busy) + 1):
        if busy.get(w, 0) / W >= low:
            cur.append(w)
        elif cur:
            runs.append(cur)
            cur = []
    if cur:
        runs.append(cur)
    main_run = max(runs, key=len)
    inside = [busy.get(w, 0) / W for w in main_run]
    print(f"{len(rows)} kernels; longest busy run {main_run[0] * win_ms:.0f}-{(main_run[-1] + 1) * win_ms:.0f} ms "
          f"({len(main_run) * win_ms:.0f} ms); kernel-time per {win_ms:g} ms window inside it: "
          f"min {min(inside):.2f}, mean {sum(inside) / len(inside):.2f}")
    gaps = [(w * win_ms, round(busy.get(w, 0) / W, 2)) for w in main_run if busy.get(w, 0) / W < 2.2]
    print("windows below 2.2:", gaps if gaps else "none")


if __name__ == "__main__":
    main(sys.argv[1])

#!/usr/bin/env python3
"""Held clock per kernel from rocprofv3 --pmc passes that include
GRBM_GUI_ACTIVE: clock = GRBM_GUI_ACTIVE / 8 (rocprofv3 sums the 8 XCDs) /
dispatch wall time (MI355X_MICROARCH.md "DVFS give-back"; the quotient reads
high on dispatches shorter than ~0.3 ms). Also the VALU issue fraction against
2.4 GHz and against the held clock. Usage: pmc_clock.py <dir> [<dir> ...]
(one table per pass; e.g. one proof at a time, then 3 proofs in flight)."""
import csv
import glob
import os
import re
import sys
from collections import defaultdict

PEAK_CLK = 2.4e9
SIMDS = 1024


def short(n):
    m = re.search(r"sezkp::(k_[A-Za-z0-9_]+)(<[^(]*>)?", n)
    return (m.group(1) + (m.group(2) or "")) if m else n.split("(")[0]


def table(d):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    per = defaultdict(lambda: defaultdict(dict))
    for f in files:
        for r in csv.DictReader(open(f, newline="")):
            k = short(r["Kernel_Name"])
            did = r["Dispatch_Id"]
            per[k][did][r["Counter_Name"]] = float(r["Counter_Value"])
            per[k][did]["_ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    rows = []
    for k, ds in per.items():
        clk, fr, frh, ns = [], [], [], []
        for c in ds.values():
            t = c["_ns"] * 1e-9
            if t <= 0 or "GRBM_GUI_ACTIVE" not in c:
                continue
            hz = c["GRBM_GUI_ACTIVE"] / 8 / t
            vi = c.get("SQ_INSTS_VALU", 0.0)
            clk.append(hz)
            fr.append(vi * 2 / (SIMDS * PEAK_CLK) / t)
            frh.append(vi * 2 / (SIMDS * hz) / t)
            ns.append(c["_ns"])
        if not clk:
            continue
        med = lambda v: sorted(v)[len(v) // 2]
        rows.append((med(ns) * len(ns), k, len(ns), med(ns) / 1e6, med(clk) / 1e9, med(fr), med(frh)))
    rows.sort(reverse=True)
    return rows


def main():
    for d in sys.argv[1:]:
        print(f"# {d}: per kernel, medians over its dispatches")
        print(f"{'kernel':46s} {'n':>4s} {'ms':>8s} {'clock_GHz':>9s} {'valu_frac@2.4':>13s} {'valu_frac@held':>14s}")
        for _, k, n, ms, ghz, fr, frh in table(d):
            print(f"{k[:46]:46s} {n:4d} {ms:8.4f} {ghz:9.3f} {fr:13.3f} {frh:14.3f}")
        print()


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Summary of tools/dict_cap_ab.sh: per table cap and round, the per-proof
device time of the dictionary kernels (rocprofv3, single-proof pass), the
single-proof ms, the col_commit stage and the in-flight bench value.
Usage: dict_cap_report.py [dir]."""
import csv
import glob
import json
import os
import re
import sys

D = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/dictcap"
KS = ("k_col_commit_dict", "k_dict_level", "k_dict_range", "k_dict_plan", "k_col_open")
runs = sorted({(int(m.group(1)), int(m.group(2))) for m in
               (re.match(r"c(\d+)_(\d+)$", os.path.basename(p)) for p in glob.glob(os.path.join(D, "c*_*"))) if m},
              key=lambda t: (t[1], -t[0]))
for cap, rep in runs:
    f = glob.glob(os.path.join(D, f"c{cap}_{rep}", "*kernel_stats.csv"))
    if not f:
        continue
    tot, calls = {}, {}
    for r in csv.DictReader(open(f[0])):
        m = re.search(r"sezkp::(k_[A-Za-z0-9_]+)", r["Name"])
        if m:
            tot[m.group(1)] = tot.get(m.group(1), 0) + float(r["TotalDurationNs"]) / 1e3
            calls[m.group(1)] = calls.get(m.group(1), 0) + int(r["Calls"])
    proofs = max(1, calls.get("k_col_commit_dict", 1))
    ks = "  ".join(f"{k} {tot.get(k, 0) / proofs:6.1f}" for k in KS)
    try:
        d1 = json.load(open(os.path.join(D, f"c{cap}_{rep}_if1.json")))
        ln = open(os.path.join(D, f"c{cap}_{rep}_bench.log")).read().strip().splitlines()[-1]
        v = json.loads(ln)["value"]
    except (OSError, ValueError, IndexError):
        continue
    print(f"cap {cap:6d} run {rep}: {ks} us/proof | one proof {d1['single_proof']['ms_per_proof']:.4f} ms "
          f"(under rocprofv3), col_commit {d1['stages_ms']['col_commit']:.4f} ms | in flight {v / 1e9:.3f}e9")

#!/usr/bin/env python3
"""Summary of tools/lib_ab.sh: per arm and round, the single-proof kernel
averages of the main kernels (rocprofv3), the single-proof ms, the col_commit
stage and the in-flight bench value. Usage: lib_ab_report.py [dir]."""
import csv
import glob
import json
import os
import re
import sys

D = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/libab"
KS = ("k_col_commit_dict", "k_forest16", "k_layer16", "k_dict_level")
for rep in (1, 2):
    for arm in ("main", "alt"):
        f = glob.glob(os.path.join(D, f"{arm}{rep}", "*kernel_stats.csv"))
        if not f:
            continue
        avg = {}
        for r in csv.DictReader(open(f[0])):
            m = re.search(r"sezkp::(k_[A-Za-z0-9_]+)(<[^(]*>)?", r["Name"])
            if m:  # template instances summed per kernel name (one instance runs per shape)
                avg[m.group(1)] = avg.get(m.group(1), 0) + float(r["TotalDurationNs"]) / 1e3 / max(1, int(r["Calls"]))
        d1 = json.load(open(os.path.join(D, f"{arm}{rep}_if1.json")))
        ln = open(os.path.join(D, f"{arm}{rep}_bench.log")).read().strip().splitlines()[-1]
        v = json.loads(ln)["value"]
        ks = "  ".join(f"{k} {avg.get(k, 0):6.1f}" for k in KS)
        print(f"{arm:4s} run {rep}: {ks} us | one proof {d1['single_proof']['ms_per_proof']:.4f} ms "
              f"(under rocprofv3), col_commit {d1['stages_ms']['col_commit']:.4f} ms | in flight {v / 1e9:.3f}e9")

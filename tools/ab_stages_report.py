#!/usr/bin/env python3
"""Report of tools/ab_stages.sh: per arm, round and P, the median proof wall
time and the stage times (ms). Usage: ab_stages_report.py <dir>"""
import json
import os
import sys

D = sys.argv[1]
KEYS = ("col_commit", "col_outer", "compose", "intt", "lde_ntt", "deep", "layer0_tree", "layer0_upper",
        "fri_fold_trees", "col_openings", "fri_paths", "total")
for P in (1, 8):
    print(f"P = {P}: " + " ".join(f"{k[:10]:>10s}" for k in ("wall",) + KEYS))
    for rep in (1, 2):
        for arm in ("main", "alt"):
            f = os.path.join(D, f"{arm}{rep}_p{P}.json")
            if not os.path.exists(f):
                continue
            d = json.loads(open(f).read().strip().splitlines()[-1])
            w = sorted(d["wall_ms"])[len(d["wall_ms"]) // 2]
            st = d["stages_ms"]
            print(f"  {arm}{rep}: " + " ".join(f"{v:10.4f}" for v in [w] + [st.get(k, 0.0) for k in KEYS]))

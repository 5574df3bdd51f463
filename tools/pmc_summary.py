#!/usr/bin/env python3
"""Per-kernel HBM traffic from two rocprofv3 PMC runs (FETCH_SIZE and
WRITE_SIZE cannot share one pass on gfx950), plus the wave64 VALU
instruction count per launch from a third (SQ_INSTS_VALU).

    rocprofv3 --pmc FETCH_SIZE --output-format csv -d <F> -o run -- python3 bench.py ...
    rocprofv3 --pmc WRITE_SIZE --output-format csv -d <W> -o run -- python3 bench.py ...
    rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES ... -d <V> -o run -- python3 bench.py ...
    python3 tools/pmc_summary.py <F> <W> [<V>] > profiles/pmc_summary.json

FETCH_SIZE / WRITE_SIZE are in KB. Per MI355X_MICROARCH.md (HBM section),
gfx950 FETCH_SIZE reports half the bytes of wide coalesced streaming reads,
so hbm_bytes_per_launch = 2 * fetch + write (the dominant kernels here load
16 B per lane).
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def _short(name: str) -> str:
    """kernel name with its template arguments (k_ntt4<...> instances differ)"""
    m = re.search(r"sezkp::(k_[A-Za-z0-9_]+)(<[^(]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name.split("(")[0]


def _load(d: str, counter: str) -> dict:
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    per = defaultdict(list)
    for f in files:
        with open(f, newline="") as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                per[_short(row["Kernel_Name"])].append(float(row["Counter_Value"]) * 1024.0)
    return per


def main():
    fdir, wdir = sys.argv[1], sys.argv[2]
    fetch, write = _load(fdir, "FETCH_SIZE"), _load(wdir, "WRITE_SIZE")
    valu = _load(sys.argv[3], "SQ_INSTS_VALU") if len(sys.argv) > 3 else {}
    out = {}
    for k in sorted(set(fetch) | set(write) | set(valu)):
        f = sum(fetch[k]) / len(fetch[k]) if fetch.get(k) else None
        w = sum(write[k]) / len(write[k]) if write.get(k) else None
        out[k] = {"launches": max(len(fetch.get(k, [])), len(write.get(k, []))),
                  "fetch_size_bytes_per_launch": f, "write_size_bytes_per_launch": w,
                  "hbm_bytes_per_launch": (2 * f + w) if f is not None and w is not None else None,
                  "correction": "fetch x2 (gfx950 wide-read undercount)"}
        if valu.get(k):  # _load scales by 1024 (KB counters); SQ_INSTS_VALU is a plain count
            out[k]["valu_instr_per_launch"] = sum(valu[k]) / len(valu[k]) / 1024.0
    json.dump(out, sys.stdout, indent=1, sort_keys=True)
    print()


if __name__ == "__main__":
    main()

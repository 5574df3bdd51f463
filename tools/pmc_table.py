#!/usr/bin/env python3
"""Per-kernel table of every counter in one or more rocprofv3 --pmc passes
(counter_collection.csv files): the median kernel duration and each
counter's mean per dispatch; SQ_* cycle counters (quad-cycles) also as a
fraction of SQ_WAVE_CYCLES. Usage: pmc_table.py csv [csv ...] [--match sub]."""
import csv
import re
import sys
from collections import defaultdict


def short(n):
    m = re.search(r"sezkp::(k_[A-Za-z0-9_]+)(<[^(]*>)?", n)
    return (m.group(1) + (m.group(2) or "")) if m else n.split("(")[0][:40]


def main(argv):
    match = None
    if "--match" in argv:
        i = argv.index("--match")
        match = argv[i + 1]
        argv = argv[:i] + argv[i + 2:]
    per = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(list)
    for path in argv:
        seen = set()
        for r in csv.DictReader(open(path)):
            k = short(r["Kernel_Name"])
            if match and match not in k:
                continue
            per[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            key = (path, r["Dispatch_Id"])
            if key not in seen:
                seen.add(key)
                dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for k in sorted(per, key=lambda k: -sum(dur[k])):
        d = sorted(dur[k])
        avg = {n: sum(v) / len(v) for n, v in per[k].items()}
        wc = avg.get("SQ_WAVE_CYCLES")
        print(f"{k}  dispatches {len(d)}  median {d[len(d) // 2]:.2f} us")
        for n in sorted(avg):
            extra = f"  ({avg[n] / wc:.3f} of SQ_WAVE_CYCLES)" if wc and n.startswith(("SQ_WAIT", "SQ_ACTIVE", "SQ_BUSY")) else ""
            w = avg.get("SQ_WAVES")
            perw = f"  per wave {avg[n] / w:.1f}" if w and n.startswith("SQ_INSTS") else ""
            print(f"    {n:28s} {avg[n]:16.1f}{extra}{perw}")


if __name__ == "__main__":
    main(sys.argv[1:])

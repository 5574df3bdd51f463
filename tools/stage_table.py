#!/usr/bin/env python3
"""DESIGN.md §6's per-rank stage table from a bench detail file: the one-GPU
proof's stages and, per P, the slowest rank of the sharded cost model.
Usage: stage_table.py <bench_detail.json>"""
import json
import sys

d = json.load(open(sys.argv[1]))
one = d.get("stages_ms", {})
sp = d["sharded_predicted"]
KEYS = ["expand", "col_commit", "col_outer", "compose", "intt", "lde_ntt", "deep", "layer0_tree", "layer0_upper",
        "fri_fold_trees", "col_openings", "fri_paths", "total"]
Ps = sorted(sp["by_gpus"], key=int)
slow = {P: max(sp["by_gpus"][P]["ranks"], key=lambda r: r["predicted_ms"]) for P in Ps}
print("| stage | 1 GPU | " + " | ".join(f"P = {P}" for P in Ps) + " |")
print("|---|---|" + "---|" * len(Ps))
for k in KEYS:
    print(f"| `{k}` | {one.get(k, float('nan')):.3f} | " + " | ".join(f"{slow[P]['stages_ms'].get(k, float('nan')):.3f}" for P in Ps) + " |")
print("| solo wall − solo collectives | — | " + " | ".join(f"{slow[P]['solo_wall_ms'] - slow[P]['solo_collective_ms']:.3f}" for P in Ps) + " |")
print("| modelled collectives (count) | — | " + " | ".join(f"{slow[P]['model_collective_ms']:.3f} ({slow[P]['collectives']})" for P in Ps) + " |")
print(f"| **predicted** (speedup) | {sp['single_gpu_ms_per_proof']:.3f} | " + " | ".join(
    f"**{sp['by_gpus'][P]['predicted_ms_per_proof']:.3f}** ({sp['by_gpus'][P]['predicted_speedup']:.2f}×)" for P in Ps) + " |")

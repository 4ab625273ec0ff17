"""Merge per-workload GEMM layout dumps (scripts/gpu/make_layout_table.sh) into the shipped table.

    python scripts/merge_layout_tables.py gpurun_out/layouts_*.json
"""
import json
import os
import sys

OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "llm_training_amd", "tuning",
                   "gemm_layouts_gfx950.json")


def main(paths):
    merged = {}
    for p in paths:
        with open(p) as f:
            for k, v in json.load(f)["layouts"].items():
                if merged.get(k, v) != v:
                    print(f"{k}: {merged[k]} ({p} says {v}); keeping the first", file=sys.stderr)
                merged.setdefault(k, v)
    doc = {"about": "GEMM layout choices (ops/fused.py _layout) per problem key "
                    "kind|M|N|K|ld...|dtype|streamK, timed on one MI355X by scripts/gpu/make_layout_table.sh",
           "layouts": dict(sorted(merged.items()))}
    with open(OUT, "w") as f:
        json.dump(doc, f, indent=1)
    print(f"{len(merged)} layouts -> {OUT}")


if __name__ == "__main__":
    main(sys.argv[1:])

#!/usr/bin/env python3
"""Merge the per-kernel JSON passes of ``scripts/gpu/r6_step_pmc.sh`` into one markdown table.

    python scripts/pmc_step_table.py gpurun_out/step_pmc_1.json gpurun_out/step_pmc_2.json \
        gpurun_out/step_pmc_3.json [--top 25]

Derived columns (per kernel, summed over its dispatches):
* clock = GRBM_GUI_ACTIVE / 8 XCDs / duration;
* MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / 1024 SIMDs / (GRBM_GUI_ACTIVE / 8), the share of the kernel's cycles
  in which the average SIMD's matrix core was busy;
* L2 fetch / write = FETCH_SIZE / WRITE_SIZE (KiB, the L2 <-> fabric traffic) over the duration of that pass.
"""
from __future__ import annotations

import argparse
import json
import re

FAMILIES = [
    ("hipBLASLt GEMMs", r"^Cijk_|^Custom_Cijk_"),
    ("own GEMM / split-K reduce", r"gemm_pp|splitk_reduce"),
    ("attention forward", r"fa_fwd"),
    ("attention dQ", r"fa_bwd_dq"),
    ("attention dK/dV", r"fa_bwd_dkdv"),
    ("SwiGLU", r"swiglu"),
    ("RMSNorm", r"rmsnorm"),
    ("transpose", r"transpose"),
    ("AdamW + grad norm", r"adamw|sumsq|sum_partials"),
    ("cross-entropy", r"ce_kernel|lse|logp"),
    ("RoPE", r"rope"),
]


def family(name: str) -> str:
    for fam, rx in FAMILIES:
        if re.search(rx, name):
            return fam
    return "other"


def derived(p1: dict, p2: dict | None, p3: dict | None) -> dict:
    c = p1["counters"]
    dur = p1["dur_ns"]
    gui = c.get("GRBM_GUI_ACTIVE", 0.0)
    out = {"ms": dur / 1e6, "n": p1["dispatches"]}
    if gui and dur:
        out["ghz"] = gui / 8 / dur
        if "SQ_VALU_MFMA_BUSY_CYCLES" in c:
            out["mfma"] = c["SQ_VALU_MFMA_BUSY_CYCLES"] / 1024 / (gui / 8)
    w = c.get("SQ_WAVE_CYCLES")
    if w:
        out["issue"] = c.get("SQ_ACTIVE_INST_ANY", 0.0) / w
        out["wait_inst"] = c.get("SQ_WAIT_INST_ANY", 0.0) / w
    for key, p, cn in (("fetch", p2, "FETCH_SIZE"), ("write", p3, "WRITE_SIZE")):
        if p and p["dur_ns"] and cn in p["counters"]:
            out[key] = p["counters"][cn] * 1024 / p["dur_ns"] / 1e3  # TB/s
    return out


def merge(ps: list[dict]) -> dict:
    """Sum kernel entries (dispatches, durations, counters) into one."""
    out = {"dispatches": 0, "dur_ns": 0.0, "counters": {}}
    for p in ps:
        out["dispatches"] += p["dispatches"]
        out["dur_ns"] += p["dur_ns"]
        for k, v in p["counters"].items():
            out["counters"][k] = out["counters"].get(k, 0.0) + v
    return out


def fmt(d: dict, k: str, spec: str) -> str:
    return format(d[k], spec) if k in d else "-"


def row(label: str, d: dict, total_ms: float) -> str:
    return (f"| {label} | {d['n']} | {d['ms']:.1f} | {100 * d['ms'] / total_ms:.1f} % | {fmt(d, 'ghz', '.2f')} | "
            f"{fmt(d, 'mfma', '.0%')} | {fmt(d, 'issue', '.2f')} | {fmt(d, 'fetch', '.2f')} | {fmt(d, 'write', '.2f')} |")


HEAD = ("| {} | dispatches | ms (profiled) | share | clock GHz | MFMA busy | issue / wave cycles | "
        "L2 fetch TB/s | L2 write TB/s |\n|---|---|---|---|---|---|---|---|---|")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("passes", nargs=3)
    ap.add_argument("--top", type=int, default=25)
    args = ap.parse_args()
    p1, p2, p3 = (json.load(open(f)) for f in args.passes)
    total = sum(v["dur_ns"] for v in p1.values()) / 1e6
    fams: dict[str, list[str]] = {}
    for k in p1:
        fams.setdefault(family(k), []).append(k)
    print(HEAD.format("family"))
    rows = []
    for fam, ks in fams.items():
        d = derived(merge([p1[k] for k in ks]), merge([p2[k] for k in ks if k in p2]) if p2 else None,
                    merge([p3[k] for k in ks if k in p3]) if p3 else None)
        rows.append((d["ms"], row(fam, d, total)))
    for _, r in sorted(rows, reverse=True):
        print(r)
    print()
    print(HEAD.format("kernel"))
    for k in sorted(p1, key=lambda k: -p1[k]["dur_ns"])[:args.top]:
        name = k if len(k) <= 90 else k[:87] + "..."
        print(row(f"`{name}`", derived(p1[k], p2.get(k), p3.get(k)), total))


if __name__ == "__main__":
    main()

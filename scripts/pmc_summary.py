#!/usr/bin/env python3
"""Per-kernel PMC counter summary of a rocprofv3 ``--pmc`` database (rocpd SQLite).

    python scripts/pmc_summary.py gpurun_out/<dir>/run_results.db [--match REGEX] [--last N]

For every kernel whose name matches: the mean over its dispatches (the last N when given) of each
collected counter, plus derived ratios when the SQ counters are present (issue / wait shares of
SQ_WAVE_CYCLES, MFMA busy per SIMD as a share of the kernel's cycles at the measured duration).
"""
from __future__ import annotations

import argparse
import collections
import re
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--match", default=".")
    ap.add_argument("--last", type=int, default=0)
    args = ap.parse_args()
    db = sqlite3.connect(args.db)
    rows = db.execute("select dispatch_id, name, duration, counter_name, counter_value from pmc_events").fetchall()
    per = collections.defaultdict(lambda: collections.defaultdict(dict))  # kernel -> dispatch -> counter
    dur = {}
    for did, name, d, cn, cv in rows:
        if not re.search(args.match, name or ""):
            continue
        k = re.sub(r"\(.*\)$", "", name)
        per[k][did][cn] = per[k][did].get(cn, 0.0) + float(cv)
        dur[(k, did)] = float(d)
    for k, ds in per.items():
        ids = sorted(ds)[-args.last:] if args.last else sorted(ds)
        mean = collections.defaultdict(float)
        for i in ids:
            for cn, v in ds[i].items():
                mean[cn] += v / len(ids)
        ms = sum(dur[(k, i)] for i in ids) / len(ids) / 1e6
        print(f"## {k[:120]}\n  dispatches {len(ids)}, mean duration {ms:.4f} ms")
        for cn in sorted(mean):
            print(f"  {cn:32s} {mean[cn]:.4g}")
        w = mean.get("SQ_WAVE_CYCLES")
        if w:
            for cn in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_LDS"):
                if cn in mean:
                    print(f"  {cn + ' / WAVE_CYCLES':32s} {mean[cn] / w:.3f}")
        if "SQ_BUSY_CYCLES" in mean and "SQ_VALU_MFMA_BUSY_CYCLES" in mean:
            print(f"  {'MFMA_BUSY / (BUSY_CYCLES*4)':32s} {mean['SQ_VALU_MFMA_BUSY_CYCLES'] / (4 * mean['SQ_BUSY_CYCLES']):.3f}")


if __name__ == "__main__":
    main()

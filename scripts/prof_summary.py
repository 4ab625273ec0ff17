#!/usr/bin/env python3
"""Summarise a rocprofv3 ``--kernel-trace`` database (rocpd SQLite) as a markdown kernel table.

    python scripts/prof_summary.py gpurun_out/<dir>/run_results.db [--steps N] [--top 30] > profiles/x.md

Groups dispatches by kernel name: calls, total / mean time, share of GPU kernel time, and the
per-step time when ``--steps`` (the number of profiled training steps, warm-up included) is given.
Also reports the registers / LDS of each kernel (from the code-object symbol table).
"""
from __future__ import annotations

import argparse
import re
import sqlite3


def _short(name: str, width: int = 90) -> str:
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"\(.*\)$", "", name)  # drop argument lists
    return name if len(name) <= width else name[: width - 3] + "..."


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--steps", type=int, default=0)
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--tail-ms", type=float, default=0.0,
                    help="only dispatches that start in the last X ms of the trace (steady-state steps; "
                         "skips warm-up, GEMM solution timing and start-up kernels)")
    ap.add_argument("--bench-log", default=None,
                    help="bench.py output of the profiled run: its JSON line sets --steps and --tail-ms "
                         "(the timed steps only)")
    args = ap.parse_args()
    if args.bench_log:
        import json
        for line in open(args.bench_log):
            if line.startswith('{"metric"'):
                r = json.loads(line)
                args.steps = int(r["steps"])
                args.tail_ms = float(r["ms_per_step"]) * args.steps
    c = sqlite3.connect(args.db)
    span = c.execute("select min(start), max(end) from rocpd_kernel_dispatch").fetchone()
    t0 = span[1] - int(args.tail_ms * 1e6) if args.tail_ms else span[0]
    rows = c.execute(
        "select s.display_name, count(*), sum(d.end - d.start), s.arch_vgpr_count, s.accum_vgpr_count, "
        "s.group_segment_size from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id "
        "where d.start >= ? group by s.display_name order by sum(d.end - d.start) desc", (t0,)).fetchall()
    span = (t0, span[1])
    total = sum(r[2] for r in rows)
    print(f"GPU kernel time {total / 1e6:.1f} ms over a {(span[1] - span[0]) / 1e6:.1f} ms trace "
          f"({len(rows)} distinct kernels)\n")
    hdr = "| kernel | calls | total ms | mean us | share |"
    if args.steps:
        hdr += " ms/step |"
    print(hdr + " vgpr/agpr | LDS B |")
    print("|" + "---|" * (hdr.count("|") + 1))
    for name, n, t, vg, ag, lds in rows[: args.top]:
        line = f"| `{_short(name)}` | {n} | {t / 1e6:.2f} | {t / n / 1e3:.1f} | {100 * t / total:.1f}% |"
        if args.steps:
            line += f" {t / 1e6 / args.steps:.2f} |"
        print(line + f" {vg}/{ag} | {lds} |")


if __name__ == "__main__":
    main()

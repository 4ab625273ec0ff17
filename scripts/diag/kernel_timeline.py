#!/usr/bin/env python3
"""Per-dispatch durations of the kernels matching a pattern over the last N ms of a rocprofv3
--kernel-trace database (rocpd SQLite), in launch order, with the count of other kernels that overlapped
each one in time (concurrent streams).   python scripts/diag/kernel_timeline.py <db> <regex> [--tail-ms X]"""
import argparse
import re
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("pattern")
    ap.add_argument("--tail-ms", type=float, default=1500.0)
    a = ap.parse_args()
    db = sqlite3.connect(a.db)
    tabs = [r[0] for r in db.execute("select name from sqlite_master where type in ('table','view')")]
    view = "kernels" if "kernels" in tabs else next(t for t in tabs if t.startswith("rocpd_kernel_dispatch"))
    cols = [r[1] for r in db.execute(f"pragma table_info({view})")]
    name_col = "name" if "name" in cols else "kernel_name"
    rows = db.execute(f"select {name_col}, start, end from {view} order by start").fetchall()
    t_end = max(r[2] for r in rows)
    rows = [r for r in rows if r[1] >= t_end - a.tail_ms * 1e6]
    pat = re.compile(a.pattern)
    for i, (n, s, e) in enumerate(rows):
        if not pat.search(n or ""):
            continue
        over = sum(1 for (n2, s2, e2) in rows if s2 < e and e2 > s and (s2, e2) != (s, e))
        print(f"{(s - rows[0][1]) / 1e6:9.2f} ms  {(e - s) / 1e3:8.1f} us  overlapping {over:3d}  {re.sub(r'[(].*', '', n)[:60]}")


if __name__ == "__main__":
    main()

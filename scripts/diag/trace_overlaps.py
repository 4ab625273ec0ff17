#!/usr/bin/env python3
"""Print what overlaps the N longest kernel dispatches of a rocprofv3 rocpd database: host API regions,
memory copies and other kernels (for diagnosing a stalled kernel), plus the table inventory.

    python scripts/diag/trace_overlaps.py <run_results.db> [N]
"""
import sqlite3
import sys


def main():
    db, n = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 3
    c = sqlite3.connect(db)
    tables = [r[0] for r in c.execute("select name from sqlite_master where type in ('table','view')")]
    print("tables:", tables)
    ks = c.execute("select s.display_name, d.start, d.end, d.stream_id from rocpd_kernel_dispatch d join "
                   "rocpd_info_kernel_symbol s on d.kernel_id = s.id order by (d.end - d.start) desc limit ?",
                   (n,)).fetchall()
    t0 = c.execute("select min(start) from rocpd_kernel_dispatch").fetchone()[0]
    for name, s, e, st in ks:
        print(f"\n=== kernel {name[:80]} stream {st} at {(s - t0) / 1e6:.1f} ms, {(e - s) / 1e6:.2f} ms")
        for t in tables:
            cols = [r[1] for r in c.execute(f"pragma table_info({t})")]
            if "start" not in cols or "end" not in cols or t == "rocpd_kernel_dispatch":
                continue
            namecol = next((x for x in ("name", "display_name", "region_name", "category") if x in cols), None)
            try:
                q = f"select {namecol or 'rowid'}, start, end from {t} where start < ? and end > ? and (end - start) > 2e5"
                rows = c.execute(q, (e, s)).fetchall()
            except sqlite3.Error:
                continue
            if rows:
                print(f"  {t}: {len(rows)} overlapping records > 0.2 ms")
                for r in sorted(rows, key=lambda r: r[2] - r[1], reverse=True)[:12]:
                    print(f"    {str(r[0])[:70]:70s} start {(r[1] - t0) / 1e6:10.1f} ms  dur {(r[2] - r[1]) / 1e6:9.2f} ms")


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Host-side HIP API time and GPU idle gaps of a rocprofv3 --sys-trace database, over the last
``window_ms`` of the trace (steady-state steps): which API calls block the host, and how long the
GPU's compute stream sits idle.

    python scripts/diag/host_api_summary.py <run_results.db> [window_ms]
"""
import collections
import sqlite3
import sys


def main():
    db = sys.argv[1]
    win = float(sys.argv[2]) if len(sys.argv) > 2 else 4000.0
    c = sqlite3.connect(db)
    kend = c.execute("select max(end) from kernels").fetchone()[0]
    t0 = kend - int(win * 1e6)
    agg = collections.defaultdict(lambda: [0, 0.0, 0.0])
    for name, s, e in c.execute("select name, start, end from regions where start >= ?", (t0,)):
        a = agg[name]
        a[0] += 1
        a[1] += (e - s) / 1e6
        a[2] = max(a[2], (e - s) / 1e6)
    print(f"host API over the last {win:.0f} ms (calls, total ms, max ms):")
    for name, (n, tot, mx) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:20]:
        print(f"  {name:40s} {n:7d} {tot:10.1f} {mx:9.2f}")
    ks = c.execute("select start, end, stream_id, name from kernels where start >= ? order by start", (t0,)).fetchall()
    busy = 0
    cur_s = cur_e = None
    for s, e, _, _ in ks:  # union of kernel intervals over all streams
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        busy += cur_e - cur_s
    span = ks[-1][1] - ks[0][0]
    print(f"GPU busy (any stream) {busy / 1e6:.1f} ms of {span / 1e6:.1f} ms ({100 * busy / span:.1f} %)")
    gaps = []
    last = None
    for s, e, st, n in ks:
        if last is not None and s - last[0] > 5e6:
            gaps.append(((s - last[0]) / 1e6, last[1][:40], n[:40]))
        last = (max(e, last[0]) if last else e, n)
    print("idle gaps > 5 ms:", len(gaps), "total", round(sum(g[0] for g in gaps), 1), "ms")
    for g in sorted(gaps, reverse=True)[:10]:
        print(f"  {g[0]:8.1f} ms after {g[1]} before {g[2]}")


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Per-kernel sums of a rocprofv3 ``--pmc`` database (rocpd SQLite) as one JSON object, so that the
passes of a multi-pass counter collection can be brought back small and merged later
(``scripts/pmc_step_table.py``).

    python scripts/pmc_kernels_json.py gpurun_out/<dir>/run_results.db > pass.json

Output: {kernel: {"dispatches": n, "dur_ns": summed duration, "counters": {name: summed value}}}.
"""
from __future__ import annotations

import collections
import json
import re
import sqlite3
import sys


def main():
    db = sqlite3.connect(sys.argv[1])
    rows = db.execute("select dispatch_id, name, duration, counter_name, counter_value from pmc_events").fetchall()
    counters = collections.defaultdict(lambda: collections.defaultdict(float))
    dur = collections.defaultdict(dict)
    for did, name, d, cn, cv in rows:
        k = re.sub(r"\(.*\)$", "", name or "?")
        counters[k][cn] += float(cv)
        dur[k][did] = float(d)
    out = {k: {"dispatches": len(dur[k]), "dur_ns": sum(dur[k].values()), "counters": dict(counters[k])}
           for k in counters}
    json.dump(out, sys.stdout, indent=0, sort_keys=True)


if __name__ == "__main__":
    main()

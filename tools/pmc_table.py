#!/usr/bin/env python3
"""Per-kernel averages of any rocprofv3 --pmc counters over several passes.

    python tools/pmc_table.py <out.json> <pass_dir> [<pass_dir> ...]

Each pass directory holds the run_counter_collection.csv of one rocprofv3
--pmc run (one counter set per run: gfx950 cannot multiplex).  Writes, per
kernel short name, the average value per launch of every counter seen, and
for FETCH_SIZE / WRITE_SIZE (KiB) the HBM bytes per launch with the gfx950
correction of MI355X_MICROARCH.md ("HBM": FETCH_SIZE tallies 128-B requests
at 64 B, so it is doubled): traffic = 2 * FETCH_SIZE + WRITE_SIZE.
"""
import csv
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import short  # noqa: E402


def main():
    out, dirs = sys.argv[1], sys.argv[2:]
    acc = defaultdict(lambda: defaultdict(lambda: [0.0, 0]))
    for d in dirs:
        path = os.path.join(d, "run_counter_collection.csv")
        if not os.path.isfile(path):
            continue
        with open(path) as f:
            for r in csv.DictReader(f):
                a = acc[short(r["Kernel_Name"])][r["Counter_Name"]]
                a[0] += float(r["Counter_Value"])
                a[1] += 1
    res = {}
    for k, cs in sorted(acc.items()):
        row = {c: round(v / max(n, 1), 1) for c, (v, n) in sorted(cs.items())}
        row["launches"] = max(n for _, n in cs.values())
        if "FETCH_SIZE" in row or "WRITE_SIZE" in row:
            row["traffic_bytes_per_launch"] = round(1024 * (2 * row.get("FETCH_SIZE", 0.0) +
                                                            row.get("WRITE_SIZE", 0.0)))
        res[k] = row
    with open(out, "w") as f:
        json.dump({"kernels": res, "passes": dirs}, f, indent=1)
    print(json.dumps(res, indent=1)[:4000])


if __name__ == "__main__":
    main()

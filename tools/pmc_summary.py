#!/usr/bin/env python3
"""Per-kernel HBM traffic from two separate rocprofv3 --pmc passes.

    python tools/pmc_summary.py <fetch_dir> <write_dir> <out.json>

Reads run_counter_collection.csv of a FETCH_SIZE pass and of a WRITE_SIZE
pass (one pass each: the TCC block cannot hold both), and writes, per kernel
short name, the average HBM bytes per launch:

    traffic = 2 * FETCH_SIZE + WRITE_SIZE      (counters are in KiB)

The factor 2 is the gfx950 correction of MI355X_MICROARCH.md ("HBM"):
FETCH_SIZE tallies 128-B requests at 64 B.  bench.py reads the entry of its
dominant kernel into roofline.traffic.
"""
import csv
import json
import re
import sys
from collections import defaultdict


def short(name: str) -> str:
    if "rocprim" in name:
        if "onesweep_iteration" in name:
            kind = "onesweep_iteration"
        elif "onesweep_global_offsets" in name:
            kind = "onesweep_global_offsets"
        else:
            kind = "other"
        key = "u64" if "radix_sort_onesweep_config<rocprim::ROCPRIM_400200_NS::default_config, unsigned long," in name else "u32"
        return f"rocprim_{kind}_{key}"
    m = re.match(r"(?:void )?(?:\(anonymous namespace\)::)?([A-Za-z_0-9]+)", name)
    return m.group(1) if m else name[:40]


def load(d: str, counter: str):
    acc = defaultdict(lambda: [0.0, 0])
    with open(f"{d}/run_counter_collection.csv") as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] != counter:
                continue
            a = acc[short(r["Kernel_Name"])]
            a[0] += float(r["Counter_Value"]) * 1024.0
            a[1] += 1
    return acc


def main():
    fdir, wdir, out = sys.argv[1:4]
    fe = load(fdir, "FETCH_SIZE")
    wr = load(wdir, "WRITE_SIZE")
    res = {}
    for k in sorted(set(fe) | set(wr)):
        fb, fn = fe.get(k, [0.0, 0])
        wb, wn = wr.get(k, [0.0, 0])
        n = max(fn, wn, 1)
        res[k] = {"launches": n, "fetch_bytes_per_launch": round(2 * fb / max(fn, 1)),
                  "write_bytes_per_launch": round(wb / max(wn, 1)),
                  "traffic_bytes_per_launch": round(2 * fb / max(fn, 1) + wb / max(wn, 1))}
    meta = {"formula": "2*FETCH_SIZE + WRITE_SIZE (KiB -> B), gfx950 FETCH_SIZE x2 correction",
            "source": [fdir, wdir]}
    with open(out, "w") as f:
        json.dump({"meta": meta, "kernels": res}, f, indent=1, sort_keys=True)
    for k, v in sorted(res.items(), key=lambda kv: -kv[1]["traffic_bytes_per_launch"] * kv[1]["launches"])[:20]:
        print(f"{k:36s} n={v['launches']:4d} traffic/launch={v['traffic_bytes_per_launch'] / 1e6:10.2f} MB")


if __name__ == "__main__":
    main()

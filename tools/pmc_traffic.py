#!/usr/bin/env python3
"""Summarise a tools/profile.sh run: average duration and HBM bytes per launch of the dominant
kernel (the fused Viterbi step kernel), from rocprofv3 CSV output.

gfx950 corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE and WRITE_SIZE are in KiB;
FETCH_SIZE reads half the bytes of a wide coalesced read, so it is doubled; WRITE_SIZE is taken
as is.  Only dispatches of the dominant kernel are averaged.
"""
from __future__ import annotations

import csv
import glob
import json
import os
import sys


def rows(pattern):
    out = []
    for f in glob.glob(pattern, recursive=True):
        with open(f) as fh:
            out.extend(csv.DictReader(fh))
    return out


def main(d):
    trace = rows(os.path.join(d, "trace", "**", "*kernel_trace.csv"))
    if not trace:
        raise SystemExit(f"no kernel_trace.csv under {d}/trace")
    per = {}
    for r in trace:
        name = r["Kernel_Name"]
        dur = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        per.setdefault(name, []).append(dur)
    dom = max(per, key=lambda k: sum(per[k]))
    durs = per[dom]
    res = {"kernel": dom, "dispatches": len(durs), "avg_ns": sum(durs) / len(durs)}

    def counter(sub, name):
        vals = [float(r["Counter_Value"]) for r in rows(os.path.join(d, sub, "**", "*counter_collection.csv"))
                if r.get("Counter_Name") == name and r.get("Kernel_Name") == dom]
        return sum(vals) / len(vals) if vals else None

    fetch_kib = counter("fetch", "FETCH_SIZE")
    write_kib = counter("write", "WRITE_SIZE")
    res["fetch_size_kib_per_launch"] = fetch_kib
    res["write_size_kib_per_launch"] = write_kib
    if fetch_kib is not None and write_kib is not None:
        res["hbm_read_bytes_per_launch"] = 2.0 * fetch_kib * 1024.0
        res["hbm_write_bytes_per_launch"] = write_kib * 1024.0
        res["hbm_bytes_per_launch"] = res["hbm_read_bytes_per_launch"] + res["hbm_write_bytes_per_launch"]
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])

#!/usr/bin/env python3
"""Reduce one tools/sq_profile.sh workload directory to per-launch figures of the dominant kernel.

Counter units (MI355X_MICROARCH.md, PMC notes): SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_*
count quad-cycles (x4 = cycles); SQ_INSTS_* count wave-instructions; GRBM_GUI_ACTIVE is summed
over the 8 XCDs (÷ 8 = GPU cycles of the dispatch); FETCH_SIZE / WRITE_SIZE are KiB, FETCH_SIZE
doubled on gfx950.  Output: JSON on stdout.
"""
from __future__ import annotations

import csv
import glob
import json
import os
import sys
from collections import defaultdict


def rows(pattern):
    out = []
    for f in glob.glob(pattern, recursive=True):
        with open(f) as fh:
            out.extend(csv.DictReader(fh))
    return out


def main(d):
    trace = rows(os.path.join(d, "trace", "**", "*kernel_trace.csv"))
    per = defaultdict(list)
    for r in trace:
        per[r["Kernel_Name"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    dom = max(per, key=lambda k: sum(per[k]))
    res = {"kernel": dom, "dispatches": len(per[dom]), "avg_ns": sum(per[dom]) / len(per[dom])}
    counters = defaultdict(list)
    for sub in ("sq1", "sq2", "fetch", "write"):
        by_disp = defaultdict(lambda: defaultdict(float))
        for r in rows(os.path.join(d, sub, "**", "*counter_collection.csv")):
            if r.get("Kernel_Name") != dom:
                continue
            by_disp[r["Counter_Name"]][r.get("Dispatch_Id")] += float(r.get("Counter_Value") or 0)
        for name, disp in by_disp.items():
            counters[name] = list(disp.values())
    avg = {k: sum(v) / len(v) for k, v in counters.items() if v}
    res["counters_per_launch"] = avg
    if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
        res["hbm_bytes_per_launch"] = 2.0 * avg["FETCH_SIZE"] * 1024 + avg["WRITE_SIZE"] * 1024
    if "SQ_INSTS_VALU" in avg and "SQ_WAVES" in avg:
        res["valu_per_wave"] = avg["SQ_INSTS_VALU"] / avg["SQ_WAVES"]
    if "GRBM_GUI_ACTIVE" in avg:
        res["gpu_cycles"] = avg["GRBM_GUI_ACTIVE"] / 8.0
        res["clock_ghz_profiled"] = res["gpu_cycles"] / res["avg_ns"]
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])

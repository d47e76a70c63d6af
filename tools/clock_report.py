#!/usr/bin/env python3
"""Effective clock per kernel from a rocprofv3 --pmc GRBM_GUI_ACTIVE run (tools/clock_probe.sh):
clock = GRBM_GUI_ACTIVE / 8 XCDs / dispatch time (MI355X_MICROARCH.md, DVFS give-back)."""
import csv
import statistics
import sys
from collections import defaultdict

for d in sys.argv[1:]:
    rows = list(csv.DictReader(open(f"{d}/run_counter_collection.csv")))
    per = defaultdict(list)
    for r in rows:
        if r["Counter_Name"] != "GRBM_GUI_ACTIVE":
            continue
        ns = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        if ns < 300_000:
            continue
        name = r["Kernel_Name"].split("(")[0][-60:]
        per[name].append((float(r["Counter_Value"]) / 8 / ns, ns / 1e6))
    for k, v in per.items():
        print(f"{d}: {k}: n={len(v)} clock {statistics.median(c for c, _ in v):.3f} GHz, "
              f"{statistics.median(t for _, t in v):.3f} ms")

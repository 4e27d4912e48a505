"""Effective shader clock per kernel from a rocprofv3 --pmc pass that collected
GRBM_GUI_ACTIVE (MI355X_MICROARCH.md DVFS note: the counter is summed over the
8 XCDs, so clock = GRBM_GUI_ACTIVE / 8 / dispatch duration).

usage: python tools/pmc_clock.py <pmc dir> [kernel substring]"""
import csv
import glob
import os
import sys
from collections import defaultdict

d = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else ""
acc = defaultdict(list)
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] != "GRBM_GUI_ACTIVE" or sub not in r["Kernel_Name"]:
            continue
        ns = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        if ns > 0:
            acc[r["Kernel_Name"].split("(")[0]].append((float(r["Counter_Value"]) / 8 / ns, ns))
for k, v in acc.items():
    ghz = sorted(x[0] for x in v)
    us = sorted(x[1] / 1e3 for x in v)
    print(f"{k[:70]:70s} n={len(v)} clock GHz median {ghz[len(ghz)//2]:.3f} "
          f"(min {ghz[0]:.3f} max {ghz[-1]:.3f}) dispatch us median {us[len(us)//2]:.1f}")

"""Per-launch-size durations of one kernel from a rocprofv3 --kernel-trace CSV.

usage: python tools/trace_by_grid.py <prof dir> <kernel prefix> <out json> [label]

The --stats summary averages every dispatch of a kernel name; the config-2 search
(8 records per launch), the one-record search and the GLONASS 5-ms search share the
fp64 correlation kernel's instantiation, so its launches are split here by grid size
(workgroups x workgroup size): the 8-record config-2 launch is the largest grid.
"""
import csv
import glob
import json
import os
import statistics
import sys


def main():
    d, prefix, out = sys.argv[1], sys.argv[2], sys.argv[3]
    label = sys.argv[4] if len(sys.argv) > 4 else ""
    by = {}
    files = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    for f in files:
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].replace("(anonymous namespace)::", "")
            if name.startswith("void "):
                name = name[5:]
            if not name.startswith(prefix):
                continue
            grid = int(r["Grid_Size_X"]) * int(r.get("Grid_Size_Y", 1) or 1) * \
                int(r.get("Grid_Size_Z", 1) or 1)
            dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            by.setdefault(str(grid), {}).setdefault(name.split("(")[0], []).append(dur)
    res = {}
    for g, kinds in by.items():
        for k, v in kinds.items():
            res.setdefault(g, {})[k] = {"dispatches": len(v), "mean_us": statistics.fmean(v),
                                        "median_us": statistics.median(v), "min_us": min(v),
                                        "max_us": max(v)}
    json.dump({"kernel_prefix": prefix, "by_grid_size": res, "files": len(files),
               "source": label}, open(out, "w"), indent=1, sort_keys=True)
    for g in sorted(res, key=int):
        for k, m in res[g].items():
            print(g, k[:60], m["dispatches"], round(m["mean_us"], 1), round(m["median_us"], 1))


if __name__ == "__main__":
    main()

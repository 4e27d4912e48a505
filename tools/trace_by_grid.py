"""Per-launch-size durations of one kernel from a rocprofv3 --kernel-trace CSV.

usage: python tools/trace_by_grid.py <prof dir> <kernel prefix> <out json> [label]
                                    [--split-us T]

The --stats summary averages every dispatch of a kernel name; the config-2 search
(8 records per launch), the one-record search and the GLONASS 5-ms search share the
fp64 correlation kernel's instantiation, so its launches are split here by grid size
(workgroups x workgroup size): the 8-record config-2 launch is the largest grid.
--split-us T further splits each grid's launches at T microseconds ("<T" / ">=T"):
osg_stream_kernel runs both single calls (PCIe-inclusive lines, ~30-40 us) and
bench.py's 10-call launches (~300 us) on the same grid.
"""
import csv
import glob
import json
import os
import statistics
import sys


def main():
    args = list(sys.argv[1:])
    split = None
    if "--split-us" in args:
        i = args.index("--split-us")
        split = float(args[i + 1])
        del args[i:i + 2]
    d, prefix, out = args[0], args[1], args[2]
    label = args[3] if len(args) > 3 else ""
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
            key = str(grid)
            if split is not None:
                key += ("/<" if dur < split else "/>=") + f"{split:g}us"
            by.setdefault(key, {}).setdefault(name.split("(")[0], []).append(dur)
    res = {}
    for g, kinds in by.items():
        for k, v in kinds.items():
            res.setdefault(g, {})[k] = {"dispatches": len(v), "mean_us": statistics.fmean(v),
                                        "median_us": statistics.median(v), "min_us": min(v),
                                        "max_us": max(v)}
    json.dump({"kernel_prefix": prefix, "by_grid_size": res, "files": len(files),
               "source": label}, open(out, "w"), indent=1, sort_keys=True)
    for g in sorted(res, key=lambda g: (int(g.split("/")[0]), g)):
        for k, m in res[g].items():
            print(g, k[:60], m["dispatches"], round(m["mean_us"], 1), round(m["median_us"], 1))


if __name__ == "__main__":
    main()

"""Summarise rocprofv3 --pmc passes (tools/prof_pmc.sh) per kernel.

usage: python tools/pmc_summary.py <pmc dir> <out json> [--traffic profiles/pmc_traffic.json]
                                   [--section NAME [--runs R]]

With --section the passes profiled ONE bench section alone (tools/bench_part.py
NAME): its kernels are merged into the traffic file as "NAME/<kernel>", so
sections sharing a kernel instantiation (the fp64 search of config 2, the
GLONASS 5-ms search and the full-sky sweep) each get their own bytes per launch.
With --runs R (the section's warmup + timed runs), "NAME/_run" also records the
HBM bytes of one whole run of the section: the kernels launched at least R
times (per-run kernels, not setup), bytes per launch x launches / R.

Per kernel (name up to the first '('): the mean of every counter over its
dispatches.  HBM bytes per launch follow MI355X_MICROARCH.md "HBM [CDNA4]":
FETCH_SIZE (KiB) reports half the bytes of wide coalesced streaming reads on
gfx950, so  traffic = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "").strip()
    if name.startswith("void "):
        name = name[5:]
    return name.split("(")[0].strip()    # template kernels keep their <args>


def summarise(d):
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            acc[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    for k, cs in acc.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        m["dispatches"] = max(len(v) for v in cs.values())
        if "FETCH_SIZE" in m and "WRITE_SIZE" in m:
            m["hbm_bytes_per_launch"] = (2 * m["FETCH_SIZE"] + m["WRITE_SIZE"]) * 1024
        if "SQ_ACTIVE_INST_VALU" in m and "SQ_WAVE_CYCLES" in m and m["SQ_WAVE_CYCLES"]:
            m["valu_active_per_wave_cycle"] = m["SQ_ACTIVE_INST_VALU"] / m["SQ_WAVE_CYCLES"]
        out[k] = m
    return out


def main():
    d, o = sys.argv[1], sys.argv[2]
    s = summarise(d)
    json.dump(s, open(o, "w"), indent=1, sort_keys=True)
    if "--traffic" in sys.argv:
        t = sys.argv[sys.argv.index("--traffic") + 1]
        sec = sys.argv[sys.argv.index("--section") + 1] if "--section" in sys.argv else None
        try:   # merged into the existing file: sections not profiled this time stay
            keep = json.load(open(t))
        except (OSError, ValueError):
            keep = {}
        if sec:
            for k, m in s.items():
                if "hbm_bytes_per_launch" in m:
                    keep[f"{sec}/{k}"] = {"hbm_bytes_per_launch": m["hbm_bytes_per_launch"],
                                          "dispatches": m["dispatches"],
                                          "source": os.path.relpath(o), "instance": k}
            if "--runs" in sys.argv:
                runs = int(sys.argv[sys.argv.index("--runs") + 1])
                per = [(k, m["hbm_bytes_per_launch"] * m["dispatches"] / runs) for k, m in s.items()
                       if "hbm_bytes_per_launch" in m and m["dispatches"] >= runs]
                keep[f"{sec}/_run"] = {"hbm_bytes_per_run": sum(b for _, b in per), "runs": runs,
                                       "kernels": sorted(k for k, _ in per),
                                       "source": os.path.relpath(o)}
            json.dump(keep, open(t, "w"), indent=1, sort_keys=True)
            s = {}
        for k, m in s.items():
            base = k.split("<")[0]
            if "hbm_bytes_per_launch" in m:
                # several instantiations of one kernel: keep the hottest
                if base not in keep or m["hbm_bytes_per_launch"] > keep[base]["hbm_bytes_per_launch"]:
                    keep[base] = {"hbm_bytes_per_launch": m["hbm_bytes_per_launch"],
                                  "source": os.path.relpath(o), "instance": k}
                if k != base:   # every template instantiation under its own name too
                    keep[k] = {"hbm_bytes_per_launch": m["hbm_bytes_per_launch"],
                               "source": os.path.relpath(o), "instance": k}
        if s:
            json.dump(keep, open(t, "w"), indent=1, sort_keys=True)
    for k, m in sorted(summarise(d).items()):
        print(k, {c: round(v, 3) for c, v in m.items() if c in
                  ("FETCH_SIZE", "WRITE_SIZE", "hbm_bytes_per_launch", "dispatches",
                   "valu_active_per_wave_cycle")})


if __name__ == "__main__":
    main()

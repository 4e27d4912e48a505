# kernel trace of the config-2 acquisition step: per-kernel averages + the last steps' timeline
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/acqkt
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/acqkt -o run -- python3 tools/bench_part.py acq 50 > gpurun_out/acqkt.log 2>&1
python3 - <<PY
import csv,glob
f=glob.glob("gpurun_out/acqkt/**/*kernel_stats.csv",recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(r["Name"][:50], r["Calls"], round(float(r["AverageNs"])/1e3,2))
f=glob.glob("gpurun_out/acqkt/**/*kernel_trace.csv",recursive=True)[0]
rows=sorted(csv.DictReader(open(f)), key=lambda r:int(r["Start_Timestamp"]))
t=[(r["Kernel_Name"][:28], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows][-11:]
t0=t[0][1]
for n,s,e in t: print("%-28s %8.2f %8.2f %6.2f" % (n, (s-t0)/1e3, (e-t0)/1e3, (e-s)/1e3))
PY

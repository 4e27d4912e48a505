# Scratch session script of round 6 (the current GPU call; earlier sessions are in git history)
set -eu
O=gpurun_out/r9c
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 tools/bench_part.py acq_generic 5 > $O/kt.log 2>&1
python3 - <<PY
import csv,glob
f=glob.glob("$O/kt/*kernel_stats.csv")[0]
for r in csv.DictReader(open(f)):
    print(r["Name"][:60], r["Calls"], round(float(r["AverageNs"])/1e3,2), round(float(r["TotalDurationNs"])/1e3,1))
PY
rm -f $O/kt/*kernel_trace.csv

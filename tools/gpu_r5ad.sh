# kernel trace of the 38.192 Msps search (four-step plan)
set -eu
export TMPDIR=/tmp
mkdir -p gpurun_out/r5ad
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5ad -o run -- python3 tools/bench_part.py acq_generic 10 > gpurun_out/r5ad/prof.log 2>&1
python3 - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/r5ad/**/run_kernel_stats.csv', recursive=True)[0]
rows = list(csv.DictReader(open(f)))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:12]:
    print(r['Name'][:70], r['Calls'], round(float(r['AverageNs'])/1e3, 1), 'us avg', round(float(r['TotalDurationNs'])/1e6, 3), 'ms total')
PY

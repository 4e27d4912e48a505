# Row statistics fused into the four-step plan's last m4_rows (per-column top-2 +
# m4_stats_kernel) against the separate stats pass (GNSSCORR_ACQ_M4STATS=0):
# generic-engine parity tests, the 38.192 Msps search A/B and a kernel trace
set -eu
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_acq_generic_gpu.py > gpurun_out/r5ah_tests.log 2>&1 || { tail -40 gpurun_out/r5ah_tests.log; exit 1; }
tail -1 gpurun_out/r5ah_tests.log
for i in 1 2; do
  for M in 1 0; do
    GNSSCORR_ACQ_M4STATS=$M timeout -k 10 200 python -u tools/bench_part.py acq_generic 10 > gpurun_out/r5ah_gen_$M$i.log 2>&1
    python3 -c "
import json
d = json.loads(open('gpurun_out/r5ah_gen_$M$i.log').read().strip().split('\n')[-1])
print('M4STATS=$M run $i', 'ms per search', round(d['dt'] / d['steps'] * 1e3, 3), 'found', d['found'], '/', d['n_planted'])"
  done
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r5ah_prof -o gen --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/bench_part.py acq_generic 10 > $GRAFT_REPO_ROOT/gpurun_out/r5ah_prof.log 2>&1
f=$(find $GRAFT_REPO_ROOT/gpurun_out/r5ah_prof -name '*kernel_stats.csv' | head -1)
python3 - "$f" <<'P'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:10]:
    print(r['Name'][:70], r['Calls'], round(float(r['AverageNs']) / 1e3, 1), 'us avg', round(float(r['TotalDurationNs']) / 1e6, 3), 'ms total')
P

# 256 MiB generic work buffers (the new default): generic-engine tests and the
# 38.192 Msps search, plus the kernel trace
set -eu
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_acq_generic_gpu.py tests/test_acq_16m_gpu.py > gpurun_out/r5ap_tests.log 2>&1 || { tail -40 gpurun_out/r5ap_tests.log; exit 1; }
tail -1 gpurun_out/r5ap_tests.log
for i in 1 2; do
  timeout -k 10 200 python -u tools/bench_part.py acq_generic 10 > gpurun_out/r5ap_gen_$i.log 2>&1
  python3 -c "
import json
d = json.loads(open('gpurun_out/r5ap_gen_$i.log').read().strip().split('\n')[-1])
print('run $i', 'ms per search', round(d['dt'] / d['steps'] * 1e3, 3), 'found', d['found'], '/', d['n_planted'])"
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r5ap_prof -o gen -- python3 $GRAFT_REPO_ROOT/tools/bench_part.py acq_generic 10 > $GRAFT_REPO_ROOT/gpurun_out/r5ap_prof.log 2>&1
f=$(find $GRAFT_REPO_ROOT/gpurun_out/r5ap_prof -name '*kernel_stats.csv' | head -1)
python3 - "$f" <<'P'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:6]:
    print(r['Name'][:70], r['Calls'], round(float(r['AverageNs']) / 1e3, 1), 'us avg', round(float(r['TotalDurationNs']) / 1e6, 3), 'ms total')
P

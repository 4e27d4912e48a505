# Four-step generic-rate FFT (m4_cols / m4_rows) against the mixed-radix passes
# (GNSSCORR_ACQ_MIX4=0): generic-engine parity tests, then the 38.192 Msps search
set -eu
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_acq_generic_gpu.py > gpurun_out/r5ac_tests.log 2>&1 || { tail -40 gpurun_out/r5ac_tests.log; exit 1; }
tail -1 gpurun_out/r5ac_tests.log
for i in 1 2; do
  for M in 1 0; do
    GNSSCORR_ACQ_MIX4=$M timeout -k 10 200 python -u tools/bench_part.py acq_generic 10 > gpurun_out/r5ac_gen_$M$i.log 2>&1
    python3 -c "
import json
d = json.loads(open('gpurun_out/r5ac_gen_$M$i.log').read().strip().split('\n')[-1])
print('MIX4=$M run $i', {k: d.get(k) for k in ('dt', 'steps', 'found', 'n_planted')}, 'ms per search', round(d['dt'] / d['steps'] * 1e3, 3))"
  done
done

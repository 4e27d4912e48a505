# Four-step generic FFT at its chosen tiles: generic and compiled-plan acquisition
# tests, then the 38.192 Msps search against the mixed-radix passes
set -eu
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -q -s --timeout 200 --timeout-method thread tests/test_acq_generic_gpu.py tests/test_acq_gpu.py tests/test_acq_16m_gpu.py > gpurun_out/r5ag_tests.log 2>&1 || { tail -40 gpurun_out/r5ag_tests.log; exit 1; }
tail -1 gpurun_out/r5ag_tests.log
grep "four-step vs" gpurun_out/r5ag_tests.log || true
for i in 1 2; do
  for M in 1 0; do
    GNSSCORR_ACQ_MIX4=$M timeout -k 10 200 python -u tools/bench_part.py acq_generic 10 > gpurun_out/r5ag_gen_$M$i.log 2>&1
    python3 -c "
import json
d = json.loads(open('gpurun_out/r5ag_gen_$M$i.log').read().strip().split('\n')[-1])
print('MIX4=$M run $i', 'ms per search', round(d['dt'] / d['steps'] * 1e3, 3), 'found', d['found'], '/', d['n_planted'])"
  done
done

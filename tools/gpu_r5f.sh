set -eu
timeout -k 10 400 python -u -m pytest tests/test_acq_generic_gpu.py tests/test_acq_gpu.py -v -x --timeout 200 --timeout-method thread 2>&1 | grep -E "PASS|FAIL|Error|error|\[" | tail -40
for B in 0 1; do
  GNSSCORR_ACQ_BLUESTEIN=$B timeout -k 10 300 python3 tools/bench_part.py acq_generic 3 | python3 -c "import json,sys; d=json.loads(sys.stdin.read().splitlines()[-1]); print('bluestein=$B generic ms per search', d['dt']/d['steps']*1e3, d['found'], d['n_planted'])"
done

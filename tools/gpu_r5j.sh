set -eu
timeout -k 10 400 python -u -m pytest tests/test_fullsky_gpu.py tests/test_acq_records_gpu.py tests/test_acq_gpu.py tests/test_acq_coh_gpu.py -q -x --timeout 200 --timeout-method thread 2>&1 | tail -2
for i in 1 2; do timeout -k 10 200 python3 tools/bench_part.py fullsky 10 | python3 -c "import json,sys; d=json.loads(sys.stdin.read().splitlines()[-1]); print('fullsky ms', round(d['dt']/d['steps']*1e3,4), json.dumps(d['projection']))"; done
bash tools/gpu_r5i.sh

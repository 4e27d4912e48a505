set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q -s --timeout 200 --timeout-method thread tests/test_acq_generic_gpu.py tests/test_acq_gpu.py tests/test_acq_16m_gpu.py tests/test_acq_coh_gpu.py tests/test_fullsky_gpu.py > gpurun_out/r2f_tests.log 2>&1
echo tests ok
timeout -k 10 60 tools/acq64_stamps.bin > gpurun_out/it_stamps.txt 2>&1
timeout -k 10 200 python -u tools/bench_part.py acq 30 > gpurun_out/it_acq.log 2>&1
cat gpurun_out/it_stamps.txt
grep -o '"corr_ms": [0-9.]*' gpurun_out/it_acq.log

# acq64: parity tests for the fp64 search, then the config-2 bench section twice.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread ${ACQ_TESTS:-tests/test_acq_gpu.py tests/test_acq_records_gpu.py tests/test_acq_16m_gpu.py tests/test_fullsky_gpu.py} > gpurun_out/acq_tests.log 2>&1
tail -2 gpurun_out/acq_tests.log
for i in 1 2; do
  timeout -k 10 200 python -u tools/bench_part.py acq 40 > gpurun_out/acq_b$i.log 2>&1
  tail -1 gpurun_out/acq_b$i.log | cut -c1-200
done

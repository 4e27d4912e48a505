set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_sgt_gpu.py > gpurun_out/sgt_tests.log 2>&1
echo tests ok
timeout -k 10 200 python -u tools/bench_part.py sgt 30 > gpurun_out/sgt_b.log 2>&1
cat gpurun_out/sgt_b.log

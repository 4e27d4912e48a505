# sgt tracking: parity tests, then the bench section under each launch shape.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_sgt_gpu.py > gpurun_out/sgt_tests.log 2>&1
tail -2 gpurun_out/sgt_tests.log
for T in ${SGT_TS:-default 64 256}; do
  if [ $T = default ]; then unset GNSSCORR_SGT_THREADS; else export GNSSCORR_SGT_THREADS=$T; fi
  timeout -k 10 200 python -u tools/bench_part.py sgt 30 > gpurun_out/sgt_b_$T.log 2>&1
  echo "T=$T $(cat gpurun_out/sgt_b_$T.log)"
done

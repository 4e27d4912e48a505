# round-2 iteration: GPU tests, tracking workgroup-size sweep, tracking layouts
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu > gpurun_out/pytest_gpu.log 2>&1
echo tests ok
for cpw in 4 3 2 1; do
  GNSSCORR_TRACK_CPW=$cpw timeout -k 10 200 python -u tools/bench_part.py track 30 > gpurun_out/cpw$cpw.log 2>&1
  echo cpw $cpw ok
done
timeout -k 10 200 python -u tools/bench_part.py track 30 > gpurun_out/cpw_auto.log 2>&1
timeout -k 10 400 python -u tools/bench_part.py track_io 20 > gpurun_out/track_io.log 2>&1
echo done

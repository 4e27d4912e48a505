set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for e in "X=0" "GNSSCORR_TRACK_STAGE_IF=0"; do
  env $e timeout -k 10 120 python -u -m pytest -q --timeout 100 --timeout-method thread tests/test_track_gpu.py tests/test_packed_gpu.py > gpurun_out/dbg_$e.log 2>&1
  echo "$e ok"; tail -1 gpurun_out/dbg_$e.log
done
timeout -k 10 300 python -u tools/bench_part.py track_io 20 > gpurun_out/track_io_d.log 2>&1
timeout -k 10 200 python -u tools/bench_part.py track 30 > gpurun_out/track_d.log 2>&1

# round-4 batch 2: tracking timings of the multi-call stream kernel
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_track_gpu.py tests/test_osg_loops_gpu.py > gpurun_out/b2_trk_tests.log 2>&1 || { tail -30 gpurun_out/b2_trk_tests.log; exit 1; }
tail -1 gpurun_out/b2_trk_tests.log
for F in 1 0; do
  GNSSCORR_OSG_FUSED=$F timeout -k 10 200 python -u tools/bench_part.py track 40 > gpurun_out/b2_track_f$F.log 2>&1
  echo "fused=$F $(tail -1 gpurun_out/b2_track_f$F.log | cut -c1-300)"
done
bash tools/gpu_trk_ab.sh "cs1_int8 cs1_packed2 rx12_int8 rx12_packed2" 2 "0:1 1:1" > gpurun_out/b2_trk_ab.log 2>&1
cat gpurun_out/b2_trk_ab.log
bash tools/trk_stream_stamps.sh > gpurun_out/b2_stamps.log 2>&1
tail -30 gpurun_out/b2_stamps.log

set -eu
timeout -k 10 300 python -u -m pytest tests/test_track_gpu.py tests/test_packed_gpu.py tests/test_osg_loops_gpu.py tests/test_e2e_gpu.py -q -x --timeout 120 --timeout-method thread 2>&1 | tail -2
for C in 12288 3072; do
  echo "== channels $C"
  TRK_C=$C bash tools/gpu_trk_libab.sh "base iv0 nd0" "cs1_int8 rx12_int8 cs1_packed2 rx12_packed2" 3 0
done

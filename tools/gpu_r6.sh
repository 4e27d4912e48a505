set -eu
export TMPDIR=/tmp
O=gpurun_out/r6g; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_track_gpu.py -k "two_slot" > $O/tests_s2.log 2>&1 || { tail -40 $O/tests_s2.log; exit 1; }
tail -1 $O/tests_s2.log
GNSSCORR_TRACK_2SLOT=1 timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_track_gpu.py tests/test_packed_gpu.py tests/test_e2e_gpu.py tests/test_trackshard_gpu.py > $O/tests_forced.log 2>&1 || { tail -40 $O/tests_forced.log; exit 1; }
tail -1 $O/tests_forced.log
export TRK_C=12288
for i in 1 2 3; do
  for V in 0 1; do
    echo "cs1_int8 2slot=$V: $(GNSSCORR_TRACK_2SLOT=$V timeout -k 10 120 python3 tools/trk_layout.py cs1_int8 40)"
  done
done | tee $O/ab.log
for V in 0 1; do
  echo "rx12_int8 2slot=$V: $(GNSSCORR_TRACK_2SLOT=$V timeout -k 10 120 python3 tools/trk_layout.py rx12_int8 40)"
done | tee -a $O/ab.log

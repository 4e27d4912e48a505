# Scratch session script of round 6 (the current GPU call; earlier sessions are in git history)
set -eu
O=gpurun_out/r8v
mkdir -p $O
export TMPDIR=/tmp
for V in ch1 ch2 ch8; do
  GNSSCORR_LIB=$PWD/gnss-sdr.ru_amd/ab/libgnsscorr_$V.so timeout -k 10 300 python -u -m pytest tests/test_track_gpu.py tests/test_packed_gpu.py -q -x --timeout 120 --timeout-method thread > $O/pytest_$V.log 2>&1
  echo "$V $(tail -1 $O/pytest_$V.log)"
done
bash tools/gpu_trk_libab.sh "base ch1 ch2 ch8" "cs1_int8 rx12_int8" 3 0 | tee $O/ab.log

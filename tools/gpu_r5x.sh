# Two LDS-DMA slots per wave (int8 pieces two ahead, counted vmcnt, slot read in
# inline asm) vs one: parity on both builds, then same-box layouts at 3072 and
# 12288 channels
set -eu
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_track_gpu.py tests/test_packed_gpu.py tests/test_osg_loops_gpu.py tests/test_e2e_gpu.py -q -x --timeout 120 --timeout-method thread 2>&1 | tail -1
GNSSCORR_LIB=$PWD/gnss-sdr.ru_amd/gnsscorr/libgnsscorr_s2.so timeout -k 10 300 python -u -m pytest tests/test_track_gpu.py tests/test_packed_gpu.py tests/test_osg_loops_gpu.py tests/test_e2e_gpu.py -q -x --timeout 120 --timeout-method thread 2>&1 | tail -1
for C in 3072 12288; do
  export TRK_C=$C
  echo "== channels $C"
  bash tools/gpu_trk_libab.sh "base s2" "cs1_int8 rx12_int8" 2 0
done

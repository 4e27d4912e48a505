# Piece LDS-DMA with the nt (streaming) cache policy vs default: parity on the
# nt build, same-box C_s = 1 and receiver layouts at 12288 channels
set -eu
export TMPDIR=/tmp
GNSSCORR_LIB=$PWD/gnss-sdr.ru_amd/gnsscorr/libgnsscorr_nt.so timeout -k 10 300 python -u -m pytest tests/test_track_gpu.py tests/test_osg_loops_gpu.py -q -x --timeout 120 --timeout-method thread 2>&1 | tail -1
export TRK_C=12288
bash tools/gpu_trk_libab.sh "base nt" "cs1_int8 rx12_int8" 3 0

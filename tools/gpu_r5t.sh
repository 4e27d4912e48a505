# Packed tracking: bytes expanded through an LDS table (TRACK_X2LUT) vs the
# spread + v_perm form (libgnsscorr_nox2.so); tracking parity tests first
set -eu
export TMPDIR=/tmp
export TRK_C=12288
bash tools/gpu_trk_libab.sh "base nox2" "cs1_packed2 rx12_packed2 cs1_int8" 3 1

# Reproduce round 2's wrong sums: the "four IF loads at a time" lane loop (TRACK_LOAD4)
# with the inline-asm v_mad_i32_i24 (TRACK_ASM_MAD) vs the __mul24 form, every lane
# on the unstaged global path (GNSSCORR_TRACK_STAGE_IF=0).
set -u
export TMPDIR=/tmp GNSSCORR_TRACK_STAGE_IF=0
for n in asm mul24; do
  echo "== load4 + $n"
  GNSSCORR_LIB=$PWD/gnss-sdr.ru_amd/gnsscorr/libgnsscorr_load4_$n.so timeout -k 10 300 \
    python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_track_gpu.py tests/test_packed_gpu.py 2>&1 | tail -4
done

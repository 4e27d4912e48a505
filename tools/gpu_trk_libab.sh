# Same-box A/B of tracking builds: bash tools/gpu_trk_libab.sh "<lib names>" [layouts] [reps] [tests]
# lib name "base" = gnss-sdr.ru_amd/gnsscorr/libgnsscorr.so, else ab/libgnsscorr_<name>.so
# (tools/build_ab.sh); prints kernel ms per call (10-call launches, tools/trk_layout.py).
# tests=1 first runs the tracking parity tests on the in-tree library.
set -eu
cd ${GRAFT_REPO_ROOT:-.}
LIBS=$1
LAYOUTS=${2:-"cs1_int8 cs1_packed2 rx12_int8 rx12_packed2"}
REPS=${3:-3}
TESTS=${4:-1}
if [ "$TESTS" = 1 ]; then
  timeout -k 10 300 python -u -m pytest tests/test_track_gpu.py tests/test_packed_gpu.py \
    tests/test_osg_loops_gpu.py tests/test_e2e_gpu.py -q -x --timeout 120 --timeout-method thread 2>&1 | tail -3
fi
for L in $LAYOUTS; do
  for i in $(seq $REPS); do
    for V in $LIBS; do
      if [ $V = base ]; then unset GNSSCORR_LIB; else export GNSSCORR_LIB=$PWD/gnss-sdr.ru_amd/ab/libgnsscorr_$V.so; fi
      echo "$L $V: $(timeout -k 10 120 python3 tools/trk_layout.py $L 40)"
    done
  done
done
unset GNSSCORR_LIB

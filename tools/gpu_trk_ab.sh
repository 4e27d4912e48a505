# Same-box A/B of osg tracking launch paths: bash tools/gpu_trk_ab.sh [layouts] [reps] [variants]
# variants: GNSSCORR_TRACK_STREAM values (0: per-call workgroup kernel, 1: osg_stream_kernel);
# prints kernel ms per call.
set -e
cd ${GRAFT_REPO_ROOT:-.}
LAYOUTS=${1:-"cs1_int8 cs1_packed2 rx12_int8 rx12_packed2"}
REPS=${2:-2}
VARS=${3:-"0 1"}
for L in $LAYOUTS; do
  for i in $(seq $REPS); do
    for V in $VARS; do
      echo "$L stream=$V: $(GNSSCORR_TRACK_STREAM=$V timeout -k 10 120 python3 tools/trk_layout.py $L 40)"
    done
  done
done

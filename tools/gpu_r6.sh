# Scratch session script of round 6 (the current GPU call; earlier sessions are in git history)
set -eu
O=gpurun_out/r6j
mkdir -p $O
export TMPDIR=/tmp
bash tools/gpu_trk_libab.sh "base trkhead" "cs1_int8 rx12_int8 cs1_packed2" 3 1 | tee $O/trk_incremental_ab.log

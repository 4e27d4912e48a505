set -eu
for C in 12288 3072; do
  echo "== channels $C"
  TRK_C=$C bash tools/gpu_trk_libab.sh "base nopf" "cs1_int8 rx12_int8 cs1_packed2 rx12_packed2" 3 0
done

set -eu
for C in 3072 6144 12288; do
  for L in cs1_int8 rx12_int8 cs1_packed2; do
    echo "$(TRK_C=$C timeout -k 10 120 python3 tools/trk_layout.py $L 20)"
  done
done

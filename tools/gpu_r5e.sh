set -eu
timeout -k 10 300 python -u -m pytest tests/test_track_gpu.py tests/test_packed_gpu.py tests/test_osg_loops_gpu.py -q -x --timeout 120 --timeout-method thread 2>&1 | tail -2
for C in 3072 12288; do
  echo "== channels $C"
  TRK_C=$C bash tools/gpu_trk_libab.sh "base w4 nopf" "cs1_int8 rx12_int8 cs1_packed2" 2 0
done
for F in base nopf; do
  if [ $F = base ]; then unset GNSSCORR_LIB; else export GNSSCORR_LIB=$PWD/gnss-sdr.ru_amd/gnsscorr/libgnsscorr_$F.so; fi
  timeout -k 10 200 python -u tools/bench_part.py track 40 > gpurun_out/r5e_track_$F.log 2>&1
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/r5e_track_$F.log').read().splitlines()[-1]); print('$F track kern_ms', d['kern_ms'], 'closed-loop ms', d['cl_ms'])"
done

# Same-box A/B of the aligned-piece path (TRACK_ALIGNED) at 12288 channels, with the
# tracking parity tests first and the C_s = 1 layout probe (stream- vs call-major IF)
set -eu
timeout -k 10 200 python -u -m pytest tests/test_track_gpu.py -q -x --timeout 120 --timeout-method thread -k batched 2>&1 | tail -2
bash tools/gpu_trk_libab.sh "base noal" "cs1_int8 rx12_int8 cs1_packed2 rx12_packed2" 3 1
echo "== main line and closed loop (tools/bench_part.py track)"
for V in base noal base noal; do
  if [ $V = base ]; then unset GNSSCORR_LIB; else export GNSSCORR_LIB=$PWD/gnss-sdr.ru_amd/gnsscorr/libgnsscorr_$V.so; fi
  timeout -k 10 200 python -u tools/bench_part.py track 40 > gpurun_out/r5n_track_$V.log 2>&1
  python3 -c "import json; d=json.loads(open('gpurun_out/r5n_track_$V.log').read().splitlines()[-1]); print('$V us/3072: main', round(d['kern_ms']*1e3*3072/d['channels'],2), 'closed loop', round(d['cl_ms']*1e3*3072/d['channels'],2))"
done
unset GNSSCORR_LIB
echo "== layout probe"
timeout -k 10 120 python3 tools/trk_callmajor.py 20

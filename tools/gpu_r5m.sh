set -eu
timeout -k 10 300 python -u -m pytest tests/test_osg_loops_gpu.py tests/test_e2e_gpu.py tests/test_track_gpu.py -q -x --timeout 120 --timeout-method thread 2>&1 | tail -2
for V in base cliv0 base cliv0; do
  if [ $V = base ]; then unset GNSSCORR_LIB; else export GNSSCORR_LIB=$PWD/gnss-sdr.ru_amd/gnsscorr/libgnsscorr_$V.so; fi
  timeout -k 10 200 python -u tools/bench_part.py track 40 > gpurun_out/r5m_track_$V.log 2>&1
  python3 -c "import json; d=json.loads(open('gpurun_out/r5m_track_$V.log').read().splitlines()[-1]); print('$V us/3072: main', round(d['kern_ms']*1e3*3072/d['channels'],2), 'closed loop', round(d['cl_ms']*1e3*3072/d['channels'],2))"
done

# sgt chip chunks: 4 waves per SIMD (128 VGPRs, some spills; w4) and without
# the IF prefetch (w4npf) against the default 3-wave build
set -eu
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_sgt_gpu.py tests/test_sgt_trackres_gpu.py > gpurun_out/r5ab_tests.log 2>&1 || { tail -40 gpurun_out/r5ab_tests.log; exit 1; }
tail -1 gpurun_out/r5ab_tests.log
for i in 1 2; do
  for V in base w4 w4npf; do
    if [ $V = base ]; then unset GNSSCORR_LIB; else export GNSSCORR_LIB=$PWD/gnss-sdr.ru_amd/gnsscorr/libgnsscorr_$V.so; fi
    timeout -k 10 200 python -u tools/bench_part.py sgt 30 > gpurun_out/r5ab_sgt_$V$i.log 2>&1
    python3 -c "
import json
d = json.loads(open('gpurun_out/r5ab_sgt_$V$i.log').read().strip().split('\n')[-1])
print('$V run $i', {k: d.get(k) for k in ('kern_ms', 'lat_ms', 'channels', 'steps', 'ok')})"
  done
done
unset GNSSCORR_LIB



# m4_rows register budget: 2 waves per SIMD (amdgpu_waves_per_eu(2), 256 VGPRs, the
# tree) against the uncapped build (270 VGPRs, gpurun_out/libgnsscorr_wpe1.so)
set -eu
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_acq_generic_gpu.py > gpurun_out/r5an_tests.log 2>&1 || { tail -40 gpurun_out/r5an_tests.log; exit 1; }
tail -1 gpurun_out/r5an_tests.log
for i in 1 2; do
  for V in wpe2 wpe1; do
    L=""; [ $V = wpe1 ] && L=$PWD/abtmp/libgnsscorr_wpe1.so
    GNSSCORR_LIB=$L timeout -k 10 200 python -u tools/bench_part.py acq_generic 10 > gpurun_out/r5an_gen_$V$i.log 2>&1
    python3 -c "
import json
d = json.loads(open('gpurun_out/r5an_gen_$V$i.log').read().strip().split('\n')[-1])
print('$V run $i', 'ms per search', round(d['dt'] / d['steps'] * 1e3, 3), 'found', d['found'], '/', d['n_planted'])"
  done
done

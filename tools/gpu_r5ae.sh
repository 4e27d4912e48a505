# Four-step tile shapes: 128-thread column / row workgroups (c128, r128, cr128)
# against the 256-thread default, 38.192 Msps search; parity on cr128 first
set -eu
export TMPDIR=/tmp
GNSSCORR_LIB=$PWD/gnss-sdr.ru_amd/gnsscorr/libgnsscorr_cr128.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_acq_generic_gpu.py 2>&1 | tail -1
for i in 1 2; do
  for V in base c128 r128 cr128; do
    if [ $V = base ]; then unset GNSSCORR_LIB; else export GNSSCORR_LIB=$PWD/gnss-sdr.ru_amd/gnsscorr/libgnsscorr_$V.so; fi
    timeout -k 10 200 python -u tools/bench_part.py acq_generic 10 > gpurun_out/r5ae_$V$i.log 2>&1
    python3 -c "
import json
d = json.loads(open('gpurun_out/r5ae_$V$i.log').read().strip().split('\n')[-1])
print('$V run $i', 'ms per search', round(d['dt'] / d['steps'] * 1e3, 3), 'found', d['found'], '/', d['n_planted'])"
  done
done

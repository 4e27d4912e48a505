set -eu
export TMPDIR=/tmp
O=gpurun_out/r6e; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_acq_16m_gpu.py tests/test_acq_gpu.py tests/test_fullsky_gpu.py tests/test_acq_coh_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2 3; do
  for V in base r5acq; do
    if [ $V = base ]; then unset GNSSCORR_LIB; else export GNSSCORR_LIB=$PWD/gnss-sdr.ru_amd/ab/libgnsscorr_$V.so; fi
    timeout -k 10 200 python3 tools/bench_part.py gps_scilab 10 > $O/scilab_${V}_${i}.log 2>&1
    python3 -c "
import json
d = json.loads(open('$O/scilab_${V}_${i}.log').read().strip().split('\n')[-1])
print('$V run $i', 'ms per search', round(d['dt'] / d['steps'] * 1e3, 4), 'found', d['found'], '/', d['n_planted'])"
  done
done
unset GNSSCORR_LIB
bash tools/pmc_kernel.sh r6e/scilab gps_scilab 5 > $O/scilab_pmc.log 2>&1
grep -A3 "acq64_corr_kernel<Plan<16000" $O/scilab/summary.txt | head -8 || true

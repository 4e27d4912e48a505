set -eu
timeout -k 10 400 python -u -m pytest tests/test_acq_generic_gpu.py -q -x --timeout 200 --timeout-method thread 2>&1 | tail -2
for V in base base; do
  if [ $V = base ]; then unset GNSSCORR_LIB; else export GNSSCORR_LIB=$PWD/gnss-sdr.ru_amd/gnsscorr/libgnsscorr_$V.so; fi
  timeout -k 10 300 python3 tools/bench_part.py acq_generic 5 | python3 -c "import json,sys; d=json.loads(sys.stdin.read().splitlines()[-1]); print('$V generic ms per search', d['dt']/d['steps']*1e3, d['found'], d['n_planted'])"
done
unset GNSSCORR_LIB
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5g/prof -o run -- python3 tools/bench_part.py acq_generic 3 > gpurun_out/r5g/prof.log 2>&1
head -12 gpurun_out/r5g/prof/run_kernel_stats.csv | cut -c1-160

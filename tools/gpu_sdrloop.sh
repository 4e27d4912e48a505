# Closed-loop kernel: SDR parity tests, then timing per channels-per-wave setting.
set -eu
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_sdr_track_gpu.py tests/test_sdr_corr_gpu.py > gpurun_out/sdrloop_tests.log 2>&1
tail -1 gpurun_out/sdrloop_tests.log
for C in ${CPWS:-1 2 3 4}; do
  echo "cpw $C: $(GNSSCORR_SDR_LOOP_CPW=$C timeout -k 10 120 python tools/bench_sdr_loop.py | tail -1)"
done

# one GPU iteration on the fp64 acquisition: parity tests, phase stamps, short bench + kernel stats
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q -s --timeout 200 --timeout-method thread tests/test_acq_gpu.py tests/test_acq_16m_gpu.py tests/test_acq_coh_gpu.py tests/test_fullsky_gpu.py > gpurun_out/it_tests.log 2>&1
timeout -k 10 60 tools/acq64_stamps.bin > gpurun_out/it_stamps.txt 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --skip-track --no-cpu-baseline > gpurun_out/it_bench.json 2> gpurun_out/it_bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/it_prof -o run -- python3 tools/bench_part.py acq 10 > gpurun_out/it_prof.log 2>&1

set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q -s --timeout 200 --timeout-method thread tests/test_acq_gpu.py tests/test_acq_16m_gpu.py tests/test_acq_coh_gpu.py tests/test_fullsky_gpu.py tests/test_acq_generic_gpu.py tests/test_packed_gpu.py > gpurun_out/r2g_tests.log 2>&1
echo tests ok
timeout -k 10 200 python -u tools/bench_part.py acq 30 > gpurun_out/it_acq.log 2>&1
timeout -k 10 200 python -u tools/bench_part.py fullsky 10 > gpurun_out/it_sky.log 2>&1
timeout -k 10 200 python -u tools/bench_part.py glo_coherent 10 > gpurun_out/it_glo.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2g_prof -o run -- python3 tools/bench_part.py acq 20 > gpurun_out/r2g_prof.log 2>&1
grep -o '"dt": [0-9.]*\|"corr_ms": [0-9.]*' gpurun_out/it_acq.log gpurun_out/it_sky.log gpurun_out/it_glo.log

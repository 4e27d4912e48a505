set -eu
export TMPDIR=/tmp
O=gpurun_out/r6a; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_acq_generic_gpu.py tests/test_track_gpu.py tests/test_packed_gpu.py tests/test_osg_loops_gpu.py \
  tests/test_e2e_gpu.py tests/test_fullsky_gpu.py tests/test_acq_records_gpu.py tests/test_acq_prn_codes_gpu.py tests/test_acq_gpu.py > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -2 $O/tests.log
export TRK_C=12288
bash tools/gpu_trk_libab.sh "r5ref swz fl base" "cs1_int8 rx12_int8 cs1_packed2" 3 0 | tee $O/ab.log
bash tools/gpu_trk_pmc_ab.sh r6a "r5ref base" "cs1_int8" | tee $O/pmc.log
timeout -k 10 300 python3 -c "
import bench
r = bench.run_acq(bench.Dist(), 0, 20, 3, records=1)
print('single search ms', r['dt'] / 20 * 1e3, 'with codes', r['with_codes'], 'cold set_codes ms', r['meta']['set_codes_ms'])
" > $O/acq1.log 2>&1
tail -3 $O/acq1.log

# Scratch session script of round 6 (the current GPU call; earlier sessions are in git history)
set -eu
O=gpurun_out/r6z
mkdir -p $O/pmc_fullsky
export TMPDIR=/tmp BENCH_FULLSKY_PROJECTION=0
timeout -k 10 600 python -u -m pytest tests/test_fullsky_gpu.py tests/test_acq_gpu.py tests/test_acq_records_gpu.py -q -x --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
tail -1 $O/pytest.log
bash tools/gpu_acq_ab.sh r6z "base ordhead" "fullsky acq" 3 0 | tee $O/order_ab.log
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d $O/pmc_fullsky/$C -o run -- \
    python3 tools/bench_part.py fullsky 10 > $O/pmc_fullsky/$C.log 2>&1
done
python tools/pmc_summary.py $O/pmc_fullsky $O/pmc_summary_fullsky.json | grep corr_kernel
for F in 1 0 1 0 1 0; do
  GNSSCORR_OSG_FUSED=$F timeout -k 10 200 python -u tools/bench_part.py track 40 > $O/track_fused$F.log 2>&1
  echo "closed loop fused=$F $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('cl_ms', round(d['cl_ms'],5), 'open kern_ms', round(d['kern_ms'],5))" $O/track_fused$F.log)" | tee -a $O/cl_fused_ab.log
done

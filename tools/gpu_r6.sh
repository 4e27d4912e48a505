# Scratch session script of round 6 (the current GPU call; earlier sessions are in git history)
set -eu
O=gpurun_out/r6y
mkdir -p $O/pmc_fullsky
export TMPDIR=/tmp BENCH_FULLSKY_PROJECTION=0
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d $O/pmc_fullsky/$C -o run -- \
    python3 tools/bench_part.py fullsky 10 > $O/pmc_fullsky/$C.log 2>&1
done
cp profiles/pmc_traffic.json $O/pmc_traffic.json
python tools/pmc_summary.py $O/pmc_fullsky $O/pmc_summary_fullsky.json --traffic $O/pmc_traffic.json --section fullsky --runs 13
bash tools/gpu_trk_libab.sh "base p1 p2" "cs1_int8 rx12_int8" 3 0 | tee $O/trk_lo_probe.log

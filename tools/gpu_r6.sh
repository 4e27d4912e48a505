# Scratch session script of round 6 (the current GPU call; earlier sessions are in git history)
set -eu
O=gpurun_out/r6h
bash tools/gpu_acq_ab.sh r6h "base r6base" "fullsky acq gps_scilab" 3 1 | tee $O.ab.log
mkdir -p $O/pmc_fullsky
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d $O/pmc_fullsky/$C -o run -- \
    python3 tools/bench_part.py fullsky 10 > $O/pmc_fullsky/$C.log 2>&1
done
python tools/pmc_summary.py $O/pmc_fullsky $O/pmc_summary_fullsky.json --section fullsky --runs 13
echo pmc ok

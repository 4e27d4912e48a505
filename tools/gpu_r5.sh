# Round-5 GPU session: parity tests, smoke, the driver's bench command, the
# self-launched 2-rank bench, kernel traces split by grid, per-section PMC passes.
# usage (via gpurun): bash tools/gpu_r5.sh <tag> [main|prof|pmc|all]
# Every GPU step has its own time limit; the first failure (other than test
# failures, rc 1) ends the script.
set -eu
TAG=${1:-r5}
PART=${2:-all}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
run_main() {
  echo "== pytest -m gpu"
  rc=0
  timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || rc=$?
  tail -3 $O/pytest.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc"; exit $rc; fi
  echo "== smoke"
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
  tail -1 $O/smoke.log
  echo "== bench (the driver's command, wall-timed)"
  s0=$(date +%s.%N)
  timeout -k 10 500 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
  s1=$(date +%s.%N)
  python3 -c "print('wall_s', round($s1-$s0, 1))" | tee $O/bench.wall
  wc -c $O/bench.json
  cp gpurun_out/bench_detail.json $O/bench_detail.json
  echo "== bench --gpus 2 (self-launched ranks, both on this box's one GPU)"
  timeout -k 10 300 python3 bench.py --gpus 2 --steps 5 --warmup 2 --skip-track --no-cpu-baseline > $O/bench_gpus2.json 2> $O/bench_gpus2.err
  cut -c1-300 $O/bench_gpus2.json
}
run_prof() {
  echo "== rocprofv3 kernel-trace stats"
  mkdir -p $O/prof
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
    python3 bench.py --no-cpu-baseline --steps 20 > $O/prof.log 2>&1
  for K in acq64_corr_kernel osg_stream_kernel sgt_track_kernel; do
    python3 tools/trace_by_grid.py $O/prof $K $O/trace_by_grid_$K.json \
      "rocprofv3 --kernel-trace of python3 bench.py --no-cpu-baseline --steps 20 ($TAG)"
  done
}
run_pmc() {
  echo "== pmc (per section; HBM bytes into a copy of profiles/pmc_traffic.json)"
  cp profiles/pmc_traffic.json $O/pmc_traffic.json
  for S in ${PMC_SECTIONS:-acq track fullsky glo_coherent gps_scilab acq_generic sgt sdr}; do
    mkdir -p $O/pmc_$S
    for C in FETCH_SIZE WRITE_SIZE; do
      BENCH_FULLSKY_PROJECTION=0 timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d $O/pmc_$S/$C -o run -- \
        python3 tools/bench_part.py $S 10 > $O/pmc_$S/$C.log 2>&1
    done
    R=""
    case $S in acq|fullsky|glo_coherent|gps_scilab|acq_generic) R="--runs 13";; esac
    python tools/pmc_summary.py $O/pmc_$S $O/pmc_summary_$S.json --traffic $O/pmc_traffic.json --section $S $R > /dev/null
    echo "pmc section $S ok"
  done
  for L in ${PMC_LAYOUTS:-cs1_int8 cs1_packed2 rx12_int8 rx12_packed2}; do
    mkdir -p $O/pmc_trk_$L
    for C in FETCH_SIZE WRITE_SIZE "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES"; do
      D=$(echo $C | cut -d' ' -f1)
      timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d $O/pmc_trk_$L/$D -o run -- \
        python3 tools/trk_layout.py $L 20 > $O/pmc_trk_$L/$D.log 2>&1
    done
    python tools/pmc_summary.py $O/pmc_trk_$L $O/pmc_summary_trk_$L.json --traffic $O/pmc_traffic.json --section trk_$L > /dev/null
    echo "pmc layout $L ok"
  done
}
case $PART in
  main) run_main;;
  prof) run_prof;;
  pmc) run_pmc;;
  all) run_main; run_prof; run_pmc;;
esac
echo "== done ($PART)"

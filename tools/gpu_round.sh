# One GPU session: parity tests, bench, kernel-trace stats, PMC passes.
# usage (via gpurun): bash tools/gpu_round.sh <tag> [main|pmc|pmcA|pmcB|all]
#   main: tests, smoke, bench, kernel-trace stats; pmc: counter passes and the tracking A/B
#   (pmcA: the whole-bench passes, pmcB: the per-section passes and the A/B, for two
#   calls within gpurun's time limit: copy pmcA's pmc_traffic.json to profiles/ first)
# Every GPU step has its own time limit; the first failure ends the script.
set -eu
TAG=${1:-r1}
PART=${2:-all}
O=gpurun_out/$TAG
mkdir -p $O/pmc $O/pmc_acq $O/pmc_track $O/pmc_fullsky $O/pmc_glo_coherent $O/pmc_acq_generic $O/pmc_gps_scilab
export TMPDIR=/tmp
if [ $PART = main ] || [ $PART = all ]; then
echo "== pytest -m gpu"
# test failures (rc 1) are recorded and the session goes on; a timeout, abort or
# crash ends it
rc=0
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || rc=$?
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
cp gpurun_out/bench_detail.json $O/bench_detail.json   # (the profiled run below rewrites it)
cut -c1-400 $O/bench.json
echo "== rocprofv3 kernel-trace stats"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 bench.py --no-cpu-baseline > $O/prof.log 2>&1
python3 tools/trace_by_grid.py $O/prof acq64_corr_kernel $O/acq64_trace_by_grid.json \
  "rocprofv3 --kernel-trace of python3 bench.py --no-cpu-baseline ($TAG)"
fi
if [ $PART = main ]; then echo "== done (main)"; exit 0; fi
echo "== pmc"
# the committed traffic file is the base: every pass below updates its entries
cp profiles/pmc_traffic.json $O/pmc_traffic.json
B="python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline"
if [ $PART != pmcB ]; then
i=0
for C in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES" \
         "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE" \
         "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d $O/pmc/p$i -o run -- $B > $O/pmc/p$i.log 2>&1
  echo "pmc pass $i ok"
done
python tools/pmc_summary.py $O/pmc $O/pmc_summary.json --traffic $O/pmc_traffic.json
rm -rf $O/pmc/p[0-9]*/   # raw counter CSVs (tens of MiB at 16-record steps): the summary stays
fi
if [ $PART = pmcA ]; then echo "== done (pmcA)"; exit 0; fi
# HBM bytes per launch of the kernels several sections share, one section at a time
# (the full-sky section without its shard projection: only the world-1 launches)
export BENCH_FULLSKY_PROJECTION=0
for S in acq track fullsky glo_coherent acq_generic gps_scilab; do
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d $O/pmc_$S/$C -o run -- \
      python3 tools/bench_part.py $S 10 > $O/pmc_$S/$C.log 2>&1
  done
  python tools/pmc_summary.py $O/pmc_$S $O/pmc_summary_$S.json --traffic $O/pmc_traffic.json --section $S --runs 13
  rm -rf $O/pmc_$S/FETCH_SIZE/ $O/pmc_$S/WRITE_SIZE/
  echo "pmc section $S ok"
done
# the tracking layouts one at a time (the layouts share kernel instantiations)
for L in cs1_int8 cs1_packed2 rx12_packed2; do
  mkdir -p $O/pmc_trk_$L
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d $O/pmc_trk_$L/$C -o run -- \
      python3 tools/trk_layout.py $L 10 > $O/pmc_trk_$L/$C.log 2>&1
  done
  python tools/pmc_summary.py $O/pmc_trk_$L $O/pmc_summary_trk_$L.json --traffic $O/pmc_traffic.json --section trk_$L
  rm -rf $O/pmc_trk_$L/FETCH_SIZE/ $O/pmc_trk_$L/WRITE_SIZE/
  echo "pmc layout $L ok"
done
for S in sgt sdr; do
  mkdir -p $O/pmc_$S
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d $O/pmc_$S/$C -o run -- \
      python3 tools/bench_part.py $S 10 > $O/pmc_$S/$C.log 2>&1
  done
  python tools/pmc_summary.py $O/pmc_$S $O/pmc_summary_$S.json --traffic $O/pmc_traffic.json --section $S
  rm -rf $O/pmc_$S/FETCH_SIZE/ $O/pmc_$S/WRITE_SIZE/
  echo "pmc section $S ok"
done
echo "== tracking A/B (same box): stream kernel, TRACK_LO_SPLIT=0 build, per-call workgroup kernel"
for L in cs1_int8 cs1_packed2 rx12_int8 rx12_packed2; do
  for V in new lo0 wg; do
    case $V in
      new) unset GNSSCORR_LIB; S=1;;
      lo0) export GNSSCORR_LIB=$PWD/gnss-sdr.ru_amd/ab/libgnsscorr_lo0.so; S=1;;
      wg) unset GNSSCORR_LIB; S=0;;
    esac
    [ $V = lo0 ] && [ ! -f gnss-sdr.ru_amd/ab/libgnsscorr_lo0.so ] && continue
    echo "$L $V: $(GNSSCORR_TRACK_STREAM=$S timeout -k 10 120 python3 tools/trk_layout.py $L 40)" | tee -a $O/trk_ab.log
  done
done
unset GNSSCORR_LIB
for F in 1 0; do
  GNSSCORR_OSG_FUSED=$F timeout -k 10 200 python -u tools/bench_part.py track 40 > $O/track_fused$F.log 2>&1
  echo "closed loop fused=$F $(tail -1 $O/track_fused$F.log | cut -c1-200)" | tee -a $O/trk_ab.log
done
echo "== done"

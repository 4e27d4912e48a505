# round-4 batch 3: tracking parity (row reuse across calls, split LO tables), then
# timings: main line + closed loop (fused / two launches), layouts new vs TRACK_LO_SPLIT=0
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/b3
O=gpurun_out/b3
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_track_gpu.py tests/test_osg_loops_gpu.py tests/test_e2e_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for F in 1 0; do
  GNSSCORR_OSG_FUSED=$F timeout -k 10 200 python -u tools/bench_part.py track 40 > $O/track_f$F.log 2>&1
  echo "fused=$F $(tail -1 $O/track_f$F.log | cut -c1-300)"
done
for L in cs1_int8 cs1_packed2 rx12_int8 rx12_packed2; do
  for i in 1 2; do
    for V in new lo0 wg; do
      case $V in
        new) unset GNSSCORR_LIB; S=1;;
        lo0) export GNSSCORR_LIB=$PWD/gnss-sdr.ru_amd/gnsscorr/libgnsscorr_lo0.so; S=1;;
        wg) unset GNSSCORR_LIB; S=0;;
      esac
      echo "$L $V: $(GNSSCORR_TRACK_STREAM=$S timeout -k 10 120 python3 tools/trk_layout.py $L 40)"
    done
  done
done
unset GNSSCORR_LIB
bash tools/trk_stream_stamps.sh > $O/stamps.log 2>&1 && tail -24 $O/stamps.log

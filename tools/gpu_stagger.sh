# acq64: correlation launch time vs the first-wave CU stagger (GNSSCORR_ACQ_STAGGER).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for S in ${STAGGERS:-0 1 2 3 4 0}; do
  GNSSCORR_ACQ_STAGGER=$S timeout -k 10 200 python -u tools/bench_part.py acq 60 > gpurun_out/stag_$S.log 2>&1
  echo "stagger=$S $(tail -1 gpurun_out/stag_$S.log | cut -c1-80)"
done

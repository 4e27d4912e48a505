# Same-box A/B timing of two builds of libgnsscorr.so (gpurun_ab/lib_A.so,
# lib_B.so): bench section ${AB_PART:-acq}, alternating A B A B A B.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for i in 1 2 3; do
  for V in A B; do
    GNSSCORR_LIB=$PWD/gpurun_ab/lib_$V.so timeout -k 10 200 python -u tools/bench_part.py ${AB_PART:-acq} ${AB_STEPS:-60} > gpurun_out/ab_$V$i.log 2>&1
    echo "$V$i $(tail -1 gpurun_out/ab_$V$i.log | cut -c1-${AB_CUT:-70})"
  done
done

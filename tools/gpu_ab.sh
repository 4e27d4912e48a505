# Same-box A/B timing of two builds of libgnsscorr.so (gpurun_ab/lib_A.so,
# lib_B.so): optional parity tests on B (AB_TESTS), then bench section
# ${AB_PART:-acq} alternating A B A B A B, printing the keys AB_KEYS.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
if [ -n "${AB_TESTS:-}" ]; then
  GNSSCORR_LIB=$PWD/gpurun_ab/lib_B.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread $AB_TESTS > gpurun_out/ab_tests.log 2>&1
  tail -1 gpurun_out/ab_tests.log
fi
for i in 1 2 3; do
  for V in ${AB_VARIANTS:-A B}; do
    GNSSCORR_LIB=$PWD/gpurun_ab/lib_$V.so timeout -k 10 200 python -u tools/bench_part.py ${AB_PART:-acq} ${AB_STEPS:-60} > gpurun_out/ab_$V$i.log 2>&1
    python -c "
import json, sys
d = json.loads(open('gpurun_out/ab_$V$i.log').read().strip().split('\n')[-1])
print('$V$i', {k: d.get(k) for k in '${AB_KEYS:-corr_ms}'.split(',')})"
  done
done

# Same-box A/B of gpurun_ab/lib_A.so and lib_B.so over several bench sections:
# optional tests on B (AB_TESTS), then acq / track / track_io alternating A B.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -n "${AB_TESTS:-}" ]; then
  GNSSCORR_LIB=$PWD/gpurun_ab/lib_B.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread $AB_TESTS > gpurun_out/ab_tests.log 2>&1 || { tail -30 gpurun_out/ab_tests.log; exit 1; }
  tail -1 gpurun_out/ab_tests.log
fi
for P in ${AB_PARTS:-acq track track_io}; do
  for i in 1 2; do
    for V in A B; do
      GNSSCORR_LIB=$PWD/gpurun_ab/lib_$V.so timeout -k 10 200 python -u tools/bench_part.py $P ${AB_STEPS:-40} > gpurun_out/ab_${P}_$V$i.log 2>&1
      python - <<PY
import json
d = json.loads(open('gpurun_out/ab_${P}_$V$i.log').read().strip().split('\n')[-1])
def pick(d):
    out = {}
    for k, v in d.items():
        if isinstance(v, dict):
            sub = {kk: vv for kk, vv in v.items() if kk in ('kern_ms', 'mean_us')}
            if sub: out[k] = sub
        elif k in ('corr_ms', 'kern_ms', 'cl_ms', 'lat_ms', 'dt'):
            out[k] = v
    return out
print('$P $V$i', pick(d))
PY
    done
  done
done

# sgt tracking A/B on one box: parity tests (chunked path, the default), then
# the bench section with the chunked path on and off (GNSSCORR_SGT_CHUNK).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_sgt_gpu.py > gpurun_out/sgt_tests.log 2>&1 || { tail -30 gpurun_out/sgt_tests.log; exit 1; }
tail -2 gpurun_out/sgt_tests.log
for i in 1 2; do
  for C in 1 0; do
    GNSSCORR_SGT_CHUNK=$C timeout -k 10 200 python -u tools/bench_part.py sgt ${SGT_STEPS:-30} > gpurun_out/sgt_ab_$C$i.log 2>&1
    python -c "
import json
d = json.loads(open('gpurun_out/sgt_ab_$C$i.log').read().strip().split('\n')[-1])
print('chunk=$C run $i', {k: d.get(k) for k in ('kern_ms', 'lat_ms', 'channels', 'steps', 'ok')})"
  done
done

# sgt A/B (lib_A / lib_B, tests on B) and the tracking layouts under
# GNSSCORR_TRACK_CPW (channels per workgroup) on the default library.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
AB_PARTS=sgt AB_STEPS=30 AB_TESTS=tests/test_sgt_gpu.py bash tools/gpu_ab2.sh
for W in 4 3 2; do
  GNSSCORR_TRACK_CPW=$W timeout -k 10 200 python -u tools/bench_part.py track_io 40 > gpurun_out/cpw_$W.log 2>&1
  python - <<PY
import json
d = json.loads(open('gpurun_out/cpw_$W.log').read().strip().split('\n')[-1])
print('cpw $W', {k: round(v['kern_ms'] * 1e3, 2) for k, v in d.items() if isinstance(v, dict) and 'kern_ms' in v})
PY
done

# sgt tracking A/B between two builds on one box: parity tests on the default
# library, then the bench section alternating it with GNSSCORR_LIB=$AB_LIB.
# usage (via gpurun): AB_LIB=gnss-sdr.ru_amd/ab/libgnsscorr_ab.so bash tools/gpu_sgt_lib_ab.sh
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
AB_LIB=${AB_LIB:-gnss-sdr.ru_amd/ab/libgnsscorr_ab.so}
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_sgt_gpu.py > gpurun_out/sgt_tests.log 2>&1 || { tail -30 gpurun_out/sgt_tests.log; exit 1; }
tail -2 gpurun_out/sgt_tests.log
for i in 1 2 3; do
  for V in new ab; do
    if [ $V = ab ]; then export GNSSCORR_LIB=$PWD/$AB_LIB; else unset GNSSCORR_LIB; fi
    timeout -k 10 200 python -u tools/bench_part.py sgt ${SGT_STEPS:-30} > gpurun_out/sgt_lab_$V$i.log 2>&1
    python -c "
import json
d = json.loads(open('gpurun_out/sgt_lab_$V$i.log').read().strip().split('\n')[-1])
print('$V run $i', {k: d.get(k) for k in ('kern_ms', 'lat_ms', 'channels', 'steps', 'ok')})"
  done
done
unset GNSSCORR_LIB

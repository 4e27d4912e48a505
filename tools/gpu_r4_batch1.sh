# round-4 batch: tracking replay debug + tracking/loop tests, then the sgt prefix A/B
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_sdr_track_gpu.py > gpurun_out/sdr_track_tests.log 2>&1 || true
tail -3 gpurun_out/sdr_track_tests.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_sgt_gpu.py tests/test_sgt_trackres_gpu.py > gpurun_out/sgt_tests.log 2>&1 || { tail -30 gpurun_out/sgt_tests.log; exit 1; }
tail -2 gpurun_out/sgt_tests.log
for i in 1 2; do
  for V in new ab ab8; do
    if [ $V = new ]; then unset GNSSCORR_LIB; else export GNSSCORR_LIB=$PWD/gnss-sdr.ru_amd/gnsscorr/libgnsscorr_$V.so; fi
    timeout -k 10 200 python -u tools/bench_part.py sgt 30 > gpurun_out/sgt_pf_$V$i.log 2>&1
    python -c "
import json
d = json.loads(open('gpurun_out/sgt_pf_$V$i.log').read().strip().split('\n')[-1])
print('$V run $i', {k: d.get(k) for k in ('kern_ms', 'lat_ms', 'channels', 'steps', 'ok')})"
  done
done
unset GNSSCORR_LIB

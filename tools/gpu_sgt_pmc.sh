# sgt: parity tests, the bench section, then PMC passes over it (tools/pmc_kernel.sh)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_sgt_gpu.py > gpurun_out/sgt_tests.log 2>&1 || { tail -30 gpurun_out/sgt_tests.log; exit 1; }
tail -1 gpurun_out/sgt_tests.log
timeout -k 10 200 python -u tools/bench_part.py sgt 30 > gpurun_out/sgt_b.log 2>&1
tail -1 gpurun_out/sgt_b.log
bash tools/pmc_kernel.sh ${PMC_TAG:-sgtpmc} sgt 10
grep -A 30 sgt_track gpurun_out/${PMC_TAG:-sgtpmc}/summary.txt | head -40

# shard test + the default bench run (what the driver runs), each under its own limit
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_trackshard_gpu.py > gpurun_out/bf_tests.log 2>&1
timeout -k 10 900 python -u bench.py > gpurun_out/bf_bench.json 2> gpurun_out/bf_bench.err

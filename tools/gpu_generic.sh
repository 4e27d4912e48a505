set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread tests/test_acq_generic_gpu.py tests/test_acq_gpu.py > gpurun_out/generic.log 2>&1

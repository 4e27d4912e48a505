set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
GNSSCORR_TRACK_STAGE_PERCH=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_track_gpu.py tests/test_packed_gpu.py tests/test_e2e_gpu.py tests/test_osg_loops_gpu.py > gpurun_out/pytest_perch.log 2>&1
echo tests ok
GNSSCORR_TRACK_STAGE_PERCH=1 timeout -k 10 300 python -u tools/bench_part.py track_io 20 > gpurun_out/track_io_perch.log 2>&1
GNSSCORR_TRACK_STAGE_PERCH=1 timeout -k 10 200 python -u tools/bench_part.py track 30 > gpurun_out/track_perch.log 2>&1
echo done

set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --skip-track --no-cpu-baseline > gpurun_out/b1.json 2> gpurun_out/b1.err
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof1 -o prof -- python3 bench.py --steps 10 --warmup 2 --skip-track --no-cpu-baseline > gpurun_out/prof1.log 2>&1

# Quick GPU session: parity tests, smoke and the driver's exact bench command (timed).
# usage (via gpurun): bash tools/gpu_quick.sh <tag>
set -eu
TAG=${1:-q}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
echo "== pytest -m gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
tail -3 $O/pytest.log
echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
echo "== bench (driver command)"
s=$(date +%s.%N)
timeout -k 10 500 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_cmd.json 2> $O/bench_driver_cmd.err
e=$(date +%s.%N)
python3 -c "print('wall_s', round($e-$s, 1))" | tee $O/bench_driver_cmd.wall
cat $O/bench_driver_cmd.json | cut -c1-600
echo "== done"

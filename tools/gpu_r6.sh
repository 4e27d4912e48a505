# Scratch session script of round 6 (the current GPU call; earlier sessions are in git history)
set -eu
O=gpurun_out/r8y
mkdir -p $O
export TMPDIR=/tmp
s0=$(date +%s.%N)
timeout -k 10 500 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
s1=$(date +%s.%N)
python3 -c "print('wall_s', round($s1-$s0, 1))" | tee $O/bench.wall
cp gpurun_out/bench_detail.json $O/bench_detail.json
cut -c1-200 $O/bench.json

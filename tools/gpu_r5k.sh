set -eu
O=gpurun_out/r5k; mkdir -p $O
echo "== full bench, --gpus 2 self-launched on one GPU (every section's distributed path)"
s0=$(date +%s.%N)
timeout -k 10 600 python3 bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_gpus2_full.json 2> $O/bench_gpus2_full.err
s1=$(date +%s.%N)
python3 -c "print('wall_s', round($s1-$s0, 1))"
wc -c $O/bench_gpus2_full.json
PMC_SECTIONS="fullsky" PMC_LAYOUTS="" bash tools/gpu_r5.sh r5k pmc

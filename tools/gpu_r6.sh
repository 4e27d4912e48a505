set -eu
export TMPDIR=/tmp
O=gpurun_out/r6c; mkdir -p $O
# 8-rank rehearsal on one GPU (ranks wrap to device 0): launcher, host group, memory
s0=$(date +%s.%N)
timeout -k 10 900 python3 bench.py --gpus 8 --steps 5 --warmup 2 --skip-track --no-cpu-baseline > $O/bench_gpus8.json 2> $O/bench_gpus8.err
s1=$(date +%s.%N)
python3 -c "print('wall_s', round($s1-$s0, 1))"
cp gpurun_out/bench_detail.json $O/bench_detail_gpus8.json
python3 - <<'P'
import json
d = json.load(open("gpurun_out/r6c/bench_detail_gpus8.json"))
print("n_gpus", d["n_gpus"], "value", d["value"])
for r in d["ranks"]:
    print(r["rank"], r["device"], r["hip_runtime"]["bound"], r["hip_runtime"]["mapped"])
P

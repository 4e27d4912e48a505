# Generic-rate work-buffer size (rows per chunk: 109 at 64 MiB) for the 38.192 Msps
# search: GNSSCORR_ACQ_GCHUNK_MB 32 / 64 / 128 / 256 (first run) and 256 / 512 / 1024 / 2048
set -eu
export TMPDIR=/tmp
for i in 1 2; do
  for M in 256 512 1024 2048; do
    GNSSCORR_ACQ_GCHUNK_MB=$M timeout -k 10 200 python -u tools/bench_part.py acq_generic 10 > gpurun_out/r5ao_gen_$M$i.log 2>&1
    python3 -c "
import json
d = json.loads(open('gpurun_out/r5ao_gen_$M$i.log').read().strip().split('\n')[-1])
print('GCHUNK_MB=$M run $i', 'ms per search', round(d['dt'] / d['steps'] * 1e3, 3), 'found', d['found'], '/', d['n_planted'])"
  done
done

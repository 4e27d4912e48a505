# Scratch session script of round 6 (the current GPU call; earlier sessions are in git history)
set -eu
O=gpurun_out/r8w
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 560 python3 bench.py --gpus 2 --steps 10 --warmup 3 > $O/bench2.json 2> $O/bench2.err
python3 -c "import json; d=json.loads(open('$O/bench2.json').read().strip().splitlines()[-1]); print('n_gpus', d['n_gpus'], 'value', d['value'], 'generic', d['acquisition_generic']['ms_per_search'], d['acquisition_generic']['planted_found'], 'scilab', d['gps_acquisition_scilab']['planted_found'], 'glo5', d['glonass_acquisition_5ms']['planted_found'], 'fullsky', d['fullsky']['planted_found'])"

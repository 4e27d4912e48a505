# Scratch session script of round 6 (the current GPU call; earlier sessions are in git history)
set -eu
O=gpurun_out/r8l
mkdir -p $O
export TMPDIR=/tmp
for i in 1 2; do
for R in 1 4 16; do
  BENCH_GLO_COH_RECORDS=$R timeout -k 10 300 python3 tools/bench_part.py glo_coherent 10 > $O/s_$R.json 2> $O/s_$R.err
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('records', d['records'], 'ms per search %.4f' % (d['dt']*1e3/(d['steps']*d['records'])), 'found %s/%s' % (d['found'], d['n_planted']))" $O/s_$R.json
done
done | tee $O/ab.log

# Scratch session script of round 6 (the current GPU call; earlier sessions are in git history)
set -eu
O=gpurun_out/r9b
mkdir -p $O
export TMPDIR=/tmp
for i in 1 2; do
for MB in 87 116 145; do
  GNSSCORR_ACQ_GCHUNK_MB=$MB timeout -k 10 300 python3 tools/bench_part.py acq_generic 10 > $O/g_$MB.json 2> $O/g_$MB.err
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('16 records, MiB of Y per lane chunk', sys.argv[2], 'ms per search %.4f' % (d['dt']*1e3/(d['steps']*d['records'])))" $O/g_$MB.json $MB
done
done | tee $O/ab.log

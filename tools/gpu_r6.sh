# Scratch session script of round 6 (the current GPU call; earlier sessions are in git history)
set -eu
O=gpurun_out/r6p
mkdir -p $O
export TMPDIR=/tmp BENCH_FULLSKY_PROJECTION=0
for i in 1 2; do
  for PC in "1 64" "1 128" "1 256" "0 128" "0 256"; do
    set -- $PC
    GNSSCORR_ACQ_M4PIPE=$1 GNSSCORR_ACQ_GCHUNK_MB=$2 timeout -k 10 300 python3 tools/bench_part.py acq_generic 20 > $O/gen_$1_$2_$i.json
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('pipe', sys.argv[2], 'chunk MiB', sys.argv[3], 'ms per search %.4f' % (d['dt']*1e3/20), 'found %s/%s' % (d['found'], d['n_planted']))" $O/gen_$1_$2_$i.json $1 $2
  done
done | tee $O/pipe_chunk_ab.log

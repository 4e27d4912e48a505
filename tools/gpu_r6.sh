# Scratch session script of round 6 (the current GPU call; earlier sessions are in git history)
set -eu
O=gpurun_out/r7o
mkdir -p $O
export TMPDIR=/tmp BENCH_FULLSKY_PROJECTION=0
for i in 1 2; do
for S in 5 10 20; do
  timeout -k 10 300 python3 tools/bench_part.py fullsky $S > $O/fs_$S.json 2> $O/fs_$S.err
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('fullsky steps', sys.argv[2], 'ms per search %.4f' % (d['dt']*1e3/d['steps']))" $O/fs_$S.json $S
done
for S in 10 20; do
  timeout -k 10 300 python3 tools/bench_part.py acq_generic $S > $O/g_$S.json 2> $O/g_$S.err
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('generic steps', sys.argv[2], 'ms per search %.4f' % (d['dt']*1e3/d['steps']))" $O/g_$S.json $S
done
done

# Same-box A/B of acquisition builds: bash tools/gpu_acq_ab.sh <tag> "<lib names>" [sections] [reps] [tests]
# lib name "base" = the in-tree library, else gnss-sdr.ru_amd/ab/libgnsscorr_<name>.so;
# sections are bench.py run_<section> names (tools/bench_part.py); tests=1 first runs
# the acquisition parity tests on the in-tree library.  Prints ms per search.
set -eu
cd ${GRAFT_REPO_ROOT:-.}
TAG=$1
LIBS=$2
SECTIONS=${3:-"fullsky acq"}
REPS=${4:-3}
TESTS=${5:-1}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp BENCH_FULLSKY_PROJECTION=0
if [ "$TESTS" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests/test_fullsky_gpu.py tests/test_acq_gpu.py \
    tests/test_acq_records_gpu.py tests/test_acq_16m_gpu.py tests/test_acq_coh_gpu.py \
    tests/test_acq_prn_codes_gpu.py -q -x --timeout 200 --timeout-method thread > $O/pytest_acq.log 2>&1
  tail -2 $O/pytest_acq.log
fi
for S in $SECTIONS; do
  for i in $(seq $REPS); do
    for V in $LIBS; do
      if [ $V = base ]; then unset GNSSCORR_LIB; else export GNSSCORR_LIB=$PWD/gnss-sdr.ru_amd/ab/libgnsscorr_$V.so; fi
      timeout -k 10 300 python3 tools/bench_part.py $S 20 > $O/${S}_${V}_$i.json 2> $O/${S}_${V}_$i.err
      # dt: seconds for the section's 20 timed steps (records per step: 'records', else 1)
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); n=20*d.get('records',1); print(sys.argv[2], sys.argv[3], 'ms per search %.4f' % (d['dt']*1e3/n), 'kernel ms %s' % d.get('corr_ms'), 'found %s/%s' % (d.get('found'), d.get('n_planted')))" $O/${S}_${V}_$i.json $S $V
    done
  done
done
unset GNSSCORR_LIB

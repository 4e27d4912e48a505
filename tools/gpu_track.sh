# Tracking kernel session: parity tests, then the tracking bench sections with the
# new kernel (osg_track2_kernel) and the round-2 kernel (GNSSCORR_TRACK_V1=1), A/B.
# usage (via gpurun): bash tools/gpu_track.sh <tag>
set -eu
TAG=${1:-t}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
echo "== tracking parity tests"
[ -n "${SKIP_TESTS:-}" ] || timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_track_gpu.py tests/test_packed_gpu.py tests/test_e2e_gpu.py tests/test_osg_loops_gpu.py \
  tests/test_trackshard_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
[ -n "${SKIP_TESTS:-}" ] || tail -2 $O/pytest.log
# TRK_VARIANTS: GNSSCORR_TRACK_<name>=1 per run (V0: no such switch, the default)
for V in ${TRK_VARIANTS:-V0 V1 V0 V1}; do
  echo "== bench track / track_io, GNSSCORR_TRACK_$V=1 (V0: default)"
  env GNSSCORR_TRACK_$V=1 timeout -k 10 200 python3 tools/bench_part.py track 20 > $O/track_v$V.json
  env GNSSCORR_TRACK_$V=1 timeout -k 10 200 python3 tools/bench_part.py track_io 20 > $O/track_io_v$V.json
  python3 - $O/track_v$V.json $O/track_io_v$V.json <<'PY'
import json, sys
a = json.load(open(sys.argv[1])); b = json.load(open(sys.argv[2]))
print("rx12 int8 kern_ms %.4f  closed-loop %.4f" % (a["kern_ms"], a["cl_ms"]))
for k in ("cs1_int8", "cs1_packed2", "rx12_packed2"):
    print(k, "kern_ms %.4f" % b[k]["kern_ms"])
print("sim_gp2021_12ch", b["sim_gp2021_12ch"])
PY
done
echo "== done"

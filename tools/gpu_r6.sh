# Scratch session script of round 6 (the current GPU call; earlier sessions are in git history)
set -eu
O=gpurun_out/r6l
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_acq_generic_gpu.py tests/test_acq_prn_codes_gpu.py -q -x --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
tail -1 $O/pytest.log
bash tools/gpu_acq_ab.sh r6l "base m4head" "acq_generic" 3 0 | tee $O/generic_pitch_ab.log
for V in base m4head; do
  if [ $V = base ]; then unset GNSSCORR_LIB; else export GNSSCORR_LIB=$PWD/gnss-sdr.ru_amd/ab/libgnsscorr_$V.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$V -o run -- \
    python3 tools/bench_part.py acq_generic 10 > $O/prof_$V.log 2>&1
done
unset GNSSCORR_LIB
for V in base m4head; do
  python3 - $O/prof_$V $V <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if any(k in r["Name"] for k in ("m4_", "g_wipe", "m4_stats")):
        print(sys.argv[2], r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2), "us")
PY
done

# Scratch session script of round 6 (the current GPU call; earlier sessions are in git history)
set -eu
O=gpurun_out/r7s
mkdir -p $O
export TMPDIR=/tmp
GNSSCORR_LIB=$PWD/gnss-sdr.ru_amd/ab/libgnsscorr_xcd.so timeout -k 10 600 python -u -m pytest tests/test_acq_generic_gpu.py -q -x --timeout 200 --timeout-method thread > $O/pytest_xcd.log 2>&1
echo "xcd $(tail -1 $O/pytest_xcd.log)"
bash tools/gpu_acq_ab.sh r7s "base xcd" "acq_generic" 4 0 | tee $O/ab.log

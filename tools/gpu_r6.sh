# Scratch session script of round 6 (the current GPU call; earlier sessions are in git history)
set -eu
O=gpurun_out/r7r
mkdir -p $O
export TMPDIR=/tmp
for V in milp mclause; do
GNSSCORR_LIB=$PWD/gnss-sdr.ru_amd/ab/libgnsscorr_$V.so timeout -k 10 600 python -u -m pytest tests/test_acq_generic_gpu.py tests/test_acq_gpu.py -q -x --timeout 200 --timeout-method thread > $O/pytest_$V.log 2>&1
echo "$V $(tail -1 $O/pytest_$V.log)"
done
bash tools/gpu_acq_ab.sh r7r "base milp mclause" "acq acq_generic" 3 0 | tee $O/ab.log

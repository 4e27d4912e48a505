# Scratch session script of round 6 (the current GPU call; earlier sessions are in git history)
set -eu
O=gpurun_out/r8b
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_acq_generic_gpu.py tests/test_acq_prn_codes_gpu.py tests/test_acq_16m_gpu.py -q -x --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
tail -1 $O/pytest.log
bash tools/gpu_acq_ab.sh r8b "base prev" "acq_generic" 4 0 | tee $O/ab.log

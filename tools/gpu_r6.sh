# Scratch session script of round 6 (the current GPU call; earlier sessions are in git history)
set -eu
O=gpurun_out/r8a
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_acq_generic_gpu.py -v -x --timeout 200 --timeout-method thread -k "multi_chunk" > $O/pytest.log 2>&1
grep -E "PASS|FAIL|passed|failed|Error" $O/pytest.log | tail -12

# sgt exact-crossing tests in wave mode (run_chips boundaries and slow path),
# tracking parity after the unguarded whole-piece DMA issue, and a same-box
# check of the tracking layouts
set -eu
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_sgt_gpu.py > gpurun_out/r5u_sgt.log 2>&1 || { tail -40 gpurun_out/r5u_sgt.log; exit 1; }
tail -1 gpurun_out/r5u_sgt.log
export TRK_C=12288
bash tools/gpu_trk_libab.sh "base" "cs1_int8 rx12_int8 cs1_packed2" 2 1

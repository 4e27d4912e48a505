# Counters at HEAD: sgt (stall + LDS) and the stream kernel at 12288 channels
# (C_s = 1 int8 vs receivers int8: what the HBM stream adds)
set -eu
export TMPDIR=/tmp
bash tools/pmc_kernel.sh r5o_sgt sgt 10
grep -A 30 "sgt_track_kernel<2, true, 64>" gpurun_out/r5o_sgt/summary.txt | head -32
bash tools/gpu_trk_stall.sh r5o_cs1 base cs1_int8 12288
bash tools/gpu_trk_stall.sh r5o_rx12 base rx12_int8 12288

# PMC passes over the tracking bench section, new kernel (V1=0) and round-2 kernel (V1=1)
set -eu
TAG=${1:-tp}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
for V in 0 1; do
  i=0; mkdir -p $O/v$V
  for C in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" ; do
    i=$((i+1))
    GNSSCORR_TRACK_V1=$V timeout -k 10 120 rocprofv3 --pmc $C --output-format csv -d $O/v$V/p$i -o run -- \
      python3 tools/bench_part.py track 10 > $O/v$V/p$i.log 2>&1
  done
  python3 tools/pmc_summary.py $O/v$V $O/pmc_v$V.json | grep track
done

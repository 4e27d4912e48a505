# PMC passes + kernel trace over one bench.py section:
#   bash tools/pmc_kernel.sh <tag> <part> [steps]
# One rocprofv3 run per counter pass (the hardware limits per block; see
# MI355X_MICROARCH.md), each under its own time limit.
set -eu
O=gpurun_out/$1
mkdir -p $O
export TMPDIR=/tmp
B="python3 tools/bench_part.py $2 ${3:-10}"
i=0
for C in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES" \
         "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
         "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/p$i -o run -- $B > $O/p$i.log 2>&1
  echo "pmc pass $i ok"
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- $B > $O/kt.log 2>&1
python3 tools/pmc_summary.py $O $O/summary.json > $O/summary.txt
echo done

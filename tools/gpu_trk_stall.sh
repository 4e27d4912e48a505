# Stall counters of one tracking layout per library build:
# bash tools/gpu_trk_stall.sh <tag> "<lib names>" [layout] [channels]
set -eu
TAG=$1; LIBS=$2; L=${3:-cs1_int8}; CH=${4:-3072}
O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
for V in $LIBS; do
  if [ $V = base ]; then unset GNSSCORR_LIB; else export GNSSCORR_LIB=$PWD/gnss-sdr.ru_amd/ab/libgnsscorr_$V.so; fi
  TRK_C=$CH timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE \
    --output-format csv -d $O/$V -o run -- python3 tools/trk_layout.py $L 20 > $O/$V.log 2>&1
  python3 tools/pmc_summary.py $O/$V $O/stall_$V.json > /dev/null
  python3 - $O/stall_$V.json $V <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for k, m in d.items():
    if "osg_stream" in k:
        w = m["SQ_WAVE_CYCLES"]
        print(sys.argv[2], k, "wait_any %.3f wait_inst %.3f active %.3f valu_insts %.0f lds_stall %.3f gui %.0f" % (
            m["SQ_WAIT_ANY"] / w, m["SQ_WAIT_INST_ANY"] / w, m["SQ_ACTIVE_INST_ANY"] / w,
            m["SQ_INSTS_VALU"], m["SQ_WAIT_INST_LDS"] / w, m["GRBM_GUI_ACTIVE"]))
PY
  tail -1 $O/$V.log
done

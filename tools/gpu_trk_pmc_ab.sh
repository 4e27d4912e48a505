# PMC passes of osg_stream_kernel per tracking build and layout (12288 channels,
# 10-call launches, tools/trk_layout.py):
#   bash tools/gpu_trk_pmc_ab.sh <tag> "<lib names>" [layouts]
# lib name "base" = the in-tree libgnsscorr.so, else ab/libgnsscorr_<name>.so
# (tools/build_ab.sh).  Writes gpurun_out/<tag>/pmc_<layout>_<lib>.json and prints
# VALU / LDS instructions, bank-conflict cycles and wait share per launch.
set -eu
cd ${GRAFT_REPO_ROOT:-.}
TAG=$1
LIBS=$2
LAYOUTS=${3:-"cs1_int8 rx12_int8"}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp TRK_C=${TRK_C:-12288}
for L in $LAYOUTS; do
  for V in $LIBS; do
    if [ $V = base ]; then unset GNSSCORR_LIB; else export GNSSCORR_LIB=$PWD/gnss-sdr.ru_amd/ab/libgnsscorr_$V.so; fi
    D=$O/${L}_$V; mkdir -p $D
    i=0
    for C in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES" \
             "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE" \
             "FETCH_SIZE"; do
      i=$((i+1))
      timeout -k 10 120 rocprofv3 --pmc $C --output-format csv -d $D/p$i -o run -- \
        python3 tools/trk_layout.py $L 20 > $D/p$i.log 2>&1
    done
    python3 tools/pmc_summary.py $D $O/pmc_${L}_$V.json > /dev/null
  done
done
unset GNSSCORR_LIB
python3 - $O <<'PY'
import glob, json, os, sys
for f in sorted(glob.glob(os.path.join(sys.argv[1], "pmc_*.json"))):
    d = json.load(open(f))
    for k, v in d.items():
        if k.startswith("osg_stream_kernel") and isinstance(v, dict) and "SQ_WAVE_CYCLES" in v:
            w = v["SQ_WAVE_CYCLES"]
            print(os.path.basename(f)[4:-5], k[17:], "VALU %.1fM LDS %.1fM conflict %.1fM "
                  "lds_active %.1fM wait/wave %.3f valu_active %.3f fetch %.3f GB" % (
                      v["SQ_INSTS_VALU"] / 1e6, v["SQ_INSTS_LDS"] / 1e6,
                      v["SQ_LDS_BANK_CONFLICT"] / 1e6, v["SQ_LDS_IDX_ACTIVE"] / 1e6,
                      v["SQ_WAIT_ANY"] / w, v["SQ_ACTIVE_INST_VALU"] / w,
                      2 * v.get("FETCH_SIZE", 0) * 1024 / 1e9))
PY

# PMC passes of osg_stream_kernel / osg_track_kernel per layout (one pass per
# counter group, separate runs).  usage (via gpurun): bash tools/gpu_trk_pmc_r4.sh <tag> [layouts] [stream]
set -eu
TAG=${1:-t4}
LAYOUTS=${2:-"cs1_int8 rx12_int8"}
S=${3:-1}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
for L in $LAYOUTS; do
  i=0; D=$O/${L}_s$S; mkdir -p $D
  for C in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE" \
           "FETCH_SIZE"; do
    i=$((i+1))
    GNSSCORR_TRACK_STREAM=$S timeout -k 10 120 rocprofv3 --pmc $C --output-format csv -d $D/p$i -o run -- \
      python3 tools/trk_layout.py $L 20 > $D/p$i.log 2>&1
  done
  python3 tools/pmc_summary.py $D $O/pmc_${L}_s$S.json > /dev/null
  echo "$L s$S: $(grep -h 'kernel ms' $D/p1.log)"
done
python3 - $O <<'PY'
import json, sys, glob, os
for f in sorted(glob.glob(os.path.join(sys.argv[1], "pmc_*.json"))):
    d = json.load(open(f))
    for k, v in d.items():
        if ("osg_track_kernel" in k or "osg_stream_kernel" in k) and isinstance(v, dict):
            w = v["SQ_WAVE_CYCLES"]
            print(os.path.basename(f), k, "VALU %.2fM SALU %.2fM LDS %.2fM wait/wave %.3f waitinst/wave %.3f valu_active/wave %.3f ldsconf %.2fM fetchMB %.1f" % (
                v["SQ_INSTS_VALU"] / 1e6, v["SQ_INSTS_SALU"] / 1e6, v["SQ_INSTS_LDS"] / 1e6,
                v["SQ_WAIT_ANY"] / w, v["SQ_WAIT_INST_ANY"] / w, v["SQ_ACTIVE_INST_VALU"] / w,
                v["SQ_LDS_BANK_CONFLICT"] / 1e6, 2 * v.get("FETCH_SIZE", 0) / 1024))
PY

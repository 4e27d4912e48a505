# Per-layout PMC passes of osg_track_kernel, default kernel (V0) against the round-2 load
# path (GNSSCORR_TRACK_V1=1).  usage (via gpurun): bash tools/gpu_trkpmc2.sh <tag>
set -eu
TAG=${1:-tl}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
for L in cs1_int8 rx12_int8; do
  for V in V0 V1; do
    i=0; D=$O/${L}_$V; mkdir -p $D
    for C in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES" \
             "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE" \
             "FETCH_SIZE"; do
      i=$((i+1))
      env GNSSCORR_TRACK_$V=1 timeout -k 10 120 rocprofv3 --pmc $C --output-format csv -d $D/p$i -o run -- \
        python3 tools/trk_layout.py $L 20 > $D/p$i.log 2>&1
    done
    python3 tools/pmc_summary.py $D $O/pmc_${L}_$V.json > /dev/null
    echo "$L $V: $(grep -h 'kernel ms' $D/p1.log)"
  done
done
python3 - $O <<'PY'
import json, sys, glob, os
for f in sorted(glob.glob(os.path.join(sys.argv[1], "pmc_*.json"))):
    d = json.load(open(f))
    for k, v in d.items():
        if k.startswith("osg_track_kernel") and isinstance(v, dict):
            w = v["SQ_WAVE_CYCLES"]
            print(os.path.basename(f), k, "VALU %.2fM SALU %.2fM wait/wave %.3f valu_active %.3f" % (
                v["SQ_INSTS_VALU"] / 1e6, v["SQ_INSTS_SALU"] / 1e6, v["SQ_WAIT_ANY"] / w,
                v.get("valu_active_per_wave_cycle", 0)))
PY

set -eu
export TMPDIR=/tmp
O=gpurun_out/r6b; mkdir -p $O
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -o /tmp/trk_slots_mb tools/trk_slots_mb.hip 2> /dev/null
timeout -k 10 120 /tmp/trk_slots_mb > $O/slots_mb.log
cat $O/slots_mb.log

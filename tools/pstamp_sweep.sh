# bash tools/prio_sweep.sh "<flags A>" "<flags B>" ... -> pipelined-kernel period per
# build variant of tools/acq_pstamps.hip (e.g. "-DACQ_LDGROUP=8" "-DACQ_LDGROUP=16")
set -e
i=0
for F in "$@"; do
  i=$((i+1))
  echo "== $F"
  PSFLAGS="$F" bash tools/pstamps.sh > gpurun_out/ps_v$i.log 2>&1
  grep period gpurun_out/ps_v$i.log
done

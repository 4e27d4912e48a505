# bash tools/pstamps.sh -> phase shares of the pipelined acquisition kernel (aligned and shifted reads)
set -e
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -DACQ_LDGROUP=${LDG:-16} ${PSFLAGS:-} -Iinclude -Ignss-sdr.ru_amd/csrc \
  -c tools/acq_pstamps.hip -o /tmp/ps.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 /tmp/ps.o gnss-sdr.ru_amd/build/common.c.o -o /tmp/ps
timeout -k 10 60 /tmp/ps
SHIFTED=1 timeout -k 10 60 /tmp/ps

# bash tools/ablate_plane.sh -> acq correlation kernels (one-unit and pipelined) vs the plane stride
set -e
for pl in ${PLANES:-1024 1040 1056 1088}; do
  for k in ${KERNELS:-old pipe}; do for sk in ${SKIPS:-0}; do
    D=""; [ $k = pipe ] && D="-DPIPE"
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -DACQ_PLANE=$pl -DACQ_LDGROUP=${LDG:-8} -DACQ_SKIP=$sk $D -Iinclude \
      -Ignss-sdr.ru_amd/csrc -c tools/acq_ablate.hip -o /tmp/abp.o
    /opt/rocm/bin/hipcc --offload-arch=gfx950 /tmp/abp.o gnss-sdr.ru_amd/build/common.c.o -o /tmp/abp
    timeout -k 10 60 /tmp/abp
  done; done
done

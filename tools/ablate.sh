# bash tools/ablate.sh -> builds and runs acq_ablate for several ACQ_SKIP values
set -e
mkdir -p gpurun_out/ablate
for k in ${SKIPS:-0 4 6 7 1 2}; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -DACQ_SKIP=$k -Iinclude \
    -Ignss-sdr.ru_amd/csrc -c tools/acq_ablate.hip -o /tmp/ab$k.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 /tmp/ab$k.o gnss-sdr.ru_amd/build/common.c.o -o /tmp/ab$k
  timeout -k 10 60 /tmp/ab$k
done

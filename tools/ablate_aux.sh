# cache-policy sweep of the row loads (load phase only, ACQ_SKIP=7, and full)
set -e
mkdir -p gpurun_out/ablate
for aux in 0 1 2 3 16 17; do
  for k in 7 0; do
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -DACQ_SKIP=$k -DACQ_LOAD_AUX=$aux -Iinclude \
      -Ignss-sdr.ru_amd/csrc -c tools/acq_ablate.hip -o /tmp/ab.o 2>/dev/null
    /opt/rocm/bin/hipcc --offload-arch=gfx950 /tmp/ab.o gnss-sdr.ru_amd/build/common.c.o -o /tmp/ab
    echo "aux=$aux"; timeout -k 10 60 /tmp/ab
  done
done

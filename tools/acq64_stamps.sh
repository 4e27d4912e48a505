# bash tools/acq64_stamps.sh -> phase shares of the fp64 correlation kernel
set -e
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 ${S64FLAGS:-} -Iinclude -Ignss-sdr.ru_amd/csrc \
  -c tools/acq64_stamps.hip -o /tmp/s64.o
OBJS=$(ls gnss-sdr.ru_amd/build/*.o | grep -v acq64.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 /tmp/s64.o $OBJS -lpthread -o /tmp/s64
timeout -k 10 60 /tmp/s64

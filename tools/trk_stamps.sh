# bash tools/trk_stamps.sh -> phase times of osg_track_kernel (diagnostic build)
set -e
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -Ignss-sdr.ru_amd/csrc \
  -c tools/trk_stamps.hip -o /tmp/ts.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 /tmp/ts.o gnss-sdr.ru_amd/build/common.c.o \
  gnss-sdr.ru_amd/build/codes.c.o -o /tmp/trk_stamps
timeout -k 10 60 /tmp/trk_stamps 3072
timeout -k 10 60 /tmp/trk_stamps 3072 cs1

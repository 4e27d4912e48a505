# bash tools/trk_stream_stamps.sh -> phase times of osg_stream_kernel (diagnostic build)
set -e
gcc -O2 -fPIC -std=gnu11 -Iinclude -Ignss-sdr.ru_amd/csrc -c gnss-sdr.ru_amd/csrc/common.c -o /tmp/tss_common.o
gcc -O2 -fPIC -std=gnu11 -Iinclude -Ignss-sdr.ru_amd/csrc -c gnss-sdr.ru_amd/csrc/codes.c -o /tmp/tss_codes.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -Ignss-sdr.ru_amd/csrc \
  -c tools/trk_stream_stamps.hip -o /tmp/tss.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 /tmp/tss.o /tmp/tss_common.o /tmp/tss_codes.o -o /tmp/trk_stream_stamps
for B in 1 0; do export GNSSCORR_TRACK_BALANCE=$B; echo balance=$B;
  timeout -k 10 60 /tmp/trk_stream_stamps 3072 cs1
  timeout -k 10 60 /tmp/trk_stream_stamps 3072
done

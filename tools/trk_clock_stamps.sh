# bash tools/trk_clock_stamps.sh -> in-kernel shader clock of osg_stream_kernel
# (diagnostic build, tools/trk_clock_stamps.hip) for C_s = 1 and receiver layouts
set -e
gcc -O2 -fPIC -std=gnu11 -Iinclude -Ignss-sdr.ru_amd/csrc -c gnss-sdr.ru_amd/csrc/common.c -o /tmp/tcs_common.o
gcc -O2 -fPIC -std=gnu11 -Iinclude -Ignss-sdr.ru_amd/csrc -c gnss-sdr.ru_amd/csrc/codes.c -o /tmp/tcs_codes.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Iinclude -Ignss-sdr.ru_amd/csrc -c gnss-sdr.ru_amd/csrc/devmem.hip -o /tmp/tcs_devmem.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -Ignss-sdr.ru_amd/csrc \
  -c tools/trk_clock_stamps.hip -o /tmp/tcs.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 /tmp/tcs.o /tmp/tcs_common.o /tmp/tcs_codes.o \
  /tmp/tcs_devmem.o -o /tmp/trk_clock_stamps
for C in 12288 3072; do
  for Lx in cs1 rx12 cs1 rx12; do timeout -k 10 120 /tmp/trk_clock_stamps $C $Lx 40; done
done

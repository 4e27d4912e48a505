# bash tools/build_ab.sh <name> <source.hip> <extra hipcc flags...>
# builds gnss-sdr.ru_amd/ab/libgnsscorr_<name>.so: the in-tree objects with
# <source> recompiled under the extra flags (A/B builds for GNSSCORR_LIB)
set -e
NAME=$1; SRC=$2; shift 2
make -s -j8 -C gnss-sdr.ru_amd && mkdir -p gnss-sdr.ru_amd/ab
B=gnss-sdr.ru_amd/build
BASE=$(basename $SRC .hip)
EXTRA=""
[ "$BASE" = sgt ] && EXTRA="-mllvm -disable-promote-alloca-to-lds"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Iinclude -Ignss-sdr.ru_amd/csrc $EXTRA "$@" \
  -c gnss-sdr.ru_amd/csrc/$BASE.hip -o /tmp/ab_$BASE.o
OBJS=$(ls $B/*.o | grep -v "/$BASE.o$")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -Wl,-z,now -o gnss-sdr.ru_amd/ab/libgnsscorr_$NAME.so \
  $OBJS /tmp/ab_$BASE.o -lm -lpthread -ldl
echo built gnss-sdr.ru_amd/ab/libgnsscorr_$NAME.so

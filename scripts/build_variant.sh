#!/bin/bash
# Build an experimental libpps_hip.so with extra defines for some source files:
#   scripts/build_variant.sh NAME "SRC1 SRC2" "-DFOO=1 ..."
# -> _variants/libpps_hip_NAME.so (load with PPS_LIB_PATH=...).
set -e
cd "$(dirname "$0")/.."
NAME=$1; SRCS=$2; DEFS=$3
make -s all
mkdir -p _variants
HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -fno-slp-vectorize"
OBJS=$(ls build/*.o)
VOBJS=""
for SRC in $SRCS; do
  /opt/rocm/bin/hipcc $HIPFLAGS $DEFS -c pps_amd/csrc/$SRC.hip -o _variants/$SRC.$NAME.o &
  OBJS=$(echo "$OBJS" | grep -v "/$SRC.o")
  VOBJS="$VOBJS _variants/$SRC.$NAME.o"
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $OBJS $VOBJS -o _variants/libpps_hip_$NAME.so
rm -f $VOBJS
echo _variants/libpps_hip_$NAME.so

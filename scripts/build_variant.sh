#!/bin/bash
# Build an experimental libpps_hip.so with extra defines for one source file:
#   scripts/build_variant.sh NAME SRC "-DFOO=1 ..."
# -> _variants/libpps_hip_NAME.so (load with PPS_LIB_PATH=...).
set -e
cd "$(dirname "$0")/.."
NAME=$1; SRC=$2; DEFS=$3
make -s all
mkdir -p _variants
HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -fno-slp-vectorize"
/opt/rocm/bin/hipcc $HIPFLAGS $DEFS -c pps_amd/csrc/$SRC.hip -o _variants/$SRC.$NAME.o
OBJS=$(ls build/*.o | grep -v "/$SRC.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $OBJS _variants/$SRC.$NAME.o \
  -o _variants/libpps_hip_$NAME.so
echo _variants/libpps_hip_$NAME.so

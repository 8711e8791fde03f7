#!/bin/bash
# build_variant.sh NAME "-DFLAG=..." : libstableavatar_hip.so with gemm.hip compiled with extra flags, into build_ab/NAME/
# (the other objects from build/obj; run the default build first).  Load with SA_LIB=build_ab/NAME/libstableavatar_hip.so
set -eu
cd "$(dirname "$0")/.."
NAME=$1; FLAGS=$2; SRC=${SRC:-gemm}
mkdir -p build_ab/$NAME
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-result -Istableavatar_amd/csrc -Iinclude $FLAGS \
  -c stableavatar_amd/csrc/$SRC.hip -o build_ab/$NAME/$SRC.o
objs=$(ls build/obj/*.o | grep -v "/$SRC.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs build_ab/$NAME/$SRC.o -o build_ab/$NAME/libstableavatar_hip.so
echo built build_ab/$NAME/libstableavatar_hip.so

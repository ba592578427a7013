#!/bin/bash
# A/B engine builds into build/lib_<name>.so with extra defines (CPU side; the box runs them with
# tools/run_ab_lib.sh).  usage: tools/ab_build.sh NAME -DFLAG ...
set -e
cd "$(dirname "$0")/.."
mkdir -p build
name=$1; shift
C=emqx_amd/csrc
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wall -Wno-unused-function \
  -Wno-unused-result "$@" $C/gm_kernels.hip $C/gm_engine.cpp $C/gm_retain.cpp $C/gm_batcher.cpp \
  -o build/lib_$name.so

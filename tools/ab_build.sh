#!/bin/bash
# A/B engine builds into ablib/lib_<name>.so with extra defines (CPU side; the box runs them with
# tools/job.sh ab=...; ablib/ is git-ignored but travels with gpurun).  usage: tools/ab_build.sh NAME -DFLAG ...
set -e
cd "$(dirname "$0")/.."
mkdir -p ablib
name=$1; shift
C=emqx_amd/csrc
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wall -Wno-unused-function \
  -Wno-unused-result "$@" $C/gm_kernels.hip $C/gm_engine.cpp $C/gm_retain.cpp $C/gm_batcher.cpp $C/gm_async.cpp \
  -pthread -o ablib/lib_$name.so

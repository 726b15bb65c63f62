#!/bin/bash
# Builds khipu_amd/libkhst_<name>.so from the working tree with extra compiler flags, for
# same-box A/B runs (scripts/gpu_ab_lib.sh "<name>:KHST_LIB_AB=khipu_amd/libkhst_<name>.so").
# Measurement only.  usage: scripts/build_ab_variant.sh NAME "-DFLAG=..."
set -e
name=$1; shift
root=$(cd "$(dirname "$0")/.." && pwd)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wall -Wno-unused-function \
  -Wno-unknown-pragmas "$@" -o "$root/khipu_amd/libkhst_$name.so" "$root/khipu_amd/csrc/khst.hip"
echo "built khipu_amd/libkhst_$name.so ($*)"

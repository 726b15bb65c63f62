#!/bin/bash
# Builds khipu_amd/libkhst_base.so from a git revision (default HEAD) for same-box A/B runs
# (scripts/gpu_ab_lib.sh "base:KHST_LIB_AB=khipu_amd/libkhst_base.so").  Measurement only.
set -e
rev=${1:-HEAD}
root=$(cd "$(dirname "$0")/.." && pwd)
tmp=$(mktemp -d)
git -C "$root" archive "$rev" khipu_amd/csrc include | tar -x -C "$tmp"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wall -Wno-unused-function \
  -Wno-unknown-pragmas -o "$root/khipu_amd/libkhst_base.so" "$tmp/khipu_amd/csrc/khst.hip"
rm -rf "$tmp"
echo "built khipu_amd/libkhst_base.so from $rev"

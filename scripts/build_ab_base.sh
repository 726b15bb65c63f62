#!/bin/bash
# Builds khipu_amd/libkhst_base.so from a git revision (default HEAD) for same-box A/B runs
# (scripts/gpu_ab_fetch.sh "base=khipu_amd/libkhst_base.so").  Measurement only.  Uses the
# revision's own __graft_entry__.build_lib when it has one with the `out` argument (its units and
# flags), else the single-unit command of earlier revisions.
set -e
rev=${1:-HEAD}
root=$(cd "$(dirname "$0")/.." && pwd)
tmp=$(mktemp -d)
git -C "$root" archive "$rev" khipu_amd/csrc include __graft_entry__.py | tar -x -C "$tmp"
if grep -q "def build_lib(force=False, out=None" "$tmp/__graft_entry__.py"; then
  (cd "$tmp" && python3 -c "import __graft_entry__ as g; g.build_lib(force=True, out='$root/khipu_amd/libkhst_base.so')")
else
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wall -Wno-unused-function \
    -Wno-unknown-pragmas -o "$root/khipu_amd/libkhst_base.so" "$tmp/khipu_amd/csrc/khst.hip"
fi
rm -rf "$tmp"
echo "built khipu_amd/libkhst_base.so from $rev"

#!/bin/bash
# Build A/B variants of libmjx355.so into mujoco-mjx-lab_amd/mjx_amd/variants/ (diagnostic; the
# product library is built by the csrc Makefile). Usage:
#   tools/build_variants.sh [--keep-prev] name1 "flags1" name2 "flags2" ...
# --keep-prev copies the current product library in as variant a_prev first.
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
SRC=$ROOT/mujoco-mjx-lab_amd/csrc
OUT=$ROOT/mujoco-mjx-lab_amd/mjx_amd/variants
mkdir -p "$OUT"
rm -f "$OUT"/*.so
if [ "$1" == "--keep-prev" ]; then
  cp "$ROOT/mujoco-mjx-lab_amd/mjx_amd/libmjx355.so" "$OUT/libmjx355_a_prev.so"
  shift
fi
F="-O2 -std=c++17 -fPIC -shared --offload-arch=gfx950 -Wno-unused-result -fapprox-func -fno-slp-vectorize"
pids=()
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  (cd "$SRC" && /opt/rocm/bin/hipcc $F $flags -o "$OUT/libmjx355_$name.so" capi.hip 2>&1 | grep -E "error" || true) &
  pids+=($!)
done
for p in "${pids[@]}"; do wait "$p"; done
ls "$OUT"

#!/bin/bash
# Build measurement variants of libtwotower_amd.so (extra -D flags) into tools/variants/lib_<name>.so,
# for A/B timing on the GPU box (tools/mb_variants.py).  Usage: tools/build_variants.sh name='-DX=1' ...
set -e
mkdir -p "$(cd "$(dirname "$0")" && pwd)/variants"
ROOT=$(cd "$(dirname "$0")/.." && pwd)
for spec in "$@"; do
  name=${spec%%=*}; flags=${spec#*=}
  make -s -C "$ROOT/twotower_amd/csrc" -j8 BUILD=/tmp/ttvar_$name OUT="$ROOT/tools/variants/lib_$name.so" EXTRA="$flags" \
    2>&1 | grep -v "hip-link" || true
  test -f "$ROOT/tools/variants/lib_$name.so"
  echo "built lib_$name.so [$flags]"
done

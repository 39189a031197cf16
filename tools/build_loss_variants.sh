#!/bin/bash
# Diagnostic builds of the whole library with -D sets (comma-separated) -> tools/_build/lib_<name>.so
set -e
cd "$(dirname "$0")/.."
mkdir -p tools/_build
SRC=normal-clustering-nerf_amd/csrc
for v in "$@"; do
  name=${v//=/_}; name=${name//,/+}
  defs=$(echo "$v" | tr ',' '\n' | sed 's/^/-D/' | tr '\n' ' ')
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -munsafe-fp-atomics $defs \
    $SRC/vren.hip $SRC/field.hip $SRC/loss.hip $SRC/optim.hip $SRC/grid.hip $SRC/distortion.hip $SRC/errors.cpp -o tools/_build/lib_${name,,}.so &
done
wait

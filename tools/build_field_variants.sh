#!/bin/bash
# Diagnostic builds of csrc/field.hip with parts of the backward compiled out (tools/field_probe.py).
set -e
cd "$(dirname "$0")/.."
mkdir -p tools/_build
SRC=normal-clustering-nerf_amd/csrc
for v in "$@"; do
  name=${v//=/_}; name=${name//,/+}
  defs=$(echo "$v" | tr ',' '\n' | sed 's/^/-D/' | tr '\n' ' ')
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -munsafe-fp-atomics -mllvm -amdgpu-kernarg-preload-count=16 $defs \
    $SRC/field.hip $SRC/errors.cpp -o tools/_build/field_${name,,}.so &
done
wait

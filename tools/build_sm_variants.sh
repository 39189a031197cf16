#!/bin/bash
# Variants of the sample-major compositor (csrc/vren.hip with -D knobs) for tools/composite_sm_probe.py.
# Diagnostic builds only; not part of the product.
set -e
cd "$(dirname "$0")/.."
SRC=normal-clustering-nerf_amd/csrc
OUT=tools/_build
mkdir -p $OUT
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -munsafe-fp-atomics -mllvm -amdgpu-kernarg-preload-count=16"
/opt/rocm/bin/hipcc -O2 -std=c++17 -fPIC -c $SRC/errors.cpp -o $OUT/errors.o
build() {  # name, defines
    /opt/rocm/bin/hipcc $FLAGS $2 -c $SRC/vren.hip -o $OUT/vren_sm_$1.o
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $OUT/vren_sm_$1.o $OUT/errors.o -o $OUT/vren_sm_$1.so
}
build base "" &
build nocont "-DSM_DIAG_NOCONT" &
build nostore "-DSM_DIAG_NOSTORE" &
wait
build loadonly "-DSM_DIAG_LOADONLY -DSM_DIAG_NOCOOP" &
build nostore_nocont "-DSM_DIAG_NOSTORE -DSM_DIAG_NOCONT -DSM_DIAG_NOCOOP" &
build nocoop "-DSM_DIAG_NOCOOP" &
wait

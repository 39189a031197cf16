#!/bin/bash
# A/B of library variants (tools/_build/libncnerf_*.so via NCN_LIB_PATH) on the bench step, plus the
# forward-grid probe; one line per variant in gpurun_out/variants.log
mkdir -p gpurun_out
: > gpurun_out/variants.log
SCATTER_PROBE_IDENTITY=1 SCATTER_PROBE_FWD=1 timeout -k 10 200 python tools/scatter_probe.py > gpurun_out/fwd_grid.log 2>&1 || exit $?
for lib in normal-clustering-nerf_amd/ncnerf_amd/libncnerf.so tools/_build/libncnerf_*.so; do
  NCN_LIB_PATH=$PWD/$lib timeout -k 10 200 python bench.py --steps 60 --no-bf16-line --no-extra-states --no-cpu-baseline > gpurun_out/v.log 2>&1 || exit $?
  echo "$lib $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/v.log | head -1)" >> gpurun_out/variants.log
done

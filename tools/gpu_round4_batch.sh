#!/bin/bash
# One gpurun call (round 4): scatter variants probe, the HIP PSNR ensembles (config #1 and #5),
# then the GPU test suite.  Each step under its own time limit; the chain stops at the first failure.
export TMPDIR=/tmp
mkdir -p gpurun_out profiles/round4
SCATTER_PROBE_IDENTITY=1 timeout -k 10 400 python -u tools/scatter_probe.py > gpurun_out/scf32.log 2>&1 && \
timeout -k 10 900 python -u tests/psnr_ensemble.py hip --repeats 3 --out gpurun_out/psnr_hip_ensemble.json \
  > gpurun_out/psnr_hip.log 2>&1 && \
timeout -k 10 600 python -u tests/psnr_ensemble.py hip --repeats 3 --fixture tests/golden/psnr_oracle_ensemble_scannet.json \
  --out gpurun_out/psnr_hip_ensemble_scannet.json > gpurun_out/psnr_hip_scannet.log 2>&1 && \
timeout -k 10 1000 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests -m gpu -p no:cacheprovider \
  > gpurun_out/gpu_tests.log 2>&1

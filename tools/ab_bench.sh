#!/bin/bash
# Step-level A/B of a library variant (NCN_LIB_PATH) against the product library, ABAB order, under
# gpurun from the repo root.  Usage: tools/ab_bench.sh TAG VARIANT.so
export TMPDIR=/tmp
TAG=$1; VAR=$2
mkdir -p gpurun_out
Q="--no-cpu-baseline --no-bf16-line --no-extra-states"
for r in 1 2; do
  timeout -k 10 300 python -u bench.py $Q > gpurun_out/ab_${TAG}_main$r.json 2> gpurun_out/ab_${TAG}_main$r.err || exit $?
  NCN_LIB_PATH=$VAR timeout -k 10 300 python -u bench.py $Q > gpurun_out/ab_${TAG}_var$r.json 2> gpurun_out/ab_${TAG}_var$r.err || exit $?
done

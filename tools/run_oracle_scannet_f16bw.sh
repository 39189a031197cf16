#!/bin/bash
# Config #5 (ScanNet-Manhattan preset) oracle seed ensemble with the HIP kernel's fp16 rounding
# emulated in the MLP forward and the field backward (--emulate fp16 --emulate-bwd), 8 members.
# Workers claim members through marker files, so more workers can be started later:
#   nohup bash tools/run_oracle_scannet_f16bw.sh > /dev/null 2>&1 &
# Test infrastructure; the outputs are the committed fixtures' sources.
cd "$(dirname "$0")/.."
dir=profiles/round4/ensemble_scannet_f16bw
mkdir -p $dir
for m in $(seq 0 7); do
  out=$dir/ref_member$m.json
  mkdir $dir/.claim$m 2>/dev/null || continue  # claimed by another worker
  python tests/psnr_trajectory.py ref --member $m --rays 2048 --steps 1000 --every 125 --impl c --emulate fp16 \
    --emulate-bwd --preset scannet_manhattan --threads 2 --out $out > $dir/ref_member$m.log 2>&1
done

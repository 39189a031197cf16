#!/bin/bash
# The round-4 oracle seed ensembles (CPU, ~40 min per member at 2 threads), 3 members at a time:
#   ensemble_f16bw:         MLP operands AND the field backward's gradients rounded as the HIP kernel's
#                           loss-scaled fp16 chain (--emulate fp16 --emulate-bwd), the device's grid sampling
#   ensemble_f16bw_refsamp: the same with the reference's own grid-refresh draws (--sampling reference)
# Test infrastructure; the outputs are the committed fixtures' sources.
cd "$(dirname "$0")/.."
jobs=()
for m in $(seq 0 11); do
  jobs+=("ensemble_f16bw $m device")
done
for m in $(seq 0 11); do
  jobs+=("ensemble_f16bw_refsamp $m reference")
done
printf '%s\n' "${jobs[@]}" | xargs -P 3 -L 1 bash -c 'dir=$0; m=$1; samp=$2; \
  out=profiles/round4/$dir/ref_member$m.json; [ -s $out ] && grep -q "\"steps\": 1000" $out && exit 0; \
  python tests/psnr_trajectory.py ref --member $m --rays 2048 --steps 1000 --every 125 --impl c --emulate fp16 \
    --emulate-bwd --sampling $samp --threads 2 --out $out > profiles/round4/$dir/ref_member$m.log 2>&1'

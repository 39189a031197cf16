#!/bin/bash
# PMC passes over the bench step (graph replays, 5 timed steps), one counter group per pass:
#   mfma: SQ_VALU_MFMA_BUSY_CYCLES, SQ_BUSY_CU_CYCLES, MFMA op counts (f16), GRBM_GUI_ACTIVE
#   FETCH_SIZE, WRITE_SIZE (separate passes: MI355X_MICROARCH.md PMC slots)
# summarise: python3 tools/pmc_step_summary.py gpurun_out/pmc_step > profiles/<round>/pmc_step.json
export TMPDIR=/tmp
out=gpurun_out/pmc_step
B="python3 bench.py --steps 5 --warmup 3 --no-cpu-baseline --no-bf16-line --no-extra-states"
i=0
for grp in "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_INSTS_VALU_MFMA_F16 GRBM_GUI_ACTIVE GRBM_COUNT" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp --output-format csv -d $out/p$i -o p -- $B > $out.p$i.log 2>&1 || exit $?
done

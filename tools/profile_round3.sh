#!/bin/bash
# Round-3 profile set (under gpurun from the repo root): the bench's kernel trace + stats, the
# composite_fw FETCH/WRITE passes (tools/profile_round.sh) and the per-kernel PMC passes of the
# step (tools/pmc_step.sh); summarise on the CPU side with tools/profile_summary.py round3,
# tools/pmc_step_summary.py gpurun_out/pmc_step and tools/step_timeline.py.
mkdir -p gpurun_out
bash tools/profile_round.sh && bash tools/pmc_step.sh

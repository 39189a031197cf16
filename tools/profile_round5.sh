#!/bin/bash
# Round-5 profile set (under gpurun from the repo root): the bench trace + composite_fw FETCH/WRITE
# passes (tools/profile_round.sh) and the per-kernel PMC passes of the step (tools/pmc_step.sh).
# Summaries on the CPU side: tools/profile_summary.py round5, tools/pmc_step_summary.py,
# tools/step_timeline.py.
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/profile_round.sh && bash tools/pmc_step.sh

#!/bin/bash
# Round-4 profile set (under gpurun from the repo root): the bench trace + composite_fw FETCH/WRITE
# passes (tools/profile_round.sh), the per-kernel PMC passes of the step (tools/pmc_step.sh) and a
# kernel trace of the test-time render of full images (tools/eval_render_probe.py).  Summaries on the
# CPU side: tools/profile_summary.py round4, tools/pmc_step_summary.py, tools/step_timeline.py,
# tools/eval_render_summary.py.
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/profile_round.sh && bash tools/pmc_step.sh && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_eval -o run -- \
  python3 tools/eval_render_probe.py --images 3 > gpurun_out/prof_eval.log 2>&1

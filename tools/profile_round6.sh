#!/bin/bash
# Round-6 validation + profile set (under gpurun from the repo root): the GPU test suite, smoke(),
# the default bench line, then the bench trace + composite_fw FETCH/WRITE passes
# (tools/profile_round.sh) and the per-kernel PMC passes of the step (tools/pmc_step.sh).
# Summaries on the CPU side: tools/profile_summary.py round6, tools/pmc_step_summary.py,
# tools/step_timeline.py.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests -m gpu -p no:cacheprovider \
  > gpurun_out/r6_final_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6_final_smoke.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py > gpurun_out/r6_final_bench.json 2> gpurun_out/r6_final_bench.err || exit $?
bash tools/profile_round.sh && bash tools/pmc_step.sh

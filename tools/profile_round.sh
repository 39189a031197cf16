#!/bin/bash
# Round profile of the bench step (run under gpurun from the repo root):
#   1. rocprofv3 --kernel-trace --stats over bench.py (30 graph-replayed steps)
#   2. FETCH_SIZE and WRITE_SIZE in separate --pmc passes (MI355X_MICROARCH.md: can't share a pass)
# then `python3 tools/profile_summary.py <round>` (on the CPU side) writes profiles/<round>/.
export TMPDIR=/tmp
out=gpurun_out/prof_round
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- \
  python3 bench.py --steps 30 --no-cpu-baseline --no-bf16-line --no-extra-states > $out.trace.log 2>&1 || exit $?
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d $out/$c -o run -- \
    python3 bench.py --steps 5 --no-cpu-baseline --no-bf16-line --no-extra-states > $out.$c.log 2>&1 || exit $?
done

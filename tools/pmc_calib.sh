#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration passes over tools/_build/pmc_calib (tools/pmc_calib.hip), one
# counter per pass, under gpurun from the repo root; summary: python3 tools/pmc_calib_summary.py
export TMPDIR=/tmp
out=gpurun_out/pmc_calib
mkdir -p $out
timeout -k 10 60 ./tools/_build/pmc_calib > $out.plain.log 2>&1 || exit $?
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 60 rocprofv3 --pmc $c --output-format csv -d $out/$c -o run -- ./tools/_build/pmc_calib > $out.$c.log 2>&1 || exit $?
done

#!/bin/bash
# One gpurun call (round 5): scatter A/B (tools/_build/field_*.so beside the product library), the GPU
# test suite, the default bench line.  Each step under its own time limit; the chain stops at the
# first failure.  Usage: tools/gpu_r5_batch.sh TAG [steps...]  (steps: probe tests bench)
export TMPDIR=/tmp
TAG=${1:-a}; shift
STEPS=${*:-probe tests bench}
mkdir -p gpurun_out
for s in $STEPS; do
  case $s in
    probe) SCATTER_PROBE_IDENTITY=1 timeout -k 10 300 python -u tools/scatter_probe.py > gpurun_out/probe_$TAG.log 2>&1 || exit $? ;;
    tests) timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests -m gpu $TESTS_EXTRA \
             -p no:cacheprovider > gpurun_out/gpu_tests_$TAG.log 2>&1 || exit $? ;;
    bench) timeout -k 10 600 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $? ;;
    new) NCN_TRAINED_STATE_RECORD=gpurun_out/trained_state_$TAG.jsonl timeout -k 10 900 python -u -m pytest -v \
             --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu ${NEW_TESTS:-tests/test_gpu_trained_state.py} \
             > gpurun_out/new_tests_$TAG.log 2>&1; rc=$?; [ $rc -le 1 ] || exit $rc ;;  # (test failures: go on)
    plateau) timeout -k 10 600 python -u tools/plateau_probe.py > gpurun_out/plateau_$TAG.log 2>&1 || exit $? ;;
    profile) bash tools/profile_round5.sh || exit $? ;;
    smoke) timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit $? ;;
  esac
done

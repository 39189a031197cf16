set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_split_step.py tests/test_gpu_ddp.py > gpurun_out/split_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 30 --no-bf16-line --no-extra-states --no-cpu-baseline > gpurun_out/bench_split.log 2>&1 && \
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_split -o run -- python3 bench.py --steps 30 --no-cpu-baseline --no-bf16-line --no-extra-states > gpurun_out/prof_split.log 2>&1

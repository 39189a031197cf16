set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_optim.py tests/test_gpu_graph.py > gpurun_out/q_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 30 --no-bf16-line --no-extra-states --no-cpu-baseline > gpurun_out/q_bench.log 2>&1 && \
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_q -o run -- python3 bench.py --steps 30 --no-cpu-baseline --no-bf16-line --no-extra-states > gpurun_out/prof_q.log 2>&1

#!/bin/bash
# One GPU verification pass: kernel/engine tests, smoke, headline bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed $?"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; cat gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/bench_n1.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench_n1.log; exit 1; }
cat gpurun_out/bench_n1.log

#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/gpt2
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { grep -B 30 "Error\|FAILED" gpurun_out/pytest_gpu.log | head -80; exit $rc; }
for M in 1; do
  timeout -k 10 240 python tools/bench_configs.py --config gpt2 --microbatches $M --steps 5 --warmup 2 > gpurun_out/gpt2/m$M.log 2>&1 || { tail -20 gpurun_out/gpt2/m$M.log; exit 1; }
  tail -1 gpurun_out/gpt2/m$M.log
done

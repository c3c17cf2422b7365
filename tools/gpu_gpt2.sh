#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/gpt2
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "layernorm" --timeout 120 --timeout-method thread > gpurun_out/pytest_ln.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_ln.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python tools/bench_configs.py --config gpt2 --steps 5 --warmup 2 > gpurun_out/gpt2/m1.log 2>&1 || { tail -20 gpurun_out/gpt2/m1.log; exit 1; }
tail -1 gpurun_out/gpt2/m1.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/gpt2/prof -o p -- python tools/bench_configs.py --config gpt2 --steps 3 --warmup 2 > gpurun_out/gpt2/prof.log 2>&1 || { tail -20 gpurun_out/gpt2/prof.log; exit 1; }

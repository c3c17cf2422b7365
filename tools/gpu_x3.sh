#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/x3_probe.py > gpurun_out/x3_probe.log 2>&1; rc=$?
cat gpurun_out/x3_probe.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gemm_x3_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_x3.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_x3.log
[ $rc -eq 0 ] || { grep -B5 Error gpurun_out/pytest_x3.log | head -60; exit $rc; }
timeout -k 10 300 python bench.py > gpurun_out/bench_n1_x3.log 2>&1 || { tail -30 gpurun_out/bench_n1_x3.log; exit 1; }
cat gpurun_out/bench_n1_x3.log

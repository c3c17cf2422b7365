#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/u8kb
export TMPDIR=/tmp
L=gpurun_out/u8kb/log.txt
timeout -k 10 300 python -u -m pytest tests/test_gemm_x3_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread -k u8 > $L 2>&1 || { tail -30 $L; exit 1; }
for kb in 32 64; do for d in 0 1; do
  echo "kb=$kb deep=$d" >> $L
  SDML_U8_WGRAD_KB=$kb SDML_X3_DEEP=$d timeout -k 10 120 python tools/bench_u8.py >> $L 2>&1 || { tail $L; exit 1; }
done; done
timeout -k 10 200 python bench.py >> $L 2>&1 || { tail $L; exit 1; }
grep -v amdgpu.ids $L | cut -c1-250

#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/u8ab
export TMPDIR=/tmp
L=gpurun_out/u8ab/log.txt
for d in 1 0; do for w in 1 2; do
  SDML_X3_DEEP=$d SDML_U8_WGRAD_WG_PER_CU=$w timeout -k 10 120 python tools/bench_u8.py >> $L 2>&1 || { tail $L; exit 1; }
done; done
timeout -k 10 300 python -u -m pytest tests/test_gemm_x3_gpu.py -x -q --timeout 120 --timeout-method thread >> $L 2>&1 || { tail -30 $L; exit 1; }
timeout -k 10 200 python bench.py --pixels f32 >> $L 2>&1 || { tail $L; exit 1; }
SDML_X3_DEEP=1 timeout -k 10 200 python bench.py >> $L 2>&1 || { tail $L; exit 1; }
SDML_X3_DEEP=0 SDML_U8_WGRAD_WG_PER_CU=2 timeout -k 10 200 python bench.py >> $L 2>&1 || { tail $L; exit 1; }
timeout -k 10 200 python tools/bench_configs.py --config mlp4x1024 --steps 20 --warmup 3 >> $L 2>&1 || { tail $L; exit 1; }
grep -v amdgpu.ids $L | cut -c1-400

#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/u8tm
export TMPDIR=/tmp
L=gpurun_out/u8tm/log.txt
: > $L
for tm in 1 2; do for d in 0 1; do for w in 1 2; do
  echo "tm=$tm deep=$d wg_per_cu=$w" >> $L
  SDML_U8_WGRAD_TM=$tm SDML_X3_DEEP=$d SDML_U8_WGRAD_WG_PER_CU=$w timeout -k 10 120 python tools/bench_u8.py >> $L 2>&1 || { tail $L; exit 1; }
done; done; done
SDML_U8_WGRAD_TM=1 timeout -k 10 300 python -u -m pytest tests/test_gemm_x3_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread -k u8 >> $L 2>&1 || { tail -30 $L; exit 1; }
grep -v amdgpu.ids $L | cut -c1-200

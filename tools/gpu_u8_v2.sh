#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/u8v2
export TMPDIR=/tmp
L=gpurun_out/u8v2/log.txt
timeout -k 10 300 python -u -m pytest tests/test_gemm_x3_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > $L 2>&1 || { tail -30 $L; exit 1; }
tail -1 $L
timeout -k 10 120 python tools/bench_u8.py >> $L 2>&1 || { tail $L; exit 1; }
timeout -k 10 200 python bench.py >> $L 2>&1 || { tail $L; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE --output-format csv -d gpurun_out/u8v2/p2 -o p2 -- python tools/bench_u8.py > gpurun_out/u8v2/p2.log 2>&1 || { tail gpurun_out/u8v2/p2.log; exit 1; }
python tools/summarize_profile.py pmc $(find gpurun_out/u8v2 -name "*counter_collection.csv") > gpurun_out/u8v2/summary.txt
grep -v amdgpu.ids $L | tail -2 | cut -c1-250
grep -A6 "gemm_x3" gpurun_out/u8v2/summary.txt

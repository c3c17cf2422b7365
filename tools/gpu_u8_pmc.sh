#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/u8pmc
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU --output-format csv -d gpurun_out/u8pmc/p1 -o p1 -- python tools/bench_u8.py > gpurun_out/u8pmc/p1.log 2>&1 || { tail gpurun_out/u8pmc/p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE FETCH_SIZE --output-format csv -d gpurun_out/u8pmc/p2 -o p2 -- python tools/bench_u8.py > gpurun_out/u8pmc/p2.log 2>&1 || { tail gpurun_out/u8pmc/p2.log; exit 1; }
python tools/summarize_profile.py pmc $(find gpurun_out/u8pmc -name "*counter_collection.csv") > gpurun_out/u8pmc/summary.txt
grep -A22 "gemm_x3" gpurun_out/u8pmc/summary.txt | head -60

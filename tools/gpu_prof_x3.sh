#!/bin/bash
set -o pipefail
cd /root/repo; mkdir -p gpurun_out/prof_x3
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU --output-format csv -d gpurun_out/prof_x3/p1 -o p1 -- python tools/x3_prof.py > gpurun_out/prof_x3/p1.log 2>&1 || { tail gpurun_out/prof_x3/p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU FETCH_SIZE --output-format csv -d gpurun_out/prof_x3/p2 -o p2 -- python tools/x3_prof.py > gpurun_out/prof_x3/p2.log 2>&1 || { tail gpurun_out/prof_x3/p2.log; exit 1; }
find gpurun_out/prof_x3 -name "*.csv" | head

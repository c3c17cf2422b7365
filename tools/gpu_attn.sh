#!/bin/bash
# attention microbench + two rocprofv3 counter passes (kernel-trace only, no sys/runtime trace)
set -o pipefail
mkdir -p gpurun_out/attn
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/attn_prof.py > gpurun_out/attn/bench.log 2>&1 || { tail -20 gpurun_out/attn/bench.log; exit 1; }
cat gpurun_out/attn/bench.log
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU --output-format csv -d gpurun_out/attn/pmc1 -o p1 -- python tools/attn_prof.py --iters 2 > gpurun_out/attn/p1.log 2>&1 || { tail gpurun_out/attn/p1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU FETCH_SIZE --output-format csv -d gpurun_out/attn/pmc2 -o p2 -- python tools/attn_prof.py --iters 2 > gpurun_out/attn/p2.log 2>&1 || { tail gpurun_out/attn/p2.log; exit 1; }
find gpurun_out/attn -name "*counter_collection.csv"

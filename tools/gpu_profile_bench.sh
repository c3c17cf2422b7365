#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/profb
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profb/stats -o b -- python bench.py --steps 20 --warmup 5 > gpurun_out/profb/stats.log 2>&1 || { tail -20 gpurun_out/profb/stats.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU --output-format csv -d gpurun_out/profb/pmc1 -o p1 -- python tools/x3_prof.py > gpurun_out/profb/p1.log 2>&1 || { tail gpurun_out/profb/p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS FETCH_SIZE --output-format csv -d gpurun_out/profb/pmc2 -o p2 -- python tools/x3_prof.py > gpurun_out/profb/p2.log 2>&1 || { tail gpurun_out/profb/p2.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profb/gpt2 -o g -- python tools/bench_configs.py --config gpt2 --steps 3 --warmup 2 > gpurun_out/profb/gpt2.log 2>&1 || { tail -20 gpurun_out/profb/gpt2.log; exit 1; }
ls -R gpurun_out/profb | head -30

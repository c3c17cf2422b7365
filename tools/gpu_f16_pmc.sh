#!/bin/bash
# fp16-plane uint8 kernels: headline kernel profile + PMC counter passes over tools/bench_u8.py
set -o pipefail
mkdir -p gpurun_out/pmc16
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pmc16/stats -o b -- python bench.py --steps 20 --warmup 5 > gpurun_out/pmc16/stats.log 2>&1 || { tail -20 gpurun_out/pmc16/stats.log; exit 1; }
f=$(find gpurun_out/pmc16/stats -name "*kernel_stats.csv" | head -1)
python tools/summarize_profile.py stats "$f" 25 > gpurun_out/pmc16/kernel_stats.txt
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU --output-format csv -d gpurun_out/pmc16/p1 -o p1 -- python tools/bench_u8.py > gpurun_out/pmc16/p1.log 2>&1 || { tail gpurun_out/pmc16/p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE FETCH_SIZE --output-format csv -d gpurun_out/pmc16/p2 -o p2 -- python tools/bench_u8.py > gpurun_out/pmc16/p2.log 2>&1 || { tail gpurun_out/pmc16/p2.log; exit 1; }
python tools/summarize_profile.py pmc $(find gpurun_out/pmc16/p1 gpurun_out/pmc16/p2 -name "*counter_collection.csv") > gpurun_out/pmc16/pmc.txt
# the factored weight gradient (u8_wgrad_kernel<true>) next to the dz form
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU --output-format csv -d gpurun_out/pmc16/p3 -o p3 -- python tools/bench_wgrad_dl.py > gpurun_out/pmc16/p3.log 2>&1 || { tail gpurun_out/pmc16/p3.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE FETCH_SIZE --output-format csv -d gpurun_out/pmc16/p4 -o p4 -- python tools/bench_wgrad_dl.py > gpurun_out/pmc16/p4.log 2>&1 || { tail gpurun_out/pmc16/p4.log; exit 1; }
python tools/summarize_profile.py pmc $(find gpurun_out/pmc16/p3 gpurun_out/pmc16/p4 -name "*counter_collection.csv") > gpurun_out/pmc16/pmc_fd.txt
head -12 gpurun_out/pmc16/kernel_stats.txt | cut -c1-140
cat gpurun_out/pmc16/pmc.txt | cut -c1-220 | head -30
cat gpurun_out/pmc16/pmc_fd.txt | cut -c1-220 | head -30

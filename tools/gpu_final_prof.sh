#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/fin
export TMPDIR=/tmp
L=gpurun_out/fin/log.txt
timeout -k 10 300 python -u -m pytest tests/test_gemm_x3_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > $L 2>&1 || { tail -30 $L; exit 1; }
tail -1 $L
timeout -k 10 200 python bench.py >> $L 2>&1 || { tail $L; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fin/stats -o b -- python bench.py --steps 20 --warmup 5 > gpurun_out/fin/stats.log 2>&1 || { tail -20 gpurun_out/fin/stats.log; exit 1; }
f=$(find gpurun_out/fin/stats -name "*kernel_stats.csv" | head -1)
python tools/summarize_profile.py stats "$f" 25 > gpurun_out/fin/kernel_stats.txt
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU --output-format csv -d gpurun_out/fin/p1 -o p1 -- python tools/bench_u8.py > gpurun_out/fin/p1.log 2>&1 || { tail gpurun_out/fin/p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE FETCH_SIZE --output-format csv -d gpurun_out/fin/p2 -o p2 -- python tools/bench_u8.py > gpurun_out/fin/p2.log 2>&1 || { tail gpurun_out/fin/p2.log; exit 1; }
python tools/summarize_profile.py pmc $(find gpurun_out/fin/p1 gpurun_out/fin/p2 -name "*counter_collection.csv") > gpurun_out/fin/pmc.txt
grep -v amdgpu.ids $L | tail -1 | cut -c1-200
head -8 gpurun_out/fin/kernel_stats.txt | cut -c1-140

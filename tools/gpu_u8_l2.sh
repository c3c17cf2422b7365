#!/bin/bash
# L2 hit rate and vector-memory instruction counts of the uint8 GEMMs (one PMC pass, its own run)
set -o pipefail
mkdir -p gpurun_out/u8l2
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU --output-format csv -d gpurun_out/u8l2/p -o p -- python tools/bench_u8.py > gpurun_out/u8l2/p.log 2>&1 || { tail gpurun_out/u8l2/p.log; exit 1; }
python tools/summarize_profile.py pmc $(find gpurun_out/u8l2/p -name "*counter_collection.csv") > gpurun_out/u8l2/pmc.txt
cat gpurun_out/u8l2/pmc.txt

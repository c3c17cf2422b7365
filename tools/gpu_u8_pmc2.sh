#!/bin/bash
# per-kernel time + SQ counters of the uint8 first-layer kernels (tools/bench_u8.py)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/u8pmc
mkdir -p $O
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/st -o st -- python3 tools/bench_u8.py > $O/st.log 2>&1 || { tail $O/st.log; exit 1; }
python tools/summarize_profile.py stats $(find $O/st -name "*kernel_stats.csv" | head -1) 55 | head -12
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU --output-format csv -d $O/p1 -o p1 -- python3 tools/bench_u8.py > $O/p1.log 2>&1 || { tail $O/p1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM_RD FETCH_SIZE --output-format csv -d $O/p2 -o p2 -- python3 tools/bench_u8.py > $O/p2.log 2>&1 || { tail $O/p2.log; exit 1; }
python tools/summarize_profile.py pmc $(find $O/p1 $O/p2 -name "*counter_collection.csv") > $O/pmc.txt
cat $O/pmc.txt

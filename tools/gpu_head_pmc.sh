#!/bin/bash
# SQ counters of the headline step's kernels (bench.py, short run)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/hpmc
mkdir -p $O
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU --output-format csv -d $O/p1 -o p1 -- python3 bench.py --steps 3 --warmup 2 > $O/p1.log 2>&1 || { tail $O/p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM_RD FETCH_SIZE --output-format csv -d $O/p2 -o p2 -- python3 bench.py --steps 3 --warmup 2 > $O/p2.log 2>&1 || { tail $O/p2.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM_WR WRITE_SIZE --output-format csv -d $O/p3 -o p3 -- python3 bench.py --steps 3 --warmup 2 > $O/p3.log 2>&1 || { tail $O/p3.log; exit 1; }
python tools/summarize_profile.py pmc $(find $O/p1 $O/p2 $O/p3 -name "*counter_collection.csv") > $O/pmc.txt
grep -A40 "head_mfma" $O/pmc.txt | head -42

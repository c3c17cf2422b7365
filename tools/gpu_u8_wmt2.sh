#!/bin/bash
# 512-row forward: timing modes + SQ counters (tools/bench_u8.py, SDML_U8_FWD_WMT=4)
set -o pipefail
export TMPDIR=/tmp SDML_U8_FWD_WMT=4
O=gpurun_out/wmt2
mkdir -p $O
for m in 0 1 2 3; do
  SDML_U8_FWD_MODE=$m timeout -k 10 120 python tools/bench_u8.py 2>/dev/null | sed "s/^/mode $m: /" || exit 1
done
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU --output-format csv -d $O/p1 -o p1 -- python3 tools/bench_u8.py > $O/p1.log 2>&1 || { tail $O/p1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM_RD FETCH_SIZE --output-format csv -d $O/p2 -o p2 -- python3 tools/bench_u8.py > $O/p2.log 2>&1 || { tail $O/p2.log; exit 1; }
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC --output-format csv -d $O/p3 -o p3 -- python3 tools/bench_u8.py > $O/p3.log 2>&1 || { tail $O/p3.log; exit 1; }
python tools/summarize_profile.py pmc $(find $O/p1 $O/p2 $O/p3 -name "*counter_collection.csv") > $O/pmc.txt
cat $O/pmc.txt

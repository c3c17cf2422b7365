#!/bin/bash
# per-kernel times of tools/bench_u8.py (the uint8 first-layer kernels)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/u8prof
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gemm_x3_gpu.py -x -q -k u8 --timeout 120 --timeout-method thread 2>&1 | tail -1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/st -o st -- python3 tools/bench_u8.py > $O/st.log 2>&1 || { tail $O/st.log; exit 1; }
python tools/summarize_profile.py stats $(find $O/st -name "*kernel_stats.csv" | head -1) 55 > $O/stats.txt
head -8 $O/stats.txt

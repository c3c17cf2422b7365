#!/bin/bash
# fused head: numerics tests + kernel time inside the headline bench
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/head
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread 2>&1 | tail -2 || exit 1
timeout -k 10 200 python bench.py --steps 50 --warmup 10 2>&1 | grep metric | cut -c1-160 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 5 > $O/prof.log 2>&1 || { tail $O/prof.log; exit 1; }
python tools/summarize_profile.py stats $(find $O/prof -name "*kernel_stats.csv" | head -1) 25 > $O/kstats.txt; head -14 $O/kstats.txt

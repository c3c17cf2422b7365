#!/bin/bash
# uint8 weight-gradient kernel: numerics, kernel timing, headline bench, kernel profile
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/wg3
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gemm_x3_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 120 python tools/bench_u8.py 2>/dev/null || exit 1
timeout -k 10 200 python bench.py --steps 50 --warmup 10 > $O/b.log 2>&1 || { tail $O/b.log; exit 1; }
echo "$(grep -o '"value": [0-9.]*' $O/b.log) $(grep -o '"ms_per_step": [0-9.]*' $O/b.log)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 5 > $O/prof.log 2>&1 || { tail $O/prof.log; exit 1; }
python tools/summarize_profile.py stats $(find $O/prof -name "*kernel_stats.csv" | head -1) 25 > $O/kstats.txt; head -12 $O/kstats.txt | cut -c1-140

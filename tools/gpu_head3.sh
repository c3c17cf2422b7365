#!/bin/bash
# MFMA head at 3 waves per SIMD: numerics, grid-size A/B (SDML_HEAD_BLOCKS), headline bench, profile
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/h3
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py tests/test_gemm_x3_gpu.py -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -1 $O/t.log
for nb in 512 768 1024; do
  SDML_HEAD_BLOCKS=$nb timeout -k 10 200 python bench.py --steps 50 --warmup 10 > $O/b$nb.log 2>&1 || { tail $O/b$nb.log; exit 1; }
  echo "blocks $nb $(grep -o '"value": [0-9.]*' $O/b$nb.log)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 5 > $O/prof.log 2>&1 || { tail $O/prof.log; exit 1; }
python tools/summarize_profile.py stats $(find $O/prof -name "*kernel_stats.csv" | head -1) 25 > $O/kstats.txt; head -12 $O/kstats.txt | cut -c1-140

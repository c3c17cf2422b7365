#!/bin/bash
# MFMA head vs the VALU head (SDML_HEAD=v1): numerics, headline bench A/B, kernel profile
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/hm
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -1 $O/t.log
for h in v1 v2; do
  SDML_HEAD=$h timeout -k 10 200 python bench.py --steps 50 --warmup 10 > $O/b$h.log 2>&1 || { tail $O/b$h.log; exit 1; }
  echo "head $h $(grep -o '"value": [0-9.]*' $O/b$h.log) $(grep -o '"ms_per_step": [0-9.]*' $O/b$h.log)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 5 > $O/prof.log 2>&1 || { tail $O/prof.log; exit 1; }
python tools/summarize_profile.py stats $(find $O/prof -name "*kernel_stats.csv" | head -1) 25 > $O/kstats.txt; head -14 $O/kstats.txt

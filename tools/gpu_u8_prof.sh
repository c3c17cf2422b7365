#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/u8p
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/u8p/stats -o b -- python bench.py --steps 20 --warmup 5 > gpurun_out/u8p/stats.log 2>&1 || { tail -20 gpurun_out/u8p/stats.log; exit 1; }
f=$(find gpurun_out/u8p/stats -name "*kernel_stats.csv" | head -1)
python tools/summarize_profile.py stats "$f" 25 | head -12

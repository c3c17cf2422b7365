#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/u8f
export TMPDIR=/tmp
L=gpurun_out/u8f/log.txt
timeout -k 10 120 python tools/bench_u8.py > $L 2>&1 || { tail $L; exit 1; }
timeout -k 10 200 python bench.py >> $L 2>&1 || { tail $L; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/u8f/stats -o b -- python bench.py --steps 20 --warmup 5 > gpurun_out/u8f/stats.log 2>&1 || { tail -20 gpurun_out/u8f/stats.log; exit 1; }
f=$(find gpurun_out/u8f/stats -name "*kernel_stats.csv" | head -1)
python tools/summarize_profile.py stats "$f" 25 > gpurun_out/u8f/kernel_stats.txt
grep -v amdgpu.ids $L | cut -c1-300
head -12 gpurun_out/u8f/kernel_stats.txt | cut -c1-150

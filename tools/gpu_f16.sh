#!/bin/bash
# fp16-plane uint8 forward: numerics, engine parity, kernel + step timing, kernel profile
set -o pipefail
mkdir -p gpurun_out/f16
export TMPDIR=/tmp
L=gpurun_out/f16/log.txt
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/f16/pytest.log 2>&1 || { tail -40 gpurun_out/f16/pytest.log; exit 1; }
tail -1 gpurun_out/f16/pytest.log
timeout -k 10 120 python tools/bench_u8.py > $L 2>&1 || { tail $L; exit 1; }
timeout -k 10 200 python bench.py >> $L 2>&1 || { tail $L; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/f16/stats -o b -- python bench.py --steps 20 --warmup 5 > gpurun_out/f16/stats.log 2>&1 || { tail -20 gpurun_out/f16/stats.log; exit 1; }
f=$(find gpurun_out/f16/stats -name "*kernel_stats.csv" | head -1)
python tools/summarize_profile.py stats "$f" 25 > gpurun_out/f16/kernel_stats.txt
grep -v amdgpu.ids $L | cut -c1-260
head -12 gpurun_out/f16/kernel_stats.txt | cut -c1-160

#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/head2
export TMPDIR=/tmp
L=gpurun_out/head2/log.txt
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > $L 2>&1 || { tail -30 $L; exit 1; }
tail -1 $L
for i in 1 2; do timeout -k 10 200 python bench.py --steps 100 >> $L 2>&1 || { tail $L; exit 1; }; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/head2/stats -o b -- python bench.py --steps 20 --warmup 5 > gpurun_out/head2/stats.log 2>&1 || { tail -20 gpurun_out/head2/stats.log; exit 1; }
f=$(find gpurun_out/head2/stats -name "*kernel_stats.csv" | head -1)
python tools/summarize_profile.py stats "$f" 25 > gpurun_out/head2/kernel_stats.txt
grep -v amdgpu.ids $L | tail -2 | cut -c1-200
grep head gpurun_out/head2/kernel_stats.txt | cut -c1-120

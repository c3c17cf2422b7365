#!/bin/bash
# ResNet-18 8-stage bf16: throughput + rocprofv3 kernel stats (3 timed steps after 2 warm-up)
set -o pipefail
mkdir -p gpurun_out/resnet
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/bench_configs.py --config resnet18 --steps 5 --warmup 2 > gpurun_out/resnet/m1.log 2>&1 || { tail -20 gpurun_out/resnet/m1.log; exit 1; }
tail -1 gpurun_out/resnet/m1.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/resnet/prof -o p -- python -u tools/bench_configs.py --config resnet18 --steps 3 --warmup 2 > gpurun_out/resnet/prof.log 2>&1 || { tail -20 gpurun_out/resnet/prof.log; exit 1; }
find gpurun_out/resnet/prof -name "*kernel_stats.csv"

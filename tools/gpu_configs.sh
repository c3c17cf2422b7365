#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/configs
export TMPDIR=/tmp
for c in mlp4x1024 resnet18 ref_cnn mlp; do
  timeout -k 10 240 python tools/bench_configs.py --config $c --steps 20 --warmup 3 > gpurun_out/configs/$c.log 2>&1 || { tail -20 gpurun_out/configs/$c.log; exit 1; }
  tail -1 gpurun_out/configs/$c.log
done
timeout -k 10 240 python tools/bench_configs.py --config resnet18 --dtype bf16 --steps 20 --warmup 3 > gpurun_out/configs/resnet18_bf16.log 2>&1 && tail -1 gpurun_out/configs/resnet18_bf16.log

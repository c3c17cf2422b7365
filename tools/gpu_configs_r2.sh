#!/bin/bash
# every BASELINE config on one MI355X (round-2 tree): JSON lines to gpurun_out/configs_r2/all.jsonl
set -o pipefail
mkdir -p gpurun_out/configs_r2
export TMPDIR=/tmp
O=gpurun_out/configs_r2/all.jsonl
: > $O
run() {
  timeout -k 10 300 python tools/bench_configs.py "$@" > gpurun_out/configs_r2/last.log 2>&1 || { tail -20 gpurun_out/configs_r2/last.log; exit 1; }
  grep '^{' gpurun_out/configs_r2/last.log | tail -1 >> $O
  tail -1 $O | cut -c1-220
}
run --config mlp --pixels f32 --steps 50 --warmup 5
run --config ref_cnn --steps 50 --warmup 5
run --config mlp4x1024 --steps 20 --warmup 3
run --config resnet18 --dtype bf16 --steps 20 --warmup 3
run --config gpt2 --steps 10 --warmup 2
timeout -k 10 200 python bench.py --steps 50 --warmup 10 2>/dev/null | grep '^{' >> $O && tail -1 $O | cut -c1-200

#!/bin/bash
# GPT-2 kernel table at HEAD: side stream off (clean per-kernel times) and the default (side stream on)
set -o pipefail
export TMPDIR=/tmp
SDML_WGRAD_STREAM=0 bash tools/gpu.sh stats r6_gpt2_final/serial 300 python3 tools/bench_configs.py --config gpt2 --steps 8 --warmup 3 || exit 1
rm -rf gpurun_out/r6_gpt2_final/serial/raw
bash tools/gpu.sh stats r6_gpt2_final/default 300 python3 tools/bench_configs.py --config gpt2 --steps 8 --warmup 3 || exit 1
f=$(find gpurun_out/r6_gpt2_final/default/raw -name "*kernel_trace.csv" | head -1)
python3 tools/trace_gaps.py "$f" --marker sgd_mixed --steps 5 --top 10 > gpurun_out/r6_gpt2_final/default/gaps.txt
head -3 gpurun_out/r6_gpt2_final/default/gaps.txt
rm -rf gpurun_out/r6_gpt2_final/default/raw

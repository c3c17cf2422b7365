#!/bin/bash
# GPT-2 config at HEAD: kernel stats + device idle gaps over the last 5 steps
set -o pipefail
export TMPDIR=/tmp
bash tools/gpu.sh stats r6_gpt2_gaps 300 python3 tools/bench_configs.py --config gpt2 --steps 8 --warmup 3 || exit 1
f=$(find gpurun_out/r6_gpt2_gaps/raw -name "*kernel_trace.csv" | head -1)
python3 tools/trace_gaps.py "$f" --marker sgd_mixed --steps 5 --top 25 > gpurun_out/r6_gpt2_gaps/gaps.txt
cat gpurun_out/r6_gpt2_gaps/gaps.txt | head -60
rm -rf gpurun_out/r6_gpt2_gaps/raw

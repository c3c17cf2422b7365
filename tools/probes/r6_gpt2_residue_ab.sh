#!/bin/bash
# Round 6: GPT-2 residue cuts (packed int32 token sort; LayerNorm passthrough for each stage's first block):
# GPT-2 / engine / multirank GPU tests, the sort microbenchmark, config runs, serial kernel table
set -o pipefail
export TMPDIR=/tmp
d=gpurun_out/r6_residue
mkdir -p $d
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpt2_ops_gpu.py tests/test_engine_gpu.py tests/test_multirank_gpu.py tests/test_graphs_gpu.py > $d/tests.txt 2>&1 || { tail -30 $d/tests.txt; exit 1; }
tail -1 $d/tests.txt
timeout -k 10 200 python tools/probes/token_sort_ab.py > $d/sort.txt 2>&1 || { tail $d/sort.txt; exit 1; }
grep -v amdgpu.ids $d/sort.txt
for rep in 1 2 3; do
  timeout -k 10 300 python tools/bench_configs.py --config gpt2 > $d/c.log 2>&1 || { tail $d/c.log; exit 1; }
  grep '^{' $d/c.log | tee -a $d/cfg.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['config'], d['value'], d['ms_per_step'], d['loss'])"
done
SDML_WGRAD_STREAM=0 bash tools/gpu.sh stats r6_residue/serial 300 python3 tools/bench_configs.py --config gpt2 --steps 8 --warmup 3 > /dev/null || exit 1
grep -E "add|sort|merge|copy|fill" $d/serial/kernel_stats.txt | cut -c1-130
rm -rf $d/serial/raw

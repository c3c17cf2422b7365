#!/bin/bash
# Round 6: LayerNorm kernels with gamma / beta held in registers and the residual gradient loaded with the row
set -o pipefail
export TMPDIR=/tmp
d=gpurun_out/r6_ln
mkdir -p $d
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpt2_ops_gpu.py tests/test_kernels_gpu.py -k "layernorm or ln or gpt2 or transformer" > $d/tests.txt 2>&1 || { tail -30 $d/tests.txt; exit 1; }
tail -1 $d/tests.txt
SDML_WGRAD_STREAM=0 bash tools/gpu.sh stats r6_ln/serial 300 python3 tools/bench_configs.py --config gpt2 --steps 8 --warmup 3 > /dev/null || exit 1
grep -E "ln_|slab_sum" $d/serial/kernel_stats.txt | cut -c1-120
rm -rf $d/serial/raw
for rep in 1 2; do
  timeout -k 10 300 python tools/bench_configs.py --config gpt2 > $d/c.log 2>&1 || { tail $d/c.log; exit 1; }
  grep '^{' $d/c.log | tee -a $d/cfg.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['config'], d['value'], d['ms_per_step'], d['loss'])"
done

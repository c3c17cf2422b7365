#!/bin/bash
# Round 6: GPT-2 weight gradients on the side stream enqueued before (default) / after the input gradient
# (SDML_LINEAR_WGRAD_AFTER), and the ResNet-18 default (conv weight gradients on the side stream, after)
set -o pipefail
export TMPDIR=/tmp
d=gpurun_out/r6_linear_after
mkdir -p $d
SDML_LINEAR_WGRAD_AFTER=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpt2_ops_gpu.py > $d/tests.txt 2>&1 || { tail -30 $d/tests.txt; exit 1; }
tail -1 $d/tests.txt
: > $d/ab.jsonl
for rep in 1 2 3; do
  for af in 0 1; do
    SDML_LINEAR_WGRAD_AFTER=$af timeout -k 10 300 python tools/bench_configs.py --config gpt2 > $d/c.log 2>&1 || { tail $d/c.log; exit 1; }
    grep '^{' $d/c.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); d['linear_after']=$af; print(json.dumps(d))" | tee -a $d/ab.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['config'], 'after', d['linear_after'], d['value'], d['ms_per_step'], d['loss'])"
  done
  timeout -k 10 300 python tools/bench_configs.py --config resnet18 > $d/c.log 2>&1 || { tail $d/c.log; exit 1; }
  grep '^{' $d/c.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); d['conv_side']='after (default)'; print(json.dumps(d))" | tee -a $d/ab.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['config'], d['conv_side'], d['value'], d['ms_per_step'], d['loss'])"
done

#!/bin/bash
# Round 6: ResNet-18 conv weight gradients on the side stream (operands held to the join), 4 more reps, both orders
set -o pipefail
export TMPDIR=/tmp
d=gpurun_out/r6_conv_side
mkdir -p $d
: > $d/ab.jsonl
for rep in 1 2; do for cs in 1 0 0 1; do
  SDML_CONV_WGRAD_STREAM=$cs timeout -k 10 300 python tools/bench_configs.py --config resnet18 > $d/c.log 2>&1 || { tail $d/c.log; exit 1; }
  grep '^{' $d/c.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); d['conv_side']=$cs; d['hold']=1; print(json.dumps(d))" | tee -a $d/ab.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['config'], 'conv_side', d['conv_side'], d['value'], d['ms_per_step'], d['loss'])"
done; done

#!/bin/bash
# Round 6: side-stream operands held until the join (SDML_SIDE_HOLD=1) instead of record_stream: GPU tests of the
# side-stream paths, then interleaved ResNet-18 (conv weight gradients on the side stream off / on) and GPT-2 (hold 0 / 1)
set -o pipefail
export TMPDIR=/tmp
d=gpurun_out/r6_side_hold
mkdir -p $d
SDML_CONV_WGRAD_STREAM=1 timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_conv_gpu.py tests/test_gpt2_ops_gpu.py tests/test_engine_gpu.py > $d/tests.txt 2>&1 || { tail -30 $d/tests.txt; exit 1; }
tail -1 $d/tests.txt
: > $d/ab.jsonl
for rep in 1 2 3; do
  for cs in 0 1; do
    SDML_CONV_WGRAD_STREAM=$cs timeout -k 10 300 python tools/bench_configs.py --config resnet18 > $d/c.log 2>&1 || { tail $d/c.log; exit 1; }
    grep '^{' $d/c.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); d['conv_side']=$cs; d['hold']=1; print(json.dumps(d))" | tee -a $d/ab.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['config'], 'conv_side', d['conv_side'], d['value'], d['ms_per_step'], d['loss'])"
  done
  for hold in 0 1; do
    SDML_SIDE_HOLD=$hold timeout -k 10 300 python tools/bench_configs.py --config gpt2 > $d/c.log 2>&1 || { tail $d/c.log; exit 1; }
    grep '^{' $d/c.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); d['hold']=$hold; print(json.dumps(d))" | tee -a $d/ab.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['config'], 'hold', d['hold'], d['value'], d['ms_per_step'], d['loss'])"
  done
done

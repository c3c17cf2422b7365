#!/bin/bash
# Round 6: ResNet-18 conv weight gradients on the side stream, enqueued before vs after the input gradient
set -o pipefail
export TMPDIR=/tmp
d=gpurun_out/r6_conv_side_order
mkdir -p $d
SDML_CONV_WGRAD_STREAM=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_conv_gpu.py tests/test_engine_gpu.py > $d/tests.txt 2>&1 || { tail -30 $d/tests.txt; exit 1; }
tail -1 $d/tests.txt
: > $d/ab.jsonl
for rep in 1 2 3 4; do for mode in off before after; do
  case $mode in off) cs=0; af=1 ;; before) cs=1; af=0 ;; after) cs=1; af=1 ;; esac
  SDML_CONV_WGRAD_STREAM=$cs SDML_CONV_WGRAD_AFTER=$af timeout -k 10 300 python tools/bench_configs.py --config resnet18 > $d/c.log 2>&1 || { tail $d/c.log; exit 1; }
  grep '^{' $d/c.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); d['conv_side']='$mode'; print(json.dumps(d))" | tee -a $d/ab.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['config'], d['conv_side'], d['value'], d['ms_per_step'], d['loss'])"
done; done

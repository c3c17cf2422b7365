#!/bin/bash
# Round 6: mixed SGD with two chunks in flight + nontemporal streams (knob SGD_MIXED_V): GPU test, kernel timing by
# rocprof on the GPT-2 config (one SGD launch over 124 M parameters per step), interleaved config A/B
set -o pipefail
export TMPDIR=/tmp
d=gpurun_out/r6_sgd_mixed
mkdir -p $d
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k sgd > $d/tests.txt 2>&1 || { tail -30 $d/tests.txt; exit 1; }
tail -1 $d/tests.txt
for v in 0 1 2; do
  SDML_KNOBS=SGD_MIXED_V=$v bash tools/gpu.sh stats r6_sgd_mixed/stats_v$v 300 python3 tools/bench_configs.py --config gpt2 --steps 8 --warmup 3 > /dev/null || exit 1
  grep sgd_mixed $d/stats_v$v/kernel_stats.txt | cut -c1-120
  rm -rf $d/stats_v$v/raw
done
: > $d/ab.jsonl
for rep in 1 2; do for cfg in gpt2 resnet18; do for v in 0 1 2; do
  SDML_KNOBS=SGD_MIXED_V=$v timeout -k 10 300 python tools/bench_configs.py --config $cfg > $d/c.log 2>&1 || { tail $d/c.log; exit 1; }
  grep '^{' $d/c.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); d['sgd_mixed_v']=$v; print(json.dumps(d))" | tee -a $d/ab.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['config'], 'v', d['sgd_mixed_v'], d['value'], d['ms_per_step'], d['loss'])"
done; done; done

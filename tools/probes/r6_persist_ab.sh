#!/bin/bash
# Round 6: persistent bf16 NT GEMM (knob GEMM_BF16_PERSIST): bit-identity tests, per-shape A/B, GPT-2 config A/B
set -o pipefail
export TMPDIR=/tmp
d=gpurun_out/r6_persist
mkdir -p $d
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpt2_ops_gpu.py -k "persistent or grouped" > $d/tests.txt 2>&1 || { tail -30 $d/tests.txt; exit 1; }
tail -1 $d/tests.txt
[ -n "$SKIP_SHAPES" ] || timeout -k 10 300 python tools/probes/gemm_persist_ab.py > $d/gemm.jsonl 2> $d/err.log || { tail $d/err.log; exit 1; }
[ -n "$SKIP_SHAPES" ] || cat $d/gemm.jsonl | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['gemm'], d['epi'], d['persist0_us'], d['persist1_us'])"
: > $d/ab.jsonl
for rep in 1 2 3; do for v in 0 -1; do
  SDML_KNOBS=GEMM_BF16_PERSIST=$v timeout -k 10 300 python tools/bench_configs.py --config gpt2 > $d/c.log 2>&1 || { tail $d/c.log; exit 1; }
  grep '^{' $d/c.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); d['persist']=$v; print(json.dumps(d))" | tee -a $d/ab.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['config'], 'persist', d['persist'], d['value'], d['ms_per_step'], d['loss'])"
done; done

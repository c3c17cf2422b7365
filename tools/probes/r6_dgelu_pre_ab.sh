#!/bin/bash
# Round 6: gelu'-multiply epilogue with its aux pieces loaded up front: GPT-2 op tests, per-shape timing, GPT-2 config
set -o pipefail
export TMPDIR=/tmp
d=gpurun_out/r6_dgelu_pre
mkdir -p $d
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpt2_ops_gpu.py > $d/tests.txt 2>&1 || { tail -30 $d/tests.txt; exit 1; }
tail -1 $d/tests.txt
timeout -k 10 300 python tools/probes/gemm_persist_ab.py > $d/gemm.jsonl 2> $d/err.log || { tail $d/err.log; exit 1; }
python3 -c "
import json
for l in open('$d/gemm.jsonl'):
    d=json.loads(l); print(d['gemm'], d['epi'], d['persist0_us'], d['persist1_us'])"
for rep in 1 2; do
  timeout -k 10 300 python tools/bench_configs.py --config gpt2 > $d/c.log 2>&1 || { tail $d/c.log; exit 1; }
  grep '^{' $d/c.log | tee -a $d/cfg.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['config'], d['value'], d['ms_per_step'], d['loss'])"
done

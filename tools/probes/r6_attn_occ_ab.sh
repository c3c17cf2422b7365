#!/bin/bash
# Round 6: attention forward register bound for 2 (default) / 3 / 4 waves per SIMD (knob ATTN_OCC): bit-identity
# (flash tests), interleaved attn_prof timings, kernel trace register counts
set -o pipefail
export TMPDIR=/tmp
d=gpurun_out/r6_attn_occ
mkdir -p $d
for o in 3 4; do
  SDML_KNOBS=ATTN_OCC=$o timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k flash > $d/tests_$o.txt 2>&1 || { tail -30 $d/tests_$o.txt; exit 1; }
  tail -1 $d/tests_$o.txt
done
: > $d/ab.jsonl
for r in 1 2 3; do for o in 2 3 4; do
  SDML_KNOBS=ATTN_OCC=$o timeout -k 10 120 python tools/attn_prof.py --iters 20 | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); d['attn_occ']=$o; print(json.dumps(d))" >> $d/ab.jsonl 2> $d/err.log || { tail $d/err.log; exit 1; }
done; done
python3 -c "
import json
for l in open('$d/ab.jsonl'):
    d=json.loads(l); print(d['attn_occ'], {k: v for k, v in d.items() if 'fwd' in k})"
for o in 2 3; do
  SDML_KNOBS=ATTN_OCC=$o STEPS=21 bash tools/gpu.sh stats r6_attn_occ/occ$o 120 python3 tools/attn_prof.py --iters 20 | grep -i "attn_fwd" | cut -c1-120
  f=$(find $d/occ$o/raw -name "*kernel_trace.csv" | head -1)
  python3 -c "
import csv
seen=set()
for r in csv.DictReader(open('$f')):
    n=r.get('Kernel_Name','')
    if 'attn_fwd' in n and n not in seen:
        seen.add(n); print({k: r[k] for k in r if 'VGPR' in k or 'Vgpr' in k or 'vgpr' in k or 'LDS' in k or 'Scratch' in k}, n[:60])"
  rm -rf $d/occ$o/raw
done

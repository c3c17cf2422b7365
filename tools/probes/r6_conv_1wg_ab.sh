#!/bin/bash
# Round 6: halo conv with one workgroup per CU (knob CONV_HALO_1WG) vs two: ResNet-18 per-kernel times and config
set -o pipefail
export TMPDIR=/tmp
d=gpurun_out/r6_conv_1wg
mkdir -p $d
for v in 0 1; do
  SDML_KNOBS=CONV_HALO_1WG=$v bash tools/gpu.sh stats r6_conv_1wg/v$v 300 python3 tools/bench_configs.py --config resnet18 --steps 10 --warmup 4 > /dev/null || exit 1
  grep -E "halo" $d/v$v/kernel_stats.txt | cut -c1-110
  rm -rf $d/v$v/raw
done
for rep in 1 2; do for v in 0 1; do
  SDML_KNOBS=CONV_HALO_1WG=$v timeout -k 10 300 python tools/bench_configs.py --config resnet18 > $d/c.log 2>&1 || { tail $d/c.log; exit 1; }
  grep '^{' $d/c.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); d['halo_1wg']=$v; print(json.dumps(d))" | tee -a $d/ab.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['config'], '1wg', d['halo_1wg'], d['value'], d['ms_per_step'], d['loss'])"
done; done

set -o pipefail
for cfg in resnet18 gpt2 mlp4x1024; do
  for g in none direct; do
    arg=""; [ $g != none ] && arg="--graph $g"
    timeout -k 10 300 python tools/bench_configs.py --config $cfg --steps 20 --warmup 4 $arg > gpurun_out/cfgg_${cfg}_$g.log 2>&1 || { tail -5 gpurun_out/cfgg_${cfg}_$g.log; exit 1; }
    echo "$cfg $g $(grep '^{' gpurun_out/cfgg_${cfg}_$g.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['loss'])")"
  done
done

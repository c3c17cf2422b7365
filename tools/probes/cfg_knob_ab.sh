# same-box A/B of knob sets on a bench_configs config: CFG=resnet18 tools/probes/cfg_knob_ab.sh "<KNOBS a>" "<KNOBS b>" ...
set -o pipefail
: > gpurun_out/${CFG}_knob_ab.jsonl
for rep in 1 2; do for k in "" "$@"; do
  SDML_KNOBS="$k" timeout -k 10 300 python tools/bench_configs.py --config "$CFG" --steps 20 --warmup 4 > gpurun_out/gk.log 2>&1 || { tail gpurun_out/gk.log; exit 1; }
  grep '^{' gpurun_out/gk.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); d['knobs']='$k'; print(json.dumps(d))" | tee -a gpurun_out/${CFG}_knob_ab.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(repr(d['knobs']), d['value'], d['ms_per_step'], d['loss'])"
done; done

# same-box A/B of knob sets on the GPT-2 step: tools/probes/gpt2_knob_ab.sh "<KNOBS a>" "<KNOBS b>" ...
set -o pipefail
: > gpurun_out/gpt2_knob_ab.jsonl
for rep in 1 2; do for k in "" "$@"; do
  SDML_KNOBS="$k" timeout -k 10 300 python tools/bench_configs.py --config gpt2 --steps 10 --warmup 3 > gpurun_out/gk.log 2>&1 || { tail gpurun_out/gk.log; exit 1; }
  grep '^{' gpurun_out/gk.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); d['knobs']='$k'; print(json.dumps(d))" | tee -a gpurun_out/gpt2_knob_ab.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(repr(d['knobs']), d['value'], d['ms_per_step'], d['loss'])"
done; done

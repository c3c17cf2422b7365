# same-box A/B of one knob on bench.py: tools/probes/knob_ab.sh "<KNOBS for new>" [rounds] [steps] [warmup]
set -o pipefail
knobs=$1; rounds=${2:-3}; steps=${3:-200}; warmup=${4:-10}
mkdir -p gpurun_out
: > gpurun_out/knob_ab.jsonl
for i in $(seq 1 "$rounds"); do
  for b in base new; do
    if [ $b = base ]; then k=""; else k="$knobs"; fi
    SDML_KNOBS="$k" timeout -k 10 120 python bench.py --gpus 1 --steps "$steps" --warmup "$warmup" > /tmp/kab.log 2>&1 || { tail -20 /tmp/kab.log; exit 1; }
    grep '^{' /tmp/kab.log | tail -1 | python -c "import sys, json; d = json.loads(sys.stdin.read()); d['build'] = '$b'; print(json.dumps(d))" >> gpurun_out/knob_ab.jsonl
  done
done
python - <<'PY'
import json, statistics
rows = [json.loads(l) for l in open("gpurun_out/knob_ab.jsonl")]
for b in ("base", "new"):
    ms = [r["ms_per_step"] for r in rows if r["build"] == b]
    med = [r["step_ms_events"]["median"] for r in rows if r["build"] == b]
    print(b, "ms_per_step", ms, "median step", round(statistics.median(med), 4))
PY

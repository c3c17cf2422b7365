#!/bin/bash
# A/B of two builds of _kernels on ONE box (box-to-box clock differences are larger than most kernel changes):
#   tools/ab_bench.sh <base.so> <new.so> [rounds=3] [steps=200] [warmup=10]
# alternates the two .so files under the package name and runs bench.py; one JSON line per run in
# gpurun_out/ab.jsonl with "build": "base" | "new" added. Each run under its own time limit; stops on the first failure.
set -o pipefail
base=$1; new=$2; rounds=${3:-3}; steps=${4:-200}; warmup=${5:-10}
pkg=simple_distributed_machine_learning_amd/_kernels.cpython-310-x86_64-linux-gnu.so
mkdir -p gpurun_out
cp "$pkg" /tmp/ab_orig.so
: > gpurun_out/ab.jsonl
for i in $(seq 1 "$rounds"); do
  for b in base new; do
    if [ "$b" = base ]; then cp "$base" "$pkg"; else cp "$new" "$pkg"; fi
    timeout -k 10 120 python bench.py --gpus 1 --steps "$steps" --warmup "$warmup" > /tmp/ab_run.log 2>&1 || {
      tail -20 /tmp/ab_run.log; cp /tmp/ab_orig.so "$pkg"; exit 1; }
    grep '^{' /tmp/ab_run.log | tail -1 | python -c "import sys, json; d = json.loads(sys.stdin.read()); d['build'] = '$b'; print(json.dumps(d))" >> gpurun_out/ab.jsonl
  done
done
cp /tmp/ab_orig.so "$pkg"
python - <<'PY'
import json, statistics
rows = [json.loads(l) for l in open("gpurun_out/ab.jsonl")]
for b in ("base", "new"):
    ms = [r["ms_per_step"] for r in rows if r["build"] == b]
    med = [r["step_ms_events"]["median"] for r in rows if r["build"] == b]
    print(b, "ms_per_step", ms, "median step", round(statistics.median(med), 4))
PY

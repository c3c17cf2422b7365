# Full GPU check: every GPU test, the driver's bench, every BASELINE config (one JSON line each).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
tools/gpu.sh test 700 tests -m gpu || exit 1
tools/gpu.sh run bench 200 python bench.py --steps 50 --warmup 10 || exit 1
: > gpurun_out/configs.jsonl
for c in mlp ref_cnn mlp4x1024 resnet18 gpt2; do
  timeout -k 10 200 python tools/bench_configs.py --config $c > gpurun_out/cfg_$c.log 2>&1 || exit 1
  grep '^{' gpurun_out/cfg_$c.log | tail -1 | tee -a gpurun_out/configs.jsonl | cut -c1-300
done

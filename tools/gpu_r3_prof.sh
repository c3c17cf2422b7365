# rocprofv3 kernel tables of the configs the README quotes (one call)
set -o pipefail
export TMPDIR=/tmp
tools/gpu.sh stats ref_cnn 200 python tools/bench_configs.py --config ref_cnn --steps 30 --warmup 5 || exit 1
tools/gpu.sh stats resnet 200 python tools/bench_configs.py --config resnet18 --steps 10 --warmup 3 || exit 1
tools/gpu.sh stats gpt2 300 python tools/bench_configs.py --config gpt2 --steps 5 --warmup 2 || exit 1
tools/gpu.sh stats mlp60 200 python tools/bench_configs.py --config mlp --steps 30 --warmup 5 || exit 1

# kernel stats of the GPT-2 and ResNet-18 steps at HEAD (10 + 3 and 10 + 4 steps; 13 / 14 steps profiled)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_gpt2 -o run -- python3 tools/bench_configs.py --config gpt2 --steps 10 --warmup 3 > gpurun_out/prof_gpt2.log 2>&1 || { tail -20 gpurun_out/prof_gpt2.log; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_resnet -o run -- python3 tools/bench_configs.py --config resnet18 --steps 10 --warmup 4 > gpurun_out/prof_resnet.log 2>&1 || { tail -20 gpurun_out/prof_resnet.log; exit 1; }
find gpurun_out/prof_gpt2 gpurun_out/prof_resnet -name "*kernel_stats.csv"

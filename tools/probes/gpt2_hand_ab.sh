set -o pipefail
for rep in 1 2; do for m in lib hand; do
  SDML_GPT2_GEMM=$m timeout -k 10 300 python tools/bench_configs.py --config gpt2 --steps 10 --warmup 3 > gpurun_out/gpt2_$m$rep.log 2>&1 || { tail gpurun_out/gpt2_$m$rep.log; exit 1; }
  echo "$m $(grep '^{' gpurun_out/gpt2_$m$rep.log | cut -c180-330)"
done; done
SDML_GPT2_GEMM=hand bash tools/gpu.sh stats gpt2hand 300 python tools/bench_configs.py --config gpt2 --steps 5 --warmup 2

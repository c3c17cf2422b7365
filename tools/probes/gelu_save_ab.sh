# A/B: c_fc forward saving gelu'(U) (SDML_GELU_SAVE=grad) vs U (=u), same .so, same box; GPT-2 bench_configs
set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpt2_ops_gpu.py tests/test_engine_gpu.py -k "gelu or gemm_bf16 or mlp or gpt2" > gpurun_out/gs_tests.log 2>&1 || { tail -30 gpurun_out/gs_tests.log; exit 1; }
tail -1 gpurun_out/gs_tests.log
for rep in 1 2; do for m in u grad; do
  SDML_GELU_SAVE=$m timeout -k 10 300 python tools/bench_configs.py --config gpt2 --steps 10 --warmup 3 > gpurun_out/gs_gpt2_$m$rep.log 2>&1 || { tail gpurun_out/gs_gpt2_$m$rep.log; exit 1; }
  echo "$m $(grep '^{' gpurun_out/gs_gpt2_$m$rep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['loss'])")"
done; done

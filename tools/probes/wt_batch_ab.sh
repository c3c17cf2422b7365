set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpt2_ops_gpu.py tests/test_engine_gpu.py -k "transpose or wt_cache or gpt2" > gpurun_out/wt_tests.log 2>&1 || { tail -30 gpurun_out/wt_tests.log; exit 1; }
tail -1 gpurun_out/wt_tests.log
pkg=simple_distributed_machine_learning_amd/_kernels.cpython-310-x86_64-linux-gnu.so
for rep in 1 2; do
  git_stash=0
  timeout -k 10 300 python tools/bench_configs.py --config gpt2 --steps 10 --warmup 3 > gpurun_out/wt_gpt2_new$rep.log 2>&1 || { tail gpurun_out/wt_gpt2_new$rep.log; exit 1; }
  echo "new $(grep '^{' gpurun_out/wt_gpt2_new$rep.log | cut -c240-330)"
  SDML_WT_BATCH=0 timeout -k 10 300 python tools/bench_configs.py --config gpt2 --steps 10 --warmup 3 > gpurun_out/wt_gpt2_old$rep.log 2>&1 || { tail gpurun_out/wt_gpt2_old$rep.log; exit 1; }
  echo "old $(grep '^{' gpurun_out/wt_gpt2_old$rep.log | cut -c240-330)"
done

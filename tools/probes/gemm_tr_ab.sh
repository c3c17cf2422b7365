set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpt2_ops_gpu.py -k "transposed or 192" > gpurun_out/tr_tests.log 2>&1 || { tail -30 gpurun_out/tr_tests.log; exit 1; }
tail -1 gpurun_out/tr_tests.log
for tr in 0 1; do
  SDML_KNOBS=GEMM_BF16_TR=$tr timeout -k 10 200 python tools/bench_gemm_bf16.py > gpurun_out/tr_gemm_$tr.log 2>&1 || { tail gpurun_out/tr_gemm_$tr.log; exit 1; }
done
for rep in 1 2; do for tr in 0 1; do
  SDML_KNOBS=GEMM_BF16_TR=$tr timeout -k 10 300 python tools/bench_configs.py --config gpt2 --steps 10 --warmup 3 > gpurun_out/tr_gpt2_$tr$rep.log 2>&1 || { tail gpurun_out/tr_gpt2_$tr$rep.log; exit 1; }
  echo "tr=$tr $(grep '^{' gpurun_out/tr_gpt2_$tr$rep.log | cut -c240-330)"
done; done

set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpt2_ops_gpu.py -k "prefetched or transposed or 192" > gpurun_out/upf_tests.log 2>&1 || { tail -30 gpurun_out/upf_tests.log; exit 1; }
tail -1 gpurun_out/upf_tests.log
for rep in 1 2; do for k in 0 1; do
  SDML_KNOBS=GEMM_BF16_UPF=$k timeout -k 10 300 python tools/bench_configs.py --config gpt2 --steps 10 --warmup 3 > gpurun_out/upf_$k$rep.log 2>&1 || { tail -5 gpurun_out/upf_$k$rep.log; exit 1; }
  echo "upf=$k $(grep '^{' gpurun_out/upf_$k$rep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['loss'])")"
done; done

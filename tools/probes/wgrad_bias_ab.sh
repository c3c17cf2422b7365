set -o pipefail
pkg=simple_distributed_machine_learning_amd/_kernels.cpython-310-x86_64-linux-gnu.so
cp $pkg /tmp/orig.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpt2_ops_gpu.py > gpurun_out/wgb_tests.log 2>&1 || { tail -30 gpurun_out/wgb_tests.log; exit 1; }
tail -1 gpurun_out/wgb_tests.log
for rep in 1 2; do for b in base new; do
  cp exp/${b}_kernels.so $pkg
  timeout -k 10 200 python tools/bench_gpt2_gemms.py > gpurun_out/wgb_$b$rep.log 2>&1 || { tail gpurun_out/wgb_$b$rep.log; cp /tmp/orig.so $pkg; exit 1; }
  echo "$b $rep"; grep -o "dW wgrad_bf16 (HIP): [0-9.]*us\|dW+db wgrad_bf16 (HIP): [0-9.]*us" gpurun_out/wgb_$b$rep.log | tr '\n' ' '; echo
done; done
cp /tmp/orig.so $pkg

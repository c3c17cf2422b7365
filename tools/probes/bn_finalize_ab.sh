set -o pipefail
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_conv_gpu.py tests/test_engine_gpu.py -k "bn or batch or resnet or conv" > gpurun_out/bn_tests.log 2>&1 || { tail -30 gpurun_out/bn_tests.log; exit 1; }
tail -1 gpurun_out/bn_tests.log
pkg=simple_distributed_machine_learning_amd/_kernels.cpython-310-x86_64-linux-gnu.so
cp $pkg /tmp/orig.so
for rep in 1 2; do for b in base new; do
  cp exp/${b}_kernels.so $pkg
  timeout -k 10 300 python tools/bench_configs.py --config resnet18 --steps 20 --warmup 4 > gpurun_out/bnab_$b$rep.log 2>&1 || { tail -5 gpurun_out/bnab_$b$rep.log; cp /tmp/orig.so $pkg; exit 1; }
  echo "$b $(grep '^{' gpurun_out/bnab_$b$rep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['loss'])")"
done; done
cp /tmp/orig.so $pkg

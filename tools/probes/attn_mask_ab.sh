set -o pipefail
pkg=simple_distributed_machine_learning_amd/_kernels.cpython-310-x86_64-linux-gnu.so
cp $pkg /tmp/orig.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attn or attention or flash" > gpurun_out/att_tests.log 2>&1 || { tail -30 gpurun_out/att_tests.log; exit 1; }
tail -1 gpurun_out/att_tests.log
for rep in 1 2; do for b in base new; do
  cp exp/${b}_kernels.so $pkg
  timeout -k 10 120 python tools/bench_attention.py --B 16 > gpurun_out/attab_$b$rep.log 2>&1 || { tail gpurun_out/attab_$b$rep.log; cp /tmp/orig.so $pkg; exit 1; }
  echo "$b $rep $(grep '^{' gpurun_out/attab_$b$rep.log | tail -1 | cut -c1-260)"
done; done
cp /tmp/orig.so $pkg

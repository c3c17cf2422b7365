set -o pipefail
pkg=simple_distributed_machine_learning_amd/_kernels.cpython-310-x86_64-linux-gnu.so
cp $pkg /tmp/orig.so
for i in 1 2; do for b in base new; do
  cp exp/${b}_kernels.so $pkg
  timeout -k 10 120 python tools/bench_attention.py --B 16 > gpurun_out/attn_$b$i.log 2>&1 || { tail gpurun_out/attn_$b$i.log; cp /tmp/orig.so $pkg; exit 1; }
  echo "$b $i $(grep '^{' gpurun_out/attn_$b$i.log | tail -3 | tr '\n' ' ' | cut -c1-400)"
done; done
cp /tmp/orig.so $pkg

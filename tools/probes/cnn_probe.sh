set -o pipefail
PYTHONPATH=. timeout -k 10 200 python tools/probes/host_cnn.py > gpurun_out/host_cnn.txt 2>&1 || { tail -20 gpurun_out/host_cnn.txt; exit 1; }
for g in none copy direct; do
  arg=""; [ $g != none ] && arg="--graph $g"
  timeout -k 10 120 python tools/bench_configs.py --config ref_cnn --steps 400 --warmup 20 $arg > gpurun_out/cnn_$g.log 2>&1 || { tail gpurun_out/cnn_$g.log; exit 1; }
  grep '^{' gpurun_out/cnn_$g.log | cut -c1-400
done

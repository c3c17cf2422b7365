set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_small_step_gpu.py tests/test_graphs_gpu.py > gpurun_out/cnn_tests.log 2>&1 || { tail -30 gpurun_out/cnn_tests.log; exit 1; }
tail -1 gpurun_out/cnn_tests.log
PYTHONPATH=. timeout -k 10 200 python tools/probes/host_cnn.py > gpurun_out/host_cnn2.txt 2>&1 || { tail -20 gpurun_out/host_cnn2.txt; exit 1; }
grep "host us" gpurun_out/host_cnn2.txt | cut -c1-200
for rep in 1 2; do
  timeout -k 10 120 python tools/bench_configs.py --config ref_cnn --steps 400 --warmup 20 > gpurun_out/cnn_e$rep.log 2>&1 || { tail gpurun_out/cnn_e$rep.log; exit 1; }
  grep '^{' gpurun_out/cnn_e$rep.log | cut -c200-330
  timeout -k 10 120 python tools/bench_configs.py --config ref_cnn --steps 400 --warmup 20 --graph direct > gpurun_out/cnn_g$rep.log 2>&1 || { tail gpurun_out/cnn_g$rep.log; exit 1; }
  grep '^{' gpurun_out/cnn_g$rep.log | cut -c200-330
done

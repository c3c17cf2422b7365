set -o pipefail
for rep in 1 2; do
timeout -k 10 120 python tools/bench_dp_split.py --steps 200 --warmup 10 --modes 0 > gpurun_out/dpg_e$rep.log 2>&1 || { tail gpurun_out/dpg_e$rep.log; exit 1; }
grep '^{' gpurun_out/dpg_e$rep.log
timeout -k 10 120 python tools/bench_dp_split.py --steps 200 --warmup 10 --modes 0 --graph > gpurun_out/dpg_g$rep.log 2>&1 || { tail gpurun_out/dpg_g$rep.log; exit 1; }
grep '^{' gpurun_out/dpg_g$rep.log
done
timeout -k 10 120 python bench.py --steps 200 --warmup 10 > gpurun_out/dpg_n1.log 2>&1 || { tail gpurun_out/dpg_n1.log; exit 1; }
grep '^{' gpurun_out/dpg_n1.log | cut -c1-200

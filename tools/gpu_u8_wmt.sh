#!/bin/bash
# forward rows-per-wave A/B (SDML_U8_FWD_WMT = 32-row MFMA tiles per wave): numerics at both
# geometries, kernel timing, headline bench
set -o pipefail
O=gpurun_out/wmt
mkdir -p $O
for w in 2 4; do
  SDML_U8_FWD_WMT=$w timeout -k 10 300 python -u -m pytest tests/test_gemm_x3_gpu.py tests/test_engine_gpu.py -x -q -k u8 --timeout 120 --timeout-method thread > $O/t$w.log 2>&1 || { tail -30 $O/t$w.log; exit 1; }
  tail -1 $O/t$w.log
done
for w in 2 4; do
  SDML_U8_FWD_WMT=$w timeout -k 10 120 python tools/bench_u8.py 2>&1 | sed "s/^/wmt$w: /" || exit 1
done
for w in 2 4; do
  SDML_U8_FWD_WMT=$w timeout -k 10 200 python bench.py --steps 50 --warmup 10 > $O/b$w.log 2>&1 || { tail $O/b$w.log; exit 1; }
  echo "wmt$w $(grep -o '"value": [0-9.]*, "unit[^,]*, "n_gpus": 1, "steps": 50, "warmup": 10, "ms_per_step": [0-9.]*' $O/b$w.log)"
done

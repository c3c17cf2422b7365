#!/bin/bash
# weight-gradient A/B: staging registers single vs double buffered (SDML_U8_WG_DB)
set -o pipefail
O=gpurun_out/wgdb
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gemm_x3_gpu.py -x -q -k wgrad --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
SDML_U8_WG_DB=1 timeout -k 10 300 python -u -m pytest tests/test_gemm_x3_gpu.py -x -q -k wgrad --timeout 120 --timeout-method thread >> $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
grep passed $O/t.log
for d in 0 1 0 1; do
  SDML_U8_WG_DB=$d timeout -k 10 120 python tools/bench_u8.py 2>/dev/null | sed "s/^/db$d: /" || exit 1
done
for d in 0 1; do
  SDML_U8_WG_DB=$d timeout -k 10 200 python bench.py --steps 50 --warmup 10 > $O/b$d.log 2>&1 || { tail $O/b$d.log; exit 1; }
  echo "db$d $(grep -o '"value": [0-9.]*' $O/b$d.log)"
done

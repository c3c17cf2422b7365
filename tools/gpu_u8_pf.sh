#!/bin/bash
# forward A/B: rows per wave (SDML_U8_FWD_WMT) x fragment prefetch (SDML_U8_FWD_PF)
set -o pipefail
O=gpurun_out/pf
mkdir -p $O
SDML_U8_FWD_PF=1 SDML_U8_FWD_WMT=4 timeout -k 10 300 python -u -m pytest tests/test_gemm_x3_gpu.py -x -q -k u8 --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for w in 2 4; do for pf in 0 1; do
  SDML_U8_FWD_PF=$pf SDML_U8_FWD_WMT=$w timeout -k 10 120 python tools/bench_u8.py 2>/dev/null | sed "s/^/wmt$w pf$pf: /" || exit 1
done; done
for w in 2 4; do for pf in 0 1; do
  SDML_U8_FWD_PF=$pf SDML_U8_FWD_WMT=$w timeout -k 10 200 python bench.py --steps 50 --warmup 10 > $O/b$w$pf.log 2>&1 || { tail $O/b$w$pf.log; exit 1; }
  echo "wmt$w pf$pf $(grep -o '"value": [0-9.]*' $O/b$w$pf.log) $(grep -o '"ms_per_step": [0-9.]*' $O/b$w$pf.log)"
done; done

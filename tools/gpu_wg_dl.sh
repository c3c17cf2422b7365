#!/bin/bash
# factored-gradient weight gradient: bit-identity tests, fused vs unfused timing, headline bench
set -o pipefail
O=gpurun_out/wgdl
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gemm_x3_gpu.py -k factor -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 120 python tools/bench_wgrad_dl.py 2>/dev/null || exit 1
timeout -k 10 200 python bench.py --steps 50 --warmup 10 > $O/b.log 2>&1 || { tail $O/b.log; exit 1; }
grep -o '"value": [0-9.]*' $O/b.log

#!/bin/bash
# new LDS-DMA uint8 forward: numerics tests + A/B timing against the bf16x3 engine kernel
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gemm_x3_gpu.py -x -q -k u8 --timeout 120 --timeout-method thread 2>&1 | tail -5 || exit 1
SDML_U8_FWD=x3 timeout -k 10 120 python tools/bench_u8.py | sed "s/^/x3 engine: /" || exit 1
timeout -k 10 120 python tools/bench_u8.py | sed "s/^/u8_fwd: /" || exit 1

#!/bin/bash
# new uint8 weight gradient (mlp_u8.hip): numerics + A/B against the bf16x3 engine kernel
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gemm_x3_gpu.py -x -q -k u8 --timeout 120 --timeout-method thread 2>&1 | tail -3 || exit 1
SDML_U8_WGRAD=x3 timeout -k 10 120 python tools/bench_u8.py | sed "s/^/x3 engine: /" || exit 1
timeout -k 10 120 python tools/bench_u8.py | sed "s/^/u8_wgrad: /" || exit 1

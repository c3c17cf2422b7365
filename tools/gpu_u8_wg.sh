#!/bin/bash
# uint8 weight gradient: numerics + A/B (SDML_U8_VARIANT=1: per-K-step fp32 partials)
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gemm_x3_gpu.py -x -q -k u8 --timeout 120 --timeout-method thread 2>&1 | tail -3 || exit 1
SDML_U8_VARIANT=1 timeout -k 10 120 python tools/bench_u8.py | sed "s/^/fresh: /" || exit 1
timeout -k 10 120 python tools/bench_u8.py | sed "s/^/default: /" || exit 1

#!/bin/bash
# A/B of the uint8 first-layer GEMM variants (SDML_U8_VARIANT, see gemm_f32x3.hip u8_variant)
set -o pipefail
for v in 0 1 2 3; do
  SDML_U8_VARIANT=$v timeout -k 10 120 python tools/bench_u8.py | sed "s/^/variant $v: /" || exit 1
done

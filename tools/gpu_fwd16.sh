#!/bin/bash
# forward geometry A/B: 8-wave (512-thread, WMT 4) vs 16-wave (1024-thread, 4 waves/SIMD) blocks
set -o pipefail
mkdir -p gpurun_out/fwd16
export TMPDIR=/tmp
for w in 8 16; do
  SDML_U8_FWD_WAVES=$w timeout -k 10 300 python -u -m pytest tests/test_gemm_x3_gpu.py -x -q --timeout 120 --timeout-method thread -k "u8" > gpurun_out/fwd16/pytest_$w.log 2>&1 || { tail -30 gpurun_out/fwd16/pytest_$w.log; exit 1; }
  echo "waves $w: $(tail -1 gpurun_out/fwd16/pytest_$w.log)"
done
for w in 8 16 8 16; do
  SDML_U8_FWD_WAVES=$w timeout -k 10 120 python tools/bench_u8.py 2>/dev/null | sed "s/^/waves $w: /" || exit 1
done
for m in 1 4 6; do
  SDML_U8_FWD_WAVES=16 SDML_U8_FWD_MODE=$m timeout -k 10 120 python tools/bench_u8.py 2>/dev/null | sed "s/^/waves 16 mode $m: /" || exit 1
done
for w in 8 16; do
  SDML_U8_FWD_WAVES=$w timeout -k 10 200 python bench.py 2>/dev/null | cut -c1-160 | sed "s/^/waves $w: /" || exit 1
done

#!/bin/bash
# fp16-plane forward timing modes (SDML_U8_FWD_MODE): 0 normal, 1 DMA pipeline alone, 2 no DMA in
# the K loop, 4 no DMA + no barrier, 5 no byte widening, 6 no output stores; both block geometries
set -o pipefail
for w in 4 2; do
  for m in 0 1 2 4 5 6; do
    SDML_U8_FWD_WMT=$w SDML_U8_FWD_MODE=$m timeout -k 10 120 python tools/bench_u8.py 2>/dev/null | sed "s/^/wmt $w mode $m: /" || exit 1
  done
done

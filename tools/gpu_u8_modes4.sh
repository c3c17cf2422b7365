#!/bin/bash
# 512-row forward timing modes (SDML_U8_FWD_MODE): 0 normal, 1 DMA only, 2 no DMA, 4 no DMA + no
# barrier, 5 no byte widening
set -o pipefail
export SDML_U8_FWD_WMT=4
for m in 0 1 2 4 5; do
  SDML_U8_FWD_MODE=$m timeout -k 10 120 python tools/bench_u8.py 2>/dev/null | sed "s/^/mode $m: /" || exit 1
done

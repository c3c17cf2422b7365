#!/bin/bash
# 512-row forward timing: normal vs no output stores (SDML_U8_FWD_MODE=6) vs no DMA / no barrier
set -o pipefail
export SDML_U8_FWD_WMT=4
for m in 0 6 4 0 6; do
  SDML_U8_FWD_MODE=$m timeout -k 10 120 python tools/bench_u8.py 2>/dev/null | sed "s/^/mode $m: /" || exit 1
done

#!/bin/bash
# uint8 forward: DMA-only / compute-only / no-LDS-read timing modes (SDML_U8_FWD_MODE)
set -o pipefail
for m in 0 1 2 3; do
  SDML_U8_FWD_MODE=$m timeout -k 10 120 python tools/bench_u8.py | sed "s/^/mode $m: /" || exit 1
done

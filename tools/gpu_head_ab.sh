#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/head
export TMPDIR=/tmp
L=gpurun_out/head/log.txt
: > $L
for b in 512 768 1024 2048; do
  echo "max_blocks=$b" >> $L
  SDML_HEAD_MAX_BLOCKS=$b timeout -k 10 200 python bench.py --steps 100 >> $L 2>&1 || { tail $L; exit 1; }
done
SDML_HEAD_MAX_BLOCKS=2048 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "head" >> $L 2>&1 || { tail -30 $L; exit 1; }
grep -v amdgpu.ids $L | cut -c1-200

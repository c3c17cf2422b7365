#!/bin/bash
# factored boundary gradient on one rank (SDML_FACTORED_R1) vs the head's dx: tests, step timing, profile
set -o pipefail
mkdir -p gpurun_out/r1f
export TMPDIR=/tmp
L=gpurun_out/r1f/log.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r1f/pytest.log 2>&1 || { tail -40 gpurun_out/r1f/pytest.log; exit 1; }
tail -1 gpurun_out/r1f/pytest.log
for f in 1 0 1 0; do
  SDML_FACTORED_R1=$f timeout -k 10 200 python bench.py 2>/dev/null | sed "s/^/factored_r1=$f: /" | cut -c1-200 >> $L || { tail $L; exit 1; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r1f/stats -o b -- python bench.py --steps 20 --warmup 5 > gpurun_out/r1f/stats.log 2>&1 || { tail -20 gpurun_out/r1f/stats.log; exit 1; }
f=$(find gpurun_out/r1f/stats -name "*kernel_stats.csv" | head -1)
python tools/summarize_profile.py stats "$f" 25 > gpurun_out/r1f/kernel_stats.txt
cat $L
head -12 gpurun_out/r1f/kernel_stats.txt | cut -c1-160

#!/bin/bash
# full GPU verification + config benches (u8 and f32 pixel storage)
set -o pipefail
mkdir -p gpurun_out/round
export TMPDIR=/tmp
L=gpurun_out/round/log.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/round/pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/round/pytest.log; exit 1; }
tail -1 gpurun_out/round/pytest.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $L 2>&1 || { cat $L; exit 1; }
timeout -k 10 200 python bench.py >> $L 2>&1 || { tail $L; exit 1; }
for px in u8 f32; do
  timeout -k 10 240 python tools/bench_configs.py --config mlp4x1024 --pixels $px --steps 20 --warmup 3 >> $L 2>&1 || { tail $L; exit 1; }
done
timeout -k 10 240 python tools/bench_configs.py --config mlp --pixels u8 --steps 50 --warmup 5 >> $L 2>&1 || { tail $L; exit 1; }
grep -v amdgpu.ids $L | cut -c1-330

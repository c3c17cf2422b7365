#!/bin/bash
# uint8-pixel first layer: tests, bench (u8 vs f32 storage), kernel profile
set -o pipefail
mkdir -p gpurun_out/u8
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gemm_x3_gpu.py tests/test_engine_gpu.py -x -v --timeout 120 --timeout-method thread -k "u8" > gpurun_out/u8/pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/u8/pytest.log; exit 1; }
tail -3 gpurun_out/u8/pytest.log
timeout -k 10 200 python bench.py > gpurun_out/u8/bench_u8.log 2>&1 || { tail -30 gpurun_out/u8/bench_u8.log; exit 1; }
cat gpurun_out/u8/bench_u8.log
timeout -k 10 200 python bench.py --pixels f32 > gpurun_out/u8/bench_f32.log 2>&1 || { tail -30 gpurun_out/u8/bench_f32.log; exit 1; }
cat gpurun_out/u8/bench_f32.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/u8/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/gpurun_out/u8/prof.log 2>&1 || { tail -30 $GRAFT_REPO_ROOT/gpurun_out/u8/prof.log; exit 1; }
find $GRAFT_REPO_ROOT/gpurun_out/u8/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c 'cut -d, -f1-8 {} | head -15'

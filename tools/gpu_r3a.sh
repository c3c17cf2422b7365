set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 250 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gemm_x2_gpu.py tests/test_kernels_gpu.py -k "x2 or attention or attn" > gpurun_out/x2t.log 2>&1; echo x2test rc=$?; grep -E "PASS|FAIL|Error" gpurun_out/x2t.log | cut -c1-150 | head -40
timeout -k 10 120 python tools/bench_x2.py > gpurun_out/x2b.log 2>&1 && tail -1 gpurun_out/x2b.log
timeout -k 10 60 python tools/bench_attention.py --B 16 > gpurun_out/attn.log 2>&1 && tail -1 gpurun_out/attn.log
timeout -k 10 400 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_multirank_gpu.py tests/test_fused_head_gpu.py > gpurun_out/mr1.log 2>&1; echo rc=$?; grep -E "PASS|FAIL" gpurun_out/mr1.log | cut -c1-150
tools/gpu.sh stats c4x2 200 python tools/bench_configs.py --config mlp4x1024 --steps 10 --warmup 3

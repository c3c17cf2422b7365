# LDS-DMA bf16 weight gradient: tests, per-shape timing (DMA vs staged), GPT-2 config A/B, kernel table
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_gemm_x2_gpu.py -k "wgrad" -m gpu > gpurun_out/wg_tests.log 2>&1 || { tail -30 gpurun_out/wg_tests.log; exit 1; }
tail -3 gpurun_out/wg_tests.log
SDML_WGRAD_DMA=0 timeout -k 10 200 python -u tools/bench_gpt2_gemms.py > gpurun_out/wg_gemms_staged.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/bench_gpt2_gemms.py > gpurun_out/wg_gemms_dma.log 2>&1 || exit 1
grep -o "^\[[^]]*\]\|wgrad_bf16 (HIP): [0-9.]*us ([0-9]* TF/s)" gpurun_out/wg_gemms_staged.log gpurun_out/wg_gemms_dma.log
SDML_WGRAD_DMA=0 timeout -k 10 300 python -u tools/bench_configs.py --config gpt2 > gpurun_out/wg_gpt2_staged.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_configs.py --config gpt2 > gpurun_out/wg_gpt2_dma.log 2>&1 || exit 1
tail -1 gpurun_out/wg_gpt2_staged.log | cut -c1-200; tail -1 gpurun_out/wg_gpt2_dma.log | cut -c1-200
tools/gpu.sh stats gpt2_dma 300 python tools/bench_configs.py --config gpt2 --steps 5 --warmup 2 || exit 1
SDML_WGRAD_DMA=0 timeout -k 10 200 python -u tools/bench_x2.py > gpurun_out/wg_x2_staged.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/bench_x2.py > gpurun_out/wg_x2_dma.log 2>&1 || exit 1
SDML_WGRAD_DMA=0 timeout -k 10 300 python -u tools/bench_configs.py --config mlp4x1024 > gpurun_out/wg_4x1024_staged.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_configs.py --config mlp4x1024 > gpurun_out/wg_4x1024_dma.log 2>&1 || exit 1

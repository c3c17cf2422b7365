# LDS-DMA conv weight gradient: tests, ResNet-18 A/B (staged, 2-stage, 3-stage), kernel table
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_conv_gpu.py -m gpu > gpurun_out/cw_tests.log 2>&1 || { tail -30 gpurun_out/cw_tests.log; exit 1; }
tail -2 gpurun_out/cw_tests.log
for mode in "0 2" "1 2" "1 3"; do
  set -- $mode
  SDML_WGRAD_DMA=$1 SDML_CONV_WGRAD_STAGES=$2 timeout -k 10 300 python -u tools/bench_configs.py --config resnet18 --dtype bf16 > gpurun_out/cw_resnet_$1_$2.log 2>&1 || exit 1
  echo "dma=$1 stages=$2 $(tail -1 gpurun_out/cw_resnet_$1_$2.log | grep -o '"value": [0-9.]*, "unit": "[a-z/]*", "ms_per_step": [0-9.]*')"
done
tools/gpu.sh stats resnet_dma 200 python tools/bench_configs.py --config resnet18 --dtype bf16 --steps 10 --warmup 3 || exit 1

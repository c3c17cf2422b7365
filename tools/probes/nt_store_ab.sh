set -o pipefail
export TMPDIR=/tmp
for nt in 0 1; do
  SDML_GEMM_NT_STORE=$nt timeout -k 10 200 python -u tools/probes/gemm_epilogue_probe.py > gpurun_out/nt_gemm_$nt.jsonl 2>&1 || exit 1
  SDML_GEMM_NT_STORE=$nt timeout -k 10 200 python -u tools/bench_x2.py > gpurun_out/nt_x2_$nt.log 2>&1 || exit 1
  SDML_GEMM_NT_STORE=$nt timeout -k 10 300 python -u tools/bench_configs.py --config mlp4x1024 > gpurun_out/nt_4x1024_$nt.log 2>&1 || exit 1
done

#!/bin/bash
# Round 6: the bf16 NT GEMM's epilogue store cost at the GPT-2 shapes (experiments build swapped in on the box only)
set -o pipefail
export TMPDIR=/tmp
d=gpurun_out/r6_gemm_store
mkdir -p $d
SO=simple_distributed_machine_learning_amd/_kernels.cpython-310-x86_64-linux-gnu.so
cp tools/probes/_exp_kernels.so $SO
SDML_KERNEL_EXPERIMENTS=1 SDML_NO_AUTOBUILD=1 timeout -k 10 300 python tools/probes/gemm_store_cost.py > $d/store.jsonl 2> $d/err.log || { tail $d/err.log; exit 1; }
cat $d/store.jsonl

#!/bin/bash
# end-to-end training through the reference CLI on one MI355X: the reference workload (CNN split,
# batch 60, 10 epochs) and the headline MLP at batch 131072 on uint8 synthetic data (3 epochs)
set -o pipefail
mkdir -p gpurun_out/train
export TMPDIR=/tmp
timeout -k 10 300 python -m simple_distributed_machine_learning_amd.train --rank 0 --world_size 1 --interface lo \
  --master_addr 127.0.0.1 --master_port 29517 --metrics gpurun_out/train/ref_cnn.jsonl > gpurun_out/train/ref_cnn.log 2>&1 \
  || { tail -20 gpurun_out/train/ref_cnn.log; exit 1; }
tail -4 gpurun_out/train/ref_cnn.log
timeout -k 10 300 python -m simple_distributed_machine_learning_amd.train --rank 0 --world_size 1 --interface lo \
  --master_addr 127.0.0.1 --master_port 29518 --model mlp --schedule rotate --batch_size 131072 --pixels u8 \
  --train_size 1048576 --test_size 65536 --epochs 3 --log_interval 2 --metrics gpurun_out/train/mlp.jsonl \
  > gpurun_out/train/mlp.log 2>&1 || { tail -20 gpurun_out/train/mlp.log; exit 1; }
grep -v amdgpu gpurun_out/train/mlp.log | tail -12

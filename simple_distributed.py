"""Drop-in entry point with the reference's name and command line.

    python simple_distributed.py --rank=0 --world_size=2 --interface=lo --master_addr=127.0.0.1 --master_port=2308
    python simple_distributed.py --rank=1 --world_size=2 --interface=lo --master_addr=127.0.0.1 --master_port=2308

Runs the reference workload (/root/reference/simple_distributed.py: MNIST CNN split after
the conv stack, batch 60, SGD lr 0.1 momentum 0.5, 10 epochs, logs every 10 batches) on the
MI355X-native engine: SPMD stages over RCCL (or Gloo on CPU) instead of RPC. Every engine
flag (--model, --schedule, --microbatches, ...) is accepted too; see
``simple_distributed_machine_learning_amd/cli.py``.
"""
import sys

from simple_distributed_machine_learning_amd.train import main

if __name__ == "__main__":
    sys.exit(main())

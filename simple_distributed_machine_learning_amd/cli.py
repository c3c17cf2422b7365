"""Command line: the reference's five flags (same names, types, defaults) plus engine flags.

Reference flags (/root/reference/simple_distributed.py:139-165):

=================  ======  ==============  =========================================
flag               type    default         effect
=================  ======  ==============  =========================================
``--rank``         int     (required*)     this process's rank
``--world_size``   int     2               number of processes
``--interface``    str     ``eth0``        -> GLOO_SOCKET_IFNAME, TP_SOCKET_IFNAME
                                           (+ NCCL_SOCKET_IFNAME for RCCL bootstrap)
``--master_addr``  str     ``localhost``   -> MASTER_ADDR (TCPStore rendezvous)
``--master_port``  str     ``"29500"``     -> MASTER_PORT
=================  ======  ==============  =========================================

(*) the reference asserts ``--rank`` is given (:160); here it may also come from torchrun's
``RANK`` env so the same entry point works under ``torch.distributed.run``.
"""
from __future__ import annotations

import argparse
import os
import sys
import warnings
from typing import List, Optional


def add_reference_args(parser: argparse.ArgumentParser):
    parser.add_argument('--rank', type=int, metavar='R', help="""Number of rank""")
    parser.add_argument('--world_size', type=int, default=None, metavar='N',
                        help="""Number of workers (default 2, or WORLD_SIZE from torchrun)""")
    parser.add_argument('--interface', type=str, default="eth0", metavar='I',
                        help="""Interface that current device is listening on. It will default to eth0 if
        not provided.""")
    parser.add_argument('--master_addr', type=str, default="localhost", metavar='MA',
                        help="""Address of master, will default to localhost if not provided.
        Master must be able to accept network traffic on the address + port.""")
    parser.add_argument('--master_port', type=str, default="29500", metavar='MP',
                        help="""Port that master is listening on, will default to 29500 if not
        provided. Master must be able to accept network traffic on the host and port.""")


def add_engine_args(parser: argparse.ArgumentParser):
    g = parser.add_argument_group("engine")
    g.add_argument("--model", default="ref_cnn",
                   choices=["ref_cnn", "mlp", "mlp4x1024", "resnet18", "gpt2", "gpt2_tiny"])
    g.add_argument("--stages", type=int, default=None, help="pipeline stages (default per model)")
    g.add_argument("--pp", type=int, default=None,
                   help="ranks per pipeline (default: min(stages, world_size); chimera: 2)")
    g.add_argument("--tp", type=int, default=1,
                   help="tensor-parallel ranks per stage (GPT-2 models; gpipe/1f1b schedules)")
    g.add_argument("--schedule", default="1f1b", choices=["gpipe", "1f1b", "chimera", "rotate"])
    g.add_argument("--microbatches", type=int, default=1)
    g.add_argument("--batch_size", type=int, default=60, help="per-replica batch (reference: 60)")
    g.add_argument("--test_batch_size", type=int, default=None)
    g.add_argument("--epochs", type=int, default=10)
    g.add_argument("--lr", type=float, default=0.1)
    g.add_argument("--momentum", type=float, default=0.5)
    g.add_argument("--weight_decay", type=float, default=0.0)
    g.add_argument("--log_interval", type=int, default=10)
    g.add_argument("--data", default="auto", choices=["auto", "synthetic", "random", "mnist"],
                   help="auto: MNIST idx files under --data_dir if present, else synthetic")
    g.add_argument("--data_dir", default="data")
    g.add_argument("--pixels", default="f32", choices=["f32", "u8"],
                   help="image storage on the device: float32 (ToTensor applied at load) or MNIST's uint8 bytes "
                        "(ToTensor's /255 applied by stage 0: fused into the first GEMM for the MLPs)")
    g.add_argument("--train_size", type=int, default=6000, help="reference keeps len(MNIST)//10")
    g.add_argument("--test_size", type=int, default=1000)
    g.add_argument("--seq_len", type=int, default=None, help="token models: sequence length")
    g.add_argument("--seed", type=int, default=1)
    g.add_argument("--data_seed", type=int, default=1234)
    g.add_argument("--device", default="auto", choices=["auto", "cpu", "cuda"])
    g.add_argument("--backend", default="auto", choices=["auto", "nccl", "rccl", "gloo"])
    g.add_argument("--timeout", type=float, default=600.0, help="process-group timeout (s), finite")
    g.add_argument("--heartbeat", type=float, default=0.0, help="peer heartbeat timeout (s); 0 = off")
    g.add_argument("--dropout", type=float, default=0.5,
                   help="ref_cnn: Dropout2d / dropout probability (reference: 0.5; 0 makes a run deterministic)")
    g.add_argument("--eval_dropout", type=int, default=1,
                   help="ref_cnn: keep stage-1 dropout active in test() like the reference (1) or not (0)")
    g.add_argument("--ckpt_dir", default=None)
    g.add_argument("--resume", action="store_true")
    g.add_argument("--save_every", type=int, default=0, help="save every N epochs (0: only at the end)")
    g.add_argument("--metrics", default=None, help="JSONL metrics file (rank 0)")
    g.add_argument("--max_steps", type=int, default=0, help="stop each epoch after N steps (0: full epoch)")
    g.add_argument("--no_test", action="store_true")
    g.add_argument("--profile", default=None, help="write a torch.profiler trace of a few steps here")
    g.add_argument("--debug_sync", action="store_true", help="device sync after every pipeline op")
    g.add_argument("--graph", action="store_true",
                   help="capture the training step in a hipGraph and replay it (ROCm, one process)")
    g.add_argument("--timing", action="store_true",
                   help="per-stage/phase device timers (fwd, bwd, recv_wait, grad_sync, optim) in the metrics")
    g.add_argument("--dtype", default="auto", choices=["auto", "fp32", "bf16"],
                   help="parameter/compute dtype (auto: the model's default; gpt2 is bf16, the rest fp32)")


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description="Distributed Machine Learning",
                                formatter_class=argparse.ArgumentDefaultsHelpFormatter)
    add_reference_args(p)
    add_engine_args(p)
    return p


def _iface_exists(name: str) -> bool:
    return os.path.exists(f"/sys/class/net/{name}")


def export_env(args) -> None:
    """Same env contract as the reference (:162-165)."""
    os.environ['MASTER_ADDR'] = args.master_addr
    os.environ['MASTER_PORT'] = str(args.master_port)
    if _iface_exists(args.interface) or args.interface != "eth0":
        os.environ['GLOO_SOCKET_IFNAME'] = args.interface
        os.environ["TP_SOCKET_IFNAME"] = args.interface
        os.environ.setdefault("NCCL_SOCKET_IFNAME", args.interface)
    else:  # reference quirk B.8: default eth0 on a host without it would break rendezvous
        warnings.warn("--interface eth0 not present on this host; leaving socket interface selection to "
                      "the libraries (pass --interface lo for single-host runs)")


def parse_args(argv: Optional[List[str]] = None):
    args = build_parser().parse_args(argv)
    if args.rank is None and "RANK" in os.environ:
        args.rank = int(os.environ["RANK"])
    if args.world_size is None:
        args.world_size = int(os.environ.get("WORLD_SIZE", "2"))
    assert args.rank is not None, "Must provide rank argument."
    if args.backend == "rccl":
        args.backend = "nccl"  # PyTorch-ROCm names RCCL "nccl"
    given = argv if argv is not None else sys.argv[1:]

    def passed(flag):
        return any(a == flag or a.startswith(flag + "=") for a in given)

    # under torchrun the rendezvous env wins unless the flag was given explicitly
    if "MASTER_ADDR" in os.environ and not passed("--master_addr"):
        args.master_addr = os.environ["MASTER_ADDR"]
    if "MASTER_PORT" in os.environ and not passed("--master_port"):
        args.master_port = os.environ["MASTER_PORT"]
    return args

"""Reference CLI compatibility (/root/reference/simple_distributed.py:139-165)."""
import os

import pytest

from simple_distributed_machine_learning_amd import cli


def test_reference_defaults(monkeypatch):
    for k in ("RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        monkeypatch.delenv(k, raising=False)
    a = cli.parse_args(["--rank", "0"])
    assert a.world_size == 2
    assert a.interface == "eth0"
    assert a.master_addr == "localhost"
    assert a.master_port == "29500" and isinstance(a.master_port, str)
    # reference hyper-parameters (:18-22)
    assert (a.batch_size, a.epochs, a.lr, a.momentum, a.log_interval) == (60, 10, 0.1, 0.5, 10)
    assert a.model == "ref_cnn"


def test_rank_required(monkeypatch):
    monkeypatch.delenv("RANK", raising=False)
    with pytest.raises(AssertionError, match="Must provide rank"):
        cli.parse_args([])


def test_torchrun_env(monkeypatch):
    monkeypatch.setenv("RANK", "3")
    monkeypatch.setenv("WORLD_SIZE", "8")
    monkeypatch.setenv("MASTER_ADDR", "10.0.0.1")
    monkeypatch.setenv("MASTER_PORT", "1234")
    a = cli.parse_args([])
    assert (a.rank, a.world_size, a.master_addr, a.master_port) == (3, 8, "10.0.0.1", "1234")
    a = cli.parse_args(["--master_port=99"])
    assert a.master_port == "99"


def test_env_export(monkeypatch):
    for k in ("GLOO_SOCKET_IFNAME", "TP_SOCKET_IFNAME", "NCCL_SOCKET_IFNAME"):
        monkeypatch.delenv(k, raising=False)
    a = cli.parse_args(["--rank=1", "--interface=lo", "--master_addr=127.0.0.1", "--master_port=2308"])
    cli.export_env(a)
    assert os.environ["MASTER_ADDR"] == "127.0.0.1"
    assert os.environ["MASTER_PORT"] == "2308"
    assert os.environ["GLOO_SOCKET_IFNAME"] == "lo"
    assert os.environ["TP_SOCKET_IFNAME"] == "lo"
    assert os.environ["NCCL_SOCKET_IFNAME"] == "lo"


def test_rccl_alias():
    assert cli.parse_args(["--rank", "0", "--backend", "rccl"]).backend == "nccl"


def test_dtype_and_timing_flags():
    from simple_distributed_machine_learning_amd import cli

    a = cli.parse_args(["--rank=0", "--dtype=bf16", "--timing", "--model=resnet18"])
    assert a.dtype == "bf16" and a.timing and a.model == "resnet18"
    assert cli.parse_args(["--rank=0"]).dtype == "auto"


def test_tp_flag_parses():
    from simple_distributed_machine_learning_amd import cli

    args = cli.build_parser().parse_args(["--rank", "0", "--model", "gpt2_tiny", "--tp", "2"])
    assert args.tp == 2
    assert cli.build_parser().parse_args(["--rank", "0"]).tp == 1

"""Per-stage checkpoint layout (reference key names) and bit-identical resume."""
import torch

from simple_distributed_machine_learning_amd.data import SyntheticMNIST
from simple_distributed_machine_learning_amd.models import get_model_spec
from simple_distributed_machine_learning_amd.parallel import PipelineEngine, init_mesh
from simple_distributed_machine_learning_amd.utils.checkpoint import load_checkpoint, save_checkpoint


def _eng(model="ref_cnn", **kw):
    mesh = init_mesh(pp=1, schedule_kind="1f1b", rank=0, world_size=1, device=torch.device("cpu"))
    return PipelineEngine(get_model_spec(model, **kw), mesh, "1f1b", 2, lr=0.1, momentum=0.5, seed=1)


def test_reference_state_dict_keys(tmp_path):
    e = _eng()
    save_checkpoint(e, str(tmp_path), epoch=1, batch=5)
    s0 = torch.load(tmp_path / "stage0.pt", weights_only=True)
    s1 = torch.load(tmp_path / "stage1.pt", weights_only=True)
    # /root/reference/simple_distributed.py:29-31 (Network1) and :63-64 (Network2)
    assert sorted(s0["model"]) == ["conv1.bias", "conv1.weight", "conv2.bias", "conv2.weight"]
    assert sorted(s1["model"]) == ["fc1.bias", "fc1.weight", "fc2.bias", "fc2.weight"]
    assert s0["model"]["conv1.weight"].shape == (10, 1, 5, 5)
    assert s1["model"]["fc1.weight"].shape == (50, 320)
    assert sum(v.numel() for v in s0["model"].values()) == 5280
    assert sum(v.numel() for v in s1["model"].values()) == 16560
    assert s0["epoch"] == 1 and s0["batch"] == 5


def test_resume_is_bit_identical(tmp_path):
    torch.manual_seed(0)
    ds = SyntheticMNIST(600, seed=3)
    kw = {"dropout": 0.0}
    a = _eng(**kw)
    for i in range(3):
        a.run(ds, i * 60, 60, train=True)
    save_checkpoint(a, str(tmp_path), epoch=1, batch=2)
    b = _eng(**kw)
    meta = load_checkpoint(b, str(tmp_path))
    assert meta == {"epoch": 1, "batch": 2, "global_step": 3}
    assert torch.equal(a.flat.params, b.flat.params)
    assert torch.equal(a.optimizer.momentum_buffer[:a.flat.numel], b.optimizer.momentum_buffer[:b.flat.numel])
    ra = a.run(ds, 180, 60, train=True)
    rb = b.run(ds, 180, 60, train=True)
    assert torch.equal(a.flat.params, b.flat.params)
    assert float(ra.loss_sum) == float(rb.loss_sum)


def test_mlp_checkpoint_roundtrip(tmp_path):
    a = _eng("mlp")
    save_checkpoint(a, str(tmp_path), 2, 9)
    sd = torch.load(tmp_path / "stage0.pt", weights_only=True)
    assert sorted(sd["model"]) == ["fc1.bias", "fc1.weight"]
    assert "momentum_buffer" in sd["optim"]

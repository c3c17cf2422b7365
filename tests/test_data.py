import gzip

import numpy as np
import torch

from simple_distributed_machine_learning_amd.data import IdxMNIST, SyntheticMNIST, SyntheticTokens, batch_ranges


def test_reference_loader_order():
    # 6,000 train / 60 -> 100 batches; 1,000 test / 60 -> 16 x 60 + 1 x 40
    b = list(batch_ranges(6000, 60))
    assert len(b) == 100 and b[0] == (0, 0, 60) and b[-1] == (99, 5940, 60)
    t = list(batch_ranges(1000, 60))
    assert len(t) == 17 and t[-1] == (16, 960, 40)
    assert list(batch_ranges(1000, 60, start_batch=16)) == [(16, 960, 40)]


def test_synthetic_deterministic_and_offset():
    a = SyntheticMNIST(100, seed=9)
    b = SyntheticMNIST(100, seed=9)
    assert torch.equal(a.x, b.x) and torch.equal(a.y, b.y)
    c = SyntheticMNIST(50, seed=9, offset=50)
    assert torch.equal(c.x, a.x[50:]) and torch.equal(c.y, a.y[50:])
    assert a.x.shape == (100, 1, 28, 28) and a.x.dtype == torch.float32
    assert 0 <= float(a.x.min()) and float(a.x.max()) <= 1
    assert set(a.y.tolist()) <= set(range(10))
    d = SyntheticMNIST(100, seed=10)
    assert not torch.equal(a.x, d.x)


def test_synthetic_is_learnable_class_structure():
    ds = SyntheticMNIST(2000, seed=1)
    means = torch.stack([ds.x[ds.y == c].mean(0).flatten() for c in range(10)])
    # class prototypes differ clearly
    d = torch.cdist(means, means)
    assert float(d[~torch.eye(10, dtype=bool)].min()) > 1.0


def test_tokens():
    t = SyntheticTokens(8, 16, 97, seed=1)
    assert t.inputs(0, 8).shape == (8, 16) and t.targets(0, 8).shape == (8, 16)
    assert torch.equal(t.inputs(0, 8)[:, 1:], t.targets(0, 8)[:, :-1])


def _write_idx(path, arr, gz=False):
    arr = np.asarray(arr, dtype=np.uint8)
    header = bytes([0, 0, 8, arr.ndim]) + b"".join(int(d).to_bytes(4, "big") for d in arr.shape)
    data = header + arr.tobytes()
    (gzip.open if gz else open)(path, "wb").write(data)


def test_idx_mnist(tmp_path):
    imgs = np.random.RandomState(0).randint(0, 256, (30, 28, 28))
    lbls = np.arange(30) % 10
    _write_idx(tmp_path / "train-images-idx3-ubyte", imgs)
    _write_idx(tmp_path / "train-labels-idx1-ubyte", lbls)
    _write_idx(tmp_path / "t10k-images-idx3-ubyte.gz", imgs[:20], gz=True)
    _write_idx(tmp_path / "t10k-labels-idx1-ubyte.gz", lbls[:20], gz=True)
    assert IdxMNIST.available(str(tmp_path))
    tr = IdxMNIST(str(tmp_path), True, fraction=0.1)  # reference keeps len // 10
    assert len(tr) == 3
    assert torch.allclose(tr.x[0, 0], torch.tensor(imgs[0], dtype=torch.float32) / 255)
    te = IdxMNIST(str(tmp_path), False, fraction=1.0)
    assert len(te) == 20 and te.y.tolist() == lbls[:20].tolist()


def test_synthetic_u8_pixels_are_mnist_bytes():
    f = SyntheticMNIST(50, seed=3)
    u = SyntheticMNIST(50, seed=3, pixels="u8")
    assert u.x.dtype == torch.uint8 and u.x.shape == f.x.shape
    assert torch.equal(u.x, (f.x * 255.0).round().to(torch.uint8))
    assert torch.equal(u.y, f.y)
    from simple_distributed_machine_learning_amd.ops import pixels_to_float

    assert torch.equal(pixels_to_float(u.x), u.x.float() / 255.0)


def test_cpu_engine_u8_pixels_equal_totensor_floats():
    from simple_distributed_machine_learning_amd.models import get_model_spec
    from simple_distributed_machine_learning_amd.parallel import PipelineEngine, init_mesh

    def eng(model):
        mesh = init_mesh(pp=1, schedule_kind="1f1b", rank=0, world_size=1, device=torch.device("cpu"))
        return PipelineEngine(get_model_spec(model, None), mesh, schedule_kind="1f1b", num_microbatches=2, lr=0.1,
                              momentum=0.5, seed=2)

    for model in ("mlp", "ref_cnn"):
        a, b = eng(model), eng(model)
        du = SyntheticMNIST(240, seed=4, pixels="u8")
        df = SyntheticMNIST(240, seed=4)
        df.x = du.x.float() / 255.0
        for s in range(2):
            if model == "ref_cnn":
                torch.manual_seed(s)
            ra = a.run(du, s * 120, 120, train=True)
            if model == "ref_cnn":
                torch.manual_seed(s)
            rb = b.run(df, s * 120, 120, train=True)
            assert float(ra.loss_sum) == float(rb.loss_sum)
        assert torch.equal(a.flat.params, b.flat.params)

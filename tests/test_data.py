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

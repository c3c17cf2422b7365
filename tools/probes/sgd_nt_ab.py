"""sgd_momentum_mixed_ on a GPT-2-sized flat buffer (124 M params): default vs non-temporal streams (knob SGD_NT)."""
import json

import torch

from simple_distributed_machine_learning_amd import _native

K = _native.kernels()
n = 124_475_904
dev = torch.device("cuda", 0)
master = torch.randn(n, device=dev)
p = master.to(torch.bfloat16)
g = (torch.randn(n, device=dev) * 1e-3).to(torch.bfloat16)
buf = torch.zeros(n, device=dev)
res = {}
for rep in range(3):
    for nt in (0, 1):
        K.set_knob("SGD_NT", nt)
        for _ in range(3):
            K.sgd_momentum_mixed_(master, p, g, buf, 0.01, 0.5, 0.0, 0.0, False, False, False)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(10):
            K.sgd_momentum_mixed_(master, p, g, buf, 0.01, 0.5, 0.0, 0.0, False, False, False)
        e1.record()
        torch.cuda.synchronize()
        res.setdefault(nt, []).append(round(e0.elapsed_time(e1) / 10 * 1e3, 1))
K.reset_knobs()
# equality of the two variants on identical inputs
outs = []
for nt in (0, 1):
    K.set_knob("SGD_NT", nt)
    m2, p2, b2 = master.clone(), p.clone(), buf.clone()
    K.sgd_momentum_mixed_(m2, p2, g.clone(), b2, 0.01, 0.5, 0.0, 0.0, False, False, False)
    torch.cuda.synchronize()
    outs.append((m2, p2, b2))
K.reset_knobs()
same = all(torch.equal(a, b) for a, b in zip(*outs))
print(json.dumps({"us_default": res[0], "us_nt": res[1], "bitwise_equal": same, "GB": round(n * 22 / 1e9, 2)}))

"""How fast can the headline's 51 MB weight-gradient slab be read? torch reductions over a [128, 100480] fp32 array
(rocprofv3 --kernel-trace --stats gives each kernel's time) against the step's slab_head_reduce kernel (11-12 us)."""
import torch

dev = torch.device("cuda", 0)
slab = torch.randn(128, 100480, device=dev)
out = torch.empty(100480, device=dev)
for _ in range(20):
    slab.mul_(1.0)                    # (rewrite: the slab arrives freshly written)
    torch.sum(slab, dim=0, out=out)   # column sums: the reduction the step does
    slab.mul_(1.0)
    s = slab.sum()                    # a contiguous full read
torch.cuda.synchronize()
print("done")

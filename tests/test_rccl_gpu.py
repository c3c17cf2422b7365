"""RCCL smoke on one MI355X: a 1-rank "nccl" (RCCL) process group created the way
parallel/mesh.py creates them (high-priority communication stream), running the collectives the
engine uses (all_to_all_single for the rotate boundary, all_reduce for gradients) from a
non-default compute stream. Runs in a subprocess so the global process-group state of the test
session stays clean."""
import os
import subprocess
import sys
import textwrap

import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():
    pytest.skip("no ROCm GPU", allow_module_level=True)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_rccl_high_priority_group_collectives():
    from conftest import free_port

    code = textwrap.dedent("""
        import datetime, torch, torch.distributed as dist
        from simple_distributed_machine_learning_amd.parallel.mesh import _pg_options
        dev = torch.device("cuda", 0)
        opts = _pg_options("nccl")
        assert opts is not None and opts.is_high_priority_stream
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev, pg_options=opts,
                                timeout=datetime.timedelta(seconds=60))
        g = dist.new_group([0], pg_options=opts)
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            x = torch.arange(4096, device=dev, dtype=torch.float32).view(1024, 4)
            y = torch.empty_like(x)
            w = dist.all_to_all_single(y, x, [1024], [1024], group=g, async_op=True)
            w.wait()
            t = torch.ones(1000, device=dev)
            dist.all_reduce(t, group=g)
        torch.cuda.synchronize()
        assert torch.equal(y, x) and float(t.sum()) == 1000.0
        dist.barrier(device_ids=[0])
        dist.destroy_process_group()
        print("rccl ok")
    """)
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()), PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=100)
    assert r.returncode == 0 and "rccl ok" in r.stdout, r.stdout[-2000:] + r.stderr[-4000:]

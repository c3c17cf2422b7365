"""Multi-process (Gloo, CPU) test harness: spawn world_size ranks on 127.0.0.1."""
from __future__ import annotations

import os
import pickle
import socket
import tempfile
import traceback

import torch.multiprocessing as mp


def free_port() -> int:
    """A free TCP port; under pytest-xdist each worker draws from its own range, so two tests that
    run at once cannot pick the same rendezvous port between its probe and its use."""
    import random

    wid = os.environ.get("PYTEST_XDIST_WORKER", "gw0")
    slot = int(wid[2:]) if wid[2:].isdigit() else 0
    lo = 20000 + (slot % 16) * 2500
    for _ in range(200):
        p = random.randint(lo, lo + 2499)
        s = socket.socket()
        try:
            s.bind(("127.0.0.1", p))
            return p
        except OSError:
            continue
        finally:
            s.close()
    raise RuntimeError("no free port")


def _entry(rank, world, port, fn, args, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), GLOO_SOCKET_IFNAME="lo")
    import torch

    torch.set_num_threads(1)
    try:
        res = fn(rank, world, *args)
        err = None
    except Exception:  # noqa: BLE001
        res, err = None, traceback.format_exc()
    finally:
        import torch.distributed as dist

        if dist.is_initialized():
            try:
                dist.destroy_process_group()
            except Exception:  # noqa: BLE001
                pass
    with open(os.path.join(outdir, f"r{rank}.pkl"), "wb") as f:
        pickle.dump((res, err), f)


def run_ranks(fn, world: int, *args, timeout: float = 240.0):
    """Run fn(rank, world, *args) in `world` processes; return the list of per-rank results."""
    port = free_port()
    with tempfile.TemporaryDirectory() as d:
        ctx = mp.get_context("spawn")
        procs = [ctx.Process(target=_entry, args=(r, world, port, fn, args, d)) for r in range(world)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(timeout)
        alive = [p for p in procs if p.is_alive()]
        for p in alive:
            p.kill()
        if alive:
            raise TimeoutError(f"{len(alive)} ranks hung")
        out = []
        for r in range(world):
            path = os.path.join(d, f"r{r}.pkl")
            if not os.path.exists(path):
                raise RuntimeError(f"rank {r} died (exit code {procs[r].exitcode})")
            with open(path, "rb") as f:
                res, err = pickle.load(f)
            if err:
                raise RuntimeError(f"rank {r} failed:\n{err}")
            out.append(res)
        return out

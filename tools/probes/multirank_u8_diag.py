"""Which run of the uint8 rotate engine disagrees: single-process vs 2 ranks (host transport, one GPU),
fused forward+head on/off. Prints step losses and the max |fc1.weight| difference to the single unfused run."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from dist_util import run_ranks  # noqa: E402
from dist_workers import train_worker  # noqa: E402


def main():
    out = {}
    for fuse in ("0", "1"):
        os.environ["SDML_FUSE_HEAD"] = fuse
        kw = {"device": "cuda:0", "pixels": "u8"}
        out[("single", fuse)] = train_worker(0, 1, "mlp", "rotate", 4, 1, 2, 16384, 3, dict(kw))
        res = run_ranks(train_worker, 2, "mlp", "rotate", 4, 2, 2, 8192, 3, dict(kw, transport="host"), timeout=400)
        out[("r2", fuse)] = res[0]
    base = out[("single", "0")]["state"]
    for k, r in out.items():
        d = max(float((v.cpu() - base[s][n].cpu()).abs().max()) for s, sd in r["state"].items() for n, v in sd.items())
        print(k, "losses", r["losses"], "eval", r["eval"], "max param diff vs single/unfused", d, flush=True)


if __name__ == "__main__":
    main()

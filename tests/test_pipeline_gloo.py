"""Multi-process parity on Gloo/CPU: an N-rank pipeline (and dp x pp mesh) must train to the
same weights and losses as one process running the whole model on the same data and seeds.
This is the framework's stand-in for "multi-node without a cluster" (SURVEY.md §4)."""
import pytest
import torch

from dist_util import run_ranks
from dist_workers import train_worker

pytestmark = pytest.mark.slow


def _single(model, M, steps, B, kind="1f1b", kw=None):
    # world 1: every stage on the one rank, global batch = B*dp of the multi-rank run
    return train_worker(0, 1, model, kind, M, 1, steps, B, 3, kw)


def _stage_states(results):
    out = {}
    for r in results:
        for s, sd in r["state"].items():
            if s in out:  # replicas (dp / chimera mirrors) must agree exactly
                for k in sd:
                    torch.testing.assert_close(sd[k], out[s][k], rtol=0, atol=0)
            else:
                out[s] = sd
    return out


def _compare(results, ref, rtol=1e-5, atol=1e-6):
    st = _stage_states(results)
    assert sorted(st) == sorted(ref["state"])
    for s in st:
        for k in st[s]:
            torch.testing.assert_close(st[s][k], ref["state"][s][k], rtol=rtol, atol=atol, msg=f"stage {s} {k}")
    for a, b in zip(results[0]["losses"], ref["losses"]):
        assert a == pytest.approx(b, rel=1e-5, abs=1e-6)
    assert results[0]["eval"][2] == ref["eval"][2]
    assert results[0]["eval"][0] == pytest.approx(ref["eval"][0], rel=1e-5)


@pytest.mark.parametrize("kind,M", [("1f1b", 1), ("1f1b", 3), ("gpipe", 4), ("chimera", 4), ("chimera", 2)])
def test_mlp_two_ranks_matches_single_process(kind, M):
    B, steps = 48, 3
    res = run_ranks(train_worker, 2, "mlp", kind, M, 2, steps, B)
    ref = _single("mlp", M, steps, B, kind)
    _compare(res, ref)
    assert all(r["bytes_sent"] > 0 for r in res)  # the boundary really crossed processes


def test_mlp_dp2_pp2_matches_single_process():
    B, steps = 24, 3
    res = run_ranks(train_worker, 4, "mlp", "1f1b", 2, 2, steps, B)
    ref = _single("mlp", 2, steps, 2 * B)
    # dp changes the micro-batch boundaries of the summed loss only through fp rounding
    _compare(res, ref, rtol=1e-4, atol=1e-5)


def test_mlp_chimera_dp2_matches_single_process():
    B, steps = 32, 2
    res = run_ranks(train_worker, 4, "mlp", "chimera", 4, 2, steps, B)
    ref = _single("mlp", 4, steps, 2 * B, "chimera")
    _compare(res, ref, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("kind", ["gpipe", "1f1b"])
def test_mlp4x1024_four_stages_four_ranks(kind):
    B, steps = 16, 2
    res = run_ranks(train_worker, 4, "mlp4x1024", kind, 4, 4, steps, B)
    ref = _single("mlp4x1024", 4, steps, B, kind)
    _compare(res, ref, rtol=1e-4, atol=1e-5)


def test_ref_cnn_two_ranks_no_dropout():
    B, steps = 30, 2
    kw = {"dropout": 0.0, "eval_dropout": False}
    res = run_ranks(train_worker, 2, "ref_cnn", "1f1b", 2, 2, steps, B, 3, kw)
    ref = _single("ref_cnn", 2, steps, B, "1f1b", kw)
    _compare(res, ref, rtol=1e-4, atol=1e-5)


def test_resnet18_eight_stages_on_four_ranks():
    B, steps = 4, 1
    kw = {"stages": 8}
    res = run_ranks(train_worker, 4, "resnet18", "1f1b", 2, 4, steps, B, 3, kw)
    ref = _single("resnet18", 2, steps, B, "1f1b", kw)
    _compare(res, ref, rtol=1e-3, atol=1e-4)


def test_gpt2_tiny_two_ranks():
    B, steps = 4, 2
    kw = {"stages": 2, "seq_len": 16}
    res = run_ranks(train_worker, 2, "gpt2_tiny", "1f1b", 2, 2, steps, B, 3, kw)
    ref = _single("gpt2_tiny", 2, steps, B, "1f1b", kw)
    _compare(res, ref, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("a2a", [True, False, "whole_grad", "u8"])
@pytest.mark.parametrize("world,M", [(2, 2), (2, 4), (4, 16), (4, 8)])
def test_mlp_rotate_matches_single_process(world, M, a2a, monkeypatch):
    """a2a=True: all-to-all boundary with the factored gradient (the head's dlogits cross, the owner
    rebuilds the boundary gradient); "whole_grad": all-to-all sending the full boundary gradient;
    False: per-peer p2p transfers; "u8": uint8 pixels, the factor going straight into stage 0's
    weight gradient (MLPStage.bwd_from_factor)."""
    B, steps = 24, 2
    if a2a == "u8":
        kw = {"pixels": "u8"}
        res = run_ranks(train_worker, world, "mlp", "rotate", M, world, steps, B, 3, kw)
        ref = _single("mlp", M, steps, world * B, "rotate", kw)
        _compare(res, ref, rtol=1e-4, atol=1e-5)
        return
    if not a2a:
        monkeypatch.setenv("SDML_ROTATE_P2P", "1")
    if a2a == "whole_grad":
        monkeypatch.setenv("SDML_ROTATE_FACTORED", "0")
    res = run_ranks(train_worker, world, "mlp", "rotate", M, world, steps, B)
    ref = _single("mlp", M, steps, world * B)
    _compare(res, ref, rtol=1e-4, atol=1e-5)
    if not a2a:
        per_owner = M // world  # micro-batch j of an owner goes to rank owner + j: j = 0 stays local
        assert all((r["bytes_sent"] > 0) == (per_owner > 1) for r in res)


def _merge_tp(results, tp, n_embd):
    """Reassemble full stage state dicts from tensor-parallel shards (parallel/tp.py layout)."""
    by_stage = {}
    for r in results:
        for s, sd in r["state"].items():
            by_stage.setdefault(s, {})[r["tp_rank"]] = sd
    C = n_embd
    out = {}
    for s, shards in by_stage.items():
        full = {}
        for k in shards[0]:
            parts = [shards[t][k] for t in range(tp)]
            if "attn.c_attn" in k:  # q, k, v column blocks of every rank's heads
                per = C // tp
                full[k] = torch.cat([parts[t][i * per:(i + 1) * per] for i in range(3) for t in range(tp)])
            elif k.endswith("attn.c_proj.weight") or k.endswith("mlp.c_proj.weight"):
                full[k] = torch.cat(parts, dim=1)
            elif "mlp.c_fc" in k:
                full[k] = torch.cat(parts, dim=0)
            else:  # replicated: identical on every tp rank
                for t in range(1, tp):
                    torch.testing.assert_close(parts[t], parts[0], rtol=0, atol=0, msg=k)
                full[k] = parts[0]
        out[s] = full
    return out


@pytest.mark.parametrize("world,pp,M", [(2, 1, 2), (4, 2, 2)])
def test_gpt2_tiny_tensor_parallel_matches_single_process(world, pp, M):
    """tp=2 (x pp) GPT-2: column/row-parallel blocks over Gloo train to the single-process weights."""
    B, steps = 4, 2
    kw = {"stages": 2, "seq_len": 16}
    res = run_ranks(train_worker, world, "gpt2_tiny", "1f1b", M, pp, steps, B, 3, kw, 2)
    ref = _single("gpt2_tiny", M, steps, B, "1f1b", kw)
    st = _merge_tp(res, 2, 32)
    assert sorted(st) == sorted(ref["state"])
    for s in st:
        for k in ref["state"][s]:
            torch.testing.assert_close(st[s][k], ref["state"][s][k], rtol=1e-4, atol=1e-5, msg=f"stage {s} {k}")
    for a, b in zip(res[0]["losses"], ref["losses"]):
        assert a == pytest.approx(b, rel=1e-5, abs=1e-6)
    assert res[0]["eval"][2] == ref["eval"][2]


def test_gpt2_tiny_rotate_alltoall_matches_single_process():
    """Token models under rotate: the all-to-all path must scale the loss per token, as the
    generic path does (a missing 1/seq_len would make the gradients seq_len times too large
    while the reported loss stays right)."""
    B, steps = 2, 2
    kw = {"stages": 2, "seq_len": 16}
    res = run_ranks(train_worker, 2, "gpt2_tiny", "rotate", 2, 2, steps, B, 3, kw)
    ref = _single("gpt2_tiny", 2, steps, 2 * B, "1f1b", kw)
    _compare(res, ref, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("B,M", [(3, 4), (1, 4), (5, 8)])
def test_mlp_rotate_alltoall_ragged_small_batches(B, M):
    """Batches smaller than waves x ranks: fewer waves, empty all-to-all parts; every rank
    must still join every collective and run its stage-0 backward."""
    steps = 2
    res = run_ranks(train_worker, 2, "mlp", "rotate", M, 2, steps, B)
    ref = _single("mlp", 1, steps, 2 * B)
    _compare(res, ref, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("world,phi", [(2, 0.0), (2, 0.25), (2, 1.0), (4, 0.5)])
@pytest.mark.parametrize("pixels", ["f32", "u8"])
def test_mlp_rotate_cross_fraction_matches_single_process(world, phi, pixels):
    """rotate with a chosen cross-GPU fraction (parallel/placement.py): phi = 0 is data parallelism over
    replicated stages (no boundary collective at all), 1.0 sends every row to a peer; every split trains
    to the single-process weights."""
    B, steps, M = 24, 2, 2 * world
    kw = {"cross_fraction": phi, "pixels": pixels, "dp_split": True}  # (the opt-in all-reduce overlap)
    res = run_ranks(train_worker, world, "mlp", "rotate", M, world, steps, B, 3, kw)
    ref = _single("mlp", M, steps, world * B, "rotate", {"pixels": pixels})
    _compare(res, ref, rtol=1e-4, atol=1e-5)
    assert all((r["bytes_sent"] > 0) == (phi > 0) for r in res)
    # nothing crossing, uint8 first layer: the weight gradient ran as two hidden ranges with the first
    # range's all-reduce issued before the second range (GradSync.issue_span)
    assert all((r["dp_split_steps"] == steps) == (phi == 0 and pixels == "u8") for r in res)


@pytest.mark.parametrize("kind,world,pp,M", [("rotate", 2, 2, 4), ("1f1b", 2, 2, 3), ("1f1b", 4, 2, 2),
                                             ("chimera", 2, 2, 4)])
def test_host_staged_transport_matches_direct(kind, world, pp, M):
    """The host-staged transport (what multi-rank runs on ONE GPU use) is interchangeable with the
    direct one: same weights, same losses, same bytes."""
    B, steps = 16, 3
    direct = run_ranks(train_worker, world, "mlp", kind, M, pp, steps, B, 3, {"transport": "direct"})
    host = run_ranks(train_worker, world, "mlp", kind, M, pp, steps, B, 3, {"transport": "host"})
    assert {r["transport"] for r in host} == {"host"} and {r["transport"] for r in direct} == {"direct"}
    for a, b in zip(host, direct):
        assert a["bytes_sent"] == b["bytes_sent"]
        for s in a["state"]:
            for k in a["state"][s]:
                torch.testing.assert_close(a["state"][s][k], b["state"][s][k], rtol=0, atol=0)
        assert a["losses"] == b["losses"]
        # persistent boundary buffers: nothing new after the first step
        assert a["pool_allocs"] == a["pool_allocs_first"]


def test_rotate_replica_with_no_samples_joins_the_same_collectives():
    """rotate with dp = 2 replicas of a 2-rank group, replica 1 given 0 samples: it must post the same
    gradient collective as the data-bearing replica (one all-reduce over the whole flat buffer), so
    nothing hangs and every rank ends with replica 0's weights (= a 2-rank run on its data alone)."""
    from dist_workers import empty_replica_worker

    B, steps = 24, 2
    res = run_ranks(empty_replica_worker, 4, 2, B, steps, timeout=200)
    ref = run_ranks(empty_replica_worker, 2, 2, B, steps, timeout=200)
    for r in res:
        for s, sd in r["state"].items():
            for k, v in sd.items():
                torch.testing.assert_close(v, ref[0]["state"][s][k], rtol=1e-5, atol=1e-6, msg=f"stage {s} {k}")


def test_empty_replica_with_planned_dp_split():
    """with the split gradient all-reduce planned (SDML_DP_SPLIT), a replica with no rows must issue the
    same two span all-reduces as the replica with data (which, on CPU, computes its gradient whole and then issues
    the spans): the same collective sequence, so no hang, and the weights of the data-only run."""
    from dist_workers import empty_replica_worker

    B, steps = 24, 2
    res = run_ranks(empty_replica_worker, 4, 2, B, steps, 3, True, 0.0, timeout=200)
    ref = run_ranks(empty_replica_worker, 2, 2, B, steps, 3, False, 0.0, timeout=200)
    for r in res:
        assert len(r["spans"]) == 2 * steps and r["spans"][0][0] == 0 and r["spans"][1][0] == r["spans"][0][1], r["spans"]
        for s, sd in r["state"].items():
            for k, v in sd.items():
                torch.testing.assert_close(v, ref[0]["state"][s][k], rtol=1e-5, atol=1e-6, msg=f"stage {s} {k}")
    assert all(not r["spans"] for r in ref)


def test_debug_sync_rotate_checks_every_owners_rows():
    """under rotate a head runs on rows of every owner, so debug_sync checks the whole replica
    group's block: a bad label in the last rank's shard is refused on rank 0 as well."""
    from dist_workers import debug_sync_rotate_worker

    res = run_ranks(debug_sync_rotate_worker, 2, 24, timeout=120)
    assert all(r is not None and "target out of range" in r for r in res), res

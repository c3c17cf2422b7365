"""Pure schedule tests (native generator + validator), no processes."""
import itertools

import pytest

from simple_distributed_machine_learning_amd import _native
from simple_distributed_machine_learning_amd.parallel.schedule import (OP_BWD, OP_FWD, OP_RECV, OP_SEND, PL_ACT,
                                                                        PL_GRAD, Instr, build_schedule, validate)

CASES = [(k, P, M, R) for k in ("gpipe", "1f1b", "chimera")
         for (P, R) in [(1, 1), (2, 1), (2, 2), (4, 4), (4, 2), (8, 8), (8, 4), (6, 3)]
         for M in (1, 2, 3, 4, 8, 13)]
CASES += [("rotate", P, M, R) for (P, R) in [(2, 1), (2, 2), (2, 4), (2, 8), (3, 4), (4, 8)] for M in (R, 2 * R, 4 * R)]


@pytest.mark.parametrize("kind,P,M,R", CASES)
def test_build_and_validate(kind, P, M, R):
    s = build_schedule(kind, P, M, R)
    assert len(s.programs) == R
    # every (stage, mb) forward and backward exactly once, on the owning rank
    seen = set()
    for r, prog in enumerate(s.programs):
        for ins in prog:
            if ins.op in (OP_FWD, OP_BWD):
                assert s.task_rank(ins.mb, ins.stage) == r
                assert ins.pipe == s.mb_pipe(ins.mb)
                key = (ins.op, ins.stage, ins.mb)
                assert key not in seen
                seen.add(key)
    assert len(seen) == 2 * P * M
    # sends/recvs pair up per channel
    for r, prog in enumerate(s.programs):
        for ins in prog:
            if ins.op == OP_SEND:
                assert any(o.op == OP_RECV and o.peer == r and (o.pipe, o.stage, o.mb, o.payload) ==
                           (ins.pipe, ins.stage, ins.mb, ins.payload) for o in s.programs[ins.peer])
    validate(s)


@pytest.mark.parametrize("kind,P,M,R", [(k, P, M, P) for k in ("gpipe", "1f1b", "chimera") for P in (2, 4) for M in (2, 4, 8)])
def test_forward_only(kind, P, M, R):
    s = build_schedule(kind, P, M, R, forward_only=True)
    assert all(i.op != OP_BWD for p in s.programs for i in p)
    assert all(i.payload != PL_GRAD for p in s.programs for i in p if i.op in (OP_SEND, OP_RECV))


def test_chimera_two_stage_is_bubble_free():
    s = build_schedule("chimera", 2, 4, 2)
    assert s.stats["makespan"] == pytest.approx(12.0)
    assert s.bubble_fraction() == pytest.approx(0.0)
    # both ranks hold both stages (one per pipe)
    assert sorted(s.local_stages(0)) == [(0, 0), (1, 1)]
    assert sorted(s.local_stages(1)) == [(0, 1), (1, 0)]


def test_1f1b_bounds_stashed_activations():
    P, M = 4, 16
    one = build_schedule("1f1b", P, M, P)
    gp = build_schedule("gpipe", P, M, P)
    assert one.stats["max_inflight"] <= P
    assert gp.stats["max_inflight"] == M
    # same work, 1F1B never slower than fill-drain in the unit-cost model
    assert one.stats["makespan"] <= gp.stats["makespan"]


def test_bubble_shrinks_with_microbatches():
    b = [build_schedule("1f1b", 4, m, 4).bubble_fraction() for m in (1, 4, 16)]
    assert b[0] > b[1] > b[2]


def _progs(s):
    return [[tuple(i) for i in p] for p in s.programs]


def test_validator_detects_order_mismatch():
    s = build_schedule("1f1b", 2, 4, 2)
    progs = _progs(s)
    # swap two receives on rank 1 (acts from rank 0 arrive in mb order)
    idx = [i for i, t in enumerate(progs[1]) if t[0] == OP_RECV]
    a, b = idx[0], idx[1]
    progs[1][a], progs[1][b] = progs[1][b], progs[1][a]
    with pytest.raises(ValueError, match="mismatch|after its consumer"):
        _native.runtime().validate_schedule("1f1b", 2, 4, 2, progs, 1.0, 2.0, False)


def test_validator_detects_deadlock():
    # rank 0 waits for a gradient before sending the activation that produces it
    prog0 = [(OP_FWD, 0, 0, 0, -1, -1), (OP_RECV, 0, 1, 0, 1, PL_GRAD), (OP_BWD, 0, 0, 0, -1, -1),
             (OP_SEND, 0, 0, 0, 1, PL_ACT)]
    prog1 = [(OP_RECV, 0, 0, 0, 0, PL_ACT), (OP_FWD, 0, 1, 0, -1, -1), (OP_BWD, 0, 1, 0, -1, -1),
             (OP_SEND, 0, 1, 0, 0, PL_GRAD)]
    with pytest.raises(ValueError, match="deadlock|before it is produced"):
        _native.runtime().validate_schedule("1f1b", 2, 1, 2, [prog0, prog1], 1.0, 2.0, False)


def test_validator_detects_missing_task():
    s = build_schedule("gpipe", 2, 2, 2)
    progs = _progs(s)
    progs[0] = [t for t in progs[0] if not (t[0] == OP_BWD and t[3] == 1)]
    with pytest.raises(ValueError, match="appears 0 times"):
        _native.runtime().validate_schedule("gpipe", 2, 2, 2, progs, 1.0, 2.0, False)


@pytest.mark.parametrize("args", [("nope", 2, 2, 2), ("1f1b", 3, 2, 2), ("1f1b", 0, 1, 1)])
def test_bad_specs(args):
    with pytest.raises(Exception):
        build_schedule(*args)


def test_instr_str():
    assert str(Instr(OP_SEND, 0, 1, 3, 2, PL_ACT)) == "S0.1.3>2a"


def test_rotate_fans_out_over_all_peers():
    R = 8
    s = build_schedule("rotate", 2, R * R, R)  # R micro-batches per owner: j -> rank owner+j
    for r, prog in enumerate(s.programs):
        peers = {i.peer for i in prog if i.op == OP_SEND and i.payload == PL_ACT}
        assert peers == set(range(R)) - {r}  # one activation message to each other GPU
    assert s.bubble_fraction() < 0.2

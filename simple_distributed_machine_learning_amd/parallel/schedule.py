"""Python view of the native pipeline schedules (csrc/runtime/schedule.cpp).

Kinds:

* ``gpipe``   — fill-drain: all forwards, then all backwards (BASELINE config 3).
* ``1f1b``    — PipeDream-flush: warm-up, steady one-forward-one-backward, cool-down;
                at most ``pp - pos`` activations stashed per rank (BASELINE config 4).
* ``chimera`` — two pipelines in opposite directions (rank r holds stage r of the "down"
                pipe and the mirrored stage of the "up" pipe); fills the bubble and, for
                a 2-stage split with a heavy first stage (the MNIST MLP: 100k of 101k
                MACs in fc1), balances the load across both GPUs.
* ``rotate``  — every rank owns a data shard and hosts every stage; micro-batch j of owner
                i runs stage s on rank (i + s*j) mod R. Each stage boundary fans out over
                ALL peers, so on an 8-GPU MI355X node the p2p traffic is spread over the 7
                xGMI links of every GPU instead of one neighbour link (and 1/R of it stays
                on-chip). Stage weights are replicated and all-reduced like DP.

The reference is the degenerate case: 2 stages, 1 micro-batch, strictly synchronous
(/root/reference/simple_distributed.py:108-113).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, NamedTuple, Tuple

from .._native import runtime

OP_FWD, OP_BWD, OP_SEND, OP_RECV = 0, 1, 2, 3
PL_ACT, PL_GRAD = 0, 1
KINDS = ("gpipe", "1f1b", "chimera", "rotate")


class Instr(NamedTuple):
    op: int
    pipe: int
    stage: int
    mb: int
    peer: int
    payload: int

    def __str__(self):
        n = {OP_FWD: "F", OP_BWD: "B", OP_SEND: "S", OP_RECV: "R"}[self.op]
        s = f"{n}{self.pipe}.{self.stage}.{self.mb}"
        if self.op in (OP_SEND, OP_RECV):
            s += f"{'>' if self.op == OP_SEND else '<'}{self.peer}{'a' if self.payload == PL_ACT else 'g'}"
        return s


@dataclass
class Schedule:
    kind: str
    num_stages: int
    num_microbatches: int
    num_ranks: int
    forward_only: bool
    programs: List[List[Instr]]
    stats: dict

    def program(self, pp_rank: int) -> List[Instr]:
        return self.programs[pp_rank]

    @property
    def num_pipes(self) -> int:
        if self.kind == "rotate":
            return self.num_ranks
        return 2 if self.kind == "chimera" else 1

    def stage_rank(self, pipe: int, stage: int) -> int:
        return stage_rank(self.kind, self.num_stages, self.num_ranks, pipe, stage)

    def task_rank(self, mb: int, stage: int) -> int:
        """Rank that computes ``stage`` of micro-batch ``mb`` (mirror of the C++ rule)."""
        if self.kind == "rotate":
            per = self.num_microbatches // self.num_ranks
            owner, j = divmod(mb, per)
            return (owner + stage * j) % self.num_ranks
        return self.stage_rank(self.mb_pipe(mb), stage)

    def mb_pipe(self, mb: int) -> int:
        if self.kind == "rotate":
            return mb // (self.num_microbatches // self.num_ranks)
        if self.num_pipes == 1:
            return 0
        half = (self.num_microbatches + 1) // 2
        return 0 if mb < half else 1

    def local_stages(self, pp_rank: int) -> List[Tuple[int, int]]:
        """(pipe, stage) pairs this rank computes, in first-use order."""
        out = []
        for ins in self.programs[pp_rank]:
            if ins.op in (OP_FWD, OP_BWD) and (ins.pipe, ins.stage) not in out:
                out.append((ins.pipe, ins.stage))
        if self.kind == "rotate":  # every rank hosts every stage
            for s in range(self.num_stages):
                if (pp_rank, s) not in out:
                    out.append((pp_rank, s))
        elif not out:  # a rank can be idle in a forward-only program with few micro-batches
            for p in range(self.num_pipes):
                for s in range(self.num_stages):
                    if self.stage_rank(p, s) == pp_rank:
                        out.append((p, s))
        return out

    def bubble_fraction(self) -> float:
        busy = self.stats.get("busy", [])
        ms = self.stats.get("makespan", 0.0)
        if not busy or ms <= 0:
            return 0.0
        return 1.0 - sum(busy) / (len(busy) * ms)

    def pretty(self) -> str:
        return "\n".join(f"rank {r}: " + " ".join(str(i) for i in p) for r, p in enumerate(self.programs))


def stage_rank(kind: str, num_stages: int, num_ranks: int, pipe: int, stage: int) -> int:
    r = stage // (num_stages // num_ranks)
    return r if pipe == 0 else num_ranks - 1 - r


def build_schedule(kind: str, num_stages: int, num_microbatches: int, num_ranks: int,
                   forward_only: bool = False, cost_f: float = 1.0, cost_b: float = 2.0,
                   validate: bool = True) -> Schedule:
    if kind not in KINDS:
        raise ValueError(f"unknown schedule kind {kind!r}; choose from {KINDS}")
    rt = runtime()
    progs, stats = rt.build_schedule(kind, num_stages, num_microbatches, num_ranks, cost_f, cost_b, forward_only)
    if validate:
        rt.validate_schedule(kind, num_stages, num_microbatches, num_ranks, progs, cost_f, cost_b, forward_only)
    programs = [[Instr(*t) for t in p] for p in progs]
    return Schedule(kind, num_stages, num_microbatches, num_ranks, forward_only, programs, stats)


def validate(schedule: Schedule) -> dict:
    """Re-validate (e.g. a hand-edited) schedule; raises ValueError on mismatch/deadlock."""
    progs = [[tuple(i) for i in p] for p in schedule.programs]
    return runtime().validate_schedule(schedule.kind, schedule.num_stages, schedule.num_microbatches,
                                       schedule.num_ranks, progs, 1.0, 2.0, schedule.forward_only)

// Pipeline schedule generator + deadlock/consistency validator (host C++).
//
// Replaces what the reference gets from PyTorch's C++ RPC/distributed-autograd runtime
// (SURVEY.md §2c): instead of a master process driving a remote stage with synchronous
// RPCs (/root/reference/simple_distributed.py:47-49, :71, :109-113), every rank executes a
// static, pre-validated instruction list (SPMD). The generator places stages on ranks,
// orders each rank's forward/backward work with a discrete-event list scheduler
// (GPipe fill-drain, 1F1B, Chimera bidirectional), inserts point-to-point sends/receives,
// and the validator replays the program under the exact stream semantics the engine uses
// on RCCL (one FIFO channel per ordered rank pair, compute stream gates) to prove that
// every message matches and nothing deadlocks.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace sdml {

enum OpType : int { OP_FWD = 0, OP_BWD = 1, OP_SEND = 2, OP_RECV = 3 };
enum Payload : int { PL_ACT = 0, PL_GRAD = 1, PL_NONE = -1 };

struct Instr {
  int op = 0;       // OpType
  int pipe = 0;     // pipeline id (Chimera runs two pipelines in opposite directions)
  int stage = 0;    // stage of the *computing* task (FWD/BWD) or of the message's producer
  int mb = 0;       // micro-batch id (global within the schedule)
  int peer = -1;    // SEND/RECV: other rank
  int payload = PL_NONE;
};

struct ScheduleSpec {
  std::string kind = "1f1b";  // gpipe | 1f1b | chimera | rotate
  int num_stages = 2;
  int num_microbatches = 1;
  int num_ranks = 2;
  double cost_f = 1.0;
  double cost_b = 2.0;
  bool forward_only = false;
};

struct SimStats {
  double makespan = 0.0;
  std::vector<double> busy;  // per rank
  int max_inflight = 0;      // max activations stashed on any rank
  int num_messages = 0;
};

// rank holding (pipe, stage) — placement-by-pipe kinds (gpipe, 1f1b, chimera)
int stage_rank(const ScheduleSpec& spec, int pipe, int stage);
// rank computing stage `stage` of micro-batch `mb` (all kinds). For "rotate": micro-batches
// are owned by ranks (owner = mb / (M/R)); local index j = mb % (M/R); stage s of it runs on
// rank (owner + s*j) mod R — every rank hosts every stage, and a stage boundary fans out to
// all peers (all xGMI links busy) instead of one neighbour.
int task_rank(const ScheduleSpec& spec, int mb, int stage);
int num_pipes(const ScheduleSpec& spec);
int mb_pipe(const ScheduleSpec& spec, int mb);

std::vector<std::vector<Instr>> build_schedule(const ScheduleSpec& spec, SimStats* stats);

// Throws std::runtime_error describing the first mismatch / deadlock.
SimStats validate_schedule(const ScheduleSpec& spec, const std::vector<std::vector<Instr>>& prog);

}  // namespace sdml

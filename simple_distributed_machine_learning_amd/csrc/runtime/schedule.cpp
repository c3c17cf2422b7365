// Pipeline schedule generator + validator. See schedule.h for the model.
//
// Reference behaviour being generalised: /root/reference/simple_distributed.py runs ONE
// micro-batch through a 2-stage split synchronously (forward :39-50 -> :69-80, backward via
// dist_autograd :112, optimizer :113). Here the same cut is scheduled over M micro-batches
// and R ranks so stages overlap instead of idling.
#include "schedule.h"

#include <algorithm>
#include <cmath>
#include <limits>
#include <map>
#include <sstream>
#include <stdexcept>
#include <tuple>

namespace sdml {

namespace {

struct Task {
  int pipe, stage, mb;
  bool bwd;
};

void check_spec(const ScheduleSpec& s) {
  if (s.num_stages < 1 || s.num_microbatches < 1 || s.num_ranks < 1)
    throw std::invalid_argument("schedule: num_stages, num_microbatches, num_ranks must be >= 1");
  if (s.kind != "rotate" && s.num_stages % s.num_ranks != 0)
    throw std::invalid_argument("schedule: num_stages must be a multiple of num_ranks");
  if (s.kind != "gpipe" && s.kind != "1f1b" && s.kind != "chimera" && s.kind != "rotate")
    throw std::invalid_argument("schedule: unknown kind '" + s.kind + "' (gpipe|1f1b|chimera|rotate)");
  if (s.kind == "rotate" && s.num_microbatches % s.num_ranks != 0)
    throw std::invalid_argument("schedule: rotate needs num_microbatches to be a multiple of num_ranks");
  if (!(s.cost_f > 0) || !(s.cost_b > 0)) throw std::invalid_argument("schedule: costs must be > 0");
}

// position of a rank along pipe p (0 = first rank to see the data)
int rank_pos(const ScheduleSpec& s, int pipe, int rank) {
  return pipe == 0 ? rank : s.num_ranks - 1 - rank;
}

int mb_index_in_pipe(const ScheduleSpec& s, int mb) {
  if (s.kind == "rotate") return mb % (s.num_microbatches / s.num_ranks);
  if (num_pipes(s) == 1) return mb;
  int half = (s.num_microbatches + 1) / 2;
  return mb < half ? mb : mb - half;
}

std::string tag_str(int payload, int pipe, int stage, int mb) {
  std::ostringstream o;
  o << (payload == PL_ACT ? "act" : "grad") << "(pipe=" << pipe << ",stage=" << stage << ",mb=" << mb << ")";
  return o.str();
}

using MsgKey = std::tuple<int, int, int, int>;  // payload, pipe, producer stage, mb

}  // namespace

int num_pipes(const ScheduleSpec& s) {
  if (s.kind == "rotate") return s.num_ranks;
  return s.kind == "chimera" ? 2 : 1;
}

int mb_pipe(const ScheduleSpec& s, int mb) {
  if (s.kind == "rotate") return mb / (s.num_microbatches / s.num_ranks);  // owner rank
  if (num_pipes(s) == 1) return 0;
  int half = (s.num_microbatches + 1) / 2;
  return mb < half ? 0 : 1;
}

int stage_rank(const ScheduleSpec& s, int pipe, int stage) {
  int r = stage / (s.num_stages / s.num_ranks);
  return pipe == 0 ? r : s.num_ranks - 1 - r;
}

int task_rank(const ScheduleSpec& s, int mb, int stage) {
  if (s.kind == "rotate") {
    int per = s.num_microbatches / s.num_ranks;
    int owner = mb / per, j = mb % per;
    return (owner + stage * j) % s.num_ranks;
  }
  return stage_rank(s, mb_pipe(s, mb), stage);
}

std::vector<std::vector<Instr>> build_schedule(const ScheduleSpec& spec, SimStats* stats_out) {
  check_spec(spec);
  const int P = spec.num_stages, M = spec.num_microbatches, R = spec.num_ranks;
  const bool fo = spec.forward_only;

  // ---- tasks ---------------------------------------------------------------------------
  // task id: ((mb * P) + stage) * 2 + bwd
  auto tid = [&](int stage, int mb, bool b) { return ((mb * P) + stage) * 2 + (b ? 1 : 0); };
  const int NT = M * P * 2;
  std::vector<double> finish(NT, -1.0);
  std::vector<char> started(NT, 0);
  std::vector<std::vector<int>> rank_tasks(R);
  for (int mb = 0; mb < M; ++mb) {
    for (int s = 0; s < P; ++s) {
      rank_tasks[task_rank(spec, mb, s)].push_back(tid(s, mb, false));
      if (!fo) rank_tasks[task_rank(spec, mb, s)].push_back(tid(s, mb, true));
    }
  }
  auto decode = [&](int t) {
    Task k;
    k.bwd = t & 1;
    int rest = t >> 1;
    k.stage = rest % P;
    k.mb = rest / P;
    k.pipe = mb_pipe(spec, k.mb);
    return k;
  };
  // dependency finish time, or -1 if not finished
  auto deps_ready = [&](const Task& k) -> double {
    double t = 0.0;
    auto need = [&](int d) -> bool {
      if (finish[d] < 0) return false;
      t = std::max(t, finish[d]);
      return true;
    };
    if (!k.bwd) {
      if (k.stage > 0 && !need(tid(k.stage - 1, k.mb, false))) return -1;
    } else {
      if (!need(tid(k.stage, k.mb, false))) return -1;
      if (k.stage < P - 1 && !need(tid(k.stage + 1, k.mb, true))) return -1;
    }
    return t;
  };

  // per (rank) bookkeeping for policies
  std::vector<int> f_total(R, 0), f_done_started(R, 0);
  for (int r = 0; r < R; ++r)
    for (int t : rank_tasks[r])
      if (!(t & 1)) f_total[r]++;
  // in-flight (F started, B not started) per (pipe, stage)
  std::vector<int> inflight((size_t)num_pipes(spec) * P, 0);
  int max_inflight_rank = 0;
  std::vector<int> rank_inflight(R, 0);

  std::vector<double> free_at(R, 0.0);
  std::vector<double> busy(R, 0.0);
  std::vector<std::vector<int>> order(R);
  int remaining = 0;
  for (int r = 0; r < R; ++r) remaining += (int)rank_tasks[r].size();

  double now = 0.0;
  const double INF = std::numeric_limits<double>::infinity();
  int guard = 0;
  while (remaining > 0) {
    if (++guard > 100000000) throw std::runtime_error("schedule: simulation did not converge");
    bool any = false;
    for (int r = 0; r < R; ++r) {
      if (free_at[r] > now + 1e-12) continue;
      // choose a task
      int best = -1;
      std::tuple<int, int, int, int> best_key{INT32_MAX, INT32_MAX, INT32_MAX, INT32_MAX};
      for (int t : rank_tasks[r]) {
        if (started[t]) continue;
        Task k = decode(t);
        double rt = deps_ready(k);
        if (rt < 0 || rt > now + 1e-12) continue;
        int pos = rank_pos(spec, k.pipe, r);
        int idx = mb_index_in_pipe(spec, k.mb);
        std::tuple<int, int, int, int> key;
        if (spec.kind == "gpipe") {
          if (k.bwd && f_done_started[r] < f_total[r]) continue;  // flush: all F before any B
          key = {k.bwd ? 1 : 0, idx, k.bwd ? -k.stage : k.stage, k.pipe};
        } else if (spec.kind == "rotate") {
          // backward first, then the deepest ready forward (frees stashed activations and
          // keeps every peer fed); own fresh micro-batches last
          key = {k.bwd ? 0 : 1, -k.stage, idx, (k.pipe - r + R) % R};
        } else {
          if (!k.bwd) {
            int limit = R - pos;  // warm-up depth of this rank along the pipe
            if (inflight[k.pipe * P + k.stage] >= limit) continue;
          }
          // Chimera: on ties prefer the pipe in which this rank sits earlier (it feeds others)
          int pkey = (num_pipes(spec) == 2) ? ((pos <= rank_pos(spec, 1 - k.pipe, r)) ? 0 : 1) : 0;
          key = {k.bwd ? 0 : 1, idx, pkey, k.bwd ? -k.stage : k.stage};
        }
        if (key < best_key) {
          best_key = key;
          best = t;
        }
      }
      if (best < 0) continue;
      Task k = decode(best);
      started[best] = 1;
      double c = k.bwd ? spec.cost_b : spec.cost_f;
      finish[best] = now + c;
      free_at[r] = now + c;
      busy[r] += c;
      order[r].push_back(best);
      remaining--;
      any = true;
      if (!k.bwd) {
        f_done_started[r]++;
        if (!fo) {
          inflight[k.pipe * P + k.stage]++;
          rank_inflight[r]++;
          max_inflight_rank = std::max(max_inflight_rank, rank_inflight[r]);
        }
      } else {
        inflight[k.pipe * P + k.stage]--;
        rank_inflight[r]--;
      }
    }
    if (remaining == 0) break;
    // advance time to next event
    double nxt = INF;
    for (int r = 0; r < R; ++r)
      if (free_at[r] > now + 1e-12) nxt = std::min(nxt, free_at[r]);
    for (int t = 0; t < NT; ++t)
      if (finish[t] > now + 1e-12) nxt = std::min(nxt, finish[t]);
    if (nxt == INF) {
      if (!any) throw std::runtime_error("schedule: policy deadlock in list scheduler (kind=" + spec.kind + ")");
      continue;
    }
    now = nxt;
  }

  // ---- instruction lists -----------------------------------------------------------------
  // 1) compute lists with sends placed right after their producer.
  std::vector<std::vector<Instr>> comp(R);
  // producer send order per channel (q -> r): list of MsgKey
  std::map<std::pair<int, int>, std::vector<MsgKey>> chan_order;
  int nmsg = 0;
  for (int r = 0; r < R; ++r) {
    for (int t : order[r]) {
      Task k = decode(t);
      Instr c;
      c.op = k.bwd ? OP_BWD : OP_FWD;
      c.pipe = k.pipe;
      c.stage = k.stage;
      c.mb = k.mb;
      comp[r].push_back(c);
      if (!k.bwd && k.stage < P - 1) {
        int dst = task_rank(spec, k.mb, k.stage + 1);
        if (dst != r) {
          Instr s{OP_SEND, k.pipe, k.stage, k.mb, dst, PL_ACT};
          comp[r].push_back(s);
          chan_order[{r, dst}].push_back(MsgKey{PL_ACT, k.pipe, k.stage, k.mb});
          nmsg++;
        }
      }
      if (k.bwd && k.stage > 0) {
        int dst = task_rank(spec, k.mb, k.stage - 1);
        if (dst != r) {
          Instr s{OP_SEND, k.pipe, k.stage, k.mb, dst, PL_GRAD};
          comp[r].push_back(s);
          chan_order[{r, dst}].push_back(MsgKey{PL_GRAD, k.pipe, k.stage, k.mb});
          nmsg++;
        }
      }
    }
  }
  // 2) receives: posted lazily, right before first use, but always in the producer's order
  //    (each ordered rank pair is one FIFO channel on the device side).
  std::vector<std::vector<Instr>> prog(R);
  for (int r = 0; r < R; ++r) {
    std::map<int, size_t> posted;  // src -> number of messages posted so far
    for (const Instr& in : comp[r]) {
      if (in.op == OP_FWD || in.op == OP_BWD) {
        int src = -1;
        MsgKey need;
        if (in.op == OP_FWD && in.stage > 0) {
          src = task_rank(spec, in.mb, in.stage - 1);
          need = MsgKey{PL_ACT, in.pipe, in.stage - 1, in.mb};
        } else if (in.op == OP_BWD && in.stage < P - 1) {
          src = task_rank(spec, in.mb, in.stage + 1);
          need = MsgKey{PL_GRAD, in.pipe, in.stage + 1, in.mb};
        }
        if (src >= 0 && src != r) {
          auto& ord = chan_order[{src, r}];
          auto it = std::find(ord.begin(), ord.end(), need);
          if (it == ord.end()) throw std::runtime_error("schedule: internal error, message never sent");
          size_t upto = (size_t)(it - ord.begin()) + 1;
          for (size_t j = posted[src]; j < upto; ++j) {
            auto [pl, pp, ps, pm] = ord[j];
            prog[r].push_back(Instr{OP_RECV, pp, ps, pm, src, pl});
          }
          posted[src] = std::max(posted[src], upto);
        }
      }
      prog[r].push_back(in);
    }
  }

  if (stats_out) {
    stats_out->makespan = 0;
    for (int r = 0; r < R; ++r) stats_out->makespan = std::max(stats_out->makespan, free_at[r]);
    stats_out->busy = busy;
    stats_out->max_inflight = max_inflight_rank;
    stats_out->num_messages = nmsg;
  }
  return prog;
}

SimStats validate_schedule(const ScheduleSpec& spec, const std::vector<std::vector<Instr>>& prog) {
  check_spec(spec);
  const int P = spec.num_stages, M = spec.num_microbatches, R = spec.num_ranks;
  if ((int)prog.size() != R) throw std::runtime_error("validate: program count != num_ranks");

  // every task exactly once, on its owner
  std::map<std::tuple<int, int, int>, int> seen;  // (stage, mb, bwd) -> count
  for (int r = 0; r < R; ++r) {
    for (const Instr& in : prog[r]) {
      if (in.op != OP_FWD && in.op != OP_BWD) continue;
      if (in.mb < 0 || in.mb >= M || in.stage < 0 || in.stage >= P)
        throw std::runtime_error("validate: task index out of range");
      int p = mb_pipe(spec, in.mb);
      if (in.pipe != p) throw std::runtime_error("validate: micro-batch on wrong pipe");
      if (task_rank(spec, in.mb, in.stage) != r) throw std::runtime_error("validate: task on wrong rank");
      seen[{in.stage, in.mb, in.op == OP_BWD}]++;
    }
  }
  for (int mb = 0; mb < M; ++mb)
    for (int s = 0; s < P; ++s)
      for (int b = 0; b < (spec.forward_only ? 1 : 2); ++b) {
        auto it = seen.find({s, mb, b == 1});
        if (it == seen.end() || it->second != 1) {
          std::ostringstream o;
          o << "validate: task " << (b ? "B" : "F") << "(stage=" << s << ",mb=" << mb << ") appears "
            << (it == seen.end() ? 0 : it->second) << " times";
          throw std::runtime_error(o.str());
        }
      }

  // channels
  struct Msg {
    MsgKey key;
    int gate;  // compute items that must be complete on the posting rank
    int pos;   // instruction index
  };
  std::map<std::pair<int, int>, std::vector<Msg>> sends, recvs;
  std::vector<std::vector<int>> comp_idx(R);  // instruction indices of compute items
  for (int r = 0; r < R; ++r) {
    int ncomp = 0;
    for (int i = 0; i < (int)prog[r].size(); ++i) {
      const Instr& in = prog[r][i];
      if (in.op == OP_FWD || in.op == OP_BWD) {
        comp_idx[r].push_back(i);
        ncomp++;
      } else if (in.op == OP_SEND || in.op == OP_RECV) {
        if (in.peer < 0 || in.peer >= R || in.peer == r) throw std::runtime_error("validate: bad peer");
        Msg m{MsgKey{in.payload, in.pipe, in.stage, in.mb}, ncomp, i};
        if (in.op == OP_SEND)
          sends[{r, in.peer}].push_back(m);
        else
          recvs[{in.peer, r}].push_back(m);
      } else {
        throw std::runtime_error("validate: unknown op");
      }
    }
  }
  for (auto& [ch, sv] : sends) {
    auto& rv = recvs[ch];
    if (sv.size() != rv.size()) {
      std::ostringstream o;
      o << "validate: channel " << ch.first << "->" << ch.second << " has " << sv.size() << " sends but "
        << rv.size() << " receives";
      throw std::runtime_error(o.str());
    }
    for (size_t k = 0; k < sv.size(); ++k)
      if (sv[k].key != rv[k].key) {
        auto [a, b, c, d] = sv[k].key;
        auto [e, f, g, h] = rv[k].key;
        std::ostringstream o;
        o << "validate: channel " << ch.first << "->" << ch.second << " message #" << k << " order mismatch: sent "
          << tag_str(a, b, c, d) << " but receiver expects " << tag_str(e, f, g, h);
        throw std::runtime_error(o.str());
      }
  }
  for (auto& [ch, rv] : recvs)
    if (!rv.empty() && sends.find(ch) == sends.end())
      throw std::runtime_error("validate: receives on a channel nobody sends on");

  // message location lookup: key -> (channel, index)
  std::map<MsgKey, std::pair<std::pair<int, int>, int>> where;
  for (auto& [ch, sv] : sends)
    for (int k = 0; k < (int)sv.size(); ++k) where[sv[k].key] = {ch, k};

  // producer-before-send and local dependency checks
  std::map<std::tuple<int, int, int>, std::pair<int, int>> task_pos;  // (stage,mb,bwd)->(rank, instr idx)
  for (int r = 0; r < R; ++r)
    for (int i = 0; i < (int)prog[r].size(); ++i) {
      const Instr& in = prog[r][i];
      if (in.op == OP_FWD || in.op == OP_BWD) task_pos[{in.stage, in.mb, in.op == OP_BWD}] = {r, i};
    }
  for (auto& [ch, sv] : sends)
    for (auto& m : sv) {
      auto [pl, pp, ps, pm] = m.key;
      auto it = task_pos.find({ps, pm, pl == PL_GRAD});
      if (it == task_pos.end() || it->second.first != ch.first || it->second.second > m.pos)
        throw std::runtime_error("validate: " + tag_str(pl, pp, ps, pm) + " sent before it is produced");
    }

  // requirements of each compute item: list of (channel, msg index) or local task
  struct Need {
    int kind;  // 0 = message, 1 = local task
    std::pair<int, int> ch;
    int k;
    int lrank, lidx;
  };
  std::vector<std::vector<std::vector<Need>>> needs(R);
  for (int r = 0; r < R; ++r) {
    needs[r].resize(comp_idx[r].size());
    for (size_t c = 0; c < comp_idx[r].size(); ++c) {
      const Instr& in = prog[r][comp_idx[r][c]];
      auto add_dep = [&](int payload, int stage_prod, bool prod_bwd) {
        int pr = task_rank(spec, in.mb, stage_prod);
        if (pr == r) {
          auto tp = task_pos.at({stage_prod, in.mb, prod_bwd});
          if (tp.second > comp_idx[r][c])
            throw std::runtime_error("validate: local dependency scheduled after its consumer");
          return;
        }
        MsgKey key{payload, in.pipe, stage_prod, in.mb};
        auto it = where.find(key);
        if (it == where.end()) throw std::runtime_error("validate: missing message " + tag_str(payload, in.pipe, stage_prod, in.mb));
        // the receive must be posted before the consumer
        auto& rv = recvs[it->second.first];
        if (rv[it->second.second].pos > comp_idx[r][c])
          throw std::runtime_error("validate: receive of " + tag_str(payload, in.pipe, stage_prod, in.mb) +
                                   " posted after its consumer");
        needs[r][c].push_back(Need{0, it->second.first, it->second.second, 0, 0});
      };
      if (in.op == OP_FWD && in.stage > 0) add_dep(PL_ACT, in.stage - 1, false);
      if (in.op == OP_BWD) {
        auto tp = task_pos.find({in.stage, in.mb, false});
        if (tp == task_pos.end() || tp->second.second > comp_idx[r][c])
          throw std::runtime_error("validate: backward before its forward");
        if (in.stage < P - 1) add_dep(PL_GRAD, in.stage + 1, true);
      }
    }
  }

  // ---- replay with device-stream semantics ------------------------------------------------
  std::vector<int> done(R, 0);
  std::vector<double> t_done(R, 0.0);  // time the compute stream finished its last item
  std::vector<std::vector<double>> comp_end(R);
  for (int r = 0; r < R; ++r) comp_end[r].assign(comp_idx[r].size(), -1);
  std::map<std::pair<int, int>, int> ch_done;
  std::map<std::pair<int, int>, std::vector<double>> ch_time;
  for (auto& [ch, sv] : sends) {
    ch_done[ch] = 0;
    ch_time[ch].assign(sv.size(), -1);
  }
  auto gate_time = [&](int r, int gate) -> double {  // time when compute stream of r passed `gate` items
    if (gate == 0) return 0.0;
    return comp_end[r][gate - 1];
  };
  bool progress = true;
  while (progress) {
    progress = false;
    for (auto& [ch, sv] : sends) {
      int& k = ch_done[ch];
      while (k < (int)sv.size()) {
        const Msg& s = sv[k];
        const Msg& rcv = recvs[ch][k];
        if (done[ch.first] < s.gate || done[ch.second] < rcv.gate) break;
        double t = std::max(gate_time(ch.first, s.gate), gate_time(ch.second, rcv.gate));
        if (k > 0) t = std::max(t, ch_time[ch][k - 1]);
        ch_time[ch][k] = t;
        k++;
        progress = true;
      }
    }
    for (int r = 0; r < R; ++r) {
      while (done[r] < (int)comp_idx[r].size()) {
        int c = done[r];
        double start = t_done[r];
        bool ok = true;
        for (auto& nd : needs[r][c]) {
          if (ch_done[nd.ch] <= nd.k) {
            ok = false;
            break;
          }
          start = std::max(start, ch_time[nd.ch][nd.k]);
        }
        if (!ok) break;
        const Instr& in = prog[r][comp_idx[r][c]];
        double cost = in.op == OP_BWD ? spec.cost_b : spec.cost_f;
        comp_end[r][c] = start + cost;
        t_done[r] = start + cost;
        done[r]++;
        progress = true;
      }
    }
  }
  for (int r = 0; r < R; ++r)
    if (done[r] < (int)comp_idx[r].size()) {
      const Instr& in = prog[r][comp_idx[r][done[r]]];
      std::ostringstream o;
      o << "validate: deadlock: rank " << r << " blocked at " << (in.op == OP_FWD ? "F" : "B") << "(pipe=" << in.pipe
        << ",stage=" << in.stage << ",mb=" << in.mb << ")";
      throw std::runtime_error(o.str());
    }

  SimStats st;
  st.busy.assign(R, 0.0);
  for (int r = 0; r < R; ++r) {
    st.makespan = std::max(st.makespan, t_done[r]);
    int infl = 0;
    for (int c = 0; c < (int)comp_idx[r].size(); ++c) {
      const Instr& in = prog[r][comp_idx[r][c]];
      st.busy[r] += in.op == OP_BWD ? spec.cost_b : spec.cost_f;
      if (!spec.forward_only) {
        infl += in.op == OP_FWD ? 1 : -1;
        st.max_inflight = std::max(st.max_inflight, infl);
      }
    }
  }
  for (auto& [ch, sv] : sends) st.num_messages += (int)sv.size();
  return st;
}

}  // namespace sdml

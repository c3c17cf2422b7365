// Host-side sanitizer driver for the native runtime (csrc/runtime/schedule.cpp and the synthetic
// data hash in csrc/common/synth_hash.h): built with -fsanitize=address,undefined by
// tests/test_native_sanitize.py and run on the CPU (GPU AddressSanitizer is not available on the
// MI355X pool, so the host code is where memory and UB checks run). It sweeps every schedule kind
// over a grid of stage / micro-batch / rank counts, validates each generated program, checks that
// corrupted programs (swapped receives, a dropped task) are rejected, and that bad specs throw.
// The multi-threaded synthetic-data fill (csrc/runtime/synth_fill.h) is checked against its
// single-threaded result; built with -fsanitize=thread and -DSDML_SYNTH_ONLY this is the data
// race check of the runtime's only threaded code.
#include <cstdio>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "schedule.h"
#include "synth_fill.h"

using namespace sdml;

static int failures = 0;

static void check(bool ok, const std::string& what) {
  if (!ok) {
    std::fprintf(stderr, "FAIL: %s\n", what.c_str());
    ++failures;
  }
}

static std::string tag(const ScheduleSpec& s) {
  return s.kind + " P=" + std::to_string(s.num_stages) + " M=" + std::to_string(s.num_microbatches) +
         " R=" + std::to_string(s.num_ranks) + (s.forward_only ? " fwd" : "");
}

// nt threads vs one thread over the same samples: bit-identical images and labels
static void synth_check(unsigned nt) {
  const int64_t n = 6000;
  const int H = 28, W = 28;
  for (int mode = 0; mode <= 1; ++mode) {
    std::vector<float> x1(n * H * W), xn(n * H * W);
    std::vector<int64_t> y1(n), yn(n);
    synth_fill_host(1234, 777, n, H, W, mode, x1.data(), y1.data(), 1);
    synth_fill_host(1234, 777, n, H, W, mode, xn.data(), yn.data(), nt);
    check(x1 == xn && y1 == yn, "threaded synthetic fill differs (mode " + std::to_string(mode) + ")");
  }
}

int main() {
  synth_check(8);
#ifdef SDML_SYNTH_ONLY
  std::printf("runtime sanitize (synth only): %d failures\n", failures);
  return failures == 0 ? 0 : 1;
#endif
  int programs = 0;
  for (const char* kind : {"gpipe", "1f1b", "chimera", "rotate"}) {
    for (int R = 1; R <= 8; ++R)
      for (int mult = 1; mult <= 2; ++mult)
        for (int M = 1; M <= 16; ++M)
          for (int fo = 0; fo <= 1; ++fo) {
            ScheduleSpec s;
            s.kind = kind;
            s.num_ranks = R;
            s.num_stages = std::string(kind) == "rotate" ? 2 : R * mult;
            s.num_microbatches = std::string(kind) == "rotate" ? M * R : M;
            s.forward_only = fo;
            if (std::string(kind) == "rotate" && mult == 2) continue;
            std::vector<std::vector<Instr>> prog;
            try {
              SimStats st;
              prog = build_schedule(s, &st);
              SimStats v = validate_schedule(s, prog);
              check(v.num_messages == st.num_messages || st.num_messages == 0, "message count " + tag(s));
              ++programs;
            } catch (const std::invalid_argument&) {
              continue;  // a spec this kind does not take (e.g. chimera's stage/rank constraints)
            } catch (const std::exception& e) {
              check(false, tag(s) + ": " + e.what());
              continue;
            }
            // corrupt: swap the first two receives of a rank that has two -> must be rejected
            for (auto& rp : prog) {
              int a = -1, b = -1;
              for (int i = 0; i < (int)rp.size(); ++i)
                if (rp[i].op == OP_RECV) {
                  if (a < 0) a = i;
                  else if (rp[i].peer == rp[a].peer && (rp[i].mb != rp[a].mb || rp[i].payload != rp[a].payload)) {
                    b = i;
                    break;
                  }
                }
              if (a >= 0 && b >= 0) {
                std::swap(rp[a], rp[b]);
                bool threw = false;
                try {
                  validate_schedule(s, prog);
                } catch (const std::runtime_error&) {
                  threw = true;
                }
                check(threw, "swapped receives accepted " + tag(s));
                std::swap(rp[a], rp[b]);
                break;
              }
            }
            // corrupt: drop the last compute task of rank 0 -> must be rejected
            for (int i = (int)prog[0].size() - 1; i >= 0; --i)
              if (prog[0][i].op == OP_FWD || prog[0][i].op == OP_BWD) {
                auto saved = prog[0][i];
                prog[0].erase(prog[0].begin() + i);
                bool threw = false;
                try {
                  validate_schedule(s, prog);
                } catch (const std::runtime_error&) {
                  threw = true;
                }
                check(threw, "dropped task accepted " + tag(s));
                prog[0].insert(prog[0].begin() + i, saved);
                break;
              }
          }
  }
  for (auto bad : {std::make_pair(0, 1), std::make_pair(3, 2)}) {  // stages < 1; stages % ranks
    ScheduleSpec s;
    s.num_stages = bad.first;
    s.num_ranks = bad.second;
    bool threw = false;
    try {
      build_schedule(s, nullptr);
    } catch (const std::invalid_argument&) {
      threw = true;
    }
    check(threw, "bad spec accepted");
  }
  std::printf("runtime sanitize: %d programs validated, %d failures\n", programs, failures);
  return failures == 0 && programs > 100 ? 0 : 1;
}

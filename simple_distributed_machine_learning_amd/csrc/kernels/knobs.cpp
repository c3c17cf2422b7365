// Kernel-variant switch table (see knobs.h).
#include "knobs.h"

#include <cstdlib>
#include <cstring>

namespace sdml {
namespace {

struct Entry {
  const char* name;  // set_knob name; the environment variable is SDML_<name> (experiments builds)
  int dflt;
  bool probe;        // timing-only switch: pinned to dflt in production builds
  const char* word;  // environment value meaning 1 (string-valued variables), else nullptr: atoi
};

// order = KnobId
const Entry kTable[KNOB_COUNT] = {
    {"CONV_FWD_IM2COL", 0, false, "im2col"},
    {"CONV_BN128_MIN", 160, false, nullptr},
    {"CONV_WG_ROWS64", 1, false, nullptr},
    {"CONV_WG_BLOCKS", 512, false, nullptr},
    {"CONV_WGRAD_DMA", 0, false, nullptr},
    {"CONV_WGRAD_STAGES", 2, false, nullptr},
    {"GEMM_NT_STORE", 0, false, nullptr},
    {"GEMM_BF16_2PHASE", 0, false, "2phase"},
    {"WGRAD_WAVES", 1, false, nullptr},
    {"WGRAD_DMA", 1, false, nullptr},
    {"X2_2PHASE", 0, false, "2phase"},
    {"X3_DEEP", -1, false, nullptr},
    {"HEAD_VALU", 0, false, "v1"},
    {"HEAD_MAX_BLOCKS", 512, false, nullptr},
    {"U8_WGRAD_XCD", 1, false, nullptr},
    {"U8_FWD_WMT", 0, false, nullptr},
    {"U8_FWD_WAVES", 0, false, nullptr},
    {"U8_FWD_X3", 0, false, "x3"},
    {"U8_WGRAD_X3", 0, false, "x3"},
    {"U8_FH_STAGES", 2, false, nullptr},
    {"U8_FWD_PRIO", 0, false, nullptr},
    {"U8_WGRAD_PRIO", 0, false, nullptr},
    {"CNN_SPLIT_BWD", 1, false, nullptr},
    {"U8_WGRAD_ILV", 0, false, nullptr},
    {"GEMM_BF16_T2", 0, false, nullptr},
    {"U8_WGRAD_RING", 1, false, nullptr},
    {"U8_WGRAD_BAL", 0, false, nullptr},
    {"U8_FWD_DMA_SPREAD", 0, false, nullptr},
    {"GEMM_BF16_N192", -1, false, nullptr},
    {"U8_FWD_PREFETCH", 1, false, nullptr},
    {"U8_SLAB_COLS", 64, false, nullptr},
    {"GEMM_BF16_TR", 1, false, nullptr},
    {"WGRAD_NFAST", -1, false, nullptr},
    {"ATTN_DKDV_KT", 1, false, nullptr},
    {"U8_FH_ROWS512", 0, false, nullptr},
    {"GEMM_GROUP_M", 8, false, nullptr},
    {"GEMM_BF16_W4", 0, false, nullptr},
    {"U8_WGRAD_PAIR", 0, false, nullptr},
    {"ATTN_FWD_QS", 1, false, nullptr},
    {"SGD_MIXED_V", 0, false, nullptr},
    {"ATTN_OCC", 2, false, nullptr},
    {"CONV_HALO_1WG", 0, false, nullptr},
    {"GEMM_BF16_PERSIST", -1, false, nullptr},
    {"GEMM_BF16_NOSTORE", 0, true, nullptr},
    {"U8_VARIANT", 0, true, nullptr},
};

#ifdef SDML_KERNEL_EXPERIMENTS
constexpr bool kExperiments = true;
// the environment variable names of rounds 1-3, for the timing tools that still set them
const char* env_name(int i) {
  switch (i) {
    case KNOB_CONV_FWD_IM2COL: return "SDML_CONV_FWD";
    case KNOB_GEMM_BF16_2PHASE: return "SDML_GEMM_BF16_NT";
    case KNOB_X2_2PHASE: return "SDML_X2_NT";
    case KNOB_HEAD_VALU: return "SDML_HEAD";
    case KNOB_U8_FWD_X3: return "SDML_U8_FWD";
    case KNOB_U8_WGRAD_X3: return "SDML_U8_WGRAD";
    default: return nullptr;
  }
}
#else
constexpr bool kExperiments = false;
#endif

struct State {
  int value[KNOB_COUNT];
  State() {
    for (int i = 0; i < KNOB_COUNT; ++i) {
      value[i] = kTable[i].dflt;
#ifdef SDML_KERNEL_EXPERIMENTS
      char buf[64] = "SDML_";
      std::strncat(buf, kTable[i].name, sizeof(buf) - 6);
      const char* e = std::getenv(buf);
      if (!e && env_name(i)) e = std::getenv(env_name(i));
      if (e && *e) value[i] = kTable[i].word ? (std::strcmp(e, kTable[i].word) == 0 ? 1 : std::atoi(e)) : std::atoi(e);
#endif
    }
  }
};

State& state() {
  static State s;  // built once (thread-safe static init)
  return s;
}

}  // namespace

int knob(KnobId id) {
  if (!kExperiments && kTable[id].probe) return kTable[id].dflt;
  return state().value[id];
}

bool set_knob(const char* name, int value) {
  for (int i = 0; i < KNOB_COUNT; ++i) {
    if (std::strcmp(kTable[i].name, name) == 0) {
      if (kTable[i].probe && !kExperiments) return false;
      state().value[i] = value;
      return true;
    }
  }
  return false;
}

void reset_knobs() {
  for (int i = 0; i < KNOB_COUNT; ++i) state().value[i] = kTable[i].dflt;
}

bool kernel_experiments_build() { return kExperiments; }

}  // namespace sdml

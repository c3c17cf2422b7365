// Host fill of the counter-based synthetic MNIST-shape data (csrc/common/synth_hash.h, the same
// hash the HIP generator uses): sample i of the batch is start + i; threads take samples
// t, t + nt, ... and write disjoint rows. Shared by the pybind11 binding and the ThreadSanitizer
// driver (tests/native/runtime_sanitize.cpp).
#pragma once

#include <algorithm>
#include <cstdint>
#include <thread>
#include <vector>

#include "synth_hash.h"

namespace sdml {

inline void synth_fill_host(uint64_t seed, int64_t start, int64_t n, int H, int W, int mode, float* x, int64_t* y,
                            unsigned nt) {
  const int D = H * W;
  nt = std::max(1u, nt);
  auto work = [&](unsigned t) {
    for (int64_t i = t; i < n; i += nt) {
      const uint64_t smp = (uint64_t)(start + i);
      if (y) y[i] = synth_label(seed, smp);
      if (x)
        for (int p = 0; p < D; ++p) x[i * D + p] = synth_pixel(seed, smp, p, H, W, mode);
    }
  };
  std::vector<std::thread> th;
  for (unsigned t = 1; t < nt; ++t) th.emplace_back(work, t);
  work(0);
  for (auto& t : th) t.join();
}

}  // namespace sdml

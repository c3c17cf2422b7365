// Counter-based synthetic data (host + device).
//
// The reference trains on torchvision MNIST (/root/reference/simple_distributed.py:87-95);
// there is no network here or on the GPU boxes, so the framework generates an MNIST-shape
// dataset from a seed. Every pixel/label is a pure function of (seed, sample, pixel), so
// every rank - and the CPU test path - materialises bit-identical data with no
// communication: the first stage reads images, the last stage reads labels (labels never
// travel over the wire).
//
// Data model ("learnable" mode): 10 class prototypes made of a few Gaussian-ish blobs,
// x = clamp(0.75 * proto[y] + 0.25 * u, 0, 1), u ~ U[0,1). Labels uniform in [0,10).
#pragma once

#include <cstdint>

#if defined(__HIPCC__)
#define SDML_HD __host__ __device__ __forceinline__
#else
#define SDML_HD inline
#endif

#if defined(__clang__)
// bit-identical host (g++/SSE) and device (hipcc) results: no FMA contraction in here
#pragma clang fp contract(off)
#endif

namespace sdml {

SDML_HD uint32_t mix32(uint64_t x) {
  // splitmix64 finaliser folded to 32 bits
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  x ^= x >> 31;
  return (uint32_t)(x ^ (x >> 32));
}

SDML_HD float u01(uint32_t h) {  // [0,1) with 24 bits
  return (float)(h >> 8) * (1.0f / 16777216.0f);
}

SDML_HD uint32_t hash3(uint64_t seed, uint64_t a, uint64_t b) {
  return mix32(seed * 0x100000001B3ull ^ mix32(a * 0x9E3779B1ull + 0x632BE5ABull) ^ ((uint64_t)mix32(b + 0x7F4A7C15ull) << 32));
}

constexpr int kSynthClasses = 10;
constexpr int kBlobs = 3;

SDML_HD int synth_label(uint64_t seed, uint64_t sample) {
  return (int)(hash3(seed, sample, 0xFFFFFFFFull) % kSynthClasses);
}

// prototype intensity of class c at pixel (py, px) of an HxW image
SDML_HD float synth_proto(uint64_t seed, int c, int py, int px, int H, int W) {
  float v = 0.f;
  for (int k = 0; k < kBlobs; ++k) {
    uint32_t h0 = hash3(seed ^ 0xC0FFEEull, (uint64_t)c * 16 + k, 1);
    uint32_t h1 = hash3(seed ^ 0xC0FFEEull, (uint64_t)c * 16 + k, 2);
    uint32_t h2 = hash3(seed ^ 0xC0FFEEull, (uint64_t)c * 16 + k, 3);
    float cy = 0.2f * H + 0.6f * H * u01(h0);
    float cx = 0.2f * W + 0.6f * W * u01(h1);
    float rad = 0.08f * H + 0.12f * H * u01(h2);
    float dy = (py - cy) / rad, dx = (px - cx) / rad;
    float d2 = dy * dy + dx * dx;
    // cheap smooth bump (no transcendental -> identical host/device results)
    float b = 1.f - d2;
    v += b > 0.f ? b * b : 0.f;
  }
  return v > 1.f ? 1.f : v;
}

// mode 0: learnable (prototype + noise); mode 1: pure uniform noise (reference harness
// style)
SDML_HD float synth_pixel(uint64_t seed, uint64_t sample, int pix, int H, int W, int mode) {
  float u = u01(hash3(seed, sample, (uint64_t)pix));
  if (mode == 1) return u;
  int y = synth_label(seed, sample);
  float p = synth_proto(seed, y, pix / W, pix % W, H, W);
  float x = 0.75f * p + 0.25f * u;
  return x < 0.f ? 0.f : (x > 1.f ? 1.f : x);
}

}  // namespace sdml

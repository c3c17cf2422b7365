// Numerics probe: does v_mfma_f32_32x32x16_bf16 round its fp32 accumulation like an fp32 fma chain
// (round-to-nearest-even), or with a bias that grows with the running sum? Compares a long MFMA
// accumulation chain (C fed back every K=16 step) against "fresh" 32-deep partials added with VALU
// adds, against fp64 and a host fp32 fmaf chain. Operands are positive so a biased rounding mode
// shows up as a signed drift.   hipcc --offload-arch=gfx950 -O3 mfma_acc_probe.hip -o probe
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <cstring>
#include <vector>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));

// A [32][K] row-major, B [32][K] row-major (B^T), both bf16 bits; C [32][32]
__global__ void probe(const unsigned short* A, const unsigned short* B, int K, float* Cchain, float* Cfresh) {
  const int l = threadIdx.x, r = l & 31, h = l >> 5;
  f32x16 acc = {}, acc2 = {};
  for (int k0 = 0; k0 < K; k0 += 32) {
    f32x16 part = {};
    for (int s = 0; s < 2; ++s) {
      bf16x8 a, b;
      for (int j = 0; j < 8; ++j) {
        a[j] = (short)A[r * K + k0 + 16 * s + 8 * h + j];
        b[j] = (short)B[r * K + k0 + 16 * s + 8 * h + j];
      }
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
      part = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, part, 0, 0, 0);
    }
    acc2 += part;
  }
  for (int i = 0; i < 16; ++i) {
    const int row = (i & 3) + 8 * (i >> 2) + 4 * h;
    Cchain[row * 32 + r] = acc[i];
    Cfresh[row * 32 + r] = acc2[i];
  }
}

static unsigned short to_bf16(float f) {  // RNE
  unsigned u;
  memcpy(&u, &f, 4);
  u += 0x7fff + ((u >> 16) & 1);
  return (unsigned short)(u >> 16);
}
static float from_bf16(unsigned short b) {
  unsigned u = (unsigned)b << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}

int main() {
  const int Ks[3] = {784, 4096, 32768};
  for (int mode = 0; mode < 2; ++mode) {
    for (int K : Ks) {
      std::mt19937 g(1234 + K);
      std::uniform_real_distribution<float> U(mode == 0 ? 0.5f : -1.f, 1.f);
      std::vector<unsigned short> A(32 * K), B(32 * K);
      for (auto& v : A) v = to_bf16(U(g));
      for (auto& v : B) v = to_bf16(U(g));
      unsigned short *dA, *dB;
      float *dC1, *dC2;
      hipMalloc(&dA, A.size() * 2);
      hipMalloc(&dB, B.size() * 2);
      hipMalloc(&dC1, 4096);
      hipMalloc(&dC2, 4096);
      hipMemcpy(dA, A.data(), A.size() * 2, hipMemcpyHostToDevice);
      hipMemcpy(dB, B.data(), B.size() * 2, hipMemcpyHostToDevice);
      probe<<<1, 64>>>(dA, dB, K, dC1, dC2);
      std::vector<float> C1(1024), C2(1024);
      hipMemcpy(C1.data(), dC1, 4096, hipMemcpyDeviceToHost);
      hipMemcpy(C2.data(), dC2, 4096, hipMemcpyDeviceToHost);
      double e[3] = {0, 0, 0}, bias[3] = {0, 0, 0}, mx[3] = {0, 0, 0};
      for (int i = 0; i < 32; ++i)
        for (int j = 0; j < 32; ++j) {
          double ex = 0, mag = 0;
          float f = 0.f;
          for (int k = 0; k < K; ++k) {
            const double p = (double)from_bf16(A[i * K + k]) * from_bf16(B[j * K + k]);
            ex += p;
            mag += fabs(p);
            f = fmaf(from_bf16(A[i * K + k]), from_bf16(B[j * K + k]), f);
          }
          const double got[3] = {C1[i * 32 + j], C2[i * 32 + j], f};
          for (int t = 0; t < 3; ++t) {
            const double d = (got[t] - ex) / mag;
            e[t] += fabs(d) / 1024;
            bias[t] += d / 1024;
            mx[t] = fmax(mx[t], fabs(d));
          }
        }
      printf("%s K=%6d  chain: mean %.3g max %.3g bias %+.3g | fresh32: mean %.3g max %.3g bias %+.3g | host fmaf chain: mean %.3g max %.3g bias %+.3g  (relative to sum|a*b|)\n",
             mode == 0 ? "pos" : "sym", K, e[0], mx[0], bias[0], e[1], mx[1], bias[1], e[2], mx[2], bias[2]);
      hipFree(dA);
      hipFree(dB);
      hipFree(dC1);
      hipFree(dC2);
    }
  }
  return 0;
}

// tanh-GELU (GPT-2's activation) and its derivative, shared by gpt2_ops.hip's standalone kernels and
// gemm_bf16.hip's fused epilogues so both produce the same bits. With s = sigmoid(2u) = (1 + tanh u) / 2,
// u = sqrt(2/pi) (x + 0.044715 x^3):
//   gelu(x)  = 0.5 x (1 + tanh u) = x s
//   gelu'(x) = 0.5 (1 + tanh u) + 0.5 x (1 - tanh^2 u) u'  = s + 2 x s (1 - s) sqrt(2/pi) (1 + 3 * 0.044715 x^2)
// (the same functions as PyTorch's approximate="tanh" formulas, evaluated with one __expf instead of
// tanhf: ~5x fewer instructions, within a few fp32 ulps, below bf16 output resolution)
#pragma once

#include <hip/hip_runtime.h>

namespace sdml {

constexpr float kGeluBeta = 0.7978845608028654f;  // sqrt(2 / pi)
constexpr float kGeluKappa = 0.044715f;

__device__ __forceinline__ float gelu_sig(float x) {
  const float u = kGeluBeta * (x + kGeluKappa * (x * x * x));
  return __fdividef(1.f, 1.f + __expf(-2.f * u));
}

__device__ __forceinline__ float gelu_f(float x) { return x * gelu_sig(x); }

__device__ __forceinline__ float gelu_grad_f(float dy, float x) {
  const float s = gelu_sig(x);
  return dy * (s + 2.f * x * s * (1.f - s) * kGeluBeta * (1.f + 3.f * kGeluKappa * (x * x)));
}

}  // namespace sdml

// Torch bindings of the gfx950 kernels (_kernels module). The only TU that includes torch
// headers. Every entry point validates shapes/dtypes/devices on the host before launching
// (a kernel must never see operands its grid does not assume) and launches on the current
// PyTorch HIP stream, so the ops compose with torch streams, events and hipGraph capture.
#include <ATen/hip/HIPContext.h>
#include <cmath>
#include <torch/extension.h>

#include "kernels.h"

namespace {

hipStream_t cur_stream() { return at::hip::getCurrentHIPStream().stream(); }

void check_f32_cuda(const torch::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a ROCm device tensor");
  TORCH_CHECK(t.scalar_type() == torch::kFloat32, name, " must be float32");
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}

void check_opt(const c10::optional<torch::Tensor>& t, const char* name, int64_t numel) {
  if (t.has_value() && t->defined()) {
    check_f32_cuda(*t, name);
    TORCH_CHECK(t->numel() == numel, name, " has ", t->numel(), " elements, expected ", numel);
  }
}

float* opt_ptr(const c10::optional<torch::Tensor>& t) {
  return (t.has_value() && t->defined()) ? t->data_ptr<float>() : nullptr;
}

// y = act(x @ w.T + b); x [M,K], w [N,K], b [N] or None
torch::Tensor linear_fwd_f32(torch::Tensor x, torch::Tensor w, c10::optional<torch::Tensor> b, bool relu) {
  check_f32_cuda(x, "x");
  check_f32_cuda(w, "w");
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && x.size(1) == w.size(1), "linear_fwd_f32: shape mismatch ",
              x.sizes(), " vs ", w.sizes());
  const int64_t M = x.size(0), K = x.size(1), N = w.size(0);
  check_opt(b, "b", N);
  auto y = torch::empty({M, N}, x.options());
  if (M == 0) return y;
  sdml::GemmArgs g;
  g.A = x.data_ptr<float>();
  g.B = w.data_ptr<float>();
  g.C = y.data_ptr<float>();
  g.bias = opt_ptr(b);
  g.M = M;
  g.N = N;
  g.K = K;
  g.lda = K;
  g.ldb = K;
  g.ldc = N;
  g.epi = g.bias ? (relu ? sdml::EPI_BIAS_RELU : sdml::EPI_BIAS) : sdml::EPI_STORE;
  TORCH_CHECK(!relu || g.bias, "relu epilogue requires a bias in this kernel");
  TORCH_CHECK(sdml::gemm_f32_supported(g), "linear_fwd_f32: unsupported shape/alignment (K % 4 != 0?)");
  torch::Tensor wsplit;
  if (sdml::gemm_f32_uses_x3(g) && sdml::gemm_f32x3_can_presplit_b(g)) {
    // the weight is shared by every row block: split it into bf16 planes once per call
    wsplit = torch::empty({3, N, K}, x.options().dtype(torch::kInt16));
    sdml::split3_planes(w.data_ptr<float>(), reinterpret_cast<unsigned short*>(wsplit.data_ptr<int16_t>()), N * K,
                        cur_stream());
    g.b_split = reinterpret_cast<const unsigned short*>(wsplit.data_ptr<int16_t>());
  }
  sdml::gemm_f32(g, cur_stream());
  return y;
}

// backward of y = relu(x w^T + b) (relu_mask) or of y = x w^T + b:
//   gz = gy * (y > 0);  gw += gz^T x ; gb += colsum(gz) ; returns gz @ w if need_dx
c10::optional<torch::Tensor> linear_bwd_f32(torch::Tensor x, c10::optional<torch::Tensor> y, torch::Tensor gy,
                                            torch::Tensor w, c10::optional<torch::Tensor> gw,
                                            c10::optional<torch::Tensor> gb, bool need_dx, bool relu_mask,
                                            bool mask_dx_by_x) {
  check_f32_cuda(x, "x");
  check_f32_cuda(gy, "gy");
  check_f32_cuda(w, "w");
  const int64_t M = x.size(0), K = x.size(1), N = w.size(0);
  TORCH_CHECK(x.dim() == 2 && gy.dim() == 2 && gy.size(0) == M && gy.size(1) == N && w.size(1) == K,
              "linear_bwd_f32: shape mismatch");
  const float* mask = nullptr;
  if (relu_mask) {
    TORCH_CHECK(y.has_value() && y->defined(), "relu_mask needs y");
    check_f32_cuda(*y, "y");
    TORCH_CHECK(y->sizes() == gy.sizes(), "y/gy shape mismatch");
    mask = y->data_ptr<float>();
  }
  check_opt(gw, "gw", N * K);
  check_opt(gb, "gb", N);
  hipStream_t s = cur_stream();
  if (M > 0 && M <= sdml::DW_SMALLK_MAX_M && opt_ptr(gw)) {
    // small batch: one deterministic VALU pass (the MFMA GEMM would run K=M in a handful of
    // blocks and spend its time in the 128x128-tile epilogue)
    sdml::dw_smallk(gy.data_ptr<float>(), mask, x.data_ptr<float>(), opt_ptr(gw), opt_ptr(gb), (int)M, (int)N, (int)K,
                    s);
  } else if (M > 0 && (opt_ptr(gw) || opt_ptr(gb))) {
    // gw[N,K] += sum_m gz[m,n] x[m,k]: A(n,m) = gy[m*N + n] (k-major), B(k,m) = x[m*K + k] (k-major)
    sdml::GemmArgs g;
    g.A = gy.data_ptr<float>();
    g.amask = mask;
    g.B = x.data_ptr<float>();
    g.M = N;
    g.N = K;
    g.K = M;
    g.lda = N;
    g.ldb = K;
    g.ldc = K;
    g.a_kmajor = true;
    g.b_kmajor = true;
    g.epi = sdml::EPI_ATOMIC;
    g.rowsum = opt_ptr(gb);
    if (opt_ptr(gw)) {
      g.C = opt_ptr(gw);
      g.splits = sdml::gemm_f32_pick_splits(g.M, g.N, g.K);
    } else {
      // only the bias grad wanted: run with a 1-column dummy B? keep it simple: torch reduce
      g.C = nullptr;
    }
    if (g.C) {
      TORCH_CHECK(sdml::gemm_f32_supported(g), "linear_bwd_f32(dW): unsupported shape/alignment");
      sdml::gemm_f32(g, s);
    } else {
      auto gz = relu_mask ? gy * (y->gt(0)).to(gy.scalar_type()) : gy;
      gb->add_(gz.sum(0));
    }
  }
  if (!need_dx) return c10::nullopt;
  auto dx = torch::empty({M, K}, x.options());
  if (M == 0) return dx;
  // dx[M,K] = gz[M,N] @ w[N,K]: A(m,n) = gy[m*N+n] (contiguous), B(k,n) = w[n*K + k] (k-major)
  sdml::GemmArgs g;
  g.A = gy.data_ptr<float>();
  g.amask = mask;
  g.B = w.data_ptr<float>();
  g.C = dx.data_ptr<float>();
  g.M = M;
  g.N = K;
  g.K = N;
  g.lda = N;
  g.ldb = K;
  g.ldc = K;
  g.a_kmajor = false;
  g.b_kmajor = true;
  g.epi = sdml::EPI_STORE;
  if (mask_dx_by_x) g.cmask = x.data_ptr<float>();  // dx *= (x > 0): ReLU backward of the producer
  TORCH_CHECK(sdml::gemm_f32_supported(g), "linear_bwd_f32(dX): unsupported shape/alignment");
  // on the bf16x3 engine, take B = W^T pre-split (one transposed split of the weight per call)
  // like the forward instead of splitting the k-major weight tile in every workgroup
  sdml::GemmArgs gt = g;
  gt.b_kmajor = false;
  gt.ldb = N;
  torch::Tensor wsplit;
  if (sdml::gemm_f32_uses_x3(gt) && sdml::gemm_f32x3_can_presplit_b(gt)) {
    wsplit = torch::empty({3, K, N}, x.options().dtype(torch::kInt16));
    sdml::split3_planes_t(w.data_ptr<float>(), reinterpret_cast<unsigned short*>(wsplit.data_ptr<int16_t>()), (int)N,
                          (int)K, s);
    gt.b_split = reinterpret_cast<const unsigned short*>(wsplit.data_ptr<int16_t>());
    sdml::gemm_f32(gt, s);
    return dx;
  }
  sdml::gemm_f32(g, s);
  return dx;
}

// uint8 pixels -> float32 the way ToTensor() does it (k / 255 for scale = 1/255, a true division)
torch::Tensor pixels_f32(const torch::Tensor& x, double scale) {
  const double d = 1.0 / scale, r = std::round(d);
  auto xf = x.to(torch::kFloat32);
  return std::abs(d - r) < 1e-9 * r ? xf.div_(r) : xf.mul_(scale);
}

// first layer fed by uint8 pixels (MNIST's native bytes): y = act(scale * x_u8 @ w.T + b), with
// scale = 1/255 this is ToTensor() fused into the GEMM's operand load. Shapes the uint8 kernel
// does not take (small batches, unaligned K) go through an fp32 copy of x * scale.
// ReLU bits of y [M][N] (N % 32 == 0): int32 [M][N / 32], bit n % 32 of word n / 32 = (y[m][n] > 0) -
// the layout u8_fwd / u8_fwd_head write (for the paths that do not go through them)
torch::Tensor relu_bits(const torch::Tensor& y) {
  const int64_t M = y.size(0), N = y.size(1);
  TORCH_CHECK(N % 32 == 0, "relu_bits: N % 32 == 0");
  auto sh = torch::arange(32, y.options().dtype(torch::kInt64));
  auto b = (y > 0).view({M, N / 32, 32}).to(torch::kInt64);
  return b.bitwise_left_shift(sh).sum(-1).to(torch::kInt32);
}

// the inverse: float 0/1 [M][32 * words]
torch::Tensor relu_bits_unpack(const torch::Tensor& mask) {
  auto sh = torch::arange(32, mask.options().dtype(torch::kInt64));
  auto w = mask.to(torch::kInt64).bitwise_and(0xffffffffLL).unsqueeze(-1);
  return w.bitwise_right_shift(sh).bitwise_and(1).view({mask.size(0), mask.size(1) * 32}).to(torch::kFloat32);
}

void check_mask_out(const c10::optional<torch::Tensor>& m, int64_t M, int64_t N) {
  if (!m.has_value() || !m->defined()) return;
  TORCH_CHECK(m->is_cuda() && m->scalar_type() == torch::kInt32 && m->is_contiguous() && m->dim() == 2 &&
                  m->size(0) == M && N % 32 == 0 && m->size(1) == N / 32,
              "mask_out must be a contiguous int32 [M, N / 32] device tensor");
}

// mask_out (optional, relu): also write the ReLU bits of y (relu_bits' layout)
torch::Tensor linear_fwd_u8(torch::Tensor x, torch::Tensor w, c10::optional<torch::Tensor> b, bool relu,
                            double scale, c10::optional<torch::Tensor> planes, bool planes_valid,
                            c10::optional<torch::Tensor> mask_out, c10::optional<torch::Tensor> wmax_out) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == torch::kUInt8 && x.is_contiguous() && x.dim() == 2,
              "linear_fwd_u8: x must be a contiguous 2-D uint8 ROCm tensor");
  check_f32_cuda(w, "w");
  TORCH_CHECK(w.dim() == 2 && x.size(1) == w.size(1), "linear_fwd_u8: shape mismatch ", x.sizes(), " vs ", w.sizes());
  const int64_t M = x.size(0), K = x.size(1), N = w.size(0);
  check_opt(b, "b", N);
  TORCH_CHECK(!relu || opt_ptr(b), "relu epilogue requires a bias");
  check_mask_out(mask_out, M, N);
  const bool want_mask = mask_out.has_value() && mask_out->defined();
  TORCH_CHECK(!want_mask || relu, "linear_fwd_u8: mask_out needs the relu epilogue");
  const bool direct = M >= 4096 && K % 16 == 0 && (reinterpret_cast<uintptr_t>(x.data_ptr()) & 15) == 0 &&
                      M * K < (int64_t(1) << 31);
  auto with_mask = [&](torch::Tensor y) {  // (the paths without the uint8 kernel's epilogue extras)
    if (want_mask) mask_out->copy_(relu_bits(y));
    if (wmax_out.has_value() && wmax_out->defined())
      wmax_out->copy_(at::linalg_vector_norm(y, INFINITY).reshape({1}).expand_as(*wmax_out));
    return y;
  };
  // a caller-owned plane cache is marked current by the caller after this call (ops.linear_relu_fwd_u8), so
  // the paths that do not read it still refresh it when it is stale (a later fused forward+head reads it)
  auto refresh_cache = [&]() {
    if (!planes.has_value() || !planes->defined() || planes_valid) return;
    const int Kp = sdml::u8_fwd_kpad((int)K);
    TORCH_CHECK(planes->is_cuda() && planes->scalar_type() == torch::kInt16 && planes->is_contiguous() &&
                    planes->dim() == 3 && planes->size(0) == sdml::kU8FwdPlanes && planes->size(1) == N &&
                    planes->size(2) == Kp,
                "linear_fwd_u8: planes must be a [u8_fwd_planes()][N][u8_fwd_kpad(K)] int16 device tensor");
    sdml::split_planes_pad(w.data_ptr<float>(), reinterpret_cast<unsigned short*>(planes->data_ptr<int16_t>()),
                           (int)N, (int)K, Kp, cur_stream());
  };
  if (!direct) {
    refresh_cache();
    return with_mask(linear_fwd_f32(pixels_f32(x, scale), w, b, relu));
  }
  auto y = torch::empty({M, N}, w.options());
  const bool legacy = sdml::knob(sdml::KNOB_U8_FWD_X3) == 1;
  if (!legacy && sdml::u8_fwd_supported((int)M, (int)N, (int)K, (int)K, x.data_ptr())) {
    const int Kp = sdml::u8_fwd_kpad((int)K);
    // planes: a caller-owned cache [2][N][Kp] (fp16 bits of W * 2^8, zero padding columns; kept
    // current by the fused SGD step, ops/optim.py); planes_valid == false -> (re)split into it
    const bool cache = planes.has_value() && planes->defined();
    if (cache)
      TORCH_CHECK(planes->is_cuda() && planes->scalar_type() == torch::kInt16 && planes->is_contiguous() &&
                      planes->dim() == 3 && planes->size(0) == sdml::kU8FwdPlanes && planes->size(1) == N &&
                      planes->size(2) == Kp,
                  "linear_fwd_u8: planes must be a [u8_fwd_planes()][N][u8_fwd_kpad(K)] int16 device tensor");
    auto wp = cache ? *planes : torch::empty({sdml::kU8FwdPlanes, N, Kp}, w.options().dtype(torch::kInt16));
    auto* wpp = reinterpret_cast<unsigned short*>(wp.data_ptr<int16_t>());
    if (!cache || !planes_valid) sdml::split_planes_pad(w.data_ptr<float>(), wpp, (int)N, (int)K, Kp, cur_stream());
    float* wm = nullptr;
    if (wmax_out.has_value() && wmax_out->defined()) {  // per-wave output maxima (a split bound downstream)
      check_f32_cuda(*wmax_out, "wmax_out");
      TORCH_CHECK(wmax_out->is_contiguous() && wmax_out->numel() == sdml::u8_fwd_wmax_slots((int)M, (int)N),
                  "linear_fwd_u8: wmax_out must hold u8_fwd_wmax_slots(M, N) floats");
      wm = wmax_out->data_ptr<float>();
    }
    sdml::u8_fwd(x.data_ptr<uint8_t>(), (int)M, (int)K, (int)K, wpp, (int)N, Kp, opt_ptr(b), y.data_ptr<float>(),
                 (int)N, relu, (float)scale, cur_stream(),
                 want_mask ? reinterpret_cast<unsigned*>(mask_out->data_ptr<int32_t>()) : nullptr, wm);
    return y;
  }
  refresh_cache();
  auto wsplit = torch::empty({3, N, K}, w.options().dtype(torch::kInt16));
  sdml::split3_planes(w.data_ptr<float>(), reinterpret_cast<unsigned short*>(wsplit.data_ptr<int16_t>()), N * K,
                      cur_stream());
  sdml::gemm_u8x3_fwd(x.data_ptr<uint8_t>(), (int)M, (int)K, (int)K,
                      reinterpret_cast<const unsigned short*>(wsplit.data_ptr<int16_t>()), (int)N, opt_ptr(b),
                      y.data_ptr<float>(), (int)N, relu, (float)scale, cur_stream());
  return with_mask(y);
}

// weight/bias gradient of the uint8-fed first layer: gw += scale * gz^T x_u8, gb += colsum(gz)
// amax: optional float tensor with |gz| <= max(amax) (the fused head's per-block |dx| maxima); the
// uint8 kernel scales gz's fp16 planes from it (computed here with a torch amax when absent)
void linear_wgrad_u8(torch::Tensor x, torch::Tensor gz, torch::Tensor gw, c10::optional<torch::Tensor> gb,
                     double scale, c10::optional<torch::Tensor> amax) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == torch::kUInt8 && x.is_contiguous() && x.dim() == 2,
              "linear_wgrad_u8: x must be a contiguous 2-D uint8 ROCm tensor");
  check_f32_cuda(gz, "gz");
  check_f32_cuda(gw, "gw");
  const int64_t M = x.size(0), K = x.size(1), N = gz.size(1);
  TORCH_CHECK(gz.dim() == 2 && gz.size(0) == M && gw.size(0) == N && gw.size(1) == K, "linear_wgrad_u8: shape mismatch");
  check_opt(gb, "gb", N);
  const bool direct = M >= 4096 && K % 8 == 0 && N % 4 == 0 && (reinterpret_cast<uintptr_t>(x.data_ptr()) & 7) == 0 &&
                      M * K < (int64_t(1) << 31);
  if (!direct) {
    // fp32 path: linear_bwd_f32 only reads w's shape when no input gradient is asked for
    linear_bwd_f32(pixels_f32(x, scale), c10::nullopt, gz, /*w=*/gw, gw, gb, false, false, false);
    return;
  }
  const bool legacy_wgrad = sdml::knob(sdml::KNOB_U8_WGRAD_X3) == 1;
  // mlp_u8.hip's kernel writes gw and gb through one [N * K + N] span: gb must follow gw
  const bool gb_follows = opt_ptr(gb) && gw.is_contiguous() && gb->is_contiguous() &&
                          opt_ptr(gb) == gw.data_ptr<float>() + N * K;
  if (!legacy_wgrad && gb_follows && sdml::u8_wgrad_supported((int)M, (int)N, (int)K, (int)K, x.data_ptr(),
                                                               gz.data_ptr())) {
    auto ws = torch::empty({sdml::u8_wgrad_slab_floats((int)M, (int)N)}, gw.options());
    // (no bound given: one reduction pass over gz, its inf-norm; abs().amax() would also write |gz|)
    torch::Tensor am =
        amax.has_value() && amax->defined() ? *amax : at::linalg_vector_norm(gz, INFINITY).reshape({1});
    check_f32_cuda(am, "amax");
    TORCH_CHECK(am.numel() >= 1 && am.is_contiguous(), "linear_wgrad_u8: amax must be a non-empty contiguous tensor");
    sdml::u8_wgrad(gz.data_ptr<float>(), x.data_ptr<uint8_t>(), (int)M, (int)N, (int)K, ws.data_ptr<float>(),
                   gw.data_ptr<float>(), (float)scale, am.data_ptr<float>(), (int)am.numel(), cur_stream());
    return;
  }
  float* slab = nullptr;
  torch::Tensor ws;
  if ((N * K) % 4 == 0 && (reinterpret_cast<uintptr_t>(gw.data_ptr()) & 15) == 0 && gw.is_contiguous()) {
    ws = torch::empty({(int64_t)sdml::u8x3_wgrad_splits((int)M, (int)N, (int)K), N, K}, gw.options());
    slab = ws.data_ptr<float>();
  }
  sdml::gemm_u8x3_wgrad(gz.data_ptr<float>(), x.data_ptr<uint8_t>(), (int)M, (int)N, (int)K, (int)K,
                        gw.data_ptr<float>(), opt_ptr(gb), (float)scale, slab, cur_stream());
}


// generic GEMM entry (tests/benchmarks): C = A(m,k) B(n,k) with layout flags
void gemm_f32_op(torch::Tensor A, torch::Tensor B, torch::Tensor C, bool a_kmajor, bool b_kmajor, int64_t epi,
                 int64_t splits, c10::optional<torch::Tensor> bias, c10::optional<torch::Tensor> rowsum) {
  check_f32_cuda(A, "A");
  check_f32_cuda(B, "B");
  check_f32_cuda(C, "C");
  TORCH_CHECK(A.dim() == 2 && B.dim() == 2 && C.dim() == 2, "2-D operands");
  const int64_t M = C.size(0), N = C.size(1);
  const int64_t K = a_kmajor ? A.size(0) : A.size(1);
  TORCH_CHECK((a_kmajor ? A.size(1) : A.size(0)) == M, "A rows != M");
  TORCH_CHECK((b_kmajor ? B.size(0) : B.size(1)) == K, "B k-extent != K");
  TORCH_CHECK((b_kmajor ? B.size(1) : B.size(0)) == N, "B rows != N");
  check_opt(bias, "bias", N);
  check_opt(rowsum, "rowsum", M);
  sdml::GemmArgs g;
  g.A = A.data_ptr<float>();
  g.B = B.data_ptr<float>();
  g.C = C.data_ptr<float>();
  g.bias = opt_ptr(bias);
  g.rowsum = opt_ptr(rowsum);
  g.M = M;
  g.N = N;
  g.K = K;
  g.lda = A.size(1);
  g.ldb = B.size(1);
  g.ldc = N;
  g.a_kmajor = a_kmajor;
  g.b_kmajor = b_kmajor;
  g.epi = (int)epi;
  g.splits = (int)splits;
  TORCH_CHECK(epi >= 0 && epi <= 4, "bad epilogue");
  TORCH_CHECK(!(epi == 1 || epi == 2) || g.bias, "bias epilogue needs bias");
  TORCH_CHECK(sdml::gemm_f32_supported(g), "gemm_f32: unsupported shape/alignment");
  sdml::gemm_f32(g, cur_stream());
}

// the bf16x3-split engine called directly (tests, any size): same contract as gemm_f32_op
void gemm_f32x3_op(torch::Tensor A, torch::Tensor B, torch::Tensor C, bool a_kmajor, bool b_kmajor, int64_t epi,
                   c10::optional<torch::Tensor> bias, c10::optional<torch::Tensor> rowsum,
                   c10::optional<torch::Tensor> amask, c10::optional<torch::Tensor> cmask) {
  check_f32_cuda(A, "A");
  check_f32_cuda(B, "B");
  check_f32_cuda(C, "C");
  TORCH_CHECK(A.dim() == 2 && B.dim() == 2 && C.dim() == 2, "2-D operands");
  const int64_t M = C.size(0), N = C.size(1);
  const int64_t K = a_kmajor ? A.size(0) : A.size(1);
  TORCH_CHECK((a_kmajor ? A.size(1) : A.size(0)) == M, "A rows != M");
  TORCH_CHECK((b_kmajor ? B.size(0) : B.size(1)) == K, "B k-extent != K");
  TORCH_CHECK((b_kmajor ? B.size(1) : B.size(0)) == N, "B rows != N");
  check_opt(bias, "bias", N);
  check_opt(rowsum, "rowsum", M);
  check_opt(amask, "amask", A.numel());
  check_opt(cmask, "cmask", C.numel());
  TORCH_CHECK(epi >= 0 && epi <= 4, "bad epilogue");
  sdml::GemmArgs g;
  g.A = A.data_ptr<float>();
  g.B = B.data_ptr<float>();
  g.C = C.data_ptr<float>();
  g.bias = opt_ptr(bias);
  g.rowsum = opt_ptr(rowsum);
  g.amask = opt_ptr(amask);
  g.cmask = opt_ptr(cmask);
  g.M = M;
  g.N = N;
  g.K = K;
  g.lda = A.size(1);
  g.ldb = B.size(1);
  g.ldc = N;
  g.a_kmajor = a_kmajor;
  g.b_kmajor = b_kmajor;
  g.epi = (int)epi;
  TORCH_CHECK(!(epi == 1 || epi == 2) || g.bias, "bias epilogue needs bias");
  TORCH_CHECK(sdml::gemm_f32x3_eligible(g), "gemm_f32x3: unsupported shape/alignment");
  sdml::gemm_f32x3(g, cur_stream());
}

// gw (bf16 [M, N], in place) += gy[T, M]^T @ x[T, N] (bf16), hand-written MFMA split-token GEMM
void wgrad_bf16_(torch::Tensor gy, torch::Tensor x, torch::Tensor gw, c10::optional<torch::Tensor> gb) {
  for (auto* t : {&gy, &x, &gw}) {
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == torch::kBFloat16, "wgrad_bf16_: bf16 ROCm tensors expected");
    TORCH_CHECK(t->dim() == 2 && t->stride(1) == 1, "wgrad_bf16_: 2-D row-major operands expected");
  }
  const int64_t T = gy.size(0), M = gy.size(1), N = x.size(1);
  TORCH_CHECK(x.size(0) == T && gw.size(0) == M && gw.size(1) == N, "wgrad_bf16_: shape mismatch");
  TORCH_CHECK(sdml::wgrad_bf16_supported(M, N, T, gy.stride(0), x.stride(0), gw.stride(0)),
              "wgrad_bf16_: unsupported shape/alignment");
  void* gbp = nullptr;
  if (gb.has_value() && gb->defined()) {
    TORCH_CHECK(gb->is_cuda() && gb->scalar_type() == torch::kBFloat16 && gb->is_contiguous() && gb->numel() == M,
                "wgrad_bf16_: gb must be a contiguous bf16 [M] tensor");
    gbp = gb->data_ptr();
  }
  if (T == 0) return;
  const size_t ws = sdml::wgrad_bf16_workspace_floats(M, N, T);
  torch::Tensor w;
  if (ws) w = torch::empty({(int64_t)ws}, gy.options().dtype(torch::kFloat32));
  sdml::wgrad_bf16(gy.data_ptr(), x.data_ptr(), gw.data_ptr(), gbp, ws ? w.data_ptr<float>() : nullptr, M, N, T,
                   gy.stride(0), x.stride(0), gw.stride(0), cur_stream());
}

// ---- fp32-accurate GEMMs from pre-split fp16 planes (gemm_f16x2.hip) ----
// x [R, C] fp32 (unit column stride) -> (planes int16 [2, R, C], scale fp32 [1] = 2^(E - 14)); amax: any fp32
// device tensor whose max |.| bounds |x| (an inf-norm, a producer's per-wave maxima, the head's bounds)
std::tuple<torch::Tensor, torch::Tensor> x2_split_op(torch::Tensor x, torch::Tensor amax) {
  check_f32_cuda(x, "x");
  check_f32_cuda(amax, "amax");
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1 && x.size(1) % 8 == 0 && x.stride(0) % 4 == 0 &&
                  x.numel() < (int64_t(1) << 34),
              "x2_split: 2-D row-major fp32 with a multiple of 8 columns (and < 2^34 elements) expected");
  TORCH_CHECK(amax.is_contiguous() && amax.numel() >= 1, "x2_split: amax must be a non-empty contiguous tensor");
  const int64_t R = x.size(0), C = x.size(1);
  auto planes = torch::empty({2, R, C}, x.options().dtype(torch::kInt16));
  auto scale = torch::empty({1}, x.options());
  if (R > 0)
    sdml::x2_split(x.data_ptr<float>(), (int)R, (int)C, (int)x.stride(0), amax.data_ptr<float>(), (int)amax.numel(),
                   planes.data_ptr(), R * C, (int)C, scale.data_ptr<float>(), cur_stream());
  return {planes, scale};
}

// planes of x^T: (planes int16 [2, C, R], scale)
std::tuple<torch::Tensor, torch::Tensor> x2_split_t_op(torch::Tensor x, torch::Tensor amax) {
  check_f32_cuda(x, "x");
  check_f32_cuda(amax, "amax");
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1, "x2_split_t: 2-D row-major fp32 expected");
  TORCH_CHECK(amax.is_contiguous() && amax.numel() >= 1, "x2_split_t: amax must be a non-empty contiguous tensor");
  const int64_t R = x.size(0), C = x.size(1);
  auto planes = torch::empty({2, C, R}, x.options().dtype(torch::kInt16));
  auto scale = torch::empty({1}, x.options());
  if (R > 0 && C > 0)
    sdml::x2_split_t(x.data_ptr<float>(), (int)R, (int)C, (int)x.stride(0), amax.data_ptr<float>(),
                     (int)amax.numel(), planes.data_ptr(), R * C, (int)R, scale.data_ptr<float>(), cur_stream());
  return {planes, scale};
}

static void check_planes(const torch::Tensor& p, const char* name) {
  TORCH_CHECK(p.is_cuda() && p.scalar_type() == torch::kInt16 && p.dim() == 3 && p.size(0) == 2 && p.is_contiguous(),
              name, ": planes must be a contiguous int16 [2, rows, cols] device tensor (x2_split)");
}

// C = sa sb A' . (b_kn ? B' : B'^T) (+ bias) (relu) (* (mask > 0)); A planes [2, M, K], B planes [2, N, K] or
// [2, K, N]. Returns (C fp32 [M, N], per-wave max |C| or None)
std::tuple<torch::Tensor, c10::optional<torch::Tensor>> x2_gemm_op(torch::Tensor A, torch::Tensor sa, torch::Tensor B,
                                                                   torch::Tensor sb, bool b_kn,
                                                                   c10::optional<torch::Tensor> bias, bool relu,
                                                                   c10::optional<torch::Tensor> mask, bool want_wmax) {
  check_planes(A, "x2_gemm A");
  check_planes(B, "x2_gemm B");
  check_f32_cuda(sa, "sa");
  check_f32_cuda(sb, "sb");
  const int64_t M = A.size(1), K = A.size(2), N = b_kn ? B.size(2) : B.size(1);
  TORCH_CHECK((b_kn ? B.size(1) : B.size(2)) == K, "x2_gemm: inner dimensions ", A.sizes(), " vs ", B.sizes());
  TORCH_CHECK(sdml::x2_gemm_supported((int)M, (int)N, (int)K, (int)K, (int)B.size(2), (int)N, b_kn),
              "x2_gemm: unsupported shape (x2_gemm_supported)");
  auto C = torch::empty({M, N}, A.options().dtype(torch::kFloat32));
  const float* bp = nullptr;
  if (bias.has_value() && bias->defined()) {
    check_f32_cuda(*bias, "bias");
    TORCH_CHECK(bias->is_contiguous() && bias->numel() == N, "x2_gemm: bias shape");
    bp = bias->data_ptr<float>();
  }
  const float* mp = nullptr;
  int64_t ldm = 0;
  if (mask.has_value() && mask->defined()) {
    check_f32_cuda(*mask, "mask");
    TORCH_CHECK(mask->dim() == 2 && mask->size(0) == M && mask->size(1) == N && mask->stride(1) == 1 &&
                    mask->stride(0) % 4 == 0,
                "x2_gemm: mask must be a row-major fp32 [M, N] tensor");
    mp = mask->data_ptr<float>();
    ldm = mask->stride(0);
  }
  c10::optional<torch::Tensor> wm;
  if (want_wmax) wm = torch::empty({(int64_t)sdml::x2_gemm_wmax_slots((int)M, (int)N)}, C.options());
  if (M > 0)
    sdml::x2_gemm(A.data_ptr(), M * K, B.data_ptr(), B.size(1) * B.size(2), C.data_ptr<float>(), (int)M, (int)N,
                  (int)K, (int)K, (int)B.size(2), (int)N, b_kn, sa.data_ptr<float>(), sb.data_ptr<float>(), bp, relu, mp,
                  (int)ldm, want_wmax ? wm->data_ptr<float>() : nullptr, cur_stream());
  return {C, wm};
}

bool x2_gemm_supported_op(int64_t M, int64_t N, int64_t K, bool b_kn) {
  return sdml::x2_gemm_supported((int)M, (int)N, (int)K, (int)K, (int)(b_kn ? N : K), (int)N, b_kn);
}

// gw [M, N] (fp32) += sdz sx dz'^T x'; gb [M] += sdz colsum(dz'). dz planes [2, T, M], x planes [2, T, N]
void x2_wgrad_(torch::Tensor dz, torch::Tensor sdz, torch::Tensor x, torch::Tensor sx, torch::Tensor gw,
               c10::optional<torch::Tensor> gb) {
  check_planes(dz, "x2_wgrad dz");
  check_planes(x, "x2_wgrad x");
  check_f32_cuda(sdz, "sdz");
  check_f32_cuda(sx, "sx");
  check_f32_cuda(gw, "gw");
  const int64_t T = dz.size(1), M = dz.size(2), N = x.size(2);
  TORCH_CHECK(x.size(1) == T && gw.dim() == 2 && gw.size(0) == M && gw.size(1) == N && gw.stride(1) == 1 &&
                  gw.stride(0) % 4 == 0 && N % 4 == 0,
              "x2_wgrad_: shape mismatch");
  TORCH_CHECK(sdml::x2_wgrad_supported((int)M, (int)N, (int)T, (int)M, (int)N), "x2_wgrad_: unsupported shape");
  float* gbp = nullptr;
  if (gb.has_value() && gb->defined()) {
    check_f32_cuda(*gb, "gb");
    TORCH_CHECK(gb->is_contiguous() && gb->numel() == M, "x2_wgrad_: gb must be a contiguous fp32 [M] tensor");
    gbp = gb->data_ptr<float>();
  }
  if (T == 0) return;
  auto ws = torch::empty({(int64_t)sdml::x2_wgrad_workspace_floats((int)M, (int)N, (int)T)}, gw.options());
  sdml::x2_wgrad(dz.data_ptr(), T * M, x.data_ptr(), T * N, sdz.data_ptr<float>(), sx.data_ptr<float>(),
                 gw.data_ptr<float>(), (int)gw.stride(0), gbp, ws.data_ptr<float>(), (int)M, (int)N, (int)T, (int)M,
                 (int)N, cur_stream());
}

bool wgrad_bf16_supported_op(int64_t M, int64_t N, int64_t T) {
  return sdml::wgrad_bf16_supported(M, N, T, M, N, N);
}

// ---- 3x3 / stride 1 / pad 1 convolutions on channels-last bf16 tensors ----
static void check_cl_bf16(const torch::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == torch::kBFloat16 && t.dim() == 4, name,
              ": 4-D bf16 ROCm tensor expected");
  TORCH_CHECK(t.is_contiguous(at::MemoryFormat::ChannelsLast), name, ": channels-last (NHWC) memory expected");
}

// weight [Co][C][3][3] -> [Co][9][C] (dgrad = false) or [C][9][Co] flipped (dgrad = true)
static void check_conv_w(const torch::Tensor& w) {
  TORCH_CHECK(w.is_cuda() && w.scalar_type() == torch::kBFloat16 && w.dim() == 4 && w.size(2) == 3 &&
              w.size(3) == 3 && w.is_contiguous(), "conv3x3 weight: contiguous [Co][C][3][3] bf16");
}

torch::Tensor conv3x3_weight_bf16(torch::Tensor w, bool dgrad) {
  check_conv_w(w);
  const int64_t Co = w.size(0), C = w.size(1);
  auto out = dgrad ? torch::empty({C, 9, Co}, w.options()) : torch::empty({Co, 9, C}, w.options());
  sdml::conv3x3_weight_transform_bf16(w.data_ptr(), dgrad ? nullptr : out.data_ptr(), dgrad ? out.data_ptr() : nullptr,
                                      Co, C, cur_stream());
  return out;
}

// both kernel layouts of one weight in one pass: (forward [Co][9][C], dgrad [C][9][Co])
std::tuple<torch::Tensor, torch::Tensor> conv3x3_weights_bf16(torch::Tensor w) {
  check_conv_w(w);
  const int64_t Co = w.size(0), C = w.size(1);
  auto f = torch::empty({Co, 9, C}, w.options());
  auto d = torch::empty({C, 9, Co}, w.options());
  sdml::conv3x3_weight_transform_bf16(w.data_ptr(), f.data_ptr(), d.data_ptr(), Co, C, cur_stream());
  return {f, d};
}

// the kernel layouts of several 3x3 weights in one launch, into caller-owned buffers (ops/conv.py keeps one pair per
// weight across optimizer steps): fwd[k] [Co][9][C], dgrad[k] [C][9][Co] or None (forward layout only)
void transpose_batched_bf16(std::vector<torch::Tensor> src, std::vector<torch::Tensor> dst) {
  TORCH_CHECK(src.size() == dst.size(), "transpose_batched_bf16: list lengths");
  const void* sp[sdml::kTransposeBatchMax];
  void* dp[sdml::kTransposeBatchMax];
  int R[sdml::kTransposeBatchMax], C[sdml::kTransposeBatchMax];
  for (size_t b0 = 0; b0 < src.size(); b0 += sdml::kTransposeBatchMax) {
    const int n = (int)std::min<size_t>(sdml::kTransposeBatchMax, src.size() - b0);
    for (int k = 0; k < n; ++k) {
      const torch::Tensor& s = src[b0 + k];
      const torch::Tensor& d = dst[b0 + k];
      TORCH_CHECK(s.is_cuda() && s.scalar_type() == torch::kBFloat16 && s.is_contiguous() && s.dim() == 2,
                  "transpose_batched_bf16: src must be a contiguous 2-D bf16 CUDA tensor");
      TORCH_CHECK(d.is_cuda() && d.scalar_type() == torch::kBFloat16 && d.is_contiguous() && d.dim() == 2 &&
                      d.size(0) == s.size(1) && d.size(1) == s.size(0) && d.device() == s.device(),
                  "transpose_batched_bf16: dst must be a contiguous [C][R] bf16 tensor on the same device");
      TORCH_CHECK(s.size(0) % 8 == 0 && s.size(1) % 8 == 0 && s.size(0) < (1 << 30) && s.size(1) < (1 << 30),
                  "transpose_batched_bf16: R and C must be multiples of 8");
      sp[k] = s.data_ptr();
      dp[k] = d.data_ptr();
      R[k] = (int)s.size(0);
      C[k] = (int)s.size(1);
    }
    sdml::transpose_batched_bf16(sp, dp, R, C, n, cur_stream());
  }
}

void conv3x3_weights_batched_bf16(std::vector<torch::Tensor> ws, std::vector<torch::Tensor> fwd,
                                  std::vector<c10::optional<torch::Tensor>> dgrad) {
  TORCH_CHECK(ws.size() == fwd.size() && ws.size() == dgrad.size(), "conv3x3_weights_batched_bf16: list lengths");
  const void* wp[sdml::kWtBatchMax];
  void* fp[sdml::kWtBatchMax];
  void* dp[sdml::kWtBatchMax];
  int co[sdml::kWtBatchMax], ci[sdml::kWtBatchMax];
  for (size_t b0 = 0; b0 < ws.size(); b0 += sdml::kWtBatchMax) {
    const int n = (int)std::min<size_t>(sdml::kWtBatchMax, ws.size() - b0);
    for (int k = 0; k < n; ++k) {
      const torch::Tensor& w = ws[b0 + k];
      check_conv_w(w);
      const int64_t Co = w.size(0), C = w.size(1);
      const torch::Tensor& f = fwd[b0 + k];
      TORCH_CHECK(f.is_cuda() && f.scalar_type() == torch::kBFloat16 && f.is_contiguous() && f.numel() == Co * 9 * C,
                  "conv3x3_weights_batched_bf16: forward layout buffer");
      wp[k] = w.data_ptr();
      fp[k] = f.data_ptr();
      dp[k] = nullptr;
      if (dgrad[b0 + k].has_value() && dgrad[b0 + k]->defined()) {
        const torch::Tensor& d = *dgrad[b0 + k];
        TORCH_CHECK(d.is_cuda() && d.scalar_type() == torch::kBFloat16 && d.is_contiguous() && d.numel() == Co * 9 * C,
                    "conv3x3_weights_batched_bf16: dgrad layout buffer");
        dp[k] = d.data_ptr();
      }
      co[k] = (int)Co;
      ci[k] = (int)C;
    }
    sdml::conv3x3_weight_transform_batched_bf16(wp, fp, dp, co, ci, n, cur_stream());
  }
}

// y (channels-last [N][Co][H][W]) = conv3x3(x, w) with wt from conv3x3_weight_bf16(w, dgrad=false)
// the optional epilogue operands of the implicit-GEMM convolutions: an addend in the output's layout
// and the BatchNorm partials [conv_part_rows][2][Co] fp32 of the output
static const void* conv_addend(const c10::optional<torch::Tensor>& add, const torch::Tensor& y, const char* fn) {
  if (!add.has_value() || !add->defined()) return nullptr;
  check_cl_bf16(*add, "add");
  TORCH_CHECK(add->sizes() == y.sizes(), fn, ": addend shape mismatch");
  return add->data_ptr();
}
static float* conv_part(const c10::optional<torch::Tensor>& part, int64_t N, int64_t OH, int64_t OW, int64_t Co,
                        const char* fn) {
  if (!part.has_value() || !part->defined()) return nullptr;
  TORCH_CHECK(part->is_cuda() && part->is_contiguous() && part->scalar_type() == torch::kFloat32 &&
                  part->numel() == (int64_t)sdml::conv_part_rows(N, OH, OW) * 2 * Co,
              fn, ": part must be a contiguous fp32 [conv_part_rows][2][Co] tensor");
  return part->data_ptr<float>();
}

int64_t conv_part_rows(int64_t N, int64_t OH, int64_t OW) { return sdml::conv_part_rows(N, OH, OW); }
int64_t conv_dgrad_s2_part_rows(int64_t N, int64_t H, int64_t W, int64_t ks, int64_t pad) {
  return sdml::conv_dgrad_s2_part_rows(N, H, W, ks, pad);
}

static void check_bn_vec(const c10::optional<torch::Tensor>& t, int64_t C, const char* name);

// the BatchNorm whose input gradient a convolution's output is (sdml::ConvBnBack): x (and y for relu 1) in the
// output's layout, fp32 [C] mean / rstd, bf16 [C] gamma / beta; relu 0 / 1 / 2
static sdml::ConvBnBack conv_bn_back(const c10::optional<torch::Tensor>& bx, const c10::optional<torch::Tensor>& by,
                                     const c10::optional<torch::Tensor>& mean, const c10::optional<torch::Tensor>& rstd,
                                     const c10::optional<torch::Tensor>& gamma, const c10::optional<torch::Tensor>& beta,
                                     int64_t relu, const torch::Tensor& out, bool have_part, const char* fn) {
  sdml::ConvBnBack b;
  if (!bx.has_value() || !bx->defined()) return b;
  TORCH_CHECK(have_part, fn, ": bn_x needs part");
  check_cl_bf16(*bx, "bn_x");
  TORCH_CHECK(bx->sizes() == out.sizes(), fn, ": bn_x must have the output's shape");
  const int64_t C = out.size(1);
  TORCH_CHECK(relu >= 0 && relu <= 2, fn, ": bn_relu must be 0, 1 or 2");
  if (relu == 1) {
    TORCH_CHECK(by.has_value() && by->defined(), fn, ": bn_relu 1 needs bn_y");
    check_cl_bf16(*by, "bn_y");
    TORCH_CHECK(by->sizes() == out.sizes(), fn, ": bn_y must have the output's shape");
    b.y = by->data_ptr();
  }
  for (const auto* t : {&mean, &rstd})
    TORCH_CHECK(t->has_value() && (*t)->defined() && (*t)->is_cuda() && (*t)->scalar_type() == torch::kFloat32 &&
                    (*t)->is_contiguous() && (*t)->numel() == C, fn, ": bn_mean / bn_rstd must be fp32 [C]");
  TORCH_CHECK(gamma.has_value() && gamma->defined() && beta.has_value() && beta->defined(), fn,
              ": bn_gamma and bn_beta are needed");
  check_bn_vec(gamma, C, "bn_gamma");
  check_bn_vec(beta, C, "bn_beta");
  b.x = bx->data_ptr();
  b.mean = mean->data_ptr<float>();
  b.rstd = rstd->data_ptr<float>();
  b.gamma = gamma->data_ptr();
  b.beta = beta->data_ptr();
  b.relu = (int)relu;
  return b;
}

torch::Tensor conv3x3_fwd_bf16(torch::Tensor x, torch::Tensor wt, c10::optional<torch::Tensor> add,
                               c10::optional<torch::Tensor> part, c10::optional<torch::Tensor> bn_x,
                               c10::optional<torch::Tensor> bn_y, c10::optional<torch::Tensor> bn_mean,
                               c10::optional<torch::Tensor> bn_rstd, c10::optional<torch::Tensor> bn_gamma,
                               c10::optional<torch::Tensor> bn_beta, int64_t bn_relu) {
  check_cl_bf16(x, "x");
  TORCH_CHECK(wt.dim() == 3 && wt.size(1) == 9 && wt.size(2) == x.size(1) && wt.is_contiguous() &&
              wt.scalar_type() == torch::kBFloat16, "conv3x3_fwd_bf16: wt must be [Co][9][C] bf16");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3), Co = wt.size(0);
  TORCH_CHECK(sdml::conv3x3_bf16_supported(C, Co), "conv3x3_fwd_bf16: channels must be multiples of 64");
  auto y = torch::empty({N, Co, H, W}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  const void* ap = conv_addend(add, y, "conv3x3_fwd_bf16");
  float* pp = conv_part(part, N, H, W, Co, "conv3x3_fwd_bf16");
  const sdml::ConvBnBack bb = conv_bn_back(bn_x, bn_y, bn_mean, bn_rstd, bn_gamma, bn_beta, bn_relu, y, pp != nullptr,
                                           "conv3x3_fwd_bf16");
  if (N * H * W > 0)
    sdml::conv3x3_fwd_bf16(x.data_ptr(), wt.data_ptr(), y.data_ptr(), N, H, W, C, Co, cur_stream(), ap, pp, &bb);
  return y;
}

// gw ([Co][C][3][3] bf16, in place) += dW of y = conv3x3(x, w) for output gradient dy
void conv3x3_wgrad_bf16_(torch::Tensor dy, torch::Tensor x, torch::Tensor gw) {
  check_cl_bf16(dy, "dy");
  check_cl_bf16(x, "x");
  TORCH_CHECK(gw.is_contiguous() && gw.scalar_type() == torch::kBFloat16 && gw.dim() == 4 &&
              gw.size(0) == dy.size(1) && gw.size(1) == x.size(1), "conv3x3_wgrad_bf16_: gw [Co][C][3][3] bf16");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3), Co = dy.size(1);
  TORCH_CHECK(dy.size(0) == N && dy.size(2) == H && dy.size(3) == W, "conv3x3_wgrad_bf16_: shape mismatch");
  TORCH_CHECK(sdml::conv3x3_bf16_supported(C, Co), "conv3x3_wgrad_bf16_: channels must be multiples of 64");
  if (N * H * W == 0) return;
  auto ws = torch::empty({(int64_t)sdml::conv3x3_wgrad_workspace_floats(N, H, W, C, Co)},
                         x.options().dtype(torch::kFloat32).memory_format(at::MemoryFormat::Contiguous));
  sdml::conv3x3_wgrad_bf16(dy.data_ptr(), x.data_ptr(), gw.data_ptr(), ws.data_ptr<float>(), N, H, W, C, Co,
                           cur_stream());
}

// ---- BatchNorm (+ residual) (+ ReLU) on channels-last bf16 activations ----
static void* opt_data(const c10::optional<torch::Tensor>& t) {
  return (t.has_value() && t->defined()) ? t->data_ptr() : nullptr;
}
static void check_bn_vec(const c10::optional<torch::Tensor>& t, int64_t C, const char* name) {
  if (t.has_value() && t->defined())
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == torch::kBFloat16 && t->is_contiguous() && t->numel() == C, name,
                ": contiguous bf16 [C] expected");
}

// general convolution (kernel 3 pad 1 / kernel 1 pad 0, stride 1 or 2), channels-last bf16; wt from
// conv3x3_weight_bf16(w, false) for 3x3 or the [Co][C][1][1] weight itself for 1x1
torch::Tensor conv_fwd_bf16(torch::Tensor x, torch::Tensor wt, int64_t ks, int64_t stride, int64_t pad,
                            c10::optional<torch::Tensor> add, c10::optional<torch::Tensor> part) {
  check_cl_bf16(x, "x");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3), Co = wt.size(0);
  TORCH_CHECK(wt.is_contiguous() && wt.scalar_type() == torch::kBFloat16 && wt.numel() == Co * ks * ks * C,
              "conv_fwd_bf16: wt must be a contiguous [Co][ks*ks][C] bf16 tensor");
  TORCH_CHECK(sdml::conv_general_supported(C, Co, ks, stride, pad), "conv_fwd_bf16: unsupported geometry");
  const int64_t OH = sdml::conv_out_size(H, ks, stride, pad), OW = sdml::conv_out_size(W, ks, stride, pad);
  auto y = torch::empty({N, Co, OH, OW}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  const void* ap = conv_addend(add, y, "conv_fwd_bf16");
  float* pp = conv_part(part, N, OH, OW, Co, "conv_fwd_bf16");
  if (N * OH * OW > 0)
    sdml::conv_fwd_bf16(x.data_ptr(), wt.data_ptr(), y.data_ptr(), N, H, W, C, Co, ks, stride, pad, cur_stream(), ap,
                        pp);
  return y;
}

// input gradient of a stride-2 convolution (3x3 pad 1 / 1x1 pad 0): dx (channels-last [N][C][H][W]) from
// dy (channels-last [N][Co][OH][OW]) and the torch weight [Co][C][ks][ks]
torch::Tensor conv_dgrad_s2_bf16(torch::Tensor dy, torch::Tensor w, int64_t H, int64_t W, int64_t pad,
                                 c10::optional<torch::Tensor> add, c10::optional<torch::Tensor> part,
                                 c10::optional<torch::Tensor> bn_x, c10::optional<torch::Tensor> bn_y,
                                 c10::optional<torch::Tensor> bn_mean, c10::optional<torch::Tensor> bn_rstd,
                                 c10::optional<torch::Tensor> bn_gamma, c10::optional<torch::Tensor> bn_beta,
                                 int64_t bn_relu) {
  check_cl_bf16(dy, "dy");
  TORCH_CHECK(w.is_cuda() && w.is_contiguous() && w.scalar_type() == torch::kBFloat16 && w.dim() == 4 &&
              w.size(2) == w.size(3) && w.size(0) == dy.size(1), "conv_dgrad_s2_bf16: w must be [Co][C][k][k] bf16");
  const int64_t N = dy.size(0), Co = dy.size(1), C = w.size(1), ks = w.size(2);
  TORCH_CHECK(sdml::conv_general_supported(C, Co, ks, 2, pad), "conv_dgrad_s2_bf16: unsupported geometry");
  TORCH_CHECK(dy.size(2) == sdml::conv_out_size(H, ks, 2, pad) && dy.size(3) == sdml::conv_out_size(W, ks, 2, pad),
              "conv_dgrad_s2_bf16: dy does not match the input size");
  auto dx = torch::empty({N, C, H, W}, dy.options().memory_format(at::MemoryFormat::ChannelsLast));
  if (dx.numel() == 0) return dx;
  conv_addend(add, dx, "conv_dgrad_s2_bf16");
  auto packed = torch::empty({(int64_t)sdml::conv_dgrad_s2_weight_elems(Co, C, ks)}, w.options());
  sdml::conv_dgrad_s2_weight_bf16(w.data_ptr(), packed.data_ptr(), Co, C, ks, pad, cur_stream());
  float* pp = nullptr;
  if (part.has_value() && part->defined()) {
    TORCH_CHECK(part->is_cuda() && part->is_contiguous() && part->scalar_type() == torch::kFloat32 &&
                    part->numel() == (int64_t)sdml::conv_dgrad_s2_part_rows(N, H, W, ks, pad) * 2 * C,
                "conv_dgrad_s2_bf16: part must be a contiguous fp32 [conv_dgrad_s2_part_rows][2][C] tensor");
    pp = part->data_ptr<float>();
  }
  const sdml::ConvBnBack bb = conv_bn_back(bn_x, bn_y, bn_mean, bn_rstd, bn_gamma, bn_beta, bn_relu, dx, pp != nullptr,
                                           "conv_dgrad_s2_bf16");
  TORCH_CHECK(!pp || bb.x, "conv_dgrad_s2_bf16: part is only written for bn_x (the backward statistics)");
  sdml::conv_dgrad_s2_bf16(dy.data_ptr(), packed.data_ptr(), dx.data_ptr(), N, H, W, C, Co, ks, pad, cur_stream(),
                           conv_addend(add, dx, "conv_dgrad_s2_bf16"), pp, &bb);
  return dx;
}

void conv_wgrad_bf16_(torch::Tensor dy, torch::Tensor x, torch::Tensor gw, int64_t stride, int64_t pad) {
  check_cl_bf16(dy, "dy");
  check_cl_bf16(x, "x");
  TORCH_CHECK(gw.is_contiguous() && gw.scalar_type() == torch::kBFloat16 && gw.dim() == 4 && gw.size(2) == gw.size(3) &&
              gw.size(0) == dy.size(1) && gw.size(1) == x.size(1), "conv_wgrad_bf16_: gw [Co][C][k][k] bf16");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3), Co = dy.size(1), ks = gw.size(2);
  TORCH_CHECK(sdml::conv_general_supported(C, Co, ks, stride, pad), "conv_wgrad_bf16_: unsupported geometry");
  TORCH_CHECK(dy.size(0) == N && dy.size(2) == sdml::conv_out_size(H, ks, stride, pad) &&
              dy.size(3) == sdml::conv_out_size(W, ks, stride, pad), "conv_wgrad_bf16_: shape mismatch");
  if (dy.numel() == 0) return;
  auto ws = torch::empty({(int64_t)sdml::conv_wgrad_workspace_floats(N, H, W, C, Co, ks, stride, pad)},
                         x.options().dtype(torch::kFloat32).memory_format(at::MemoryFormat::Contiguous));
  sdml::conv_wgrad_bf16(dy.data_ptr(), x.data_ptr(), gw.data_ptr(), ws.data_ptr<float>(), N, H, W, C, Co, ks, stride,
                        pad, cur_stream());
}

// stem convolution, one input channel: y (channels-last [N][Co][H][W]) = conv3x3(x [N][1][H][W], w)
torch::Tensor conv_c1_fwd_bf16(torch::Tensor x, torch::Tensor w) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == torch::kBFloat16 && x.dim() == 4 && x.size(1) == 1 && x.is_contiguous(),
              "conv_c1_fwd_bf16: x must be contiguous [N][1][H][W] bf16");
  TORCH_CHECK(w.is_cuda() && w.scalar_type() == torch::kBFloat16 && w.dim() == 4 && w.size(1) == 1 && w.size(2) == 3 &&
              w.size(3) == 3 && w.is_contiguous() && sdml::conv_c1_supported(w.size(0)),
              "conv_c1_fwd_bf16: w must be contiguous [Co][1][3][3] bf16, Co % 16 == 0, Co <= 512");
  const int64_t N = x.size(0), H = x.size(2), W = x.size(3), Co = w.size(0);
  auto y = torch::empty({N, Co, H, W}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  if (N * H * W > 0) sdml::conv_c1_fwd_bf16(x.data_ptr(), w.data_ptr(), y.data_ptr(), N, H, W, Co, cur_stream());
  return y;
}

// gw ([Co][1][3][3] bf16, in place) += dW of the stem convolution for output gradient dy (channels-last)
void conv_c1_wgrad_bf16_(torch::Tensor dy, torch::Tensor x, torch::Tensor gw) {
  check_cl_bf16(dy, "dy");
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == torch::kBFloat16 && x.dim() == 4 && x.size(1) == 1 && x.is_contiguous(),
              "conv_c1_wgrad_bf16_: x must be contiguous [N][1][H][W] bf16");
  TORCH_CHECK(gw.is_contiguous() && gw.scalar_type() == torch::kBFloat16 && gw.dim() == 4 && gw.size(0) == dy.size(1) &&
              gw.size(1) == 1 && sdml::conv_c1_supported(gw.size(0)), "conv_c1_wgrad_bf16_: gw [Co][1][3][3] bf16");
  const int64_t N = x.size(0), H = x.size(2), W = x.size(3), Co = dy.size(1);
  TORCH_CHECK(dy.size(0) == N && dy.size(2) == H && dy.size(3) == W, "conv_c1_wgrad_bf16_: shape mismatch");
  if (N * H * W == 0) return;
  auto ws = torch::empty({(int64_t)sdml::conv_c1_wgrad_workspace_floats(N, H, W, Co)},
                         x.options().dtype(torch::kFloat32));
  sdml::conv_c1_wgrad_bf16(dy.data_ptr(), x.data_ptr(), gw.data_ptr(), ws.data_ptr<float>(), N, H, W, Co, cur_stream());
}

std::tuple<torch::Tensor, torch::Tensor, torch::Tensor> bn_nhwc_fwd(
    torch::Tensor x, c10::optional<torch::Tensor> res, torch::Tensor gamma, torch::Tensor beta,
    c10::optional<torch::Tensor> rmean, c10::optional<torch::Tensor> rvar, double eps, double momentum, bool relu,
    c10::optional<torch::Tensor> num_batches_tracked, c10::optional<torch::Tensor> part) {
  check_cl_bf16(x, "x");
  int64_t* nbt = nullptr;
  if (num_batches_tracked.has_value() && num_batches_tracked->defined()) {
    TORCH_CHECK(num_batches_tracked->is_cuda() && num_batches_tracked->scalar_type() == torch::kLong &&
                    num_batches_tracked->numel() == 1, "bn_nhwc_fwd: num_batches_tracked must be a device int64 scalar");
    nbt = num_batches_tracked->data_ptr<int64_t>();
  }
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3), M = N * H * W;
  TORCH_CHECK(sdml::bn_nhwc_supported(C), "bn_nhwc_fwd: C must be a multiple of 8 and <= 2048");
  if (res.has_value() && res->defined()) {
    check_cl_bf16(*res, "res");
    TORCH_CHECK(res->sizes() == x.sizes(), "bn_nhwc_fwd: residual shape mismatch");
  }
  check_bn_vec(gamma, C, "gamma");
  check_bn_vec(beta, C, "beta");
  check_bn_vec(rmean, C, "running_mean");
  check_bn_vec(rvar, C, "running_var");
  auto y = torch::empty_like(x, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  auto f = x.options().dtype(torch::kFloat32).memory_format(at::MemoryFormat::Contiguous);
  auto mean = torch::empty({C}, f), rstd = torch::empty({C}, f);
  auto ws = torch::empty({(int64_t)sdml::bn_nhwc_workspace_floats(M, C)}, f);
  // part: the producing convolution's per-tile partials of x (conv_part_rows(N, H, W) rows), instead of
  // the statistics pass over x
  const float* pp = conv_part(part, N, H, W, C, "bn_nhwc_fwd");
  const int prow = pp ? sdml::conv_part_rows(N, H, W) : 0;
  if (M > 0)
    sdml::bn_nhwc_fwd_bf16(x.data_ptr(), opt_data(res), gamma.data_ptr(), beta.data_ptr(), opt_data(rmean),
                           opt_data(rvar), M, C, (float)eps, (float)momentum, relu, y.data_ptr(), mean.data_ptr<float>(),
                           rstd.data_ptr<float>(), ws.data_ptr<float>(), cur_stream(), nbt, pp, prow);
  return {y, mean, rstd};
}

// returns (dx, dres or None); ggamma/gbeta (bf16) are accumulated in place
std::tuple<torch::Tensor, c10::optional<torch::Tensor>> bn_nhwc_bwd(
    torch::Tensor x, torch::Tensor dy, c10::optional<torch::Tensor> y, torch::Tensor mean, torch::Tensor rstd,
    torch::Tensor gamma, bool relu, bool need_dres, c10::optional<torch::Tensor> ggamma,
    c10::optional<torch::Tensor> gbeta, c10::optional<torch::Tensor> beta, c10::optional<torch::Tensor> part,
    int64_t part_rows) {
  check_cl_bf16(x, "x");
  check_cl_bf16(dy, "dy");
  TORCH_CHECK(dy.sizes() == x.sizes(), "bn_nhwc_bwd: dy shape mismatch");
  const bool have_y = y.has_value() && y->defined();
  if (relu) {  // the mask comes from y, or is recomputed from x with beta (no residual)
    TORCH_CHECK(have_y || (beta.has_value() && beta->defined()), "bn_nhwc_bwd: relu needs y or beta");
    if (have_y) check_cl_bf16(*y, "y");
  }
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3), M = N * H * W;
  check_bn_vec(gamma, C, "gamma");
  check_bn_vec(ggamma, C, "ggamma");
  check_bn_vec(gbeta, C, "gbeta");
  check_bn_vec(beta, C, "beta");
  TORCH_CHECK(mean.numel() == C && rstd.numel() == C && mean.scalar_type() == torch::kFloat32, "bn_nhwc_bwd: stats");
  auto cl = x.options().memory_format(at::MemoryFormat::ChannelsLast);
  auto dx = torch::empty_like(x, cl);
  c10::optional<torch::Tensor> dres;
  if (need_dres) dres = torch::empty_like(x, cl);
  auto ws = torch::empty({(int64_t)sdml::bn_nhwc_workspace_floats(M, C)},
                         x.options().dtype(torch::kFloat32).memory_format(at::MemoryFormat::Contiguous));
  // part: the per-tile backward sums the convolution that produced dy wrote (conv3x3_fwd_bf16 / conv_dgrad_s2_bf16
  // with bn_x = x), part_rows rows of [2][C]
  const float* pp = nullptr;
  if (part.has_value() && part->defined()) {
    TORCH_CHECK(part->is_cuda() && part->is_contiguous() && part->scalar_type() == torch::kFloat32 && part_rows > 0 &&
                    part->numel() == part_rows * 2 * C, "bn_nhwc_bwd: part must be a contiguous fp32 [part_rows][2][C]");
    pp = part->data_ptr<float>();
  }
  if (M > 0)
    sdml::bn_nhwc_bwd_bf16(x.data_ptr(), dy.data_ptr(), (relu && have_y) ? y->data_ptr() : nullptr,
                           mean.data_ptr<float>(), rstd.data_ptr<float>(), gamma.data_ptr(), M, C, relu, dx.data_ptr(),
                           need_dres ? dres->data_ptr() : nullptr, opt_data(ggamma), opt_data(gbeta),
                           ws.data_ptr<float>(), cur_stream(), opt_data(beta), pp, (int)part_rows);
  return {dx, dres};
}

torch::Tensor bn_nhwc_eval(torch::Tensor x, c10::optional<torch::Tensor> res, torch::Tensor scale, torch::Tensor shift,
                           bool relu) {
  check_cl_bf16(x, "x");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3), M = N * H * W;
  TORCH_CHECK(scale.numel() == C && shift.numel() == C && scale.scalar_type() == torch::kFloat32 &&
              shift.scalar_type() == torch::kFloat32 && scale.is_contiguous() && shift.is_contiguous(),
              "bn_nhwc_eval: fp32 [C] scale/shift");
  if (res.has_value() && res->defined()) check_cl_bf16(*res, "res");
  auto y = torch::empty_like(x, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  if (M > 0)
    sdml::bn_nhwc_eval_bf16(x.data_ptr(), opt_data(res), scale.data_ptr<float>(), shift.data_ptr<float>(), M, C, relu,
                            y.data_ptr(), cur_stream());
  return y;
}

using HeadOut = std::tuple<torch::Tensor, c10::optional<torch::Tensor>, c10::optional<torch::Tensor>>;

// fused head; returns (stats[2] = {loss_sum, correct}, dx or None, dx_amax or None), dx_amax = the
// MFMA head's per-block bounds on |dx| (what linear_wgrad_u8 takes for dz). If `stats_acc` is given
// the kernel accumulates into it (and returns it) instead of allocating a new one; with
// `stats_init` it overwrites it (stats_acc may then hold anything: no zero-fill launch).
HeadOut head_logsoftmax_nll_f32(
    torch::Tensor x, torch::Tensor w, torch::Tensor b, torch::Tensor target, c10::optional<torch::Tensor> gw,
    c10::optional<torch::Tensor> gb, double scale, bool need_dx, c10::optional<torch::Tensor> stats_acc,
    bool mask_dx, bool stats_init) {
  check_f32_cuda(x, "x");
  check_f32_cuda(w, "w");
  check_f32_cuda(b, "b");
  TORCH_CHECK(target.is_cuda() && target.scalar_type() == torch::kInt64 && target.is_contiguous(),
              "target must be a contiguous int64 device tensor");
  const int64_t M = x.size(0), K = x.size(1), C = w.size(0);
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && w.size(1) == K && b.numel() == C && target.numel() == M,
              "head: shape mismatch");
  TORCH_CHECK(C >= 1 && C <= 32, "head: 1..32 classes supported");
  check_opt(gw, "gw", C * K);
  check_opt(gb, "gb", C);
  check_opt(stats_acc, "stats_acc", 2);
  const bool fresh = !opt_ptr(stats_acc);
  auto stats = fresh ? torch::empty({2}, x.options()) : *stats_acc;
  const bool overwrite = fresh || stats_init;
  const bool train = opt_ptr(gw) != nullptr || opt_ptr(gb) != nullptr || need_dx;
  c10::optional<torch::Tensor> dx;
  if (M == 0) {
    if (overwrite) stats.zero_();
    return {stats, need_dx ? c10::optional<torch::Tensor>(torch::empty({0, K}, x.options())) : c10::nullopt,
            c10::nullopt};
  }
  hipStream_t s = cur_stream();
  const bool fusable = sdml::head_fused_supported((int)K, (int)C) || sdml::head_lds_supported((int)M, (int)K, (int)C);
  const bool fused = fusable && (!train || (opt_ptr(gw) && opt_ptr(gb)));
  torch::Tensor ws;
  if (fused) ws = torch::empty({(int64_t)sdml::head_workspace_floats(M, K, C)}, x.options());
  float* wsp = fused ? ws.data_ptr<float>() : nullptr;
  if (!train) {
    sdml::head_logsoftmax_nll(x.data_ptr<float>(), w.data_ptr<float>(), b.data_ptr<float>(),
                              target.data_ptr<int64_t>(), M, K, C, (float)scale, stats.data_ptr<float>(), nullptr,
                              nullptr, nullptr, nullptr, wsp, false, s, nullptr, overwrite);
    return {stats, c10::nullopt, c10::nullopt};
  }
  auto dxt = torch::empty({M, K}, x.options());
  c10::optional<torch::Tensor> amax;
  if (fused) {
    auto am = torch::empty({sdml::kHeadAmaxMax}, x.options());
    int n_am = 0;
    sdml::head_logsoftmax_nll(x.data_ptr<float>(), w.data_ptr<float>(), b.data_ptr<float>(),
                              target.data_ptr<int64_t>(), M, K, C, (float)scale, stats.data_ptr<float>(),
                              dxt.data_ptr<float>(), opt_ptr(gw), opt_ptr(gb), nullptr, wsp, mask_dx, s, nullptr,
                              overwrite, am.data_ptr<float>(), &n_am);
    if (n_am > 0) amax = am.narrow(0, 0, n_am);
  } else {
    auto dz = torch::empty({M, C}, x.options());
    sdml::head_logsoftmax_nll(x.data_ptr<float>(), w.data_ptr<float>(), b.data_ptr<float>(),
                              target.data_ptr<int64_t>(), M, K, C, (float)scale, stats.data_ptr<float>(),
                              dxt.data_ptr<float>(), nullptr, nullptr, dz.data_ptr<float>(), nullptr, mask_dx, s, nullptr,
                              overwrite);
    if (opt_ptr(gw)) {
      sdml::GemmArgs g;  // gw[C,K] += dz^T x ; gb += colsum(dz)
      g.A = dz.data_ptr<float>();
      g.B = x.data_ptr<float>();
      g.C = opt_ptr(gw);
      g.rowsum = opt_ptr(gb);
      g.M = C;
      g.N = K;
      g.K = M;
      g.lda = C;
      g.ldb = K;
      g.ldc = K;
      g.a_kmajor = true;
      g.b_kmajor = true;
      g.epi = sdml::EPI_ATOMIC;
      g.splits = sdml::gemm_f32_pick_splits(g.M, g.N, g.K);
      TORCH_CHECK(sdml::gemm_f32_supported(g), "head dW: unsupported");
      sdml::gemm_f32(g, s);
    } else if (opt_ptr(gb)) {
      gb->add_(dz.sum(0));
    }
  }
  if (need_dx) dx = dxt;
  return {stats, dx, need_dx ? amax : c10::nullopt};
}

// training head that returns its boundary gradient as the factor dl = scale * (softmax - onehot) [M, C]
// (dx = dl @ w, rebuilt by head_dx_from_dl wherever w is held); gw/gb accumulated, loss and correct
// count accumulated into stats_acc [2] (overwritten with stats_init). Returns (dl, bound or None):
// the MFMA head's per-block bounds on |dl @ w| (what linear_wgrad_u8_dl takes as amax)
// A head reduction deferred by head_logsoftmax_nll_dl_f32(defer_reduce=True): keeps the slab workspace
// (and the outputs) alive until it runs - inside linear_wgrad_u8_dl's reduction launch, or alone via
// run() - exactly once.
struct HeadPending {
  sdml::HeadReduceArgs args;
  torch::Tensor ws, gw, gb, stats;
  bool pending() const { return args.part != nullptr; }
  void run() {
    if (!pending()) return;
    sdml::head_reduce_run(args, cur_stream());
    done();
  }
  void done() {
    args = sdml::HeadReduceArgs();
    ws = torch::Tensor();
  }
};

std::tuple<torch::Tensor, c10::optional<torch::Tensor>, std::shared_ptr<HeadPending>> head_logsoftmax_nll_dl_f32(
    torch::Tensor x, torch::Tensor w, torch::Tensor b, torch::Tensor target, torch::Tensor gw, torch::Tensor gb,
    double scale, torch::Tensor stats_acc, bool stats_init, bool defer_reduce) {
  check_f32_cuda(x, "x");
  check_f32_cuda(w, "w");
  check_f32_cuda(b, "b");
  check_f32_cuda(gw, "gw");
  check_f32_cuda(gb, "gb");
  check_f32_cuda(stats_acc, "stats_acc");
  TORCH_CHECK(target.is_cuda() && target.scalar_type() == torch::kInt64 && target.is_contiguous(),
              "target must be a contiguous int64 device tensor");
  const int64_t M = x.size(0), K = x.size(1), C = w.size(0);
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && w.size(1) == K && b.numel() == C && target.numel() == M &&
                  gw.numel() == C * K && gb.numel() == C && stats_acc.numel() == 2,
              "head_dl: shape mismatch");
  TORCH_CHECK(sdml::head_fused_supported((int)K, (int)C), "head_dl: needs the fused head (K == 128, C in {2, 10, 16})");
  auto dl = torch::empty({M, C}, x.options());
  if (M == 0) {
    if (stats_init) stats_acc.zero_();
    return {dl, c10::nullopt, nullptr};
  }
  auto ws = torch::empty({(int64_t)sdml::head_workspace_floats(M, K, C)}, x.options());
  auto am = torch::empty({sdml::kHeadAmaxMax}, x.options());
  int n_am = 0;
  auto pend = std::make_shared<HeadPending>();
  sdml::head_logsoftmax_nll(x.data_ptr<float>(), w.data_ptr<float>(), b.data_ptr<float>(), target.data_ptr<int64_t>(),
                            M, K, C, (float)scale, stats_acc.data_ptr<float>(), nullptr, gw.data_ptr<float>(),
                            gb.data_ptr<float>(), nullptr, ws.data_ptr<float>(), false, cur_stream(),
                            dl.data_ptr<float>(), stats_init, am.data_ptr<float>(), &n_am,
                            defer_reduce ? &pend->args : nullptr);
  std::shared_ptr<HeadPending> out;
  if (pend->pending()) {
    pend->ws = ws;
    pend->gw = gw;
    pend->gb = gb;
    pend->stats = stats_acc;
    out = pend;
  }
  return {dl, n_am > 0 ? c10::optional<torch::Tensor>(am.narrow(0, 0, n_am)) : c10::nullopt, out};
}

// ResNet's last layer: average pool over P positions + Linear + log_softmax + NLL + backward (head_pool.hip).
// x [M, P, K] contiguous (a channels-last activation viewed as [M, H*W, C]); w [C, K]; b [C]; gw/gb the
// parameter gradients (accumulated); stats [2] accumulated (overwritten with stats_init). Returns dx like x.
torch::Tensor head_pool_xent(torch::Tensor x, torch::Tensor w, torch::Tensor b, torch::Tensor target, torch::Tensor gw,
                             torch::Tensor gb, double scale, torch::Tensor stats, bool stats_init) {
  TORCH_CHECK(x.is_cuda() && x.dim() == 3 && x.is_contiguous(), "head_pool_xent: x must be a contiguous [M, P, K] device tensor");
  const auto dt = x.scalar_type();
  TORCH_CHECK(dt == torch::kBFloat16 || dt == torch::kFloat32, "head_pool_xent: bf16 or fp32");
  for (auto* t : {&w, &b, &gw, &gb})
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == dt && t->is_contiguous(), "head_pool_xent: w/b/gw/gb must match x");
  check_f32_cuda(stats, "stats");
  TORCH_CHECK(target.is_cuda() && target.scalar_type() == torch::kInt64 && target.is_contiguous(),
              "target must be a contiguous int64 device tensor");
  const int64_t M = x.size(0), P = x.size(1), K = x.size(2), C = w.size(0);
  TORCH_CHECK(w.dim() == 2 && w.size(1) == K && b.numel() == C && gw.numel() == C * K && gb.numel() == C &&
                  target.numel() == M && stats.numel() == 2,
              "head_pool_xent: shape mismatch");
  TORCH_CHECK(sdml::head_pool_supported((int)M, (int)P, (int)K, (int)C), "head_pool_xent: unsupported shape");
  TORCH_CHECK((reinterpret_cast<uintptr_t>(x.data_ptr()) & 15) == 0 && (reinterpret_cast<uintptr_t>(w.data_ptr()) & 15) == 0,
              "head_pool_xent: x and w must be 16-B aligned (16-B loads)");
  auto dx = torch::empty_like(x);
  auto ws = torch::empty({sdml::head_pool_workspace_floats((int)M, (int)K, (int)C)}, stats.options());
  sdml::head_pool_xent(x.data_ptr(), w.data_ptr(), b.data_ptr(), target.data_ptr<int64_t>(), (int)M, (int)P, (int)K,
                       (int)C, (float)scale, dx.data_ptr(), gw.data_ptr(), gb.data_ptr(), stats.data_ptr<float>(),
                       stats_init, ws.data_ptr<float>(), dt == torch::kBFloat16, cur_stream());
  return dx;
}

// dx = (dl @ w) * (x > 0 if mask): the fused head's boundary gradient rebuilt from its factor
torch::Tensor head_dx_from_dl(torch::Tensor dl, torch::Tensor w, torch::Tensor x, bool mask) {
  check_f32_cuda(dl, "dl");
  check_f32_cuda(w, "w");
  check_f32_cuda(x, "x");
  const int64_t M = dl.size(0), C = dl.size(1), K = w.size(1);
  TORCH_CHECK(dl.dim() == 2 && w.dim() == 2 && w.size(0) == C && x.dim() == 2 && x.size(0) == M && x.size(1) == K,
              "head_dx_from_dl: shape mismatch");
  TORCH_CHECK(sdml::head_fused_supported((int)K, (int)C), "head_dx_from_dl: K == 128, C in {2, 10, 16}");
  auto dx = torch::empty({M, K}, x.options());
  sdml::head_dx_from_dl(dl.data_ptr<float>(), w.data_ptr<float>(), x.data_ptr<float>(), dx.data_ptr<float>(), (int)M,
                        (int)K, (int)C, mask, cur_stream());
  return dx;
}

// first layer's weight gradient from the FACTORED boundary gradient: gw += scale * dz^T x_u8,
// gb += colsum(dz) with dz = (dl @ w2) * (h > 0) - expanded inside mlp_u8.hip's wgrad kernel when
// it applies (bit-identical to head_dx_from_dl followed by linear_wgrad_u8), else those two
// head: a deferred head reduction (HeadPending) to run in this call's reduction launch (or before it).
// sgd (optional, with head): (params, grads, momentum_buffer, lr, momentum, dampening, weight_decay,
// nesterov, first, zero_grad, planes | None, plane_offset, plane_rows, plane_k) of the flat buffers
// gw/gb and the head's gW/gb live in - when these are the step's last gradients, the optimizer step is
// applied inside the same reduction launch. Returns whether it was (else the caller steps).
// act: the layer's output h [M][N] fp32, or its ReLU bits [M][N / 32] int32 (linear_fwd_u8's mask_out /
// linear_relu_head_u8) - only the mask is used
bool linear_wgrad_u8_dl(torch::Tensor x, torch::Tensor dl, torch::Tensor w2, torch::Tensor act, torch::Tensor gw,
                        torch::Tensor gb, double scale, c10::optional<torch::Tensor> amax,
                        std::shared_ptr<HeadPending> head, c10::optional<py::tuple> sgd,
                        c10::optional<py::tuple> groups) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == torch::kUInt8 && x.is_contiguous() && x.dim() == 2,
              "linear_wgrad_u8_dl: x must be a contiguous 2-D uint8 ROCm tensor");
  check_f32_cuda(dl, "dl");
  check_f32_cuda(w2, "w2");
  check_f32_cuda(gw, "gw");
  check_f32_cuda(gb, "gb");
  const bool bits = act.scalar_type() == torch::kInt32;
  if (bits) {
    TORCH_CHECK(act.is_cuda() && act.is_contiguous() && act.dim() == 2, "linear_wgrad_u8_dl: bad mask");
  } else {
    check_f32_cuda(act, "h");
  }
  const int64_t M = x.size(0), K = x.size(1), N = bits ? act.size(1) * 32 : act.size(1), C = dl.size(1);
  TORCH_CHECK(dl.dim() == 2 && dl.size(0) == M && w2.dim() == 2 && w2.size(0) == C && w2.size(1) == N &&
                  act.dim() == 2 && act.size(0) == M && gw.size(0) == N && gw.size(1) == K && gb.numel() == N,
              "linear_wgrad_u8_dl: shape mismatch");
  const bool gb_follows = gw.is_contiguous() && gb.is_contiguous() && gb.data_ptr<float>() == gw.data_ptr<float>() + N * K;
  if (gb_follows && sdml::head_fused_supported((int)N, (int)C) &&
      sdml::u8_wgrad_dl_supported((int)M, (int)N, (int)K, (int)K, x.data_ptr(), act.data_ptr(), (int)C)) {
    sdml::WgradGroups grp{0, 0, 0};
    if (groups.has_value()) {  // (g_first, g_count, blocks): one hidden-group range (data-parallel split)
      const py::tuple& g = *groups;
      TORCH_CHECK(g.size() == 3, "linear_wgrad_u8_dl: groups = (g_first, g_count, blocks)");
      grp.g_first = g[0].cast<int>();
      grp.g_count = g[1].cast<int>();
      grp.blocks = g[2].cast<int>();
      TORCH_CHECK(grp.g_first >= 0 && grp.g_count >= 1 && (grp.g_first + grp.g_count) * 64 <= N && grp.blocks >= 1 &&
                      !sgd.has_value(),
                  "linear_wgrad_u8_dl: groups must be whole 64-unit hidden groups inside N, without sgd");
    }
    auto ws = torch::empty({sdml::u8_wgrad_slab_floats((int)M, (int)N, groups.has_value() ? grp.blocks : 0)},
                           gw.options());
    const bool has_am = amax.has_value() && amax->defined();
    if (has_am) {
      check_f32_cuda(*amax, "amax");
      TORCH_CHECK(amax->numel() >= 1 && amax->is_contiguous(), "linear_wgrad_u8_dl: amax must be non-empty");
    }
    const bool fuse_head = head && head->pending();
    sdml::SgdFuse sg;
    if (fuse_head && sgd.has_value() && (head->args.flags & 1) &&
        head->args.gb == head->args.gW + head->args.CK) {
      const py::tuple& t = *sgd;
      TORCH_CHECK(t.size() == 14, "linear_wgrad_u8_dl: sgd tuple of 14");
      auto P = t[0].cast<torch::Tensor>(), G = t[1].cast<torch::Tensor>(), B = t[2].cast<torch::Tensor>();
      check_f32_cuda(P, "params");
      check_f32_cuda(G, "grads");
      const int64_t nflat = G.numel();
      const int64_t off_w = gw.data_ptr<float>() - G.data_ptr<float>();
      const int64_t off_h = head->args.gW - G.data_ptr<float>();
      const float mom = (float)t[4].cast<double>();
      TORCH_CHECK(P.numel() == nflat && off_w >= 0 && off_w % 4 == 0 && off_w + N * K + N <= nflat && off_h >= 0 &&
                      off_h % 4 == 0 && off_h + head->args.CK + head->args.C <= nflat &&
                      (mom == 0.f || B.numel() == nflat),
                  "linear_wgrad_u8_dl: gradients outside the flat buffers");
      sg.p = P.data_ptr<float>() + off_w;
      sg.hp = P.data_ptr<float>() + off_h;
      sg.buf = mom != 0.f ? B.data_ptr<float>() + off_w : nullptr;
      sg.hbuf = mom != 0.f ? B.data_ptr<float>() + off_h : nullptr;
      sg.lr = (float)t[3].cast<double>();
      sg.mom = mom;
      sg.damp = (float)t[5].cast<double>();
      sg.wd = (float)t[6].cast<double>();
      sg.nesterov = t[7].cast<bool>() ? 1 : 0;
      sg.first = t[8].cast<bool>() ? 1 : 0;
      sg.zero_grad = t[9].cast<bool>() ? 1 : 0;
      if (!t[10].is_none()) {
        auto planes = t[10].cast<torch::Tensor>();
        const int64_t poff = t[11].cast<int64_t>(), prows = t[12].cast<int64_t>(), pk = t[13].cast<int64_t>();
        TORCH_CHECK(planes.is_cuda() && planes.scalar_type() == torch::kInt16 && planes.is_contiguous() &&
                        planes.dim() == 3 && planes.size(0) == sdml::kU8FwdPlanes && planes.size(1) == prows &&
                        poff >= off_w && (poff - off_w) % 4 == 0 && pk % 4 == 0 && poff + prows * pk <= off_w + N * K,
                    "linear_wgrad_u8_dl: planes must cover a weight inside gw");
        sg.planes = reinterpret_cast<unsigned short*>(planes.data_ptr<int16_t>());
        sg.pl_off4 = (poff - off_w) / 4;
        sg.pl_n4 = prows * pk / 4;
        sg.K = pk;
        sg.Kp = planes.size(2);
        sg.plane_stride = prows * planes.size(2);
      }
    }
    sdml::u8_wgrad_dl(dl.data_ptr<float>(), w2.data_ptr<float>(), bits ? nullptr : act.data_ptr<float>(),
                      bits ? reinterpret_cast<const unsigned*>(act.data_ptr<int32_t>()) : nullptr, (int)C,
                      x.data_ptr<uint8_t>(), (int)M, (int)N, (int)K, ws.data_ptr<float>(), gw.data_ptr<float>(), (float)scale,
                      has_am ? amax->data_ptr<float>() : nullptr, has_am ? (int)amax->numel() : 0, cur_stream(),
                      fuse_head ? &head->args : nullptr, sg.p ? &sg : nullptr, groups.has_value() ? &grp : nullptr);
    if (fuse_head) head->done();
    return sg.p != nullptr;
  }
  if (head) head->run();
  torch::Tensor dz;
  if (bits) dz = at::matmul(dl, w2).mul_(relu_bits_unpack(act));
  else dz = sdml::head_fused_supported((int)N, (int)C) ? head_dx_from_dl(dl, w2, act, true)
                                                       : at::matmul(dl, w2).mul_((act > 0).to(act.scalar_type()));
  if (groups.has_value()) {  // only the hidden-group range asked for
    const py::tuple& g = *groups;
    const int64_t lo = g[0].cast<int64_t>() * 64, cnt = g[1].cast<int64_t>() * 64;
    TORCH_CHECK(lo >= 0 && cnt > 0 && lo + cnt <= N, "linear_wgrad_u8_dl: bad hidden-group range");
    auto gws = gw.narrow(0, lo, cnt), gbs = gb.narrow(0, lo, cnt);
    linear_wgrad_u8(x, dz.narrow(1, lo, cnt).contiguous(), gws, gbs, scale, c10::nullopt);
    return false;
  }
  linear_wgrad_u8(x, dz, gw, gb, scale, amax);
  return false;
}

// The uint8 first layer + classifier head in one launch (mlp_u8.hip u8_fwd_head, training): h =
// relu(scale x @ w1.T + b1) never leaves the chip; writes dl = loss_scale (softmax - onehot) into
// dl_out [M, C] and the ReLU bits into mask_out [M, 4]; loss sum / correct count go to stats (overwritten
// with stats_init), dW2/db2 to gw2/gb2 through a slab reduction - deferred (returned as HeadPending, for
// linear_wgrad_u8_dl's reduction launch) with `defer`, else run here. Returns (dl bounds, pending).
std::tuple<torch::Tensor, std::shared_ptr<HeadPending>> linear_relu_head_u8(
    torch::Tensor x, torch::Tensor w1, torch::Tensor b1, double scale, torch::Tensor planes, bool planes_valid,
    torch::Tensor w2, torch::Tensor b2, torch::Tensor target, torch::Tensor gw2, torch::Tensor gb2, double loss_scale,
    torch::Tensor stats, bool stats_init, torch::Tensor dl_out, torch::Tensor mask_out, bool defer) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == torch::kUInt8 && x.is_contiguous() && x.dim() == 2,
              "linear_relu_head_u8: x must be a contiguous 2-D uint8 ROCm tensor");
  for (auto* t : {&w1, &b1, &w2, &b2, &gw2, &gb2, &stats, &dl_out}) check_f32_cuda(*t, "linear_relu_head_u8");
  TORCH_CHECK(target.is_cuda() && target.scalar_type() == torch::kInt64 && target.is_contiguous(),
              "target must be a contiguous int64 device tensor");
  const int64_t M = x.size(0), K = x.size(1), N = w1.size(0), C = w2.size(0);
  TORCH_CHECK(w1.dim() == 2 && w1.size(1) == K && b1.numel() == N && w2.dim() == 2 && w2.size(1) == N &&
                  b2.numel() == C && target.numel() == M && gw2.numel() == C * N && gb2.numel() == C &&
                  stats.numel() == 2 && dl_out.dim() == 2 && dl_out.size(0) == M && dl_out.size(1) == C,
              "linear_relu_head_u8: shape mismatch");
  check_mask_out(mask_out, M, N);
  TORCH_CHECK(sdml::u8_fwd_head_supported((int)M, (int)N, (int)K, (int)K, x.data_ptr(), (int)C),
              "linear_relu_head_u8: unsupported shape (u8_fwd_head_supported)");
  const int Kp = sdml::u8_fwd_kpad((int)K);
  TORCH_CHECK(planes.is_cuda() && planes.scalar_type() == torch::kInt16 && planes.is_contiguous() &&
                  planes.dim() == 3 && planes.size(0) == sdml::kU8FwdPlanes && planes.size(1) == N && planes.size(2) == Kp,
              "linear_relu_head_u8: planes must be a [u8_fwd_planes()][N][u8_fwd_kpad(K)] int16 device tensor");
  auto* wpp = reinterpret_cast<unsigned short*>(planes.data_ptr<int16_t>());
  if (!planes_valid) sdml::split_planes_pad(w1.data_ptr<float>(), wpp, (int)N, (int)K, Kp, cur_stream());
  const int blocks = sdml::u8_fwd_head_blocks((int)M);
  auto ws = torch::empty({(int64_t)blocks * (C * N + C + 2)}, w1.options());
  auto bound = torch::empty({blocks}, w1.options());
  sdml::U8HeadArgs h;
  h.w2 = w2.data_ptr<float>();
  h.b2 = b2.data_ptr<float>();
  h.target = target.data_ptr<int64_t>();
  h.C = (int)C;
  h.loss_scale = (float)loss_scale;
  h.dl = dl_out.data_ptr<float>();
  h.mask = reinterpret_cast<unsigned*>(mask_out.data_ptr<int32_t>());
  h.part = ws.data_ptr<float>();
  h.bound = bound.data_ptr<float>();
  sdml::u8_fwd_head(x.data_ptr<uint8_t>(), (int)M, (int)K, (int)K, wpp, (int)N, Kp, b1.data_ptr<float>(), (float)scale, h,
                    cur_stream());
  auto pend = std::make_shared<HeadPending>();
  pend->args.part = ws.data_ptr<float>();
  pend->args.nblocks = blocks;
  pend->args.CK = (int)(C * N);
  pend->args.C = (int)C;
  pend->args.gW = gw2.data_ptr<float>();
  pend->args.gb = gb2.data_ptr<float>();
  pend->args.stats = stats.data_ptr<float>();
  pend->args.flags = 1 | (stats_init ? 2 : 0);
  pend->ws = ws;
  pend->gw = gw2;
  pend->gb = gb2;
  pend->stats = stats;
  if (!defer) {
    pend->run();
    return {bound, nullptr};
  }
  return {bound, pend};
}

void check_bf16_cuda(const torch::Tensor& t, const char* name);  // (defined with the transformer ops)

torch::Tensor gelu_fwd_bf16(torch::Tensor x) {
  check_bf16_cuda(x, "x");
  TORCH_CHECK(x.numel() % 8 == 0, "gelu: numel % 8 == 0");
  auto y = torch::empty_like(x);
  sdml::gelu_fwd_bf16(x.data_ptr(), y.data_ptr(), x.numel(), cur_stream());
  return y;
}

// gx = gy * gelu'(x); in place into gy when `inplace`
torch::Tensor gelu_bwd_bf16(torch::Tensor gy, torch::Tensor x, bool inplace) {
  check_bf16_cuda(gy, "gy");
  check_bf16_cuda(x, "x");
  TORCH_CHECK(gy.numel() == x.numel() && x.numel() % 8 == 0, "gelu_bwd: shape mismatch");
  auto gx = inplace ? gy : torch::empty_like(gy);
  sdml::gelu_bwd_bf16(gy.data_ptr(), x.data_ptr(), gx.data_ptr(), x.numel(), cur_stream());
  return gx;
}

torch::Tensor embedding_fwd_bf16(torch::Tensor tok, torch::Tensor wte, torch::Tensor wpe) {
  TORCH_CHECK(tok.is_cuda() && tok.scalar_type() == torch::kInt64 && tok.is_contiguous() && tok.dim() == 2,
              "embedding: tokens must be a contiguous int64 [B, S] device tensor");
  check_bf16_cuda(wte, "wte");
  check_bf16_cuda(wpe, "wpe");
  const int64_t B = tok.size(0), S = tok.size(1), C = wte.size(1);
  TORCH_CHECK(wpe.size(1) == C && wpe.size(0) >= S && C % 4 == 0, "embedding: shape mismatch");
  auto out = torch::empty({B, S, C}, wte.options());
  sdml::embedding_fwd_bf16(tok.data_ptr<int64_t>(), wte.data_ptr(), wpe.data_ptr(), out.data_ptr(), (int)(B * S),
                           (int)S, (int)C, (int)wte.size(0), cur_stream());
  return out;
}

void embedding_bwd_bf16(torch::Tensor g, torch::Tensor sorted_tok, torch::Tensor perm,
                        c10::optional<torch::Tensor> gwte, c10::optional<torch::Tensor> gwpe) {
  check_bf16_cuda(g, "g");
  TORCH_CHECK(g.dim() == 3 && sorted_tok.is_cuda() && perm.is_cuda() && sorted_tok.scalar_type() == torch::kInt64 &&
                  perm.scalar_type() == torch::kInt64 && sorted_tok.numel() == g.size(0) * g.size(1) &&
                  perm.numel() == sorted_tok.numel() && sorted_tok.is_contiguous() && perm.is_contiguous(),
              "embedding_bwd: shape mismatch");
  const int64_t B = g.size(0), S = g.size(1), C = g.size(2);
  int64_t V = 0;
  void* pw = nullptr;
  void* pp = nullptr;
  if (gwte.has_value() && gwte->defined()) {
    check_bf16_cuda(*gwte, "gwte");
    TORCH_CHECK(gwte->size(1) == C, "embedding_bwd: wte grad shape");
    V = gwte->size(0);
    pw = gwte->data_ptr();
  }
  if (gwpe.has_value() && gwpe->defined()) {
    check_bf16_cuda(*gwpe, "gwpe");
    TORCH_CHECK(gwpe->size(1) == C && gwpe->size(0) >= S, "embedding_bwd: wpe grad shape");
    pp = gwpe->data_ptr();
  }
  sdml::embedding_bwd_bf16(g.data_ptr(), sorted_tok.data_ptr<int64_t>(), perm.data_ptr<int64_t>(), pw, pp, (int)B,
                           (int)S, (int)C, (int)V, cur_stream());
}

// the whole 784-128-10 training step in two launches (mlp_small.hip); params/momentum are
// views into the flat buffers (momentum views None without momentum). Returns False if not launched.
bool mlp_small_step(torch::Tensor x, torch::Tensor target, torch::Tensor w1, torch::Tensor b1, torch::Tensor w2,
                    torch::Tensor b2, c10::optional<torch::Tensor> m1, c10::optional<torch::Tensor> mb1,
                    c10::optional<torch::Tensor> m2, c10::optional<torch::Tensor> mb2, double lr, double mom,
                    double damp, double wd, bool nesterov, bool first, double scale, torch::Tensor stats) {
  TORCH_CHECK(x.is_cuda() && x.is_contiguous() && x.dim() == 2 && x.size(1) == 784 &&
                  (x.scalar_type() == torch::kFloat32 || x.scalar_type() == torch::kUInt8),
              "mlp_small_step: x must be a contiguous [B, 784] fp32 or uint8 device tensor");
  TORCH_CHECK(target.is_cuda() && target.scalar_type() == torch::kInt64 && target.is_contiguous() &&
                  target.numel() == x.size(0),
              "mlp_small_step: target");
  for (auto* t : {&w1, &b1, &w2, &b2, &stats}) check_f32_cuda(*t, "mlp_small_step");
  TORCH_CHECK(w1.numel() == 128 * 784 && b1.numel() == 128 && w2.numel() == 10 * 128 && b2.numel() == 10 &&
                  stats.numel() == 2,
              "mlp_small_step: the 784-128-10 MLP only");
  const bool has_m = m1.has_value() && m1->defined();
  if (has_m) {
    TORCH_CHECK(mb1 && m2 && mb2 && m1->numel() == w1.numel() && mb1->numel() == 128 && m2->numel() == 1280 &&
                    mb2->numel() == 10,
                "mlp_small_step: momentum buffers");
  }
  const int64_t B = x.size(0);
  if (B < 1 || B > sdml::mlp_small_step_max_batch()) return false;
  auto h = torch::empty({B * 128 + 10 * 128 + 10}, w1.options());  // h, then the W2/b2 snapshot
  auto mp = [&](c10::optional<torch::Tensor>& t) { return has_m ? t->data_ptr<float>() : nullptr; };
  return sdml::mlp_small_step(x.data_ptr(), x.scalar_type() == torch::kUInt8, target.data_ptr<int64_t>(), (int)B,
                              (float)scale, w1.data_ptr<float>(), b1.data_ptr<float>(), w2.data_ptr<float>(),
                              b2.data_ptr<float>(), mp(m1), mp(mb1), mp(m2), mp(mb2), (float)lr, (float)mom,
                              (float)damp, (float)wd, nesterov, first, h.data_ptr<float>(),
                              h.data_ptr<float>() + B * 128, stats.data_ptr<float>(), cur_stream());
}

// the reference CNN's training step (both stages, SGD of all 8 tensors) in two launches (ref_cnn.hip)
void ref_cnn_step_op(torch::Tensor x, torch::Tensor target, std::vector<torch::Tensor> params,
                     std::vector<c10::optional<torch::Tensor>> bufs, int64_t seed0, int64_t seed1,
                     c10::optional<torch::Tensor> ctr, double p0, bool drop0, double p1, bool drop1, double scale,
                     double lr, double mom, double damp, double wd, bool nesterov, bool first, torch::Tensor stats,
                     c10::optional<torch::Tensor> stamps) {
  check_f32_cuda(x, "x");
  TORCH_CHECK(x.is_contiguous() && x.numel() % 784 == 0, "ref_cnn_step: x must be contiguous [B, 1, 28, 28]");
  const int64_t B = x.numel() / 784;
  TORCH_CHECK(target.is_cuda() && target.scalar_type() == torch::kInt64 && target.is_contiguous() &&
                  target.numel() == B,
              "ref_cnn_step: target");
  TORCH_CHECK(params.size() == 8 && bufs.size() == 8, "ref_cnn_step: 8 parameter tensors");
  static const int64_t sizes[8] = {250, 10, 5000, 20, 16000, 50, 500, 10};
  float* pp[8];
  float* bp[8];
  for (int i = 0; i < 8; ++i) {
    check_f32_cuda(params[i], "param");
    TORCH_CHECK(params[i].is_contiguous() && params[i].numel() == sizes[i], "ref_cnn_step: parameter ", i, " shape");
    pp[i] = params[i].data_ptr<float>();
    bp[i] = nullptr;
    if (bufs[i].has_value() && bufs[i]->defined()) {
      check_f32_cuda(*bufs[i], "momentum");
      TORCH_CHECK(bufs[i]->is_contiguous() && bufs[i]->numel() == sizes[i], "ref_cnn_step: momentum ", i, " shape");
      bp[i] = bufs[i]->data_ptr<float>();
    }
    TORCH_CHECK(mom == 0 || bp[i], "ref_cnn_step: momentum buffers required");
  }
  check_f32_cuda(stats, "stats");
  long long* cp = nullptr;
  if (ctr.has_value() && ctr->defined()) {
    TORCH_CHECK(ctr->is_cuda() && ctr->scalar_type() == torch::kInt64 && ctr->numel() == 1, "ref_cnn_step: ctr");
    cp = reinterpret_cast<long long*>(ctr->data_ptr<int64_t>());
  }
  auto rec = torch::empty({(int64_t)sdml::ref_cnn_step_workspace_floats((int)B)}, x.options());
  sdml::ref_cnn_step(x.data_ptr<float>(), target.data_ptr<int64_t>(), (int)B, pp, bp, (unsigned long long)seed0,
                     (unsigned long long)seed1, cp, (float)p0, drop0, (float)p1, drop1, (float)scale, (float)lr,
                     (float)mom, (float)damp, (float)wd, nesterov, first, rec.data_ptr<float>(),
                     stats.data_ptr<float>(), cur_stream(),
                     stamps.has_value() && stamps->defined() ? reinterpret_cast<long long*>(stamps->data_ptr<int64_t>())
                                                              : nullptr);
}

// C = A . (b_kn ? B : B^T) with a fused epilogue (gemm_bf16.hip); A [M, K] (row stride lda), B [N, K] or
// [K, N]; returns C [M, N] bf16. epi: 0 store, 1 bias, 5 bias+GELU (aux out, allocated here and returned),
// 6 gelu' (aux in).
std::tuple<torch::Tensor, c10::optional<torch::Tensor>> gemm_bf16_op(torch::Tensor A, torch::Tensor B,
                                                                     c10::optional<torch::Tensor> bias, bool b_kn,
                                                                     int64_t epi, c10::optional<torch::Tensor> aux) {
  TORCH_CHECK(A.is_cuda() && A.scalar_type() == torch::kBFloat16 && A.dim() == 2 && A.stride(1) == 1,
              "gemm_bf16: A must be a 2-D bf16 device tensor with unit column stride");
  check_bf16_cuda(B, "B");
  TORCH_CHECK(B.dim() == 2, "gemm_bf16: B must be 2-D");
  const int64_t M = A.size(0), K = A.size(1), N = b_kn ? B.size(1) : B.size(0);
  TORCH_CHECK((b_kn ? B.size(0) : B.size(1)) == K, "gemm_bf16: inner dimensions ", A.sizes(), " vs ", B.sizes());
  TORCH_CHECK(sdml::gemm_bf16_supported((int)M, (int)N, (int)K, (int)A.stride(0), (int)B.stride(0), (int)N, b_kn),
              "gemm_bf16: unsupported shape (gemm_bf16_supported)");
  auto C = torch::empty({M, N}, A.options());
  c10::optional<torch::Tensor> u;
  const void* bp = nullptr;
  if (epi == sdml::EPI_BIAS || epi == sdml::EPI_BIAS_GELU || epi == sdml::EPI_BIAS_GELU_SAVE_GRAD) {
    TORCH_CHECK(bias.has_value() && bias->defined(), "gemm_bf16: bias required");
    check_bf16_cuda(*bias, "bias");
    TORCH_CHECK(bias->numel() == N, "gemm_bf16: bias shape");
    bp = bias->data_ptr();
  }
  void* ap = nullptr;
  int64_t ldaux = N;
  if (epi == sdml::EPI_BIAS_GELU || epi == sdml::EPI_BIAS_GELU_SAVE_GRAD) {
    u = torch::empty({M, N}, A.options());
    ap = u->data_ptr();
  } else if (epi == sdml::EPI_DGELU || epi == sdml::EPI_MUL_GRAD) {
    TORCH_CHECK(aux.has_value() && aux->defined(), "gemm_bf16: pre-activation required");
    check_bf16_cuda(*aux, "aux");
    TORCH_CHECK(aux->numel() == M * N, "gemm_bf16: pre-activation shape");
    ap = aux->data_ptr();
  } else {
    TORCH_CHECK(epi == sdml::EPI_STORE || epi == sdml::EPI_BIAS, "gemm_bf16: unknown epilogue ", epi);
  }
  sdml::gemm_bf16(A.data_ptr(), B.data_ptr(), C.data_ptr(), (int)M, (int)N, (int)K, (int)A.stride(0),
                  (int)B.stride(0), (int)N, b_kn, (int)epi, bp, ap, (int)ldaux, cur_stream());
  return {C, u};
}

bool gemm_bf16_supported_op(int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb, bool b_kn) {
  return sdml::gemm_bf16_supported((int)M, (int)N, (int)K, (int)lda, (int)ldb, (int)N, b_kn);
}

bool u8_fwd_head_supported_op(int64_t M, int64_t N, int64_t K, int64_t C) {
  return sdml::u8_fwd_head_supported((int)M, (int)N, (int)K, (int)K, nullptr, (int)C);
}

void sgd_momentum_(torch::Tensor p, torch::Tensor g, torch::Tensor buf, double lr, double momentum, double dampening,
                   double wd, bool nesterov, bool first, bool zero_grad, c10::optional<torch::Tensor> planes,
                   int64_t plane_offset, int64_t plane_rows, int64_t plane_k) {
  check_f32_cuda(p, "p");
  check_f32_cuda(g, "g");
  check_f32_cuda(buf, "buf");
  TORCH_CHECK(p.numel() == g.numel(), "sgd: p/g size mismatch");
  TORCH_CHECK(momentum == 0 || buf.numel() == p.numel(), "sgd: momentum buffer size mismatch");
  TORCH_CHECK(p.numel() % 4 == 0, "sgd: flat buffers must be padded to a multiple of 4");
  sdml::SgdPlanes pl;
  if (planes.has_value() && planes->defined()) {
    // planes [2][rows][Kp] int16 (fp16 bits, u8_planes.h) of the [rows][K] weight at float offset plane_offset
    TORCH_CHECK(planes->is_cuda() && planes->scalar_type() == torch::kInt16 && planes->is_contiguous() &&
                    planes->dim() == 3 && planes->size(0) == sdml::kU8FwdPlanes && planes->size(1) == plane_rows,
                "sgd planes: [u8_fwd_planes()][rows][Kp] int16 device tensor");
    const int64_t Kp = planes->size(2);
    TORCH_CHECK(plane_k % 4 == 0 && plane_offset % 4 == 0 && Kp % 4 == 0 && Kp >= plane_k &&
                    plane_offset + plane_rows * plane_k <= p.numel(),
                "sgd planes: K, offset and Kp must be multiples of 4 and the weight inside the buffer");
    pl.planes = reinterpret_cast<unsigned short*>(planes->data_ptr<int16_t>());
    pl.off4 = plane_offset / 4;
    pl.n4 = plane_rows * plane_k / 4;
    pl.K = plane_k;
    pl.Kp = Kp;
    pl.plane_stride = plane_rows * Kp;
  }
  sdml::sgd_momentum(p.data_ptr<float>(), g.data_ptr<float>(), buf.data_ptr<float>(), p.numel(), (float)lr,
                     (float)momentum, (float)dampening, (float)wd, nesterov, first, zero_grad, cur_stream(), pl);
}

void sgd_momentum_mixed_(torch::Tensor master, torch::Tensor p, torch::Tensor g, torch::Tensor buf, double lr,
                         double momentum, double dampening, double wd, bool nesterov, bool first, bool zero_grad) {
  check_f32_cuda(master, "master");
  check_f32_cuda(buf, "buf");
  TORCH_CHECK(p.is_cuda() && g.is_cuda() && p.scalar_type() == torch::kBFloat16 && g.scalar_type() == torch::kBFloat16,
              "sgd_mixed: p/g must be bf16 device tensors");
  TORCH_CHECK(p.is_contiguous() && g.is_contiguous(), "sgd_mixed: contiguous");
  TORCH_CHECK(p.numel() == master.numel() && g.numel() == master.numel() && p.numel() % 8 == 0,
              "sgd_mixed: sizes (a multiple of 8: the flat buffers pad every view to 64 elements)");
  TORCH_CHECK(momentum == 0 || buf.numel() == p.numel(), "sgd_mixed: momentum buffer size");
  auto al = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
  TORCH_CHECK(al(master.data_ptr()) && al(buf.data_ptr()) && al(p.data_ptr()) && al(g.data_ptr()),
              "sgd_mixed: 16-B alignment");
  sdml::sgd_momentum_mixed(master.data_ptr<float>(), p.data_ptr(), g.data_ptr(), buf.data_ptr<float>(), p.numel(),
                           (float)lr, (float)momentum, (float)dampening, (float)wd, nesterov, first, zero_grad,
                           cur_stream());
}

void synth_mnist(int64_t seed, int64_t start, int64_t n, int64_t H, int64_t W, int64_t mode, torch::Tensor x,
                 torch::Tensor y) {
  check_f32_cuda(x, "x");
  TORCH_CHECK(y.is_cuda() && y.scalar_type() == torch::kInt64 && y.is_contiguous(), "y: int64 device tensor");
  TORCH_CHECK(x.numel() == n * H * W && y.numel() == n, "synth_mnist: size mismatch");
  sdml::synth_mnist((uint64_t)seed, start, n, (int)H, (int)W, (int)mode, x.data_ptr<float>(), y.data_ptr<int64_t>(),
                    cur_stream());
}

void check_bf16_cuda(const torch::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a ROCm device tensor");
  TORCH_CHECK(t.scalar_type() == torch::kBFloat16, name, " must be bfloat16");
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}

// returns (row_loss fp32 [rows], row_correct fp32 [rows], dlogits bf16 or None)
std::tuple<torch::Tensor, torch::Tensor, c10::optional<torch::Tensor>> cross_entropy_bf16(
    torch::Tensor logits, torch::Tensor target, double scale, int64_t ignore_index, bool need_grad) {
  TORCH_CHECK(logits.is_cuda() && logits.scalar_type() == torch::kBFloat16, "logits must be a bf16 device tensor");
  TORCH_CHECK(logits.dim() == 2, "logits [rows, V]");
  // rows may be padded (row stride ld >= V, e.g. the lm_head's padded vocabulary): dlogits gets the same row stride,
  // its pad columns written as zeros by the kernel, and is returned as the [rows, V] view
  const int64_t rows = logits.size(0), V = logits.size(1);
  const int64_t ld = rows > 1 ? logits.stride(0) : V;
  TORCH_CHECK(logits.stride(1) == 1 && ld >= V, "logits rows must be contiguous (row stride >= V)");
  TORCH_CHECK(target.is_cuda() && target.scalar_type() == torch::kInt64 && target.is_contiguous(), "target int64");
  TORCH_CHECK(target.numel() == rows, "target size");
  auto f = logits.options().dtype(torch::kFloat32);
  auto loss = torch::empty({rows}, f), ok = torch::empty({rows}, f);
  c10::optional<torch::Tensor> g;
  if (need_grad) g = torch::empty({rows, ld}, logits.options()).narrow(1, 0, V);
  sdml::cross_entropy_bf16(logits.data_ptr(), target.data_ptr<int64_t>(), rows, V, ld, (float)scale, (int)ignore_index,
                           loss.data_ptr<float>(), ok.data_ptr<float>(), need_grad ? g->data_ptr() : nullptr,
                           cur_stream());
  return {loss, ok, g};
}

// returns (y, mean, rstd)
std::tuple<torch::Tensor, torch::Tensor, torch::Tensor> layernorm_fwd_bf16(torch::Tensor x, torch::Tensor w,
                                                                          torch::Tensor b, double eps) {
  check_bf16_cuda(x, "x");
  check_bf16_cuda(w, "w");
  check_bf16_cuda(b, "b");
  const int64_t D = x.size(-1), rows = x.numel() / D;
  TORCH_CHECK(D % 8 == 0 && D <= 4096 && w.numel() == D && b.numel() == D, "layernorm: D % 8 == 0, D <= 4096");
  auto y = torch::empty_like(x);
  auto f = x.options().dtype(torch::kFloat32);
  auto mean = torch::empty({rows}, f), rstd = torch::empty({rows}, f);
  sdml::layernorm_fwd_bf16(x.data_ptr(), w.data_ptr(), b.data_ptr(), y.data_ptr(), mean.data_ptr<float>(),
                           rstd.data_ptr<float>(), rows, D, (float)eps, cur_stream());
  return {y, mean, rstd};
}

// fused residual add + LayerNorm: xs = x + h (bf16, exactly the unfused add), y = LN(xs);
// returns (xs, y, mean, rstd)
std::tuple<torch::Tensor, torch::Tensor, torch::Tensor, torch::Tensor> add_layernorm_fwd_bf16(
    torch::Tensor x, torch::Tensor h, torch::Tensor w, torch::Tensor b, double eps) {
  check_bf16_cuda(x, "x");
  check_bf16_cuda(h, "h");
  check_bf16_cuda(w, "w");
  check_bf16_cuda(b, "b");
  TORCH_CHECK(x.sizes() == h.sizes(), "add_layernorm: x / h shape mismatch");
  const int64_t D = x.size(-1), rows = x.numel() / D;
  TORCH_CHECK(D % 8 == 0 && D <= 4096 && w.numel() == D && b.numel() == D, "layernorm: D % 8 == 0, D <= 4096");
  auto xs = torch::empty_like(x);
  auto y = torch::empty_like(x);
  auto f = x.options().dtype(torch::kFloat32);
  auto mean = torch::empty({rows}, f), rstd = torch::empty({rows}, f);
  sdml::layernorm_fwd_bf16(x.data_ptr(), w.data_ptr(), b.data_ptr(), y.data_ptr(), mean.data_ptr<float>(),
                           rstd.data_ptr<float>(), rows, D, (float)eps, cur_stream(), h.data_ptr(), xs.data_ptr());
  return {xs, y, mean, rstd};
}

// returns (dx bf16, dw fp32 [D], db fp32 [D])
std::tuple<torch::Tensor, torch::Tensor, torch::Tensor> layernorm_bwd_bf16(torch::Tensor x, torch::Tensor w,
                                                                          torch::Tensor gy, torch::Tensor mean,
                                                                          torch::Tensor rstd) {
  check_bf16_cuda(x, "x");
  check_bf16_cuda(w, "w");
  check_bf16_cuda(gy, "gy");
  check_f32_cuda(mean, "mean");
  check_f32_cuda(rstd, "rstd");
  const int64_t D = x.size(-1), rows = x.numel() / D;
  TORCH_CHECK(gy.sizes() == x.sizes() && mean.numel() == rows && rstd.numel() == rows && w.numel() == D, "ln bwd shapes");
  auto dx = torch::empty_like(x);
  auto f = x.options().dtype(torch::kFloat32);
  auto ws = torch::empty({(int64_t)sdml::layernorm_bwd_blocks(rows) * 2 * D}, f);
  auto dwdb = torch::zeros({2 * D}, f);
  sdml::layernorm_bwd_bf16(x.data_ptr(), w.data_ptr(), gy.data_ptr(), mean.data_ptr<float>(), rstd.data_ptr<float>(),
                           dx.data_ptr(), ws.data_ptr<float>(), dwdb.data_ptr<float>(), nullptr, rows, D,
                           cur_stream());
  return {dx, dwdb.narrow(0, 0, D), dwdb.narrow(0, D, D)};
}

// layernorm backward accumulating dw/db into bf16 parameter grads; returns dx
torch::Tensor layernorm_bwd_bf16_accum(torch::Tensor x, torch::Tensor w, torch::Tensor gy, torch::Tensor mean,
                                       torch::Tensor rstd, torch::Tensor gw, torch::Tensor gb,
                                       c10::optional<torch::Tensor> gadd) {
  check_bf16_cuda(x, "x");
  check_bf16_cuda(w, "w");
  check_bf16_cuda(gy, "gy");
  check_bf16_cuda(gw, "gw");
  check_bf16_cuda(gb, "gb");
  check_f32_cuda(mean, "mean");
  check_f32_cuda(rstd, "rstd");
  const int64_t D = x.size(-1), rows = x.numel() / D;
  TORCH_CHECK(gy.sizes() == x.sizes() && mean.numel() == rows && rstd.numel() == rows && w.numel() == D &&
                  gw.numel() == D && gb.numel() == D,
              "ln bwd shapes");
  const void* ga = nullptr;
  if (gadd.has_value() && gadd->defined()) {
    check_bf16_cuda(*gadd, "gadd");
    TORCH_CHECK(gadd->sizes() == x.sizes() && gadd->is_contiguous(), "ln bwd: gadd must match x (contiguous)");
    ga = gadd->data_ptr();
  }
  auto dx = torch::empty_like(x);
  auto ws = torch::empty({(int64_t)sdml::layernorm_bwd_blocks(rows) * 2 * D}, x.options().dtype(torch::kFloat32));
  sdml::layernorm_bwd_bf16_accum(x.data_ptr(), w.data_ptr(), gy.data_ptr(), mean.data_ptr<float>(),
                                 rstd.data_ptr<float>(), dx.data_ptr(), ws.data_ptr<float>(), gw.data_ptr(),
                                 gb.data_ptr(), rows, D, cur_stream(), ga);
  return dx;
}

// gb (bf16 [N]) += column sums of gy (bf16 [..., N], last dim contiguous)
void bias_grad_bf16_(torch::Tensor gy, torch::Tensor gb) {
  TORCH_CHECK(gy.is_cuda() && gy.scalar_type() == torch::kBFloat16 && gy.stride(-1) == 1,
              "bias_grad: gy must be a bf16 device tensor with a contiguous last dim");
  check_bf16_cuda(gb, "gb");
  const int64_t N = gy.size(-1);
  TORCH_CHECK(gb.numel() == N, "bias_grad: gb size");
  auto g2 = gy.reshape({-1, N});
  TORCH_CHECK(g2.stride(1) == 1, "bias_grad: rows must be addressable with one stride");
  const int64_t M = g2.size(0);
  if (M == 0) return;
  auto ws = torch::empty({(int64_t)sdml::bias_grad_blocks(M) * N}, gy.options().dtype(torch::kFloat32));
  sdml::bias_grad_bf16(g2.data_ptr(), (int)M, (int)N, (int)g2.stride(0), gb.data_ptr(), ws.data_ptr<float>(),
                       cur_stream());
}

// q, k, v: [B, S, H, 64] bf16 views sharing strides (d contiguous), e.g. slices of the fused
// qkv projection. Returns (out [B, S, H, 64] contiguous, lse fp32 [B*H*S]).
std::tuple<torch::Tensor, torch::Tensor> attention_fwd(torch::Tensor q, torch::Tensor k, torch::Tensor v, double scale,
                                                       bool causal) {
  TORCH_CHECK(q.is_cuda() && q.scalar_type() == torch::kBFloat16, "attention: bf16 device tensors");
  TORCH_CHECK(q.dim() == 4 && q.size(3) == 64 && q.stride(3) == 1, "attention: [B, S, H, 64] with contiguous d");
  TORCH_CHECK(k.sizes() == q.sizes() && v.sizes() == q.sizes() && k.strides() == q.strides() &&
                  v.strides() == q.strides(),
              "attention: q/k/v must share shape and strides");
  TORCH_CHECK(q.stride(2) % 8 == 0 && q.stride(1) % 8 == 0 && (reinterpret_cast<uintptr_t>(q.data_ptr()) & 15) == 0 &&
                  (reinterpret_cast<uintptr_t>(k.data_ptr()) & 15) == 0 &&
                  (reinterpret_cast<uintptr_t>(v.data_ptr()) & 15) == 0,
              "attention: 16-B aligned rows required");
  const int64_t B = q.size(0), S = q.size(1), H = q.size(2);
  auto out = torch::empty({B, S, H, 64}, q.options());
  auto lse = torch::empty({B * H * S}, q.options().dtype(torch::kFloat32));
  sdml::AttnShape a;
  a.q = q.data_ptr();
  a.k = k.data_ptr();
  a.v = v.data_ptr();
  a.out = out.data_ptr();
  a.lse = lse.data_ptr<float>();
  a.B = B;
  a.H = H;
  a.S = S;
  a.sqb = q.stride(0);
  a.sqs = q.stride(1);
  a.sqh = q.stride(2);
  a.sob = out.stride(0);
  a.sos = out.stride(1);
  a.soh = out.stride(2);
  a.scale = (float)scale;
  a.causal = causal ? 1 : 0;
  sdml::attention_fwd_bf16(a, cur_stream());
  return {out, lse};
}

// grads written into dqkv (same strides as q/k/v views of it: pass dq, dk, dv views)
void attention_bwd(torch::Tensor q, torch::Tensor k, torch::Tensor v, torch::Tensor out, torch::Tensor dout,
                   torch::Tensor lse, torch::Tensor dq, torch::Tensor dk, torch::Tensor dv, double scale, bool causal) {
  TORCH_CHECK(out.is_contiguous() && dout.is_contiguous() && out.sizes() == dout.sizes(), "attention bwd: out/dout");
  TORCH_CHECK(dq.strides() == q.strides() && dk.strides() == q.strides() && dv.strides() == q.strides(),
              "attention bwd: grads must use the q/k/v strides");
  const int64_t B = q.size(0), S = q.size(1), H = q.size(2);
  auto delta = torch::empty({B * H * S}, q.options().dtype(torch::kFloat32));
  sdml::AttnShape a;
  a.q = q.data_ptr();
  a.k = k.data_ptr();
  a.v = v.data_ptr();
  a.o = out.data_ptr();
  a.dout = dout.data_ptr();
  a.dq = dq.data_ptr();
  a.dk = dk.data_ptr();
  a.dv = dv.data_ptr();
  a.lse = lse.data_ptr<float>();
  a.delta = delta.data_ptr<float>();
  a.B = B;
  a.H = H;
  a.S = S;
  a.sqb = q.stride(0);
  a.sqs = q.stride(1);
  a.sqh = q.stride(2);
  a.sob = out.stride(0);
  a.sos = out.stride(1);
  a.soh = out.stride(2);
  a.scale = (float)scale;
  a.causal = causal ? 1 : 0;
  sdml::attention_bwd_bf16(a, cur_stream());
}


// ---- reference CNN ----------------------------------------------------------------------
void check_cnn_params(const torch::Tensor& w1, const torch::Tensor& b1, const torch::Tensor& w2,
                      const torch::Tensor& b2, int64_t n1, int64_t nb1, int64_t n2, int64_t nb2) {
  check_f32_cuda(w1, "w1");
  check_f32_cuda(b1, "b1");
  check_f32_cuda(w2, "w2");
  check_f32_cuda(b2, "b2");
  TORCH_CHECK(w1.numel() == n1 && b1.numel() == nb1 && w2.numel() == n2 && b2.numel() == nb2,
              "ref_cnn: parameter shapes do not match the reference CNN");
}

const long long* ctr_ptr(const c10::optional<torch::Tensor>& c) {
  if (!c.has_value() || !c->defined()) return nullptr;
  TORCH_CHECK(c->is_cuda() && c->scalar_type() == torch::kInt64 && c->numel() >= 1, "ctr must be an int64 device tensor");
  return reinterpret_cast<const long long*>(c->data_ptr<int64_t>());
}

// returns (out [B,320], z1 [B,1440] or None, idx [B,NIDX] uint8 or None); save = training
std::tuple<torch::Tensor, c10::optional<torch::Tensor>, c10::optional<torch::Tensor>> ref_cnn_stage0_fwd(
    torch::Tensor x, torch::Tensor w1, torch::Tensor b1, torch::Tensor w2, torch::Tensor b2, int64_t seed,
    c10::optional<torch::Tensor> ctr, int64_t sample0, double p, bool drop, bool save) {
  check_f32_cuda(x, "x");
  TORCH_CHECK(x.numel() % 784 == 0 && x.size(0) * 784 == x.numel(), "ref_cnn stage0: x must be [B,1,28,28]");
  check_cnn_params(w1, b1, w2, b2, 250, 10, 5000, 20);
  const int64_t B = x.size(0);
  auto out = torch::empty({B, 320}, x.options());
  c10::optional<torch::Tensor> z1, idx;
  if (save) {
    z1 = torch::empty({B, (int64_t)sdml::ref_cnn_z1_floats()}, x.options());
    idx = torch::empty({B, (int64_t)sdml::ref_cnn_idx_bytes()}, x.options().dtype(torch::kUInt8));
  }
  sdml::ref_cnn_stage0_fwd(x.data_ptr<float>(), w1.data_ptr<float>(), b1.data_ptr<float>(), w2.data_ptr<float>(),
                           b2.data_ptr<float>(), out.data_ptr<float>(), save ? z1->data_ptr<float>() : nullptr,
                           save ? idx->data_ptr<uint8_t>() : nullptr, (int)B, (unsigned long long)seed, ctr_ptr(ctr),
                           (unsigned)sample0, (float)p, drop, cur_stream());
  return {out, z1, idx};
}

void ref_cnn_stage0_bwd(torch::Tensor x, torch::Tensor w2, torch::Tensor out, torch::Tensor gout, torch::Tensor z1,
                        torch::Tensor idx, int64_t seed, c10::optional<torch::Tensor> ctr, int64_t sample0, double p,
                        bool drop, torch::Tensor gw1, torch::Tensor gb1, torch::Tensor gw2, torch::Tensor gb2) {
  check_f32_cuda(x, "x");
  check_f32_cuda(w2, "w2");
  check_f32_cuda(out, "out");
  check_f32_cuda(gout, "gout");
  check_f32_cuda(z1, "z1");
  const int64_t B = x.size(0);
  TORCH_CHECK(x.numel() == B * 784 && out.numel() == B * 320 && gout.numel() == B * 320 && w2.numel() == 5000 &&
                  z1.numel() == B * sdml::ref_cnn_z1_floats(),
              "ref_cnn stage0 bwd: shape mismatch");
  TORCH_CHECK(idx.is_cuda() && idx.scalar_type() == torch::kUInt8 && idx.is_contiguous() &&
                  idx.numel() == B * sdml::ref_cnn_idx_bytes(),
              "ref_cnn stage0 bwd: idx must be the forward's uint8 argmax tensor");
  check_cnn_params(gw1, gb1, gw2, gb2, 250, 10, 5000, 20);
  sdml::ref_cnn_stage0_bwd(x.data_ptr<float>(), w2.data_ptr<float>(), out.data_ptr<float>(), gout.data_ptr<float>(),
                           z1.data_ptr<float>(), idx.data_ptr<uint8_t>(), (int)B, (unsigned long long)seed,
                           ctr_ptr(ctr), (unsigned)sample0, (float)p, drop, gw1.data_ptr<float>(),
                           gb1.data_ptr<float>(), gw2.data_ptr<float>(), gb2.data_ptr<float>(), cur_stream());
}

// returns dx if grads are given (training), else None; loss/correct accumulate into stats[2]
c10::optional<torch::Tensor> ref_cnn_stage1(torch::Tensor x, torch::Tensor w1, torch::Tensor b1, torch::Tensor w2,
                                            torch::Tensor b2, torch::Tensor target, int64_t seed,
                                            c10::optional<torch::Tensor> ctr, int64_t sample0, double p, bool drop, double scale, torch::Tensor stats,
                                            c10::optional<torch::Tensor> gw1, c10::optional<torch::Tensor> gb1,
                                            c10::optional<torch::Tensor> gw2, c10::optional<torch::Tensor> gb2) {
  check_f32_cuda(x, "x");
  check_f32_cuda(stats, "stats");
  const int64_t B = x.size(0);
  TORCH_CHECK(x.dim() == 2 && x.size(1) == 320, "ref_cnn stage1: x must be [B,320]");
  TORCH_CHECK(target.is_cuda() && target.scalar_type() == torch::kInt64 && target.is_contiguous() &&
                  target.numel() == B,
              "ref_cnn stage1: target must be a contiguous int64 [B] device tensor");
  TORCH_CHECK(stats.numel() == 2, "stats must have 2 elements");
  check_cnn_params(w1, b1, w2, b2, 16000, 50, 500, 10);
  const bool train = opt_ptr(gw1) != nullptr;
  c10::optional<torch::Tensor> dx;
  if (train) {
    TORCH_CHECK(opt_ptr(gb1) && opt_ptr(gw2) && opt_ptr(gb2), "ref_cnn stage1: all four grads or none");
    check_cnn_params(*gw1, *gb1, *gw2, *gb2, 16000, 50, 500, 10);
    dx = torch::empty({B, 320}, x.options());
  }
  sdml::ref_cnn_stage1(x.data_ptr<float>(), w1.data_ptr<float>(), b1.data_ptr<float>(), w2.data_ptr<float>(),
                       b2.data_ptr<float>(), target.data_ptr<int64_t>(), (int)B, (unsigned long long)seed,
                       ctr_ptr(ctr), (unsigned)sample0, (float)p, drop, (float)scale, stats.data_ptr<float>(),
                       train ? dx->data_ptr<float>() : nullptr, opt_ptr(gw1), opt_ptr(gb1), opt_ptr(gw2), opt_ptr(gb2),
                       cur_stream());
  return dx;
}
}  // namespace

// ---- stream memory operations for the IPC transport (parallel/p2p.py IpcTransport): the command processor of the
// current stream writes / waits for a 32-bit word in device memory (this process's or a peer process's buffer opened
// through hipIPC), so a boundary hand-off between processes is ordered on the device, with no host round trip.
void stream_write_value32(int64_t ptr, int64_t value) {
  const hipError_t e = hipStreamWriteValue32(cur_stream(), reinterpret_cast<void*>(ptr), (uint32_t)value, 0);
  TORCH_CHECK(e == hipSuccess, "hipStreamWriteValue32: ", hipGetErrorString(e));
}
void stream_wait_value32(int64_t ptr, int64_t value) {
  const hipError_t e = hipStreamWaitValue32(cur_stream(), reinterpret_cast<void*>(ptr), (uint32_t)value,
                                            hipStreamWaitValueGte, 0xFFFFFFFFu);
  TORCH_CHECK(e == hipSuccess, "hipStreamWaitValue32: ", hipGetErrorString(e));
}

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "sdml gfx950 HIP kernels";
  m.def("linear_fwd_u8", &linear_fwd_u8, "act(scale * x_u8 @ w.T + b): uint8-pixel first layer", py::arg("x"),
        py::arg("w"), py::arg("b"), py::arg("relu"), py::arg("scale"), py::arg("planes") = py::none(),
        py::arg("planes_valid") = false, py::arg("mask_out") = py::none(), py::arg("wmax_out") = py::none());
  m.def("u8_fwd_wmax_slots", &sdml::u8_fwd_wmax_slots, "per-wave maxima linear_fwd_u8 writes into wmax_out (M, N)");
  m.def("linear_relu_head_u8", &linear_relu_head_u8,
        "uint8 first layer + classifier head in one launch (h stays on chip): dl, ReLU bits, head slab");
  m.def(
      "u8_set_stamps",
      [](c10::optional<torch::Tensor> buf) {
        if (!buf) return sdml::u8_set_stamps(nullptr);
        TORCH_CHECK(buf->is_cuda() && buf->scalar_type() == torch::kInt64 && buf->is_contiguous(),
                    "u8_set_stamps: contiguous int64 device tensor");
        return sdml::u8_set_stamps(buf->data_ptr());
      },
      "experiments builds: phase stamps of the fused uint8 forward + head (tools/probes/u8_fwd_stamps.py)");
  m.def("u8_stamp_slots", &sdml::u8_stamp_slots, "stamps per (block, wave) of u8_set_stamps");
  m.def(
      "u8_tr8_probe",
      [](torch::Tensor img, torch::Tensor addr) {
        TORCH_CHECK(img.is_cuda() && img.scalar_type() == torch::kUInt8 && img.is_contiguous() && img.numel() == 1024,
                    "u8_tr8_probe: img uint8 [1024]");
        TORCH_CHECK(addr.is_cuda() && addr.scalar_type() == torch::kInt32 && addr.is_contiguous() && addr.numel() == 64,
                    "u8_tr8_probe: addr int32 [64]");
        auto out = torch::empty({64, 2}, addr.options());
        sdml::u8_tr8_probe(img.data_ptr<uint8_t>(), addr.data_ptr<int>(), out.data_ptr<int>(), cur_stream());
        return out;
      },
      "test probe: the 8 bytes ds_read_b64_tr_b8 gives each lane of one wave (img in LDS, per-lane byte addresses)");
  m.def(
      "u8_set_wgrad_stamps",
      [](c10::optional<torch::Tensor> buf) {
        if (!buf) return sdml::u8_set_wgrad_stamps(nullptr);
        TORCH_CHECK(buf->is_cuda() && buf->scalar_type() == torch::kInt64 && buf->is_contiguous(),
                    "u8_set_wgrad_stamps: contiguous int64 device tensor");
        return sdml::u8_set_wgrad_stamps(buf->data_ptr());
      },
      "experiments builds: phase stamps of the uint8 weight gradient (tools/u8_wgrad_stamps.py)");
  m.def("u8_fwd_head_supported", &u8_fwd_head_supported_op, "shape check for linear_relu_head_u8 (M, N, K, C)");
  m.def("relu_bits", &relu_bits, "int32 [M, N/32] ReLU bits of y (the uint8 kernels' mask layout)");
  m.def("gemm_bf16", &gemm_bf16_op, "bf16 GEMM with fused bias / bias+GELU / GELU-backward epilogues",
        py::arg("A"), py::arg("B"), py::arg("bias") = py::none(), py::arg("b_kn") = false, py::arg("epi") = 0,
        py::arg("aux") = py::none());
  m.def("x2_split", &x2_split_op, "fp32 -> two fp16 planes of x * 2^(14 - E) (+ the dequantisation scale)",
        py::arg("x"), py::arg("amax"));
  m.def("x2_split_t", &x2_split_t_op, "planes of x^T (the input gradient's NT weight operand)", py::arg("x"),
        py::arg("amax"));
  m.def("x2_gemm", &x2_gemm_op, "fp32-accurate GEMM from fp16 planes (3 MFMA products) with fused epilogues",
        py::arg("A"), py::arg("sa"), py::arg("B"), py::arg("sb"), py::arg("b_kn") = false,
        py::arg("bias") = py::none(), py::arg("relu") = false, py::arg("mask") = py::none(),
        py::arg("want_wmax") = false);
  m.def("x2_gemm_supported", &x2_gemm_supported_op, "shape check for x2_gemm (M, N, K, b_kn)");
  m.def("x2_wgrad_", &x2_wgrad_, "gw += dz^T x, gb += colsum(dz) from fp16 planes (fp32-accurate)",
        py::arg("dz"), py::arg("sdz"), py::arg("x"), py::arg("sx"), py::arg("gw"), py::arg("gb") = py::none());
  m.def("gemm_bf16_supported", &gemm_bf16_supported_op, "shape check for gemm_bf16 (M, N, K, lda, ldb, b_kn)");
  m.def("ref_cnn_step", &ref_cnn_step_op, "reference CNN training step (both stages + SGD) in two launches",
        py::arg("x"), py::arg("target"), py::arg("params"), py::arg("bufs"), py::arg("seed0"), py::arg("seed1"),
        py::arg("ctr"), py::arg("p0"), py::arg("drop0"), py::arg("p1"), py::arg("drop1"), py::arg("scale"),
        py::arg("lr"), py::arg("mom"), py::arg("damp"), py::arg("wd"), py::arg("nesterov"), py::arg("first"),
        py::arg("stats"), py::arg("stamps") = py::none());
  m.def("mlp_small_step", &mlp_small_step, "784-128-10 MLP training step (fwd, loss, bwd, SGD) in one launch");
  m.def("mlp_small_step_max_batch", &sdml::mlp_small_step_max_batch);
  m.def("gelu_fwd_bf16", &gelu_fwd_bf16, "tanh-GELU forward (bf16)");
  m.def("gelu_bwd_bf16", &gelu_bwd_bf16, "tanh-GELU backward (bf16): gy * gelu'(x)", py::arg("gy"), py::arg("x"),
        py::arg("inplace") = false);
  m.def("embedding_fwd_bf16", &embedding_fwd_bf16, "token + position embedding (bf16)");
  m.def("embedding_bwd_bf16", &embedding_bwd_bf16, "deterministic embedding backward into bf16 grads",
        py::arg("g"), py::arg("sorted_tok"), py::arg("perm"), py::arg("gwte") = py::none(),
        py::arg("gwpe") = py::none());
  m.def("u8_fwd_kpad", [](int64_t K) { return (int64_t)sdml::u8_fwd_kpad((int)K); },
        "padded K of the uint8 forward's weight planes");
  m.def("u8_fwd_planes", []() { return (int64_t)sdml::kU8FwdPlanes; }, "number of the uint8 forward's weight planes");
  m.def("linear_wgrad_u8", &linear_wgrad_u8, "gw += scale * gz^T x_u8, gb += colsum(gz)", py::arg("x"), py::arg("gz"),
        py::arg("gw"), py::arg("gb"), py::arg("scale"), py::arg("amax") = py::none());
  m.def("linear_fwd_f32", &linear_fwd_f32, "relu?(x @ w.T + b) on fp32 MFMA", py::arg("x"), py::arg("w"),
        py::arg("b"), py::arg("relu"));
  m.def("linear_bwd_f32", &linear_bwd_f32, "backward of linear(+relu): accumulates gw/gb, returns dx",
        py::arg("x"), py::arg("y"), py::arg("gy"), py::arg("w"), py::arg("gw"), py::arg("gb"), py::arg("need_dx"),
        py::arg("relu_mask"), py::arg("mask_dx_by_x") = false);
  m.def("gemm_f32", &gemm_f32_op, "generic fp32 MFMA GEMM", py::arg("A"), py::arg("B"), py::arg("C"),
        py::arg("a_kmajor"), py::arg("b_kmajor"), py::arg("epi"), py::arg("splits") = 1,
        py::arg("bias") = py::none(), py::arg("rowsum") = py::none());
  m.def("head_logsoftmax_nll_f32", &head_logsoftmax_nll_f32, "fused fc + log_softmax + NLL (+ backward)",
        py::arg("x"), py::arg("w"), py::arg("b"), py::arg("target"), py::arg("gw"), py::arg("gb"), py::arg("scale"),
        py::arg("need_dx"), py::arg("stats_acc") = py::none(), py::arg("mask_dx") = false,
        py::arg("stats_init") = false);
  m.def("head_logsoftmax_nll_dl_f32", &head_logsoftmax_nll_dl_f32,
        "fused head returning the boundary gradient as its factor dl = scale * (softmax - onehot)", py::arg("x"),
        py::arg("w"), py::arg("b"), py::arg("target"), py::arg("gw"), py::arg("gb"), py::arg("scale"),
        py::arg("stats_acc"), py::arg("stats_init") = false, py::arg("defer_reduce") = false);
  py::class_<HeadPending, std::shared_ptr<HeadPending>>(m, "HeadPending")
      .def("run", &HeadPending::run, "launch the deferred head reduction now (once)")
      .def_property_readonly("pending", &HeadPending::pending);
  m.def("head_pool_supported", &sdml::head_pool_supported, "head_pool_xent shape support (M, P, K, C)");
  m.def("head_pool_xent", &head_pool_xent,
        "avg-pool + Linear + log_softmax + NLL + backward (ResNet head); returns dx, accumulates gw/gb/stats",
        py::arg("x"), py::arg("w"), py::arg("b"), py::arg("target"), py::arg("gw"), py::arg("gb"), py::arg("scale"),
        py::arg("stats"), py::arg("stats_init") = false);
  m.def("linear_wgrad_u8_dl", &linear_wgrad_u8_dl,
        "gw += scale * dz^T x_u8, gb += colsum(dz), dz = (dl @ w2) * (h > 0) (factored boundary gradient)",
        py::arg("x"), py::arg("dl"), py::arg("w2"), py::arg("h"), py::arg("gw"), py::arg("gb"), py::arg("scale"),
        py::arg("amax") = py::none(), py::arg("head") = nullptr, py::arg("sgd") = py::none(),
        py::arg("groups") = py::none());
  m.def("head_dx_from_dl", &head_dx_from_dl, "dx = (dl @ w) * (x > 0): boundary gradient from its factor",
        py::arg("dl"), py::arg("w"), py::arg("x"), py::arg("mask"));
  m.def("sgd_momentum_", &sgd_momentum_, "fused SGD with momentum over a flat buffer (optionally also writing a "
        "weight's fp16 plane cache)", py::arg("p"), py::arg("g"), py::arg("buf"), py::arg("lr"), py::arg("momentum"),
        py::arg("dampening"), py::arg("wd"), py::arg("nesterov"), py::arg("first"), py::arg("zero_grad") = false,
        py::arg("planes") = py::none(), py::arg("plane_offset") = 0, py::arg("plane_rows") = 0,
        py::arg("plane_k") = 0);
  m.def("sgd_momentum_mixed_", &sgd_momentum_mixed_, "SGD: fp32 master + momentum, bf16 grads/params");
  m.def("cross_entropy_bf16", &cross_entropy_bf16, "vocab cross-entropy on bf16 logits (+ dlogits)");
  m.def("layernorm_fwd_bf16", &layernorm_fwd_bf16, "LayerNorm forward (bf16, fp32 stats)");
  m.def("layernorm_bwd_bf16", &layernorm_bwd_bf16, "LayerNorm backward (bf16)");
  m.def("layernorm_bwd_bf16_accum", &layernorm_bwd_bf16_accum, "LayerNorm backward, dw/db added into bf16 grads",
        py::arg("x"), py::arg("w"), py::arg("gy"), py::arg("mean"), py::arg("rstd"), py::arg("gw"), py::arg("gb"),
        py::arg("gadd") = py::none());
  m.def("add_layernorm_fwd_bf16", &add_layernorm_fwd_bf16, "fused residual add + LayerNorm forward (bf16)");
  m.def("bias_grad_bf16_", &bias_grad_bf16_, "gb += column sums of gy (bf16, deterministic)");
  m.def("attention_fwd", &attention_fwd, "causal flash attention forward (bf16, d=64)");
  m.def("attention_bwd", &attention_bwd, "causal flash attention backward (bf16, d=64)");
  m.def("attention_set_fwd_kb", &sdml::attention_set_fwd_kb, "attention forward keys per tile (tuning)");
  m.def("gemm_f32x3", &gemm_f32x3_op, "fp32 GEMM via the bf16x3 split on bf16 MFMA", py::arg("A"), py::arg("B"),
        py::arg("C"), py::arg("a_kmajor"), py::arg("b_kmajor"), py::arg("epi") = 0, py::arg("bias") = py::none(),
        py::arg("rowsum") = py::none(), py::arg("amask") = py::none(), py::arg("cmask") = py::none());
  m.def("gemm_f32x3_set_variant", &sdml::gemm_f32x3_set_variant, "x3 engine accumulation variant (A/B)");
  m.def("wgrad_bf16_", &wgrad_bf16_, "gw += gy^T x, gb += colsum(gy) (bf16 Linear weight/bias gradient)",
        py::arg("gy"), py::arg("x"), py::arg("gw"), py::arg("gb") = py::none());
  m.def("wgrad_bf16_supported", &wgrad_bf16_supported_op, "shape check for wgrad_bf16_ (contiguous operands)");
  m.def("conv3x3_weight_bf16", &conv3x3_weight_bf16, "3x3 conv weight -> kernel layout (forward / dgrad)");
  m.def("conv3x3_weights_bf16", &conv3x3_weights_bf16, "3x3 conv weight -> (forward, dgrad) kernel layouts");
  m.def("transpose_batched_bf16", &transpose_batched_bf16,
        "dst[k] = src[k]^T for a list of contiguous 2-D bf16 matrices (R, C multiples of 8), one launch");
  m.def("conv3x3_weights_batched_bf16", &conv3x3_weights_batched_bf16,
        "several 3x3 conv weights -> their kernel layouts in caller-owned buffers, one launch");
  m.def("conv3x3_fwd_bf16", &conv3x3_fwd_bf16, "3x3 stride-1 pad-1 conv, channels-last bf16 (implicit GEMM)",
        py::arg("x"), py::arg("wt"), py::arg("add") = py::none(), py::arg("part") = py::none(),
        py::arg("bn_x") = py::none(), py::arg("bn_y") = py::none(), py::arg("bn_mean") = py::none(),
        py::arg("bn_rstd") = py::none(), py::arg("bn_gamma") = py::none(), py::arg("bn_beta") = py::none(),
        py::arg("bn_relu") = 0);
  m.def("conv_part_rows", &conv_part_rows, "rows of the BatchNorm partials a convolution epilogue writes");
  m.def("conv_dgrad_s2_part_rows", &conv_dgrad_s2_part_rows,
        "rows of the BatchNorm backward partials conv_dgrad_s2_bf16 writes", py::arg("N"), py::arg("H"), py::arg("W"),
        py::arg("ks"), py::arg("pad"));
  m.def("conv3x3_wgrad_bf16_", &conv3x3_wgrad_bf16_, "3x3 conv weight gradient, accumulated into bf16 grad");
  m.def("conv_fwd_bf16", &conv_fwd_bf16, "conv (3x3 pad 1 / 1x1, stride 1|2), channels-last bf16 (implicit GEMM)",
        py::arg("x"), py::arg("wt"), py::arg("ks"), py::arg("stride"), py::arg("pad"), py::arg("add") = py::none(),
        py::arg("part") = py::none());
  m.def("conv_dgrad_s2_bf16", &conv_dgrad_s2_bf16, "input gradient of a stride-2 conv (3x3 pad 1 / 1x1), parity-class GEMMs",
        py::arg("dy"), py::arg("w"), py::arg("H"), py::arg("W"), py::arg("pad"), py::arg("add") = py::none(),
        py::arg("part") = py::none(), py::arg("bn_x") = py::none(), py::arg("bn_y") = py::none(),
        py::arg("bn_mean") = py::none(), py::arg("bn_rstd") = py::none(), py::arg("bn_gamma") = py::none(),
        py::arg("bn_beta") = py::none(), py::arg("bn_relu") = 0);
  m.def("conv_wgrad_bf16_", &conv_wgrad_bf16_, "conv weight gradient (3x3 / 1x1, stride 1|2), accumulated");
  m.def("conv_c1_fwd_bf16", &conv_c1_fwd_bf16, "stem 3x3 conv with one input channel -> channels-last bf16");
  m.def("conv_c1_wgrad_bf16_", &conv_c1_wgrad_bf16_, "stem conv weight gradient, accumulated into bf16 grad");
  m.def("bn_nhwc_fwd", &bn_nhwc_fwd, "training BatchNorm (+residual)(+ReLU), channels-last bf16", py::arg("x"),
        py::arg("res"), py::arg("gamma"), py::arg("beta"), py::arg("rmean"), py::arg("rvar"), py::arg("eps"),
        py::arg("momentum"), py::arg("relu"), py::arg("num_batches_tracked") = py::none(), py::arg("part") = py::none());
  m.def("bn_nhwc_bwd", &bn_nhwc_bwd, "BatchNorm (+residual)(+ReLU) backward, channels-last bf16", py::arg("x"),
        py::arg("dy"), py::arg("y"), py::arg("mean"), py::arg("rstd"), py::arg("gamma"), py::arg("relu"),
        py::arg("need_dres"), py::arg("ggamma"), py::arg("gbeta"), py::arg("beta") = py::none(),
        py::arg("part") = py::none(), py::arg("part_rows") = 0);
  m.def("bn_nhwc_eval", &bn_nhwc_eval, "BatchNorm with running statistics (+residual)(+ReLU)");
  m.def("set_knob", [](const std::string& name, int value) {
          TORCH_CHECK(sdml::set_knob(name.c_str(), value), "unknown kernel knob, or a timing probe that only ",
                      "SDML_KERNEL_EXPERIMENTS builds accept: ", name);
        }, "set a kernel-variant switch (csrc/kernels/knobs.h)", py::arg("name"), py::arg("value"));
  m.def("reset_knobs", &sdml::reset_knobs, "every kernel-variant switch back to its default");
  m.def("kernel_experiments_build", &sdml::kernel_experiments_build,
        "whether timing-probe switches are live (SDML_KERNEL_EXPERIMENTS build)");
  m.def("gemm_f32_set_mode", &sdml::gemm_f32_set_mode, "fp32 GEMM engine: 1 = bf16x3 split (default), 0 = fp32 MFMA");
  m.def("gemm_f32_mode", &sdml::gemm_f32_mode, "current fp32 GEMM engine");
  m.def("gemm_f32_set_variant", &sdml::gemm_f32_set_variant, "fp32 GEMM variant (tuning: 0 auto, 16, 32)");
  m.def("ref_cnn_stage0_fwd", &ref_cnn_stage0_fwd, "reference CNN stage 0 forward (one launch)");
  m.def("ref_cnn_stage0_bwd", &ref_cnn_stage0_bwd, "reference CNN stage 0 backward (one launch)");
  m.def("ref_cnn_stage1", &ref_cnn_stage1, "reference CNN stage 1 forward+loss+backward (one launch)");
  m.def("synth_mnist", &synth_mnist, "on-device synthetic MNIST-shape data");
  m.def("stream_write_value32", &stream_write_value32, "current stream: *ptr = value (uint32) after prior work");
  m.def("stream_wait_value32", &stream_wait_value32, "current stream: later work waits until *ptr >= value (uint32)");
}

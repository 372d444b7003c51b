// Python bindings for the fused NHWC BatchNorm(+residual)(+ReLU) kernels (csrc/kernels/bn.hip).
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>

#include <cstdlib>

#include <stdexcept>
#include <string>

extern "C" {
int dtfk_bn_partial_rows(int M, int C);
hipError_t dtfk_bn_fwd(const void* x, const void* res, const float* gamma, const float* beta, void* y, float* part,
                       float* mean, float* invstd, float* scale, float* shift, float* run_mean, float* run_var,
                       int M, int C, float momentum, float eps, int relu, hipStream_t st);
hipError_t dtfk_bn_apply(const void* x, const void* res, const float* scale, const float* shift, void* y, int M, int C,
                         int relu, hipStream_t st);
hipError_t dtfk_bn_bwd(const void* dy, const void* x, const void* res, const float* gamma, const float* mean,
                       const float* invstd, const float* scale, const float* shift, float* part, float* coef,
                       void* dx, void* dres, float* dgamma, float* dbeta, int M, int C, int relu, int accum,
                       int write_g, hipStream_t st);
hipError_t dtfk_strided_add(void* full, const void* comp, int N, int H, int W, int C, int Ho, int Wo, int s,
                            hipStream_t st);
hipError_t dtfk_maxpool_fwd(const void* x, void* y, void* idx, int N, int H, int W, int C, int Ho, int Wo, int k,
                            int s, int p, hipStream_t st);
hipError_t dtfk_maxpool_bwd(const void* dy, const void* idx, void* dx, int N, int H, int W, int C, int Ho, int Wo,
                            int k, int s, int p, hipStream_t st);
int dtfk_conv3x3_supported(int N, int H, int W, int C, int K, int stride);
hipError_t dtfk_conv3x3_fwd(const void* x, const void* w, void* y, float* part, int N, int H, int W, int C, int K,
                            int stride, int bn, hipStream_t stream);
long long dtfk_conv3x3_tiles(int N, int H, int W, int stride);
hipError_t dtfk_conv3x3_wflip(const void* w, void* wt, int K, int C, hipStream_t stream);
hipError_t dtfk_conv3x3_wgrad(const void* dy, const void* x, float* dw, float* ws, int N, int H, int W, int C, int K,
                              int stride, int kcrs, hipStream_t stream);
long long dtfk_conv3x3_wgrad_plan(int N, int H, int W, int C, int K, int stride, int* splits_out, int* sps_out);
int dtfk_conv_supported(int N, int H, int W, int C, int K, int stride, int ks);
hipError_t dtfk_conv_fwd(const void* x, const void* w, void* y, float* part, int N, int H, int W, int C, int K,
                         int stride, int bn, int ks, int accum, const void* bnx, const float* bnst,
                         const void* bnres, hipStream_t stream);
hipError_t dtfk_bn_bwd_parts(const void* g, const void* x, const float* gamma, const float* mean, const float* invstd,
                             const float* part, int P, float* coef, void* dx, float* dgamma, float* dbeta, int M, int C,
                             int accum, hipStream_t st);
long long dtfk_conv_tiles(int N, int H, int W, int stride, int ks);
hipError_t dtfk_conv_wflip(const void* w, void* wt, int K, int C, int ks, hipStream_t stream);
hipError_t dtfk_conv_wflip_multi(const long long* tab, const int* tiles, int ntiles, hipStream_t stream);
long long dtfk_conv_wgrad_plan(int N, int H, int W, int C, int K, int stride, int ks, int* splits_out, int* sps_out);
hipError_t dtfk_conv_wgrad(const void* dy, const void* x, float* dw, float* ws, int N, int H, int W, int C, int K,
                           int stride, int ks, int kcrs, hipStream_t stream);
hipError_t dtfk_bn_stat_partials(const void* x, float* part, int M, int C, hipStream_t st);
hipError_t dtfk_bn_fwd_parts(const void* x, const void* res, const float* gamma, const float* beta, void* y,
                             const float* part, int P, float* mean, float* invstd, float* scale, float* shift,
                             float* run_mean, float* run_var, int M, int C, float momentum, float eps, int relu,
                             hipStream_t st);
}

namespace dtf {
namespace {
hipStream_t cs() { return c10::hip::getCurrentHIPStream().stream(); }
void ck(hipError_t e, const char* w) {
  if (e != hipSuccess) throw std::runtime_error(std::string(w) + ": " + hipGetErrorString(e));
}
// NHWC bf16 activation viewed as [M, C]: channels_last 4-D or plain 2-D row-major
int64_t rows_of(const at::Tensor& t, int64_t C) {
  if (!t.is_cuda() || t.scalar_type() != at::kBFloat16) throw std::runtime_error("bn: bf16 GPU activations");
  const bool ok = t.dim() == 4 ? (t.size(1) == C && t.is_contiguous(at::MemoryFormat::ChannelsLast))
                               : (t.dim() == 2 && t.size(1) == C && t.is_contiguous());
  if (!ok) throw std::runtime_error("bn: activation must be channels_last NCHW (or [M, C]) with C channels");
  return t.numel() / C;
}
void f32(const at::Tensor& t, int64_t n, const char* w) {
  if (!t.is_cuda() || t.scalar_type() != at::kFloat || !t.is_contiguous() || t.numel() < n)
    throw std::runtime_error(std::string("bn: ") + w + " must be a contiguous fp32 GPU tensor");
}
float* optf(const c10::optional<at::Tensor>& t) { return t.has_value() ? t->data_ptr<float>() : nullptr; }
}  // namespace

// ---- NHWC bf16 max pooling (kernels/pool.hip); idx: uint8 window position of each output's max
static void pool_check(const at::Tensor& t, const char* w) {
  if (!t.is_cuda() || t.scalar_type() != at::kBFloat16 || t.dim() != 4 ||
      !t.is_contiguous(at::MemoryFormat::ChannelsLast) || t.size(1) % 8)
    throw std::runtime_error(std::string("maxpool: ") + w + " must be channels_last bf16 [N, C % 8 == 0, H, W]");
}

void maxpool_fwd(at::Tensor x, at::Tensor y, at::Tensor idx, int64_t k, int64_t s, int64_t p) {
  pool_check(x, "x");
  pool_check(y, "y");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3), Ho = y.size(2), Wo = y.size(3);
  if (y.size(0) != N || y.size(1) != C || Ho != (H + 2 * p - k) / s + 1 || Wo != (W + 2 * p - k) / s + 1)
    throw std::runtime_error("maxpool_fwd: output shape");
  if (k < 1 || k * k > 255 || s < 1 || p < 0 || 2 * p > k) throw std::runtime_error("maxpool_fwd: window");
  if (!idx.is_cuda() || idx.scalar_type() != at::kByte || idx.numel() != y.numel())
    throw std::runtime_error("maxpool_fwd: idx must be a uint8 GPU tensor like y");
  ck(dtfk_maxpool_fwd(x.data_ptr(), y.data_ptr(), idx.data_ptr(), (int)N, (int)H, (int)W, (int)C, (int)Ho, (int)Wo,
                      (int)k, (int)s, (int)p, cs()),
     "maxpool_fwd");
}

void maxpool_bwd(at::Tensor dy, at::Tensor idx, at::Tensor dx, int64_t k, int64_t s, int64_t p) {
  pool_check(dy, "dy");
  pool_check(dx, "dx");
  const int64_t N = dx.size(0), C = dx.size(1), H = dx.size(2), W = dx.size(3), Ho = dy.size(2), Wo = dy.size(3);
  if (dy.size(0) != N || dy.size(1) != C || Ho != (H + 2 * p - k) / s + 1 || Wo != (W + 2 * p - k) / s + 1)
    throw std::runtime_error("maxpool_bwd: shapes");
  if (!idx.is_cuda() || idx.scalar_type() != at::kByte || idx.numel() != dy.numel())
    throw std::runtime_error("maxpool_bwd: idx must be a uint8 GPU tensor like dy");
  ck(dtfk_maxpool_bwd(dy.data_ptr(), idx.data_ptr(), dx.data_ptr(), (int)N, (int)H, (int)W, (int)C, (int)Ho, (int)Wo,
                      (int)k, (int)s, (int)p, cs()),
     "maxpool_bwd");
}

int64_t bn_partial_rows(int64_t M, int64_t C) { return dtfk_bn_partial_rows((int)M, (int)C); }

void bn_fwd(at::Tensor x, c10::optional<at::Tensor> res, at::Tensor gamma, at::Tensor beta, at::Tensor y,
            at::Tensor part, at::Tensor stats, c10::optional<at::Tensor> run_mean, c10::optional<at::Tensor> run_var,
            double momentum, double eps, bool relu) {
  const int64_t C = gamma.numel();
  const int64_t M = rows_of(x, C);
  if (rows_of(y, C) != M) throw std::runtime_error("bn_fwd: y shape");
  if (res.has_value() && rows_of(*res, C) != M) throw std::runtime_error("bn_fwd: residual shape");
  f32(gamma, C, "gamma"); f32(beta, C, "beta"); f32(stats, 4 * C, "stats");
  f32(part, 2 * (int64_t)dtfk_bn_partial_rows((int)M, (int)C) * C, "part");
  float* s = stats.data_ptr<float>();
  ck(dtfk_bn_fwd(x.data_ptr(), res.has_value() ? res->data_ptr() : nullptr, gamma.data_ptr<float>(),
                 beta.data_ptr<float>(), y.data_ptr(), part.data_ptr<float>(), s, s + C, s + 2 * C, s + 3 * C,
                 optf(run_mean), optf(run_var), (int)M, (int)C, (float)momentum, (float)eps, relu ? 1 : 0, cs()),
     "bn_fwd");
}

// bn_fwd with the statistics partials [2, P, C] supplied by the producer of x
void bn_fwd_parts(at::Tensor x, c10::optional<at::Tensor> res, at::Tensor gamma, at::Tensor beta, at::Tensor y,
                  at::Tensor part, int64_t P, at::Tensor stats, c10::optional<at::Tensor> run_mean,
                  c10::optional<at::Tensor> run_var, double momentum, double eps, bool relu) {
  const int64_t C = gamma.numel();
  const int64_t M = rows_of(x, C);
  if (rows_of(y, C) != M) throw std::runtime_error("bn_fwd_parts: y shape");
  if (res.has_value() && rows_of(*res, C) != M) throw std::runtime_error("bn_fwd_parts: residual shape");
  f32(gamma, C, "gamma"); f32(beta, C, "beta"); f32(stats, 4 * C, "stats"); f32(part, 2 * P * C, "part");
  float* s = stats.data_ptr<float>();
  ck(dtfk_bn_fwd_parts(x.data_ptr(), res.has_value() ? res->data_ptr() : nullptr, gamma.data_ptr<float>(),
                       beta.data_ptr<float>(), y.data_ptr(), part.data_ptr<float>(), (int)P, s, s + C, s + 2 * C,
                       s + 3 * C, optf(run_mean), optf(run_var), (int)M, (int)C, (float)momentum, (float)eps,
                       relu ? 1 : 0, cs()),
     "bn_fwd_parts");
}

void bn_apply(at::Tensor x, c10::optional<at::Tensor> res, at::Tensor scale, at::Tensor shift, at::Tensor y,
              bool relu) {
  const int64_t C = scale.numel();
  const int64_t M = rows_of(x, C);
  ck(dtfk_bn_apply(x.data_ptr(), res.has_value() ? res->data_ptr() : nullptr, scale.data_ptr<float>(),
                   shift.data_ptr<float>(), y.data_ptr(), (int)M, (int)C, relu ? 1 : 0, cs()),
     "bn_apply");
}

void bn_bwd(at::Tensor dy, at::Tensor x, c10::optional<at::Tensor> res, at::Tensor gamma, at::Tensor stats,
            at::Tensor part, at::Tensor coef, at::Tensor dx, c10::optional<at::Tensor> dres, at::Tensor dgamma,
            at::Tensor dbeta, bool relu, bool accum) {
  const int64_t C = gamma.numel();
  const int64_t M = rows_of(x, C);
  if (rows_of(dy, C) != M || rows_of(dx, C) != M) throw std::runtime_error("bn_bwd: shapes");
  if (res.has_value() != dres.has_value()) throw std::runtime_error("bn_bwd: res and dres go together");
  f32(stats, 4 * C, "stats"); f32(coef, 3 * C, "coef"); f32(dgamma, C, "dgamma"); f32(dbeta, C, "dbeta");
  f32(part, 2 * (int64_t)dtfk_bn_partial_rows((int)M, (int)C) * C, "part");
  const float* s = stats.data_ptr<float>();
  // residual + ReLU blocks: the partials pass stores g = dres and the apply pass reads
  // (g, x) -- one tensor pass fewer (DTF_BN_WRITE_G=0: recompute g from dy, x, res twice)
  static const bool write_g = [] {
    const char* e = getenv("DTF_BN_WRITE_G");
    return e == nullptr || e[0] != '0';
  }();
  ck(dtfk_bn_bwd(dy.data_ptr(), x.data_ptr(), res.has_value() ? res->data_ptr() : nullptr, gamma.data_ptr<float>(),
                 s, s + C, s + 2 * C, s + 3 * C, part.data_ptr<float>(), coef.data_ptr<float>(), dx.data_ptr(),
                 dres.has_value() ? dres->data_ptr() : nullptr, dgamma.data_ptr<float>(), dbeta.data_ptr<float>(),
                 (int)M, (int)C, relu ? 1 : 0, accum ? 1 : 0, write_g ? 1 : 0, cs()),
     "bn_bwd");
}

// full[:, :, s*i, s*j] += comp (channels_last bf16 [N, C, H, W] and [N, C, Ho, Wo])
void strided_add(at::Tensor full, at::Tensor comp, int64_t s) {
  for (const at::Tensor* t : {&full, &comp})
    if (!t->is_cuda() || t->scalar_type() != at::kBFloat16 || t->dim() != 4 ||
        !t->is_contiguous(at::MemoryFormat::ChannelsLast))
      throw std::runtime_error("strided_add: channels_last bf16 4-D CUDA tensors");
  if (full.size(0) != comp.size(0) || full.size(1) != comp.size(1)) throw std::runtime_error("strided_add: N / C differ");
  ck(dtfk_strided_add(full.data_ptr(), comp.data_ptr(), (int)full.size(0), (int)full.size(2), (int)full.size(3),
                      (int)full.size(1), (int)comp.size(2), (int)comp.size(3), (int)s, cs()),
     "strided_add");
}

// 3x3 (pad 1) or 1x1 (pad 0), stride 1 or 2 convolution on channels_last bf16
// tensors as an in-tree implicit GEMM (csrc/kernels/conv_igemm.hip; the filter
// size comes from w); `part` [2, P, K] fp32 receives the BatchNorm statistics
// partials of y (P = conv3x3_tiles).
static void cl_bf16(const at::Tensor& t, const char* what) {
  if (!t.is_cuda() || t.scalar_type() != at::kBFloat16 || t.dim() != 4 || !t.is_contiguous(at::MemoryFormat::ChannelsLast))
    throw std::runtime_error(std::string(what) + ": channels_last bf16 4-D CUDA tensor expected");
}
static int ksize(const at::Tensor& w) {
  if (w.dim() != 4 || w.size(2) != w.size(3) || (w.size(2) != 1 && w.size(2) != 3)) return 0;
  return (int)w.size(2);
}

bool conv3x3_supported(at::Tensor x, at::Tensor w, int64_t stride) {
  const int ks = ksize(w);
  if (x.dim() != 4 || ks == 0 || w.size(1) != x.size(1)) return false;
  return dtfk_conv_supported((int)x.size(0), (int)x.size(2), (int)x.size(3), (int)x.size(1), (int)w.size(0),
                             (int)stride, ks) != 0;
}

int64_t conv3x3_tiles(int64_t N, int64_t H, int64_t W, int64_t stride) {
  return dtfk_conv_tiles((int)N, (int)H, (int)W, (int)stride, 3);   // same rows for 1x1 / pad 0
}

// bn_x / bn_stats (EPI 2): y is the output gradient of a BatchNorm(+ReLU) whose
// input was bn_x ([N, K, Ho, Wo]) with statistics bn_stats [4, K] -- y is stored as
// the ReLU-masked g and part receives the BN backward's [2, P, K] partials.
// bn_res (EPI 3, with accumulate): that BN also added a residual (mask from
// bn_x * scale + shift + bn_res) and y already holds the residual branch's
// gradient, so g is formed from y + the convolution.
void conv3x3_fwd(at::Tensor x, at::Tensor w, at::Tensor y, c10::optional<at::Tensor> part, int64_t stride,
                 int64_t bn, bool accumulate, c10::optional<at::Tensor> bn_x, c10::optional<at::Tensor> bn_stats,
                 c10::optional<at::Tensor> bn_res) {
  cl_bf16(x, "conv_fwd x");
  cl_bf16(w, "conv_fwd w");
  cl_bf16(y, "conv_fwd y");
  const int ks = ksize(w);
  const int N = (int)x.size(0), C = (int)x.size(1), H = (int)x.size(2), W = (int)x.size(3), K = (int)w.size(0);
  const int Ho = (H - 1) / (int)stride + 1, Wo = (W - 1) / (int)stride + 1;
  if (ks == 0 || w.size(1) != C || y.size(0) != N || y.size(1) != K || y.size(2) != Ho || y.size(3) != Wo)
    throw std::runtime_error("conv_fwd: shapes");
  float* pp = nullptr;
  if (part.has_value()) {
    const int64_t P = dtfk_conv_tiles(N, H, W, (int)stride, ks);
    if (!part->is_cuda() || part->scalar_type() != at::kFloat || !part->is_contiguous() || part->numel() < 2 * P * K)
      throw std::runtime_error("conv_fwd: part must hold [2, P, K] fp32");
    pp = part->data_ptr<float>();
  }
  const void* bx = nullptr;
  const void* br = nullptr;
  const float* bst = nullptr;
  if (bn_x.has_value()) {
    cl_bf16(*bn_x, "conv_fwd bn_x");
    if (!bn_stats.has_value() || pp == nullptr || accumulate != bn_res.has_value() || bn_x->sizes() != y.sizes())
      throw std::runtime_error("conv_fwd: bn_x needs bn_stats, part, y's shape, and accumulate iff bn_res");
    f32(*bn_stats, 4LL * K, "bn_stats");
    bx = bn_x->data_ptr();
    bst = bn_stats->data_ptr<float>();
    if (bn_res.has_value()) {
      cl_bf16(*bn_res, "conv_fwd bn_res");
      if (bn_res->sizes() != y.sizes()) throw std::runtime_error("conv_fwd: bn_res must have y's shape");
      br = bn_res->data_ptr();
    }
  } else if (bn_res.has_value()) {
    throw std::runtime_error("conv_fwd: bn_res needs bn_x");
  }
  ck(dtfk_conv_fwd(x.data_ptr(), w.data_ptr(), y.data_ptr(), pp, N, H, W, C, K, (int)stride, (int)bn, ks,
                   accumulate ? 1 : 0, bx, bst, br, cs()),
     "conv_fwd");
}

// wt [C, K, ks, ks] channels_last = the flipped, transposed filter of the stride-1 input gradient
void conv3x3_wflip(at::Tensor w, at::Tensor wt) {
  cl_bf16(w, "conv_wflip w");
  cl_bf16(wt, "conv_wflip wt");
  const int ks = ksize(w);
  if (ks == 0 || wt.size(0) != w.size(1) || wt.size(1) != w.size(0) || wt.size(2) != ks || wt.size(3) != ks)
    throw std::runtime_error("conv_wflip: shapes");
  ck(dtfk_conv_wflip(w.data_ptr(), wt.data_ptr(), (int)w.size(0), (int)w.size(1), ks, cs()), "conv_wflip");
}

// Several filters flipped in one launch.  tab: int64 [n, 5] rows {w, wt, K, C, ks}
// (device pointers of channels_last bf16 filters, checked by the caller:
// ops/conv.py _flipped), tiles: int32 [m, 4] (row, tap, k0, c0) per 64 x 64
// tile, both on the device.
void conv_wflip_multi(at::Tensor tab, at::Tensor tiles) {
  if (!tab.is_cuda() || tab.scalar_type() != at::kLong || tab.dim() != 2 || tab.size(1) != 5 || !tab.is_contiguous() ||
      !tiles.is_cuda() || tiles.scalar_type() != at::kInt || tiles.dim() != 2 || tiles.size(1) != 4 ||
      !tiles.is_contiguous())
    throw std::runtime_error("conv_wflip_multi: tab int64 [n, 5], tiles int32 [m, 4] on the device");
  ck(dtfk_conv_wflip_multi(reinterpret_cast<const long long*>(tab.data_ptr<int64_t>()), tiles.data_ptr<int>(),
                           (int)tiles.size(0), cs()),
     "conv_wflip_multi");
}

// dw (fp32 [K, C, ks, ks], channels_last or contiguous) += the weight gradient of
// y = conv(x, w, stride) for y's gradient dy
void conv3x3_wgrad(at::Tensor dy, at::Tensor x, at::Tensor dw, int64_t stride) {
  cl_bf16(dy, "conv_wgrad dy");
  cl_bf16(x, "conv_wgrad x");
  if (!dw.is_cuda() || dw.scalar_type() != at::kFloat || dw.dim() != 4 || dw.size(2) != dw.size(3) ||
      (dw.size(2) != 3 && dw.size(2) != 1))
    throw std::runtime_error("conv_wgrad: dw must be an fp32 [K, C, ks, ks] CUDA tensor, ks 1 or 3");
  const int ks = (int)dw.size(2);
  int kcrs;
  if (dw.is_contiguous()) kcrs = 1;
  else if (dw.is_contiguous(at::MemoryFormat::ChannelsLast)) kcrs = 0;
  else throw std::runtime_error("conv_wgrad: dw must be contiguous or channels_last");
  const int N = (int)x.size(0), C = (int)x.size(1), H = (int)x.size(2), W = (int)x.size(3), K = (int)dy.size(1);
  const int Ho = (H - 1) / (int)stride + 1, Wo = (W - 1) / (int)stride + 1;
  if (dw.size(0) != K || dw.size(1) != C || dy.size(0) != N || dy.size(2) != Ho || dy.size(3) != Wo)
    throw std::runtime_error("conv_wgrad: shapes");
  // split slabs from the caching allocator (freed back to it on return; the
  // stream-ordered reuse is safe)
  const long long wsn = dtfk_conv_wgrad_plan(N, H, W, C, K, (int)stride, ks, nullptr, nullptr);
  at::Tensor ws;
  if (wsn > 0) ws = at::empty({wsn}, dw.options());
  ck(dtfk_conv_wgrad(dy.data_ptr(), x.data_ptr(), dw.data_ptr<float>(), wsn > 0 ? ws.data_ptr<float>() : nullptr, N,
                     H, W, C, K, (int)stride, ks, kcrs, cs()),
     "conv_wgrad");
}

// BatchNorm backward when its output gradient arrived already ReLU-masked as g
// together with the [2, P, C] partials (sum g, sum g x_hat) -- written by the
// producing convolution's epilogue (conv3x3_fwd bn_x): finalize + apply only.
void bn_bwd_parts(at::Tensor g, at::Tensor x, at::Tensor gamma, at::Tensor stats, at::Tensor part, int64_t P,
                  at::Tensor coef, at::Tensor dx, at::Tensor dgamma, at::Tensor dbeta, bool accum) {
  const int64_t C = gamma.numel();
  const int64_t M = rows_of(x, C);
  if (rows_of(g, C) != M || rows_of(dx, C) != M) throw std::runtime_error("bn_bwd_parts: shapes");
  f32(stats, 4 * C, "stats"); f32(coef, 3 * C, "coef"); f32(dgamma, C, "dgamma"); f32(dbeta, C, "dbeta");
  f32(part, 2 * P * C, "part");
  const float* s = stats.data_ptr<float>();
  ck(dtfk_bn_bwd_parts(g.data_ptr(), x.data_ptr(), gamma.data_ptr<float>(), s, s + C, part.data_ptr<float>(), (int)P,
                       coef.data_ptr<float>(), dx.data_ptr(), dgamma.data_ptr<float>(), dbeta.data_ptr<float>(),
                       (int)M, (int)C, accum ? 1 : 0, cs()),
     "bn_bwd_parts");
}

// BatchNorm statistics partials of x alone ([2, P, C], P = bn_partial_rows(M, C));
// returns P.  The convolution engine choice prices a conv without a statistics
// epilogue with this pass (ops/conv.py).
int64_t bn_stat_partials(at::Tensor x, at::Tensor part) {
  const int64_t C = x.dim() == 4 ? x.size(1) : x.size(1);
  const int64_t M = rows_of(x, C);
  const int P = dtfk_bn_partial_rows((int)M, (int)C);
  f32(part, 2LL * P * C, "part");
  ck(dtfk_bn_stat_partials(x.data_ptr(), part.data_ptr<float>(), (int)M, (int)C, cs()), "bn_stat_partials");
  return P;
}

void init_bn(pybind11::module& m) {
  m.def("bn_stat_partials", &bn_stat_partials);
  m.def("bn_bwd_parts", &bn_bwd_parts);
  m.def("conv3x3_wgrad", &conv3x3_wgrad);
  m.def("bn_fwd_parts", &bn_fwd_parts);
  m.def("conv3x3_supported", &conv3x3_supported);
  m.def("conv3x3_tiles", &conv3x3_tiles);
  m.def("conv3x3_fwd", &conv3x3_fwd, py::arg("x"), py::arg("w"), py::arg("y"), py::arg("part") = py::none(),
        py::arg("stride") = 1, py::arg("bn") = 0, py::arg("accumulate") = false, py::arg("bn_x") = py::none(),
        py::arg("bn_stats") = py::none(), py::arg("bn_res") = py::none());
  m.def("conv3x3_wflip", &conv3x3_wflip);
  m.def("conv_wflip_multi", &conv_wflip_multi);
  m.def("strided_add", &strided_add);
  m.def("bn_partial_rows", &bn_partial_rows);
  m.def("maxpool_fwd", &maxpool_fwd);
  m.def("maxpool_bwd", &maxpool_bwd);
  m.def("bn_fwd", &bn_fwd);
  m.def("bn_apply", &bn_apply);
  m.def("bn_bwd", &bn_bwd);
}

}  // namespace dtf

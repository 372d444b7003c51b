// Python bindings for the generic op / optimizer kernels (csrc/kernels/gemm.hip, ops.hip).
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>

#include <stdexcept>
#include <vector>
#include <string>

extern "C" {
hipError_t dtfk_hogwild_pull(const float* shared, float* local, long long n, hipStream_t s);
hipError_t dtfk_hogwild_sgd(float* shared, const float* g, float* local, float lr, long long n, int locking,
                            unsigned long long* counter, long long* gstep_out, hipStream_t s);
hipError_t dtfk_hogwild_counter(unsigned long long* counter, long long* out, long long set, int do_set, hipStream_t s);
hipError_t dtfk_hogwild_gather_rows(const long long* ids, int n, int D, const float* const* shards, int W, float* out,
                                   hipStream_t s);
hipError_t dtfk_sparse_rows_apply(float* table, float* slot_a, float* slot_b, const long long* rows, const float* g,
                                  long long n, int D, int kind, float lr, float mu, int nesterov, float rho, float eps,
                                  const int* skip, hipStream_t s);
hipError_t dtfk_hogwild_scatter_sgd(const long long* ids, const float* g, int n, int D, float* const* shards, int W,
                                    float lr, int locking, hipStream_t s);
hipError_t dtfk_bucket_pack(const float* g, uint16_t* c, int64_t n, float scale, int fp16, hipStream_t s);
hipError_t dtfk_bucket_unpack(const uint16_t* c, float* g, int64_t n, float scale, int fp16, hipStream_t s);
int dtfk_route_max_world();
hipError_t dtfk_route_flags(const void* sids, int ids32, int N, int W, int* flag, int* onehot, hipStream_t stream);
hipError_t dtfk_route_scatter(const void* sids, int ids32, const int64_t* perm, const int* incl, const int* owncum,
                              int N, int W, int cap, int* inv_sorted, int64_t* inverse, int64_t* uniq, int* dest,
                              int64_t* send, int* count, hipStream_t stream);
hipError_t dtfk_philox_normal(float* out, long long rows, int dim, long long row_mul, long long row_add,
                              unsigned long long seed, float mean, float stddev, hipStream_t stream);
hipError_t dtfk_gemm(const void* A, int a_bf16, int lda, int transA, const void* B, int b_bf16, int ldb,
                     int transB, void* C, int c_bf16, int ldc, float* Z, const float* bias, int M, int N,
                     int K, float alpha, float beta, int act, hipStream_t stream);
hipError_t dtfk_gemm_big(const void* A, int lda, int transA, const void* B, int ldb, int transB, void* C,
                         int c_bf16, int ldc, const float* bias, int M, int N, int K, float alpha, float beta,
                         int act, int split_k, int variant, void* ws, hipStream_t stream);
long long dtfk_gemm_big_workspace(int M, int N, int K, int c_bf16, float beta, int act, int split_k, int variant);
int dtfk_gemm_big_supported(const void* A, int lda, int transA, const void* B, int ldb, int transB, int c_bf16, int M,
                            int N, int K, float beta, int act, int split_k);
hipError_t dtfk_gemm_bn_stats(const void* A, int lda, int transA, const void* B, int ldb, int transB, void* C, int ldc,
                              float* colpart, int M, int N, int K, hipStream_t stream);
int dtfk_gemm_bn_stat_rows(int M);
hipError_t dtfk_gemm_dgelu(const void* A, int lda, int transA, const void* B, int ldb, int transB, void* C, int ldc,
                           const void* aux, const float* bias, float* colpart, int M, int N, int K, hipStream_t stream);
hipError_t dtfk_gemm_gelu_aux(const void* A, int lda, int transA, const void* B, int ldb, int transB, void* C,
                              int ldc, void* aux, const float* bias, int M, int N, int K, hipStream_t stream);
hipError_t dtfk_colsum_partials_multi(const float* const* parts, float* const* outs, int nbuf, int P, int H,
                                      int accumulate, hipStream_t st);
hipError_t dtfk_gemm_big_cfg(int cfg, const void* A, int lda, const void* B, int ldb, void* C, int ldc, int M, int N,
                             int K, hipStream_t stream);
hipError_t dtfk_act_backward(const float* dy, const float* y, const float* z, float* dz, int64_t n, int act,
                             hipStream_t s);
hipError_t dtfk_col_sum(const float* X, float* out, int M, int N, int accum, hipStream_t s);
hipError_t dtfk_logit3_xent(const float* a, const float* b, const float* bias, const float* t, float* loss,
                            float* dz, int n, hipStream_t s);
hipError_t dtfk_logit3_xent_bwd(const float* dz, const float* g, float* d, float* gbias, int accum, int n,
                                hipStream_t s);
hipError_t dtfk_multi_copy(const void* const* src, void* const* dst, const long long* bytes, int n, hipStream_t s);
hipError_t dtfk_bag_index(const int64_t* offsets, int B, int* bag_of, int64_t N, hipStream_t s);
hipError_t dtfk_softmax_xent(const float* logits, const int64_t* labels, const float* ydense, float* loss_rows,
                             float* grad, int64_t* correct, int B, int C, float grad_scale, int naive,
                             hipStream_t s);
hipError_t dtfk_sigmoid_xent(const float* x, const float* t, float* loss, float* grad, int64_t n,
                             float grad_scale, hipStream_t s);
hipError_t dtfk_xent_fwd_bf16(const void* logits, const float* bias, const int64_t* labels, float* lse_rows,
                              float* loss_rows, int B, int C, hipStream_t s);
hipError_t dtfk_xent_bwd_bf16(const void* logits, const float* bias, const int64_t* labels, const float* lse_rows,
                              const float* dloss, void* grad, int B, int C, float scale, hipStream_t s);
hipError_t dtfk_embedding_bag_fwd(const float* W, int64_t V, int D, const int64_t* ids, const int64_t* offsets,
                                  const float* psw, int B, int mode, float* out, int64_t* bad, const int64_t* remap, hipStream_t s);
hipError_t dtfk_embedding_bag_bwd(float* target, int64_t V, int D, const int64_t* ids, const int64_t* offsets,
                                  const float* psw, const float* dout, int B, int mode, float lr,
                                  hipStream_t s);
hipError_t dtfk_embedding_bag_bwd_sorted(float* target, int64_t V, int D, const int* rows, const int64_t* occ,
                                         const int* bag_of, const float* psw, const float* dout, int64_t N,
                                         hipStream_t s);
hipError_t dtfk_argmax_correct(const float* x, const int64_t* labels, int B, int C, int64_t* count,
                               hipStream_t s);
hipError_t dtfk_auc_hist(const float* pred, const float* label, int64_t n, int nbins, unsigned long long* pos,
                         unsigned long long* neg, hipStream_t s);
hipError_t dtfk_multi_tensor_apply(const void* tab, const void* chunks, int nchunks, int kind, int gbf,
                                   const float* lr_ptr, float lr, float gscale, float wd, float b1, float b2,
                                   float eps, float momentum, int nesterov, const long long* step,
                                   const int* skip, hipStream_t s);
hipError_t dtfk_multi_tensor_sumsq(const void* tab, const void* chunks, int nchunks, int gbf, float* out,
                                   hipStream_t s);
int dtfk_mt_chunk();
int dtfk_tensor_rec_bytes();
}

namespace dtf {

static hipStream_t cs() { return c10::hip::getCurrentHIPStream().stream(); }
static void ck(hipError_t e, const char* w) {
  if (e != hipSuccess) throw std::runtime_error(std::string(w) + ": " + hipGetErrorString(e));
}
static void gpu(const at::Tensor& t, const char* n) {
  if (!t.is_cuda()) throw std::runtime_error(std::string(n) + " must be a GPU tensor");
}
static void f32c(const at::Tensor& t, const char* n) {
  gpu(t, n);
  if (t.scalar_type() != at::kFloat) throw std::runtime_error(std::string(n) + " must be float32");
  if (!t.is_contiguous()) throw std::runtime_error(std::string(n) + " must be contiguous");
}
static void i64c(const at::Tensor& t, const char* n) {
  gpu(t, n);
  if (t.scalar_type() != at::kLong) throw std::runtime_error(std::string(n) + " must be int64");
  if (!t.is_contiguous()) throw std::runtime_error(std::string(n) + " must be contiguous");
}
template <typename T>
static T* opt_ptr(const c10::optional<at::Tensor>& t) {
  return t.has_value() ? t->data_ptr<T>() : nullptr;
}

// out = act(alpha * op(A) @ op(B) + bias) (+ beta * out); Z (optional) gets the pre-activation.
void gemm(at::Tensor A, bool transA, at::Tensor B, bool transB, at::Tensor out,
          c10::optional<at::Tensor> bias, int act, double alpha, double beta, c10::optional<at::Tensor> Z) {
  gpu(A, "A"); gpu(B, "B"); gpu(out, "out");
  if (A.dim() != 2 || B.dim() != 2 || out.dim() != 2) throw std::runtime_error("gemm operands must be 2-D");
  if (A.stride(1) != 1 || B.stride(1) != 1 || out.stride(1) != 1)
    throw std::runtime_error("gemm operands must have unit inner stride");
  auto dt_ok = [](const at::Tensor& t) { return t.scalar_type() == at::kFloat || t.scalar_type() == at::kBFloat16; };
  if (!dt_ok(A) || !dt_ok(B) || !dt_ok(out)) throw std::runtime_error("gemm supports float32/bfloat16");
  const int M = (int)(transA ? A.size(1) : A.size(0));
  const int K = (int)(transA ? A.size(0) : A.size(1));
  const int KB = (int)(transB ? B.size(1) : B.size(0));
  const int N = (int)(transB ? B.size(0) : B.size(1));
  if (K != KB) throw std::runtime_error("gemm inner dimensions differ");
  if (out.size(0) != M || out.size(1) != N) throw std::runtime_error("gemm out has wrong shape");
  if (bias.has_value()) { f32c(*bias, "bias"); if (bias->numel() != N) throw std::runtime_error("bias size"); }
  if (Z.has_value()) { f32c(*Z, "Z"); if (Z->size(0) != M || Z->size(1) != N) throw std::runtime_error("Z shape"); }
  ck(dtfk_gemm(A.data_ptr(), A.scalar_type() == at::kBFloat16, (int)A.stride(0), transA, B.data_ptr(),
               B.scalar_type() == at::kBFloat16, (int)B.stride(0), transB, out.data_ptr(),
               out.scalar_type() == at::kBFloat16, (int)out.stride(0), opt_ptr<float>(Z), opt_ptr<float>(bias),
               M, N, K, (float)alpha, (float)beta, act, cs()),
     "gemm");
}

// Large-tile bf16 GEMM (gemm_big.hip): out = act(alpha * op(A) @ op(B) + bias) (+ beta * out).
// bf16 operands, bf16 or fp32 out.  Returns false (nothing launched) when the
// shape is outside the kernel's contract (K % 64, alignment), so callers can
// pick another GEMM; dtype / rank errors throw.
bool gemm_big(at::Tensor A, bool transA, at::Tensor B, bool transB, at::Tensor out, c10::optional<at::Tensor> bias,
              int act, double alpha, double beta, int split_k, int variant) {
  gpu(A, "A"); gpu(B, "B"); gpu(out, "out");
  if (A.dim() != 2 || B.dim() != 2 || out.dim() != 2) throw std::runtime_error("gemm_big operands must be 2-D");
  if (variant != 0 && variant != 4 && variant != 8 && variant != 9)
    throw std::runtime_error("gemm_big: variant 0 (auto), 4, 8 or 9");
  if (A.scalar_type() != at::kBFloat16 || B.scalar_type() != at::kBFloat16)
    throw std::runtime_error("gemm_big: bf16 operands");
  if (out.scalar_type() != at::kBFloat16 && out.scalar_type() != at::kFloat)
    throw std::runtime_error("gemm_big: bf16 or float32 output");
  if (A.stride(1) != 1 || B.stride(1) != 1 || out.stride(1) != 1)
    throw std::runtime_error("gemm_big operands must have unit inner stride");
  const int M = (int)(transA ? A.size(1) : A.size(0));
  const int K = (int)(transA ? A.size(0) : A.size(1));
  const int KB = (int)(transB ? B.size(1) : B.size(0));
  const int N = (int)(transB ? B.size(0) : B.size(1));
  if (K != KB) throw std::runtime_error("gemm_big inner dimensions differ");
  if (out.size(0) != M || out.size(1) != N) throw std::runtime_error("gemm_big out has wrong shape");
  if (bias.has_value()) { f32c(*bias, "bias"); if (bias->numel() != N) throw std::runtime_error("bias size"); }
  const int obf = out.scalar_type() == at::kBFloat16;
  if (!dtfk_gemm_big_supported(A.data_ptr(), (int)A.stride(0), transA, B.data_ptr(), (int)B.stride(0), transB, obf, M,
                               N, K, (float)beta, act, split_k))
    return false;   // outside the kernel's contract: the caller picks another GEMM
  // split-K slabs: an fp32 workspace from the caching allocator (freed -- and
  // reusable -- once the stream has passed the reduction)
  const long long wsb = dtfk_gemm_big_workspace(M, N, K, obf, (float)beta, act, split_k, variant);
  at::Tensor ws;
  if (wsb > 0) ws = at::empty({wsb / 4}, A.options().dtype(at::kFloat));
  ck(dtfk_gemm_big(A.data_ptr(), (int)A.stride(0), transA, B.data_ptr(), (int)B.stride(0), transB, out.data_ptr(), obf,
                   (int)out.stride(0), opt_ptr<float>(bias), M, N, K, (float)alpha, (float)beta, act, split_k, variant,
                   wsb > 0 ? ws.data_ptr() : nullptr, cs()),
     "gemm_big");   // any launch error is a real error
  return true;
}

// out = op(A) op(B) in bf16 plus the BatchNorm statistics partials of out in
// colpart ([2, ceil(M/128), N] fp32: per-column sums and sums of squares of the
// stored values per 128 rows) -- a 1x1 convolution feeding a BatchNorm
// (gemm_big.hip dtfk_gemm_bn_stats).  False (nothing launched) outside the
// kernel's contract.
bool gemm_bn_stats(at::Tensor A, bool transA, at::Tensor B, bool transB, at::Tensor out, at::Tensor colpart) {
  gpu(A, "A"); gpu(B, "B"); gpu(out, "out"); f32c(colpart, "colpart");
  if (A.dim() != 2 || B.dim() != 2 || out.dim() != 2) throw std::runtime_error("gemm_bn_stats: 2-D");
  for (const at::Tensor* t : {&A, &B, &out})
    if (t->scalar_type() != at::kBFloat16 || t->stride(1) != 1)
      throw std::runtime_error("gemm_bn_stats: bf16, unit inner stride");
  const int M = (int)(transA ? A.size(1) : A.size(0));
  const int K = (int)(transA ? A.size(0) : A.size(1));
  const int N = (int)(transB ? B.size(0) : B.size(1));
  if ((transB ? B.size(1) : B.size(0)) != K) throw std::runtime_error("gemm_bn_stats inner dimensions differ");
  if (out.size(0) != M || out.size(1) != N) throw std::runtime_error("gemm_bn_stats: out shape");
  if (colpart.numel() < 2LL * dtfk_gemm_bn_stat_rows(M) * N)
    throw std::runtime_error("gemm_bn_stats: colpart needs 2 * ceil(M/128) * N floats");
  const hipError_t e = dtfk_gemm_bn_stats(A.data_ptr(), (int)A.stride(0), transA, B.data_ptr(), (int)B.stride(0),
                                          transB, out.data_ptr(), (int)out.stride(0), colpart.data_ptr<float>(), M, N,
                                          K, cs());
  if (e == hipErrorInvalidValue) { (void)hipGetLastError(); return false; }   // shape / alignment contract
  ck(e, "gemm_bn_stats");
  return true;
}

// Input gradient of a linear layer fed by bias + GELU, with the GELU backward
// in the GEMM epilogue (gemm_big.hip dtfk_gemm_dgelu): out = (op(A) op(B)) *
// gelu'(aux + bias) in bf16, and dbias (fp32) = (or +=, accumulate) the column
// sums, via the kernel's [M/128, N] partials in `colpart`.  False (nothing
// launched) outside the kernel's contract.
bool gemm_dgelu(at::Tensor A, bool transA, at::Tensor B, bool transB, at::Tensor out, at::Tensor aux,
                c10::optional<at::Tensor> bias, at::Tensor colpart, at::Tensor dbias, bool accumulate) {
  gpu(A, "A"); gpu(B, "B"); gpu(out, "out"); gpu(aux, "aux");
  if (bias.has_value()) f32c(*bias, "bias");
  f32c(colpart, "colpart"); f32c(dbias, "dbias");
  if (A.dim() != 2 || B.dim() != 2 || out.dim() != 2 || aux.dim() != 2) throw std::runtime_error("gemm_dgelu: 2-D");
  for (const at::Tensor* t : {&A, &B, &out, &aux})
    if (t->scalar_type() != at::kBFloat16 || t->stride(1) != 1) throw std::runtime_error("gemm_dgelu: bf16, unit inner stride");
  const int M = (int)(transA ? A.size(1) : A.size(0));
  const int K = (int)(transA ? A.size(0) : A.size(1));
  const int N = (int)(transB ? B.size(0) : B.size(1));
  if ((transB ? B.size(1) : B.size(0)) != K) throw std::runtime_error("gemm_dgelu inner dimensions differ");
  if (out.size(0) != M || out.size(1) != N || aux.size(0) != M || aux.size(1) != N || aux.stride(0) != out.stride(0))
    throw std::runtime_error("gemm_dgelu: out / aux shape or leading dimension");
  if ((bias.has_value() && bias->numel() != N) || dbias.numel() != N || !dbias.is_contiguous())
    throw std::runtime_error("gemm_dgelu: bias size");
  if (M % 256 || N % 256 || K % 128) return false;
  if (colpart.numel() < (int64_t)(M / 128) * N) throw std::runtime_error("gemm_dgelu: colpart needs M/128 * N floats");
  const hipError_t e = dtfk_gemm_dgelu(A.data_ptr(), (int)A.stride(0), transA, B.data_ptr(), (int)B.stride(0), transB,
                                       out.data_ptr(), (int)out.stride(0), aux.data_ptr(), opt_ptr<float>(bias),
                                       colpart.data_ptr<float>(), M, N, K, cs());
  if (e == hipErrorInvalidValue) { (void)hipGetLastError(); return false; }   // alignment contract
  ck(e, "gemm_dgelu");
  const float* pp[1] = {colpart.data_ptr<float>()};
  float* po[1] = {dbias.data_ptr<float>()};
  ck(dtfk_colsum_partials_multi(pp, po, 1, M / 128, N, accumulate ? 1 : 0, cs()), "gemm_dgelu colsum");
  return true;
}

// Forward of a linear layer followed by bias + GELU (gemm_big.hip
// dtfk_gemm_gelu_aux): aux = op(A) op(B) + bias (the pre-activation, bf16) and
// out = gelu(aux) (bf16) from one epilogue.  False outside the contract.
bool gemm_gelu_aux(at::Tensor A, bool transA, at::Tensor B, bool transB, at::Tensor out, at::Tensor aux,
                   at::Tensor bias) {
  gpu(A, "A"); gpu(B, "B"); gpu(out, "out"); gpu(aux, "aux"); f32c(bias, "bias");
  if (A.dim() != 2 || B.dim() != 2 || out.dim() != 2 || aux.dim() != 2) throw std::runtime_error("gemm_gelu_aux: 2-D");
  for (const at::Tensor* t : {&A, &B, &out, &aux})
    if (t->scalar_type() != at::kBFloat16 || t->stride(1) != 1)
      throw std::runtime_error("gemm_gelu_aux: bf16, unit inner stride");
  const int M = (int)(transA ? A.size(1) : A.size(0));
  const int K = (int)(transA ? A.size(0) : A.size(1));
  const int N = (int)(transB ? B.size(0) : B.size(1));
  if ((transB ? B.size(1) : B.size(0)) != K) throw std::runtime_error("gemm_gelu_aux inner dimensions differ");
  if (out.size(0) != M || out.size(1) != N || aux.size(0) != M || aux.size(1) != N || aux.stride(0) != out.stride(0))
    throw std::runtime_error("gemm_gelu_aux: out / aux shape or leading dimension");
  if (bias.numel() != N) throw std::runtime_error("gemm_gelu_aux: bias size");
  if (M % 256 || N % 256 || K % 128) return false;
  const hipError_t e = dtfk_gemm_gelu_aux(A.data_ptr(), (int)A.stride(0), transA, B.data_ptr(), (int)B.stride(0),
                                          transB, out.data_ptr(), (int)out.stride(0), aux.data_ptr(),
                                          bias.data_ptr<float>(), M, N, K, cs());
  if (e == hipErrorInvalidValue) { (void)hipGetLastError(); return false; }
  ck(e, "gemm_gelu_aux");
  return true;
}

// tiling experiments of gemm_big (forward layout only): out[M,N] = A[M,K] B[N,K]^T, bf16
void gemm_big_cfg(int cfg, at::Tensor A, at::Tensor B, at::Tensor out) {
  gpu(A, "A"); gpu(B, "B"); gpu(out, "out");
  if (A.scalar_type() != at::kBFloat16 || B.scalar_type() != at::kBFloat16 || out.scalar_type() != at::kBFloat16 ||
      !A.is_contiguous() || !B.is_contiguous() || !out.is_contiguous() || A.size(1) != B.size(1) ||
      out.size(0) != A.size(0) || out.size(1) != B.size(0))
    throw std::runtime_error("gemm_big_cfg: contiguous bf16 A[M,K], B[N,K], out[M,N]");
  ck(dtfk_gemm_big_cfg(cfg, A.data_ptr(), (int)A.size(1), B.data_ptr(), (int)B.size(1), out.data_ptr(),
                       (int)out.size(1), (int)A.size(0), (int)B.size(0), (int)A.size(1), cs()),
     "gemm_big_cfg");
}

void act_backward(at::Tensor dy, c10::optional<at::Tensor> y, c10::optional<at::Tensor> z, at::Tensor dz,
                  int act) {
  f32c(dy, "dy"); f32c(dz, "dz");
  if (y.has_value()) f32c(*y, "y");
  if (z.has_value()) f32c(*z, "z");
  ck(dtfk_act_backward(dy.data_ptr<float>(), opt_ptr<float>(y), opt_ptr<float>(z), dz.data_ptr<float>(),
                       dy.numel(), act, cs()),
     "act_backward");
}

// Wide&Deep head (fused): loss[0] = mean xent(a + b + bias[0], t), dz
void logit3_xent(at::Tensor a, at::Tensor b, at::Tensor bias, at::Tensor t, at::Tensor loss, at::Tensor dz) {
  f32c(a, "a"); f32c(b, "b"); f32c(bias, "bias"); f32c(t, "t"); f32c(loss, "loss"); f32c(dz, "dz");
  const int64_t n = a.numel();
  if (b.numel() != n || t.numel() != n || dz.numel() != n || bias.numel() < 1 || loss.numel() < 1)
    throw std::runtime_error("logit3_xent: size mismatch");
  ck(dtfk_logit3_xent(a.data_ptr<float>(), b.data_ptr<float>(), bias.data_ptr<float>(), t.data_ptr<float>(),
                      loss.data_ptr<float>(), dz.data_ptr<float>(), (int)n, cs()),
     "logit3_xent");
}
void logit3_xent_bwd(at::Tensor dz, at::Tensor g, at::Tensor d, c10::optional<at::Tensor> gbias, bool accumulate) {
  f32c(dz, "dz"); f32c(g, "g"); f32c(d, "d");
  if (gbias.has_value()) f32c(*gbias, "gbias");
  ck(dtfk_logit3_xent_bwd(dz.data_ptr<float>(), g.data_ptr<float>(), d.data_ptr<float>(),
                          gbias.has_value() ? gbias->data_ptr<float>() : nullptr, accumulate ? 1 : 0, (int)dz.numel(), cs()),
     "logit3_xent_bwd");
}
// dst[i].copy_(src[i]) for up to 8 contiguous same-size pairs in one launch
void multi_copy(std::vector<at::Tensor> dst, std::vector<at::Tensor> src) {
  if (dst.size() != src.size() || dst.empty() || dst.size() > 8) throw std::runtime_error("multi_copy: 1..8 pairs");
  const void* sp[8];
  void* dp[8];
  long long nb[8];
  for (size_t i = 0; i < dst.size(); ++i) {
    gpu(dst[i], "dst"); gpu(src[i], "src");
    if (!dst[i].is_contiguous() || !src[i].is_contiguous() || dst[i].scalar_type() != src[i].scalar_type() ||
        dst[i].numel() != src[i].numel())
      throw std::runtime_error("multi_copy: contiguous pairs of one dtype and size expected");
    sp[i] = src[i].data_ptr();
    dp[i] = dst[i].data_ptr();
    nb[i] = (long long)(src[i].numel() * src[i].element_size());
  }
  ck(dtfk_multi_copy(sp, dp, nb, (int)dst.size(), cs()), "multi_copy");
}

void col_sum(at::Tensor X, at::Tensor out, bool accumulate) {
  f32c(X, "X"); f32c(out, "out");
  const int N = (int)X.size(-1);
  const int M = (int)(X.numel() / std::max<int64_t>(1, N));
  ck(dtfk_col_sum(X.data_ptr<float>(), out.data_ptr<float>(), M, N, accumulate ? 1 : 0, cs()), "col_sum");
}

static void bf16xent_check(const at::Tensor& logits, const c10::optional<at::Tensor>& bias, const at::Tensor& labels) {
  if (!logits.is_cuda() || logits.scalar_type() != at::kBFloat16 || !logits.is_contiguous() || logits.dim() != 2 ||
      logits.size(1) % 2)
    throw std::runtime_error("xent_bf16: logits must be contiguous [B, C] bf16 on GPU with C even");
  i64c(labels, "labels");
  if (labels.numel() != logits.size(0)) throw std::runtime_error("xent_bf16: labels must be [B]");
  if (bias.has_value()) {
    f32c(*bias, "bias");
    if (bias->numel() != logits.size(1)) throw std::runtime_error("xent_bf16: bias must be [C]");
  }
}

void xent_fwd_bf16(at::Tensor logits, c10::optional<at::Tensor> bias, at::Tensor labels, at::Tensor lse_rows,
                   at::Tensor loss_rows) {
  bf16xent_check(logits, bias, labels);
  f32c(lse_rows, "lse_rows"); f32c(loss_rows, "loss_rows");
  ck(dtfk_xent_fwd_bf16(logits.data_ptr(), opt_ptr<float>(bias), labels.data_ptr<int64_t>(), lse_rows.data_ptr<float>(),
                        loss_rows.data_ptr<float>(), (int)logits.size(0), (int)logits.size(1), cs()),
     "xent_fwd_bf16");
}

void xent_bwd_bf16(at::Tensor logits, c10::optional<at::Tensor> bias, at::Tensor labels, at::Tensor lse_rows,
                   c10::optional<at::Tensor> dloss, at::Tensor grad, double scale) {
  bf16xent_check(logits, bias, labels);
  f32c(lse_rows, "lse_rows");
  if (dloss.has_value()) f32c(*dloss, "dloss");
  if (!grad.is_cuda() || grad.scalar_type() != at::kBFloat16 || !grad.is_contiguous() ||
      grad.numel() != logits.numel())
    throw std::runtime_error("xent_bwd_bf16: grad must be a contiguous bf16 tensor like logits");
  ck(dtfk_xent_bwd_bf16(logits.data_ptr(), opt_ptr<float>(bias), labels.data_ptr<int64_t>(), lse_rows.data_ptr<float>(),
                        opt_ptr<float>(dloss), grad.data_ptr(), (int)logits.size(0), (int)logits.size(1),
                        (float)scale, cs()),
     "xent_bwd_bf16");
}

void softmax_xent(at::Tensor logits, c10::optional<at::Tensor> labels, c10::optional<at::Tensor> ydense,
                  at::Tensor loss_rows, c10::optional<at::Tensor> grad, c10::optional<at::Tensor> correct,
                  double grad_scale, bool naive) {
  f32c(logits, "logits"); f32c(loss_rows, "loss_rows");
  const int B = (int)logits.size(0), C = (int)logits.size(1);
  if (labels.has_value()) i64c(*labels, "labels");
  if (ydense.has_value()) f32c(*ydense, "ydense");
  if (!labels.has_value() && !ydense.has_value()) throw std::runtime_error("labels or ydense required");
  if (grad.has_value()) f32c(*grad, "grad");
  if (correct.has_value()) i64c(*correct, "correct");
  ck(dtfk_softmax_xent(logits.data_ptr<float>(), opt_ptr<int64_t>(labels), opt_ptr<float>(ydense),
                       loss_rows.data_ptr<float>(), opt_ptr<float>(grad), opt_ptr<int64_t>(correct), B, C,
                       (float)grad_scale, naive ? 1 : 0, cs()),
     "softmax_xent");
}

void sigmoid_xent(at::Tensor x, at::Tensor t, at::Tensor loss, c10::optional<at::Tensor> grad, double gs) {
  f32c(x, "x"); f32c(t, "t"); f32c(loss, "loss");
  if (grad.has_value()) f32c(*grad, "grad");
  ck(dtfk_sigmoid_xent(x.data_ptr<float>(), t.data_ptr<float>(), loss.data_ptr<float>(), opt_ptr<float>(grad),
                       x.numel(), (float)gs, cs()),
     "sigmoid_xent");
}

void embedding_bag_fwd(at::Tensor W, at::Tensor ids, at::Tensor offsets, c10::optional<at::Tensor> psw, int mode,
                       at::Tensor out, c10::optional<at::Tensor> bad, c10::optional<at::Tensor> remap) {
  f32c(W, "weight"); i64c(ids, "ids"); i64c(offsets, "offsets"); f32c(out, "out");
  if (psw.has_value()) f32c(*psw, "per_sample_weights");
  if (bad.has_value()) i64c(*bad, "bad");
  if (remap.has_value()) i64c(*remap, "remap");
  const int B = (int)offsets.numel() - 1;
  const int D = W.dim() == 1 ? 1 : (int)W.size(1);
  ck(dtfk_embedding_bag_fwd(W.data_ptr<float>(), W.size(0), D, ids.data_ptr<int64_t>(),
                            offsets.data_ptr<int64_t>(), opt_ptr<float>(psw), B, mode, out.data_ptr<float>(),
                            opt_ptr<int64_t>(bad), opt_ptr<int64_t>(remap), cs()),
     "embedding_bag_fwd");
}

// offsets None: one id per bag (B = ids.numel())
void embedding_bag_bwd(at::Tensor target, at::Tensor ids, c10::optional<at::Tensor> offsets,
                       c10::optional<at::Tensor> psw, at::Tensor dout, int mode, double lr) {
  f32c(target, "target"); i64c(ids, "ids"); f32c(dout, "dout");
  if (offsets.has_value()) i64c(*offsets, "offsets");
  if (psw.has_value()) f32c(*psw, "per_sample_weights");
  const int B = offsets.has_value() ? (int)offsets->numel() - 1 : (int)ids.numel();
  const int D = target.dim() == 1 ? 1 : (int)target.size(1);
  ck(dtfk_embedding_bag_bwd(target.data_ptr<float>(), target.size(0), D, ids.data_ptr<int64_t>(),
                            opt_ptr<int64_t>(offsets), opt_ptr<float>(psw), dout.data_ptr<float>(), B, mode,
                            (float)lr, cs()),
     "embedding_bag_bwd");
}
void bag_index(at::Tensor offsets, at::Tensor bag_of) {
  i64c(offsets, "offsets");
  gpu(bag_of, "bag_of");
  if (bag_of.scalar_type() != at::kInt || !bag_of.is_contiguous()) throw std::runtime_error("bag_index: int32 out");
  ck(dtfk_bag_index(offsets.data_ptr<int64_t>(), (int)offsets.numel() - 1, bag_of.data_ptr<int>(), bag_of.numel(),
                    cs()),
     "bag_index");
}

void embedding_bag_bwd_sorted(at::Tensor target, at::Tensor rows, at::Tensor occ, at::Tensor bag_of,
                              c10::optional<at::Tensor> psw, at::Tensor dout) {
  f32c(target, "target"); i64c(occ, "occ"); f32c(dout, "dout");
  gpu(rows, "rows"); gpu(bag_of, "bag_of");
  if (rows.scalar_type() != at::kInt || bag_of.scalar_type() != at::kInt || !rows.is_contiguous() ||
      !bag_of.is_contiguous())
    throw std::runtime_error("embedding_bag_bwd_sorted: rows / bag_of must be contiguous int32");
  if (psw.has_value()) f32c(*psw, "per_sample_weights");
  const int64_t N = rows.numel();
  const int D = target.dim() == 1 ? 1 : (int)target.size(1);
  if (occ.numel() != N || bag_of.numel() != N) throw std::runtime_error("embedding_bag_bwd_sorted: length mismatch");
  if (psw.has_value() && psw->numel() != N) throw std::runtime_error("embedding_bag_bwd_sorted: psw length");
  if (dout.dim() != 2 || dout.size(1) != D) throw std::runtime_error("embedding_bag_bwd_sorted: dout must be [B, D]");
  ck(dtfk_embedding_bag_bwd_sorted(target.data_ptr<float>(), target.size(0), D, rows.data_ptr<int>(),
                                   occ.data_ptr<int64_t>(), bag_of.data_ptr<int>(), opt_ptr<float>(psw),
                                   dout.data_ptr<float>(), N, cs()),
     "embedding_bag_bwd_sorted");
}

void argmax_correct(at::Tensor x, at::Tensor labels, at::Tensor count) {
  f32c(x, "x"); i64c(labels, "labels"); i64c(count, "count");
  ck(dtfk_argmax_correct(x.data_ptr<float>(), labels.data_ptr<int64_t>(), (int)x.size(0), (int)x.size(1),
                         count.data_ptr<int64_t>(), cs()),
     "argmax_correct");
}

void auc_hist(at::Tensor pred, at::Tensor label, at::Tensor pos, at::Tensor neg) {
  f32c(pred, "pred"); f32c(label, "label"); i64c(pos, "pos"); i64c(neg, "neg");
  ck(dtfk_auc_hist(pred.data_ptr<float>(), label.data_ptr<float>(), pred.numel(), (int)pos.numel(),
                   reinterpret_cast<unsigned long long*>(pos.data_ptr<int64_t>()),
                   reinterpret_cast<unsigned long long*>(neg.data_ptr<int64_t>()), cs()),
     "auc_hist");
}

void multi_tensor_apply(at::Tensor tab, at::Tensor chunks, int kind, bool grad_bf16,
                        c10::optional<at::Tensor> lr_t, double lr, double gscale, double wd, double b1,
                        double b2, double eps, double momentum, bool nesterov, c10::optional<at::Tensor> step,
                        c10::optional<at::Tensor> skip) {
  gpu(tab, "table"); gpu(chunks, "chunks");
  if (tab.dim() != 2 || tab.size(1) * 8 != dtfk_tensor_rec_bytes())
    throw std::runtime_error("multi_tensor_apply: table rows must be TensorRec {p, g, m, v, n, shadow}");
  if (lr_t.has_value()) f32c(*lr_t, "lr");
  if (step.has_value()) i64c(*step, "step");
  if (skip.has_value() && (!skip->is_cuda() || skip->scalar_type() != at::kInt))
    throw std::runtime_error("multi_tensor_apply: skip must be a device int32 flag");
  ck(dtfk_multi_tensor_apply(tab.data_ptr(), chunks.data_ptr(), (int)chunks.size(0), kind, grad_bf16 ? 1 : 0,
                             opt_ptr<float>(lr_t), (float)lr, (float)gscale, (float)wd, (float)b1, (float)b2,
                             (float)eps, (float)momentum, nesterov ? 1 : 0,
                             step.has_value() ? reinterpret_cast<const long long*>(step->data_ptr<int64_t>()) : nullptr,
                             skip.has_value() ? skip->data_ptr<int>() : nullptr, cs()),
     "multi_tensor_apply");
}

void multi_tensor_sumsq(at::Tensor tab, at::Tensor chunks, bool grad_bf16, at::Tensor out) {
  gpu(tab, "table"); gpu(chunks, "chunks"); f32c(out, "out");
  ck(dtfk_multi_tensor_sumsq(tab.data_ptr(), chunks.data_ptr(), (int)chunks.size(0), grad_bf16 ? 1 : 0,
                             out.data_ptr<float>(), cs()),
     "multi_tensor_sumsq");
}

void philox_normal(at::Tensor out, int64_t row_mul, int64_t row_add, uint64_t seed, double mean, double stddev) {
  f32c(out, "out");
  if (out.dim() != 2) throw std::runtime_error("philox_normal: out must be [rows, dim]");
  ck(dtfk_philox_normal(out.data_ptr<float>(), out.size(0), (int)out.size(1), row_mul, row_add, seed, (float)mean,
                        (float)stddev, cs()),
     "philox_normal");
}

// Dedup + owner bucketing of sorted ids (csrc/kernels/sparse_route.hip: flags,
// rocPRIM scans, one scatter pass).
std::vector<at::Tensor> sparse_route(at::Tensor sids, at::Tensor perm, int W, int64_t cap) {
  gpu(sids, "sids"); i64c(perm, "perm");
  if (!sids.is_contiguous() || (sids.scalar_type() != at::kInt && sids.scalar_type() != at::kLong))
    throw std::runtime_error("sparse_route: sorted ids must be contiguous int32/int64");
  if (W < 1 || W > dtfk_route_max_world()) throw std::runtime_error("sparse_route: world size out of range");
  const int64_t N = sids.numel();
  if (W > 1 && cap < 1) throw std::runtime_error("sparse_route: per-peer capacity must be >= 1");
  if (std::max(N, cap) * std::max(W, 1) >= (1LL << 31)) throw std::runtime_error("sparse_route: batch too large");
  auto o32 = sids.options().dtype(at::kInt), o64 = sids.options().dtype(at::kLong);
  at::Tensor inv = at::empty({N}, o32), inverse = at::empty({N}, o64), uniq = at::empty({N}, o64);
  at::Tensor dest = at::empty({W > 1 ? N : 0}, o32), send = at::empty({W > 1 ? (int64_t)W * cap : 0}, o64);
  at::Tensor count = at::empty({1}, o32);
  const int ids32 = sids.scalar_type() == at::kInt ? 1 : 0;
  // [flags | owner one-hot rows (W > 1)], owner-major, scanned flat in ONE pass
  const int64_t nrow = W > 1 ? W + 1 : 1;
  at::Tensor fl = at::empty({nrow * N}, o32);
  ck(dtfk_route_flags(sids.data_ptr(), ids32, (int)N, W, fl.data_ptr<int>(), W > 1 ? fl.data_ptr<int>() + N : nullptr,
                      cs()),
     "route_flags");
  at::Tensor scan = at::cumsum(fl, 0, at::kInt);
  ck(dtfk_route_scatter(sids.data_ptr(), ids32, perm.data_ptr<int64_t>(), scan.data_ptr<int>(),
                        W > 1 ? scan.data_ptr<int>() + N : nullptr, (int)N, W, (int)cap, inv.data_ptr<int>(),
                        inverse.data_ptr<int64_t>(), uniq.data_ptr<int64_t>(), W > 1 ? dest.data_ptr<int>() : nullptr,
                        W > 1 ? send.data_ptr<int64_t>() : nullptr, count.data_ptr<int>(), cs()),
     "route_scatter");
  // unique ids per owner (differences of the scan at the row ends): the
  // caller's overflow test (> cap) and capacity adaptation, no host read-back
  at::Tensor ocnt = count;
  if (W > 1) {
    at::Tensor ends = scan.view({nrow, N}).select(1, N - 1);
    ocnt = (ends.slice(0, 1, nrow) - ends.slice(0, 0, nrow - 1)).contiguous();
  }
  return {inv, inverse, uniq, dest, send, count, ocnt};
}

// DDP bucket <-> 16-bit (bf16 / fp16) comm buffer with the 1/N scale folded in
// (csrc/kernels/ops.hip K16); the comm buffer's dtype picks the format.
static int comm16(const at::Tensor& g, const at::Tensor& c, const char* who) {
  f32c(g, "grad bucket"); gpu(c, "comm buffer");
  if ((c.scalar_type() != at::kBFloat16 && c.scalar_type() != at::kHalf) || !c.is_contiguous() ||
      c.numel() != g.numel())
    throw std::runtime_error(std::string(who) + ": contiguous bf16 / fp16 comm buffer of the bucket's size expected");
  if ((reinterpret_cast<uintptr_t>(g.data_ptr()) & 15) || (reinterpret_cast<uintptr_t>(c.data_ptr()) & 15))
    throw std::runtime_error(std::string(who) + ": 16-byte aligned buffers expected");
  return c.scalar_type() == at::kHalf;
}
void bucket_pack(at::Tensor g, at::Tensor c, double scale) {
  const int f16 = comm16(g, c, "bucket_pack");
  ck(dtfk_bucket_pack(g.data_ptr<float>(), reinterpret_cast<uint16_t*>(c.data_ptr()), g.numel(), (float)scale, f16,
                      cs()),
     "bucket_pack");
}
void bucket_unpack(at::Tensor c, at::Tensor g, double scale) {
  const int f16 = comm16(g, c, "bucket_unpack");
  ck(dtfk_bucket_unpack(reinterpret_cast<const uint16_t*>(c.data_ptr()), g.data_ptr<float>(), g.numel(),
                        (float)scale, f16, cs()),
     "bucket_unpack");
}

// Hogwild parameter store (csrc/kernels/hogwild.hip): `shared` / `counter` are
// raw device addresses (an IPC-mapped peer buffer); local / grads / gstep_out GPU tensors.
static void hogwild_pull(int64_t shared, at::Tensor local) {
  gpu(local, "local");
  if (local.scalar_type() != at::kFloat || !local.is_contiguous()) throw std::runtime_error("hogwild: fp32 contiguous");
  ck(dtfk_hogwild_pull(reinterpret_cast<const float*>(shared), local.data_ptr<float>(), local.numel(), cs()),
     "hogwild_pull");
}
static void hogwild_sgd(int64_t shared, at::Tensor grads, at::Tensor local, double lr, bool locking, int64_t counter,
                        at::Tensor gstep_out) {
  gpu(grads, "grads"); gpu(local, "local"); gpu(gstep_out, "gstep_out");
  if (grads.scalar_type() != at::kFloat || local.scalar_type() != at::kFloat || !grads.is_contiguous() ||
      !local.is_contiguous() || grads.numel() != local.numel() || gstep_out.scalar_type() != at::kLong)
    throw std::runtime_error("hogwild_sgd: fp32 contiguous grads/local of one size, int64 gstep_out");
  ck(dtfk_hogwild_sgd(reinterpret_cast<float*>(shared), grads.data_ptr<float>(), local.data_ptr<float>(), (float)lr,
                      local.numel(), locking ? 1 : 0, reinterpret_cast<unsigned long long*>(counter),
                      reinterpret_cast<long long*>(gstep_out.data_ptr<int64_t>()), cs()),
     "hogwild_sgd");
}
static void hogwild_counter(int64_t counter, at::Tensor out, int64_t set, bool do_set) {
  gpu(out, "out");
  ck(dtfk_hogwild_counter(reinterpret_cast<unsigned long long*>(counter), reinterpret_cast<long long*>(out.data_ptr<int64_t>()), set, do_set ? 1 : 0,
                          cs()),
     "hogwild_counter");
}

// rows of IPC-mapped table shards (`shards`: device table of W shard addresses)
static void hogwild_gather_rows(at::Tensor ids, int64_t shards, int W, at::Tensor out) {
  i64c(ids, "ids"); f32c(out, "out");
  if (out.dim() != 2 || out.size(0) != ids.numel()) throw std::runtime_error("hogwild_gather_rows: out [n, D]");
  ck(dtfk_hogwild_gather_rows(reinterpret_cast<const long long*>(ids.data_ptr<int64_t>()), (int)ids.numel(),
                              (int)out.size(1), reinterpret_cast<const float* const*>(shards), W,
                              out.data_ptr<float>(), cs()),
     "hogwild_gather_rows");
}
static void hogwild_scatter_sgd(at::Tensor ids, at::Tensor grads, int64_t shards, int W, double lr, bool locking) {
  i64c(ids, "ids"); f32c(grads, "grads");
  if (grads.dim() != 2 || grads.size(0) != ids.numel()) throw std::runtime_error("hogwild_scatter_sgd: grads [n, D]");
  ck(dtfk_hogwild_scatter_sgd(reinterpret_cast<const long long*>(ids.data_ptr<int64_t>()),
                              grads.data_ptr<float>(), (int)ids.numel(), (int)grads.size(1),
                              reinterpret_cast<float* const*>(shards), W, (float)lr, locking ? 1 : 0, cs()),
     "hogwild_scatter_sgd");
}

// Row-sparse optimizer update of a table shard (sparse_optim.hip): rows[i] >= 0
// distinct (the owner summed the duplicates), -1 = no update.
static void sparse_rows_apply(at::Tensor table, c10::optional<at::Tensor> slot_a, c10::optional<at::Tensor> slot_b,
                              at::Tensor rows, at::Tensor g, int kind, double lr, double mu, bool nesterov,
                              double rho, double eps, c10::optional<at::Tensor> skip) {
  f32c(table, "table"); i64c(rows, "rows"); f32c(g, "g");
  if (table.dim() != 2 || g.dim() != 2 || g.size(0) != rows.numel() || g.size(1) != table.size(1))
    throw std::runtime_error("sparse_rows_apply: table [R, D], g [n, D], rows [n]");
  for (auto* t : {&slot_a, &slot_b})
    if (t->has_value()) {
      f32c(**t, "slot");
      if ((*t)->sizes() != table.sizes()) throw std::runtime_error("sparse_rows_apply: slot shape != table shape");
    }
  if (skip.has_value() && (skip->scalar_type() != at::kInt || !skip->is_cuda()))
    throw std::runtime_error("sparse_rows_apply: skip must be a device int32 tensor");
  ck(dtfk_sparse_rows_apply(table.data_ptr<float>(), opt_ptr<float>(slot_a), opt_ptr<float>(slot_b),
                            reinterpret_cast<const long long*>(rows.data_ptr<int64_t>()), g.data_ptr<float>(),
                            rows.numel(), (int)table.size(1), kind, (float)lr, (float)mu, nesterov ? 1 : 0,
                            (float)rho, (float)eps, opt_ptr<int>(skip), cs()),
     "sparse_rows_apply");
}

void init_ops(py::module& m) {
  m.def("sparse_rows_apply", &sparse_rows_apply, py::arg("table"), py::arg("slot_a"), py::arg("slot_b"),
        py::arg("rows"), py::arg("g"), py::arg("kind"), py::arg("lr"), py::arg("mu") = 0.0,
        py::arg("nesterov") = false, py::arg("rho") = 0.9, py::arg("eps") = 1e-10, py::arg("skip") = py::none());
  m.def("hogwild_gather_rows", &hogwild_gather_rows, py::arg("ids"), py::arg("shards"), py::arg("W"), py::arg("out"));
  m.def("hogwild_scatter_sgd", &hogwild_scatter_sgd, py::arg("ids"), py::arg("grads"), py::arg("shards"), py::arg("W"),
        py::arg("lr"), py::arg("locking"));
  m.def("hogwild_pull", &hogwild_pull, py::arg("shared"), py::arg("local"));
  m.def("hogwild_sgd", &hogwild_sgd, py::arg("shared"), py::arg("grads"), py::arg("local"), py::arg("lr"),
        py::arg("locking"), py::arg("counter"), py::arg("gstep_out"));
  m.def("hogwild_counter", &hogwild_counter, py::arg("counter"), py::arg("out"), py::arg("set") = 0,
        py::arg("do_set") = false);
  m.def("bucket_pack", &bucket_pack, py::arg("g"), py::arg("c"), py::arg("scale"));
  m.def("bucket_unpack", &bucket_unpack, py::arg("c"), py::arg("g"), py::arg("scale"));
  m.def("bucket_pack_bf16", &bucket_pack);     // round-2 names
  m.def("bucket_unpack_bf16", &bucket_unpack);
  m.def("sparse_route", &sparse_route, py::arg("sids"), py::arg("perm"), py::arg("W"), py::arg("cap"));
  m.def("route_max_world", &dtfk_route_max_world);
  m.def("philox_normal", &philox_normal, py::arg("out"), py::arg("row_mul"), py::arg("row_add"), py::arg("seed"),
        py::arg("mean"), py::arg("stddev"));
  m.def("gemm", &gemm, py::arg("A"), py::arg("transA"), py::arg("B"), py::arg("transB"), py::arg("out"),
        py::arg("bias") = py::none(), py::arg("act") = 0, py::arg("alpha") = 1.0, py::arg("beta") = 0.0,
        py::arg("Z") = py::none());
  m.def("gemm_big", &gemm_big, py::arg("A"), py::arg("transA"), py::arg("B"), py::arg("transB"), py::arg("out"),
        py::arg("bias") = py::none(), py::arg("act") = 0, py::arg("alpha") = 1.0, py::arg("beta") = 0.0,
        py::arg("split_k") = 0, py::arg("variant") = 0);
  m.def("gemm_big_cfg", &gemm_big_cfg);
  m.def("gemm_bn_stats", &gemm_bn_stats, py::arg("A"), py::arg("transA"), py::arg("B"), py::arg("transB"),
        py::arg("out"), py::arg("colpart"));
  m.def("gemm_bn_stat_rows", [](int64_t M) { return dtfk_gemm_bn_stat_rows((int)M); });
  m.def("gemm_dgelu", &gemm_dgelu, py::arg("A"), py::arg("transA"), py::arg("B"), py::arg("transB"), py::arg("out"),
        py::arg("aux"), py::arg("bias"), py::arg("colpart"), py::arg("dbias"), py::arg("accumulate") = false);
  m.def("gemm_gelu_aux", &gemm_gelu_aux, py::arg("A"), py::arg("transA"), py::arg("B"), py::arg("transB"),
        py::arg("out"), py::arg("aux"), py::arg("bias"));
  m.def("act_backward", &act_backward);
  m.def("col_sum", &col_sum, py::arg("X"), py::arg("out"), py::arg("accumulate") = false);
  m.def("logit3_xent", &logit3_xent);
  m.def("logit3_xent_bwd", &logit3_xent_bwd);
  m.def("multi_copy", &multi_copy);
  m.def("bag_index", &bag_index);
  m.def("softmax_xent", &softmax_xent);
  m.def("xent_fwd_bf16", &xent_fwd_bf16);
  m.def("xent_bwd_bf16", &xent_bwd_bf16);
  m.def("sigmoid_xent", &sigmoid_xent);
  m.def("embedding_bag_fwd", &embedding_bag_fwd, py::arg("W"), py::arg("ids"), py::arg("offsets"), py::arg("psw"),
        py::arg("mode"), py::arg("out"), py::arg("bad") = py::none(), py::arg("remap") = py::none());
  m.def("embedding_bag_bwd", &embedding_bag_bwd);
  m.def("embedding_bag_bwd_sorted", &embedding_bag_bwd_sorted);
  m.def("argmax_correct", &argmax_correct);
  m.def("auc_hist", &auc_hist);
  m.def("multi_tensor_apply", &multi_tensor_apply, py::arg("tab"), py::arg("chunks"), py::arg("kind"),
        py::arg("grad_bf16"), py::arg("lr_t"), py::arg("lr"), py::arg("gscale"), py::arg("wd"), py::arg("b1"),
        py::arg("b2"), py::arg("eps"), py::arg("momentum"), py::arg("nesterov"), py::arg("step"),
        py::arg("skip") = py::none());
  m.def("multi_tensor_sumsq", &multi_tensor_sumsq);
  m.def("mt_chunk", &dtfk_mt_chunk);
  m.def("tensor_rec_bytes", &dtfk_tensor_rec_bytes);
}

}  // namespace dtf

// Python bindings for the fused transformer kernels (csrc/kernels/transformer.hip).
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>

#include <stdexcept>
#include <string>

extern "C" {
hipError_t dtfk_bdrln_fwd(const void* x, const float* bias, const void* res, const float* gamma, const float* beta,
                          void* y, void* s_out, float* mean, float* rstd, int N, int H, float eps, float p,
                          unsigned long long seed, hipStream_t st);
hipError_t dtfk_emb_ln_fwd(const float* word, const int64_t* ids, const float* typ, const int64_t* tt,
                           const float* pos, int S, const float* gamma, const float* beta, void* y, void* s_out,
                           float* mean, float* rstd, int N, int H, float eps, float p, unsigned long long seed,
                           hipStream_t st);
hipError_t dtfk_emb_bwd_aux(const void* ds, const int64_t* tt, int B, int S, int H, float* pos_grad, float* part,
                            int accumulate, hipStream_t st);
hipError_t dtfk_ln_fwd_f32in(const float* x, const float* gamma, const float* beta, void* y, void* s_out,
                             float* mean, float* rstd, int N, int H, float eps, float p, unsigned long long seed,
                             hipStream_t st);
hipError_t dtfk_ln_bwd(const void* dy, const void* s, const float* mean, const float* rstd, const float* gamma,
                       void* ds, void* dxb, float* part_g, float* part_b, float* part_bias, int grid, int N, int H,
                       float p, unsigned long long seed, hipStream_t st);
hipError_t dtfk_colsum_partials(const float* part, float* out, int P, int H, hipStream_t st);
hipError_t dtfk_colsum_partials_multi(const float* const* parts, float* const* outs, int nbuf, int P, int H,
                                      int accumulate, hipStream_t st);
hipError_t dtfk_colsum_bf16(const void* x, float* part, float* out, int N, int H, int P, int accumulate,
                            hipStream_t st);
hipError_t dtfk_slab_sum(const float* slabs, float* out, int S, long long n, int accumulate, hipStream_t st);
hipError_t dtfk_bias_gelu_fwd(const void* x, const float* bias, void* y, long long n, int H, hipStream_t st);
hipError_t dtfk_bias_gelu_bwd(const void* dy, const void* x, const float* bias, void* dx, float* part, int N, int H,
                              int row_slices, hipStream_t st);
hipError_t dtfk_softmax_fwd(const void* S, const float* mask, void* P, void* Pd, int rows, int Sk, int rows_per_batch,
                            float scale, float p, unsigned long long seed, hipStream_t st);
hipError_t dtfk_softmax_bwd(const void* dPd, const void* P, void* dS, int rows, int Sk, float scale, float p,
                            unsigned long long seed, hipStream_t st);
hipError_t dtfk_dropout_bf16(const void* x, void* y, long long n, float p, unsigned long long seed, hipStream_t st);
int dtfk_attn_supported(int S, int d);
hipError_t dtfk_attn_fwd(const void* qkv, const float* bias, const float* mask, void* ctx, float* lse, int B, int S,
                         int NH, float scale, float p, unsigned long long seed, hipStream_t st);
hipError_t dtfk_attn_bwd(const void* qkv, const float* bias, const float* mask, const void* ctx, const void* dctx,
                         const float* lse, float* Dbuf, void* dqkv, int B, int S, int NH, float scale, float p,
                         unsigned long long seed, float* bpart, hipStream_t st);
}

namespace dtf {
namespace {
hipStream_t cs() { return c10::hip::getCurrentHIPStream().stream(); }
void ck(hipError_t e, const char* w) {
  if (e != hipSuccess) throw std::runtime_error(std::string(w) + ": " + hipGetErrorString(e));
}
void req(const at::Tensor& t, at::ScalarType dt, const char* n) {
  if (!t.is_cuda()) throw std::runtime_error(std::string(n) + " must be a GPU tensor");
  if (t.scalar_type() != dt) throw std::runtime_error(std::string(n) + " has the wrong dtype");
  if (!t.is_contiguous()) throw std::runtime_error(std::string(n) + " must be contiguous");
}
void* optp(const c10::optional<at::Tensor>& t) { return t.has_value() ? t->data_ptr() : nullptr; }
float* optf(const c10::optional<at::Tensor>& t) { return t.has_value() ? t->data_ptr<float>() : nullptr; }
int rows_of(const at::Tensor& t, int H) { return (int)(t.numel() / H); }
}  // namespace

// y = LN(dropout(x + bias) + res) ; x, res, y, s bf16 [N, H]; bias/gamma/beta fp32 [H]
void bdrln_fwd(at::Tensor x, at::Tensor bias, c10::optional<at::Tensor> res, at::Tensor gamma, at::Tensor beta,
               at::Tensor y, c10::optional<at::Tensor> s, at::Tensor mean, at::Tensor rstd, double eps, double p,
               int64_t seed) {
  const int H = (int)x.size(-1);
  req(x, at::kBFloat16, "x"); req(y, at::kBFloat16, "y"); req(bias, at::kFloat, "bias");
  req(gamma, at::kFloat, "gamma"); req(beta, at::kFloat, "beta"); req(mean, at::kFloat, "mean");
  req(rstd, at::kFloat, "rstd");
  if (res.has_value()) req(*res, at::kBFloat16, "res");
  if (s.has_value()) req(*s, at::kBFloat16, "s");
  const int N = rows_of(x, H);
  if (mean.numel() < N || rstd.numel() < N || y.numel() != x.numel()) throw std::runtime_error("bdrln_fwd shapes");
  ck(dtfk_bdrln_fwd(x.data_ptr(), bias.data_ptr<float>(), optp(res), gamma.data_ptr<float>(), beta.data_ptr<float>(),
                    y.data_ptr(), optp(s), mean.data_ptr<float>(), rstd.data_ptr<float>(), N, H, (float)eps,
                    (float)p, (unsigned long long)seed, cs()),
     "bdrln_fwd");
}

void ln_fwd_f32in(at::Tensor x, at::Tensor gamma, at::Tensor beta, at::Tensor y, c10::optional<at::Tensor> s,
                  at::Tensor mean, at::Tensor rstd, double eps, double p, int64_t seed) {
  const int H = (int)x.size(-1);
  req(x, at::kFloat, "x"); req(y, at::kBFloat16, "y");
  if (s.has_value()) req(*s, at::kBFloat16, "s");
  const int N = rows_of(x, H);
  ck(dtfk_ln_fwd_f32in(x.data_ptr<float>(), gamma.data_ptr<float>(), beta.data_ptr<float>(), y.data_ptr(), optp(s),
                       mean.data_ptr<float>(), rstd.data_ptr<float>(), N, H, (float)eps, (float)p,
                       (unsigned long long)seed, cs()),
     "ln_fwd_f32in");
}

// BERT embedding block: y = dropout(LN(word[ids] + typ[tt] + pos[t % S])), s = bf16 of the sum
void emb_ln_fwd(at::Tensor word, at::Tensor ids, at::Tensor typ, at::Tensor tt, at::Tensor pos, int64_t S,
                at::Tensor gamma, at::Tensor beta, at::Tensor y, at::Tensor s, at::Tensor mean, at::Tensor rstd,
                double eps, double p, int64_t seed) {
  const int H = (int)word.size(-1);
  req(word, at::kFloat, "word"); req(typ, at::kFloat, "typ"); req(pos, at::kFloat, "pos");
  req(gamma, at::kFloat, "gamma"); req(beta, at::kFloat, "beta");
  req(y, at::kBFloat16, "y"); req(s, at::kBFloat16, "s"); req(mean, at::kFloat, "mean"); req(rstd, at::kFloat, "rstd");
  req(ids, at::kLong, "ids"); req(tt, at::kLong, "tt");
  const int64_t N = ids.numel();
  if (tt.numel() != N || y.numel() != N * H || s.numel() != N * H || mean.numel() < N || rstd.numel() < N ||
      typ.size(-1) != H || pos.size(-1) != H || pos.size(0) < S || S < 1 || N % S)
    throw std::runtime_error("emb_ln_fwd shapes");
  ck(dtfk_emb_ln_fwd(word.data_ptr<float>(), ids.data_ptr<int64_t>(), typ.data_ptr<float>(), tt.data_ptr<int64_t>(),
                     pos.data_ptr<float>(), (int)S, gamma.data_ptr<float>(), beta.data_ptr<float>(), y.data_ptr(),
                     s.data_ptr(), mean.data_ptr<float>(), rstd.data_ptr<float>(), (int)N, H, (float)eps, (float)p,
                     (unsigned long long)seed, cs()),
     "emb_ln_fwd");
}
// position / 2-row token-type gradients of the embedding block from ds [B*S, H] bf16:
// pos_grad rows [0, S) (+)= sum over b; typ_grad [2, H] (+)= per-type sums
void emb_bwd_aux(at::Tensor ds, at::Tensor tt, int64_t S, at::Tensor pos_grad, at::Tensor typ_grad, at::Tensor part,
                 bool accumulate) {
  const int H = (int)ds.size(-1);
  req(ds, at::kBFloat16, "ds"); req(tt, at::kLong, "tt"); req(pos_grad, at::kFloat, "pos_grad");
  req(typ_grad, at::kFloat, "typ_grad"); req(part, at::kFloat, "part");
  const int64_t N = tt.numel();
  if (S < 1 || N % S || ds.numel() != N * H || pos_grad.numel() < S * H || typ_grad.numel() < 2 * H ||
      part.numel() < 2 * S * H)
    throw std::runtime_error("emb_bwd_aux shapes");
  ck(dtfk_emb_bwd_aux(ds.data_ptr(), tt.data_ptr<int64_t>(), (int)(N / S), (int)S, H, pos_grad.data_ptr<float>(),
                      part.data_ptr<float>(), accumulate ? 1 : 0, cs()),
     "emb_bwd_aux");
  const float* parts[2] = {part.data_ptr<float>(), part.data_ptr<float>() + S * H};
  float* outs[2] = {typ_grad.data_ptr<float>(), typ_grad.data_ptr<float>() + H};
  ck(dtfk_colsum_partials_multi(parts, outs, 2, (int)S, H, accumulate ? 1 : 0, cs()), "emb_bwd_aux colsum");
}

// returns nothing; dgamma/dbeta/dbias (fp32 [H]) written if given
void ln_bwd(at::Tensor dy, at::Tensor s, at::Tensor mean, at::Tensor rstd, at::Tensor gamma, at::Tensor ds,
            c10::optional<at::Tensor> dxb, at::Tensor part, c10::optional<at::Tensor> dgamma,
            c10::optional<at::Tensor> dbeta, c10::optional<at::Tensor> dbias, double p, int64_t seed,
            bool accumulate) {
  const int H = (int)dy.size(-1);
  req(dy, at::kBFloat16, "dy"); req(s, at::kBFloat16, "s"); req(ds, at::kBFloat16, "ds");
  req(part, at::kFloat, "part");
  if (dxb.has_value()) req(*dxb, at::kBFloat16, "dxb");
  const int N = rows_of(dy, H);
  const int grid = (int)(part.numel() / (3LL * H));
  if (grid < 1) throw std::runtime_error("ln_bwd: partial buffer too small (needs 3*grid*H floats)");
  float* pg = part.data_ptr<float>();
  float* pb = pg + (size_t)grid * H;
  float* px = pb + (size_t)grid * H;
  ck(dtfk_ln_bwd(dy.data_ptr(), s.data_ptr(), mean.data_ptr<float>(), rstd.data_ptr<float>(), gamma.data_ptr<float>(),
                 ds.data_ptr(), optp(dxb), dgamma.has_value() ? pg : nullptr, dbeta.has_value() ? pb : nullptr,
                 dbias.has_value() ? px : nullptr, grid, N, H, (float)p, (unsigned long long)seed, cs()),
     "ln_bwd");
  // dgamma / dbeta / dbias: one finishing launch (accumulate: += into sunk .grad)
  const float* parts[3];
  float* outs[3];
  int nb = 0;
  auto add = [&](const c10::optional<at::Tensor>& t, const float* pp) {
    if (!t.has_value()) return;
    req(*t, at::kFloat, "param grad");
    if (t->numel() < H) throw std::runtime_error("ln_bwd: gradient output too small");
    parts[nb] = pp;
    outs[nb++] = t->data_ptr<float>();
  };
  add(dgamma, pg);
  add(dbeta, pb);
  add(dbias, px);
  if (nb) ck(dtfk_colsum_partials_multi(parts, outs, nb, grid, H, accumulate ? 1 : 0, cs()), "colsum");
}

// bias gradient of a bf16 [N, H] matrix: out (+)= column sums (part: P*H floats)
void colsum_bf16(at::Tensor x, at::Tensor part, at::Tensor out, bool accumulate) {
  req(x, at::kBFloat16, "x"); req(part, at::kFloat, "part"); req(out, at::kFloat, "out");
  const int H = (int)x.size(-1);
  const int N = rows_of(x, H);
  const int P = (int)(part.numel() / H);
  if (P < 1 || out.numel() < H) throw std::runtime_error("colsum_bf16 shapes");
  ck(dtfk_colsum_bf16(x.data_ptr(), part.data_ptr<float>(), out.data_ptr<float>(), N, H, P, accumulate ? 1 : 0, cs()),
     "colsum_bf16");
}

// out (+)= sum over the leading dim of slabs [S, n] (fp32; 16-byte vector path when aligned)
void slab_sum(at::Tensor slabs, at::Tensor out, bool accumulate) {
  req(slabs, at::kFloat, "slabs"); req(out, at::kFloat, "out");
  const int64_t n = out.numel();
  if (n == 0 || slabs.numel() % n) throw std::runtime_error("slab_sum shapes");
  if (!slabs.is_contiguous() || !out.is_contiguous()) throw std::runtime_error("slab_sum: contiguous tensors only");
  const int S = (int)(slabs.numel() / n);
  ck(dtfk_slab_sum(slabs.data_ptr<float>(), out.data_ptr<float>(), S, n, accumulate ? 1 : 0, cs()), "slab_sum");
}

void bias_gelu_fwd(at::Tensor x, at::Tensor bias, at::Tensor y) {
  req(x, at::kBFloat16, "x"); req(y, at::kBFloat16, "y"); req(bias, at::kFloat, "bias");
  const int H = (int)x.size(-1);
  if (H % 4) throw std::runtime_error("bias_gelu: H % 4 != 0");
  ck(dtfk_bias_gelu_fwd(x.data_ptr(), bias.data_ptr<float>(), y.data_ptr(), x.numel(), H, cs()), "bias_gelu_fwd");
}

void bias_gelu_bwd(at::Tensor dy, at::Tensor x, at::Tensor bias, at::Tensor dx, at::Tensor part, at::Tensor dbias,
                   bool accumulate) {
  req(dy, at::kBFloat16, "dy"); req(x, at::kBFloat16, "x"); req(dx, at::kBFloat16, "dx");
  req(part, at::kFloat, "part"); req(dbias, at::kFloat, "dbias");
  const int H = (int)x.size(-1);
  const int N = rows_of(x, H);
  const int slices = (int)(part.numel() / H);
  if (slices < 1 || H % 4) throw std::runtime_error("bias_gelu_bwd shapes");
  ck(dtfk_bias_gelu_bwd(dy.data_ptr(), x.data_ptr(), bias.data_ptr<float>(), dx.data_ptr(), part.data_ptr<float>(), N,
                        H, slices, cs()),
     "bias_gelu_bwd");
  const float* pp[1] = {part.data_ptr<float>()};
  float* po[1] = {dbias.data_ptr<float>()};
  ck(dtfk_colsum_partials_multi(pp, po, 1, slices, H, accumulate ? 1 : 0, cs()), "colsum");
}

void softmax_fwd(at::Tensor S, c10::optional<at::Tensor> mask, at::Tensor P, c10::optional<at::Tensor> Pd,
                 int64_t rows_per_batch, double scale, double p, int64_t seed) {
  req(S, at::kBFloat16, "S"); req(P, at::kBFloat16, "P");
  if (Pd.has_value()) req(*Pd, at::kBFloat16, "Pd");
  if (mask.has_value()) req(*mask, at::kFloat, "mask");
  const int Sk = (int)S.size(-1);
  const int rows = (int)(S.numel() / Sk);
  ck(dtfk_softmax_fwd(S.data_ptr(), optf(mask), P.data_ptr(), optp(Pd), rows, Sk, (int)rows_per_batch, (float)scale,
                      (float)p, (unsigned long long)seed, cs()),
     "softmax_fwd");
}

void softmax_bwd(at::Tensor dPd, at::Tensor P, at::Tensor dS, double scale, double p, int64_t seed) {
  req(dPd, at::kBFloat16, "dPd"); req(P, at::kBFloat16, "P"); req(dS, at::kBFloat16, "dS");
  const int Sk = (int)P.size(-1);
  const int rows = (int)(P.numel() / Sk);
  ck(dtfk_softmax_bwd(dPd.data_ptr(), P.data_ptr(), dS.data_ptr(), rows, Sk, (float)scale, (float)p,
                      (unsigned long long)seed, cs()),
     "softmax_bwd");
}

void dropout_bf16(at::Tensor x, at::Tensor y, double p, int64_t seed) {
  req(x, at::kBFloat16, "x"); req(y, at::kBFloat16, "y");
  if (x.numel() % 4) throw std::runtime_error("dropout_bf16: numel % 4 != 0");
  ck(dtfk_dropout_bf16(x.data_ptr(), y.data_ptr(), x.numel(), (float)p, (unsigned long long)seed, cs()), "dropout");
}

// qkv [B, S, 3*NH*64] bf16 (pre-bias projection), bias [3*NH*64] fp32 or None,
// mask [B, S] additive fp32 or None -> ctx [B, S, NH*64] bf16, lse [B, NH, S] fp32
void attn_check(const at::Tensor& qkv, const c10::optional<at::Tensor>& bias, const c10::optional<at::Tensor>& mask,
                int64_t NH) {
  req(qkv, at::kBFloat16, "qkv");
  if (qkv.dim() != 3 || qkv.size(2) != 3 * NH * 64) throw std::runtime_error("attn: qkv must be [B, S, 3*NH*64]");
  if (!dtfk_attn_supported((int)qkv.size(1), 64)) throw std::runtime_error("attn: unsupported sequence length");
  if (bias.has_value()) {
    req(*bias, at::kFloat, "bias");
    if (bias->numel() != qkv.size(2)) throw std::runtime_error("attn: bias size");
  }
  if (mask.has_value()) {
    req(*mask, at::kFloat, "mask");
    if (mask->numel() != qkv.size(0) * qkv.size(1)) throw std::runtime_error("attn: mask must be [B, S]");
  }
}

void attn_fwd(at::Tensor qkv, c10::optional<at::Tensor> bias, c10::optional<at::Tensor> mask, at::Tensor ctx,
              at::Tensor lse, int64_t NH, double scale, double p, int64_t seed) {
  attn_check(qkv, bias, mask, NH);
  const int64_t B = qkv.size(0), S = qkv.size(1);
  req(ctx, at::kBFloat16, "ctx"); req(lse, at::kFloat, "lse");
  if (ctx.numel() != B * S * NH * 64 || lse.numel() != B * NH * S) throw std::runtime_error("attn_fwd: output sizes");
  ck(dtfk_attn_fwd(qkv.data_ptr(), optf(bias), optf(mask), ctx.data_ptr(), lse.data_ptr<float>(), (int)B, (int)S,
                   (int)NH, (float)scale, (float)p, (unsigned long long)seed, cs()),
     "attn_fwd");
}

// dbias (optional, with bpart [B * S / 16, 3 * NH * 64] fp32 scratch): the qkv
// bias gradient = column sums of dqkv, from per-wave partial sums the backward
// kernels write (no pass over dqkv); accumulate: dbias +=.
void attn_bwd(at::Tensor qkv, c10::optional<at::Tensor> bias, c10::optional<at::Tensor> mask, at::Tensor ctx,
              at::Tensor dctx, at::Tensor lse, at::Tensor Dbuf, at::Tensor dqkv, int64_t NH, double scale, double p,
              int64_t seed, c10::optional<at::Tensor> bpart, c10::optional<at::Tensor> dbias, bool accumulate) {
  attn_check(qkv, bias, mask, NH);
  const int64_t B = qkv.size(0), S = qkv.size(1);
  req(ctx, at::kBFloat16, "ctx"); req(dctx, at::kBFloat16, "dctx"); req(dqkv, at::kBFloat16, "dqkv");
  req(lse, at::kFloat, "lse"); req(Dbuf, at::kFloat, "Dbuf");
  if (ctx.numel() != B * S * NH * 64 || dctx.numel() != ctx.numel() || dqkv.numel() != qkv.numel() ||
      lse.numel() != B * NH * S || Dbuf.numel() != lse.numel())
    throw std::runtime_error("attn_bwd: sizes");
  const int64_t H3 = 3 * NH * 64, P = B * S / 16;
  if (bpart.has_value() != dbias.has_value()) throw std::runtime_error("attn_bwd: bpart and dbias go together");
  if (bpart.has_value()) {
    req(*bpart, at::kFloat, "bpart"); req(*dbias, at::kFloat, "dbias");
    if (bpart->numel() < P * H3 || dbias->numel() != H3 || !dbias->is_contiguous())
      throw std::runtime_error("attn_bwd: bpart needs B*S/16 x 3*NH*64 floats, dbias 3*NH*64");
  }
  ck(dtfk_attn_bwd(qkv.data_ptr(), optf(bias), optf(mask), ctx.data_ptr(), dctx.data_ptr(), lse.data_ptr<float>(),
                   Dbuf.data_ptr<float>(), dqkv.data_ptr(), (int)B, (int)S, (int)NH, (float)scale, (float)p,
                   (unsigned long long)seed, bpart.has_value() ? bpart->data_ptr<float>() : nullptr, cs()),
     "attn_bwd");
  if (bpart.has_value()) {
    const float* pp[1] = {bpart->data_ptr<float>()};
    float* po[1] = {dbias->data_ptr<float>()};
    ck(dtfk_colsum_partials_multi(pp, po, 1, (int)P, (int)H3, accumulate ? 1 : 0, cs()), "attn_bwd dbias");
  }
}

void init_transformer(pybind11::module& m) {
  m.def("attn_supported", [](int64_t S, int64_t d) { return dtfk_attn_supported((int)S, (int)d) != 0; });
  m.def("attn_fwd", &attn_fwd);
  m.def("attn_bwd", &attn_bwd, py::arg("qkv"), py::arg("bias"), py::arg("mask"), py::arg("ctx"), py::arg("dctx"),
        py::arg("lse"), py::arg("Dbuf"), py::arg("dqkv"), py::arg("NH"), py::arg("scale"), py::arg("p"),
        py::arg("seed"), py::arg("bpart") = py::none(), py::arg("dbias") = py::none(), py::arg("accumulate") = false);
  m.def("bdrln_fwd", &bdrln_fwd);
  m.def("ln_fwd_f32in", &ln_fwd_f32in);
  m.def("emb_ln_fwd", &emb_ln_fwd);
  m.def("emb_bwd_aux", &emb_bwd_aux);
  m.def("ln_bwd", &ln_bwd, py::arg("dy"), py::arg("s"), py::arg("mean"), py::arg("rstd"), py::arg("gamma"),
        py::arg("ds"), py::arg("dxb"), py::arg("part"), py::arg("dgamma"), py::arg("dbeta"), py::arg("dbias"),
        py::arg("p"), py::arg("seed"), py::arg("accumulate") = false);
  m.def("colsum_bf16", &colsum_bf16, py::arg("x"), py::arg("part"), py::arg("out"), py::arg("accumulate") = false);
  m.def("slab_sum", &slab_sum, py::arg("slabs"), py::arg("out"), py::arg("accumulate") = false);
  m.def("bias_gelu_fwd", &bias_gelu_fwd);
  m.def("bias_gelu_bwd", &bias_gelu_bwd, py::arg("dy"), py::arg("x"), py::arg("bias"), py::arg("dx"), py::arg("part"),
        py::arg("dbias"), py::arg("accumulate") = false);
  m.def("softmax_fwd", &softmax_fwd);
  m.def("softmax_bwd", &softmax_bwd);
  m.def("dropout_bf16", &dropout_bf16);
}

}  // namespace dtf

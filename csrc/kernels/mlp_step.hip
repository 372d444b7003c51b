// Fused training step for the reference's 784-100-10 MLP
// (reference: example.py:84-118 -- x*W1+b1 -> sigmoid -> *W2+b2 -> softmax ->
// -sum(y log y_hat) mean -> GradientDescentOptimizer.minimize).
//
// MI355X design (not a translation of the TF graph): the whole step is three
// launches that a hipGraph replays back to back.
//
//   A  mlp_rows_fwd_bwd   one 512-thread block per 16 batch rows.  Layer-1 GEMM
//                         on 16x16x32 bf16 MFMA (W1 read from a bf16 shadow laid
//                         out K-contiguous so every B fragment is one 16-byte
//                         load), fused bias+activation epilogue, layer-2 MFMA,
//                         softmax cross-entropy (stable log-sum-exp), backward
//                         through layer 2 and the activation, per-block partial
//                         dW2/db1/db2 slabs, and K-major (transposed) copies of
//                         x and dz2 so the weight-gradient GEMM gets contiguous
//                         fragments too.
//   B  mlp_wgrad          dW1 = x^T dz2 on MFMA, one wave per 16-row strip of
//                         dW1 (all 7 column tiles share the A fragment).  The
//                         last block reduces block A's slabs (deterministic, no
//                         atomics) and writes loss/accuracy into a device-side
//                         metrics ring and bumps the device global_step.
//                         mode FUSED (1 GPU): SGD is applied in the epilogue and
//                         the bf16 shadows refreshed -- no gradient round trip.
//                         mode GRAD: gradients go to one flat bucket (fp32 or
//                         bf16) for the RCCL all-reduce.
//   C  mlp_apply_flat     after the all-reduce: p -= lr*scale*g over the flat
//                         bucket + shadow refresh (also used to build shadows
//                         after init / checkpoint restore with g = nullptr).
//
// Flat parameter layout == TF variable order of example.py:
//   W1 [784,100] @0, W2 [100,10] @78400, b1 [100] @79400, b2 [10] @79500.
#include "common.h"

namespace dtfk {
namespace mlp {

constexpr int DIN = 784, DINP = 800;   // K of layer 1, padded to 25*32
constexpr int HID = 100, HIDP = 112;   // N of layer 1 (7 MFMA col tiles)
constexpr int HIDK = 128;              // K of layer 2 padded to 4*32
constexpr int NCLS = 10;
constexpr int OFF_W1 = 0, OFF_W2 = 78400, OFF_B1 = 79400, OFF_B2 = 79500;
constexpr int NPARAM = 79510;
constexpr int PART = 1112;             // dW2(1000) db1(100) db2(10) loss correct
constexpr int XS = 808;                // LDS row stride (bf16) of the x tile
constexpr int A2S = 136;               // LDS row stride (bf16) of a2
constexpr int ROWS = 16;

__global__ __launch_bounds__(512) void mlp_rows_fwd_bwd(
    const uint8_t* __restrict__ xin, int x_kind, const uint8_t* __restrict__ labels, int B,
    const uint16_t* __restrict__ W1T, const uint16_t* __restrict__ W2T,
    const float* __restrict__ params, uint16_t* __restrict__ xT, uint16_t* __restrict__ dz2T,
    int BP, float* __restrict__ partials, float inv_batch, int act, int naive_loss) {
  __shared__ __attribute__((aligned(16))) uint16_t xs[ROWS * XS];
  __shared__ __attribute__((aligned(16))) uint16_t a2b[ROWS * A2S];
  __shared__ float a2f[ROWS * HIDK];
  __shared__ float dz3s[ROWS * 16];
  __shared__ float dz2s[ROWS * HIDP];
  __shared__ float red[2];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 15, lh = lane >> 4;
  const int r0 = blockIdx.x * ROWS;

  // (1) Issue this wave's whole W1 column-tile stream first (25 x 16 B per
  // lane); its latency hides under the x staging below.
  bf16x8 bw[25];
  if (wave < 7) {
    const uint16_t* p = W1T + (size_t)(wave * 16 + lr) * DINP + lh * 8;
#pragma unroll
    for (int ks = 0; ks < 25; ++ks) bw[ks] = ld_bf16x8(p + ks * 32);
  }

  // (2) Stage 16 rows of x as bf16 in LDS (zero K-pad / rows past B).
  for (int i = tid; i < ROWS * (DINP / 8); i += 512) {
    const int r = i / (DINP / 8), c8 = (i % (DINP / 8)) * 8;
    const int row = r0 + r;
    float v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (row < B && c8 < DIN) {
      const size_t e = (size_t)row * DIN + c8;
      if (x_kind == 0) {
        const uint2 u = *reinterpret_cast<const uint2*>(xin + e);
        const float s = 1.f / 255.f;
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = (float)((u.x >> (8 * j)) & 255u) * s;
#pragma unroll
        for (int j = 0; j < 4; ++j) v[4 + j] = (float)((u.y >> (8 * j)) & 255u) * s;
      } else if (x_kind == 1) {
        const float4* f = reinterpret_cast<const float4*>(reinterpret_cast<const float*>(xin) + e);
        const float4 a = f[0], b = f[1];
        v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
        v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
      } else {
        const uint4 u = *reinterpret_cast<const uint4*>(reinterpret_cast<const uint16_t*>(xin) + e);
        const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) { v[2 * j] = bf2f(w[j] & 0xffff); v[2 * j + 1] = bf2f(w[j] >> 16); }
      }
    }
    uint4 o;
    o.x = pack2bf(v[0], v[1]); o.y = pack2bf(v[2], v[3]);
    o.z = pack2bf(v[4], v[5]); o.w = pack2bf(v[6], v[7]);
    *reinterpret_cast<uint4*>(&xs[r * XS + c8]) = o;
  }
  __syncthreads();

  // (3) x^T for the weight-gradient GEMM: xT[k][r0 + 8h .. +8], one 16-B store.
  for (int i = tid; i < DIN * 2; i += 512) {
    const int k = i >> 1, h = i & 1;
    uint32_t w[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
      w[j] = (uint32_t)xs[(8 * h + 2 * j) * XS + k] | ((uint32_t)xs[(8 * h + 2 * j + 1) * XS + k] << 16);
    *reinterpret_cast<uint4*>(&xT[(size_t)k * BP + r0 + 8 * h]) = make_uint4(w[0], w[1], w[2], w[3]);
  }

  // (4) Layer 1: z2 = x W1 + b1, a2 = act(z2). Wave w owns column tile w.
  if (wave < 7) {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    const uint16_t* xa = xs + lr * XS + lh * 8;
#pragma unroll
    for (int ks = 0; ks < 25; ++ks) acc = mfma16x16x32(ld_bf16x8(xa + ks * 32), bw[ks], acc);
    const int n = wave * 16 + lr;
    const float bias = n < HID ? params[OFF_B1 + n] : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = 4 * lh + i;
      const float z = acc[i] + bias;
      float a = act == 0 ? sigmoidf_(z) : fmaxf(z, 0.f);
      if (n >= HID || r0 + r >= B) a = 0.f;
      a2f[r * HIDK + n] = a;
      a2b[r * A2S + n] = f2bf(a);
    }
  } else {
    for (int i = lane; i < ROWS * 16; i += 64) {
      const int r = i >> 4, c = HIDP + (i & 15);
      a2f[r * HIDK + c] = 0.f;
      a2b[r * A2S + c] = 0;
    }
  }
  __syncthreads();

  // (5) Layer 2 + softmax cross-entropy + dz3 (wave 0).
  if (wave == 0) {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < HIDK / 32; ++ks) {
      const bf16x8 a = ld_bf16x8(a2b + lr * A2S + ks * 32 + lh * 8);
      const bf16x8 b = ld_bf16x8(W2T + lr * HIDK + ks * 32 + lh * 8);
      acc = mfma16x16x32(a, b, acc);
    }
    const int c = lr;
    const bool cv = c < NCLS;
    const float b2 = cv ? params[OFF_B2 + c] : 0.f;
    float lsum = 0.f, csum = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = 4 * lh + i, row = r0 + r;
      const bool valid = row < B;
      const float z = acc[i] + b2;
      const float v = cv ? z : -3.0e38f;
      const float m = group16_max(v);
      const float e = cv ? __expf(v - m) : 0.f;
      const float s = group16_sum(e);
      const float p = e / s;
      int y = valid ? (int)labels[row] : 0;
      y = y < NCLS ? y : 0;  // corrupt label ids never index past the row group
      const int src = (lane & 48) | y;
      const float zy = __shfl(z, src, 64);
      const float py = __shfl(p, src, 64);
      // tf.argmax picks the first maximal index
      float cand = (cv && v == m) ? (float)c : 1e9f;
#pragma unroll
      for (int off = 8; off > 0; off >>= 1) cand = fminf(cand, __shfl_xor(cand, off, 16));
      const float loss = naive_loss ? -__logf(py) : (m + __logf(s) - zy);
      dz3s[r * 16 + c] = (valid && cv) ? (p - (c == y ? 1.f : 0.f)) * inv_batch : 0.f;
      if (c == 0 && valid) { lsum += loss; csum += ((int)cand == y) ? 1.f : 0.f; }
    }
    lsum = wave_sum(lsum);
    csum = wave_sum(csum);
    if (lane == 0) { red[0] = lsum; red[1] = csum; }
  }
  __syncthreads();

  // (6) dz2 = (dz3 W2^T) * act'(z2)
  for (int i = tid; i < ROWS * HIDP; i += 512) {
    const int r = i / HIDP, n = i % HIDP;
    float d = 0.f;
    if (n < HID && r0 + r < B) {
      float s = 0.f;
#pragma unroll
      for (int c = 0; c < NCLS; ++c) s += dz3s[r * 16 + c] * params[OFF_W2 + n * NCLS + c];
      const float a = a2f[r * HIDK + n];
      d = act == 0 ? s * a * (1.f - a) : (a > 0.f ? s : 0.f);
    }
    dz2s[r * HIDP + n] = d;
  }
  __syncthreads();

  // (7) dz2^T (bf16) for the weight-gradient GEMM, and this block's partials.
  if (tid < HIDP * 2) {
    const int n = tid >> 1, h = tid & 1;
    uint32_t w[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
      w[j] = pack2bf(dz2s[(8 * h + 2 * j) * HIDP + n], dz2s[(8 * h + 2 * j + 1) * HIDP + n]);
    *reinterpret_cast<uint4*>(&dz2T[(size_t)n * BP + r0 + 8 * h]) = make_uint4(w[0], w[1], w[2], w[3]);
  }
  float* part = partials + (size_t)blockIdx.x * PART;
  for (int i = tid; i < 1110; i += 512) {
    float s = 0.f;
    if (i < 1000) {
      const int n = i / NCLS, c = i % NCLS;
#pragma unroll
      for (int r = 0; r < ROWS; ++r) s += a2f[r * HIDK + n] * dz3s[r * 16 + c];
    } else if (i < 1100) {
      const int n = i - 1000;
#pragma unroll
      for (int r = 0; r < ROWS; ++r) s += dz2s[r * HIDP + n];
    } else {
      const int c = i - 1100;
#pragma unroll
      for (int r = 0; r < ROWS; ++r) s += dz3s[r * 16 + c];
    }
    part[i] = s;
  }
  if (tid == 0) { part[1110] = red[0]; part[1111] = red[1]; }
}

// grad_kind: 0 = fused SGD update, 1 = fp32 grads, 2 = bf16 grads
__global__ __launch_bounds__(256) void mlp_wgrad(
    const uint16_t* __restrict__ xT, const uint16_t* __restrict__ dz2T, int BP, int B,
    const float* __restrict__ partials, int nblk_rows, float* __restrict__ params,
    uint16_t* __restrict__ W1T, uint16_t* __restrict__ W2T, void* __restrict__ grads, int grad_kind,
    const float* __restrict__ lr_ptr, float* __restrict__ metrics, long long* __restrict__ gstep,
    int ring) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 15, lh = lane >> 4;
  const float lrate = *lr_ptr;
  constexpr int NSTRIP = DIN / 16;  // 49
  const int nstrip_blocks = (NSTRIP + 3) / 4;

  if ((int)blockIdx.x < nstrip_blocks) {
    const int s = blockIdx.x * 4 + wave;
    if (s >= NSTRIP) return;
    const int k0 = s * 16;
    f32x4 acc[7];
#pragma unroll
    for (int t = 0; t < 7; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    const uint16_t* pa = xT + (size_t)(k0 + lr) * BP + lh * 8;
    const uint16_t* pb = dz2T + (size_t)lr * BP + lh * 8;
    for (int kb = 0; kb < BP; kb += 32) {
      const bf16x8 a = ld_bf16x8(pa + kb);
      bf16x8 b[7];
#pragma unroll
      for (int t = 0; t < 7; ++t) b[t] = ld_bf16x8(pb + (size_t)t * 16 * BP + kb);
#pragma unroll
      for (int t = 0; t < 7; ++t) acc[t] = mfma16x16x32(a, b[t], acc[t]);
    }
#pragma unroll
    for (int t = 0; t < 7; ++t) {
      const int n = t * 16 + lr;
      if (n >= HID) continue;
      const int kr = k0 + 4 * lh;
      if (grad_kind == 0) {
        float p[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          float* q = &params[OFF_W1 + (kr + i) * HID + n];
          p[i] = *q - lrate * acc[t][i];
          *q = p[i];
        }
        *reinterpret_cast<uint2*>(&W1T[(size_t)n * DINP + kr]) =
            make_uint2(pack2bf(p[0], p[1]), pack2bf(p[2], p[3]));
      } else if (grad_kind == 1) {
        float* g = reinterpret_cast<float*>(grads);
#pragma unroll
        for (int i = 0; i < 4; ++i) g[OFF_W1 + (kr + i) * HID + n] = acc[t][i];
      } else {
        uint16_t* g = reinterpret_cast<uint16_t*>(grads);
#pragma unroll
        for (int i = 0; i < 4; ++i) g[OFF_W1 + (kr + i) * HID + n] = f2bf(acc[t][i]);
      }
    }
    return;
  }

  // Reducer block: small-parameter gradients, metrics, global_step.
  for (int i = tid; i < 1110; i += 256) {
    float s = 0.f;
    for (int b = 0; b < nblk_rows; ++b) s += partials[(size_t)b * PART + i];
    if (grad_kind == 0) {
      const float p = params[OFF_W2 + i] - lrate * s;
      params[OFF_W2 + i] = p;
      if (i < 1000) W2T[(i % NCLS) * HIDK + i / NCLS] = f2bf(p);
    } else if (grad_kind == 1) {
      reinterpret_cast<float*>(grads)[OFF_W2 + i] = s;
    } else {
      reinterpret_cast<uint16_t*>(grads)[OFF_W2 + i] = f2bf(s);
    }
  }
  if (tid == 0) {
    float l = 0.f, c = 0.f;
    for (int b = 0; b < nblk_rows; ++b) { l += partials[(size_t)b * PART + 1110]; c += partials[(size_t)b * PART + 1111]; }
    const long long st = *gstep;
    const int slot = (int)(st % ring);
    metrics[2 * slot] = l / (float)B;
    metrics[2 * slot + 1] = c / (float)B;
    *gstep = st + 1;
  }
}

__global__ __launch_bounds__(256) void mlp_apply_flat(
    float* __restrict__ params, const void* __restrict__ grads, int grad_kind,
    const float* __restrict__ lr_ptr, float scale, uint16_t* __restrict__ W1T,
    uint16_t* __restrict__ W2T) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= NPARAM) return;
  float p = params[i];
  if (grads != nullptr) {
    const float g = grad_kind == 1 ? reinterpret_cast<const float*>(grads)[i]
                                   : bf2f(reinterpret_cast<const uint16_t*>(grads)[i]);
    p -= (*lr_ptr) * scale * g;
    params[i] = p;
  }
  if (i < OFF_W2) {
    W1T[(size_t)(i % HID) * DINP + i / HID] = f2bf(p);
  } else if (i < OFF_B1) {
    const int j = i - OFF_W2;
    W2T[(j % NCLS) * HIDK + j / NCLS] = f2bf(p);
  }
}

}  // namespace mlp
}  // namespace dtfk

// ---------------------------------------------------------------- launchers
extern "C" {

int dtfk_mlp_nblk_rows(int B) { return (B + 15) / 16; }
int dtfk_mlp_bp(int B) { return ((B + 31) / 32) * 32; }

hipError_t dtfk_mlp_fwd_bwd(const void* x, int x_kind, const void* labels, int B,
                            const void* W1T, const void* W2T, const float* params, void* xT,
                            void* dz2T, int BP, float* partials, float inv_batch, int act,
                            int naive_loss, hipStream_t stream) {
  using namespace dtfk::mlp;
  const int nb = (B + 15) / 16;
  hipLaunchKernelGGL(mlp_rows_fwd_bwd, dim3(nb), dim3(512), 0, stream,
                     (const uint8_t*)x, x_kind, (const uint8_t*)labels, B, (const uint16_t*)W1T,
                     (const uint16_t*)W2T, params, (uint16_t*)xT, (uint16_t*)dz2T, BP, partials,
                     inv_batch, act, naive_loss);
  return hipGetLastError();
}

hipError_t dtfk_mlp_wgrad(const void* xT, const void* dz2T, int BP, int B, const float* partials,
                          float* params, void* W1T, void* W2T, void* grads, int grad_kind,
                          const float* lr, float* metrics, long long* gstep, int ring,
                          hipStream_t stream) {
  using namespace dtfk::mlp;
  const int nstrip_blocks = (DIN / 16 + 3) / 4;
  hipLaunchKernelGGL(mlp_wgrad, dim3(nstrip_blocks + 1), dim3(256), 0, stream,
                     (const uint16_t*)xT, (const uint16_t*)dz2T, BP, B, partials, (B + 15) / 16,
                     params, (uint16_t*)W1T, (uint16_t*)W2T, grads, grad_kind, lr, metrics, gstep,
                     ring);
  return hipGetLastError();
}

hipError_t dtfk_mlp_apply_flat(float* params, const void* grads, int grad_kind, const float* lr,
                               float scale, void* W1T, void* W2T, hipStream_t stream) {
  using namespace dtfk::mlp;
  hipLaunchKernelGGL(mlp_apply_flat, dim3((NPARAM + 255) / 256), dim3(256), 0, stream, params,
                     grads, grad_kind, lr, scale, (uint16_t*)W1T, (uint16_t*)W2T);
  return hipGetLastError();
}

}  // extern "C"

// Large-batch MLP step (784-100-10, example.py:69-128): three launches.
//
// The fused / persistent engines (mlp_step.hip, mlp_persist_f32.hip) are
// latency engines for the reference's batch of 100: one wave owns a 16x16
// weight-gradient tile and contracts the whole batch serially -- right at
// B=100, 4x too slow at B=4096 (424 us/step).  The generic fp32 GEMM is no
// better here: [B,784]x[784,100] has 2*ceil(B/64) 64x64 tiles, i.e. 32 f32-MFMA
// workgroups at B=1024 (57 us, rocprofv3).  This step is shaped for the batch:
//
//   mlpg_fwd    one workgroup per 64 rows (4 waves x 16 rows x all 112 hidden
//               columns): z = x W1 on bf16 MFMA with W1 as an exact 3-way bf16
//               split (hi + mid + lo == the fp32 weight; uint8 pixels are exact
//               in bf16) -> exact products, fp32 accumulate; then, per row and
//               without leaving the workgroup, a2 = act(z/255 + b1), logits,
//               softmax-xent, dlog, dz2 = (dlog W2^T) act'(a2), and this block's
//               partial dW2 / db1 / db2 / loss / correct (slab P1).  dz2 leaves
//               as its exact 3-way split, hidden-major [3][112][BP] bf16.
//   mlpg_wgrad  dW1 = x^T dz2 / 255 over a (pixel block x batch chunk) grid:
//               x tiles transposed into LDS as bf16, dz2 split from LDS,
//               3 MFMAs per tile and k-step; one fp32 slab per batch chunk (P2).
//   mlpg_apply  sums the slabs in a fixed order (deterministic), SGD, refreshes
//               the W1 split, metrics ring + global step.  N > 1: the same
//               kernel first writes the reduced gradient (RCCL all-reduce), then
//               applies it.
//
// Every staged operand goes global -> registers (one k-step ahead) -> LDS
// (double-buffered, one barrier per k-step).
#include "common.h"

namespace dtfk {
namespace mlpg {

constexpr int DIN = 784, DINP = 800, HID = 100, HIDP = 112, NCLS = 10;
constexpr int OFF_W2 = 78400, OFF_B1 = 79400, OFF_B2 = 79500, NPARAM = 79510;
constexpr int KSTEPS = DINP / 32;          // 25
constexpr int BLD = 40;                    // LDS row stride (bf16) of a staged 32-wide k slice
constexpr int SLICE = 3 * HIDP * BLD;      // one staged [3][112][32] slice
constexpr int SLICE_CHUNKS = 3 * HIDP * 4; // 16-byte chunks per slice (1344)
constexpr int R1 = 64;                     // rows per mlpg_fwd block
constexpr int ALD = 101;                   // LDS row stride (fp32) of a2 / dz2 (odd: row-varying reads conflict-free)
constexpr int P1N = 1112;                  // [dW2 1000 | db1 100 | db2 10 | loss | correct]
constexpr int XTLD = 40;                   // LDS row stride (bf16) of a transposed x tile [64 px][32 batch]

__device__ __forceinline__ bf16x8 u8x8_to_bf16(uint2 w) {
  // integers 0..255 are exact in bf16
  uint32_t p[4];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const uint32_t v = j == 0 ? w.x : w.y;
    p[2 * j] = pack2bf((float)(v & 255u), (float)((v >> 8) & 255u));
    p[2 * j + 1] = pack2bf((float)((v >> 16) & 255u), (float)(v >> 24));
  }
  return __builtin_bit_cast(bf16x8, make_uint4(p[0], p[1], p[2], p[3]));
}

// fp32 -> hi + mid + lo bf16, exact for normal values (8 + 8 + 8 mantissa bits)
__device__ __forceinline__ void split3(float v, uint16_t& h, uint16_t& m, uint16_t& l) {
  h = f2bf(v);
  const float r1 = v - bf2f(h);
  m = f2bf(r1);
  l = f2bf(r1 - bf2f(m));
}

// [3][112][ld] bf16 operand, 32-wide k slice at column k0 -> registers
__device__ __forceinline__ void load_slice(const uint16_t* __restrict__ src, long long ld, int k0, uint4 (&v)[6]) {
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const int c = threadIdx.x + 256 * i;
    if (c < SLICE_CHUNKS) {
      const int row = c >> 2, q = c & 3;   // row = s * 112 + n
      v[i] = *reinterpret_cast<const uint4*>(src + (size_t)row * ld + k0 + 8 * q);
    }
  }
}
__device__ __forceinline__ void store_slice(uint16_t* dst, const uint4 (&v)[6]) {
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const int c = threadIdx.x + 256 * i;
    if (c < SLICE_CHUNKS) *reinterpret_cast<uint4*>(dst + (c >> 2) * BLD + 8 * (c & 3)) = v[i];
  }
}

__global__ __launch_bounds__(256) void mlpg_fwd(const uint8_t* __restrict__ x, const uint8_t* __restrict__ labels,
                                                int B, int BP, const uint16_t* __restrict__ W1S,
                                                const float* __restrict__ params, float* __restrict__ P1,
                                                uint16_t* __restrict__ dz2S, int act, int naive, float gscale,
                                                int stop) {
  __shared__ __attribute__((aligned(16))) uint16_t bs[2 * SLICE];   // 53.8 KB; a2 / dz2 after the K loop
  __shared__ float w2[HID * NCLS], b2[NCLS], lg[R1][NCLS + 1], dl[R1][NCLS + 1], red[2][R1];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int r0 = blockIdx.x * R1;
  const int row = r0 + wave * 16 + (lane & 15);
  const int kq = 8 * (lane >> 4);
  const uint8_t* xr = x + (size_t)min(row, B - 1) * DIN;
  for (int i = t; i < HID * NCLS; i += 256) w2[i] = params[OFF_W2 + i];
  if (t < NCLS) b2[t] = params[OFF_B2 + t];

  f32x4 acc[7];
#pragma unroll
  for (int j = 0; j < 7; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  uint4 v[6];
  uint2 xa = make_uint2(0u, 0u);
  load_slice(W1S, DINP, 0, v);
  if (row < B) xa = *reinterpret_cast<const uint2*>(xr + kq);
  for (int ks = 0; ks < KSTEPS; ++ks) {
    uint16_t* cur = bs + (ks & 1) * SLICE;
    store_slice(cur, v);
    const bf16x8 a = u8x8_to_bf16(xa);
    __syncthreads();
    if (ks + 1 < KSTEPS) {
      load_slice(W1S, DINP, (ks + 1) * 32, v);
      const int k = (ks + 1) * 32 + kq;
      xa = (row < B && k < DIN) ? *reinterpret_cast<const uint2*>(xr + k) : make_uint2(0u, 0u);
    }
    const uint16_t* bl = cur + (lane & 15) * BLD + kq;
#pragma unroll
    for (int j = 0; j < 7; ++j) {
#pragma unroll
      for (int s = 0; s < 3; ++s) acc[j] = mfma16x16x32(a, ld_bf16x8(bl + (s * HIDP + j * 16) * BLD), acc[j]);
    }
  }
  __syncthreads();   // the slices are dead: a2 / dz2 reuse the LDS
  float* a2s = reinterpret_cast<float*>(bs);
  float* dzs = a2s + R1 * ALD;
#pragma unroll
  for (int j = 0; j < 7; ++j) {
    const int h = j * 16 + (lane & 15);
    if (h < HID) {
      const float bb = params[OFF_B1 + h];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float z = acc[j][i] * (1.f / 255.f) + bb;
        a2s[(wave * 16 + 4 * (lane >> 4) + i) * ALD + h] = act == 0 ? sigmoidf_(z) : fmaxf(z, 0.f);
      }
    }
  }
  __syncthreads();
  if (stop == 1) return;
  for (int o = t; o < R1 * NCLS; o += 256) {   // logits
    const int r = o / NCLS, c = o % NCLS;
    float s = b2[c];
#pragma unroll 10
    for (int h = 0; h < HID; ++h) s = fmaf(a2s[r * ALD + h], w2[h * NCLS + c], s);
    lg[r][c] = s;
  }
  __syncthreads();
  if (t < R1) {   // softmax-xent of row t
    float loss = 0.f, corr = 0.f;
    if (r0 + t < B) {
      const int y = labels[r0 + t];
      float m = lg[t][0];
      int am = 0;
      for (int c = 1; c < NCLS; ++c)
        if (lg[t][c] > m) { m = lg[t][c]; am = c; }
      float s = 0.f;
      for (int c = 0; c < NCLS; ++c) s += __expf(lg[t][c] - m);
      const float inv = 1.f / s;
      loss = naive ? -__logf(__expf(lg[t][y] - m) * inv) : (m + __logf(s)) - lg[t][y];
      corr = am == y ? 1.f : 0.f;
      for (int c = 0; c < NCLS; ++c) dl[t][c] = (__expf(lg[t][c] - m) * inv - (c == y ? 1.f : 0.f)) * gscale;
    } else {
      for (int c = 0; c < NCLS; ++c) dl[t][c] = 0.f;
    }
    red[0][t] = loss;
    red[1][t] = corr;
  }
  __syncthreads();
  if (stop == 2) return;
  for (int o = t; o < R1 * HID; o += 256) {   // dz2 (rows fastest: coalesced split stores)
    const int r = o % R1, h = o / R1;
    float d = 0.f;
#pragma unroll
    for (int c = 0; c < NCLS; ++c) d = fmaf(dl[r][c], w2[h * NCLS + c], d);
    const float av = a2s[r * ALD + h];
    const float dz = act == 0 ? d * av * (1.f - av) : (av > 0.f ? d : 0.f);
    dzs[r * ALD + h] = dz;
    uint16_t hi, mi, lo;
    split3(dz, hi, mi, lo);
    const size_t col = (size_t)r0 + r;
    dz2S[(size_t)h * BP + col] = hi;
    dz2S[(size_t)(HIDP + h) * BP + col] = mi;
    dz2S[(size_t)(2 * HIDP + h) * BP + col] = lo;
  }
  __syncthreads();
  if (stop == 3) return;
  float* p1 = P1 + (size_t)blockIdx.x * P1N;
  for (int o = t; o < P1N; o += 256) {   // this block's partial sums
    float s = 0.f;
    if (o < HID * NCLS) {
      const int h = o / NCLS, c = o % NCLS;
      for (int r = 0; r < R1; ++r) s = fmaf(a2s[r * ALD + h], dl[r][c], s);
    } else if (o < HID * NCLS + HID) {
      const int h = o - HID * NCLS;
      for (int r = 0; r < R1; ++r) s += dzs[r * ALD + h];
    } else if (o < HID * NCLS + HID + NCLS) {
      const int c = o - HID * NCLS - HID;
      for (int r = 0; r < R1; ++r) s += dl[r][c];
    } else {
      const int k = o - (HID * NCLS + HID + NCLS);
      for (int r = 0; r < R1; ++r) s += red[k][r];
    }
    p1[o] = s;
  }
}

// grid (13 pixel blocks of 64, nchunk batch chunks of kchunk rows)
__global__ __launch_bounds__(256) void mlpg_wgrad(const uint8_t* __restrict__ x, int B, int BP,
                                                  const uint16_t* __restrict__ dz2S, float* __restrict__ P2,
                                                  int kchunk) {
  __shared__ __attribute__((aligned(16))) uint16_t ds[2 * SLICE];
  __shared__ __attribute__((aligned(16))) uint16_t xs[2 * 64 * XTLD];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int p0 = blockIdx.x * 64;
  const int b0 = blockIdx.y * kchunk, b1 = min(BP, b0 + kchunk);
  const int kq = 8 * (lane >> 4);
  // x staging: threads 0..127 load 16 pixels of one batch row
  const int xb = t >> 2, xq = t & 3;
  const bool xload = t < 128 && p0 + 16 * xq < DIN;
  f32x4 acc[7];
#pragma unroll
  for (int j = 0; j < 7; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  uint4 v[6];
  uint4 xv = make_uint4(0u, 0u, 0u, 0u);
  auto load_x = [&](int k0) {
    const int r = min(k0 + xb, B - 1);   // rows >= B: dz2 is 0 there
    xv = xload ? *reinterpret_cast<const uint4*>(x + (size_t)r * DIN + p0 + 16 * xq) : make_uint4(0u, 0u, 0u, 0u);
  };
  load_slice(dz2S, BP, b0, v);
  load_x(b0);
  for (int k0 = b0; k0 < b1; k0 += 32) {
    const int par = ((k0 - b0) >> 5) & 1;
    uint16_t* cur = ds + par * SLICE;
    uint16_t* xc = xs + par * 64 * XTLD;
    store_slice(cur, v);
    if (t < 128) {
      const uint32_t w[4] = {xv.x, xv.y, xv.z, xv.w};
#pragma unroll
      for (int j = 0; j < 16; ++j)
        xc[(16 * xq + j) * XTLD + xb] = f2bf((float)((w[j >> 2] >> (8 * (j & 3))) & 255u));
    }
    __syncthreads();
    if (k0 + 32 < b1) {
      load_slice(dz2S, BP, k0 + 32, v);
      load_x(k0 + 32);
    }
    const bf16x8 a = ld_bf16x8(xc + (wave * 16 + (lane & 15)) * XTLD + kq);
    const uint16_t* bl = cur + (lane & 15) * BLD + kq;
#pragma unroll
    for (int j = 0; j < 7; ++j) {
#pragma unroll
      for (int s = 0; s < 3; ++s) acc[j] = mfma16x16x32(a, ld_bf16x8(bl + (s * HIDP + j * 16) * BLD), acc[j]);
    }
  }
  float* p2 = P2 + (size_t)blockIdx.y * OFF_W2;
#pragma unroll
  for (int j = 0; j < 7; ++j) {
    const int h = j * 16 + (lane & 15);
    if (h >= HID) continue;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int p = p0 + wave * 16 + 4 * (lane >> 4) + i;
      if (p < DIN) p2[(size_t)p * HID + h] = acc[j][i];
    }
  }
}

// sum of n values at p[0], p[ld], ... in a fixed order, 8 loads in flight
__device__ __forceinline__ float sum_strided(const float* __restrict__ p, size_t ld, int n) {
  float s = 0.f;
  int c = 0;
  for (; c + 8 <= n; c += 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = p[(size_t)(c + u) * ld];
#pragma unroll
    for (int u = 0; u < 8; ++u) s += v[u];
  }
  for (; c < n; ++c) s += p[(size_t)c * ld];
  return s;
}

// mode 0: reduce the slabs + SGD + W1 split refresh + metrics (1 GPU)
// mode 1: reduce the slabs into gout (TF flat layout) + metrics (before the all-reduce)
// mode 2: SGD from gin (all-reduced, x scale) + W1 split refresh
// mode 3: W1 split refresh only (after set_params)
__global__ __launch_bounds__(256) void mlpg_apply(float* __restrict__ params, const float* __restrict__ P1, int n1,
                                                  const float* __restrict__ P2, int n2, const float* __restrict__ gin,
                                                  float* __restrict__ gout, const float* __restrict__ lr_ptr,
                                                  float scale, uint16_t* __restrict__ W1S,
                                                  float* __restrict__ metrics, int ring,
                                                  long long* __restrict__ gstep, float inv_b, int mode) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < NPARAM && mode != 3) {
    float g = 0.f;
    if (mode == 2) {
      g = gin[i];
    } else if (i < OFF_W2) {
      g = sum_strided(P2 + i, OFF_W2, n2) * (1.f / 255.f);
    } else {
      const int j = i < OFF_B1 ? i - OFF_W2 : (i < OFF_B2 ? HID * NCLS + (i - OFF_B1) : HID * NCLS + HID + (i - OFF_B2));
      g = sum_strided(P1 + j, P1N, n1);
    }
    if (mode == 1) gout[i] = g;
    else params[i] -= (*lr_ptr) * scale * g;
  }
  if (i < OFF_W2 && mode != 1) {
    uint16_t hi, mi, lo;
    split3(params[i], hi, mi, lo);
    const int k = i / HID, n = i % HID;
    W1S[(size_t)n * DINP + k] = hi;
    W1S[(size_t)(HIDP + n) * DINP + k] = mi;
    W1S[(size_t)(2 * HIDP + n) * DINP + k] = lo;
  }
  if (blockIdx.x == 0 && threadIdx.x < 64 && (mode == 0 || mode == 1)) {
    // wave 0 of block 0: lanes over the row blocks, fixed-order wave sum
    float ls = 0.f, cs = 0.f;
    for (int b = threadIdx.x; b < n1; b += 64) {
      ls += P1[(size_t)b * P1N + P1N - 2];
      cs += P1[(size_t)b * P1N + P1N - 1];
    }
    ls = wave_sum(ls);
    cs = wave_sum(cs);
    if (threadIdx.x != 0) return;
    const long long st = *gstep;
    const int slot = (int)(st % ring);
    metrics[2 * slot] = ls * inv_b;
    metrics[2 * slot + 1] = cs * inv_b;
    *gstep = st + 1;
  }
}

}  // namespace mlpg
}  // namespace dtfk

static int g_stop = 0;   // probe knob (scripts/probes/mlpg_stages.py): end mlpg_fwd after stage 1/2/3

extern "C" {

void dtfk_mlpg_set_stop(int s) { g_stop = s; }

int dtfk_mlpg_p1_floats() { return dtfk::mlpg::P1N; }

hipError_t dtfk_mlpg_fwd(const void* x, const void* labels, int B, int BP, const void* W1S, const float* params,
                         float* P1, void* dz2S, int act, int naive, float gscale, hipStream_t s) {
  using namespace dtfk::mlpg;
  hipLaunchKernelGGL(mlpg_fwd, dim3(BP / R1), dim3(256), 0, s, (const uint8_t*)x, (const uint8_t*)labels, B, BP,
                     (const uint16_t*)W1S, params, P1, (uint16_t*)dz2S, act, naive, gscale, g_stop);
  return hipGetLastError();
}

hipError_t dtfk_mlpg_wgrad(const void* x, int B, int BP, const void* dz2S, float* P2, int nchunk, hipStream_t s) {
  using namespace dtfk::mlpg;
  const int kchunk = BP / nchunk;
  hipLaunchKernelGGL(mlpg_wgrad, dim3((DIN + 63) / 64, nchunk), dim3(256), 0, s, (const uint8_t*)x, B, BP,
                     (const uint16_t*)dz2S, P2, kchunk);
  return hipGetLastError();
}

hipError_t dtfk_mlpg_apply(float* params, const float* P1, int n1, const float* P2, int n2, const float* gin,
                           float* gout, const float* lr, float scale, void* W1S, float* metrics, int ring,
                           long long* gstep, int B, int mode, hipStream_t s) {
  using namespace dtfk::mlpg;
  hipLaunchKernelGGL(mlpg_apply, dim3((NPARAM + 255) / 256), dim3(256), 0, s, params, P1, n1, P2, n2, gin, gout, lr,
                     scale, (uint16_t*)W1S, metrics, ring, gstep, 1.f / (float)B, mode);
  return hipGetLastError();
}

}  // extern "C"

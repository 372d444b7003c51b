// Reached by: bench.py at per-GPU batch >= 256 (models/mlp.py GemmMLPTrainer); tests/test_mlp_gemm_gpu.py
// Large-batch MLP step (784-100-10, example.py:69-128): four launches.
//
// The fused / persistent engines (mlp_step.hip, mlp_persist_f32.hip) are
// latency engines for the reference's batch of 100: one wave owns a 16x16
// weight-gradient tile and contracts the whole batch serially -- right at
// B=100, 4x too slow at B=4096 (424 us/step).  The generic fp32 GEMM is no
// better here: [B,784]x[784,100] has 2*ceil(B/64) 64x64 tiles, i.e. 32 f32-MFMA
// workgroups at B=1024 (57 us, rocprofv3).  This step is shaped for the batch:
//
//   mlpg_l1     one workgroup per (64 rows, 16 hidden units): its 4 waves
//               split the 25 k-steps and request their whole operand slice in
//               one shot -- W1 kept as a fragment image of its exact 3-way
//               bf16 split (hi + mid + lo == the fp32 weight; uint8 pixels are
//               exact in bf16: exact products, fp32 accumulate), 1 KB coalesced
//               fragment loads -- partials meet in LDS, a2 = act(z/255 + b1).
//   mlpg_head   one workgroup per 16 rows: logits, softmax-xent, dlog,
//               dz2 = (dlog W2^T) act'(a2) and the [dW2; db2] partials on
//               exact-f32 MFMA, the waves splitting the hidden tiles; dz2
//               leaves as its exact split in the weight-gradient kernel's
//               fragment order.
//   mlpg_wgrad  [dW1; db1] = [x | 255]^T dz2 / 255 per (64-pixel block,
//               128- or 256-row chunk): waves split the chunk, x tiles transposed
//               through wave-private LDS, dz2 straight from its fragment
//               image; one fp32 slab per chunk.
//   mlpg_apply  sums the slabs in a fixed order (deterministic), SGD, refreshes
//               the W1 fragment image, metrics ring + global step.  N > 1: the
//               same kernel first writes the reduced gradient (RCCL
//               all-reduce), then applies it.
//
// Measured (scripts/probes/mlpg_stages.py, profiles/mlp_large_batch_r4.md) --
// the first cut staged operands through LDS with one barrier per k-step and
// paid a full load latency per k-step (a load under a branch, and a HIP uint4
// array kept in scratch); a fused forward streaming all of W1 through every
// workgroup was latency-chained over 7 k-step rounds.
#include "common.h"

namespace dtfk {
namespace mlpg {

constexpr int DIN = 784, DINP = 800, HID = 100, HIDP = 112, NCLS = 10;
constexpr int OFF_W2 = 78400, OFF_B1 = 79400, OFF_B2 = 79500, NPARAM = 79510;
constexpr int KSTEPS = DINP / 32;          // 25
constexpr int P1N = 1112;                  // [dW2 1000 | (unused 100) | db2 10 | loss | correct]
constexpr int XTLD = 40;                   // LDS row stride (bf16) of a transposed x tile [64 px][32 batch]
// register staging in native vectors (an array of HIP's struct uint4 stayed in scratch memory)
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ bf16x8 u8x8_to_bf16(u32x2 w) {
  // integers 0..255 are exact in bf16
  uint32_t p[4];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const uint32_t v = w[j];
    p[2 * j] = pack2bf((float)(v & 255u), (float)((v >> 8) & 255u));
    p[2 * j + 1] = pack2bf((float)((v >> 16) & 255u), (float)(v >> 24));
  }
  return __builtin_bit_cast(bf16x8, u32x4{p[0], p[1], p[2], p[3]});
}

// fp32 -> hi + mid + lo bf16, exact for normal values (8 + 8 + 8 mantissa bits)
__device__ __forceinline__ void split3(float v, uint16_t& h, uint16_t& m, uint16_t& l) {
  h = f2bf(v);
  const float r1 = v - bf2f(h);
  m = f2bf(r1);
  l = f2bf(r1 - bf2f(m));
}

// W1 as MFMA B fragments: [ks 25][split 3][col tile 7][lane 64][8] bf16, so each
// (k-step, split, col tile) fragment is one coalesced 1 KB wave load.  Pads
// (hidden >= 100, pixel >= 784) stay zero.
__device__ __forceinline__ size_t w1f_index(int k, int n, int s) {
  const int ks = k >> 5, kk = k & 31;
  const int lane = (kk >> 3) * 16 + (n & 15);
  return ((((size_t)ks * 3 + s) * 7 + (n >> 4)) * 64 + lane) * 8 + (kk & 7);
}

__device__ __forceinline__ f32x4 mfma16x16x4f32(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

constexpr int NW = 4;            // waves per block (mlpg_l1 / mlpg_wgrad split K over them)
constexpr int NT = 28;           // mlpg_wgrad: 4 pixel tiles x 7 hidden tiles
constexpr int ALD = 112;         // row stride (fp32) of the a2 buffer [BP][112]: col 100 = 1 (db2's column)
constexpr int KPW = (KSTEPS + NW - 1) / NW;   // 7 k-steps per wave

// Hidden layer: one workgroup per (64 rows, 16 hidden units).  Its 4 waves
// split the 25 k-steps (7 each; waves 1-3 run a 7th, all-zero step) and each
// covers the 4 row tiles of the column tile, so a wave's whole operand set --
// 7 x 3 W1 fragments from the fragment image and 7 x 4 x fragments, ~140
// VGPRs -- is requested up front: ONE memory latency, then 84 back-to-back
// MFMAs.  (Covering all 112 hidden units per workgroup streamed the whole
// 537 KB W1 image through every workgroup in 7 dependent rounds: 13 us.)
// Partials meet in LDS (tile rt summed by wave rt, wave order), then
// a2 = act(z / 255 + b1) goes to global fp32 [BP][112].
__global__ __launch_bounds__(256) void mlpg_l1(const uint8_t* __restrict__ x, int B, const uint16_t* __restrict__ W1F,
                                               const float* __restrict__ params, float* __restrict__ a2g, int act) {
  __shared__ __attribute__((aligned(16))) f32x4 red[NW][4][64];
  const int t = threadIdx.x, lane = t & 63, wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int lr = lane & 15, lg4 = lane >> 4;
  const int r0 = blockIdx.x * 64, ct = blockIdx.y;
  const int h = 16 * ct + lr;
  const float bb = params[OFF_B1 + min(h, HID - 1)];
  const bf16x8* wf = reinterpret_cast<const bf16x8*>(W1F) + lane;
  const uint8_t* xr[4];
#pragma unroll
  for (int rt = 0; rt < 4; ++rt) xr[rt] = x + (size_t)min(r0 + 16 * rt + lr, B - 1) * DIN;   // rows >= B: zeroed later
  bf16x8 bq[KPW][3];
  u32x2 xq[KPW][4];
#pragma unroll
  for (int i = 0; i < KPW; ++i) {
    const int kc = min(wave + NW * i, KSTEPS - 1);
#pragma unroll
    for (int sp = 0; sp < 3; ++sp) bq[i][sp] = wf[((size_t)(kc * 3 + sp) * 7 + ct) * 64];
    // pixels >= 784 re-read 776.. (times W1's zero padding)
#pragma unroll
    for (int rt = 0; rt < 4; ++rt) xq[i][rt] = *reinterpret_cast<const u32x2*>(xr[rt] + min(kc * 32 + 8 * lg4, DIN - 8));
  }
  f32x4 acc[4];
#pragma unroll
  for (int rt = 0; rt < 4; ++rt) acc[rt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < KPW; ++i) {
    const bool live = wave + NW * i < KSTEPS;
#pragma unroll
    for (int rt = 0; rt < 4; ++rt) {
      const bf16x8 a = u8x8_to_bf16(live ? xq[i][rt] : u32x2{0u, 0u});
#pragma unroll
      for (int sp = 0; sp < 3; ++sp) acc[rt] = mfma16x16x32(a, bq[i][sp], acc[rt]);
    }
  }
#pragma unroll
  for (int rt = 0; rt < 4; ++rt) red[wave][rt][lane] = acc[rt];
  __syncthreads();
  f32x4 z = red[0][wave][lane];
#pragma unroll
  for (int w = 1; w < NW; ++w) z += red[w][wave][lane];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float zz = z[i] * (1.f / 255.f) + bb;
    const float av = act == 0 ? sigmoidf_(zz) : fmaxf(zz, 0.f);
    a2g[(size_t)(r0 + 16 * wave + 4 * lg4 + i) * ALD + h] = h < HID ? av : (h == HID ? 1.f : 0.f);
  }
}

// Head: one workgroup per 16 rows, no block barrier.  Every wave computes the
// rows' logits and softmax-xent (the cheap, serial part: 25 dependent f32
// MFMAs and DPP row reductions) and then its share of the 7 hidden tiles --
// wave w takes tiles w and w + 4 -- for dz2 = (dlog W2^T) act'(a2) (stored as
// its exact split in mlpg_wgrad's fragment order) and [dW2; db2] = [a2 | 1]^T
// dlog (a2's column 100 is 1) into the tile's P1 slab.  All operands are
// requested up front (one memory latency), on exact-f32 MFMA throughout.
__global__ __launch_bounds__(256) void mlpg_head(const float* __restrict__ a2g, const uint8_t* __restrict__ labels,
                                                 int B, const float* __restrict__ params, float* __restrict__ P1,
                                                 uint16_t* __restrict__ dz2F, int act, int naive, float gscale) {
  __shared__ float dlx[NW][16][17];
  const int t = threadIdx.x, lane = t & 63, wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int lr = lane & 15, lg4 = lane >> 4;
  const int r0 = 16 * blockIdx.x;
  const float* W2 = params + OFF_W2;
  // ---- operands, all in flight at once
  float la[HID / 4], lw[HID / 4];              // logits: A = a2[row lr][k], B = W2[k][class lr]
#pragma unroll
  for (int s = 0; s < HID / 4; ++s) {
    const int k = 4 * s + lg4;
    la[s] = a2g[(size_t)(r0 + lr) * ALD + k];
    lw[s] = W2[k * NCLS + min(lr, NCLS - 1)];
  }
  float ad[2][4], aw[2][4], w2t[2][3];
#pragma unroll
  for (int m = 0; m < 2; ++m) {
    const int ct = min(wave + NW * m, 6), h = 16 * ct + lr;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      ad[m][i] = a2g[(size_t)(r0 + 4 * lg4 + i) * ALD + h];   // D layout: act' of dz2
      aw[m][i] = a2g[(size_t)(r0 + 4 * i + lg4) * ALD + h];   // dW2's A operand: [h][row 4i + lg4]
    }
#pragma unroll
    for (int s = 0; s < 3; ++s) w2t[m][s] = W2[min(h, HID - 1) * NCLS + min(4 * s + lg4, NCLS - 1)];
  }
  const float b2v = params[OFF_B2 + min(lr, NCLS - 1)];
  int yl[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) yl[i] = labels[min(r0 + 4 * lg4 + i, B - 1)];
  // ---- logits [16 x 10] = a2 [16 x 100] W2 [100 x 10]
  f32x4 lgt = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < HID / 4; ++s) lgt = mfma16x16x4f32(la[s], lr < NCLS ? lw[s] : 0.f, lgt);
  // ---- softmax-xent per row (rows 4*lg4 + i, class lr: one 16-lane DPP row per lane group)
  float lsum = 0.f, csum = 0.f;
  const bool cv = lr < NCLS;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int rl = 4 * lg4 + i, row = r0 + rl;
    const float z = cv ? lgt[i] + b2v : -INFINITY;
    const float m = row16_max(z);
    const float e = cv ? __expf(z - m) : 0.f;
    const float se = row16_sum(e);
    const int y = yl[i];
    const float zy = row16_sum(lr == y ? z : 0.f);
    const float ey = row16_sum(lr == y ? e : 0.f);
    const float am = row16_min(cv && z == m ? (float)lr : 16.f);
    float g = 0.f;
    if (row < B) {
      if (lr == 0) {
        lsum += naive ? -__logf(ey / se) : (m + __logf(se)) - zy;
        csum += (int)am == y ? 1.f : 0.f;
      }
      g = cv ? (e / se - (lr == y ? 1.f : 0.f)) * gscale : 0.f;
    }
    dlx[wave][rl][lr] = g;                      // transposed through wave-private LDS
  }
  float dlk[3];                                 // dz2's A operand: dl[row lr][class 4s + lg4]
#pragma unroll
  for (int s = 0; s < 3; ++s) dlk[s] = dlx[wave][lr][4 * s + lg4];
  float dlr[4];                                 // dW2's B operand: dl[row 4i + lg4][class lr]
#pragma unroll
  for (int i = 0; i < 4; ++i) dlr[i] = dlx[wave][4 * i + lg4][lr];
  float* p1 = P1 + (size_t)blockIdx.x * P1N;
  // ---- this wave's hidden tiles: dz2 -> the B-fragment image of mlpg_wgrad
  //      [row / 32][split][col tile][lane ((row % 32) / 8) * 16 + h % 16][row % 8], and [dW2; db2]
  const int R = r0 + 4 * lg4;                   // this lane's 4 rows R .. R+3 (one 8-byte run of e)
  uint16_t* dbase = dz2F + (((size_t)(R >> 5) * 3) * 7) * 512 + (size_t)(((R & 31) >> 3) * 16 + lr) * 8 + (R & 7);
#pragma unroll
  for (int m = 0; m < 2; ++m) {
    const int ct = wave + NW * m;
    if (ct >= 7) break;
    const int h = 16 * ct + lr;
    f32x4 d = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 3; ++s) d = mfma16x16x4f32(dlk[s], (4 * s + lg4 < NCLS && h < HID) ? w2t[m][s] : 0.f, d);
    uint16_t hv[4], mv[4], lv[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float av = ad[m][i];
      const float dz = h < HID ? (act == 0 ? d[i] * av * (1.f - av) : (av > 0.f ? d[i] : 0.f)) : 0.f;
      split3(dz, hv[i], mv[i], lv[i]);
    }
#pragma unroll
    for (int sp = 0; sp < 3; ++sp) {
      const uint16_t* v = sp == 0 ? hv : (sp == 1 ? mv : lv);
      *reinterpret_cast<u32x2*>(dbase + (size_t)(sp * 7 + ct) * 512) =
          u32x2{(uint32_t)v[0] | ((uint32_t)v[1] << 16), (uint32_t)v[2] | ((uint32_t)v[3] << 16)};
    }
    f32x4 w = f32x4{0.f, 0.f, 0.f, 0.f};        // [dW2; db2] tile: M = hidden, N = class, K = 16 rows
#pragma unroll
    for (int i = 0; i < 4; ++i) w = mfma16x16x4f32(aw[m][i], dlr[i], w);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int hh = 16 * ct + 4 * lg4 + i;
      if (lr < NCLS) {
        if (hh < HID) p1[hh * NCLS + lr] = w[i];
        else if (hh == HID) p1[HID * NCLS + HID + lr] = w[i];
      }
    }
  }
  if (wave == 0) {
    lsum = wave_sum(lsum);
    csum = wave_sum(csum);
    if (lane == 0) {
      p1[P1N - 2] = lsum;
      p1[P1N - 1] = csum;
    }
  }
}

// mlpg_wgrad: WKPW 32-row k-steps per wave, chunk = 4 waves x WKPW x 32 rows:
// 128 (WKPW 1) up to B = 2048 -- more workgroups for a small batch -- else 256
__host__ __device__ constexpr int wchunk_of(int wkpw) { return NW * wkpw * 32; }
inline int wkpw_for(int B) { return B <= 2048 ? 1 : 2; }
constexpr int P2N = (DIN + 1) * HID;     // one dW1 slab: 784 pixel rows + the db1 row

// [dW1; db1] partial of one 256-row batch chunk for 64 pixels (+ the constant
// pixel 784 = 255 in the last block: db1 = sum(255 dz2) / 255).  Wave w
// contracts k-steps w and w+4 for all 4 x 7 output tiles: x rows go through
// a wave-private LDS tile transposed to [pixel][batch] bf16 (A fragments),
// dz2 comes straight from its fragment image (B), no block barrier until
// the 4 partials meet in LDS (owner wave per tile, wave order).
template <int WKPW>
__global__ __launch_bounds__(256, 1) void mlpg_wgrad(const uint8_t* __restrict__ x, int B,
                                                     const uint16_t* __restrict__ dz2F, float* __restrict__ P2) {
  __shared__ __attribute__((aligned(16))) float zred[NW * NT * 256];   // 112 KB (x tiles before the reduction)
  const int t = threadIdx.x, lane = t & 63, wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int lr = lane & 15, lg4 = lane >> 4;
  const int p0 = blockIdx.x * 64;
  const int c0 = blockIdx.y * wchunk_of(WKPW);
  uint16_t* xt = reinterpret_cast<uint16_t*>(zred) + wave * (WKPW * 64 * XTLD);   // [step][64 px][XTLD]
  // x: lane -> batch row (lane & 31) of the step, pixels p0 + 32 * (lane >> 5) .. + 32
  const int xb = lane & 31, xh = lane >> 5;
  u32x4 xv[WKPW][2];
  bf16x8 bq[WKPW][21];
  const bf16x8* df = reinterpret_cast<const bf16x8*>(dz2F) + lane;
#pragma unroll
  for (int st = 0; st < WKPW; ++st) {
    const int kb = (c0 >> 5) + wave + NW * st;   // global 32-row k-step
    const int r = min(32 * kb + xb, B - 1);      // rows >= B: dz2 is 0 there
#pragma unroll
    for (int q = 0; q < 2; ++q)
      xv[st][q] = *reinterpret_cast<const u32x4*>(x + (size_t)r * DIN + min(p0 + 32 * xh + 16 * q, DIN - 16));
#pragma unroll
    for (int i = 0; i < 21; ++i) bq[st][i] = df[((size_t)kb * 21 + i) * 64];
  }
#pragma unroll
  for (int st = 0; st < WKPW; ++st) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int pl = 32 * xh + 16 * q + j, p = p0 + pl;
        const float v = p < DIN ? (float)((xv[st][q][j >> 2] >> (8 * (j & 3))) & 255u) : (p == DIN ? 255.f : 0.f);
        xt[(st * 64 + pl) * XTLD + xb] = f2bf(v);
      }
    }
  }
  f32x4 acc[4][7];
#pragma unroll
  for (int pt = 0; pt < 4; ++pt)
#pragma unroll
    for (int ct = 0; ct < 7; ++ct) acc[pt][ct] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int st = 0; st < WKPW; ++st) {
#pragma unroll
    for (int pt = 0; pt < 4; ++pt) {
      const bf16x8 a = ld_bf16x8(xt + (st * 64 + 16 * pt + lr) * XTLD + 8 * lg4);
#pragma unroll
      for (int sp = 0; sp < 3; ++sp)
#pragma unroll
        for (int ct = 0; ct < 7; ++ct) acc[pt][ct] = mfma16x16x32(a, bq[st][sp * 7 + ct], acc[pt][ct]);
    }
  }
  __syncthreads();   // every wave's x tiles read: the partials reuse the LDS
  f32x4* zr = reinterpret_cast<f32x4*>(zred);
#pragma unroll
  for (int pt = 0; pt < 4; ++pt)
#pragma unroll
    for (int ct = 0; ct < 7; ++ct) zr[(wave * NT + pt * 7 + ct) * 64 + lane] = acc[pt][ct];
  __syncthreads();
  float* p2 = P2 + (size_t)blockIdx.y * P2N;
#pragma unroll
  for (int m = 0; m < 7; ++m) {
    const int tile = wave + NW * m, pt = tile / 7, ct = tile % 7;
    f32x4 z = zr[tile * 64 + lane];
#pragma unroll
    for (int w = 1; w < NW; ++w) z += zr[(w * NT + tile) * 64 + lane];
    const int h = 16 * ct + lr;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int p = p0 + 16 * pt + 4 * lg4 + i;
      if (h < HID && p <= DIN) p2[(size_t)p * HID + h] = z[i];
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

// mode 0: reduce the slabs + SGD + W1 fragment-image refresh + metrics (1 GPU)
// mode 1: reduce the slabs into gout (TF flat layout) + metrics (before the all-reduce)
// mode 2: SGD from gin (all-reduced, x scale) + W1 refresh
// mode 3: W1 refresh only (after set_params)
// Blocks [0, NB2): one thread per W1 / b1 parameter (P2 slabs: n2 batch chunks).
// Blocks [NB2, ..): one WAVE per W2 / b2 parameter: the P1 slabs (one per 16
// batch rows, hundreds at large B) summed lane-strided + a fixed-order wave sum.
constexpr int NP2 = OFF_W2 + HID;                 // W1 + b1
constexpr int NB2 = (NP2 + 255) / 256;
constexpr int NP1 = HID * NCLS + NCLS;            // W2 + b2
__device__ __forceinline__ void apply_one(float* params, int i, float g, const float* gin, float* gout,
                                          const float* lr_ptr, float scale, int mode) {
  if (mode == 2) g = gin[i];
  if (mode == 1) gout[i] = g;
  else params[i] -= (*lr_ptr) * scale * g;
}

__global__ __launch_bounds__(256) void mlpg_apply(float* __restrict__ params, const float* __restrict__ P1, int n1,
                                                  const float* __restrict__ P2, int n2, const float* __restrict__ gin,
                                                  float* __restrict__ gout, const float* __restrict__ lr_ptr,
                                                  float scale, uint16_t* __restrict__ W1S,
                                                  float* __restrict__ metrics, int ring,
                                                  long long* __restrict__ gstep, float inv_b, int mode) {
  if (blockIdx.x >= NB2) {
    if (mode == 3) return;
    const int pi = (blockIdx.x - NB2) * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (pi >= NP1) return;
    const int i = pi < HID * NCLS ? OFF_W2 + pi : OFF_B2 + (pi - HID * NCLS);
    const int j = pi < HID * NCLS ? pi : HID * NCLS + HID + (pi - HID * NCLS);
    float g = 0.f;
    if (mode != 2) {
      for (int b = lane; b < n1; b += 64) g += P1[(size_t)b * P1N + j];
      g = wave_sum(g);
    }
    if (lane == 0) apply_one(params, i, g, gin, gout, lr_ptr, scale, mode);
    return;
  }
  const int il = blockIdx.x * blockDim.x + threadIdx.x;
  if (il < NP2) {
    const int i = il < OFF_W2 ? il : OFF_B1 + (il - OFF_W2);
    if (mode != 3) {
      // db1 = the pixel-784 row of the slabs
      const float g = mode == 2 ? 0.f : sum_strided(P2 + il, P2N, n2) * (1.f / 255.f);
      apply_one(params, i, g, gin, gout, lr_ptr, scale, mode);
    }
    if (il < OFF_W2 && mode != 1) {
      uint16_t hi, mi, lo;
      split3(params[i], hi, mi, lo);
      const int k = i / HID, n = i % HID;
      W1S[w1f_index(k, n, 0)] = hi;
      W1S[w1f_index(k, n, 1)] = mi;
      W1S[w1f_index(k, n, 2)] = lo;
    }
  }
  if (blockIdx.x == 0 && threadIdx.x < 64 && (mode == 0 || mode == 1)) {
    // wave 0 of block 0: lanes over the row tiles, fixed-order wave sum
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

extern "C" {

int dtfk_mlpg_p1_floats() { return dtfk::mlpg::P1N; }

hipError_t dtfk_mlpg_fwd(const void* x, const void* labels, int B, int BP, const void* W1F, const float* params,
                         float* a2g, float* P1, void* dz2F, int act, int naive, float gscale, hipStream_t s) {
  using namespace dtfk::mlpg;
  if (BP % 64) return hipErrorInvalidValue;
  hipLaunchKernelGGL(mlpg_l1, dim3(BP / 64, 7), dim3(256), 0, s, (const uint8_t*)x, B, (const uint16_t*)W1F, params,
                     a2g, act);
  hipLaunchKernelGGL(mlpg_head, dim3(BP / 16), dim3(256), 0, s, a2g, (const uint8_t*)labels, B, params, P1,
                     (uint16_t*)dz2F, act, naive, gscale);
  return hipGetLastError();
}

int dtfk_mlpg_wchunk(int B) { return dtfk::mlpg::wchunk_of(dtfk::mlpg::wkpw_for(B)); }
int dtfk_mlpg_p2_floats() { return dtfk::mlpg::P2N; }

hipError_t dtfk_mlpg_wgrad(const void* x, int B, const void* dz2F, float* P2, int nchunk, hipStream_t s) {
  using namespace dtfk::mlpg;
  if (wkpw_for(B) == 1)
    hipLaunchKernelGGL(mlpg_wgrad<1>, dim3((DIN + 64) / 64, nchunk), dim3(256), 0, s, (const uint8_t*)x, B,
                       (const uint16_t*)dz2F, P2);
  else
    hipLaunchKernelGGL(mlpg_wgrad<2>, dim3((DIN + 64) / 64, nchunk), dim3(256), 0, s, (const uint8_t*)x, B,
                       (const uint16_t*)dz2F, P2);
  return hipGetLastError();
}

hipError_t dtfk_mlpg_apply(float* params, const float* P1, int n1, const float* P2, int n2, const float* gin,
                           float* gout, const float* lr, float scale, void* W1S, float* metrics, int ring,
                           long long* gstep, int B, int mode, hipStream_t s) {
  using namespace dtfk::mlpg;
  hipLaunchKernelGGL(mlpg_apply, dim3(NB2 + (NP1 + 3) / 4), dim3(256), 0, s, params, P1, n1, P2, n2, gin, gout, lr,
                     scale, (uint16_t*)W1S, metrics, ring, gstep, 1.f / (float)B, mode);
  return hipGetLastError();
}

}  // extern "C"

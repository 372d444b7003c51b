// Large-batch MLP step (784-100-10, example.py:69-128): three launches.
//
// The fused / persistent engines (mlp_step.hip, mlp_persist_f32.hip) are
// latency engines for the reference's batch of 100: one wave owns a 16x16
// weight-gradient tile and contracts the whole batch serially -- right at
// B=100, 4x too slow at B=4096 (424 us/step).  The generic fp32 GEMM is no
// better here: [B,784]x[784,100] has 2*ceil(B/64) 64x64 tiles, i.e. 32 f32-MFMA
// workgroups at B=1024 (57 us, rocprofv3).  This step is shaped for the batch:
//
//   mlpg_fwd    one workgroup per 64 rows; its 4 waves split the 25 k-steps
//               and each covers all 64 x 112 outputs, so every operand is
//               loaded once per workgroup straight into MFMA fragments (W1 is
//               kept as a fragment image, 1 KB coalesced loads), with the next
//               k-step's loads in flight under 84 MFMAs and no barrier in the
//               K loop.  W1 rides as an exact 3-way bf16 split (hi + mid + lo
//               == the fp32 weight; uint8 pixels are exact in bf16): exact
//               products, fp32 accumulate.  Partials meet in LDS, then per
//               row: a2 = act(z/255 + b1), logits, softmax-xent, dlog,
//               dz2 = (dlog W2^T) act'(a2) and this block's [dW2; db2] on
//               exact-f32 MFMA.  dz2 leaves as its exact split, in the
//               weight-gradient kernel's fragment order.
//   mlpg_wgrad  [dW1; db1] = [x | 255]^T dz2 / 255 per (64-pixel block,
//               256-row chunk): waves split the chunk, x tiles transposed
//               through wave-private LDS, dz2 straight from its fragment
//               image; one fp32 slab per chunk.
//   mlpg_apply  sums the slabs in a fixed order (deterministic), SGD, refreshes
//               the W1 fragment image, metrics ring + global step.  N > 1: the
//               same kernel first writes the reduced gradient (RCCL
//               all-reduce), then applies it.
//
// Measured (scripts/probes/mlpg_stages.py) -- the first cut staged operands
// through LDS with one barrier per k-step and paid a full load latency per
// k-step (a load under a branch, and a HIP uint4 array kept in scratch).
#include "common.h"

namespace dtfk {
namespace mlpg {

constexpr int DIN = 784, DINP = 800, HID = 100, HIDP = 112, NCLS = 10;
constexpr int OFF_W2 = 78400, OFF_B1 = 79400, OFF_B2 = 79500, NPARAM = 79510;
constexpr int KSTEPS = DINP / 32;          // 25
constexpr int R1 = 64;                     // rows per mlpg_fwd block
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

constexpr int NW = 4;            // waves per mlpg_fwd block: they split K, each covers all 64 x 112 outputs
constexpr int NT = 28;           // 4 row tiles x 7 col tiles
constexpr int ZLD = 113;         // LDS row stride (fp32) of a2 / dz2 after the reduction

// One block per 64 rows.  Wave w contracts k-steps w, w+4, ... for every
// output tile, B fragments straight from the fragment image (no LDS staging,
// no barrier in the K loop), next k-step's loads in flight under this one's 84
// MFMAs.  The 4 partial sums meet in LDS (each tile summed by one owner wave in
// wave order: deterministic), then the head runs on exact-f32 MFMA.
__global__ __launch_bounds__(256, 1) void mlpg_fwd(const uint8_t* __restrict__ x, const uint8_t* __restrict__ labels,
                                                   int B, int BP, const uint16_t* __restrict__ W1F,
                                                   const float* __restrict__ params, float* __restrict__ P1,
                                                   uint16_t* __restrict__ dz2S, int act, int naive, float gscale,
                                                   int stop) {
  __shared__ __attribute__((aligned(16))) float zred[NW * NT * 256];   // 112 KB; a2 / dz2 after the reduction
  __shared__ float w2[HID * NCLS], b2[16], b1[HIDP], dls[R1][16], lred[2][NW];
  __shared__ int lab[R1];
  const int t = threadIdx.x, lane = t & 63, wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int lr = lane & 15, lg4 = lane >> 4;
  const int r0 = blockIdx.x * R1;
  // small operands into registers now, into LDS after the K loop (a load
  // waited for here would stall the K loop's start)
  float pw[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) pw[k] = params[OFF_W2 + min(t + 256 * k, HID * NCLS - 1)];
  const float pb1 = params[OFF_B1 + min(t, HID - 1)];
  const float pb2 = params[OFF_B2 + min(t, NCLS - 1)];
  const int plab = labels[min(r0 + (t & 63), B - 1)];

  const uint8_t* xr[4];
#pragma unroll
  for (int rt = 0; rt < 4; ++rt) xr[rt] = x + (size_t)min(r0 + 16 * rt + lr, B - 1) * DIN;   // rows >= B: grads zeroed
  const bf16x8* wf = reinterpret_cast<const bf16x8*>(W1F) + lane;
  f32x4 acc[4][7];
#pragma unroll
  for (int rt = 0; rt < 4; ++rt)
#pragma unroll
    for (int ct = 0; ct < 7; ++ct) acc[rt][ct] = f32x4{0.f, 0.f, 0.f, 0.f};
  // 7 k-steps per wave, fully unrolled, the next k-step's loads in flight
  // under this one's MFMAs; waves 1-3 run a 7th, all-zero step (ks >= 25
  // re-reads step 24 and multiplies a zero x fragment) -- no branch around a
  // load, so the compiler's waits stay counted (a conditional load made it
  // wait for the just-issued next step at every join).  Loading two steps
  // ahead (3 register sets) measured slower: 15.1 vs 13.0 us (VGPRs spill
  // into AGPR copies).
  bf16x8 bq[2][21];
  u32x2 xq[2][4];
  auto load = [&](int ks, bf16x8 (&b)[21], u32x2 (&xv)[4]) {
    const int kc = min(ks, KSTEPS - 1);
#pragma unroll
    for (int i = 0; i < 21; ++i) b[i] = wf[((size_t)kc * 21 + i) * 64];   // i = s * 7 + ct
    // pixels >= 784 re-read 776.. (times W1's zero padding)
#pragma unroll
    for (int rt = 0; rt < 4; ++rt) xv[rt] = *reinterpret_cast<const u32x2*>(xr[rt] + min(kc * 32 + 8 * lg4, DIN - 8));
  };
  auto compute = [&](int ks, const bf16x8 (&b)[21], const u32x2 (&xv)[4]) {
    const bool live = ks < KSTEPS;
#pragma unroll
    for (int rt = 0; rt < 4; ++rt) {
      const bf16x8 a = u8x8_to_bf16(live ? xv[rt] : u32x2{0u, 0u});
#pragma unroll
      for (int s = 0; s < 3; ++s)
#pragma unroll
        for (int ct = 0; ct < 7; ++ct) acc[rt][ct] = mfma16x16x32(a, b[s * 7 + ct], acc[rt][ct]);
    }
  };
  constexpr int KPW = (KSTEPS + NW - 1) / NW;   // 7
  load(wave, bq[0], xq[0]);
#pragma unroll
  for (int i = 0; i < KPW; ++i) {
    if (i + 1 < KPW) load(wave + NW * (i + 1), bq[(i + 1) & 1], xq[(i + 1) & 1]);
    __builtin_amdgcn_sched_barrier(0);   // the next step's loads go out before this step's MFMAs
    compute(wave + NW * i, bq[i & 1], xq[i & 1]);
  }
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (t + 256 * k < HID * NCLS) w2[t + 256 * k] = pw[k];
  if (t < 16) b2[t] = t < NCLS ? pb2 : 0.f;
  if (t < HIDP) b1[t] = t < HID ? pb1 : 0.f;
  if (t < R1) lab[t] = plab;
  // partial sums -> LDS [wave][tile][lane][4]
  f32x4* zr = reinterpret_cast<f32x4*>(zred);
#pragma unroll
  for (int rt = 0; rt < 4; ++rt)
#pragma unroll
    for (int ct = 0; ct < 7; ++ct) zr[(wave * NT + rt * 7 + ct) * 64 + lane] = acc[rt][ct];
  __syncthreads();
  float av[7][4];
#pragma unroll
  for (int m = 0; m < 7; ++m) {   // owned tiles: wave + 4m
    const int tile = wave + NW * m, rt = tile / 7, ct = tile % 7;
    f32x4 z = zr[tile * 64 + lane];
#pragma unroll
    for (int w = 1; w < NW; ++w) z += zr[(w * NT + tile) * 64 + lane];
    const int h = 16 * ct + lr;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float zz = z[i] * (1.f / 255.f) + b1[h];
      const float a = act == 0 ? sigmoidf_(zz) : fmaxf(zz, 0.f);
      av[m][i] = h < HID ? a : (h == HID ? 1.f : 0.f);   // column 100 = 1: db2 rides dW2's product
    }
    (void)rt;
  }
  __syncthreads();   // every partial read: a2 / dz2 reuse the LDS
  float* a2s = zred;
  float* dzs = zred + R1 * ZLD;
#pragma unroll
  for (int m = 0; m < 7; ++m) {
    const int tile = wave + NW * m, rt = tile / 7, ct = tile % 7;
#pragma unroll
    for (int i = 0; i < 4; ++i) a2s[(16 * rt + 4 * lg4 + i) * ZLD + 16 * ct + lr] = av[m][i];
  }
  __syncthreads();
  if (stop == 1) return;
  // logits of row tile `wave`: [16 x 100] x [100 x 10] on f32 MFMA (exact products)
  f32x4 lgt = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 5
  for (int s = 0; s < HID / 4; ++s) {
    const int k = 4 * s + lg4;
    lgt = mfma16x16x4f32(a2s[(16 * wave + lr) * ZLD + k], lr < NCLS ? w2[k * NCLS + lr] : 0.f, lgt);
  }
  float lsum = 0.f, csum = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {   // rows 16*wave + 4*lg4 + i, class lr (16-lane DPP rows)
    const int rl = 16 * wave + 4 * lg4 + i, row = r0 + rl;
    const bool cv = lr < NCLS;
    const float z = cv ? lgt[i] + b2[lr] : -INFINITY;
    const float m = row16_max(z);
    const float e = cv ? __expf(z - m) : 0.f;
    const float se = row16_sum(e);
    float g = 0.f;
    if (row < B) {
      const int y = lab[rl];
      const float zy = row16_sum(lr == y ? z : 0.f);
      const float ey = row16_sum(lr == y ? e : 0.f);
      const float am = row16_min(cv && z == m ? (float)lr : 16.f);
      const float loss = naive ? -__logf(ey / se) : (m + __logf(se)) - zy;
      if (lr == 0) {
        lsum += loss;
        csum += (int)am == y ? 1.f : 0.f;
      }
      g = cv ? (e / se - (lr == y ? 1.f : 0.f)) * gscale : 0.f;
    }
    dls[rl][lr] = g;
  }
  lsum = wave_sum(lsum);
  csum = wave_sum(csum);
  if (lane == 0) {
    lred[0][wave] = lsum;
    lred[1][wave] = csum;
  }
  __syncthreads();
  if (stop == 2) return;
  // dz2 of row tile `wave` = dl [16 x 10] x W2^T [10 x 100] (K padded to 12), times act'(a2)
#pragma unroll
  for (int ct = 0; ct < 7; ++ct) {
    f32x4 d = f32x4{0.f, 0.f, 0.f, 0.f};
    const int h = 16 * ct + lr;
#pragma unroll
    for (int s = 0; s < 3; ++s) {
      const int c = 4 * s + lg4;
      d = mfma16x16x4f32(dls[16 * wave + lr][c], (c < NCLS && h < HID) ? w2[h * NCLS + c] : 0.f, d);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int rl = 16 * wave + 4 * lg4 + i;
      const float a = a2s[rl * ZLD + h];
      dzs[rl * ZLD + h] = h < HID ? (act == 0 ? d[i] * a * (1.f - a) : (a > 0.f ? d[i] : 0.f)) : 0.f;
    }
  }
  __syncthreads();
  // dz2 as its exact split in the wgrad's B-fragment image (dz2F: [row/32][split][col tile][lane][8]):
  // one task = 8 consecutive rows of one hidden unit -> three 16-byte stores
  for (int task = t; task < (R1 / 8) * HID; task += 256) {
    const int h = task % HID, rg = task / HID;
    u32x4 hv, mv, lv;
#pragma unroll
    for (int e = 0; e < 8; e += 2) {
      uint16_t h0, m0, l0, h1, m1, l1;
      split3(dzs[(8 * rg + e) * ZLD + h], h0, m0, l0);
      split3(dzs[(8 * rg + e + 1) * ZLD + h], h1, m1, l1);
      hv[e / 2] = (uint32_t)h0 | ((uint32_t)h1 << 16);
      mv[e / 2] = (uint32_t)m0 | ((uint32_t)m1 << 16);
      lv[e / 2] = (uint32_t)l0 | ((uint32_t)l1 << 16);
    }
    const int row = r0 + 8 * rg;
    const size_t base = (((size_t)(row >> 5) * 3) * 7 + (h >> 4)) * 64 + ((row & 31) >> 3) * 16 + (h & 15);
    u32x4* dst = reinterpret_cast<u32x4*>(dz2S);
    dst[base] = hv;
    dst[base + 7 * 64] = mv;
    dst[base + 14 * 64] = lv;
  }
  if (stop == 3) return;
  // this block's [dW2; db2] = [a2 | 1]^T dl on f32 MFMA: hidden tiles ct = wave, wave + 4
  float* p1 = P1 + (size_t)blockIdx.x * P1N;
  for (int ct = wave; ct < 7; ct += NW) {
    f32x4 d = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
    for (int s = 0; s < R1 / 4; ++s) {
      const int r = 4 * s + lg4;
      d = mfma16x16x4f32(a2s[r * ZLD + 16 * ct + lr], dls[r][lr], d);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int h = 16 * ct + 4 * lg4 + i;
      if (lr < NCLS) {
        if (h < HID) p1[h * NCLS + lr] = d[i];
        else if (h == HID) p1[HID * NCLS + HID + lr] = d[i];
      }
    }
  }
  if (t == 0) {   // (db1 rides the weight gradient: pixel column 784 == 255 in mlpg_wgrad)
    float ls = 0.f, cs = 0.f;
    for (int w = 0; w < NW; ++w) { ls += lred[0][w]; cs += lred[1][w]; }
    p1[P1N - 2] = ls;
    p1[P1N - 1] = cs;
  }
}

constexpr int WKPW = 2;                 // mlpg_wgrad: 32-row k-steps per wave (chunk = 4 waves x 2 x 32 = 256 rows)
constexpr int WCHUNK = NW * WKPW * 32;
constexpr int P2N = (DIN + 1) * HID;     // one dW1 slab: 784 pixel rows + the db1 row

// [dW1; db1] partial of one 256-row batch chunk for 64 pixels (+ the constant
// pixel 784 = 255 in the last block: db1 = sum(255 dz2) / 255).  Wave w
// contracts k-steps w and w+4 for all 4 x 7 output tiles: x rows go through
// a wave-private LDS tile transposed to [pixel][batch] bf16 (A fragments),
// dz2 comes straight from its fragment image (B), no block barrier until
// the 4 partials meet in LDS (owner wave per tile, wave order).
__global__ __launch_bounds__(256, 1) void mlpg_wgrad(const uint8_t* __restrict__ x, int B,
                                                     const uint16_t* __restrict__ dz2F, float* __restrict__ P2) {
  __shared__ __attribute__((aligned(16))) float zred[NW * NT * 256];   // 112 KB (x tiles before the reduction)
  const int t = threadIdx.x, lane = t & 63, wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int lr = lane & 15, lg4 = lane >> 4;
  const int p0 = blockIdx.x * 64;
  const int c0 = blockIdx.y * WCHUNK;
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
      g = sum_strided(P2 + i, P2N, n2) * (1.f / 255.f);
    } else if (i >= OFF_B1 && i < OFF_B2) {
      g = sum_strided(P2 + OFF_W2 + (i - OFF_B1), P2N, n2) * (1.f / 255.f);   // db1 = the pixel-784 row
    } else {
      const int j = i < OFF_B1 ? i - OFF_W2 : HID * NCLS + HID + (i - OFF_B2);
      g = sum_strided(P1 + j, P1N, n1);
    }
    if (mode == 1) gout[i] = g;
    else params[i] -= (*lr_ptr) * scale * g;
  }
  if (i < OFF_W2 && mode != 1) {
    uint16_t hi, mi, lo;
    split3(params[i], hi, mi, lo);
    const int k = i / HID, n = i % HID;
    W1S[w1f_index(k, n, 0)] = hi;
    W1S[w1f_index(k, n, 1)] = mi;
    W1S[w1f_index(k, n, 2)] = lo;
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

int dtfk_mlpg_wchunk() { return dtfk::mlpg::WCHUNK; }
int dtfk_mlpg_p2_floats() { return dtfk::mlpg::P2N; }

hipError_t dtfk_mlpg_wgrad(const void* x, int B, const void* dz2F, float* P2, int nchunk, hipStream_t s) {
  using namespace dtfk::mlpg;
  hipLaunchKernelGGL(mlpg_wgrad, dim3((DIN + 64) / 64, nchunk), dim3(256), 0, s, (const uint8_t*)x, B,
                     (const uint16_t*)dz2F, P2);
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

// Reached by: ops/conv.py ShadowConv2d (ResNet-50 convolutions); tests/test_conv_igemm_gpu.py
// 3x3 (pad 1) and 1x1 (pad 0) convolutions, stride 1 or 2, on NHWC bf16
// activations as implicit GEMMs on the gfx950 matrix cores, with an optional
// BatchNorm statistics epilogue (ResNet-50, BASELINE.json configs[2]).  KS is
// the filter size (template): 9 or 1 taps per 64-channel chunk.
//
//   y[p][k] = sum_{r,s,c} x[n, ho*st + r - 1, wo*st + s - 1, c] * w[k][r][s][c]
//
// GEMM view: M = N*Ho*Wo output pixels (rows), N = K output channels, the
// reduction runs over (r, s, 64-channel chunk) steps: no im2col buffer -- each
// step's A tile is 128 pixels x 64 channels gathered straight from x (one
// 128-byte channel run per pixel, zero for padding pixels via out-of-range
// buffer loads), its B tile the matching [BN][64] slice of w (KRSC =
// channels_last [K, C, 3, 3]).
//
//  * 256 threads = 4 waves in a 2 x 2 grid over the BM x BN tile (BM = 128,
//    BN = 128 or 64): each wave owns (BM/2) x (BN/2) of the output as 16x16
//    v_mfma_f32_16x16x32_bf16 tiles, fp32 accumulate.
//  * Global -> registers (16-B buffer loads, 4 + BN/32 per thread per step) ->
//    LDS: two register sets and two LDS buffers, a step's loads issued two
//    steps before its MFMAs (the first version's one-step lookahead left every
//    step waiting ~1 us on HBM: per-step time was the load latency).  LDS rows are 128 B with the 16-B chunk XOR
//    (chunk ^ ((row >> 1) & 7)) that puts the 16 lanes of a ds_read_b128 group
//    on 16 distinct slots of a bank row (MI355X_MICROARCH.md).
//  * Epilogue through LDS: the bf16 tile is written back as whole 16-B row
//    segments.  EPI 1: the workgroup also writes per-channel sums of y and
//    y^2 over its valid rows -- the [2, P, K] partials bn_finalize
//    (csrc/kernels/bn.hip) reduces, so the BatchNorm after this conv skips its
//    statistics pass over y.  EPI 2 / 3 (this conv computes an input gradient
//    that feeds a BatchNorm (+ residual) + ReLU backward): y is stored
//    ReLU-masked and the partials are that BN backward's sums of g and
//    g * x_hat (EPI 3 first adds the residual branch's gradient already in y).
//    The HBM operands of the epilogue are loaded while the last K step
//    multiplies (with the operands' first loads for <= 2 steps).
//  * ONE (a 1x1 over 64 channels: a single K step): one operand buffer and the
//    LDS sized for the epilogue -- three workgroups per CU instead of two.
//
// The input gradient of a stride-1 conv is the same convolution of dy with the
// flipped, channel-transposed filter (wflip; wflip_multi re-flips every conv's
// filter in one launch after an optimizer step, ops/conv.py _flipped).  The
// weight gradient (conv_wgrad) is split over pixels into fp32 slabs summed in
// split order by wgrad_reduce (profiles/conv_wgrad_sweep_r5.txt).
#include "common.h"
#include <cstdlib>

#include <type_traits>

namespace dtfk {
namespace cig {

typedef __attribute__((ext_vector_type(4))) uint32_t u32x4;

constexpr int BM = 128, BK = 64, NTHR = 256;
constexpr int OOB = 0x7ffffff0;

__device__ __forceinline__ int swz(int row, int ch) { return ch ^ ((row >> 1) & 7); }

// EPI: 0 plain, 1 BN statistics of y (forward), 2 BN backward of the BatchNorm
// whose OUTPUT gradient y is (an input gradient feeding BN(+ReLU)'s backward):
// y is stored as g = y * relu'(bn(bnx)) and part receives the per-channel sums
// of g and g * x_hat (bnst = [mean, invstd, scale, shift] of that BN) -- the
// partials pass of csrc/kernels/bn.hip bn_bwd, done in this epilogue.
// EPI 3: the same for a BatchNorm + residual add + ReLU (mask from
// bnx * scale + shift + bnres), with accum: the output gradient is the
// convolution plus the residual branch's gradient already in y (the fold of
// ops/conv.py), so g is formed from the complete gradient.
// ONE: a single 64-channel K step (1x1 over C = 64): one operand buffer, the
// LDS sized for the epilogue, three workgroups per CU instead of two -- the
// load -> MFMA -> epilogue chain of such a tile is latency bound.
template <int KS, int BN, int EPI>
constexpr int fwd_lds_bytes(bool one) {
  constexpr int BUF = BM * BK * 2 + BN * BK * 2, PITCH = BN * 2 + 16;
  constexpr int EPI_B = ((BM * PITCH + 15) & ~15) + (EPI >= 2 ? NTHR * 16 * 4 : (EPI == 1 ? 2 * NTHR * 4 : 0));
  return one ? (BUF > EPI_B ? BUF : EPI_B) : 2 * BUF;
}
template <int KS, int BN, int EPI, bool ONE = false>
__global__ __launch_bounds__(NTHR, ONE ? 3 : 2) void conv_fwd(const uint16_t* __restrict__ x, const uint16_t* __restrict__ w,
                                                    uint16_t* __restrict__ y, float* __restrict__ part, int N,
                                                    int H, int W, int C, int K, int Ho, int Wo, int stride,
                                                    long long xbytes, int accum, const uint16_t* __restrict__ bnx,
                                                    const float* __restrict__ bnst,
                                                    const uint16_t* __restrict__ bnres, int xcd) {
  constexpr bool STATS = EPI == 1, BNB = EPI >= 2, BNR = EPI == 3;
  constexpr int PAD = KS / 2, TAPS = KS * KS;
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2, BUF = A_BYTES + B_BYTES;
  constexpr int WM = BM / 2, WN = BN / 2;          // per-wave output block
  constexpr int TM = WM / 16, TN = WN / 16;        // 16x16 tiles per wave
  constexpr int NB = BN * 8 / NTHR;                // B chunks per thread per step
  __shared__ __attribute__((aligned(16))) uint8_t smem[fwd_lds_bytes<KS, BN, EPI>(ONE)];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wm = wv >> 1, wn = wv & 1;
  const long long M = (long long)N * Ho * Wo;
  // xcd: the channel tiles of one pixel tile (they share its A rows) on one XCD,
  // consecutive pixel tiles dealt over the 8 XCDs (1-D grid, ids round robin)
  int bx, by;
  if (xcd) {
    const int nt = K / BN, L = blockIdx.x, i = L >> 3;
    bx = (i / nt) * 8 + (L & 7);
    by = i % nt;
    if ((long long)bx * BM >= (long long)N * Ho * Wo) return;   // grid rounded up to 8 pixel tiles
  } else {
    bx = blockIdx.x;
    by = blockIdx.y;
  }
  const long long m0 = (long long)bx * BM;
  const int k0 = by * BN;

  // this thread's 4 A rows (pixel coordinates fixed over the K loop) and chunk
  const int ach = tid & 7;
  int an[4], aho[4], awo[4];
  bool arow[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const long long m = m0 + (tid >> 3) + 32 * i;
    arow[i] = m < M;
    const long long mm = arow[i] ? m : 0;
    awo[i] = (int)(mm % Wo);
    const long long t = mm / Wo;
    aho[i] = (int)(t % Ho);
    an[i] = (int)(t / Ho);
  }
  const auto xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(x), 0, (int)(xbytes > 0x7ffffff0 ? 0x7ffffff0 : xbytes), 0x00020000);
  const long long wbytes = (long long)K * TAPS * C * 2;
  const auto wr = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(w), 0, (int)wbytes, 0x00020000);
  const int ncc = C / BK;
  const int nsteps = TAPS * ncc;

  // two register sets: a step's operands are loaded two steps ahead (issued
  // while the step before it is multiplied), so one HBM round trip hides
  // behind two steps of MFMAs instead of one
  u32x4 ra[2][4], rb[2][NB];
  auto load = [&](int step, auto pc) {
    constexpr int P = decltype(pc)::value;
    const int rs = step / ncc, c0 = (step % ncc) * BK;
    const int r = rs / KS, s = rs % KS;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int hi = aho[i] * stride + r - PAD, wi = awo[i] * stride + s - PAD;
      const bool ok = arow[i] && hi >= 0 && hi < H && wi >= 0 && wi < W;
      const long long off = ((((long long)an[i] * H + hi) * W + wi) * C + c0 + 8 * ach) * 2;
      ra[P][i] = __builtin_amdgcn_raw_buffer_load_b128(xr, ok ? (int)off : OOB, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int row = (tid >> 3) + 32 * i;   // output channel within the tile
      const long long off = (((long long)(k0 + row) * TAPS + rs) * C + c0 + 8 * ach) * 2;
      rb[P][i] = __builtin_amdgcn_raw_buffer_load_b128(wr, (int)off, 0, 0);
    }
  };
  auto store = [&](auto pc) {   // register set P -> LDS buffer P
    constexpr int P = decltype(pc)::value;
    uint8_t* A = smem + P * BUF;
    uint8_t* Bs = A + A_BYTES;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = (tid >> 3) + 32 * i;
      *reinterpret_cast<u32x4*>(A + row * 128 + 16 * swz(row, ach)) = ra[P][i];
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int row = (tid >> 3) + 32 * i;
      *reinterpret_cast<u32x4*>(Bs + row * 128 + 16 * swz(row, ach)) = rb[P][i];
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // epilogue operands read from HBM (BNB: the BN input x; accum: the gradient
  // added onto) are loaded at the start of the last K step, so their latency
  // hides behind its MFMAs instead of stalling the store loop
  constexpr int CPR = BN / 8;                 // 16-B chunks per output row
  constexpr int EIT = BM * CPR / NTHR;        // store-loop iterations per thread
  static_assert(NTHR % CPR == 0, "a thread's chunk column is fixed over the store loop");
  // EPI 3 on 64-wide tiles also prefetches the folded gradient and the residual
  // (on 128-wide tiles those registers would spill: loaded in the store loop)
  constexpr bool PRE3 = BNR && BN == 64;
  // ... and on 128-wide tiles right after the K loop (the operand registers are
  // dead by then), ahead of the accumulator write-out and its barrier
  // (not in the single-step variant: its 3-workgroup register budget spills)
  constexpr bool POST3 = BNR && !PRE3 && !ONE;
  u32x4 pre[EIT], pre_y[PRE3 || POST3 ? EIT : 1], pre_r[PRE3 || POST3 ? EIT : 1];
  auto prefetch = [&]() {
    if (!(BNB || accum)) return;
    const uint16_t* src = BNB ? bnx : y;
#pragma unroll
    for (int it = 0; it < EIT; ++it) {
      const int t = tid + it * NTHR;
      const long long m = m0 + t / CPR;
      if (m < M) {
        const long long e = m * K + k0 + 8 * (t % CPR);
        pre[it] = *reinterpret_cast<const u32x4*>(src + e);
        if constexpr (PRE3) {
          pre_y[it] = *reinterpret_cast<const u32x4*>(y + e);
          pre_r[it] = *reinterpret_cast<const u32x4*>(bnres + e);
        }
      }
    }
  };
  // with one or two K steps (a 1x1 over 64 / 128 channels: the epilogue's HBM
  // traffic dominates) the epilogue loads go out with the operands' first loads
  const bool early = nsteps <= 2;

  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  load(0, I0{});
  if (!ONE && nsteps > 1) load(1, I1{});
  if (early) prefetch();
  store(I0{});
  __syncthreads();
  const int fr = lane & 15, fk = lane >> 4;   // fragment row / k-chunk of this lane
  // step s: its operands sit in LDS buffer s & 1; first the next step's operands
  // go from their registers into the other buffer (free since the last
  // barrier), then the step after that is loaded into the registers just freed
  auto body = [&](int step, auto pc) {
    constexpr int P = decltype(pc)::value;
    using Q = std::integral_constant<int, P ^ 1>;
    if (!ONE && step + 1 < nsteps) store(Q{});
    if (!ONE && step + 2 < nsteps) load(step + 2, pc);
    if (step + 1 == nsteps && !early) prefetch();
    const uint8_t* A = smem + P * BUF;
    const uint8_t* Bs = A + A_BYTES;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {   // two 32-deep k halves of the 64-channel step
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = wm * WM + 16 * i + fr;
        af[i] = *reinterpret_cast<const bf16x8*>(A + row * 128 + 16 * swz(row, 4 * kk + fk));
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int row = wn * WN + 16 * j + fr;
        bfr[j] = *reinterpret_cast<const bf16x8*>(Bs + row * 128 + 16 * swz(row, 4 * kk + fk));
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma16x16x32(af[i], bfr[j], acc[i][j]);
    }
    __syncthreads();
  };
  if constexpr (ONE) {
    body(0, I0{});
  } else for (int step = 0; step < nsteps; step += 2) {
    body(step, I0{});
    if (step + 1 < nsteps) body(step + 1, I1{});
  }

  if constexpr (POST3) {
#pragma unroll
    for (int it = 0; it < EIT; ++it) {
      const int t = tid + it * NTHR;
      const long long m = m0 + t / CPR;
      if (m < M) {
        const long long e = m * K + k0 + 8 * (t % CPR);
        pre_y[it] = *reinterpret_cast<const u32x4*>(y + e);
        pre_r[it] = *reinterpret_cast<const u32x4*>(bnres + e);
      }
    }
  }

  // ---- epilogue: bf16 tile through LDS [BM][BN] (row pitch BN*2 + 16 B)
  constexpr int PITCH = BN * 2 + 16;
  static_assert(BM * PITCH <= (int)sizeof(smem), "epilogue tile fits the operand buffers");
  uint8_t* E = smem;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = wm * WM + 16 * i + 4 * fk + e;   // C[4*(l>>4)+e][l&15]
        const int col = wn * WN + 16 * j + fr;
        *reinterpret_cast<uint16_t*>(E + row * PITCH + 2 * col) = f2bf(acc[i][j][e]);
      }
  float bmu[8], bis[8], bsc[8], bsh[8];      // BNB: the BN's statistics for this thread's 8 channels
  if constexpr (BNB) {
    const int c8 = k0 + 8 * (tid % CPR);
#pragma unroll
    for (int q = 0; q < 8; q += 4) {
      *reinterpret_cast<f32x4*>(bmu + q) = *reinterpret_cast<const f32x4*>(bnst + c8 + q);
      *reinterpret_cast<f32x4*>(bis + q) = *reinterpret_cast<const f32x4*>(bnst + K + c8 + q);
      *reinterpret_cast<f32x4*>(bsc + q) = *reinterpret_cast<const f32x4*>(bnst + 2 * K + c8 + q);
      *reinterpret_cast<f32x4*>(bsh + q) = *reinterpret_cast<const f32x4*>(bnst + 3 * K + c8 + q);
    }
  }
  __syncthreads();
  float sg[8], sgx[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) sg[q] = sgx[q] = 0.f;
#pragma unroll
  for (int it = 0; it < EIT; ++it) {
    const int t = tid + it * NTHR;
    const int row = t / CPR, ch = t % CPR;
    const long long m = m0 + row;
    if (m < M) {
      u32x4 v = *reinterpret_cast<const u32x4*>(E + row * PITCH + 16 * ch);
      if constexpr (BNB) {
        // g = dy * relu'(x * scale + shift) with the BN input x; sums of g and g * x_hat
        const u32x4 xo = pre[it];
        u32x4 ro = {0u, 0u, 0u, 0u};
        if constexpr (BNR) {   // the complete gradient: conv + the folded residual gradient (rounded as stored)
          const long long e = m * K + k0 + 8 * ch;
          constexpr bool HELD = PRE3 || POST3;
          const u32x4 o = HELD ? pre_y[HELD ? it : 0] : *reinterpret_cast<const u32x4*>(y + e);
          ro = HELD ? pre_r[HELD ? it : 0] : *reinterpret_cast<const u32x4*>(bnres + e);
#pragma unroll
          for (int q = 0; q < 4; ++q)
            v[q] = pack2bf(bf2f(v[q] & 0xffff) + bf2f(o[q] & 0xffff), bf2f(v[q] >> 16) + bf2f(o[q] >> 16));
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float x0 = bf2f(xo[q] & 0xffff), x1 = bf2f(xo[q] >> 16);
          const float r0 = BNR ? bf2f(ro[q] & 0xffff) : 0.f, r1 = BNR ? bf2f(ro[q] >> 16) : 0.f;
          const float g0 = x0 * bsc[2 * q] + bsh[2 * q] + r0 > 0.f ? bf2f(v[q] & 0xffff) : 0.f;
          const float g1 = x1 * bsc[2 * q + 1] + bsh[2 * q + 1] + r1 > 0.f ? bf2f(v[q] >> 16) : 0.f;
          sg[2 * q] += g0;
          sg[2 * q + 1] += g1;
          sgx[2 * q] += g0 * (x0 - bmu[2 * q]) * bis[2 * q];
          sgx[2 * q + 1] += g1 * (x1 - bmu[2 * q + 1]) * bis[2 * q + 1];
          v[q] = pack2bf(g0, g1);
        }
      } else if (accum) {   // y += conv (an input gradient folded into an existing one)
        const u32x4 o = pre[it];
#pragma unroll
        for (int q = 0; q < 4; ++q)
          v[q] = pack2bf(bf2f(v[q] & 0xffff) + bf2f(o[q] & 0xffff), bf2f(v[q] >> 16) + bf2f(o[q] >> 16));
      }
      *reinterpret_cast<u32x4*>(y + m * K + k0 + 8 * ch) = v;
    }
  }
  if constexpr (BNB) {
    // the NTHR / CPR threads of each chunk column -> per-channel tile sums (fixed order)
    float* red = reinterpret_cast<float*>(smem + ((BM * PITCH + 15) & ~15));   // behind the tile
    static_assert(((BM * PITCH + 15) & ~15) + NTHR * 16 * 4 <= (int)sizeof(smem), "BN-backward scratch fits");
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      red[tid * 16 + q] = sg[q];
      red[tid * 16 + 8 + q] = sgx[q];
    }
    __syncthreads();
    if (tid < BN) {
      const int ch = tid / 8, q = tid % 8;
      float a = 0.f, b = 0.f;
      for (int j = ch; j < NTHR; j += CPR) {
        a += red[j * 16 + q];
        b += red[j * 16 + 8 + q];
      }
      const int P = (int)((M + BM - 1) / BM);
      part[((size_t)0 * P + bx) * K + k0 + tid] = a;
      part[((size_t)1 * P + bx) * K + k0 + tid] = b;
    }
  }
  if constexpr (STATS) {
    // per-channel sum / sum of squares of the bf16 outputs over the valid rows
    const int rows = (int)(M - m0 < BM ? M - m0 : BM);
    constexpr int RG = NTHR / BN;   // row groups
    const int col = tid % BN, g = tid / BN;
    float s = 0.f, q = 0.f;
    for (int row = g; row < rows; row += RG) {
      const float v = bf2f(*reinterpret_cast<const uint16_t*>(E + row * PITCH + 2 * col));
      s += v;
      q += v * v;
    }
    float* red = reinterpret_cast<float*>(smem + ((BM * PITCH + 15) & ~15));   // behind the tile
    static_assert(((BM * PITCH + 15) & ~15) + 2 * NTHR * 4 <= (int)sizeof(smem), "stats scratch fits");
    red[tid] = s;
    red[NTHR + tid] = q;
    __syncthreads();
    if (g == 0) {
#pragma unroll
      for (int k = 1; k < RG; ++k) {
        s += red[k * BN + col];
        q += red[NTHR + k * BN + col];
      }
      const int P = (int)((M + BM - 1) / BM);
      part[((size_t)0 * P + bx) * K + k0 + col] = s;
      part[((size_t)1 * P + bx) * K + k0 + col] = q;
    }
  }
}

// ---- weight gradient -------------------------------------------------------
//   dW[k][r][s][c] += sum_p dy[p][k] * x[n, ho*st + r - 1, wo*st + s - 1, c]
// GEMM: M = K (output channels), N = 9 C (filter columns (r, s, c) -- the KRSC
// layout), reduction over the P = N*Ho*Wo output pixels, split over gridDim.z.
// Each split writes its fp32 tile as a plain slab (fragment order, 16-byte
// stores) and wgrad_reduce adds the slabs into dW in split order -- the
// gradient is deterministic and accumulates into an existing fp32 gradient.
// (The first version added every split's tile with float atomics: ~16M
// atomics per call, 5x slower than MIOpen -- profiles/conv3x3_paths_r5.jsonl.)
// With one split the workgroup adds its tile into dW directly.  Both
// operands arrive pixel-major -- dy rows [P][K], x rows [.][C] -- so the LDS
// images are [64 pixels][BM] and [64 pixels][BN] ("M/N-contiguous") and the MFMA
// fragments are read with the gfx950 transposed LDS read ds_read_b64_tr_b16
// (4 x 16-bit down a column per lane, two per 8-deep fragment).  Pixel rows
// advance 64 per step by a carried (n, ho, wo) counter, no divisions in the loop.
// chunk XOR of pixel row k (as gemm_big.hip mn_sw: R = 64 rows are 128 B, two
// per bank row, so k bit 0 picks the half and the XOR takes bits 1 and 3)
__device__ __forceinline__ int mn_swz(int k) { return (k & 3) | (((k >> 3) & 1) << 2); }
template <int R>
__device__ __forceinline__ int mn_sw(int k) {
  if constexpr (R == 64) return (((k >> 1) & 1) | (((k >> 3) & 1) << 1)) << 1;
  else return (mn_swz(k) << 1) & (R / 8 - 1);
}
template <int R>
__device__ __forceinline__ int mn_off(int k, int ch) {   // byte offset of (k, 16-byte chunk ch) in [64][R]
  return k * (2 * R) + ((ch ^ mn_sw<R>(k)) << 4);
}
typedef __attribute__((ext_vector_type(4))) short v4s;
typedef __attribute__((address_space(3))) v4s lds_v4s;
// MFMA 16x16x32 fragment of rows [rb, rb+16), k-sub s of a [64][R] image
template <int R>
__device__ __forceinline__ bf16x8 frag_tr(const uint8_t* img, int rb, int s, int lane) {
  const int k = s * 32 + 8 * (lane >> 4) + ((lane & 15) >> 2);
  const int mn = rb + 4 * (lane & 3);
  const int off = mn_off<R>(k, mn >> 3) + ((mn & 7) << 1);
  const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(img + off));
  const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(img + off + 4 * 2 * R));
  typedef __attribute__((ext_vector_type(8))) short v8s;
  const v8s v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, v);
}

// DEPTH: register sets of operands in flight -- a step's loads go out DEPTH
// steps ahead (2: the original two-ahead prefetch; 3: one more set, which the
// 128x128 tile's 220 VGPRs leave room for at the same two workgroups per CU)
template <int KS, int BMW, int BNW, int DEPTH = 2>
__global__ __launch_bounds__(NTHR, 2) void conv_wgrad(const uint16_t* __restrict__ dy, const uint16_t* __restrict__ x,
                                                         float* __restrict__ dw, int N, int H, int W, int C, int K,
                                                         int Ho, int Wo, int stride, long long xbytes,
                                                         int steps_per_split, int kcrs, float* __restrict__ ws,
                                                         long long slab, int tiles_x, int tiles_y, int xcd) {
  constexpr int PAD = KS / 2, TAPS = KS * KS;
  constexpr int PK = 64;                                        // pixels per step
  constexpr int A_BYTES = PK * BMW * 2, B_BYTES = PK * BNW * 2, BUF = A_BYTES + B_BYTES;
  constexpr int ACPR = BMW / 8, BCPR = BNW / 8;                 // 16-B chunks per image row
  constexpr int NA = PK * ACPR / NTHR, NB = PK * BCPR / NTHR;   // chunks per thread per step
  constexpr int WM = BMW / 2, WN = BNW / 2, TM = WM / 16, TN = WN / 16;
  __shared__ __attribute__((aligned(16))) uint8_t smem[2 * BUF];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wm = wv >> 1, wn = wv & 1;
  const long long P = (long long)N * Ho * Wo;
  // 1-D grid of splits x tiles.  xcd: the tiles of one pixel split share its dy / x
  // rows, so every workgroup of split z runs on XCD z % 8 (workgroups are dealt to
  // the XCDs round robin by id) and those rows come from one L2
  int bx, by, bz;
  {
    const int T = tiles_x * tiles_y, L = blockIdx.x;
    const int logical = xcd ? ((L >> 3) / T * 8 + (L & 7)) * T + (L >> 3) % T : L;
    bz = logical / T;
    const int t = logical - bz * T;
    bx = t % tiles_x;
    by = t / tiles_x;
  }
  const int m0 = bx * BMW;                    // output-channel tile
  const int n0 = by * BNW;                    // filter-column tile over (r, s, c)
  const int NC = TAPS * C;
  const long long pb = (long long)bz * steps_per_split * PK;
  long long pe = pb + (long long)steps_per_split * PK;
  if (pe > P) pe = P;
  const int nsteps = pb < pe ? (int)((pe - pb + PK - 1) / PK) : 0;
  const auto dyr = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(dy), 0,
                                                     (int)((P * K * 2) > 0x7ffffff0LL ? 0x7ffffff0LL : P * K * 2), 0x00020000);
  const auto xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(x), 0,
                                                    (int)(xbytes > 0x7ffffff0LL ? 0x7ffffff0LL : xbytes), 0x00020000);
  // A: thread's chunk column and pixel rows (fixed), B: chunk column -> (r, s, c) and pixel rows
  const int ach = tid % ACPR, arow0 = tid / ACPR;               // rows arow0 + (NTHR/ACPR) i
  const int bch = tid % BCPR, brow0 = tid / BCPR;
  constexpr int ARS = NTHR / ACPR, BRS = NTHR / BCPR;           // row strides between a thread's chunks
  // the B chunk's physical (swizzled) column and its filter column
  int bphys[NB], br[NB], bs[NB], bc[NB];
  bool bval[NB];
  // carried pixel coordinates of each B row (advanced by PK per step)
  int bn_[NB], bho[NB], bwo[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int row = brow0 + BRS * i;
    const int lch = bch ^ mn_sw<BNW>(row);   // logical chunk stored at this slot
    bphys[i] = bch;
    const int col = n0 + 8 * lch;
    bval[i] = col < NC;
    const int rs = bval[i] ? col / C : 0;
    bc[i] = bval[i] ? col % C : 0;
    br[i] = rs / KS;
    bs[i] = rs % KS;
    const long long p = pb + row;
    const long long pp = p < P ? p : 0;
    bwo[i] = (int)(pp % Wo);
    const long long t = pp / Wo;
    bho[i] = (int)(t % Ho);
    bn_[i] = (int)(t / Ho);
  }
  int alch[NA];
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    const int row = arow0 + ARS * i;
    alch[i] = ach ^ mn_sw<BMW>(row);
  }
  const int dq = PK / Wo, dr = PK % Wo;
  auto advance = [&]() {
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      bwo[i] += dr;
      bho[i] += dq;
      if (bwo[i] >= Wo) { bwo[i] -= Wo; bho[i] += 1; }
      while (bho[i] >= Ho) { bho[i] -= Ho; bn_[i] += 1; }
    }
  };
  static_assert(DEPTH == 2 || DEPTH == 3, "two or three operand sets in flight");
  u32x4 ra[DEPTH][NA], rb[DEPTH][NB];
  auto load = [&](int step, auto pc) {
    constexpr int Q = decltype(pc)::value;
    const long long p0 = pb + (long long)step * PK;
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const long long p = p0 + arow0 + ARS * i;
      const bool ok = p < pe;
      ra[Q][i] = __builtin_amdgcn_raw_buffer_load_b128(dyr, ok ? (int)((p * K + m0 + 8 * alch[i]) * 2) : OOB, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const long long p = p0 + brow0 + BRS * i;
      const int hi = bho[i] * stride + br[i] - PAD, wi = bwo[i] * stride + bs[i] - PAD;
      const bool ok = bval[i] && p < pe && hi >= 0 && hi < H && wi >= 0 && wi < W;
      const long long off = ((((long long)bn_[i] * H + hi) * W + wi) * C + bc[i]) * 2;
      rb[Q][i] = __builtin_amdgcn_raw_buffer_load_b128(xr, ok ? (int)off : OOB, 0, 0);
    }
    advance();
  };
  auto store = [&](auto pr, auto pl) {   // register set R -> LDS buffer L
    constexpr int R = decltype(pr)::value, L = decltype(pl)::value;
    uint8_t* A = smem + L * BUF;
    uint8_t* Bs = A + A_BYTES;
#pragma unroll
    for (int i = 0; i < NA; ++i)
      *reinterpret_cast<u32x4*>(A + (arow0 + ARS * i) * (2 * BMW) + 16 * ach) = ra[R][i];
#pragma unroll
    for (int i = 0; i < NB; ++i)
      *reinterpret_cast<u32x4*>(Bs + (brow0 + BRS * i) * (2 * BNW) + 16 * bphys[i]) = rb[R][i];
  };
  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  if (nsteps > 0) {
    load(0, I0{});
    if (nsteps > 1) load(1, I1{});
    if constexpr (DEPTH == 3) {
      if (nsteps > 2) load(2, I2{});
    }
    store(I0{}, I0{});
  }
  __syncthreads();
  // step s: its operands sit in LDS buffer s & 1 and came from register set
  // s % DEPTH; first step s + 1's set goes into the other buffer (free since the
  // last barrier), then step s + DEPTH is loaded into set s % DEPTH (stored already)
  auto body = [&](int step, auto pr, auto pl) {
    constexpr int R = decltype(pr)::value, L = decltype(pl)::value;
    using Rn = std::integral_constant<int, (R + 1) % DEPTH>;
    using Ln = std::integral_constant<int, L ^ 1>;
    if (step + 1 < nsteps) store(Rn{}, Ln{});
    if (step + DEPTH < nsteps) load(step + DEPTH, pr);
    const uint8_t* A = smem + L * BUF;
    const uint8_t* Bs = A + A_BYTES;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = frag_tr<BMW>(A, wm * WM + 16 * i, kk, lane);
#pragma unroll
      for (int j = 0; j < TN; ++j) bfr[j] = frag_tr<BNW>(Bs, wn * WN + 16 * j, kk, lane);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma16x16x32(af[i], bfr[j], acc[i][j]);
    }
    __syncthreads();
  };
  if constexpr (DEPTH == 2) {
    for (int step = 0; step < nsteps; step += 2) {
      body(step, I0{}, I0{});
      if (step + 1 < nsteps) body(step + 1, I1{}, I1{});
    }
  } else {
    for (int step = 0; step < nsteps; step += 6) {   // (set, buffer) repeats every 6 steps
      body(step, I0{}, I0{});
      if (step + 1 < nsteps) body(step + 1, I1{}, I1{});
      if (step + 2 < nsteps) body(step + 2, I2{}, I0{});
      if (step + 3 < nsteps) body(step + 3, I0{}, I1{});
      if (step + 4 < nsteps) body(step + 4, I1{}, I0{});
      if (step + 5 < nsteps) body(step + 5, I2{}, I1{});
    }
  }
  const int fr = lane & 15, fk = lane >> 4;
  if (ws != nullptr) {
    // slab of split z, tile (x, y): [wave][TM][TN][64 lanes] f32x4 (zeros for an empty split)
    float* sl = ws + bz * slab + ((long long)by * tiles_x + bx) * (BMW * BNW);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
        *reinterpret_cast<f32x4*>(sl + (((wv * TM + i) * TN + j) * 64 + lane) * 4) = acc[i][j];
    return;
  }
  if (nsteps == 0) return;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = n0 + wn * WN + 16 * j + fr;
      if (col >= NC) continue;
      // KRSC (channels_last) or KCRS (contiguous) gradient layout
      const int cidx = kcrs ? (col % C) * TAPS + col / C : col;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = m0 + wm * WM + 16 * i + 4 * fk + e;
        dw[(long long)row * NC + cidx] += acc[i][j][e];
      }
    }
}

// dW += sum_z slab_z: G threads per f32x4 of the fragment-order tiles (the
// wgrad epilogue's layout), thread g summing slabs g, g + G, ... in order and
// the G partials then combined in LDS in g order -- a fixed summation order
// (deterministic).  With one thread per output (the first version) a 2-tile
// 1x1 weight gradient at 56x56 (256 slabs) ran 16 workgroups of 256-long
// serial load chains.  Each output is mapped back to (output channel, filter
// column) and added into dW once.
template <int KS, int BMW, int BNW>
__global__ __launch_bounds__(256) void wgrad_reduce(const float* __restrict__ ws, int S, long long slab,
                                                    float* __restrict__ dw, int C, int tiles_x, int kcrs, int G) {
  constexpr int WM = BMW / 2, WN = BNW / 2, TM = WM / 16, TN = WN / 16;
  constexpr int Q = BMW * BNW / 4;                      // f32x4 per tile
  __shared__ f32x4 red[256];
  const int OPB = 256 / G;                              // outputs per block
  const int lo = threadIdx.x % OPB, g = threadIdx.x / OPB;
  const long long e = (long long)blockIdx.x * OPB + lo;
  const bool valid = e * 4 < slab;
  f32x4 z = {0.f, 0.f, 0.f, 0.f};
  if (valid) {
    const float* src = ws + e * 4;
    for (int s = g; s < S; s += G) z += *reinterpret_cast<const f32x4*>(src + s * slab);
  }
  red[threadIdx.x] = z;
  __syncthreads();
  if (g != 0 || !valid) return;
  for (int q = 1; q < G; ++q) z += red[q * OPB + lo];
  const int tile = (int)(e / Q), qq = (int)(e - (long long)tile * Q);
  const int lane = qq & 63, f = qq >> 6;                // f = (wave * TM + i) * TN + j
  const int j = f % TN, i = (f / TN) % TM, wv = f / (TN * TM);
  const int wm = wv >> 1, wn = wv & 1;
  const int NC = KS * KS * C;
  const int col = (tile / tiles_x) * BNW + wn * WN + 16 * j + (lane & 15);
  if (col >= NC) return;
  const int row0 = (tile % tiles_x) * BMW + wm * WM + 16 * i + 4 * (lane >> 4);
  const int cidx = kcrs ? (col % C) * (KS * KS) + col / C : col;
#pragma unroll
  for (int r = 0; r < 4; ++r) dw[(long long)(row0 + r) * NC + cidx] += z[r];
}

// w' [C][KS][KS][K] = w [K][KS-1-r][KS-1-s][C]: the filter of the stride-1
// input gradient (KS = 1: the channel transpose)
template <int KS>
__global__ void wflip(const uint16_t* __restrict__ w, uint16_t* __restrict__ wt, int K, int C) {
  constexpr int TAPS = KS * KS;
  const long long n = (long long)K * TAPS * C;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    // i indexes wt = [c][rs'][k]
    const int k = (int)(i % K);
    const long long t = i / K;
    const int rs = (int)(t % TAPS), c = (int)(t / TAPS);
    const int r = KS - 1 - rs / KS, s = KS - 1 - rs % KS;
    wt[i] = w[((long long)k * TAPS + r * KS + s) * C + c];
  }
}

// Every conv's flipped filter in one launch, as LDS-tiled transposes: for
// each tap rs, w[k][rs][c] -> wt[c][TAPS-1-rs][k].  Rows of `tab` are
// {w, wt, K, C, ks} (int64); `tiles` lists (row, rs, k0, c0) per 64 x 64 tile.
// Once per optimizer step instead of one wflip launch per conv backward.
__global__ __launch_bounds__(256) void wflip_multi(const long long* __restrict__ tab, const int4* __restrict__ tiles) {
  __shared__ uint16_t t[64][66];
  const int4 d = tiles[blockIdx.x];
  const long long* r = tab + 5LL * d.x;
  const uint16_t* __restrict__ w = reinterpret_cast<const uint16_t*>(r[0]);
  uint16_t* __restrict__ wt = reinterpret_cast<uint16_t*>(r[1]);
  const int K = (int)r[2], C = (int)r[3], KS = (int)r[4], TAPS = KS * KS;
  const int rs = d.y, k0 = d.z, c0 = d.w;
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  for (int kk = ty; kk < 64; kk += 16) {      // read 64 k rows x 64 c (c contiguous)
    const int k = k0 + kk;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = c0 + 4 * tx + j;
      t[kk][4 * tx + j] = (k < K && c < C) ? w[((long long)k * TAPS + rs) * C + c] : (uint16_t)0;
    }
  }
  __syncthreads();
  const int rsf = TAPS - 1 - rs;
  for (int cc = ty; cc < 64; cc += 16) {      // write 64 c rows x 64 k (k contiguous)
    const int c = c0 + cc;
    if (c >= C) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = k0 + 4 * tx + j;
      if (k < K) wt[((long long)c * TAPS + rsf) * K + k] = t[4 * tx + j][cc];
    }
  }
}

}  // namespace cig
}  // namespace dtfk

extern "C" {

hipError_t dtfk_conv_wflip_multi(const long long* tab, const int* tiles, int ntiles, hipStream_t stream) {
  if (ntiles <= 0) return hipSuccess;
  hipLaunchKernelGGL(dtfk::cig::wflip_multi, dim3((unsigned)ntiles), dim3(256), 0, stream, tab,
                     reinterpret_cast<const int4*>(tiles));
  return hipGetLastError();
}

// 0: ok; invalid shapes return hipErrorInvalidValue (the caller uses MIOpen).
// ks: 3 (pad 1) or 1 (pad 0)
int dtfk_conv_supported(int N, int H, int W, int C, int K, int stride, int ks) {
  if (N < 1 || H < 1 || W < 1 || (stride != 1 && stride != 2) || (ks != 1 && ks != 3)) return 0;
  if (C % 64 != 0 || K % 64 != 0) return 0;
  const long long xbytes = (long long)N * H * W * C * 2;
  if (xbytes >= 0x7ffffff0LL || (long long)K * ks * ks * C * 2 >= 0x7ffffff0LL) return 0;   // 32-bit buffer offsets
  return 1;
}
int dtfk_conv3x3_supported(int N, int H, int W, int C, int K, int stride) {
  return dtfk_conv_supported(N, H, W, C, K, stride, 3);
}

static inline int conv_out(int H, int stride, int ks) { return (H + 2 * (ks / 2) - ks) / stride + 1; }

// y = conv(x, w) (+ y when accum); part (optional): the output's BN statistics partials
hipError_t dtfk_conv_fwd(const void* x, const void* w, void* y, float* part, int N, int H, int W, int C, int K,
                         int stride, int bn, int ks, int accum, const void* bnx, const float* bnst, const void* bnres,
                         hipStream_t stream) {
  using namespace dtfk::cig;
  if (!dtfk_conv_supported(N, H, W, C, K, stride, ks)) return hipErrorInvalidValue;
  const int Ho = conv_out(H, stride, ks), Wo = conv_out(W, stride, ks);
  const long long M = (long long)N * Ho * Wo;
  if (bn != 64 && bn != 128) {
    // 128-wide channel tiles unless that leaves fewer than one workgroup per CU
    // -- the late stages (7x7 / 14x14, 512 channels) have few pixels
    const long long t128 = (M + BM - 1) / BM * (K / 128);
    bn = (K % 128 == 0 && t128 >= 256) ? 128 : 64;
  }
  if (K % bn) return hipErrorInvalidValue;
  // DTF_CONV_FWD_XCD=1: the channel tiles of a pixel tile on one XCD (measured
  // neutral on ResNet-50: 9,275 vs 9,250-9,280 img/s; profiles/conv_wgrad_xcd_r5.txt)
  static const int fwd_xcd = [] {
    const char* e = getenv("DTF_CONV_FWD_XCD");
    return (e && e[0] == '1') ? 1 : 0;
  }();
  const long long mt = (M + BM - 1) / BM;
  const dim3 grid = fwd_xcd ? dim3((unsigned)((mt + 7) / 8 * 8 * (K / bn))) : dim3((unsigned)mt, (unsigned)(K / bn));
  const long long xbytes = (long long)N * H * W * C * 2;
  auto xs = static_cast<const uint16_t*>(x);
  auto ws = static_cast<const uint16_t*>(w);
  auto ys = static_cast<uint16_t*>(y);
  // EPI 2 (BN backward) overwrites y; EPI 3 (BN + residual backward) needs the folded gradient in y
  if (bnx != nullptr && (part == nullptr || bnst == nullptr || (bnres != nullptr) != (accum != 0)))
    return hipErrorInvalidValue;
  if (bnx == nullptr && bnres != nullptr) return hipErrorInvalidValue;
  const int epi = bnx != nullptr ? (bnres != nullptr ? 3 : 2) : (part != nullptr ? 1 : 0);
  auto bx = static_cast<const uint16_t*>(bnx);
  auto br = static_cast<const uint16_t*>(bnres);
  // one 64-channel K step: the single-buffer, three-workgroups-per-CU variant
  const bool one = ks == 1 && C == BK;
#define DTFK_CF(KSV, BNV, EP)                                                                                        \
  if constexpr (KSV == 1) {                                                                                         \
    if (one)                                                                                                        \
      hipLaunchKernelGGL((conv_fwd<KSV, BNV, EP, true>), grid, dim3(NTHR), 0, stream, xs, ws, ys, part, N, H, W, C,  \
                         K, Ho, Wo, stride, xbytes, accum, bx, bnst, br, fwd_xcd);                                  \
    else                                                                                                            \
      hipLaunchKernelGGL((conv_fwd<KSV, BNV, EP>), grid, dim3(NTHR), 0, stream, xs, ws, ys, part, N, H, W, C, K, Ho, \
                         Wo, stride, xbytes, accum, bx, bnst, br, fwd_xcd);                                         \
  } else {                                                                                                          \
    hipLaunchKernelGGL((conv_fwd<KSV, BNV, EP>), grid, dim3(NTHR), 0, stream, xs, ws, ys, part, N, H, W, C, K, Ho,   \
                       Wo, stride, xbytes, accum, bx, bnst, br, fwd_xcd);                                           \
  }
#define DTFK_CF_EPI(KSV, BNV)                                                                               \
  switch (epi) {                                                                                            \
    case 3: DTFK_CF(KSV, BNV, 3); break;                                                                    \
    case 2: DTFK_CF(KSV, BNV, 2); break;                                                                    \
    case 1: DTFK_CF(KSV, BNV, 1); break;                                                                    \
    default: DTFK_CF(KSV, BNV, 0);                                                                          \
  }
#define DTFK_CF_BN(KSV)                                                                      \
  if (bn == 128) {                                                                           \
    DTFK_CF_EPI(KSV, 128)                                                                    \
  } else {                                                                                   \
    DTFK_CF_EPI(KSV, 64)                                                                     \
  }
  if (ks == 3) { DTFK_CF_BN(3) } else { DTFK_CF_BN(1) }
#undef DTFK_CF_BN
#undef DTFK_CF_EPI
#undef DTFK_CF
  return hipGetLastError();
}
hipError_t dtfk_conv3x3_fwd(const void* x, const void* w, void* y, float* part, int N, int H, int W, int C, int K,
                            int stride, int bn, hipStream_t stream) {
  return dtfk_conv_fwd(x, w, y, part, N, H, W, C, K, stride, bn, 3, 0, nullptr, nullptr, nullptr, stream);
}

long long dtfk_conv_tiles(int N, int H, int W, int stride, int ks) {
  return ((long long)N * conv_out(H, stride, ks) * conv_out(W, stride, ks) + dtfk::cig::BM - 1) / dtfk::cig::BM;
}
long long dtfk_conv3x3_tiles(int N, int H, int W, int stride) { return dtfk_conv_tiles(N, H, W, stride, 3); }

hipError_t dtfk_conv_wflip(const void* w, void* wt, int K, int C, int ks, hipStream_t stream) {
  const long long n = (long long)K * ks * ks * C;
  const unsigned blocks = (unsigned)((n + 255) / 256 < 4096 ? (n + 255) / 256 : 4096);
  if (ks == 3)
    hipLaunchKernelGGL(dtfk::cig::wflip<3>, dim3(blocks), dim3(256), 0, stream, static_cast<const uint16_t*>(w),
                       static_cast<uint16_t*>(wt), K, C);
  else if (ks == 1)
    hipLaunchKernelGGL(dtfk::cig::wflip<1>, dim3(blocks), dim3(256), 0, stream, static_cast<const uint16_t*>(w),
                       static_cast<uint16_t*>(wt), K, C);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}
hipError_t dtfk_conv3x3_wflip(const void* w, void* wt, int K, int C, hipStream_t stream) {
  return dtfk_conv_wflip(w, wt, K, C, 3, stream);
}

// Split plan of the weight gradient: the number of pixel splits (gridDim.z)
// and the fp32 workspace (floats) its slabs need (0 with one split).  About two
// workgroups per CU in total (both resident at once) and at least 8 steps of 64
// pixels per split: each extra split costs a 64 KB slab write + read.
// XCD-aware weight-gradient dispatch for 8-16 tiles per split (3x3 over 128
// channels: 73 -> 55 us; 1x1 at 14x14: 37 -> 35 us); with fewer tiles the
// rounded-up split count, with more the one-XCD-per-split concentration lost
// (3x3 over 256 / 512 channels: 61 -> 75 us; profiles/conv_wgrad_xcd_r5.txt).
// DTF_CONV_XCD=0: plain split-major order everywhere.
static bool wgrad_xcd(long long tiles) {
  static const bool on = [] {
    const char* e = getenv("DTF_CONV_XCD");
    return !(e && e[0] == '0');
  }();
  return on && tiles >= 8 && tiles <= 16;
}

// filter-column tile of the weight gradient: 128 wide when it divides 9C / C,
// or when the last, partial tile wastes at most 1/8 (3x3 over 64 channels:
// 576 columns = 4.5 tiles -- the 64-wide tiling ran 1.2x MIOpen's time)
static int wgrad_bnw(int NC) {
  if (NC % 128 == 0) return 128;
  return (NC >= 512 && ((NC + 127) / 128) * 128 - NC <= NC / 8) ? 128 : 64;
}

long long dtfk_conv_wgrad_plan(int N, int H, int W, int C, int K, int stride, int ks, int* splits_out, int* sps_out) {
  using namespace dtfk::cig;
  const long long P = (long long)N * conv_out(H, stride, ks) * conv_out(W, stride, ks);
  const int NC = ks * ks * C;
  const int bm = K % 128 == 0 ? 128 : 64;
  const int bnw = wgrad_bnw(NC);
  const long long tiles = (long long)(K / bm) * ((NC + bnw - 1) / bnw);
  const long long steps = (P + 63) / 64;
  // target workgroups: 512 (two per CU); 256 for the few-tile 1x1 gradients
  // (56x56 / 28x28: fewer, longer splits), 1024 for the many-tile 3x3 ones
  // (profiles/conv_wgrad_sweep_r5.txt; DTF_CONV_WGRAD_WGS overrides), and the
  // minimum 64-pixel steps per split (DTF_CONV_WGRAD_MINSTEPS, default 8)
  static const long long env_target = [] {
    const char* e = getenv("DTF_CONV_WGRAD_WGS");
    return e ? atoll(e) : 0LL;
  }();
  const long long target = env_target > 0 ? env_target
                                          : (ks == 1 ? (tiles <= 4 ? 256 : 512) : (tiles >= 32 ? 1024 : 512));
  static const long long minsteps = [] {
    const char* e = getenv("DTF_CONV_WGRAD_MINSTEPS");
    return e ? atoll(e) : 8LL;
  }();
  long long splits = (target + tiles - 1) / tiles;
  if (splits > steps / minsteps) splits = steps / minsteps;
  if (splits < 1) splits = 1;
  int sps = (int)((steps + splits - 1) / splits);
  splits = (steps + sps - 1) / sps;
  // XCD-aware dispatch (conv_wgrad): a multiple of 8 splits, each XCD its own
  // splits (trailing splits may be empty: they write zero slabs)
  if (wgrad_xcd(tiles) && splits >= 8) {
    splits = (splits + 7) / 8 * 8;
    sps = (int)((steps + splits - 1) / splits);
  }
  if (splits_out) *splits_out = (int)splits;
  if (sps_out) *sps_out = sps;
  return splits > 1 ? splits * tiles * bm * bnw : 0;
}
long long dtfk_conv3x3_wgrad_plan(int N, int H, int W, int C, int K, int stride, int* splits_out, int* sps_out) {
  return dtfk_conv_wgrad_plan(N, H, W, C, K, stride, 3, splits_out, sps_out);
}

// dW (fp32 [K][ks][ks][C] channels_last or [K][C][ks][ks] with kcrs, accumulated
// into) of y = conv(x, w, stride); dy is y's gradient; ws: dtfk_conv_wgrad_plan's
// workspace (may be null when it is 0)
hipError_t dtfk_conv_wgrad(const void* dy, const void* x, float* dw, float* ws, int N, int H, int W, int C, int K,
                           int stride, int ks, int kcrs, hipStream_t stream) {
  using namespace dtfk::cig;
  if (!dtfk_conv_supported(N, H, W, C, K, stride, ks)) return hipErrorInvalidValue;
  const int Ho = conv_out(H, stride, ks), Wo = conv_out(W, stride, ks);
  const long long P = (long long)N * Ho * Wo;
  if (P * K * 2 >= 0x7ffffff0LL) return hipErrorInvalidValue;
  const int NC = ks * ks * C;
  const int bm = K % 128 == 0 ? 128 : 64;
  const int bnw = wgrad_bnw(NC);
  int splits = 1, sps = 1;
  const long long wsn = dtfk_conv_wgrad_plan(N, H, W, C, K, stride, ks, &splits, &sps);
  if (wsn > 0 && ws == nullptr) return hipErrorInvalidValue;
  float* wsp = wsn > 0 ? ws : nullptr;
  const long long slab = wsn > 0 ? wsn / splits : 0;
  const int tiles_x = K / bm, tiles_y = (NC + bnw - 1) / bnw;
  const dim3 grid((unsigned)(tiles_x * tiles_y * splits));
  const int xcd = (wgrad_xcd((long long)tiles_x * tiles_y) && splits >= 8 && splits % 8 == 0) ? 1 : 0;
  const long long xbytes = (long long)N * H * W * C * 2;
  // reduce threads per output: up to 16, ~128K threads in all
  int G = 1;
  while (G < 16 && 2 * G <= splits && (slab / 4) * G < 131072) G *= 2;
  auto d = static_cast<const uint16_t*>(dy);
  auto xs = static_cast<const uint16_t*>(x);
  // operand sets in flight (DTF_CONV_WGRAD_DEPTH: 2 or 3; 3 where it keeps the occupancy)
  static const int depth = [] {
    const char* e = getenv("DTF_CONV_WGRAD_DEPTH");
    return e && atoi(e) == 2 ? 2 : 3;
  }();
#define DTFK_WG(KSV, A, B)                                                                                         \
  do {                                                                                                             \
    if (depth == 3 && !(A == 64 && B == 128)) /* 64x128: 192 VGPRs at depth 3, one wave/SIMD less */              \
      hipLaunchKernelGGL((conv_wgrad<KSV, A, B, 3>), grid, dim3(NTHR), 0, stream, d, xs, dw, N, H, W, C, K, Ho,    \
                         Wo, stride, xbytes, sps, kcrs, wsp, slab, tiles_x, tiles_y, xcd);                         \
    else                                                                                                           \
      hipLaunchKernelGGL((conv_wgrad<KSV, A, B, 2>), grid, dim3(NTHR), 0, stream, d, xs, dw, N, H, W, C, K, Ho,    \
                         Wo, stride, xbytes, sps, kcrs, wsp, slab, tiles_x, tiles_y, xcd);                         \
    if (wsp)                                                                                                       \
      hipLaunchKernelGGL((wgrad_reduce<KSV, A, B>), dim3((unsigned)((slab / 4 + 256 / G - 1) / (256 / G))),        \
                         dim3(256), 0, stream, wsp, splits, slab, dw, C, tiles_x, kcrs, G);                        \
  } while (0)
#define DTFK_WG_T(KSV)                                 \
  if (bm == 128 && bnw == 128) DTFK_WG(KSV, 128, 128); \
  else if (bm == 128) DTFK_WG(KSV, 128, 64);           \
  else if (bnw == 128) DTFK_WG(KSV, 64, 128);          \
  else DTFK_WG(KSV, 64, 64);
  if (ks == 3) { DTFK_WG_T(3) } else { DTFK_WG_T(1) }
#undef DTFK_WG_T
#undef DTFK_WG
  return hipGetLastError();
}
hipError_t dtfk_conv3x3_wgrad(const void* dy, const void* x, float* dw, float* ws, int N, int H, int W, int C, int K,
                              int stride, int kcrs, hipStream_t stream) {
  return dtfk_conv_wgrad(dy, x, dw, ws, N, H, W, C, K, stride, 3, kcrs, stream);
}

}  // extern "C"

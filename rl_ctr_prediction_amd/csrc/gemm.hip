// fp32 GEMM on CDNA4 matrix cores for the DeepFM / policy MLPs.
//
// v_mfma_f32_32x32x2_f32: exact fp32 inputs and accumulation (bit-for-bit a k-ordered fmaf
// chain), 64 FLOP/clk/SIMD — gfx950 has no xf32/TF32, and fp32 is what the reference
// computes in. Block = 4 waves (256 threads), tile BM x BN x BK=32, each wave a WM x WN
// sub-tile of (WM/32) x (WN/32) accumulators of 16 VGPRs. Operands are staged in LDS
// k-major ([BK][BM+pad], [BK][BN+pad]) so a fragment read is one ds_read_b32 per lane over
// 32 consecutive dwords (conflict-free); tiles that arrive row-major along k are
// transposed on the LDS write with an odd row stride (conflict-free ds_write_b32), tiles
// that arrive along m/n are written with ds_write_b128. The next k-tile is loaded into
// registers while the current one feeds the MFMAs.
//
// Epilogues fuse what follows each Linear in nn.Sequential(Linear, ReLU, Dropout): bias,
// ReLU, dropout (stateless counter hash, so no mask tensor is stored), and in the
// backward the Dropout+ReLU gradient mask read from the saved activation.
// Long-K products (weight gradients, K = batch) are split over blockIdx.z into fp32
// slabs and summed in slab order by a second kernel: deterministic, no atomics.
#include <stdlib.h>

#include "ctr_common.h"

namespace ctr {

typedef float floatx16 __attribute__((ext_vector_type(16)));

struct GemmArgs {
  int64_t M, N, K;
  const float* A;
  int64_t lda;
  const float* B;
  int64_t ldb;
  float* C;
  int64_t ldc;
  int epi;
  const float* bias;
  const float* aux;
  int64_t ldaux;
  float scale;        // GRAD_MASK multiplier
  uint32_t drop_thr;  // keep iff hash >= drop_thr
  float drop_scale;   // 1/(1-p)
  uint64_t seed, offset;
  int64_t k_per_split;
  int64_t slab_stride;  // elements between split-K slabs (0: no split)
  bool vec_a, vec_b;
};

__device__ __forceinline__ float apply_epi(const GemmArgs& a, int epi, float acc, int64_t m,
                                           int64_t n) {
  switch (epi) {
    case CTR_EPI_BIAS:
      return acc + a.bias[n];
    case CTR_EPI_BIAS_RELU: {
      const float v = acc + a.bias[n];
      return v > 0.f ? v : 0.f;
    }
    case CTR_EPI_BIAS_RELU_DROP: {
      float v = acc + a.bias[n];
      v = v > 0.f ? v : 0.f;
      const uint32_t hsh = hash_u32(a.seed, a.offset + (uint64_t)(m * a.N + n));
      return hsh >= a.drop_thr ? v * a.drop_scale : 0.f;
    }
    case CTR_EPI_GRAD_MASK:
      return a.aux[m * a.ldaux + n] > 0.f ? acc * a.scale : 0.f;
    default:
      return acc;
  }
}

// ------------------------------------------------------------------- the kernel ------
// Block = WAVES_M x WAVES_N x KSPLIT waves (4: one per SIMD), tile BM x BN x BK=32; a wave
// owns a WM x WN = (BM/WAVES_M) x (BN/WAVES_N) sub-tile of TM x TN 32x32 accumulators over
// 1/KSPLIT of every k-tile (the KSPLIT partial tiles are added in wave order through LDS
// at the end: deterministic). Tiles are sized per GEMM shape so that the grid is about one
// round of the 256 CUs (choose_tiles): e.g. 64x160 (k-split 2) for the 8192x300 forward,
// 128x416 for the 8192x1664 input gradient, 160x128 (split-K 9) for the 300x1664 weight
// gradient — tile quantisation, not the MFMA loop, was what the previous 64/128-only
// tilings lost.
//
// LDS images, per operand:
//  - k-contiguous in memory (A [M][K], nn.Linear weights [N][K]): row-major [rows][36]; a
//    lane reads its row's 4 consecutive k with one ds_read_b128 (conflict-free at stride
//    36) and feeds 4 MFMA k-steps. The MFMA's k order inside each 8-wide group is permuted
//    (step j, lane half h -> k = 8g + 4h + j) identically for A and B, so every product
//    A[m,k]B[k,n] is formed once; only the accumulation order differs from plain k order.
//  - rows-contiguous (A^T, B [K][N]): k-major [32][rows+4]; ds_read_b32 per k-step at the
//    permuted k (32 consecutive rows per half-wave: conflict-free).
// Global loads of k-tile t+1 are in flight (registers) while the MFMAs of k-tile t run;
// rows beyond M/N are clamped to row 0 (never stored), the K tail is zeroed at LDS store.
template <int BM, int BN, int WAVES_M, int WAVES_N, int KSPLIT, bool TA, bool TB, bool VEC>
__global__ __launch_bounds__(WAVES_M* WAVES_N* KSPLIT * 64) void gemm_f32_kernel(GemmArgs a) {
  constexpr int BK = 32;
  constexpr int NT = WAVES_M * WAVES_N * KSPLIT * 64;
  constexpr int WM = BM / WAVES_M, WN = BN / WAVES_N;
  constexpr int TM = WM / 32, TN = WN / 32;
  constexpr bool A_KC = !TA, B_KC = TB;
  constexpr int SKC = BK + 4;
  constexpr int SA = A_KC ? SKC : BM + 4;
  constexpr int SB = B_KC ? SKC : BN + 4;
  constexpr int A_IMG = A_KC ? BM * SKC : BK * (BM + 4);
  constexpr int B_IMG = B_KC ? BN * SKC : BK * (BN + 4);
  constexpr int NA = BM * BK / 4 / NT, NB = BN * BK / 4 / NT;
  constexpr int GPW = (BK / 8) / KSPLIT;  // 8-k groups per wave per k-tile
  static_assert(WM % 32 == 0 && WN % 32 == 0, "wave tile in 32x32 MFMA blocks");
  static_assert(NA * NT * 4 == BM * BK && NB * NT * 4 == BN * BK, "loads split evenly");
  static_assert(GPW * KSPLIT == BK / 8, "k-split divides the 4 groups of a k-tile");
  static_assert((KSPLIT - 1) * WAVES_M * WAVES_N * WM * WN <= 2 * (A_IMG + B_IMG),
                "k-split partials fit the tile buffers");
  __shared__ __attribute__((aligned(16))) float smem[2 * (A_IMG + B_IMG)];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int kw = wave / (WAVES_M * WAVES_N);
  const int wmn = wave % (WAVES_M * WAVES_N);
  const int wm0 = (wmn / WAVES_N) * WM;
  const int wn0 = (wmn % WAVES_N) * WN;
  const int h = lane >> 5, il = lane & 31;

  // tile of this block: tiles sharing A rows are consecutive, and consecutive tiles are
  // kept on one XCD (blocks b, b+8, b+16... share an XCD under round-robin dispatch)
  const int64_t gn = (a.N + BN - 1) / BN;
  const int64_t T = gridDim.x;
  int64_t tix = blockIdx.x;
  if (T % 8 == 0) tix = (tix % 8) * (T / 8) + tix / 8;
  const int64_t m0 = (tix / gn) * BM;
  const int64_t n0 = (tix % gn) * BN;
  const int64_t kb = (int64_t)blockIdx.z * a.k_per_split;
  const int64_t ke = min(a.K, kb + a.k_per_split);

  // per-thread load coordinates: (row, k-offset) of each float4 it stages
  const float* pa[NA];
  const float* pb[NB];
  int ka[NA], kbv[NB], la[NA], lb[NB];  // k offset in the tile; LDS float offset
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    const int q = tid + NT * i;
    if (A_KC) {
      const int r = q / (BK / 4), k4 = q % (BK / 4);
      const int64_t gm = m0 + r;
      ka[i] = k4 * 4;
      la[i] = r * SKC + k4 * 4;
      pa[i] = a.A + (gm < a.M ? gm : 0) * a.lda + kb + ka[i];
    } else {
      const int k = q / (BM / 4), r4 = q % (BM / 4);
      const int64_t gm = m0 + r4 * 4;
      ka[i] = k;
      la[i] = k * SA + r4 * 4;
      pa[i] = a.A + (kb + k) * a.lda + (gm < a.M ? gm : 0);
    }
  }
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int q = tid + NT * i;
    if (B_KC) {
      const int r = q / (BK / 4), k4 = q % (BK / 4);
      const int64_t gnn = n0 + r;
      kbv[i] = k4 * 4;
      lb[i] = r * SKC + k4 * 4;
      pb[i] = a.B + (gnn < a.N ? gnn : 0) * a.ldb + kb + kbv[i];
    } else {
      const int k = q / (BN / 4), r4 = q % (BN / 4);
      const int64_t gnn = n0 + r4 * 4;
      kbv[i] = k;
      lb[i] = k * SB + r4 * 4;
      pb[i] = a.B + (kb + k) * a.ldb + (gnn < a.N ? gnn : 0);
    }
  }
  const int64_t stepA = A_KC ? BK : BK * a.lda;
  const int64_t stepB = B_KC ? BK : BK * a.ldb;

  float4 ra[NA], rb[NB];
  auto load_tile = [&](int t) {
    const int64_t k0 = kb + (int64_t)t * BK;
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const float* p = pa[i] + t * stepA;
      const bool okk = k0 + ka[i] < ke;
      if (VEC) {
        ra[i] = *reinterpret_cast<const float4*>(okk ? p : pa[i]);
      } else {
        float4 v;
        if (A_KC) {
          v.x = (k0 + ka[i] + 0 < ke) ? p[0] : 0.f;
          v.y = (k0 + ka[i] + 1 < ke) ? p[1] : 0.f;
          v.z = (k0 + ka[i] + 2 < ke) ? p[2] : 0.f;
          v.w = (k0 + ka[i] + 3 < ke) ? p[3] : 0.f;
        } else {
          const int64_t gm = m0 + (((tid + NT * i) % (BM / 4)) * 4);
          v.x = (okk && gm + 0 < a.M) ? p[0] : 0.f;
          v.y = (okk && gm + 1 < a.M) ? p[1] : 0.f;
          v.z = (okk && gm + 2 < a.M) ? p[2] : 0.f;
          v.w = (okk && gm + 3 < a.M) ? p[3] : 0.f;
        }
        ra[i] = v;
      }
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const float* p = pb[i] + t * stepB;
      const bool okk = k0 + kbv[i] < ke;
      if (VEC) {
        rb[i] = *reinterpret_cast<const float4*>(okk ? p : pb[i]);
      } else {
        float4 v;
        if (B_KC) {
          v.x = (k0 + kbv[i] + 0 < ke) ? p[0] : 0.f;
          v.y = (k0 + kbv[i] + 1 < ke) ? p[1] : 0.f;
          v.z = (k0 + kbv[i] + 2 < ke) ? p[2] : 0.f;
          v.w = (k0 + kbv[i] + 3 < ke) ? p[3] : 0.f;
        } else {
          const int64_t gnn = n0 + (((tid + NT * i) % (BN / 4)) * 4);
          v.x = (okk && gnn + 0 < a.N) ? p[0] : 0.f;
          v.y = (okk && gnn + 1 < a.N) ? p[1] : 0.f;
          v.z = (okk && gnn + 2 < a.N) ? p[2] : 0.f;
          v.w = (okk && gnn + 3 < a.N) ? p[3] : 0.f;
        }
        rb[i] = v;
      }
    }
  };

  auto store_tile = [&](int buf, int t) {
    const int64_t k0 = kb + (int64_t)t * BK;
    float* as = smem + buf * (A_IMG + B_IMG);
    float* bs = as + A_IMG;
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      float4 v = ra[i];
      if (VEC && !(k0 + ka[i] < ke)) v = make_float4(0.f, 0.f, 0.f, 0.f);  // K tail
      *reinterpret_cast<float4*>(as + la[i]) = v;
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      float4 v = rb[i];
      if (VEC && !(k0 + kbv[i] < ke)) v = make_float4(0.f, 0.f, 0.f, 0.f);
      *reinterpret_cast<float4*>(bs + lb[i]) = v;
    }
  };

  floatx16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // fragments of one 8-k group: [operand tile][k-step]
  auto read_frags = [&](float (&af)[TM][4], float (&bf)[TN][4], const float* as, const float* bs,
                        int g) {
    const int k0 = g * 8;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      if (A_KC) {
        const float4 v =
            *reinterpret_cast<const float4*>(as + (wm0 + i * 32 + il) * SKC + k0 + 4 * h);
        af[i][0] = v.x; af[i][1] = v.y; af[i][2] = v.z; af[i][3] = v.w;
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) af[i][j] = as[(k0 + 4 * h + j) * SA + wm0 + i * 32 + il];
      }
    }
#pragma unroll
    for (int t = 0; t < TN; ++t) {
      if (B_KC) {
        const float4 v =
            *reinterpret_cast<const float4*>(bs + (wn0 + t * 32 + il) * SKC + k0 + 4 * h);
        bf[t][0] = v.x; bf[t][1] = v.y; bf[t][2] = v.z; bf[t][3] = v.w;
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) bf[t][j] = bs[(k0 + 4 * h + j) * SB + wn0 + t * 32 + il];
      }
    }
  };

  if (kb < ke) {
    const int nt = (int)((ke - kb + BK - 1) / BK);
    load_tile(0);
    store_tile(0, 0);
    __syncthreads();
    for (int t = 0; t < nt; ++t) {
      const int buf = t & 1;
      const bool more = t + 1 < nt;
      if (more) load_tile(t + 1);  // in flight under the MFMAs below
      const float* as = smem + buf * (A_IMG + B_IMG);
      const float* bs = as + A_IMG;
      float afc[TM][4], bfc[TN][4];
      read_frags(afc, bfc, as, bs, kw * GPW);
#pragma unroll
      for (int gg = 0; gg < GPW; ++gg) {
        float afn[TM][4], bfn[TN][4];  // next group's fragments, read under these MFMAs
        if (gg + 1 < GPW) read_frags(afn, bfn, as, bs, kw * GPW + gg + 1);
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int tn = 0; tn < TN; ++tn)
              acc[i][tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(afc[i][j], bfc[tn][j],
                                                                acc[i][tn], 0, 0, 0);
        if (gg + 1 < GPW) {
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) afc[i][j] = afn[i][j];
#pragma unroll
          for (int tn = 0; tn < TN; ++tn)
#pragma unroll
            for (int j = 0; j < 4; ++j) bfc[tn][j] = bfn[tn][j];
        }
      }
      if (more) store_tile(buf ^ 1, t + 1);  // the other stage: last read one barrier ago
      __syncthreads();
    }
  }

  // in-block k-split: waves kw > 0 hand their partial tiles to wave kw = 0 through LDS
  if (KSPLIT > 1) {
    constexpr int PW = WM * WN;  // floats per wave partial, stored [i][t][r][lane]
    if (kw > 0) {
      float* dst = smem + ((kw - 1) * WAVES_M * WAVES_N + wmn) * PW;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)
#pragma unroll
          for (int r = 0; r < 16; ++r) dst[((i * TN + tn) * 16 + r) * 64 + lane] = acc[i][tn][r];
    }
    __syncthreads();
    if (kw > 0) return;
#pragma unroll
    for (int s = 1; s < KSPLIT; ++s) {
      const float* src = smem + ((s - 1) * WAVES_M * WAVES_N + wmn) * PW;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[i][tn][r] += src[((i * TN + tn) * 16 + r) * 64 + lane];
    }
  }

  // C/D map of the 32x32 f32 MFMA: col = lane & 31, row = (r&3) + 8*(r>>2) + 4*(lane>>5).
  float* C = a.C + (int64_t)blockIdx.z * a.slab_stride;
  const int epi = a.slab_stride ? (int)CTR_EPI_NONE : a.epi;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int tn = 0; tn < TN; ++tn)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t m = m0 + wm0 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        const int64_t n = n0 + wn0 + tn * 32 + il;
        if (m < a.M && n < a.N) C[m * a.ldc + n] = apply_epi(a, epi, acc[i][tn][r], m, n);
      }
}

// Split-K slabs [splits][M][N] -> C with the epilogue, summed in slab order.
__global__ __launch_bounds__(256) void splitk_reduce_kernel(GemmArgs a, const float* __restrict__ slabs,
                                                            int splits) {
  const int64_t total = a.M * a.N;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    float s = slabs[t];
    for (int z = 1; z < splits; ++z) s += slabs[(int64_t)z * total + t];
    const int64_t m = t / a.N, n = t - m * a.N;
    a.C[m * a.ldc + n] = apply_epi(a, a.epi, s, m, n);
  }
}

// Compiled tilings: (BM, BN, WAVES_M, WAVES_N, KSPLIT), 4 waves each.
struct TileDef {
  int bm, bn, wm, wn, ks;
  double eff;  // sustained fraction of the 0.614 TFLOP/s per-CU fp32 MFMA peak (MI355X)
};
static const TileDef kTiles[] = {
    {64, 64, 2, 2, 1, 0.40},   {64, 128, 2, 2, 1, 0.50},  {128, 64, 2, 2, 1, 0.50},
    {128, 128, 2, 2, 1, 0.60}, {64, 160, 2, 1, 2, 0.62},  {128, 416, 4, 1, 1, 0.72},
    {160, 128, 1, 4, 1, 0.62}, {64, 224, 2, 1, 2, 0.60},
};
constexpr int kNumTiles = sizeof(kTiles) / sizeof(kTiles[0]);

struct TileCfg {
  int tile;  // index into kTiles
  int splits;
  int64_t kps;
};

// Pick (tiling, split-K) by a makespan model: blocks are dealt to the 256 CUs in rounds;
// a round costs one block's padded flops at the tiling's sustained per-CU rate plus ~2 us
// of prologue/epilogue; split-K adds its fp32 slab round trip (2 * splits * M * N * 4 B at
// ~5 TB/s) and a reduce launch. CTR_GEMM_CFG="tile,splits" forces a choice (tuning only).
static TileCfg choose_tiles(int64_t M, int64_t N, int64_t K) {
  TileCfg best{0, 1, std::max<int64_t>(K, 1)};
  if (const char* env = getenv("CTR_GEMM_CFG")) {
    int ti = -1, sp = 1;
    if (sscanf(env, "%d,%d", &ti, &sp) >= 1 && ti >= 0 && ti < kNumTiles && sp >= 1) {
      TileCfg c{ti, 1, std::max<int64_t>(K, 1)};
      if (sp > 1 && K >= 64) {
        c.kps = align_up(ceil_div(K, sp), 32);
        c.splits = (int)ceil_div(K, c.kps);
      }
      return c;
    }
  }
  double best_t = 1e30;
  for (int ti = 0; ti < kNumTiles; ++ti) {
    const TileDef& d = kTiles[ti];
    const int64_t tiles = ceil_div(M, d.bm) * ceil_div(N, d.bn);
    for (int s = 1; s <= 32; ++s) {
      if (s > 1 && K / s < 256) break;  // keep >= 8 k-tiles per split
      const int64_t kps = s == 1 ? K : align_up(ceil_div(K, s), 32);
      const int splits = s == 1 ? 1 : (int)ceil_div(K, kps);
      if (splits != s) continue;
      const int64_t blocks = tiles * splits;
      const double rounds = (double)ceil_div(blocks, 256);
      const double kpad = (double)align_up(std::max<int64_t>(kps, 1), 32);
      const double t_block = 2.0 * d.bm * d.bn * kpad / (0.614 * d.eff * 1e6) + 2.0;
      double t = rounds * t_block;
      if (splits > 1) t += 2.0 * splits * (double)M * N * 4 / 5e6 + 3.0;  // us
      if (t < best_t * 0.98) {
        best_t = t;
        best = TileCfg{ti, splits, splits > 1 ? kps : std::max<int64_t>(K, 1)};
      }
    }
  }
  return best;
}

template <int BM, int BN, int WMW, int WNW, int KS, bool VEC>
static void launch_vec(const GemmArgs& a, bool ta, bool tb, dim3 grid, hipStream_t st) {
  constexpr int NT = WMW * WNW * KS * 64;
  if (!ta && !tb)
    hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, WMW, WNW, KS, false, false, VEC>), grid, NT, 0, st, a);
  else if (!ta && tb)
    hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, WMW, WNW, KS, false, true, VEC>), grid, NT, 0, st, a);
  else if (ta && !tb)
    hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, WMW, WNW, KS, true, false, VEC>), grid, NT, 0, st, a);
  else
    hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, WMW, WNW, KS, true, true, VEC>), grid, NT, 0, st, a);
}

template <int BM, int BN, int WMW, int WNW, int KS>
static void launch_cfg(const GemmArgs& a, bool ta, bool tb, dim3 grid, hipStream_t st) {
  if (a.vec_a && a.vec_b)
    launch_vec<BM, BN, WMW, WNW, KS, true>(a, ta, tb, grid, st);
  else
    launch_vec<BM, BN, WMW, WNW, KS, false>(a, ta, tb, grid, st);
}

static void launch_tile(int ti, const GemmArgs& a, bool ta, bool tb, dim3 grid, hipStream_t st) {
  switch (ti) {
    case 0: launch_cfg<64, 64, 2, 2, 1>(a, ta, tb, grid, st); break;
    case 1: launch_cfg<64, 128, 2, 2, 1>(a, ta, tb, grid, st); break;
    case 2: launch_cfg<128, 64, 2, 2, 1>(a, ta, tb, grid, st); break;
    case 3: launch_cfg<128, 128, 2, 2, 1>(a, ta, tb, grid, st); break;
    case 4: launch_cfg<64, 160, 2, 1, 2>(a, ta, tb, grid, st); break;
    case 5: launch_cfg<128, 416, 4, 1, 1>(a, ta, tb, grid, st); break;
    case 6: launch_cfg<160, 128, 1, 4, 1>(a, ta, tb, grid, st); break;
    case 7: launch_cfg<64, 224, 2, 1, 2>(a, ta, tb, grid, st); break;
  }
}

}  // namespace ctr

using namespace ctr;

extern "C" int64_t ctr_gemm_f32_workspace_bytes(int trans_a, int trans_b, int64_t M, int64_t N,
                                                int64_t K) {
  (void)trans_a;
  (void)trans_b;
  if (M < 0 || N < 0 || K < 0) return -1;
  const TileCfg c = choose_tiles(M, N, K);
  return c.splits > 1 ? (int64_t)c.splits * M * N * (int64_t)sizeof(float) : 0;
}

extern "C" int ctr_gemm_f32(int trans_a, int trans_b, int64_t M, int64_t N, int64_t K,
                            const float* A, int64_t lda, const float* B, int64_t ldb, float* C,
                            int64_t ldc, int epi, const float* bias, const float* aux,
                            int64_t ldaux, float scale, float drop_p, uint64_t seed,
                            uint64_t offset, void* ws, int64_t ws_bytes, ctr_stream_t stream) {
  CTR_REQUIRE(M >= 0 && N >= 0 && K >= 0, "ctr_gemm_f32: negative size");
  CTR_REQUIRE(epi >= CTR_EPI_NONE && epi <= CTR_EPI_GRAD_MASK, "ctr_gemm_f32: bad epilogue %d",
              epi);
  if (M == 0 || N == 0) return CTR_OK;
  CTR_REQUIRE(C && ldc >= N, "ctr_gemm_f32: bad C");
  CTR_REQUIRE(K == 0 || (A && B), "ctr_gemm_f32: null operand");
  CTR_REQUIRE(trans_a ? lda >= M : lda >= K, "ctr_gemm_f32: lda too small");
  CTR_REQUIRE(trans_b ? ldb >= K : ldb >= N, "ctr_gemm_f32: ldb too small");
  CTR_REQUIRE(epi == CTR_EPI_NONE || epi == CTR_EPI_GRAD_MASK || bias, "ctr_gemm_f32: bias missing");
  CTR_REQUIRE(epi != CTR_EPI_GRAD_MASK || (aux && ldaux >= N), "ctr_gemm_f32: aux missing");
  CTR_REQUIRE(drop_p >= 0.f && drop_p < 1.f, "ctr_gemm_f32: dropout p must be in [0,1)");
  CTR_REQUIRE(M < (int64_t(1) << 31) / 128 * 128 && N < (int64_t(1) << 31),
              "ctr_gemm_f32: size too large");
  hipStream_t st = as_stream(stream);

  GemmArgs a;
  a.M = M; a.N = N; a.K = K;
  a.A = A; a.lda = lda; a.B = B; a.ldb = ldb;
  a.C = C; a.ldc = ldc;
  a.epi = epi; a.bias = bias; a.aux = aux; a.ldaux = ldaux; a.scale = scale;
  const double thr = (double)drop_p * 4294967296.0;
  a.drop_thr = (uint32_t)std::min(thr, 4294967295.0);
  a.drop_scale = (float)(1.0 / (1.0 - (double)drop_p));
  a.seed = seed; a.offset = offset;
  // float4 path: 16-B aligned rows whose contiguous extent is a multiple of 4 (then a
  // float4 is entirely inside or entirely outside the matrix; split-K bounds are
  // multiples of 32)
  a.vec_a = (reinterpret_cast<uintptr_t>(A) % 16 == 0) && (lda % 4 == 0) &&
            ((trans_a ? M : K) % 4 == 0);
  a.vec_b = (reinterpret_cast<uintptr_t>(B) % 16 == 0) && (ldb % 4 == 0) &&
            ((trans_b ? K : N) % 4 == 0);

  const TileCfg c = choose_tiles(M, N, K);
  a.k_per_split = c.splits > 1 ? c.kps : std::max<int64_t>(K, 1);
  a.slab_stride = 0;
  if (c.splits > 1) {
    const int64_t need = (int64_t)c.splits * M * N * (int64_t)sizeof(float);
    if (!ws || ws_bytes < need) {
      set_error("ctr_gemm_f32: split-K workspace %lld < %lld bytes", (long long)ws_bytes,
                (long long)need);
      return CTR_ERR_WORKSPACE;
    }
    a.C = static_cast<float*>(ws);
    a.ldc = N;
    a.slab_stride = M * N;
  }
  const TileDef& d = kTiles[c.tile];
  const dim3 grid((unsigned)(ceil_div(N, d.bn) * ceil_div(M, d.bm)), 1, (unsigned)c.splits);
  launch_tile(c.tile, a, trans_a != 0, trans_b != 0, grid, st);
  CTR_LAUNCH_CHECK("gemm_f32_kernel");
  if (c.splits > 1) {
    GemmArgs r = a;
    r.C = C;
    r.ldc = ldc;
    const unsigned g2 = (unsigned)std::min<int64_t>(ceil_div(M * N, 256), 4096);
    hipLaunchKernelGGL(splitk_reduce_kernel, g2, 256, 0, st, r, static_cast<const float*>(ws),
                       c.splits);
    CTR_LAUNCH_CHECK("splitk_reduce_kernel");
  }
  return CTR_OK;
}

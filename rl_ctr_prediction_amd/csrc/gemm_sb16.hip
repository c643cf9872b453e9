// fp32-accurate GEMM on the bf16 matrix cores: "split-bf16" (3 planes, 6 products).
//
// gfx950's fp32-input MFMA (v_mfma_f32_32x32x2_f32) runs at 1/16 of the bf16 rate. Every
// fp32 operand x is split EXACTLY into three bf16 planes, x = x0 + x1 + x2:
//   x0 = bf16_rne(x), r1 = x - x0 (exact: Sterbenz), x1 = bf16_rne(r1), x2 = r1 - x1
// (r1 has <= 16 significant bits and r1 - x1 <= 8, so x2 is exactly a bf16). A product
// a*b = sum_{i,j} a_i b_j; the six terms with i + j <= 2 are formed on
// v_mfma_f32_32x32x16_bf16 (bf16 x bf16 products are exact in fp32, accumulation fp32);
// the dropped terms a1b2 + a2b1 + a2b2 are bounded by 2^-23 |ab| (|a1| <= 2^-8 |a|,
// |a2| <= 2^-16 |a|, RNE splits: signs random), i.e. the rounding error of one fp32
// multiply. 6 bf16 MFMAs of 32 cycles per 16-deep k step replace 8 fp32 MFMAs of 64:
// 2.7x the fp32 matrix rate, with fp32 accumulation — the GEMMs of DeepFM's MLP (and of
// the PG policy) keep the reference's fp32 results to fp32 rounding (tests/test_gpu_kernels.py
// bounds every output against an fp64 product with the same bar as the exact kernel).
//
// Operands stay fp32 in HBM (no producer changes). A block stages each k-tile global ->
// registers (prefetched one tile ahead) -> split -> three bf16 LDS images, [rows][BK] per
// plane, k-contiguous, 16-B chunks XOR-swizzled so that a fragment read (ds_read_b128 of
// 8 consecutive k of one row by 32 rows) is conflict-free. Operands stored with k
// contiguous (A [M][K], nn.Linear weights [N][K]) are staged as float4 along k; operands
// stored rows-contiguous (A^T, B [K][N]) as 4x4 blocks transposed in registers, so both
// land in the same image. Each element is split once per block (not once per wave
// fragment read), which keeps the VALU share of a k-tile under the MFMA time.
#include "gemm_common.h"

// tuning-only experiment knobs (tools/build_variant.py): drop the global loads, the split
// VALU, or the MFMAs, to see which one bounds the k-loop. Results are wrong when set.
#ifndef CTR_SB16_NOLOAD
#define CTR_SB16_NOLOAD 0
#endif
#ifndef CTR_SB16_NOSPLIT
#define CTR_SB16_NOSPLIT 0
#endif
#ifndef CTR_SB16_NOMFMA
#define CTR_SB16_NOMFMA 0
#endif

namespace ctr {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));

// (x, y) -> packed (bf16_rne(x), bf16_rne(y)) and the exact fp32 residuals
__device__ __forceinline__ uint32_t split_pair(float x, float y, float& rx, float& ry) {
  const bf16x2_t hv = __builtin_convertvector((f32x2_t){x, y}, bf16x2_t);
  const f32x2_t hf = __builtin_convertvector(hv, f32x2_t);
  rx = x - hf.x;
  ry = y - hf.y;
  return __builtin_bit_cast(uint32_t, hv);
}

__device__ __forceinline__ uint32_t pack_pair(float x, float y) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2_t){x, y}, bf16x2_t));
}

// four consecutive k of one row -> that row's 8-byte piece of each of the three planes
struct Split4 {
  uint2 p[3];
};
__device__ __forceinline__ Split4 split4(float a, float b, float c, float d) {
  Split4 s;
  if (CTR_SB16_NOSPLIT) {
    s.p[0] = make_uint2(__float_as_uint(a), __float_as_uint(b));
    s.p[1] = make_uint2(__float_as_uint(c), __float_as_uint(d));
    s.p[2] = s.p[0];
    return s;
  }
  float r0, r1, r2, r3, q0, q1, q2, q3;
  s.p[0].x = split_pair(a, b, r0, r1);
  s.p[0].y = split_pair(c, d, r2, r3);
  s.p[1].x = split_pair(r0, r1, q0, q1);
  s.p[1].y = split_pair(r2, r3, q2, q3);
  s.p[2].x = pack_pair(q0, q1);
  s.p[2].y = pack_pair(q2, q3);
  return s;
}

// 16-B chunk swizzle of a [rows][BK] bf16 image (BK/8 chunks per row): the 16-lane groups
// of a gfx950 ds_read_b128 ({0-3,12-15,20-27}, {4-11,16-19,28-31}, ...) then touch 16
// distinct 4-bank slots.
template <int BK>
__device__ __forceinline__ int sb_swz(int r) {
  return BK == 32 ? ((r >> 2) & 3) : ((r >> 1) & 7);
}

__device__ __forceinline__ float f4c(const float4& v, int i) {
  return i == 0 ? v.x : i == 1 ? v.y : i == 2 ? v.z : v.w;
}

// ---- staging: global fp32 -> registers ----------------------------------------------
// KC (k-contiguous, element (row, k) at X[row*ld + k]): unit = one float4 along k.
// RC (rows-contiguous, element at X[k*ld + row]): unit = 4 rows x 4 k (4 float4 loads).
// Rows past `extent` read clamped in-bounds addresses (finite data that only reaches
// never-stored outputs), so a full k-tile needs no select on loaded data and the loads
// stay in flight until the store after the MFMAs; only the TAIL tile (k past `ke`, which
// would add into stored outputs) zeroes what it loaded.
template <int ROWS, int BK, bool KC, bool VEC, bool TAIL, int NU, int R>
__device__ __forceinline__ void sb_load(float4 (&r)[NU][R], const float* __restrict__ X,
                                        int64_t ld, int64_t row0, int64_t extent, int64_t k0,
                                        int64_t ke, int tid) {
  constexpr int KQ = BK / 4;
  constexpr int U = KC ? ROWS * KQ : (ROWS / 4) * KQ;
  const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
  if (CTR_SB16_NOLOAD) {
#pragma unroll
    for (int i = 0; i < NU; ++i)
#pragma unroll
      for (int j = 0; j < R; ++j) r[i][j] = make_float4((float)(tid + i), (float)j, (float)k0, 1.f);
    return;
  }
#pragma unroll
  for (int i = 0; i < NU; ++i) {
    const int q = tid + 256 * i;
    if (U % 256 != 0 && q >= U) {
#pragma unroll
      for (int j = 0; j < R; ++j) r[i][j] = z;
      continue;
    }
    if (KC) {
      const int64_t row = row0 + q / KQ;
      const int64_t k = k0 + 4 * (q % KQ);
      const float* p = X + (row < extent ? row : 0) * ld;
      if (VEC) {
        const bool ok = !TAIL || k < ke;
        const float4 v = *reinterpret_cast<const float4*>(p + (ok ? k : k0));
        r[i][0] = ok ? v : z;
      } else {
        float e[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const bool ok = !TAIL || k + j < ke;
          const float v = p[ok ? k + j : k0];
          e[j] = ok ? v : 0.f;
        }
        r[i][0] = make_float4(e[0], e[1], e[2], e[3]);
      }
    } else {
      const int64_t rowb = row0 + 4 * (q % (ROWS / 4));
      const int64_t kq = k0 + 4 * (q / (ROWS / 4));
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int64_t k = kq + j;
        const bool okk = !TAIL || k < ke;
        const float* p = X + (okk ? k : k0) * ld;
        if (VEC) {
          const float4 v = *reinterpret_cast<const float4*>(p + (rowb < extent ? rowb : 0));
          r[i][j] = okk ? v : z;
        } else {
          float e[4];
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            const float v = p[rowb + c < extent ? rowb + c : 0];
            e[c] = okk ? v : 0.f;
          }
          r[i][j] = make_float4(e[0], e[1], e[2], e[3]);
        }
      }
    }
  }
}

// ---- staging: registers -> split -> the three bf16 planes ----------------------------
// `img` = plane 0 of this stage; image row = rbase + operand row; planes PLANE apart.
template <int ROWS, int BK, bool KC, int NU, int R, int PLANE>
__device__ __forceinline__ void sb_store(uint16_t* img, int rbase, const float4 (&r)[NU][R],
                                         int tid) {
  constexpr int KQ = BK / 4;
  constexpr int U = KC ? ROWS * KQ : (ROWS / 4) * KQ;
#pragma unroll
  for (int i = 0; i < NU; ++i) {
    const int q = tid + 256 * i;
    if (U % 256 != 0 && q >= U) break;
    if (KC) {
      const int row = rbase + q / KQ, c4 = q % KQ;
      const Split4 s = split4(r[i][0].x, r[i][0].y, r[i][0].z, r[i][0].w);
      const int off = row * BK + 8 * ((c4 >> 1) ^ sb_swz<BK>(row)) + 4 * (c4 & 1);
#pragma unroll
      for (int p = 0; p < 3; ++p) *reinterpret_cast<uint2*>(img + p * PLANE + off) = s.p[p];
    } else {
      const int rg = q % (ROWS / 4), kq = q / (ROWS / 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) {  // row 4rg + e: its 4 k are element e of the 4 loads
        const int row = rbase + 4 * rg + e;
        const Split4 s = split4(f4c(r[i][0], e), f4c(r[i][1], e), f4c(r[i][2], e), f4c(r[i][3], e));
        const int off = row * BK + 8 * ((kq >> 1) ^ sb_swz<BK>(row)) + 4 * (kq & 1);
#pragma unroll
        for (int p = 0; p < 3; ++p) *reinterpret_cast<uint2*>(img + p * PLANE + off) = s.p[p];
      }
    }
  }
}

// ---- the kernel --------------------------------------------------------------------
// Block = 4 waves (WAVES_M x WAVES_N), tile BM x BN x BK; a wave owns WM x WN =
// (BM/WAVES_M) x (BN/WAVES_N) as TM x TN 32x32 accumulators. NS = LDS stages: 2 (one
// barrier per k-tile) or 1 (half the LDS, so more blocks share a CU; two barriers).
template <int BM, int BN, int BK, int WAVES_M, int WAVES_N, int NS, bool TA, bool TB, bool VEC>
__global__ __launch_bounds__(256) void gemm_sb16_kernel(GemmArgs a) {
  static_assert(WAVES_M * WAVES_N == 4, "4 waves");
  static_assert(BK == 32 || BK == 64, "k-tile of 32 or 64");
  constexpr int ROWS = BM + BN;
  constexpr int PLANE = ROWS * BK;  // bf16 elements per plane image
  constexpr int STAGE = 3 * PLANE;
  constexpr int WM = BM / WAVES_M, WN = BN / WAVES_N;
  constexpr int TM = WM / 32, TN = WN / 32;
  static_assert(WM % 32 == 0 && WN % 32 == 0, "wave tile in 32x32 MFMA blocks");
  static_assert(BM % 4 == 0 && BN % 4 == 0, "4-row staging units");
  constexpr bool A_KC = !TA, B_KC = TB;
  constexpr int KQ = BK / 4;
  constexpr int UA = A_KC ? BM * KQ : (BM / 4) * KQ;
  constexpr int UB = B_KC ? BN * KQ : (BN / 4) * KQ;
  constexpr int NUA = (UA + 255) / 256, NUB = (UB + 255) / 256;
  constexpr int RA = A_KC ? 1 : 4, RB = B_KC ? 1 : 4;
  constexpr int LDS_ELEMS = NS * STAGE > 4 * 32 * 36 * 2 ? NS * STAGE : 4 * 32 * 36 * 2;
  __shared__ __attribute__((aligned(16))) uint16_t smem[LDS_ELEMS];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm0 = (wave / WAVES_N) * WM;
  const int wn0 = (wave % WAVES_N) * WN;
  const int h = lane >> 5, il = lane & 31;

  const int64_t gn = (a.N + BN - 1) / BN;
  const int64_t tix = xcd_tile_index();
  const int64_t m0 = (tix / gn) * BM;
  const int64_t n0 = (tix % gn) * BN;
  const int64_t kb = (int64_t)blockIdx.z * a.k_per_split;
  const int64_t ke = min(a.K, kb + a.k_per_split);
  const int nt = kb < ke ? (int)((ke - kb + BK - 1) / BK) : 0;

  floatx16 acc[TM][TN], lo[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = lo[i][j][r] = 0.f;

  // two register sets: the loads of k-tile t+2 are issued before the MFMAs of tile t, so a
  // tile's global loads have two tiles' MFMAs to land (one tile was too short a window)
  float4 ra0[NUA][RA], rb0[NUB][RB], ra1[NUA][RA], rb1[NUB][RB];
  auto load = [&](int t, float4 (&ra)[NUA][RA], float4 (&rb)[NUB][RB]) {
    const int64_t k0 = kb + (int64_t)t * BK;
    if (k0 + BK <= ke) {
      sb_load<BM, BK, A_KC, VEC, false>(ra, a.A, a.lda, m0, a.M, k0, ke, tid);
      sb_load<BN, BK, B_KC, VEC, false>(rb, a.B, a.ldb, n0, a.N, k0, ke, tid);
    } else {
      sb_load<BM, BK, A_KC, VEC, true>(ra, a.A, a.lda, m0, a.M, k0, ke, tid);
      sb_load<BN, BK, B_KC, VEC, true>(rb, a.B, a.ldb, n0, a.N, k0, ke, tid);
    }
  };
  auto sb_load_full = [&](int t, float4 (&ra)[NUA][RA], float4 (&rb)[NUB][RB]) {
    const int64_t k0 = kb + (int64_t)t * BK;
    sb_load<BM, BK, A_KC, VEC, false>(ra, a.A, a.lda, m0, a.M, k0, ke, tid);
    sb_load<BN, BK, B_KC, VEC, false>(rb, a.B, a.ldb, n0, a.N, k0, ke, tid);
  };
  auto store = [&](uint16_t* st, const float4 (&ra)[NUA][RA], const float4 (&rb)[NUB][RB]) {
    sb_store<BM, BK, A_KC, NUA, RA, PLANE>(st, 0, ra, tid);
    sb_store<BN, BK, B_KC, NUB, RB, PLANE>(st, BM, rb, tid);
  };
  // MFMAs over one stage: per 16-deep k step, the fragments of the wave's TM A rows and
  // TN B rows (3 planes each, ds_read_b128), then 6 products per accumulator, smallest
  // first (a1b1, a0b2, a2b0, a0b1, a1b0, a0b0)
  auto compute = [&](const uint16_t* st) {
#pragma unroll
    for (int s = 0; s < BK / 16; ++s) {
      const int c = 2 * s + h;
      bf16x8 af[TM][3];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = wm0 + 32 * i + il;
        const int off = row * BK + 8 * (c ^ sb_swz<BK>(row));
#pragma unroll
        for (int p = 0; p < 3; ++p) af[i][p] = *reinterpret_cast<const bf16x8*>(st + p * PLANE + off);
      }
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) {
        const int row = BM + wn0 + 32 * tn + il;
        const int off = row * BK + 8 * (c ^ sb_swz<BK>(row));
        bf16x8 bf[3];
#pragma unroll
        for (int p = 0; p < 3; ++p) bf[p] = *reinterpret_cast<const bf16x8*>(st + p * PLANE + off);
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          if (CTR_SB16_NOMFMA) {
            acc[i][tn][0] += (float)af[i][0][0] + (float)bf[0][0] + (float)af[i][1][1] +
                             (float)bf[1][1] + (float)af[i][2][2] + (float)bf[2][2];
            continue;
          }
          // a0b0 adds into the main accumulator, the five smaller products (<= 2^-7 of
          // it) into a second one, summed at the end: the main accumulator rounds once per
          // 16 k (the fp32 kernel: 8 times), so the split path is the more accurate one
          floatx16 v = lo[i][tn];
          v = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i][1], bf[1], v, 0, 0, 0);
          v = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i][0], bf[2], v, 0, 0, 0);
          v = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i][2], bf[0], v, 0, 0, 0);
          v = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i][0], bf[1], v, 0, 0, 0);
          v = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i][1], bf[0], v, 0, 0, 0);
          lo[i][tn] = v;
          acc[i][tn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i][0], bf[0], acc[i][tn], 0, 0, 0);
        }
      }
    }
  };

  auto stage = [&](int t) { return smem + (NS == 2 ? (t & 1) * STAGE : 0); };
  // one k-tile: prefetch tile t+2 into the free register set, MFMAs on tile t, then split
  // tile t+1 (loaded a tile earlier) into LDS
  auto step = [&](int t, float4 (&fa)[NUA][RA], float4 (&fb)[NUB][RB], float4 (&na)[NUA][RA],
                  float4 (&nb)[NUB][RB]) {
    if (t + 2 < nt) load(t + 2, fa, fb);
    compute(stage(t));
    if (NS == 1) __syncthreads();
    if (t + 1 < nt) store(stage(t + 1), na, nb);
    __syncthreads();
  };
  if (nt > 0) load(0, ra0, rb0);
  if (nt > 1) load(1, ra1, rb1);
  if (nt > 0) {
    store(stage(0), ra0, rb0);
    __syncthreads();
  }
  // steady state (NS == 2): a branch-free pair of k-tiles whose loads are never the K tail,
  // so each tile's MFMAs, the split of the next tile and its LDS stores form one scheduling
  // region; the group barriers ask for the split VALU to be threaded between the MFMAs
  // (an MFMA holds the issue port 8 of its 32 cycles; the rest is free for VALU)
  int t = 0;
  if (NS == 2) {
    constexpr int MF = (BK / 16) * TM * TN * 6;  // MFMAs per wave per k-tile
    auto full = [&](int tt, float4 (&fa)[NUA][RA], float4 (&fb)[NUB][RB],
                    float4 (&na)[NUA][RA], float4 (&nb)[NUB][RB]) {
      sb_load_full(tt + 2, fa, fb);
      compute(stage(tt));
      store(stage(tt + 1), na, nb);
#pragma unroll
      for (int i = 0; i < MF; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // 1 MFMA
        __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);  // 4 VALU

      }
      __syncthreads();
    };
    for (; t + 4 < nt; t += 2) {
      full(t, ra0, rb0, ra1, rb1);
      full(t + 1, ra1, rb1, ra0, rb0);
    }
  }
  for (; t < nt; t += 2) {
    step(t, ra0, rb0, ra1, rb1);  // set 0 is free (tile t is in LDS), set 1 holds t+1
    if (t + 1 < nt) step(t + 1, ra1, rb1, ra0, rb0);
  }
  __syncthreads();  // every stage read before the epilogue reuses the LDS
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] += lo[i][j];
  gemm_store_tiles<TM, TN>(a, acc, reinterpret_cast<float*>(smem) + wave * (32 * 36), m0 + wm0,
                           n0 + wn0, lane);
}

// ---- tilings + chooser -------------------------------------------------------------
struct Sb16Def {
  int bm, bn, bk, wm, wn, ns;
  int occ;     // blocks resident per CU (LDS / VGPR bound)
  double eff;  // sustained fraction of the per-CU split-bf16 peak (2.5 PF / 6 / 256)
};
static const Sb16Def kSb16[] = {
    {64, 64, 32, 2, 2, 2, 2, 0.45},   {128, 64, 32, 2, 2, 2, 2, 0.55},
    {64, 128, 32, 2, 2, 2, 2, 0.55},  {128, 128, 32, 2, 2, 2, 1, 0.65},
    {128, 160, 32, 4, 1, 2, 1, 0.65}, {64, 320, 32, 2, 2, 2, 1, 0.65},
    {128, 128, 32, 2, 2, 1, 2, 0.65},
    // M = 300 (DeepFM's dW0 = dH1^T.X): two 160-row tiles waste 6 % where 128 wastes 22 %
    {160, 128, 32, 1, 4, 2, 1, 0.65},
};
constexpr int kNumSb16 = sizeof(kSb16) / sizeof(kSb16[0]);

int sb16_num_tiles() { return kNumSb16; }

void sb16_tile_dims(int tile, int& bm, int& bn) {
  bm = kSb16[tile].bm;
  bn = kSb16[tile].bn;
}

// Makespan model as the exact kernel's chooser: blocks are dealt to 256 CUs x occ slots in
// rounds; a round costs one block's padded flops at the tiling's sustained per-CU rate
// (divided among the blocks sharing the CU) plus ~2 us; split-K adds its slab round trip.
// CTR_GEMM_CFG="tile,splits" forces a choice (tuning only).
Sb16Cfg sb16_choose(int64_t M, int64_t N, int64_t K) {
  auto mk = [&](int ti, int s) {
    Sb16Cfg c{ti, 1, std::max<int64_t>(K, 1), kSb16[ti].bm, kSb16[ti].bn};
    if (s > 1 && K >= 64) {
      c.kps = align_up(ceil_div(K, s), 32);
      c.splits = (int)ceil_div(K, c.kps);
    }
    return c;
  };
  if (const char* env = getenv("CTR_GEMM_CFG")) {
    int ti = -1, sp = 1;
    if (sscanf(env, "%d,%d", &ti, &sp) >= 1 && ti >= 0 && ti < kNumSb16 && sp >= 1)
      return mk(ti, sp);
  }
  const double per_cu = 2.5e15 / 6.0 / 256.0 / 1e6;  // flop per us per CU
  Sb16Cfg best = mk(0, 1);
  double best_t = 1e30;
  for (int ti = 0; ti < kNumSb16; ++ti) {
    const Sb16Def& d = kSb16[ti];
    const int64_t tiles = ceil_div(M, d.bm) * ceil_div(N, d.bn);
    for (int s = 1; s <= 32; ++s) {
      if (s > 1 && K / s < 256) break;
      const Sb16Cfg c = mk(ti, s);
      if (c.splits != s) continue;
      const int64_t blocks = tiles * c.splits;
      const int64_t slots = 256 * (int64_t)d.occ;
      const double rounds = (double)ceil_div(blocks, slots);
      const int64_t per_cu_blocks = std::min<int64_t>(d.occ, ceil_div(blocks, 256));
      const double kpad = (double)align_up(c.kps, d.bk);
      const double t_block =
          2.0 * d.bm * d.bn * kpad * per_cu_blocks / (per_cu * d.eff) + 2.0;
      double t = rounds * t_block;
      if (c.splits > 1) t += 2.0 * c.splits * (double)M * N * 4 / 5e6 + 3.0;
      if (t < best_t * 0.98) {
        best_t = t;
        best = c;
      }
    }
  }
  return best;
}

template <int BM, int BN, int BK, int WMW, int WNW, int NS, bool VEC>
static void sb16_launch_vec(const GemmArgs& a, bool ta, bool tb, dim3 grid, hipStream_t st) {
#define CTR_SB16_LAUNCH(TA_, TB_) \
  hipLaunchKernelGGL((gemm_sb16_kernel<BM, BN, BK, WMW, WNW, NS, TA_, TB_, VEC>), grid, 256, 0, st, a)
  if (!ta && !tb) CTR_SB16_LAUNCH(false, false);
  else if (!ta && tb) CTR_SB16_LAUNCH(false, true);
  else if (ta && !tb) CTR_SB16_LAUNCH(true, false);
  else CTR_SB16_LAUNCH(true, true);
#undef CTR_SB16_LAUNCH
}

template <int BM, int BN, int BK, int WMW, int WNW, int NS>
static void sb16_launch_cfg(const GemmArgs& a, bool ta, bool tb, dim3 grid, hipStream_t st) {
  if (a.vec_a && a.vec_b)
    sb16_launch_vec<BM, BN, BK, WMW, WNW, NS, true>(a, ta, tb, grid, st);
  else
    sb16_launch_vec<BM, BN, BK, WMW, WNW, NS, false>(a, ta, tb, grid, st);
}

void sb16_launch(const Sb16Cfg& c, const GemmArgs& a, bool ta, bool tb, dim3 grid, hipStream_t st) {
  switch (c.tile) {
    case 0: sb16_launch_cfg<64, 64, 32, 2, 2, 2>(a, ta, tb, grid, st); break;
    case 1: sb16_launch_cfg<128, 64, 32, 2, 2, 2>(a, ta, tb, grid, st); break;
    case 2: sb16_launch_cfg<64, 128, 32, 2, 2, 2>(a, ta, tb, grid, st); break;
    case 3: sb16_launch_cfg<128, 128, 32, 2, 2, 2>(a, ta, tb, grid, st); break;
    case 4: sb16_launch_cfg<128, 160, 32, 4, 1, 2>(a, ta, tb, grid, st); break;
    case 5: sb16_launch_cfg<64, 320, 32, 2, 2, 2>(a, ta, tb, grid, st); break;
    case 6: sb16_launch_cfg<128, 128, 32, 2, 2, 1>(a, ta, tb, grid, st); break;
    case 7: sb16_launch_cfg<160, 128, 32, 1, 4, 2>(a, ta, tb, grid, st); break;
  }
}

}  // namespace ctr

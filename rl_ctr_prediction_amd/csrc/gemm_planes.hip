// fp32-accurate GEMM on PRE-SPLIT operand planes — the DeepFM / IPNN MLP of the fused
// training step (p_model.py:276-293,322: Linear(F*K,300) -> Linear(300,200) -> Linear(200,1),
// forward and backward: 6 GEMMs per step, SURVEY.md §8d C3: 27.5 GFLOP).
//
// Numerics (as csrc/gemm_sb16.hip): every fp32 operand x is split EXACTLY into three bf16
// planes x = x0 + x1 + x2 (x0 = bf16_rne(x), x1 = bf16_rne(x - x0), x2 = x - x0 - x1); a
// product sums the six plane products with i + j <= 2 on the bf16 matrix cores, fp32
// accumulation (a0b0 in one accumulator, the five smaller products in a second; the
// dropped terms are <= 2^-23 |ab|). The fp32 value is recovered exactly as x0 + (x1 + x2).
//
// What is different here: the operands arrive ALREADY split, written once by their
// producers (the forward gather writes the MLP input's planes, each GEMM epilogue and the
// head kernel write the planes of the activations / gradients they produce, the weights
// are split once per step). A plane tensor is bf16 [3][rows_pad][cols_pad], rows and
// columns padded to multiples of 32 with ZEROS, so the k loop never has a tail and the
// kernel's staging is pure data movement: LDS-DMA (global_load_lds_dwordx4, 1 KiB per
// wave-instruction) straight into a 3-deep LDS ring, no VALU split, no register staging.
// Operands are read in the orientation they are stored in:
//   KC (k contiguous: X [B][F*K] for fwd0, nn.Linear weights [out][in]):
//       LDS image [rows][32 k] per plane, fragments by ds_read_b128;
//   RC (rows contiguous, k strided: W0 [300][1664] as dX's B operand, dH1 / X as dW0's
//       operands — the transposed products of the backward):
//       LDS image [32 k][rows] per plane, fragments by ds_read_b64_tr_b16 (the hardware
//       transpose read), so no transposed copy of any operand is ever written.
// Both images are XOR-swizzled (on the DMA's per-lane SOURCE address; the DMA destination is
// lane-linear) so that every fragment read is bank-conflict free.
//
// MFMA: v_mfma_f32_16x16x32_bf16 — a 32-deep k step per instruction (one LDS stage), 16-row
// granularity (N = 300 pads to 320, not 384), and per the MI355X measurements the shape the
// chip holds the higher clock on.
#include "gemm_common.h"

namespace ctr {

typedef __bf16 pbf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 pbf16x4 __attribute__((ext_vector_type(4)));
typedef float pf32x4 __attribute__((ext_vector_type(4)));
#define CTR_LDS __attribute__((address_space(3)))

constexpr int kPBK = 32;  // k per LDS stage = one 16x16x32 MFMA

// the software-pipelined stage of the k-contiguous x k-contiguous products with >= 4
// 16-column groups per wave (fwd0's 64 x 160 tiling: B fragments of group tn+1 read under the
// MFMAs of group tn, the DMA pieces spread between the groups): fwd0 69.2 -> 59.7 us
// standalone at C3 (tools/gemm_planes_bench.py, profiles/r06_gemm_pipe.txt); fwd1's 32 x 32
// waves (two groups) ran slower that way (17.4 -> 19.1 us) and keep the burst form
#ifndef CTR_PL_PIPE
#define CTR_PL_PIPE 1
#endif
#ifndef CTR_PL_PIPE2
#define CTR_PL_PIPE2 0
#endif

struct PlaneSrc {
  const uint16_t* p;  // plane 0 (bf16 bits); planes `ps` elements apart
  int64_t ld;         // elements per storage row
  int64_t ps;         // elements between planes
  int64_t rows;       // storage rows
  int64_t cols;       // storage columns
};

struct PlanesArgs {
  int64_t Kp;           // padded k extent (multiple of 32)
  int64_t k_per_split;  // multiple of 32
  PlaneSrc A, B;
  GemmArgs g;           // M, N, C, ldc, epilogue, split-K slab stride
  uint16_t* cpl;        // output planes (nullptr: none)
  int64_t cpl_ld, cpl_ps;
  float* last_col;      // non-null: result column N-1 goes to last_col[m], C has N-1 columns
  int xcd_ngroups;      // tiles partitioned over the 8 XCDs as (8/g) M-groups x g N-groups
  int splits;           // > 1: split-K, (tile, split) flattened into blockIdx.x (see below)
  int64_t tiles;        // output tiles per split
};

// ---- LDS image swizzles ----------------------------------------------------------------
// KC image: [rows][32 k] bf16 = 64-B rows, four 16-B chunks. The 16x16x32 A/B fragment of
// lane l is row (l & 15), chunk (l >> 4); a ds_read_b128 is serviced in 16-lane groups
// {0-3,12-15,20-27}, {4-11,16-19,28-31}, ... The chunk is XORed with g(row quad) where
// g = {0, 2, 3, 1}: every group then touches 16 distinct 16-B slots of a 256-B bank row.
__device__ __forceinline__ int kc_swz(int r) { return (0x78 >> (2 * ((r >> 2) & 3))) & 3; }

// RC image: [32 k][R] bf16, R in {64, 128} (128- or 256-B rows) in 32-B blocks of 16
// columns. A ds_read_b64_tr_b16 16-lane group reads 4 k rows x one block; the two groups of
// a 32-lane half read k rows {4j..4j+3} and {8+4j..8+4j+3} of the same block. The block is
// XORed with a key of the row that spreads those 8 rows over 8 distinct 32-B slots.
template <int R>
__device__ __forceinline__ int rc_swz(int k) {
  if (R == 128) return (k & 3) | (((k >> 3) & 1) << 2);
  return ((k >> 1) & 1) | (((k >> 3) & 1) << 1);  // R == 64: two rows per bank row
}

// ---- LDS-DMA source addresses (one lane's 16 B of a 1 KiB piece) -------------------
// KC: piece c covers image rows 16c..16c+15, lane -> (row lane/4, swizzled chunk lane%4).
__device__ __forceinline__ const uint16_t* piece_kc(const PlaneSrc& s, int plane, int c,
                                                    int64_t row0, int64_t k0, int lane) {
  const int r = c * 16 + (lane >> 2);
  const int ch = (lane & 3) ^ kc_swz(r);
  int64_t row = row0 + r;
  row = row < s.rows ? row : s.rows - 1;  // clamped rows only feed never-stored outputs
  return s.p + plane * s.ps + row * s.ld + k0 + 8 * ch;
}

// RC: piece c covers image rows c*RPI .. +RPI-1 (k), lane -> (row, 16-B piece of the row).
template <int R>
__device__ __forceinline__ const uint16_t* piece_rc(const PlaneSrc& s, int plane, int c,
                                                    int64_t col0, int64_t k0, int lane) {
  constexpr int PPR = R / 8;     // 16-B pieces per image row
  constexpr int RPI = 64 / PPR;  // image rows per 1 KiB piece
  const int kr = c * RPI + lane / PPR;
  const int pc = lane % PPR;
  const int blk = (pc >> 1) ^ rc_swz<R>(kr);
  int64_t col = col0 + 16 * blk;
  col = col <= s.cols - 16 ? col : s.cols - 16;
  return s.p + plane * s.ps + (k0 + kr) * s.ld + col + 8 * (pc & 1);
}

// An RC operand tile wider than 128 (the weight gradients' whole-M tiles: 192, 256, 320)
// is held as several [32 k][64] images side by side (4 KiB each per plane); 64 and 128 are
// one image. Piece c of a plane: image c / (R/16), piece c % (R/16) of that image.
template <int BX>
constexpr int rc_img() { return BX == 128 ? 128 : 64; }

template <int R>
__device__ __forceinline__ const uint16_t* piece_rc_img(const PlaneSrc& s, int plane, int c,
                                                        int64_t col0, int64_t k0, int lane) {
  constexpr int PPI = R / 16;  // 1 KiB pieces per image
  return piece_rc<R>(s, plane, c % PPI, col0 + (int64_t)R * (c / PPI), k0, lane);
}

// ---- fragment reads ---------------------------------------------------------------
// Byte offsets (within one plane image) of a lane's fragment reads: computed once per
// kernel, so the k loop issues bare LDS reads.
__device__ __forceinline__ int frag_kc_off(int rb, int lane) {
  const int r = rb + (lane & 15);
  return r * 64 + ((lane >> 4) ^ kc_swz(r)) * 16;
}

template <int R>
__device__ __forceinline__ int frag_rc_off(int cb, int lane, int j) {
  const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
  const int k = 8 * g + 4 * j + q;
  return k * (2 * R) + 32 * ((cb >> 4) ^ rc_swz<R>(k)) + 8 * pp;
}

template <int R>
__device__ __forceinline__ int frag_rc_img_off(int cb, int lane, int j) {
  return (cb / R) * (R * kPBK * 2) + frag_rc_off<R>(cb % R, lane, j);
}

__device__ __forceinline__ pbf16x8 frag_kc_at(const char* p) {
  return *reinterpret_cast<const pbf16x8*>(p);
}

// the same read as an asm statement (waited for by hand, CTR_PL_PIPE2)
__device__ __forceinline__ pbf16x8 frag_kc_asm(const char* p) {
  pbf16x8 v;
  const uint32_t a = (uint32_t)(uintptr_t)(const CTR_LDS char*)p;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(a));
  return v;
}

// The transpose reads as inline asm (CTR_PL_TR_ASM, default): with the builtin, hipcc 7.2
// cannot tell the read from the LDS-DMA writes in flight and waits vmcnt(0) before it — the
// next stage's DMA then lands before the current stage computes (no load/compute overlap in
// any GEMM with a k-strided operand). The asm form is invisible to the wait pass, so its
// results are waited for explicitly (planes_wait_lds) before the MFMAs that use them.
#ifndef CTR_PL_TR_ASM
#define CTR_PL_TR_ASM 1
#endif
__device__ __forceinline__ pbf16x8 frag_rc_at(const char* p0, const char* p1) {
#if CTR_PL_TR_ASM
  pbf16x4 v0, v1;
  const uint32_t a0 = (uint32_t)(uintptr_t)(const CTR_LDS char*)p0;
  const uint32_t a1 = (uint32_t)(uintptr_t)(const CTR_LDS char*)p1;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v0) : "v"(a0));
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v1) : "v"(a1));
#else
  const pbf16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((CTR_LDS pbf16x4*)p0);
  const pbf16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((CTR_LDS pbf16x4*)p1);
#endif
  return __builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7);
}

// every LDS read issued so far has landed (the asm transpose reads are not tracked by the
// compiler), and no MFMA is hoisted above this point (cdna_hip_programming.md rule 18)
__device__ __forceinline__ void planes_wait_lds() {
#if CTR_PL_TR_ASM
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
#endif
}

// ---- epilogue --------------------------------------------------------------------
__device__ __forceinline__ void store_planes4(const PlanesArgs& a, int64_t m, int64_t n, float4 o) {
  uint16_t* base = a.cpl + m * a.cpl_ld + n;
  if (n + 3 < a.g.N) {
    uint2 pl[3];
    psplit4(o, pl);
#pragma unroll
    for (int p = 0; p < 3; ++p) *reinterpret_cast<uint2*>(base + p * a.cpl_ps) = pl[p];
  } else {
    const float e[4] = {o.x, o.y, o.z, o.w};
    for (int j = 0; j < 4 && n + j < a.g.N; ++j) {
      uint16_t h[3];
      psplit1(e[j], h);
#pragma unroll
      for (int p = 0; p < 3; ++p) base[p * a.cpl_ps + j] = h[p];
    }
  }
}

// one wave's TM x TN 16x16 accumulators (C/D map: col = lane & 15, row = 4*(lane>>4) + r)
// through a wave-private [16][WN+4] LDS strip, then row-contiguous float4 stores
template <int TM, int TN>
__device__ __forceinline__ void planes_store(const PlanesArgs& a, pf32x4 (&acc)[TM][TN],
                                             float* strip, int64_t mb, int64_t nb, int lane,
                                             int64_t split) {
  constexpr int WN = 16 * TN, LD = WN + 4, C4 = WN / 4;
  const GemmArgs& g = a.g;
  float* C = g.C + split * g.slab_stride;
  const bool slab = g.slab_stride != 0;
  const int epi = slab ? (int)CTR_EPI_NONE : g.epi;
  GemmArgs ge = g;
  if (epi == CTR_EPI_BIAS_RELU_DROP && ge.step_ptr) ge.offset += (uint64_t)(*ge.step_ptr) << 32;
  const bool planes = a.cpl && !slab;
  float* const lastc = slab ? nullptr : a.last_col;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
#pragma unroll
    for (int tn = 0; tn < TN; ++tn)
#pragma unroll
      for (int r = 0; r < 4; ++r) strip[(4 * (lane >> 4) + r) * LD + 16 * tn + (lane & 15)] = acc[i][tn][r];
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): wave-private strip, no barrier
    __builtin_amdgcn_wave_barrier();
    for (int idx = lane; idx < 16 * C4; idx += 64) {
      const int row = idx / C4, c4 = idx - row * C4;
      const int64_t m = mb + 16 * i + row;
      const int64_t n = nb + 4 * c4;
      if (m >= g.M || n >= g.N) continue;
      const float4 v = *reinterpret_cast<const float4*>(strip + row * LD + 4 * c4);
      float4 o;
      o.x = apply_epi(ge, epi, v.x, m, n + 0);
      o.y = n + 1 < g.N ? apply_epi(ge, epi, v.y, m, n + 1) : 0.f;
      o.z = n + 2 < g.N ? apply_epi(ge, epi, v.z, m, n + 2) : 0.f;
      o.w = n + 3 < g.N ? apply_epi(ge, epi, v.w, m, n + 3) : 0.f;
      if (C) {
        float* crow = C + m * g.ldc;
        const int64_t nc = lastc ? g.N - 1 : g.N;  // columns that go to C
        if (g.vec_c && n + 3 < nc) {
          *reinterpret_cast<float4*>(crow + n) = o;
        } else {
          const float e[4] = {o.x, o.y, o.z, o.w};
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            if (n + j < nc) crow[n + j] = e[j];
            else if (lastc && n + j == nc) lastc[m] = e[j];
          }
        }
      }
      if (planes) store_planes4(a, m, n, o);
    }
    __builtin_amdgcn_wave_barrier();
  }
}

// Block -> output tile. Under round-robin dispatch blocks b, b+8, b+16... share an XCD; the
// tiles are dealt so that each XCD owns a contiguous (M-group x N-group) sub-grid and walks
// it M-row by M-row (the row's tiles back to back, its A strip L2-hot for all of them):
// g = 1 gives each XCD whole M rows (every XCD reads all of B), g = 2 gives each XCD half
// of the N tiles of a quarter of the M rows (dX: each XCD's share of W0 is 1.6 of 3.2 MB,
// so it stays in the 4 MiB L2 beside the streamed dH1 rows). Falls back to g = 1, then to
// the identity, where the grid does not divide.
// g = 3: whole M rows per XCD as g = 1, but each XCD walks its rows N-tile-major (one B
// column strip for all of its M rows, then the next): its A rows (dX: 16 x 123 KB of dH1
// planes) stay L2-resident while each B strip streams through once per XCD, instead of all
// of B once per M row (round-4 counters: dX 160 MB of HBM traffic against 72 algorithmic).
__device__ __forceinline__ int64_t planes_tile_index(int64_t gn, int g) {
  const int64_t T = gridDim.x;
  const int64_t b = blockIdx.x;
  if (T % 8 != 0) return b;
  const int64_t x = b % 8, i = b / 8;
  const int64_t gm = T / gn;
  if (g == 3 && gm % 8 == 0) {
    const int64_t gmx = gm / 8;
    return (x * gmx + i % gmx) * gn + i / gmx;
  }
  if (g > 1 && 8 % g == 0 && gn % g == 0 && gm % (8 / g) == 0) {
    const int64_t gnn = gn / g, gmm = gm / (8 / g);
    const int64_t mt = (x / g) * gmm + i / gnn, nt = (x % g) * gnn + i % gnn;
    return mt * gn + nt;
  }
  return x * (T / 8) + i;
}

// ---- the kernel ---------------------------------------------------------------------
// Block = WAVES_M x WAVES_N waves, tile BM x BN; a wave owns (BM/WAVES_M) x (BN/WAVES_N) as
// TM x TN 16x16 accumulators (x2: the a0b0 accumulator and the small-products one).
// NS-deep LDS ring of 32-deep k stages; one barrier per stage; the DMA of stage t+NS-1 is
// issued right after the barrier of stage t and stays in flight (counted vmcnt) under the
// MFMAs of stages t .. t+NS-2.
// KS: 32-deep MFMA k-steps per ring stage (1 or 2): KS = 2 halves the barriers per k
// (the guide's BK 32 -> 64) at twice the LDS per stage.
template <int BM, int BN, int WAVES_M, int WAVES_N, bool A_RC, bool B_RC, int NS, int KS = 1>
__global__ __launch_bounds__(64 * WAVES_M* WAVES_N) void gemm_planes_kernel(PlanesArgs a) {
  constexpr int NW = WAVES_M * WAVES_N;
  constexpr int WM = BM / WAVES_M, WN = BN / WAVES_N;
  constexpr int TM = WM / 16, TN = WN / 16;
  static_assert(WM % 16 == 0 && WN % 16 == 0, "wave tile in 16x16 MFMA blocks");
  static_assert(!A_RC || BM == 128 || BM % 64 == 0, "RC operand tiles of 128 or 64 * n");
  static_assert(!B_RC || BN == 128 || BN % 64 == 0, "RC operand tiles of 128 or 64 * n");
  constexpr int RA = rc_img<BM>(), RB = rc_img<BN>();  // RC image widths
  static_assert(NS >= 2 && NS <= 7, "2- to 7-deep LDS ring");
  static_assert(KS == 1 || KS == 2, "1 or 2 MFMA k-steps per stage");
  constexpr int A_PL = BM * kPBK * 2, B_PL = BN * kPBK * 2;  // bytes per plane image
  constexpr int SUB = 3 * (A_PL + B_PL);                     // one 32-deep k-step's images
  constexpr int STAGE = KS * SUB;
  constexpr int NIA1 = 3 * BM / 16, NIB1 = 3 * BN / 16;  // 1 KiB pieces per k-step
  constexpr int NIA = KS * NIA1, NIB = KS * NIB1;        // ... per stage
  constexpr int EPI = NW * 16 * (WN + 4) * 4;
  constexpr int LDS = NS * STAGE > EPI ? NS * STAGE : EPI;
  // ONE shared object: a second one can make hipcc wait vmcnt(0) before LDS reads
  __shared__ __attribute__((aligned(1024))) char smem[LDS];

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm0 = (wave / WAVES_N) * WM;
  const int wn0 = (wave % WAVES_N) * WN;

  const int64_t gn = (a.g.N + BN - 1) / BN;
  int64_t tix, split = 0;
  if (a.splits > 1) {
    // split-K: block b -> XCD b % 8 -> the XCD's contiguous range of (split, tile) pairs,
    // split-major, so the blocks of one k range (which share both operands' k slices) run
    // on one XCD and each operand slice is fetched into ~one L2 (grid padded to 8 | T; the
    // padding blocks exit here, before any barrier)
    const int64_t T = gridDim.x, b = blockIdx.x;
    const int64_t j = (b % 8) * (T / 8) + b / 8;
    if (j >= a.tiles * a.splits) return;
    split = j / a.tiles;
    tix = j % a.tiles;
  } else {
    tix = planes_tile_index(gn, a.xcd_ngroups);
  }
  const int64_t m0 = (tix / gn) * BM;
  const int64_t n0 = (tix % gn) * BN;
  const int64_t kb = split * a.k_per_split;
  const int64_t ke = min(a.Kp, kb + a.k_per_split);
  const int nt = kb < ke ? (int)((ke - kb) / (kPBK * KS)) : 0;  // stages

  pf32x4 acc[TM][TN], lo[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = lo[i][j] = (pf32x4){0.f, 0.f, 0.f, 0.f};

  // The wave's LDS-DMA pieces: A's 3*BM/16 and B's 3*BN/16 1-KiB pieces of a stage are dealt
  // round-robin over the waves (a wave short of a piece re-issues the operand's last one:
  // the same bytes to the same place), so every wave issues exactly IPW per stage and the
  // counted vmcnt is a constant. Per piece: the lane's byte offset from the operand base at
  // the split's first k (computed once) and the uniform LDS offset in a stage; stage t adds
  // t * (32 k) to the base.
  constexpr int IPWA = (NIA + NW - 1) / NW, IPWB = (NIB + NW - 1) / NW;
  const PlaneSrc SA = a.A, SB = a.B;
  uint32_t offA[IPWA], offB[IPWB];
  int ldsA[IPWA], ldsB[IPWB];
#pragma unroll
  for (int j = 0; j < IPWA; ++j) {
    const int ins = min(wave + NW * j, NIA - 1);
    const int ks = ins / NIA1, r = ins % NIA1;
    const int plane = r / (BM / 16), c = r % (BM / 16);
    ldsA[j] = ks * SUB + plane * A_PL + c * 1024;
    const int64_t k0 = kb + ks * kPBK;
    const uint16_t* p = A_RC ? piece_rc_img<RA>(SA, plane, c, m0, k0, lane)
                             : piece_kc(SA, plane, c, m0, k0, lane);
    offA[j] = (uint32_t)((const char*)p - (const char*)SA.p);
  }
#pragma unroll
  for (int j = 0; j < IPWB; ++j) {
    const int ins = min(wave + NW * j, NIB - 1);
    const int ks = ins / NIB1, r = ins % NIB1;
    const int plane = r / (BN / 16), c = r % (BN / 16);
    ldsB[j] = ks * SUB + 3 * A_PL + plane * B_PL + c * 1024;
    const int64_t k0 = kb + ks * kPBK;
    const uint16_t* p = B_RC ? piece_rc_img<RB>(SB, plane, c, n0, k0, lane)
                             : piece_kc(SB, plane, c, n0, k0, lane);
    offB[j] = (uint32_t)((const char*)p - (const char*)SB.p);
  }
  const int64_t stepA = 2 * (A_RC ? kPBK * KS * SA.ld : kPBK * KS);  // bytes per stage along k
  const int64_t stepB = 2 * (B_RC ? kPBK * KS * SB.ld : kPBK * KS);
#define CTR_PL_ISSUE(t_)                                                                       \
  do {                                                                                         \
    char* st_ = smem + ((t_) % NS) * STAGE;                                                    \
    const char* ba_ = (const char*)SA.p + (int64_t)(t_) * stepA;                               \
    const char* bb_ = (const char*)SB.p + (int64_t)(t_) * stepB;                               \
    _Pragma("unroll") for (int j_ = 0; j_ < IPWA; ++j_)                                        \
        __builtin_amdgcn_global_load_lds((const void*)(ba_ + offA[j_]), (CTR_LDS void*)(st_ + ldsA[j_]), 16, 0, 0); \
    _Pragma("unroll") for (int j_ = 0; j_ < IPWB; ++j_)                                        \
        __builtin_amdgcn_global_load_lds((const void*)(bb_ + offB[j_]), (CTR_LDS void*)(st_ + ldsB[j_]), 16, 0, 0); \
  } while (0)

  int aoff[TM][2], boff[TN][2];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    aoff[i][0] = A_RC ? frag_rc_img_off<RA>(wm0 + 16 * i, lane, 0) : frag_kc_off(wm0 + 16 * i, lane);
    aoff[i][1] = A_RC ? frag_rc_img_off<RA>(wm0 + 16 * i, lane, 1) : 0;
  }
#pragma unroll
  for (int i = 0; i < TN; ++i) {
    boff[i][0] = B_RC ? frag_rc_img_off<RB>(wn0 + 16 * i, lane, 0) : frag_kc_off(wn0 + 16 * i, lane);
    boff[i][1] = B_RC ? frag_rc_img_off<RB>(wn0 + 16 * i, lane, 1) : 0;
  }

  auto compute_sub = [&](const char* st) {
    pbf16x8 af[TM][3];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        const char* img = st + p * A_PL;
        af[i][p] = A_RC ? frag_rc_at(img + aoff[i][0], img + aoff[i][1]) : frag_kc_at(img + aoff[i][0]);
      }
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) {
      pbf16x8 bf[3];
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        const char* img = st + 3 * A_PL + p * B_PL;
        bf[p] = B_RC ? frag_rc_at(img + boff[tn][0], img + boff[tn][1]) : frag_kc_at(img + boff[tn][0]);
      }
      if (A_RC || B_RC) planes_wait_lds();
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        // a0b0 into the main accumulator; the five products <= 2^-7 of it (smallest first)
        // into the second, summed at the end
        pf32x4 v = lo[i][tn];
        v = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][1], bf[1], v, 0, 0, 0);
        v = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][0], bf[2], v, 0, 0, 0);
        v = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][2], bf[0], v, 0, 0, 0);
        v = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][0], bf[1], v, 0, 0, 0);
        v = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][1], bf[0], v, 0, 0, 0);
        lo[i][tn] = v;
        acc[i][tn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][0], bf[0], acc[i][tn], 0, 0, 0);
      }
    }
  };
  auto compute = [&](int slot) {
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) compute_sub(smem + slot * STAGE + ks * SUB);
  };

  constexpr int IPW = IPWA + IPWB;
#if CTR_PL_PIPE2
  if constexpr ((A_RC || B_RC) && KS == 1) {
    // The pipelined stage for products with a k-strided operand: every fragment read is an
    // asm statement (the compiler's wait pass cannot count the transpose reads, and its
    // conservative lgkmcnt(0) for its own reads would drain them too), waited for by hand:
    // the B fragments of group tn+1 are in flight (lgkmcnt(NBR)) under the MFMAs of group
    // tn, and the next stage's DMA pieces are spread between the groups.
    constexpr int NBR = 3 * (B_RC ? 2 : 1);
    const int tlast = nt - 1;
    auto issue_piece = [&](int j, int ts) {
      char* st_ = smem + (ts % NS) * STAGE;
      const int tsrc = min(ts, tlast);
      if (j < IPWA)
        __builtin_amdgcn_global_load_lds((const void*)((const char*)SA.p + (int64_t)tsrc * stepA + offA[j]),
                                         (CTR_LDS void*)(st_ + ldsA[j]), 16, 0, 0);
      else
        __builtin_amdgcn_global_load_lds((const void*)((const char*)SB.p + (int64_t)tsrc * stepB + offB[j - IPWA]),
                                         (CTR_LDS void*)(st_ + ldsB[j - IPWA]), 16, 0, 0);
    };
    if (nt > 0) {
#pragma unroll
      for (int s = 0; s < NS - 1; ++s)
#pragma unroll
        for (int j = 0; j < IPW; ++j) issue_piece(j, s);
    }
    for (int t = 0; t < nt; ++t) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(IPW * (NS - 2)) : "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      const char* st = smem + (t % NS) * STAGE;
      if constexpr (NS <= 2) {  // a 2-deep ring: the next stage's pieces go out first
#pragma unroll
        for (int j = 0; j < IPW; ++j) issue_piece(j, t + NS - 1);
      }
      pbf16x8 af[TM][3], bf[2][3];
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int p = 0; p < 3; ++p) {
          const char* img = st + p * A_PL;
          af[i][p] = A_RC ? frag_rc_at(img + aoff[i][0], img + aoff[i][1])
                          : frag_kc_asm(img + aoff[i][0]);
        }
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        const char* img = st + 3 * A_PL + p * B_PL;
        bf[0][p] = B_RC ? frag_rc_at(img + boff[0][0], img + boff[0][1])
                        : frag_kc_asm(img + boff[0][0]);
      }
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) {
        const int cb = tn & 1;
        if (tn + 1 < TN) {
#pragma unroll
          for (int p = 0; p < 3; ++p) {
            const char* img = st + 3 * A_PL + p * B_PL;
            bf[cb ^ 1][p] = B_RC ? frag_rc_at(img + boff[tn + 1][0], img + boff[tn + 1][1])
                                 : frag_kc_asm(img + boff[tn + 1][0]);
          }
          asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(NBR) : "memory");
        } else {
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        }
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (NS > 2) {  // deeper rings: the pieces spread between the groups
          const int j0 = (IPW * tn) / TN, j1 = (IPW * (tn + 1)) / TN;
#pragma unroll
          for (int j = 0; j < IPW; ++j)
            if (j >= j0 && j < j1) issue_piece(j, t + NS - 1);
        }
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          pf32x4 v = lo[i][tn];
          v = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][1], bf[cb][1], v, 0, 0, 0);
          v = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][0], bf[cb][2], v, 0, 0, 0);
          v = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][2], bf[cb][0], v, 0, 0, 0);
          v = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][0], bf[cb][1], v, 0, 0, 0);
          v = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][1], bf[cb][0], v, 0, 0, 0);
          lo[i][tn] = v;
          acc[i][tn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][0], bf[cb][0], acc[i][tn], 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  } else
#endif
#if CTR_PL_PIPE
  if constexpr (!A_RC && !B_RC && KS == 1 && TN >= 4) {
    // Software-pipelined stage (both operands k-contiguous): the B fragments of 16-column
    // group tn+1 are read while the MFMAs of group tn run, and the stage's LDS-DMA pieces
    // for stage t+NS-1 are issued between the groups instead of in one burst at the
    // barrier (the scheduler order is pinned by sched_group_barrier). The DMA is issued
    // every iteration — past the last stage it re-loads the last stage into the ring slot
    // nobody reads again — so the wait count is the constant IPW * (NS-2).
    const int tlast = nt - 1;
    auto issue_piece = [&](int j, int ts) {
      char* st_ = smem + (ts % NS) * STAGE;
      const int tsrc = min(ts, tlast);
      if (j < IPWA)
        __builtin_amdgcn_global_load_lds((const void*)((const char*)SA.p + (int64_t)tsrc * stepA + offA[j]),
                                         (CTR_LDS void*)(st_ + ldsA[j]), 16, 0, 0);
      else
        __builtin_amdgcn_global_load_lds((const void*)((const char*)SB.p + (int64_t)tsrc * stepB + offB[j - IPWA]),
                                         (CTR_LDS void*)(st_ + ldsB[j - IPWA]), 16, 0, 0);
    };
    if (nt > 0) {
#pragma unroll
      for (int s = 0; s < NS - 1; ++s)
#pragma unroll
        for (int j = 0; j < IPW; ++j) issue_piece(j, s);
    }
    for (int t = 0; t < nt; ++t) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(IPW * (NS - 2)) : "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      const char* st = smem + (t % NS) * STAGE;
      pbf16x8 af[TM][3], bf[2][3];
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int p = 0; p < 3; ++p) af[i][p] = frag_kc_at(st + p * A_PL + aoff[i][0]);
#pragma unroll
      for (int p = 0; p < 3; ++p) bf[0][p] = frag_kc_at(st + 3 * A_PL + p * B_PL + boff[0][0]);
      __builtin_amdgcn_sched_group_barrier(0x100, 3 * TM + 3, 0);
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) {
        const int cb = tn & 1;
        if (tn + 1 < TN) {
#pragma unroll
          for (int p = 0; p < 3; ++p)
            bf[cb ^ 1][p] = frag_kc_at(st + 3 * A_PL + p * B_PL + boff[tn + 1][0]);
          __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);
        }
        // this group's share of the next stage's DMA pieces
        const int j0 = (IPW * tn) / TN, j1 = (IPW * (tn + 1)) / TN;
#pragma unroll
        for (int j = 0; j < IPW; ++j)
          if (j >= j0 && j < j1) {
            issue_piece(j, t + NS - 1);
            __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
          }
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          pf32x4 v = lo[i][tn];
          v = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][1], bf[cb][1], v, 0, 0, 0);
          v = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][0], bf[cb][2], v, 0, 0, 0);
          v = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][2], bf[cb][0], v, 0, 0, 0);
          v = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][0], bf[cb][1], v, 0, 0, 0);
          v = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][1], bf[cb][0], v, 0, 0, 0);
          lo[i][tn] = v;
          acc[i][tn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][0], bf[cb][0], acc[i][tn], 0, 0, 0);
        }
        __builtin_amdgcn_sched_group_barrier(0x008, 6 * TM, 0);
      }
    }
  } else
#endif
  {
  // prologue: stages 0 .. NS-2 in flight
#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < nt) CTR_PL_ISSUE(s);
  for (int t = 0; t < nt; ++t) {
    // this wave's pieces of stage t have landed; the q younger stages stay in flight ...
    const int q = min(nt - 1 - t, NS - 2);
    if (q <= 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#define CTR_PL_WAITQ(Q_)                                                          \
    if constexpr (NS - 2 >= Q_) {                                                 \
      if (q == Q_) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(IPW * Q_) : "memory"); \
    }
    CTR_PL_WAITQ(1) CTR_PL_WAITQ(2) CTR_PL_WAITQ(3) CTR_PL_WAITQ(4) CTR_PL_WAITQ(5)
#undef CTR_PL_WAITQ
    // ... and every wave's (and every wave is done reading the slot refilled next)
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (t + NS - 1 < nt) CTR_PL_ISSUE(t + NS - 1);
    compute(t % NS);
  }
  }
#undef CTR_PL_ISSUE
  __syncthreads();  // every stage read before the epilogue reuses the LDS
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] += lo[i][j];
  planes_store<TM, TN>(a, acc, reinterpret_cast<float*>(smem) + wave * 16 * (WN + 4),
                       m0 + wm0, n0 + wn0, lane, split);
}

// split-K: sum the fp32 slabs in split order (16 independent loads in flight per step of
// the chain), then the epilogue (fp32 out and/or planes); one thread per 4 columns
// slabs: [splits][M][sld], sld = align_up(N, 4) (the padding columns are never read as
// results), so every row starts 16-B aligned and the float4 path always applies
__global__ __launch_bounds__(64) void planes_reduce_kernel(PlanesArgs a, const float* __restrict__ slabs,
                                                           int splits, int64_t sld) {
  GemmArgs g = a.g;
  if (g.epi == CTR_EPI_BIAS_RELU_DROP && g.step_ptr) g.offset += (uint64_t)(*g.step_ptr) << 32;
  const int64_t n4 = (g.N + 3) / 4;
  const int64_t total = g.M * n4;
  const int64_t slab = g.M * sld;
  const bool vec = true;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t m = t / n4, n = 4 * (t - m * n4);
    const int64_t o = m * sld + n;
    float e[4];
    if (vec) {
      // up to 16 slabs' loads in flight per step of the (ordered) sum chain: dW0's 9 slabs in
      // one memory round trip, dW1's 32 in two (a first load, then batches of 8, took 2 and
      // 5: 11 us per reduce at C3)
      float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
      for (int z = 0; z < splits; z += 16) {
        float4 v[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) {  // past the last slab: a clamped (unused) load, no branch
          const int zj = min(z + j, splits - 1);
          v[j] = *reinterpret_cast<const float4*>(slabs + (int64_t)zj * slab + o);
        }
#pragma unroll
        for (int j = 0; j < 16; ++j) {  // selects, not branches (the loads stay batched)
          const bool first = z + j == 0, add = z + j < splits && !first;
          s.x = first ? v[j].x : add ? s.x + v[j].x : s.x;
          s.y = first ? v[j].y : add ? s.y + v[j].y : s.y;
          s.z = first ? v[j].z : add ? s.z + v[j].z : s.z;
          s.w = first ? v[j].w : add ? s.w + v[j].w : s.w;
        }
      }
      e[0] = s.x; e[1] = s.y; e[2] = s.z; e[3] = s.w;
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        e[j] = 0.f;
        if (n + j >= g.N) continue;
        float s = slabs[o + j];
        for (int z = 1; z < splits; ++z) s += slabs[(int64_t)z * slab + o + j];
        e[j] = s;
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (n + j < g.N) e[j] = apply_epi(g, g.epi, e[j], m, n + j);
    if (g.C) {
      float* crow = g.C + m * g.ldc;
      const int64_t nc = a.last_col ? g.N - 1 : g.N;
      for (int j = 0; j < 4 && n + j < g.N; ++j) {
        if (n + j < nc) crow[n + j] = e[j];
        else a.last_col[m] = e[j];
      }
    }
    if (a.cpl) store_planes4(a, m, n, make_float4(e[0], e[1], e[2], e[3]));
  }
}

// fp32 [rows][cols] (row stride ld) -> planes [3][.][.] (row stride dst_ld, plane stride
// dst_ps); only the valid region is written (the zero padding is the allocation's)
__global__ __launch_bounds__(256) void split_planes_kernel(const float* __restrict__ src, int64_t rows,
                                                           int64_t cols, int64_t ld,
                                                           uint16_t* __restrict__ dst,
                                                           int64_t dst_ld, int64_t dst_ps,
                                                           bool vec) {
  const int64_t c4 = (cols + 3) / 4;
  const int64_t total = rows * c4;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = t / c4, c = 4 * (t - r * c4);
    const float* s = src + r * ld + c;
    uint16_t* d = dst + r * dst_ld + c;
    if (vec && c + 3 < cols) {
      uint2 pl[3];
      psplit4(*reinterpret_cast<const float4*>(s), pl);
#pragma unroll
      for (int p = 0; p < 3; ++p) *reinterpret_cast<uint2*>(d + p * dst_ps) = pl[p];
    } else {
      for (int j = 0; j < 4 && c + j < cols; ++j) {
        uint16_t h[3];
        psplit1(s[j], h);
#pragma unroll
        for (int p = 0; p < 3; ++p) d[p * dst_ps + j] = h[p];
      }
    }
  }
}

// ---- tilings + chooser ----------------------------------------------------------------
struct PlDef {
  int bm, bn, wm, wn, ns;
  int occ;     // blocks resident per CU (LDS bound)
  double eff;  // sustained fraction of the per-CU bf16 MFMA peak (model only)
  int ks = 1;  // 32-deep k-steps per ring stage
};
static const PlDef kPl[] = {
    {64, 160, 2, 2, 3, 1, 0.60},   // 0: fwd0 / dH1-shaped (N = 300 -> 320), 256 blocks at B = 8192
    {128, 128, 2, 2, 3, 1, 0.62},  // 1
    {64, 128, 2, 2, 3, 1, 0.58},   // 2
    {128, 64, 2, 2, 3, 1, 0.58},   // 3
    {64, 64, 2, 2, 3, 2, 0.50},    // 4
    {128, 128, 2, 2, 2, 1, 0.55},  // 5
    {64, 160, 2, 2, 2, 1, 0.55},   // 6
    {64, 64, 2, 2, 2, 3, 0.45},    // 7
    // 8 waves (two per SIMD: one wave's LDS / barrier waits under the other's MFMAs)
    {64, 160, 4, 2, 3, 1, 0.70},   // 8
    {64, 160, 4, 2, 2, 1, 0.65},   // 9
    {128, 128, 4, 2, 3, 1, 0.70},  // 10
    {64, 128, 4, 2, 3, 1, 0.65},   // 11
    {128, 64, 4, 2, 3, 1, 0.65},   // 12
    {64, 64, 4, 2, 3, 2, 0.55},    // 13
    // deep rings: more bytes in flight per CU (the k loop waits on its DMA otherwise)
    {64, 64, 2, 2, 6, 1, 0.55},    // 14
    {64, 64, 4, 2, 6, 1, 0.60},    // 15
    {64, 128, 4, 2, 4, 1, 0.68},   // 16
    {128, 64, 4, 2, 4, 1, 0.68},   // 17
    {64, 64, 4, 2, 4, 1, 0.60},    // 18
    {64, 64, 4, 2, 2, 3, 0.55},    // 19: 8 waves, 3 blocks per CU
    // 64-deep stages (KS = 2): one barrier per two MFMA k-steps
    {64, 64, 2, 2, 3, 1, 0.60, 2},   // 20: 144 KB
    {64, 64, 4, 2, 2, 1, 0.60, 2},   // 21: 96 KB
    {128, 64, 4, 2, 2, 1, 0.65, 2},  // 22: 144 KB
    {64, 128, 4, 2, 2, 1, 0.65, 2},  // 23: 144 KB
    {64, 64, 2, 2, 2, 1, 0.55, 2},   // 24: 96 KB, 4 waves
    // whole-M weight-gradient tiles (dW = G^T X over the batch, split-K): the k-strided
    // X / H operand streams through ONCE (each of its column strips belongs to one block
    // per split) instead of once per 64-row M tile; the narrow G^T operand is the re-read
    // one (L2). RC images of 64 side by side.
    {320, 64, 4, 2, 2, 1, 0.60},   // 25: 144 KB (dW0: M = 300)
    {256, 64, 4, 2, 2, 1, 0.60},   // 26: 120 KB (dW1: M = 200)
    {192, 64, 4, 2, 2, 1, 0.60},   // 27: 96 KB
    {320, 64, 2, 2, 2, 1, 0.60},   // 28: 144 KB, 4 waves (TM 10)
    // taller forward tiles (fwd0: N = 300 in two 160 strips; with split-K 2 still 256
    // blocks): W0's strip is re-read by half as many blocks, 27 KB of fill per
    // 64 x 160 x 32 of work instead of 43
    {128, 160, 4, 2, 2, 1, 0.62},  // 29: 110 KB
    // one N tile for N <= 224 (fwd1: N = 200): the A operand (H1's planes) is read once
    // instead of once per 64-wide N tile; 16 x 112 per wave (TN = 7: the pipelined stage)
    {32, 224, 2, 2, 3, 1, 0.60},   // 30: 147 KB, 4 waves
    {64, 224, 4, 2, 2, 1, 0.60},   // 31: 110 KB, 8 waves
    // one wave per SIMD holding a 64 x 80 tile (TM 4, TN 5: 4.4x fewer LDS fragment bytes
    // per MFMA than 16 x 80), the pipelined stage hiding its own reads
    {128, 160, 2, 2, 2, 1, 0.60},  // 32: 110 KB, 4 waves
};
constexpr int kNumPl = sizeof(kPl) / sizeof(kPl[0]);

struct PlCfg {
  int tile, splits;
  int64_t kps;
  int xg = 1;  // XCD N-groups of a single-pass launch (planes_tile_index)
};

static bool pl_valid(int ti, bool a_rc, bool b_rc) {
  const PlDef& d = kPl[ti];
  return (!a_rc || d.bm == 128 || d.bm % 64 == 0) && (!b_rc || d.bn == 128 || d.bn % 64 == 0);
}

// a KS = 2 tiling needs every split's k range in whole 64-deep stages
static bool pl_ks_ok(const PlDef& d, int64_t Kp, int64_t kps) {
  return d.ks == 1 || (Kp % 64 == 0 && kps % 64 == 0);
}

// dX (dH1 . W0: M = B, N = 1664, K = 300) on the 4-wave 64 x 64 tiling, three blocks per CU:
// in the step it runs 64.3 us (median of 93 launches, rocprofv3) against 74.8 on the 8-wave
// tiling 19 that standalone timing had picked (70.7 vs 74.3 us alone), C3 12.51 / 12.49 /
// 12.81 vs 12.30 / 12.44 / 12.53 M ex/s alternating (profiles/r03_dx_tiling.txt)
#ifndef CTR_PL_DX_TILE
#define CTR_PL_DX_TILE 7  // (A/B builds: 19, the 8-wave 64 x 64 tiling)
#endif
// dX's XCD walk: whole M rows per XCD, N-tile-major inside the XCD (3, round 5): HBM traffic
// 160 -> 100 MB per launch at C3 (profiles/r05_gemm_mfma_busy.json vs
// r05_gemm_counters_dx_xg3.json), in-step C3 13.26 / 13.39 / 13.22 / 13.20 / 13.22 vs M-row-
// major (1) 13.21 / 13.21 / 13.26 / 13.24 / 13.42 M ex/s, alternating: the same time for 60 MB
// less traffic beside the scatter chain
#ifndef CTR_PL_DX_XG
#define CTR_PL_DX_XG 3
#endif
#ifndef CTR_PL_FWD0_TILE
#define CTR_PL_FWD0_TILE 8
#endif
static PlCfg pl_choose(bool a_rc, bool b_rc, int64_t M, int64_t N, int64_t Kp) {
  auto mk = [&](int ti, int s) {
    PlCfg c{ti, 1, Kp};
    if (s > 1) {
      c.kps = align_up(ceil_div(Kp, s), kPBK * kPl[ti].ks);
      c.splits = (int)ceil_div(Kp, c.kps);
    }
    return c;
  };
  // per-shape override for in-step A/B (tuning only): CTR_GEMM_PLANES_SHAPE_CFG =
  // "M,N,Kp,a_rc,b_rc=tile,splits,xg;..." (Kp: the 32-padded k extent)
  if (const char* env = getenv("CTR_GEMM_PLANES_SHAPE_CFG")) {
    const char* q = env;
    while (q && *q) {
      long long m, n, k;
      int ar, br, ti = -1, sp = 1, xg = 1, used = 0;
      if (sscanf(q, "%lld,%lld,%lld,%d,%d=%d,%d,%d%n", &m, &n, &k, &ar, &br, &ti, &sp, &xg,
                 &used) >= 8 && m == M && n == N && k == Kp && ar == (int)a_rc &&
          br == (int)b_rc && ti >= 0 && ti < kNumPl && sp >= 1 && pl_valid(ti, a_rc, b_rc)) {
        PlCfg c = mk(ti, sp);
        c.xg = xg == 2 || xg == 3 || xg == 4 || xg == 8 ? xg : 1;
        if (pl_ks_ok(kPl[ti], Kp, c.kps)) return c;
      }
      q = strchr(q, ';');
      if (q) ++q;
    }
  }
  if (const char* env = getenv("CTR_GEMM_PLANES_CFG")) {
    int ti = -1, sp = 1, xg = 1;
    if (sscanf(env, "%d,%d,%d", &ti, &sp, &xg) >= 1 && ti >= 0 && ti < kNumPl && sp >= 1 &&
        pl_valid(ti, a_rc, b_rc)) {
      PlCfg c = mk(ti, sp);
      c.xg = xg == 2 || xg == 3 || xg == 4 || xg == 8 ? xg : 1;
      if (pl_ks_ok(kPl[ti], Kp, c.kps)) return c;
    }
  }
  // measured on MI355X (tools/gemm_planes_bench.py --sweep, profiles/r02_gemm_planes_sweep.jsonl;
  // fwd1 (N = 200) 14.6 us on 17 vs 16.2 on 8, dX (N = 1664) 70.7 on 19 vs 74.3 on 7):
  // large-M products with a narrow N (the forward) on the 8-wave 64x160 tiling, large-M
  // products with a k-strided B (the dH1 / dX backward) on 64x64 x3 blocks per CU, the
  // transposed weight gradients (both operands k-strided, long K) on 64x64 with split-K
  // sized to ~2 blocks per CU
  // fwd0 (N = 300) on the 64 x 160 tiling (8): a direct-to-register A variant (round 3,
  // removed) was faster standalone (59.1 vs 65.2 us, profiles/r03_gemm_direct_a.txt) but not
  // in the step, where it read the X planes 4 times instead of 2
  if (!a_rc && !b_rc && M >= 2048 && N > 256 && N <= 320) return mk(CTR_PL_FWD0_TILE, 1);
  // round 5 (tools/gemm_planes_bench.py --pg --sweep, gpurun_out/r05_pg_sweep.jsonl; the C4
  // policy MLP at an episode of 4096): longer-k products on the 64-deep-stage tilings —
  // N <= 256 with K >= 512 (4096 x 256 x 512: tile 21 11.9 us vs 17.3 on 17), 320 < N <= 768
  // with K >= 1024 (4096 x 512 x 1024: tile 22 30.7 vs 35.0 on 16) — and a k-strided B with
  // K >= 512 on 128 x 128 tiles (4096 x 1024 x 512: tile 10 31.2 vs 33.6 on 7). The C3 shapes
  // (K 300 / 320) keep their in-step-measured tilings. CTR_PL_RULES_R05=0: the round-4 rules.
  static const bool r05 = [] {
    const char* e = getenv("CTR_PL_RULES_R05");
    return !(e && e[0] == '0');
  }();
  if (r05 && !a_rc && !b_rc && M >= 2048 && N <= 256 && Kp >= 512 && Kp % 64 == 0)
    return mk(21, 1);
  if (r05 && !a_rc && !b_rc && M >= 2048 && N > 320 && N <= 768 && Kp >= 1024 && Kp % 64 == 0)
    return mk(22, 1);
  if (r05 && !a_rc && b_rc && M >= 2048 && N >= 1024 && N <= 1024 + 64 && Kp >= 512)
    return mk(10, 1);
  if (!a_rc && !b_rc && M >= 2048 && N <= 256) return mk(17, 1);
  if (!a_rc && b_rc && M >= 2048 && N >= 1024) {
    PlCfg c = mk(CTR_PL_DX_TILE, 1);
    // XCD tile groups (planes_tile_index): with the 4-wave tiling, whole M rows per XCD (1)
    // measured C3 13.05 / 13.02 / 13.04 vs 12.93 / 12.70 / 12.93 M ex/s with halves of the
    // N tiles per XCD (2), 4 no better (alternating, per-shape override); walked N-major
    // inside the XCD (3) the same time with 60 MB less HBM traffic (round 5, above)
    c.xg = CTR_PL_DX_XG;
    return c;
  }
  if (!a_rc && b_rc && M >= 2048) return mk(7, 1);
  if (a_rc && b_rc && Kp >= 2048 && M > 128 && M <= 320 && N >= 768) {
    // whole-M tile (the wide operand read once), split-K to about one block per CU.
    // Standalone (operands MALL-warm) it is no faster than 64x64 tiles (dW0 71 vs 66 us
    // with the compiler's transpose reads); in the step, where dW0 runs beside the scatter
    // chain and the two compete for HBM, reading X's planes once instead of once per
    // 64-row M tile measured C3 11.94 -> 12.32 M ex/s (12.48 -> 12.75 with plan lookahead;
    // two alternating runs each). Not for narrower N: the policy net's 256 x 512 weight
    // gradient (C4) measured 8.49 wide vs 8.72 M transitions/s on the 64x64 tiles.
    const int ti = M <= 192 ? 27 : M <= 256 ? 26 : 25;
    const int64_t tiles = ceil_div(N, 64);
    const int s = (int)std::max<int64_t>(1, std::min<int64_t>(std::min<int64_t>(256 / tiles, Kp / 256), 64));
    return mk(ti, s);
  }
  if (a_rc && b_rc && Kp >= 2048) {
    // target block count of the weight-gradient GEMMs: ~1170 (4.5 per CU) with the
    // split-major XCD map — measured dW0 (130 tiles) 9 splits 66 us vs 4 splits 73, dW1
    // (20 tiles) 24-32 splits 22.5-23 us vs 16 24
    // round 5: at K <= 4096 (the C4 policy weight gradients) ~600 blocks, 2-3 per CU — dW1
    // (128 tiles) 4 splits 35.5 us vs 10 41.6, dW0 (192 tiles) 4 splits 47.1 vs 7 53.9
    const int64_t wg_blocks = (r05 && Kp <= 4096) ? 600 : 1170;
    const int64_t tiles = ceil_div(M, 64) * ceil_div(N, 64);
    const int s = (int)std::max<int64_t>(1, std::min<int64_t>(std::min<int64_t>(
                      ceil_div(wg_blocks, tiles), Kp / 256), 64));
    return mk(7, s);
  }
  // otherwise a makespan model: blocks dealt to 256 CUs x occ slots in rounds; a round costs one block's
  // padded bf16 MFMA work (6 products) at the tiling's sustained per-CU rate, plus fill and
  // drain; split-K adds its fp32 slab round trip and the reduce launch
  const double per_cu = 2.5e15 / 256.0 / 1e6;  // bf16 flop per us per CU
  PlCfg best = mk(0, 1);
  double best_t = 1e30;
  for (int ti = 0; ti < kNumPl; ++ti) {
    // the model: KS = 1 only, the round-2 tilings (later ones by measured rules only)
    if (!pl_valid(ti, a_rc, b_rc) || kPl[ti].ks != 1 || ti >= 29) continue;
    const PlDef& d = kPl[ti];
    const int64_t tiles = ceil_div(M, d.bm) * ceil_div(N, d.bn);
    for (int s = 1; s <= 32; ++s) {
      if (s > 1 && Kp / s < 128) break;
      const PlCfg c = mk(ti, s);
      if (c.splits != s) continue;
      const int64_t blocks = tiles * c.splits;
      const double rounds = (double)ceil_div(blocks, 256 * (int64_t)d.occ);
      const int64_t per_cu_blocks = std::min<int64_t>(d.occ, ceil_div(blocks, 256));
      const double t_block =
          6.0 * 2.0 * d.bm * d.bn * (double)c.kps * per_cu_blocks / (per_cu * d.eff) + 2.5;
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

// every (tiling, orientation) pair is instantiated explicitly (RC operands only on 64- or
// 128-wide tiles; pl_valid keeps the chooser inside this list)
#define CTR_PL_K(BM, BN, WMW, WNW, NS, AR, BR, KS)                                        \
  hipLaunchKernelGGL((gemm_planes_kernel<BM, BN, WMW, WNW, AR, BR, NS, KS>), grid,             \
                     64 * WMW * WNW, 0, st, a)
#define CTR_PL_ALL4K(BM, BN, WMW, WNW, NS, KS)                          \
  if (!a_rc && !b_rc) CTR_PL_K(BM, BN, WMW, WNW, NS, false, false, KS); \
  else if (!a_rc) CTR_PL_K(BM, BN, WMW, WNW, NS, false, true, KS);      \
  else if (!b_rc) CTR_PL_K(BM, BN, WMW, WNW, NS, true, false, KS);      \
  else CTR_PL_K(BM, BN, WMW, WNW, NS, true, true, KS);
#define CTR_PL_ALL4(BM, BN, WMW, WNW, NS) CTR_PL_ALL4K(BM, BN, WMW, WNW, NS, 1)
#define CTR_PL_AONLY(BM, BN, WMW, WNW, NS)                          \
  if (!a_rc) CTR_PL_K(BM, BN, WMW, WNW, NS, false, false, 1);       \
  else CTR_PL_K(BM, BN, WMW, WNW, NS, true, false, 1);

static void pl_launch(const PlCfg& c, const PlanesArgs& a, bool a_rc, bool b_rc, dim3 grid,
                      hipStream_t st) {
  switch (c.tile) {
    case 0: CTR_PL_AONLY(64, 160, 2, 2, 3) break;
    case 1: CTR_PL_ALL4(128, 128, 2, 2, 3) break;
    case 2: CTR_PL_ALL4(64, 128, 2, 2, 3) break;
    case 3: CTR_PL_ALL4(128, 64, 2, 2, 3) break;
    case 4: CTR_PL_ALL4(64, 64, 2, 2, 3) break;
    case 5: CTR_PL_ALL4(128, 128, 2, 2, 2) break;
    case 6: CTR_PL_AONLY(64, 160, 2, 2, 2) break;
    case 7: CTR_PL_ALL4(64, 64, 2, 2, 2) break;
    case 8: CTR_PL_AONLY(64, 160, 4, 2, 3) break;
    case 9: CTR_PL_AONLY(64, 160, 4, 2, 2) break;
    case 10: CTR_PL_ALL4(128, 128, 4, 2, 3) break;
    case 11: CTR_PL_ALL4(64, 128, 4, 2, 3) break;
    case 12: CTR_PL_ALL4(128, 64, 4, 2, 3) break;
    case 13: CTR_PL_ALL4(64, 64, 4, 2, 3) break;
    case 14: CTR_PL_ALL4(64, 64, 2, 2, 6) break;
    case 15: CTR_PL_ALL4(64, 64, 4, 2, 6) break;
    case 16: CTR_PL_ALL4(64, 128, 4, 2, 4) break;
    case 17: CTR_PL_ALL4(128, 64, 4, 2, 4) break;
    case 18: CTR_PL_ALL4(64, 64, 4, 2, 4) break;
    case 19: CTR_PL_ALL4(64, 64, 4, 2, 2) break;
    case 20: CTR_PL_ALL4K(64, 64, 2, 2, 3, 2) break;
    case 21: CTR_PL_ALL4K(64, 64, 4, 2, 2, 2) break;
    case 22: CTR_PL_ALL4K(128, 64, 4, 2, 2, 2) break;
    case 23: CTR_PL_ALL4K(64, 128, 4, 2, 2, 2) break;
    case 24: CTR_PL_ALL4K(64, 64, 2, 2, 2, 2) break;
    case 25: CTR_PL_ALL4(320, 64, 4, 2, 2) break;
    case 26: CTR_PL_ALL4(256, 64, 4, 2, 2) break;
    case 27: CTR_PL_ALL4(192, 64, 4, 2, 2) break;
    case 28: CTR_PL_ALL4(320, 64, 2, 2, 2) break;
    case 29: CTR_PL_AONLY(128, 160, 4, 2, 2) break;
    case 30: if (!a_rc && !b_rc) CTR_PL_K(32, 224, 2, 2, 3, false, false, 1); break;
    case 31: CTR_PL_AONLY(64, 224, 4, 2, 2) break;
    case 32: CTR_PL_AONLY(128, 160, 2, 2, 2) break;
  }
}
#undef CTR_PL_AONLY
#undef CTR_PL_ALL4
#undef CTR_PL_ALL4K
#undef CTR_PL_K

static int64_t pl_ws_bytes(const PlCfg& c, int64_t M, int64_t N) {
  return c.splits > 1 ? (int64_t)c.splits * M * align_up(N, 4) * 4 : 0;
}

}  // namespace ctr

using namespace ctr;

static bool plane_src_ok(const ctr_planes* p) {
  return p && p->data && p->ld > 0 && p->ld % 8 == 0 && p->plane_stride % 8 == 0 &&
         p->rows > 0 && p->cols > 0 && p->cols <= p->ld &&
         p->plane_stride >= p->rows * p->ld && (uintptr_t)p->data % 16 == 0;
}

extern "C" int ctr_split_planes(const float* src, int64_t rows, int64_t cols, int64_t ld,
                                const ctr_planes* dst, ctr_stream_t stream) {
  CTR_REQUIRE(rows >= 0 && cols >= 0, "ctr_split_planes: bad sizes");
  if (rows == 0 || cols == 0) return CTR_OK;
  CTR_REQUIRE(src && plane_src_ok(dst), "ctr_split_planes: bad pointers / plane layout");
  CTR_REQUIRE(ld >= cols && dst->rows >= rows && dst->cols >= cols,
              "ctr_split_planes: destination smaller than the source");
  const bool vec = ld % 4 == 0 && (uintptr_t)src % 16 == 0;
  const int64_t total = rows * ceil_div(cols, 4);
  const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>(ceil_div(total, 256), 8192));
  hipLaunchKernelGGL(split_planes_kernel, grid, 256, 0, as_stream(stream), src, rows, cols, ld,
                     static_cast<uint16_t*>(dst->data), dst->ld, dst->plane_stride, vec);
  CTR_LAUNCH_CHECK("split_planes_kernel");
  return CTR_OK;
}

extern "C" int64_t ctr_gemm_planes_workspace_bytes(int a_rc, int b_rc, int64_t M, int64_t N,
                                                   int64_t K) {
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  const PlCfg c = pl_choose(a_rc != 0, b_rc != 0, M, N, align_up(K, kPBK));
  return pl_ws_bytes(c, M, N);
}

extern "C" int ctr_gemm_planes_lastcol(int a_rc, int b_rc, int64_t M, int64_t N, int64_t K,
                                       const ctr_planes* A, const ctr_planes* B, float* C,
                                       int64_t ldc, const ctr_planes* Cp, int epi,
                                       const float* bias, const float* aux, int64_t ldaux,
                                       float scale, float drop_p, uint64_t seed, uint64_t offset,
                                       const int32_t* step_ptr, float* last_col, void* ws,
                                       int64_t ws_bytes, ctr_stream_t stream) {
  CTR_REQUIRE(M >= 0 && N >= 0 && K >= 0, "ctr_gemm_planes: negative size");
  if (M == 0 || N == 0) return CTR_OK;
  CTR_REQUIRE(C || Cp, "ctr_gemm_planes: no output");
  CTR_REQUIRE(!last_col || (C && !Cp && N >= 2),
              "ctr_gemm_planes: last_col needs an fp32 output C of N-1 >= 1 columns, no planes");
  CTR_REQUIRE(plane_src_ok(A) && plane_src_ok(B), "ctr_gemm_planes: bad operand plane layout");
  CTR_REQUIRE(!Cp || (plane_src_ok(Cp) && Cp->rows >= M && Cp->cols >= N),
              "ctr_gemm_planes: bad output plane layout");
  CTR_REQUIRE(!C || ldc >= (last_col ? N - 1 : N), "ctr_gemm_planes: ldc < N");
  const int64_t Kp = align_up(std::max<int64_t>(K, 1), kPBK);
  // KC operand: storage [rows >= extent][cols >= Kp]; RC: storage [rows >= Kp][cols >= extent]
  CTR_REQUIRE(a_rc ? (A->rows >= Kp && A->cols >= M && A->cols % 16 == 0)
                   : (A->rows >= M && A->cols >= Kp),
              "ctr_gemm_planes: A planes must cover the (32-padded) operand, zero-padded");
  CTR_REQUIRE(b_rc ? (B->rows >= Kp && B->cols >= N && B->cols % 16 == 0)
                   : (B->rows >= N && B->cols >= Kp),
              "ctr_gemm_planes: B planes must cover the (32-padded) operand, zero-padded");
  CTR_REQUIRE(epi != CTR_EPI_BIAS_RELU_DROP || (drop_p >= 0.f && drop_p < 1.f),
              "ctr_gemm_planes: drop_p out of range");
  CTR_REQUIRE(epi != CTR_EPI_GRAD_MASK || aux, "ctr_gemm_planes: GRAD_MASK needs aux");
  CTR_REQUIRE((epi != CTR_EPI_BIAS && epi != CTR_EPI_BIAS_RELU && epi != CTR_EPI_BIAS_RELU_DROP) || bias,
              "ctr_gemm_planes: bias epilogue without bias");
  const bool arc = a_rc != 0, brc = b_rc != 0;
  const PlCfg c = pl_choose(arc, brc, M, N, Kp);
  const PlDef& d = kPl[c.tile];
  const int64_t need = pl_ws_bytes(c, M, N);
  CTR_REQUIRE(ws_bytes >= need && (need == 0 || ws), "ctr_gemm_planes: workspace too small");

  PlanesArgs a{};
  a.Kp = Kp;
  a.k_per_split = c.kps;
  auto src = [](const ctr_planes* p) {
    return PlaneSrc{static_cast<const uint16_t*>(p->data), p->ld, p->plane_stride, p->rows, p->cols};
  };
  a.A = src(A);
  a.B = src(B);
  GemmArgs& g = a.g;
  g.M = M;
  g.N = N;
  g.K = K;
  g.C = C;
  g.ldc = ldc;
  g.epi = epi;
  g.bias = bias;
  g.aux = aux;
  g.ldaux = ldaux;
  g.scale = scale;
  g.drop_thr = epi == CTR_EPI_BIAS_RELU_DROP
                   ? (uint32_t)std::min<double>((double)drop_p * 4294967296.0, 4294967295.0)
                   : 0u;
  g.drop_scale = epi == CTR_EPI_BIAS_RELU_DROP ? 1.0f / (1.0f - drop_p) : 1.0f;
  g.seed = seed;
  g.offset = offset;
  g.step_ptr = step_ptr;
  g.vec_c = C && ldc % 4 == 0 && (uintptr_t)C % 16 == 0;
  if (Cp) {
    a.cpl = static_cast<uint16_t*>(Cp->data);
    a.cpl_ld = Cp->ld;
    a.cpl_ps = Cp->plane_stride;
  }
  a.last_col = last_col;
  if (last_col) g.vec_c = g.vec_c && (N - 1) % 4 == 0;
  hipStream_t st = as_stream(stream);
  const int64_t tiles = ceil_div(M, d.bm) * ceil_div(N, d.bn);
  CTR_REQUIRE(tiles * c.splits + 8 <= INT32_MAX, "ctr_gemm_planes: grid too large");
  a.xcd_ngroups = c.xg;
  a.splits = c.splits;
  a.tiles = tiles;
  // split-K: every (tile, split) pair in blockIdx.x, padded to a multiple of 8
  const dim3 grid((unsigned)(c.splits > 1 ? align_up(tiles * c.splits, 8) : tiles), 1, 1);
  if (c.splits > 1) {
    PlanesArgs s = a;
    const int64_t sld = align_up(N, 4);
    s.g.C = static_cast<float*>(ws);
    s.g.ldc = sld;
    s.g.slab_stride = M * sld;
    s.g.vec_c = (uintptr_t)ws % 16 == 0;
    s.cpl = nullptr;
    s.last_col = nullptr;
    pl_launch(c, s, arc, brc, grid, st);
    CTR_LAUNCH_CHECK("gemm_planes_kernel (split-K)");
    const int64_t total = M * ceil_div(N, 4);
    const unsigned g2 = (unsigned)std::min<int64_t>(ceil_div(total, 64), 16384);
    hipLaunchKernelGGL(planes_reduce_kernel, g2, 64, 0, st, a, static_cast<const float*>(ws),
                       c.splits, sld);
    CTR_LAUNCH_CHECK("planes_reduce_kernel");
    return CTR_OK;
  }
  pl_launch(c, a, arc, brc, grid, st);
  CTR_LAUNCH_CHECK("gemm_planes_kernel");
  return CTR_OK;
}

extern "C" int ctr_gemm_planes(int a_rc, int b_rc, int64_t M, int64_t N, int64_t K,
                               const ctr_planes* A, const ctr_planes* B, float* C, int64_t ldc,
                               const ctr_planes* Cp, int epi, const float* bias, const float* aux,
                               int64_t ldaux, float scale, float drop_p, uint64_t seed,
                               uint64_t offset, const int32_t* step_ptr, void* ws,
                               int64_t ws_bytes, ctr_stream_t stream) {
  return ctr_gemm_planes_lastcol(a_rc, b_rc, M, N, K, A, B, C, ldc, Cp, epi, bias, aux, ldaux,
                                 scale, drop_p, seed, offset, step_ptr, nullptr, ws, ws_bytes,
                                 stream);
}

extern "C" int ctr_gemm_planes_config(int a_rc, int b_rc, int64_t M, int64_t N, int64_t K,
                                      int* tile, int* splits, int* bm, int* bn) {
  const PlCfg c = pl_choose(a_rc != 0, b_rc != 0, M, N, align_up(std::max<int64_t>(K, 1), kPBK));
  if (tile) *tile = c.tile;
  if (splits) *splits = c.splits;
  if (bm) *bm = kPl[c.tile].bm;
  if (bn) *bn = kPl[c.tile].bn;
  return CTR_OK;
}

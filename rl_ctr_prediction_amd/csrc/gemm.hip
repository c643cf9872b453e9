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

#include "gemm_common.h"

namespace ctr {

// ------------------------------------------------------------------- the kernel ------
// Block = WAVES_M x WAVES_N x KSPLIT waves (4: one per SIMD), tile BM x BN x BK=32; a wave
// owns a WM x WN = (BM/WAVES_M) x (BN/WAVES_N) sub-tile of TM x TN 32x32 accumulators over
// 1/KSPLIT of every k-tile (the KSPLIT partial tiles are added in wave order through LDS
// at the end: deterministic). Tiles are sized per GEMM shape so that the grid is about one
// round of the 256 CUs (choose_tiles): e.g. 64x160 (k-split 2) for the 8192x300 forward,
// 128x416 for the 8192x1664 input gradient, 160x128 (split-K) for the 300x1664 weight
// gradient — tile quantisation was what 64/128-only tilings lost on these shapes.
//
// LDS images (unpadded, so LDS-DMA can fill them lane-linearly), per operand:
//  - k-contiguous in memory (A [M][K], nn.Linear weights [N][K]): [rows][32] with the 16-B
//    chunk c of row r stored at chunk c ^ ((r >> 1) & 7); a lane reads its row's 4
//    consecutive k with one conflict-free ds_read_b128 and feeds 4 MFMA k-steps. The MFMA's
//    k order inside each 8-wide group is permuted (step j, lane half h -> k = 8g + 4h + j)
//    identically for A and B, so every product A[m,k]B[k,n] is formed once; only the
//    accumulation order differs from plain k order.
//  - rows-contiguous (A^T, B [K][N]): [32][rows]; ds_read_b32 per k-step at the permuted k
//    (32 consecutive rows per half-wave: conflict-free).
// Staging (VEC = 16-B aligned operands whose contiguous extents are multiples of 4):
// global_load_lds_dwordx4 into a STAGES-deep LDS ring (the swizzle is applied to the
// per-lane SOURCE address), counted s_waitcnt vmcnt + raw s_barrier, so STAGES-1 k-tiles
// are in flight while one is multiplied; otherwise a register-staged path with the same
// images. Rows beyond M/N read row 0 (never stored); the K tail of the last k-tile is
// zeroed in LDS before use.
typedef __attribute__((address_space(3))) void* lds_void_ptr;

#ifndef CTR_GEMM_TRACE
#define CTR_GEMM_TRACE 0
#endif
#if CTR_GEMM_TRACE
// tuning builds only: per block [realtime start, memtime start, memtime after the k-loop,
// memtime end, xcc<<8 | se<<4 | cu]
__device__ unsigned long long g_gemm_trace[16384 * 5];
#endif

// global_load_lds_dwordx4 in inline asm: hipcc (ROCm 7.2) treats the builtin's LDS write
// as aliasing every later ds_read and puts an s_waitcnt vmcnt(0) before the first fragment
// read of each k-tile, draining the ring; hidden from its waitcnt model, the ring is
// retired only by the counted waits below. `lds` is the wave-uniform LDS byte address.
__device__ __forceinline__ void glds16(const float* gsrc, uint32_t lds) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(lds)
      : "memory");
}

__device__ __forceinline__ uint32_t lds_addr(const float* p) {
  return (uint32_t)(uintptr_t)(lds_void_ptr)p;
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ void block_barrier_lds() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// 16-B chunk swizzle of a k-contiguous image row (BK/4 chunks): conflict-free ds_read_b128
// of one logical chunk by 32 consecutive rows (the 4x16-lane groups of gfx950's b128 read).
template <int BK>
__device__ __forceinline__ int kc_swz(int r) {
  return BK == 32 ? ((r >> 1) & 7) : (r & 15);
}

template <int BM, int BN, int BK, int WAVES_M, int WAVES_N, int KSPLIT, int STAGES, bool TA,
          bool TB, bool VEC>
__global__ __launch_bounds__(WAVES_M* WAVES_N* KSPLIT * 64) void gemm_f32_kernel(GemmArgs a) {
  static_assert(BK == 32 || BK == 64, "k-tile of 32 or 64");
  constexpr int CPR = BK / 4;     // 16-B chunks per k-contiguous image row
  constexpr int RPP = 256 / BK;   // image rows per 1-KB DMA piece
  constexpr int NW = WAVES_M * WAVES_N * KSPLIT;
  constexpr int NT = NW * 64;
  constexpr int WM = BM / WAVES_M, WN = BN / WAVES_N;
  constexpr int TM = WM / 32, TN = WN / 32;
  constexpr bool A_KC = !TA, B_KC = TB;
  constexpr int A_IMG = BM * BK, B_IMG = BN * BK;
  constexpr int STAGE = A_IMG + B_IMG;
  constexpr int NS = VEC ? STAGES : 2;  // LDS stages
  constexpr int IA = A_IMG / 256 / NW, IB = B_IMG / 256 / NW;  // DMA instr per wave per tile
  constexpr int G = IA + IB;
  constexpr int NA = A_IMG / 4 / NT, NB = B_IMG / 4 / NT;  // register path: float4 per thread
  constexpr int GPW = (BK / 8) / KSPLIT;                   // 8-k groups per wave per k-tile
  static_assert(WM % 32 == 0 && WN % 32 == 0, "wave tile in 32x32 MFMA blocks");
  static_assert(IA * NW * 256 == A_IMG && IB * NW * 256 == B_IMG, "DMA pieces split evenly");
  static_assert(NA * NT * 4 == A_IMG && NB * NT * 4 == B_IMG, "loads split evenly");
  static_assert(GPW * KSPLIT == BK / 8, "k-split divides the 8-k groups of a k-tile");
  static_assert(G <= 63, "vmcnt range");
  static_assert((KSPLIT - 1) * WAVES_M * WAVES_N * WM * WN <= NS * STAGE, "k-split partials fit");
  static_assert(NW * 32 * 36 <= NS * STAGE, "epilogue tiles fit");
  __shared__ __attribute__((aligned(16))) float smem[NS * STAGE];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
#if CTR_GEMM_TRACE
  const unsigned long long tr_rt = wall_clock64(), tr_t0 = clock64();
  const int tr_b = blockIdx.x + gridDim.x * blockIdx.z;
#endif
  const int kw = wave / (WAVES_M * WAVES_N);
  const int wmn = wave % (WAVES_M * WAVES_N);
  const int wm0 = (wmn / WAVES_N) * WM;
  const int wn0 = (wmn % WAVES_N) * WN;
  const int h = lane >> 5, il = lane & 31;

  // tile of this block: tiles sharing A rows are consecutive, and consecutive tiles are
  // kept on one XCD (blocks b, b+8, b+16... share an XCD under round-robin dispatch)
  const int64_t gn = (a.N + BN - 1) / BN;
  const int64_t tix = xcd_tile_index();
  const int64_t m0 = (tix / gn) * BM;
  const int64_t n0 = (tix % gn) * BN;
  const int64_t kb = (int64_t)blockIdx.z * a.k_per_split;
  const int64_t ke = min(a.K, kb + a.k_per_split);
  const int nt = kb < ke ? (int)((ke - kb + BK - 1) / BK) : 0;

  // ---- fragments of one 8-k group: [operand tile][k-step] ---------------------------
  auto read_frags = [&](float (&af)[TM][4], float (&bf)[TN][4], const float* as, const float* bs,
                        int g) {
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int r = wm0 + i * 32 + il;
      if (A_KC) {
        const float4 v = *reinterpret_cast<const float4*>(
            as + r * BK + 4 * ((2 * g + h) ^ kc_swz<BK>(r)));
        af[i][0] = v.x; af[i][1] = v.y; af[i][2] = v.z; af[i][3] = v.w;
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) af[i][j] = as[(8 * g + 4 * h + j) * BM + r];
      }
    }
#pragma unroll
    for (int t = 0; t < TN; ++t) {
      const int r = wn0 + t * 32 + il;
      if (B_KC) {
        const float4 v = *reinterpret_cast<const float4*>(
            bs + r * BK + 4 * ((2 * g + h) ^ kc_swz<BK>(r)));
        bf[t][0] = v.x; bf[t][1] = v.y; bf[t][2] = v.z; bf[t][3] = v.w;
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) bf[t][j] = bs[(8 * g + 4 * h + j) * BN + r];
      }
    }
  };

  floatx16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // one k-tile: MFMAs over one LDS stage, fragments read one 8-k group ahead
  auto compute_tile = [&](const float* as) {
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
  };

  // zero the LDS image positions of k >= ke (last k-tile of a split only)
  auto zero_k_tail = [&](float* as, int64_t k0) {
    const int kv = (int)(ke - k0);  // valid k in this tile (< BK)
    float* bs = as + A_IMG;
    if (A_KC) {
      for (int q = tid; q < BM * CPR; q += NT) {
        const int r = q / CPR, c = q % CPR;
        if (4 * c >= kv)
          *reinterpret_cast<float4*>(as + r * BK + 4 * (c ^ kc_swz<BK>(r))) =
              make_float4(0.f, 0.f, 0.f, 0.f);
      }
    } else {
      for (int q = tid + kv * BM; q < BK * BM; q += NT) as[q] = 0.f;
    }
    if (B_KC) {
      for (int q = tid; q < BN * CPR; q += NT) {
        const int r = q / CPR, c = q % CPR;
        if (4 * c >= kv)
          *reinterpret_cast<float4*>(bs + r * BK + 4 * (c ^ kc_swz<BK>(r))) =
              make_float4(0.f, 0.f, 0.f, 0.f);
      }
    } else {
      for (int q = tid + kv * BN; q < BK * BN; q += NT) bs[q] = 0.f;
    }
  };

  if (VEC) {
    // ---- LDS-DMA ring ----------------------------------------------------------------
    // DMA piece q of an image = 256 consecutive floats of it; wave w issues pieces
    // w*I .. w*I+I-1. Per lane: the source of its 16 B in piece q at k-tile 0.
    const float* srcA[IA];
    const float* srcB[IB];
#pragma unroll
    for (int j = 0; j < IA; ++j) {
      const int q = wave * IA + j;
      if (A_KC) {  // piece = RPP rows x CPR chunks; lane -> (row, stored chunk)
        const int r = RPP * q + lane / CPR, p = lane % CPR;
        const int c = p ^ kc_swz<BK>(r);
        const int64_t gm = m0 + r;
        srcA[j] = a.A + (gm < a.M ? gm : 0) * a.lda + kb + 4 * c;
      } else {  // piece = floats [256q, 256q+256) of [32][BM]
        const int idx = 256 * q + 4 * lane;
        const int k = idx / BM, r = idx % BM;
        const int64_t gm = m0 + r;
        srcA[j] = a.A + (kb + k) * a.lda + (gm < a.M ? gm : 0);
      }
    }
#pragma unroll
    for (int j = 0; j < IB; ++j) {
      const int q = wave * IB + j;
      if (B_KC) {
        const int r = RPP * q + lane / CPR, p = lane % CPR;
        const int c = p ^ kc_swz<BK>(r);
        const int64_t gnn = n0 + r;
        srcB[j] = a.B + (gnn < a.N ? gnn : 0) * a.ldb + kb + 4 * c;
      } else {
        const int idx = 256 * q + 4 * lane;
        const int k = idx / BN, r = idx % BN;
        const int64_t gnn = n0 + r;
        srcB[j] = a.B + (kb + k) * a.ldb + (gnn < a.N ? gnn : 0);
      }
    }
    const int64_t stepA = A_KC ? BK : BK * a.lda;
    const int64_t stepB = B_KC ? BK : BK * a.ldb;
    // k of each lane's float4 inside the tile (for the K tail: never read past K)
    int kA[IA], kB[IB];
#pragma unroll
    for (int j = 0; j < IA; ++j) {
      const int q = wave * IA + j;
      kA[j] = A_KC ? 4 * ((lane % CPR) ^ kc_swz<BK>(RPP * q + lane / CPR)) : (256 * q + 4 * lane) / BM;
    }
#pragma unroll
    for (int j = 0; j < IB; ++j) {
      const int q = wave * IB + j;
      kB[j] = B_KC ? 4 * ((lane % CPR) ^ kc_swz<BK>(RPP * q + lane / CPR)) : (256 * q + 4 * lane) / BN;
    }
    auto issue = [&](int t) {
      const float* st = smem + (t % NS) * STAGE;
      const int64_t k0 = kb + (int64_t)t * BK;
      const bool tail = k0 + BK > ke;
#pragma unroll
      for (int j = 0; j < IA; ++j) {
        const float* src = srcA[j] + t * stepA;
        if (tail && !(k0 + kA[j] < ke)) src = srcA[j];  // in-bounds; zeroed before use
        glds16(src, __builtin_amdgcn_readfirstlane(lds_addr(st + (wave * IA + j) * 256)));
      }
#pragma unroll
      for (int j = 0; j < IB; ++j) {
        const float* src = srcB[j] + t * stepB;
        if (tail && !(k0 + kB[j] < ke)) src = srcB[j];
        glds16(src, __builtin_amdgcn_readfirstlane(lds_addr(st + A_IMG + (wave * IB + j) * 256)));
      }
    };
    // prologue: NS-1 tiles in flight
#pragma unroll
    for (int s = 0; s < NS - 1; ++s)
      if (s < nt) issue(s);
    for (int t = 0; t < nt; ++t) {
      // this wave's pieces of k-tile t have landed when at most the later tiles' are pending
      if (NS == 3 && t + 1 < nt) wait_vmcnt<G>();
      else wait_vmcnt<0>();
      block_barrier_lds();  // every wave's pieces landed; stage (t-1)%NS no longer read
      float* st = smem + (t % NS) * STAGE;
      if (kb + (int64_t)(t + 1) * BK > ke) {
        zero_k_tail(st, kb + (int64_t)t * BK);
        block_barrier_lds();
      }
      if (t + NS - 1 < nt) issue(t + NS - 1);
      compute_tile(st);
    }
  } else {
    // ---- register staging (unaligned / odd extents) ------------------------------------
    float4 ra[NA], rb[NB];
    auto load_tile = [&](int t) {
      const int64_t k0 = kb + (int64_t)t * BK;
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        const int q = tid + NT * i;
        float4 v;
        if (A_KC) {
          const int r = q / CPR, c = q % CPR;
          const int64_t gm = m0 + r;
          const float* p = a.A + (gm < a.M ? gm : 0) * a.lda + k0 + 4 * c;
          const int64_t k = k0 + 4 * c;
          v.x = (k + 0 < ke) ? p[0] : 0.f;
          v.y = (k + 1 < ke) ? p[1] : 0.f;
          v.z = (k + 2 < ke) ? p[2] : 0.f;
          v.w = (k + 3 < ke) ? p[3] : 0.f;
        } else {
          const int k = q / (BM / 4), r = 4 * (q % (BM / 4));
          const int64_t gm = m0 + r;
          const bool okk = k0 + k < ke;
          const float* p = a.A + (okk ? k0 + k : kb) * a.lda + gm;
          v.x = (okk && gm + 0 < a.M) ? p[0] : 0.f;
          v.y = (okk && gm + 1 < a.M) ? p[1] : 0.f;
          v.z = (okk && gm + 2 < a.M) ? p[2] : 0.f;
          v.w = (okk && gm + 3 < a.M) ? p[3] : 0.f;
        }
        ra[i] = v;
      }
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        const int q = tid + NT * i;
        float4 v;
        if (B_KC) {
          const int r = q / CPR, c = q % CPR;
          const int64_t gnn = n0 + r;
          const float* p = a.B + (gnn < a.N ? gnn : 0) * a.ldb + k0 + 4 * c;
          const int64_t k = k0 + 4 * c;
          v.x = (k + 0 < ke) ? p[0] : 0.f;
          v.y = (k + 1 < ke) ? p[1] : 0.f;
          v.z = (k + 2 < ke) ? p[2] : 0.f;
          v.w = (k + 3 < ke) ? p[3] : 0.f;
        } else {
          const int k = q / (BN / 4), r = 4 * (q % (BN / 4));
          const int64_t gnn = n0 + r;
          const bool okk = k0 + k < ke;
          const float* p = a.B + (okk ? k0 + k : kb) * a.ldb + gnn;
          v.x = (okk && gnn + 0 < a.N) ? p[0] : 0.f;
          v.y = (okk && gnn + 1 < a.N) ? p[1] : 0.f;
          v.z = (okk && gnn + 2 < a.N) ? p[2] : 0.f;
          v.w = (okk && gnn + 3 < a.N) ? p[3] : 0.f;
        }
        rb[i] = v;
      }
    };
    auto store_tile = [&](float* st) {
      float* bs = st + A_IMG;
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        const int q = tid + NT * i;
        if (A_KC) {
          const int r = q / CPR, c = q % CPR;
          *reinterpret_cast<float4*>(st + r * BK + 4 * (c ^ kc_swz<BK>(r))) = ra[i];
        } else {
          *reinterpret_cast<float4*>(st + 4 * q) = ra[i];
        }
      }
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        const int q = tid + NT * i;
        if (B_KC) {
          const int r = q / CPR, c = q % CPR;
          *reinterpret_cast<float4*>(bs + r * BK + 4 * (c ^ kc_swz<BK>(r))) = rb[i];
        } else {
          *reinterpret_cast<float4*>(bs + 4 * q) = rb[i];
        }
      }
    };
    if (nt > 0) {
      load_tile(0);
      store_tile(smem);
      __syncthreads();
    }
    for (int t = 0; t < nt; ++t) {
      const bool more = t + 1 < nt;
      if (more) load_tile(t + 1);  // in flight under the MFMAs below
      compute_tile(smem + (t & 1) * STAGE);
      if (more) store_tile(smem + ((t + 1) & 1) * STAGE);  // stage last read a barrier ago
      __syncthreads();
    }
  }
  __syncthreads();  // every stage read before the buffers are reused below
#if CTR_GEMM_TRACE
  const unsigned long long tr_t1 = clock64();
  if (tid == 0 && tr_b < 16384) {
    const unsigned hw = __builtin_amdgcn_s_getreg(GETREG_IMMED(31, 0, 4));
    const unsigned xcc = __builtin_amdgcn_s_getreg(GETREG_IMMED(3, 0, 20));
    g_gemm_trace[tr_b * 5 + 0] = tr_rt;
    g_gemm_trace[tr_b * 5 + 1] = tr_t0;
    g_gemm_trace[tr_b * 5 + 2] = tr_t1;
    g_gemm_trace[tr_b * 5 + 4] = ((unsigned long long)xcc << 8) | (((hw >> 13) & 3) << 4) | ((hw >> 8) & 15);
  }
#endif

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
    if (kw == 0) {
#pragma unroll
      for (int s = 1; s < KSPLIT; ++s) {
        const float* src = smem + ((s - 1) * WAVES_M * WAVES_N + wmn) * PW;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int tn = 0; tn < TN; ++tn)
#pragma unroll
            for (int r = 0; r < 16; ++r)
              acc[i][tn][r] += src[((i * TN + tn) * 16 + r) * 64 + lane];
      }
    }
    __syncthreads();  // partials consumed before the epilogue reuses the buffer
  }
  if (kw > 0) return;

  gemm_store_tiles<TM, TN>(a, acc, smem + wmn * (32 * 36), m0 + wm0, n0 + wn0, lane);
#if CTR_GEMM_TRACE
  if (tid == 0 && tr_b < 16384) g_gemm_trace[tr_b * 5 + 3] = clock64();
#endif
}

// Split-K slabs [splits][M][N] -> C with the epilogue, summed in slab order.
__global__ __launch_bounds__(256) void splitk_reduce_kernel(GemmArgs a, const float* __restrict__ slabs,
                                                            int splits) {
  if (a.epi == CTR_EPI_BIAS_RELU_DROP && a.step_ptr) a.offset += (uint64_t)(*a.step_ptr) << 32;
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
  int bm, bn, bk, wm, wn, ks, stages;
  double eff;  // sustained fraction of the 0.614 TFLOP/s per-CU fp32 MFMA peak, measured on
               // MI355X per tiling (tools/gemm_bench.py, profiles/r01_gemm_tuning.txt)
};
static const TileDef kTiles[] = {
    {64, 64, 32, 2, 2, 1, 3, 0.57},   {64, 128, 32, 2, 2, 1, 3, 0.57},
    {128, 64, 32, 2, 2, 1, 3, 0.57},  {128, 128, 64, 2, 2, 1, 2, 0.70},
    {64, 160, 64, 2, 1, 2, 2, 0.61},  {128, 416, 32, 4, 1, 1, 2, 0.61},
    {160, 128, 64, 1, 4, 1, 2, 0.64}, {64, 224, 64, 2, 1, 2, 2, 0.58},
    {64, 160, 32, 2, 1, 2, 3, 0.57},  {160, 128, 32, 1, 4, 1, 3, 0.65},
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

template <int BM, int BN, int BK, int WMW, int WNW, int KS, int PF, bool VEC>
static void launch_vec(const GemmArgs& a, bool ta, bool tb, dim3 grid, hipStream_t st) {
  constexpr int NT = WMW * WNW * KS * 64;
#define CTR_GEMM_LAUNCH(TA_, TB_)                                                               \
  hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, BK, WMW, WNW, KS, PF, TA_, TB_, VEC>), grid, NT, \
                     0, st, a)
  if (!ta && !tb) CTR_GEMM_LAUNCH(false, false);
  else if (!ta && tb) CTR_GEMM_LAUNCH(false, true);
  else if (ta && !tb) CTR_GEMM_LAUNCH(true, false);
  else CTR_GEMM_LAUNCH(true, true);
#undef CTR_GEMM_LAUNCH
}

template <int BM, int BN, int BK, int WMW, int WNW, int KS, int PF>
static void launch_cfg(const GemmArgs& a, bool ta, bool tb, dim3 grid, hipStream_t st) {
  if (a.vec_a && a.vec_b)
    launch_vec<BM, BN, BK, WMW, WNW, KS, PF, true>(a, ta, tb, grid, st);
  else
    launch_vec<BM, BN, BK, WMW, WNW, KS, PF, false>(a, ta, tb, grid, st);
}

static void launch_tile(int ti, const GemmArgs& a, bool ta, bool tb, dim3 grid, hipStream_t st) {
  switch (ti) {
    case 0: launch_cfg<64, 64, 32, 2, 2, 1, 3>(a, ta, tb, grid, st); break;
    case 1: launch_cfg<64, 128, 32, 2, 2, 1, 3>(a, ta, tb, grid, st); break;
    case 2: launch_cfg<128, 64, 32, 2, 2, 1, 3>(a, ta, tb, grid, st); break;
    case 3: launch_cfg<128, 128, 64, 2, 2, 1, 2>(a, ta, tb, grid, st); break;
    case 4: launch_cfg<64, 160, 64, 2, 1, 2, 2>(a, ta, tb, grid, st); break;
    case 5: launch_cfg<128, 416, 32, 4, 1, 1, 2>(a, ta, tb, grid, st); break;
    case 6: launch_cfg<160, 128, 64, 1, 4, 1, 2>(a, ta, tb, grid, st); break;
    case 7: launch_cfg<64, 224, 64, 2, 1, 2, 2>(a, ta, tb, grid, st); break;
    case 8: launch_cfg<64, 160, 32, 2, 1, 2, 3>(a, ta, tb, grid, st); break;
    case 9: launch_cfg<160, 128, 32, 1, 4, 1, 3>(a, ta, tb, grid, st); break;
  }
}

}  // namespace ctr

using namespace ctr;

// CTR_GEMM_AUTO resolves to CTR_GEMM_SPLIT_BF16 unless CTR_GEMM_ALGO=exact is set in the
// environment (read once per process).
static int resolve_algo(int algo) {
  if (algo != CTR_GEMM_AUTO) return algo;
  static const int dflt = [] {
    const char* e = getenv("CTR_GEMM_ALGO");
    return (e && (strcmp(e, "exact") == 0 || strcmp(e, "f32") == 0)) ? (int)CTR_GEMM_EXACT_F32
                                                                       : (int)CTR_GEMM_SPLIT_BF16;
  }();
  return dflt;
}

// Measured winners (MI355X, tools/gemm_bench.py sweeps of both kernels over every tiling x
// split-K; profiles/r01_gemm_tuning_sb16.txt) for the shapes of the hot path: the DeepFM
// MLP at B=8192 (C3) and the PG policy MLP at B=4096 (C4). Other shapes use the model.
struct KnownGemm {
  int64_t M, N, K;
  int ta, tb, algo, tile, splits;
};
static const KnownGemm kKnown[] = {
    {8192, 300, 1664, 0, 1, CTR_GEMM_SPLIT_BF16, 4, 2},   // DeepFM fwd0  X.W0^T
    {8192, 200, 300, 0, 1, CTR_GEMM_SPLIT_BF16, 0, 1},    // fwd1  H1.W1^T
    {8192, 300, 200, 0, 0, CTR_GEMM_SPLIT_BF16, 0, 1},    // dH1 = dH2.W1
    {8192, 1664, 300, 0, 0, CTR_GEMM_SPLIT_BF16, 1, 1},   // dX  = dH1.W0
    {200, 300, 8192, 1, 0, CTR_GEMM_EXACT_F32, 0, 16},    // dW1 = dH2^T.H1
    {300, 1664, 8192, 1, 0, CTR_GEMM_SPLIT_BF16, 7, 8},   // dW0 = dH1^T.X (160x128 tiles)
    {4096, 1024, 741, 0, 1, CTR_GEMM_SPLIT_BF16, 2, 1},   // PG policy fwd0
    {1024, 741, 4096, 1, 0, CTR_GEMM_SPLIT_BF16, 3, 4},   // dW0
    {4096, 512, 1024, 0, 1, CTR_GEMM_SPLIT_BF16, 0, 1},   // fwd1
    {4096, 1024, 512, 0, 0, CTR_GEMM_SPLIT_BF16, 3, 1},   // dX1
    {512, 1024, 4096, 1, 0, CTR_GEMM_SPLIT_BF16, 3, 8},   // dW1
};

struct GemmPlan {
  int algo;
  int tile;  // exact kernel's tiling (algo == EXACT)
  Sb16Cfg sc;  // split kernel's config (algo == SPLIT)
  int splits;
  int64_t kps;
  int bm, bn;
};

static GemmPlan plan_gemm(int algo, int ta, int tb, int64_t M, int64_t N, int64_t K) {
  GemmPlan p{};
  auto k_split = [&](int sp, int& splits, int64_t& kps) {
    splits = 1;
    kps = std::max<int64_t>(K, 1);
    if (sp > 1 && K >= 64) {
      kps = align_up(ceil_div(K, sp), 32);
      splits = (int)ceil_div(K, kps);
    }
  };
  const bool forced_cfg = getenv("CTR_GEMM_CFG") != nullptr;
  if (algo == CTR_GEMM_AUTO && !forced_cfg) {
    for (const KnownGemm& k : kKnown) {
      if (k.M != M || k.N != N || k.K != K || k.ta != (ta != 0) || k.tb != (tb != 0)) continue;
      if (k.algo == CTR_GEMM_SPLIT_BF16 && resolve_algo(CTR_GEMM_AUTO) != CTR_GEMM_SPLIT_BF16)
        break;  // the environment asked for the exact kernel everywhere
      p.algo = k.algo;
      k_split(k.splits, p.splits, p.kps);
      if (p.algo == CTR_GEMM_SPLIT_BF16) {
        p.sc = Sb16Cfg{k.tile, p.splits, p.kps, 0, 0};
        sb16_tile_dims(k.tile, p.sc.bm, p.sc.bn);
        p.bm = p.sc.bm, p.bn = p.sc.bn;
      } else {
        p.tile = k.tile;
        p.bm = kTiles[k.tile].bm, p.bn = kTiles[k.tile].bn;
      }
      return p;
    }
  }
  p.algo = resolve_algo(algo);
  if (p.algo == CTR_GEMM_SPLIT_BF16) {
    p.sc = sb16_choose(M, N, K);
    p.splits = p.sc.splits, p.kps = p.sc.kps, p.bm = p.sc.bm, p.bn = p.sc.bn;
  } else {
    const TileCfg c = choose_tiles(M, N, K);
    p.tile = c.tile, p.splits = c.splits, p.kps = c.kps;
    p.bm = kTiles[c.tile].bm, p.bn = kTiles[c.tile].bn;
  }
  return p;
}

extern "C" int64_t ctr_gemm_f32_ex_workspace_bytes(int algo, int trans_a, int trans_b, int64_t M,
                                                   int64_t N, int64_t K) {
  if (M < 0 || N < 0 || K < 0) return -1;
  if (algo < CTR_GEMM_AUTO || algo > CTR_GEMM_SPLIT_BF16) return -1;
  const int64_t s = plan_gemm(algo, trans_a, trans_b, M, N, K).splits;
  return s > 1 ? s * M * N * (int64_t)sizeof(float) : 0;
}

extern "C" int64_t ctr_gemm_f32_workspace_bytes(int trans_a, int trans_b, int64_t M, int64_t N,
                                                int64_t K) {
  return ctr_gemm_f32_ex_workspace_bytes(CTR_GEMM_AUTO, trans_a, trans_b, M, N, K);
}

extern "C" int ctr_gemm_resolved_algo(int algo) { return resolve_algo(algo); }

#if CTR_GEMM_TRACE
extern "C" int ctr_debug_gemm_trace(unsigned long long* host, int n_blocks) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_gemm_trace),
                                  sizeof(unsigned long long) * 5 * std::min(n_blocks, 16384));
}
#endif

extern "C" int ctr_gemm_f32_ex(int algo, int trans_a, int trans_b, int64_t M, int64_t N,
                               int64_t K, const float* A, int64_t lda, const float* B,
                               int64_t ldb, float* C, int64_t ldc, int epi, const float* bias,
                               const float* aux, int64_t ldaux, float scale, float drop_p,
                               uint64_t seed, uint64_t offset, const int32_t* step_ptr, void* ws,
                               int64_t ws_bytes, ctr_stream_t stream) {
  CTR_REQUIRE(algo >= CTR_GEMM_AUTO && algo <= CTR_GEMM_SPLIT_BF16, "ctr_gemm_f32: bad algo %d",
              algo);
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
  a.seed = seed; a.offset = offset; a.step_ptr = step_ptr;
  // float4 path: 16-B aligned rows whose contiguous extent is a multiple of 4 (then a
  // float4 is entirely inside or entirely outside the matrix; split-K bounds are
  // multiples of 32)
  a.vec_a = (reinterpret_cast<uintptr_t>(A) % 16 == 0) && (lda % 4 == 0) &&
            ((trans_a ? M : K) % 4 == 0);
  a.vec_b = (reinterpret_cast<uintptr_t>(B) % 16 == 0) && (ldb % 4 == 0) &&
            ((trans_b ? K : N) % 4 == 0);
  a.vec_c = (reinterpret_cast<uintptr_t>(C) % 16 == 0) && (ldc % 4 == 0);

  const GemmPlan pl = plan_gemm(algo, trans_a, trans_b, M, N, K);
  const int splits = pl.splits;
  const int64_t kps = pl.kps;
  a.k_per_split = splits > 1 ? kps : std::max<int64_t>(K, 1);
  a.slab_stride = 0;
  if (splits > 1) {
    const int64_t need = (int64_t)splits * M * N * (int64_t)sizeof(float);
    if (!ws || ws_bytes < need) {
      set_error("ctr_gemm_f32: split-K workspace %lld < %lld bytes", (long long)ws_bytes,
                (long long)need);
      return CTR_ERR_WORKSPACE;
    }
    a.C = static_cast<float*>(ws);
    a.ldc = N;
    a.slab_stride = M * N;
    a.vec_c = (reinterpret_cast<uintptr_t>(ws) % 16 == 0) && (N % 4 == 0) && ((M * N) % 4 == 0);
  }
  const dim3 grid((unsigned)(ceil_div(N, pl.bn) * ceil_div(M, pl.bm)), 1, (unsigned)splits);
  if (pl.algo == CTR_GEMM_SPLIT_BF16) {
    sb16_launch(pl.sc, a, trans_a != 0, trans_b != 0, grid, st);
    CTR_LAUNCH_CHECK("gemm_sb16_kernel");
  } else {
    launch_tile(pl.tile, a, trans_a != 0, trans_b != 0, grid, st);
    CTR_LAUNCH_CHECK("gemm_f32_kernel");
  }
  if (splits > 1) {
    GemmArgs r = a;
    r.C = C;
    r.ldc = ldc;
    const unsigned g2 = (unsigned)std::min<int64_t>(ceil_div(M * N, 256), 4096);
    hipLaunchKernelGGL(splitk_reduce_kernel, g2, 256, 0, st, r, static_cast<const float*>(ws),
                       splits);
    CTR_LAUNCH_CHECK("splitk_reduce_kernel");
  }
  return CTR_OK;
}

extern "C" int ctr_gemm_f32(int trans_a, int trans_b, int64_t M, int64_t N, int64_t K,
                            const float* A, int64_t lda, const float* B, int64_t ldb, float* C,
                            int64_t ldc, int epi, const float* bias, const float* aux,
                            int64_t ldaux, float scale, float drop_p, uint64_t seed,
                            uint64_t offset, const int32_t* step_ptr, void* ws, int64_t ws_bytes,
                            ctr_stream_t stream) {
  return ctr_gemm_f32_ex(CTR_GEMM_AUTO, trans_a, trans_b, M, N, K, A, lda, B, ldb, C, ldc, epi,
                         bias, aux, ldaux, scale, drop_p, seed, offset, step_ptr, ws, ws_bytes,
                         stream);
}

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

// Global->register staging, built so the loads of k-tile t+1 really overlap the MFMAs of
// k-tile t: no select or branch touches a loaded value until the LDS store that follows
// the MFMA loop (a select right after a load makes hipcc wait vmcnt there). Addresses are
// clamped instead: a row beyond M (or a column beyond N) is read from row 0 — it only
// feeds C entries that are never stored — and the K tail, which feeds every output, is
// zeroed at LDS-store time. Per-thread row pointers are computed once; a k-tile step is
// one pointer increment. VEC: 16-B aligned rows, contiguous extents multiple of 4.
template <int BM, int BN, int WM, int WN, bool TA, bool TB, bool VEC>
__global__ __launch_bounds__((BM / WM) * (BN / WN) * 64) void gemm_f32_kernel(GemmArgs a) {
  constexpr int BK = 32;
  constexpr int PADA = TA ? 4 : 1;  // k-major images; odd stride for transposed writes
  constexpr int PADB = TB ? 1 : 4;
  constexpr int SA = BM + PADA, SB = BN + PADB;
  constexpr int WAVES_N = BN / WN;
  constexpr int NT = (BM / WM) * (BN / WN) * 64;  // 4 waves (1/SIMD) or 8 (2/SIMD)
  constexpr int TM = WM / 32, TN = WN / 32;
  constexpr int NA = BM * BK / 4 / NT;  // float4 loads per thread per k-tile
  constexpr int NB = BN * BK / 4 / NT;
  static_assert(NT == 256 || NT == 512, "4 or 8 waves per block");
  static_assert(NA >= 1 && NB >= 1, "tile too small for the block");

  // two LDS stages: the next k-tile is written while the current one feeds the MFMAs,
  // one barrier per k-tile
  __shared__ __attribute__((aligned(16))) float As[2][BK * SA];
  __shared__ __attribute__((aligned(16))) float Bs[2][BK * SB];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm0 = (wave / WAVES_N) * WM;
  const int wn0 = (wave % WAVES_N) * WN;
  const int64_t m0 = (int64_t)blockIdx.y * BM;
  const int64_t n0 = (int64_t)blockIdx.x * BN;
  const int64_t kb = (int64_t)blockIdx.z * a.k_per_split;
  const int64_t ke = min(a.K, kb + a.k_per_split);

  // per-thread fixed tile coordinates and row pointers (at k = kb)
  const float* pa[NA];
  const float* pb[NB];
  int ka[NA], kbv[NB];  // k offset inside the tile this thread's float4 starts at
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    const int q = tid + NT * i;
    if (!TA) {  // A[m][k], k contiguous
      const int m = q / (BK / 4), k4 = q % (BK / 4);
      const int64_t gm = m0 + m;
      ka[i] = k4 * 4;
      pa[i] = a.A + (gm < a.M ? gm : 0) * a.lda + kb + ka[i];
    } else {  // A stored [k][m], m contiguous
      const int k = q / (BM / 4), m4 = q % (BM / 4);
      const int64_t gm = m0 + m4 * 4;
      ka[i] = k;
      pa[i] = a.A + (kb + k) * a.lda + (gm < a.M ? gm : 0);
    }
  }
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int q = tid + NT * i;
    if (!TB) {  // B[k][n], n contiguous
      const int k = q / (BN / 4), n4 = q % (BN / 4);
      const int64_t gn = n0 + n4 * 4;
      kbv[i] = k;
      pb[i] = a.B + (kb + k) * a.ldb + (gn < a.N ? gn : 0);
    } else {  // B stored [n][k] (nn.Linear weight), k contiguous
      const int n = q / (BK / 4), k4 = q % (BK / 4);
      const int64_t gn = n0 + n;
      kbv[i] = k4 * 4;
      pb[i] = a.B + (gn < a.N ? gn : 0) * a.ldb + kb + kbv[i];
    }
  }
  const int64_t stepA = TA ? BK * a.lda : BK;  // pointer advance per k-tile
  const int64_t stepB = TB ? BK : BK * a.ldb;

  float4 ra[NA], rb[NB];
  auto load_tile = [&](int t) {  // k-tile t of this split, rows clamped, K tail not masked
    const int64_t k0 = kb + (int64_t)t * BK;
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const float* p = pa[i] + t * stepA;
      if (VEC) {
        // a float4 wholly past the K end reads the split's first tile instead (masked later)
        const bool okk = k0 + ka[i] < ke;
        ra[i] = *reinterpret_cast<const float4*>(okk ? p : pa[i]);
      } else {
        const int kl0 = (int)(k0 + ka[i] - kb);
        float4 v;
        if (!TA) {
          v.x = (k0 + ka[i] + 0 < ke) ? p[0] : 0.f;
          v.y = (k0 + ka[i] + 1 < ke) ? p[1] : 0.f;
          v.z = (k0 + ka[i] + 2 < ke) ? p[2] : 0.f;
          v.w = (k0 + ka[i] + 3 < ke) ? p[3] : 0.f;
        } else {
          const int q = tid + NT * i;
          const int64_t gm = m0 + (q % (BM / 4)) * 4;
          const bool okk = k0 + ka[i] < ke;
          v.x = (okk && gm + 0 < a.M) ? p[0] : 0.f;
          v.y = (okk && gm + 1 < a.M) ? p[1] : 0.f;
          v.z = (okk && gm + 2 < a.M) ? p[2] : 0.f;
          v.w = (okk && gm + 3 < a.M) ? p[3] : 0.f;
        }
        (void)kl0;
        ra[i] = v;
      }
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const float* p = pb[i] + t * stepB;
      if (VEC) {
        const bool okk = k0 + kbv[i] < ke;
        rb[i] = *reinterpret_cast<const float4*>(okk ? p : pb[i]);
      } else {
        float4 v;
        if (TB) {
          v.x = (k0 + kbv[i] + 0 < ke) ? p[0] : 0.f;
          v.y = (k0 + kbv[i] + 1 < ke) ? p[1] : 0.f;
          v.z = (k0 + kbv[i] + 2 < ke) ? p[2] : 0.f;
          v.w = (k0 + kbv[i] + 3 < ke) ? p[3] : 0.f;
        } else {
          const int q = tid + NT * i;
          const int64_t gn = n0 + (q % (BN / 4)) * 4;
          const bool okk = k0 + kbv[i] < ke;
          v.x = (okk && gn + 0 < a.N) ? p[0] : 0.f;
          v.y = (okk && gn + 1 < a.N) ? p[1] : 0.f;
          v.z = (okk && gn + 2 < a.N) ? p[2] : 0.f;
          v.w = (okk && gn + 3 < a.N) ? p[3] : 0.f;
        }
        rb[i] = v;
      }
    }
  };

  auto store_tile = [&](int buf, int t) {
    const int64_t k0 = kb + (int64_t)t * BK;
    float* as = As[buf];
    float* bs = Bs[buf];
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int q = tid + NT * i;
      float4 v = ra[i];
      if (VEC && !(k0 + ka[i] < ke)) v = make_float4(0.f, 0.f, 0.f, 0.f);  // K tail
      if (!TA) {
        const int m = q / (BK / 4), k4 = q % (BK / 4);
        as[(k4 * 4 + 0) * SA + m] = v.x;
        as[(k4 * 4 + 1) * SA + m] = v.y;
        as[(k4 * 4 + 2) * SA + m] = v.z;
        as[(k4 * 4 + 3) * SA + m] = v.w;
      } else {
        const int k = q / (BM / 4), m4 = q % (BM / 4);
        *reinterpret_cast<float4*>(&as[k * SA + m4 * 4]) = v;
      }
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int q = tid + NT * i;
      float4 v = rb[i];
      if (VEC && !(k0 + kbv[i] < ke)) v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (!TB) {
        const int k = q / (BN / 4), n4 = q % (BN / 4);
        *reinterpret_cast<float4*>(&bs[k * SB + n4 * 4]) = v;
      } else {
        const int n = q / (BK / 4), k4 = q % (BK / 4);
        bs[(k4 * 4 + 0) * SB + n] = v.x;
        bs[(k4 * 4 + 1) * SB + n] = v.y;
        bs[(k4 * 4 + 2) * SB + n] = v.z;
        bs[(k4 * 4 + 3) * SB + n] = v.w;
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

  const int kl = lane >> 5;  // k within the MFMA's K=2
  const int il = lane & 31;
  if (kb < ke) {
    const int nt = (int)((ke - kb + BK - 1) / BK);
    load_tile(0);
    store_tile(0, 0);
    __syncthreads();
    for (int t = 0; t < nt; ++t) {
      const int buf = t & 1;
      const bool more = t + 1 < nt;
      if (more) load_tile(t + 1);  // in flight under the MFMAs below
      const float* as = As[buf] + kl * SA + wm0 + il;
      const float* bs = Bs[buf] + kl * SB + wn0 + il;
      // every fragment of the k-tile is read first; the MFMA chain then only waits for
      // the reads it consumes (progressive lgkmcnt), not a full LDS round trip per step
      float af[BK / 2][TM], bf[BK / 2][TN];
#pragma unroll
      for (int kk = 0; kk < BK / 2; ++kk) {
#pragma unroll
        for (int i = 0; i < TM; ++i) af[kk][i] = as[kk * 2 * SA + i * 32];
#pragma unroll
        for (int j = 0; j < TN; ++j) bf[kk][j] = bs[kk * 2 * SB + j * 32];
      }
      // keep the reads ahead of the chain: hipcc's scheduler otherwise re-interleaves them
      // with an lgkmcnt(0) before every MFMA group
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int kk = 0; kk < BK / 2; ++kk)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[kk][i], bf[kk][j], acc[i][j],
                                                             0, 0, 0);
      if (more) store_tile(buf ^ 1, t + 1);  // the other stage: last read one barrier ago
      __syncthreads();
    }
  }

  // C/D map of the 32x32 f32 MFMA: col = lane & 31, row = (r&3) + 8*(r>>2) + 4*(lane>>5).
  float* C = a.C + (int64_t)blockIdx.z * a.slab_stride;
  const int epi = a.slab_stride ? (int)CTR_EPI_NONE : a.epi;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t m = m0 + wm0 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * kl;
        const int64_t n = n0 + wn0 + j * 32 + il;
        if (m < a.M && n < a.N) C[m * a.ldc + n] = apply_epi(a, epi, acc[i][j][r], m, n);
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

struct TileCfg {
  int bm, bn;
  int splits;
  int64_t kps;
  int waves;  // 4 (one per SIMD) or 8 (two per SIMD)
};

// Pick (tile, split-K, waves) by a makespan model calibrated on MI355X (tools/gemm_bench.py,
// profiles/r01_gemm_tuning.txt): every tiling sustains about the same per-CU rate
// (~0.36 TFLOP/s), so the choice is about load balance — blocks are dealt to 256 CUs in
// rounds, a round costs one block's flops at that rate plus ~1.5 us of prologue/epilogue,
// and split-K adds its fp32 slab round trip (2 * splits * M * N * 4 B at ~5 TB/s) and a
// reduce launch. CTR_GEMM_CFG="bm,bn,splits[,waves]" forces a choice (tuning only).
static TileCfg choose_tiles(int64_t M, int64_t N, int64_t K) {
  static const struct { int bm, bn, waves; } cands[] = {
      {128, 128, 4}, {128, 64, 4}, {64, 128, 4}, {64, 64, 4}, {128, 64, 8}, {64, 128, 8}};
  const double cu_tflops = 0.36;
  TileCfg best{64, 64, 1, std::max<int64_t>(K, 1), 4};
  double best_t = 1e30;
  if (const char* env = getenv("CTR_GEMM_CFG")) {
    int bm = 0, bn = 0, sp = 0, wv = 4;
    const int nf = sscanf(env, "%d,%d,%d,%d", &bm, &bn, &sp, &wv);
    if (nf >= 3 && (bm == 64 || bm == 128) && (bn == 64 || bn == 128) && sp >= 1 &&
        (wv == 4 || (wv == 8 && bm * bn >= 128 * 64))) {
      TileCfg c{bm, bn, 1, std::max<int64_t>(K, 1), wv};
      if (sp > 1 && K >= 64) {
        c.kps = align_up(ceil_div(K, sp), 32);
        c.splits = (int)ceil_div(K, c.kps);
      }
      return c;
    }
  }
  for (const auto& cd : cands) {
    const int64_t tiles = ceil_div(M, cd.bm) * ceil_div(N, cd.bn);
    for (int s = 1; s <= 32; ++s) {
      if (s > 1 && K / s < 256) break;  // keep >= 8 k-tiles per split
      const int64_t kps = s == 1 ? K : align_up(ceil_div(K, s), 32);
      const int splits = s == 1 ? 1 : (int)ceil_div(K, kps);
      if (splits != s) continue;
      const int64_t blocks = tiles * splits;
      const double rounds = (double)ceil_div(blocks, 256);
      const double t_block = 2.0 * cd.bm * cd.bn * (double)kps / (cu_tflops * 1e6) + 1.5;
      double t = rounds * t_block;
      if (splits > 1) t += 2.0 * splits * (double)M * N * 4 / 5e6 + 3.0;  // us
      if (t < best_t * 0.98) {
        best_t = t;
        best = TileCfg{cd.bm, cd.bn, splits, splits > 1 ? kps : std::max<int64_t>(K, 1), cd.waves};
      }
    }
  }
  return best;
}

template <int BM, int BN, int WM, int WN, bool VEC>
static void launch_vec(const GemmArgs& a, bool ta, bool tb, dim3 grid, hipStream_t st) {
  constexpr int NT = (BM / WM) * (BN / WN) * 64;
  if (!ta && !tb)
    hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, WM, WN, false, false, VEC>), grid, NT, 0, st, a);
  else if (!ta && tb)
    hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, WM, WN, false, true, VEC>), grid, NT, 0, st, a);
  else if (ta && !tb)
    hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, WM, WN, true, false, VEC>), grid, NT, 0, st, a);
  else
    hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, WM, WN, true, true, VEC>), grid, NT, 0, st, a);
}

template <int BM, int BN, int WM, int WN>
static void launch_cfg(const GemmArgs& a, bool ta, bool tb, dim3 grid, hipStream_t st) {
  if (a.vec_a && a.vec_b)
    launch_vec<BM, BN, WM, WN, true>(a, ta, tb, grid, st);
  else
    launch_vec<BM, BN, WM, WN, false>(a, ta, tb, grid, st);
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
  const dim3 grid((unsigned)ceil_div(N, c.bn), (unsigned)ceil_div(M, c.bm), (unsigned)c.splits);
  const bool ta = trans_a != 0, tb = trans_b != 0;
  if (c.waves == 8) {  // two waves per SIMD: one's LDS-store/barrier phase hides under the
                      // other's MFMA chain
    if (c.bm == 128 && c.bn == 128) launch_cfg<128, 128, 64, 32>(a, ta, tb, grid, st);
    else if (c.bm == 128) launch_cfg<128, 64, 32, 32>(a, ta, tb, grid, st);
    else launch_cfg<64, 128, 32, 32>(a, ta, tb, grid, st);
  } else if (c.bm == 128 && c.bn == 128) launch_cfg<128, 128, 64, 64>(a, ta, tb, grid, st);
  else if (c.bm == 128) launch_cfg<128, 64, 64, 32>(a, ta, tb, grid, st);
  else if (c.bn == 128) launch_cfg<64, 128, 32, 64>(a, ta, tb, grid, st);
  else launch_cfg<64, 64, 32, 32>(a, ta, tb, grid, st);
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

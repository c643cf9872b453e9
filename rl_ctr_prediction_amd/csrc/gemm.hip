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

template <int BM, int BN, int WM, int WN, bool TA, bool TB>
__global__ __launch_bounds__(256) void gemm_f32_kernel(GemmArgs a) {
  constexpr int BK = 32;
  constexpr int PADA = TA ? 4 : 1;
  constexpr int PADB = TB ? 1 : 4;
  constexpr int SA = BM + PADA, SB = BN + PADB;
  constexpr int WAVES_N = BN / WN;
  constexpr int TM = WM / 32, TN = WN / 32;
  constexpr int NA = BM * BK / 4 / 256;  // float4 loads per thread per k-tile
  constexpr int NB = BN * BK / 4 / 256;
  static_assert((BM / WM) * (BN / WN) == 4, "4 waves per block");
  static_assert(NA >= 1 && NB >= 1, "tile too small for 256 threads");

  __shared__ __attribute__((aligned(16))) float As[BK * SA];
  __shared__ __attribute__((aligned(16))) float Bs[BK * SB];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm0 = (wave / WAVES_N) * WM;
  const int wn0 = (wave % WAVES_N) * WN;
  const int64_t m0 = (int64_t)blockIdx.y * BM;
  const int64_t n0 = (int64_t)blockIdx.x * BN;
  const int64_t kb = (int64_t)blockIdx.z * a.k_per_split;
  const int64_t ke = min(a.K, kb + a.k_per_split);

  float4 ra[NA], rb[NB];

  auto load_tile = [&](int64_t k0) {
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int q = tid + 256 * i;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (!TA) {  // A[m][k], k contiguous
        const int m = q / (BK / 4), k4 = q % (BK / 4);
        const int64_t gm = m0 + m, gk = k0 + k4 * 4;
        if (gm < a.M) {
          const float* src = a.A + gm * a.lda + gk;
          if (a.vec_a && gk + 3 < ke) {
            v = *reinterpret_cast<const float4*>(src);
          } else {
            if (gk + 0 < ke) v.x = src[0];
            if (gk + 1 < ke) v.y = src[1];
            if (gk + 2 < ke) v.z = src[2];
            if (gk + 3 < ke) v.w = src[3];
          }
        }
      } else {  // A stored [k][m], m contiguous
        const int k = q / (BM / 4), m4 = q % (BM / 4);
        const int64_t gk = k0 + k, gm = m0 + m4 * 4;
        if (gk < ke) {
          const float* src = a.A + gk * a.lda + gm;
          if (a.vec_a && gm + 3 < a.M) {
            v = *reinterpret_cast<const float4*>(src);
          } else {
            if (gm + 0 < a.M) v.x = src[0];
            if (gm + 1 < a.M) v.y = src[1];
            if (gm + 2 < a.M) v.z = src[2];
            if (gm + 3 < a.M) v.w = src[3];
          }
        }
      }
      ra[i] = v;
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int q = tid + 256 * i;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (!TB) {  // B[k][n], n contiguous
        const int k = q / (BN / 4), n4 = q % (BN / 4);
        const int64_t gk = k0 + k, gn = n0 + n4 * 4;
        if (gk < ke) {
          const float* src = a.B + gk * a.ldb + gn;
          if (a.vec_b && gn + 3 < a.N) {
            v = *reinterpret_cast<const float4*>(src);
          } else {
            if (gn + 0 < a.N) v.x = src[0];
            if (gn + 1 < a.N) v.y = src[1];
            if (gn + 2 < a.N) v.z = src[2];
            if (gn + 3 < a.N) v.w = src[3];
          }
        }
      } else {  // B stored [n][k] (nn.Linear weight), k contiguous
        const int n = q / (BK / 4), k4 = q % (BK / 4);
        const int64_t gn = n0 + n, gk = k0 + k4 * 4;
        if (gn < a.N) {
          const float* src = a.B + gn * a.ldb + gk;
          if (a.vec_b && gk + 3 < ke) {
            v = *reinterpret_cast<const float4*>(src);
          } else {
            if (gk + 0 < ke) v.x = src[0];
            if (gk + 1 < ke) v.y = src[1];
            if (gk + 2 < ke) v.z = src[2];
            if (gk + 3 < ke) v.w = src[3];
          }
        }
      }
      rb[i] = v;
    }
  };

  auto store_tile = [&]() {
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int q = tid + 256 * i;
      if (!TA) {
        const int m = q / (BK / 4), k4 = q % (BK / 4);
        As[(k4 * 4 + 0) * SA + m] = ra[i].x;
        As[(k4 * 4 + 1) * SA + m] = ra[i].y;
        As[(k4 * 4 + 2) * SA + m] = ra[i].z;
        As[(k4 * 4 + 3) * SA + m] = ra[i].w;
      } else {
        const int k = q / (BM / 4), m4 = q % (BM / 4);
        *reinterpret_cast<float4*>(&As[k * SA + m4 * 4]) = ra[i];
      }
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int q = tid + 256 * i;
      if (!TB) {
        const int k = q / (BN / 4), n4 = q % (BN / 4);
        *reinterpret_cast<float4*>(&Bs[k * SB + n4 * 4]) = rb[i];
      } else {
        const int n = q / (BK / 4), k4 = q % (BK / 4);
        Bs[(k4 * 4 + 0) * SB + n] = rb[i].x;
        Bs[(k4 * 4 + 1) * SB + n] = rb[i].y;
        Bs[(k4 * 4 + 2) * SB + n] = rb[i].z;
        Bs[(k4 * 4 + 3) * SB + n] = rb[i].w;
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
    load_tile(kb);
    store_tile();
    __syncthreads();
    for (int64_t k0 = kb; k0 < ke; k0 += BK) {
      const bool more = k0 + BK < ke;
      if (more) load_tile(k0 + BK);
#pragma unroll
      for (int kk = 0; kk < BK / 2; ++kk) {
        float af[TM], bf[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) af[i] = As[(kk * 2 + kl) * SA + wm0 + i * 32 + il];
#pragma unroll
        for (int j = 0; j < TN; ++j) bf[j] = Bs[(kk * 2 + kl) * SB + wn0 + j * 32 + il];
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i], bf[j], acc[i][j], 0, 0, 0);
      }
      __syncthreads();
      if (more) {
        store_tile();
        __syncthreads();
      }
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
};

static TileCfg choose_tiles(int64_t M, int64_t N, int64_t K) {
  constexpr int64_t kTarget = 256;  // one workgroup per CU at least
  const int64_t t128 = ceil_div(M, 128) * ceil_div(N, 128);
  const int64_t t12864 = ceil_div(M, 128) * ceil_div(N, 64);
  const int64_t t64128 = ceil_div(M, 64) * ceil_div(N, 128);
  const int64_t t64 = ceil_div(M, 64) * ceil_div(N, 64);
  TileCfg c{64, 64, 1, K};
  int64_t tiles = t64;
  if (t128 >= kTarget) {
    c.bm = 128; c.bn = 128; tiles = t128;
  } else if (t12864 >= kTarget && M >= N) {
    c.bm = 128; c.bn = 64; tiles = t12864;
  } else if (t64128 >= kTarget) {
    c.bm = 64; c.bn = 128; tiles = t64128;
  }
  // Few output tiles and a long K (weight gradients: K = batch): split K so the grid
  // covers the chip; each split keeps >= 512 of K.
  if (tiles < kTarget && K >= 1024) {
    int64_t s = std::min<int64_t>(ceil_div(2 * kTarget, tiles), K / 512);
    s = std::max<int64_t>(1, std::min<int64_t>(s, 64));
    if (s > 1) {
      c.kps = align_up(ceil_div(K, s), 32);
      c.splits = (int)ceil_div(K, c.kps);
    }
  }
  return c;
}

template <int BM, int BN, int WM, int WN>
static void launch_cfg(const GemmArgs& a, bool ta, bool tb, dim3 grid, hipStream_t st) {
  if (!ta && !tb)
    hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, WM, WN, false, false>), grid, 256, 0, st, a);
  else if (!ta && tb)
    hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, WM, WN, false, true>), grid, 256, 0, st, a);
  else if (ta && !tb)
    hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, WM, WN, true, false>), grid, 256, 0, st, a);
  else
    hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, WM, WN, true, true>), grid, 256, 0, st, a);
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
  a.vec_a = (reinterpret_cast<uintptr_t>(A) % 16 == 0) && (lda % 4 == 0);
  a.vec_b = (reinterpret_cast<uintptr_t>(B) % 16 == 0) && (ldb % 4 == 0);

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
  if (c.bm == 128 && c.bn == 128) launch_cfg<128, 128, 64, 64>(a, ta, tb, grid, st);
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

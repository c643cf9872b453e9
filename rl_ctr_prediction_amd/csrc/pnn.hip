// Inner-product network (IPNN): the pairwise-interaction input of
// p_model.InnerPNN (reference src/models/p_model.py:146-200) and its backward.
//
// Forward (p_model.py:187-195): for every example b of F fields with embeddings e_f = E[x_bf]
//   cat[b] = [ flat(e_0..e_{F-1}) (F*K) | <e_i, e_j> for i < j in row-major pair order (P) ]
// (P = F(F-1)/2, the reference's self.row / self.col lists, p_model.py:179-182), which feeds
// the MLP GEMMs. Backward: given dcat = dL/dcat (the dX GEMM's output), the gradient of
// slot (b, f):
//   dslot[b*F+f, k] = dcat[b, f*K+k] + sum_{j != f} dcat[b, F*K + pair(f,j)] * e_j[k]
// (the view's gradient plus the two index backwards of embedding_x[:, row] / [:, col]),
// written per slot; the per-row sums then go through the deterministic segmented sum
// (ctr_segment_sum_rows) exactly like the FM / DeepFM scatter.
//
// One wave per example: the example's F x K embeddings are staged once in a wave-private
// LDS tile (row stride K+1: lanes reading different fields at the same k hit different
// banks), every global access is a coalesced run of a K-float row; the products are
// VALU work (F^2 K per example, ~0.3 GFLOP per C3 batch: far under the HBM time of the
// gathers), so no MFMA.
#include "ctr_common.h"

namespace ctr {

// pair ordinal of (i, j), i < j, in row-major order: (0,1),(0,2)..(0,F-1),(1,2)..
__device__ __forceinline__ int pair_index(int i, int j, int F) {
  return i * (2 * F - i - 1) / 2 + (j - i - 1);
}

// xpl (optional): the MLP input written as its three bf16 planes (the split-bf16 GEMMs'
// operand, csrc/gemm_planes.hip) — flat part from the staged tile, pair part as computed —
// so no fp32 copy of cat and no split pass; cat may then be NULL.
template <typename IdxT>
__global__ __launch_bounds__(256) void ipnn_forward_kernel(const IdxT* __restrict__ idx,
                                                           int64_t B, int F, int K, int64_t V,
                                                           const float* __restrict__ emb,
                                                           float* __restrict__ cat, int64_t ldc,
                                                           int32_t* err,
                                                           uint16_t* __restrict__ xpl,
                                                           int64_t xpl_ld, int64_t xpl_ps) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int wave = threadIdx.x / kWave;
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t b = (int64_t)blockIdx.x * (blockDim.x / kWave) + wave;
  if (b >= B) return;  // wave-uniform; the tile is wave-private (no block barrier)
  // row stride: K + 4 when K % 4 == 0 (16-B aligned rows: the dots read float4s; the 16
  // lanes of a ds_read_b128 quarter-wave read rows j..j+15 of one field pair walk, banks
  // 4j + k, all distinct), else K + 1
  const bool vec = (K & 3) == 0;
  const int ld = vec ? K + 4 : K + 1;
  float* tile = lds + (int64_t)wave * F * ld;
  float* ob = cat ? cat + b * ldc : nullptr;
  stage_rows_wave(idx, b, F, K, V, emb, tile, ld, ob, err, lane);
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS stores are done
  __builtin_amdgcn_wave_barrier();
  const int P = F * (F - 1) / 2;
  uint16_t* xb = xpl ? xpl + b * xpl_ld : nullptr;
  // lane -> pairs p = lane, lane + 64, ...; (i, j) walked incrementally
  int i = 0, rem = lane;
  for (int p = lane; p < P; p += kWave) {
    while (rem >= F - 1 - i) {
      rem -= F - 1 - i;
      ++i;
    }
    const int j = i + 1 + rem;
    const float* ei = tile + i * ld;
    const float* ej = tile + j * ld;
    float acc = 0.f;
    {
#pragma clang fp contract(off)
      if (vec) {  // the same products and sums in the same k order, four k per LDS read
        for (int k = 0; k < K; k += 4) {
          const float4 x = *reinterpret_cast<const float4*>(ei + k);
          const float4 y = *reinterpret_cast<const float4*>(ej + k);
          acc += x.x * y.x;
          acc += x.y * y.y;
          acc += x.z * y.z;
          acc += x.w * y.w;
        }
      } else {
        for (int k = 0; k < K; ++k) acc += ei[k] * ej[k];  // torch.mul, then torch.sum
      }
    }
    if (ob) ob[(int64_t)F * K + p] = acc;
    if (xb) {
      uint16_t h3[3];
      psplit1(acc, h3);
#pragma unroll
      for (int q = 0; q < 3; ++q) xb[q * xpl_ps + (int64_t)F * K + p] = h3[q];
    }
    rem += kWave;
  }
  if (xb) {  // the flat part's planes (columns 0 .. F*K), 4 consecutive elements per lane
    if ((K & 3) == 0 && (xpl_ld & 3) == 0) {
      for (int t = 4 * lane; t < F * K; t += 4 * kWave) {
        const int f = t / K, k = t - f * K;
        const float* r = tile + f * ld + k;
        store_planes4_at(xb + t, xpl_ps, make_float4(r[0], r[1], r[2], r[3]));
      }
    } else {
      for (int t = lane; t < F * K; t += kWave) {
        const int f = t / K, k = t - f * K;
        uint16_t h3[3];
        psplit1(tile[f * ld + k], h3);
#pragma unroll
        for (int q = 0; q < 3; ++q) xb[q * xpl_ps + t] = h3[q];
      }
    }
  }
}

template <typename IdxT>
__global__ __launch_bounds__(256) void ipnn_backward_kernel(const IdxT* __restrict__ idx,
                                                            int64_t B, int F, int K, int64_t V,
                                                            const float* __restrict__ emb,
                                                            const float* __restrict__ dcat,
                                                            int64_t ldd,
                                                            float* __restrict__ dslot) {
#pragma clang fp contract(off)  // torch.mul, then the index_put accumulation: rounded apart
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int wave = threadIdx.x / kWave;
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t b = (int64_t)blockIdx.x * (blockDim.x / kWave) + wave;
  if (b >= B) return;
  const int ld = K + 1;
  const int P = F * (F - 1) / 2;
  float* tile = lds + (int64_t)wave * (F * ld + P);
  float* dp = tile + F * ld;
  stage_rows_wave(idx, b, F, K, V, emb, tile, ld, (float*)nullptr, (int32_t*)nullptr, lane);
  const float* db = dcat + b * ldd;
  for (int p = lane; p < P; p += kWave) dp[p] = db[(int64_t)F * K + p];
  __builtin_amdgcn_s_waitcnt(0xc07f);
  __builtin_amdgcn_wave_barrier();
  float* out = dslot + b * (int64_t)F * K;
  for (int t = lane; t < F * K; t += kWave) {  // output (f, k), contiguous per example
    const int f = t / K, k = t - f * K;
    float g = db[t];
    // j ascending, j != f (the reference's order): pairs (j, f) for j < f sit at strides
    // F - j - 2 from pair_index(0, f) = f - 1; pairs (f, j) for j > f are contiguous from
    // pair_index(f, f + 1) — no per-j branch or index arithmetic, so the loops unroll
    int q = f - 1;
#pragma unroll 4
    for (int j = 0; j < f; ++j) {
      g += dp[q] * tile[j * ld + k];
      q += F - j - 2;
    }
    const int base = (f * (2 * F - f - 1)) / 2 - (f + 1);  // dp[base + j] = pair (f, j)
#pragma unroll 4
    for (int j = f + 1; j < F; ++j) g += dp[base + j] * tile[j * ld + k];
    out[t] = g;
  }
}

// The backward with the example's rows held in registers (lane = column k; FMAX >= F
// fields, KC columns per lane): ONE walk over the pairs in row-major order, each pair's
// dcat read once (an LDS broadcast) and applied to both its fields,
//   g_i += dp(i,j) * e_j,  g_j += dp(i,j) * e_i.
// For a field f the pairs (j, f), j < f, come before (f, j), j > f, in that walk, so g_f
// receives its terms in ascending j — the same operations in the same order as
// ipnn_backward_kernel (bitwise equal; tests/test_gpu_kernels.py), with one LDS read per
// pair instead of two per term, and no row staging in LDS.
template <typename IdxT, int FMAX, int KC>
__global__ __launch_bounds__(256) void ipnn_backward_reg(const IdxT* __restrict__ idx,
                                                         int64_t B, int F, int K, int64_t V,
                                                         const float* __restrict__ emb,
                                                         const float* __restrict__ dcat,
                                                         int64_t ldd,
                                                         float* __restrict__ dslot) {
#pragma clang fp contract(off)  // torch.mul, then the index_put accumulation: rounded apart
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int wave = threadIdx.x / kWave;
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t b = (int64_t)blockIdx.x * (blockDim.x / kWave) + wave;
  if (b >= B) return;  // wave-uniform; the LDS slice is wave-private
  const int P = F * (F - 1) / 2;
  float* dp = lds + (int64_t)wave * (FMAX * (FMAX - 1) / 2);
  const float* db = dcat + b * ldd;
  for (int p = lane; p < P; p += kWave) dp[p] = db[(int64_t)F * K + p];
  const long long my_row = lane < F ? (long long)load_row(idx, b * F + lane, V, (int32_t*)nullptr)
                                    : 0ll;
  float e[FMAX][KC], g[FMAX][KC];
#pragma unroll
  for (int j = 0; j < FMAX; ++j) {
    const long long row = __shfl(my_row, j < F ? j : 0, kWave);
#pragma unroll
    for (int c = 0; c < KC; ++c) {
      const int k = lane + kWave * c;
      const bool ok = j < F && k < K;
      e[j][c] = ok ? emb[(int64_t)row * K + k] : 0.f;
      g[j][c] = ok ? db[(int64_t)j * K + k] : 0.f;
    }
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's dp stores are done
  __builtin_amdgcn_wave_barrier();
  int p = 0;
#pragma unroll
  for (int i = 0; i < FMAX - 1; ++i) {
#pragma unroll
    for (int j = i + 1; j < FMAX; ++j) {
      if (j < F) {  // wave-uniform
        const float d = dp[p++];
#pragma unroll
        for (int c = 0; c < KC; ++c) {
          g[i][c] += d * e[j][c];
          g[j][c] += d * e[i][c];
        }
      }
    }
  }
  float* out = dslot + b * (int64_t)F * K;
#pragma unroll
  for (int f = 0; f < FMAX; ++f)
#pragma unroll
    for (int c = 0; c < KC; ++c) {
      const int k = lane + kWave * c;
      if (f < F && k < K) out[(int64_t)f * K + k] = g[f][c];
    }
}

// The register walk for a compile-time field count (the CTR layouts: F = 26 Criteo, 22
// Avazu): every pair slot is static, so each pair value is read into an SGPR at a fixed lane
// of a fixed register, and each update is one VALU multiply by that SGPR operand plus one
// add: no LDS, no per-pair
// branch or wait (the pair values come in by coalesced vector loads, then v_readlane). The same
// pair walk and operations as ipnn_backward_reg (bitwise equal).
template <typename IdxT, int F>
__global__ __launch_bounds__(256) void ipnn_backward_sreg(const IdxT* __restrict__ idx,
                                                          int64_t B, int K, int64_t V,
                                                          const float* __restrict__ emb,
                                                          const float* __restrict__ dcat,
                                                          int64_t ldd,
                                                          float* __restrict__ dslot) {
#pragma clang fp contract(off)  // torch.mul, then the index_put accumulation: rounded apart
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t b = (int64_t)blockIdx.x * (blockDim.x / kWave) + wave;
  if (b >= B) return;
  const float* db = dcat + b * ldd;
  const float* dp = db + (int64_t)F * K;  // the F(F-1)/2 pair gradients
  constexpr int P = F * (F - 1) / 2, ND = (P + kWave - 1) / kWave;
  const long long my_row = lane < F ? (long long)load_row(idx, b * F + lane, V, (int32_t*)nullptr)
                                    : 0ll;
  // the pair values: one coalesced vector load per 64 pairs (lane l holds pair c*64 + l),
  // in flight with the rows; each pair's value then reaches the wave by v_readlane
  float vd[ND];
#pragma unroll
  for (int c = 0; c < ND; ++c) vd[c] = c * kWave + lane < P ? dp[c * kWave + lane] : 0.f;
  const bool ok = lane < K;
  float e[F], g[F];
#pragma unroll
  for (int j = 0; j < F; ++j) {
    const long long row = __shfl(my_row, j, kWave);
    e[j] = ok ? emb[(int64_t)row * K + lane] : 0.f;
    g[j] = ok ? db[(int64_t)j * K + lane] : 0.f;
  }
  int p = 0;
#pragma unroll
  for (int i = 0; i < F - 1; ++i) {
#pragma unroll
    for (int j = i + 1; j < F; ++j, ++p) {
      const float d = __builtin_bit_cast(
          float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, vd[p / kWave]), p % kWave));
      g[i] += d * e[j];
      g[j] += d * e[i];
      // no scheduling across 32-pair groups: the readlanes of a group stay beside its
      // updates (hoisted, 325 SGPR values spill)
      if (p % 32 == 31) __builtin_amdgcn_sched_barrier(0);
    }
  }
  if (ok) {
    float* out = dslot + b * (int64_t)F * K + lane;
#pragma unroll
    for (int f = 0; f < F; ++f) out[(int64_t)f * K] = g[f];
  }
}

// The backward as one small product per example on the fp32 matrix cores: with D the
// symmetric F x F matrix of the pair gradients (zero diagonal) and E the example's F
// embedding rows, the slot gradients are G = dflat + D E. One wave per example, one
// v_mfma_f32_32x32x2_f32 chain per 32 columns: F padded to 32, the chain starts from dflat
// (the accumulator's initial value) and runs 16 k-steps of two fields each. Lane l holds
// A = D[l & 31][2i + (l >> 5)] (gathered from the pair row of dcat) and B = E[2i + (l >> 5)]
// [32 nb + (l & 31)] (the rows' 128-B halves). The products accumulate inside the matrix
// core, so the sums are not in the LDS / register walks' order (within fp32 rounding of
// them; tests/test_gpu_kernels.py) — the same result for every run and launch shape.
typedef float pnnf32x16 __attribute__((ext_vector_type(16)));

template <typename IdxT>
__global__ __launch_bounds__(256) void ipnn_backward_mfma(const IdxT* __restrict__ idx,
                                                          int64_t B, int F, int K, int64_t V,
                                                          const float* __restrict__ emb,
                                                          const float* __restrict__ dcat,
                                                          int64_t ldd,
                                                          float* __restrict__ dslot) {
  const int wave = threadIdx.x / kWave;
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t b = (int64_t)blockIdx.x * (blockDim.x / kWave) + wave;
  if (b >= B) return;  // wave-uniform
  const float* db = dcat + b * ldd;
  const float* dp = db + (int64_t)F * K;
  const long long my_row = lane < F ? (long long)load_row(idx, b * F + lane, V, (int32_t*)nullptr)
                                    : 0ll;
  const int f = lane & 31, kk = lane >> 5;
  // A fragments: D[f][j], j = 2i + kk (the pair (min, max) in row-major order; 0 on the
  // diagonal and past F)
  float a[16];
  long long rj[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int j = 2 * i + kk;
    const int lo = f < j ? f : j, hi = f < j ? j : f;
    const bool on = f < F && j < F && f != j;
    a[i] = on ? dp[lo * (2 * F - lo - 1) / 2 + (hi - lo - 1)] : 0.f;
    rj[i] = __shfl(my_row, j < F ? j : 0, kWave);
  }
  float* out = dslot + b * (int64_t)F * K;
  for (int nb = 0; nb < K / 32; ++nb) {
    const int n = 32 * nb + f;
    pnnf32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = (r & 3) + 8 * (r >> 2) + 4 * kk;
      acc[r] = row < F ? db[(int64_t)row * K + n] : 0.f;
    }
    float e[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int j = 2 * i + kk;
      e[i] = j < F ? emb[rj[i] * K + n] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], e[i], acc, 0, 0, 0);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = (r & 3) + 8 * (r >> 2) + 4 * kk;
      if (row < F) out[(int64_t)row * K + n] = acc[r];
    }
  }
}

}  // namespace ctr

using namespace ctr;

// Default: the matrix-core product where F <= 32 and K % 32 == 0 (40.7 us at the C3 IPNN
// shape against 53.8 for the scalar-operand walk, profiles/r04_ipnn_bwd.txt), else the
// scalar-operand walk for F = 26 / 22 (K <= 64), the register walk where F <= 32 and K <= 64
// (one column per lane), the LDS-tile kernel beyond. CTR_IPNN_BWD=lds / reg / sreg / m forces
// one (A/B runs and the tests: the three walks are bitwise one another, the product within
// fp32 rounding of them).
template <typename IdxT>
static bool launch_ipnn_backward_reg(const IdxT* idx, int64_t B, int F, int K, int64_t V,
                                     const float* emb, const float* dcat, int64_t ldd,
                                     float* dslot, hipStream_t st) {
  const char* env = getenv("CTR_IPNN_BWD");
  const char e = env ? env[0] : '\0';
  const unsigned grid = (unsigned)ceil_div(B, 4);
  if ((e == '\0' || e == 'm') && F <= 32 && K % 32 == 0) {  // the matrix-core product
    hipLaunchKernelGGL((ipnn_backward_mfma<IdxT>), grid, 256, 0, st, idx, B, F, K, V, emb, dcat,
                       ldd, dslot);
    return true;
  }
  if (e == 'l' || F > 32 || K > 64) return false;
  if (e != 'r') {  // the scalar-operand walk
    if (F == 26) {
      hipLaunchKernelGGL((ipnn_backward_sreg<IdxT, 26>), grid, 256, 0, st, idx, B, K, V, emb,
                         dcat, ldd, dslot);
      return true;
    }
    if (F == 22) {
      hipLaunchKernelGGL((ipnn_backward_sreg<IdxT, 22>), grid, 256, 0, st, idx, B, K, V, emb,
                         dcat, ldd, dslot);
      return true;
    }
  }
  constexpr int FM = 32;
  hipLaunchKernelGGL((ipnn_backward_reg<IdxT, FM, 1>), (unsigned)ceil_div(B, 4), 256,
                     4 * (FM * (FM - 1) / 2) * sizeof(float), st, idx, B, F, K, V, emb, dcat,
                     ldd, dslot);
  return true;
}

static int ipnn_check(const void* idx, int idx_type, int64_t B, int F, int K, int64_t V,
                      size_t per_wave_floats) {
  CTR_REQUIRE(idx, "ipnn: null ids");
  CTR_REQUIRE(B >= 0 && F > 1 && K > 0 && V > 0, "ipnn: bad sizes");
  CTR_REQUIRE(idx_type == CTR_IDX_I32 || idx_type == CTR_IDX_I64, "bad idx_type %d", idx_type);
  CTR_REQUIRE(4 * per_wave_floats * sizeof(float) <= 160 * 1024, "ipnn: F*K too large for LDS");
  return CTR_OK;
}

extern "C" int ctr_ipnn_forward_planes(const void* idx, int idx_type, int64_t B, int F, int K,
                                       int64_t V, const float* emb, float* cat, int64_t ldc,
                                       const ctr_planes* cat_planes, int32_t* err_flag,
                                       ctr_stream_t stream) {
  const size_t per_wave = (size_t)F * (K % 4 == 0 ? K + 4 : K + 1);
  int rc = ipnn_check(idx, idx_type, B, F, K, V, per_wave);
  if (rc != CTR_OK) return rc;
  const int64_t W = (int64_t)F * K + F * (F - 1) / 2;
  CTR_REQUIRE(emb && (cat || cat_planes) && (!cat || ldc >= W),
              "ctr_ipnn_forward: bad output");
  CTR_REQUIRE(!cat_planes || (cat_planes->data && cat_planes->rows >= B && cat_planes->cols >= W &&
                              cat_planes->ld >= W && (uintptr_t)cat_planes->data % 8 == 0 &&
                              cat_planes->plane_stride >= cat_planes->rows * cat_planes->ld),
              "ctr_ipnn_forward_planes: planes smaller than cat [B, %lld]", (long long)W);
  if (B == 0) return CTR_OK;
  uint16_t* xpl = cat_planes ? static_cast<uint16_t*>(cat_planes->data) : nullptr;
  const int64_t xld = cat_planes ? cat_planes->ld : 0;
  const int64_t xps = cat_planes ? cat_planes->plane_stride : 0;
  const size_t lds = 4 * per_wave * sizeof(float);
  const unsigned grid = (unsigned)ceil_div(B, 4);
  hipStream_t st = as_stream(stream);
  if (idx_type == CTR_IDX_I64)
    hipLaunchKernelGGL(ipnn_forward_kernel<int64_t>, grid, 256, lds, st,
                       static_cast<const int64_t*>(idx), B, F, K, V, emb, cat, ldc, err_flag,
                       xpl, xld, xps);
  else
    hipLaunchKernelGGL(ipnn_forward_kernel<int32_t>, grid, 256, lds, st,
                       static_cast<const int32_t*>(idx), B, F, K, V, emb, cat, ldc, err_flag,
                       xpl, xld, xps);
  CTR_LAUNCH_CHECK("ctr_ipnn_forward");
  return CTR_OK;
}

extern "C" int ctr_ipnn_forward(const void* idx, int idx_type, int64_t B, int F, int K,
                                int64_t V, const float* emb, float* cat, int64_t ldc,
                                int32_t* err_flag, ctr_stream_t stream) {
  CTR_REQUIRE(cat, "ctr_ipnn_forward: null output");
  return ctr_ipnn_forward_planes(idx, idx_type, B, F, K, V, emb, cat, ldc, nullptr, err_flag,
                                 stream);
}

extern "C" int ctr_ipnn_backward(const void* idx, int idx_type, int64_t B, int F, int K,
                                 int64_t V, const float* emb, const float* dcat, int64_t ldd,
                                 float* dslot, ctr_stream_t stream) {
  const size_t per_wave = (size_t)F * (K + 1) + (size_t)F * (F - 1) / 2;
  int rc = ipnn_check(idx, idx_type, B, F, K, V, per_wave);
  if (rc != CTR_OK) return rc;
  CTR_REQUIRE(emb && dcat && dslot && ldd >= (int64_t)F * K + F * (F - 1) / 2,
              "ctr_ipnn_backward: bad arguments");
  if (B == 0) return CTR_OK;
  const size_t lds = 4 * per_wave * sizeof(float);
  const unsigned grid = (unsigned)ceil_div(B, 4);
  hipStream_t st = as_stream(stream);
  const bool reg = idx_type == CTR_IDX_I64
      ? launch_ipnn_backward_reg(static_cast<const int64_t*>(idx), B, F, K, V, emb, dcat, ldd,
                                 dslot, st)
      : launch_ipnn_backward_reg(static_cast<const int32_t*>(idx), B, F, K, V, emb, dcat, ldd,
                                 dslot, st);
  if (!reg) {
    if (idx_type == CTR_IDX_I64)
      hipLaunchKernelGGL(ipnn_backward_kernel<int64_t>, grid, 256, lds, st,
                         static_cast<const int64_t*>(idx), B, F, K, V, emb, dcat, ldd, dslot);
    else
      hipLaunchKernelGGL(ipnn_backward_kernel<int32_t>, grid, 256, lds, st,
                         static_cast<const int32_t*>(idx), B, F, K, V, emb, dcat, ldd, dslot);
  }
  CTR_LAUNCH_CHECK("ctr_ipnn_backward");
  return CTR_OK;
}

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

template <typename IdxT>
__global__ __launch_bounds__(256) void ipnn_forward_kernel(const IdxT* __restrict__ idx,
                                                           int64_t B, int F, int K, int64_t V,
                                                           const float* __restrict__ emb,
                                                           float* __restrict__ cat, int64_t ldc,
                                                           int32_t* err) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int wave = threadIdx.x / kWave;
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t b = (int64_t)blockIdx.x * (blockDim.x / kWave) + wave;
  if (b >= B) return;  // wave-uniform; the tile is wave-private (no block barrier)
  const int ld = K + 1;
  float* tile = lds + (int64_t)wave * F * ld;
  float* ob = cat + b * ldc;
  stage_rows_wave(idx, b, F, K, V, emb, tile, ld, ob, err, lane);
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS stores are done
  __builtin_amdgcn_wave_barrier();
  const int P = F * (F - 1) / 2;
  float* op = ob + (int64_t)F * K;
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
      for (int k = 0; k < K; ++k) acc += ei[k] * ej[k];  // torch.mul, then torch.sum
    }
    op[p] = acc;
    rem += kWave;
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

}  // namespace ctr

using namespace ctr;

static int ipnn_check(const void* idx, int idx_type, int64_t B, int F, int K, int64_t V,
                      size_t per_wave_floats) {
  CTR_REQUIRE(idx, "ipnn: null ids");
  CTR_REQUIRE(B >= 0 && F > 1 && K > 0 && V > 0, "ipnn: bad sizes");
  CTR_REQUIRE(idx_type == CTR_IDX_I32 || idx_type == CTR_IDX_I64, "bad idx_type %d", idx_type);
  CTR_REQUIRE(4 * per_wave_floats * sizeof(float) <= 160 * 1024, "ipnn: F*K too large for LDS");
  return CTR_OK;
}

extern "C" int ctr_ipnn_forward(const void* idx, int idx_type, int64_t B, int F, int K,
                                int64_t V, const float* emb, float* cat, int64_t ldc,
                                int32_t* err_flag, ctr_stream_t stream) {
  const size_t per_wave = (size_t)F * (K + 1);
  int rc = ipnn_check(idx, idx_type, B, F, K, V, per_wave);
  if (rc != CTR_OK) return rc;
  CTR_REQUIRE(emb && cat && ldc >= (int64_t)F * K + F * (F - 1) / 2,
              "ctr_ipnn_forward: bad output");
  if (B == 0) return CTR_OK;
  const size_t lds = 4 * per_wave * sizeof(float);
  const unsigned grid = (unsigned)ceil_div(B, 4);
  hipStream_t st = as_stream(stream);
  if (idx_type == CTR_IDX_I64)
    hipLaunchKernelGGL(ipnn_forward_kernel<int64_t>, grid, 256, lds, st,
                       static_cast<const int64_t*>(idx), B, F, K, V, emb, cat, ldc, err_flag);
  else
    hipLaunchKernelGGL(ipnn_forward_kernel<int32_t>, grid, 256, lds, st,
                       static_cast<const int32_t*>(idx), B, F, K, V, emb, cat, ldc, err_flag);
  CTR_LAUNCH_CHECK("ctr_ipnn_forward");
  return CTR_OK;
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
  if (idx_type == CTR_IDX_I64)
    hipLaunchKernelGGL(ipnn_backward_kernel<int64_t>, grid, 256, lds, st,
                       static_cast<const int64_t*>(idx), B, F, K, V, emb, dcat, ldd, dslot);
  else
    hipLaunchKernelGGL(ipnn_backward_kernel<int32_t>, grid, 256, lds, st,
                       static_cast<const int32_t*>(idx), B, F, K, V, emb, dcat, ldd, dslot);
  CTR_LAUNCH_CHECK("ctr_ipnn_backward");
  return CTR_OK;
}

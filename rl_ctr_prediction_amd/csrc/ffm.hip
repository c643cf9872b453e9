// Field-aware FM (FFM): p_model.FFM (reference
// src/models/p_model.py:59-100). F embedding tables E_t [V, K] (one per field t); for a
// pair of fields i < j the interaction is E_j[x_i] . E_i[x_j] (the embedding of feature x_i
// in the table of field j, times that of x_j in the table of field i, line 91):
//
//   z = bias + sum_f w[x_f] + sum_k sum_{i<j} E_j[x_i, k] * E_i[x_j, k]          (line 97)
//
// Forward: one wave per example; with G = 64 / K pair groups per wave, lane (g, k) sums the
// products of pairs g, g+G, ... at column k (each load a coalesced K-float run), then lane 0
// adds the G partials of each column and the K columns (pairs first, then k, as line 97). The BCE head (the reference's unfused sigmoid + BCELoss
// gradient, ctr_common.h) is fused when labels are given.
//
// Backward: the gradient of table t at row x_bf (t != f) from pair (f, t) is
//   g_b * E_f[x_bt]
// — F(F-1) row gradients per example, written as (key, row) pairs with key = t*V + x_bf,
// position (b*F + f)*(F-1) + t' (t' = t minus one past f), so a stable sort of the keys
// keeps each row's contributions in slot order (embedding_dense_backward's order); the
// per-row sums then go through the ordinary sparse plan + segmented sum over the F*V-row
// key space. Tables are passed as a device array of F row pointers: the module's F
// nn.Embedding weights stay separate Parameters (state_dict unchanged).
#include "ctr_common.h"

namespace ctr {

template <typename IdxT>
__global__ __launch_bounds__(256) void ffm_forward_kernel(
    const IdxT* __restrict__ idx, int64_t B, int F, int K, int64_t V,
    const float* const* __restrict__ tabs, const float* __restrict__ lin,
    const float* __restrict__ bias, float* __restrict__ z, const float* __restrict__ labels,
    float mean_div, float* __restrict__ p, float* __restrict__ loss, float* __restrict__ gz,
    int32_t* err) {
  __shared__ float s_part[4][kWave];
  const int wave = threadIdx.x / kWave;
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t b = (int64_t)blockIdx.x * (blockDim.x / kWave) + wave;
  if (b >= B) return;  // wave-uniform; s_part is wave-private
  const int G = kWave / K;  // pair groups (K <= 64); lanes past G*K idle
  const int g = lane / K, k = lane % K;
  const int P = F * (F - 1) / 2;
  float acc = 0.f;
  int i = 0, rem = g;
  for (int q = g; g < G && q < P; q += G) {
    while (rem >= F - 1 - i) {
      rem -= F - 1 - i;
      ++i;
    }
    const int j = i + 1 + rem;
    const int64_t xi = load_row(idx, b * F + i, V, err);
    const int64_t xj = load_row(idx, b * F + j, V, err);
    const float a = tabs[j][xi * K + k], c = tabs[i][xj * K + k];
    {
#pragma clang fp contract(off)
      acc += a * c;  // torch.mul, then the sums over pairs and k
    }
    rem += G;
  }
  // per column k the pair groups' partials, then the K columns (the reference's order:
  // sum over pairs, then over k)
  s_part[wave][lane] = acc;
  __builtin_amdgcn_s_waitcnt(0xc07f);
  __builtin_amdgcn_wave_barrier();
  if (lane == 0) {
    acc = 0.f;
    for (int kk = 0; kk < K; ++kk) {
      float col = 0.f;
      for (int gg = 0; gg < G; ++gg) col += s_part[wave][gg * K + kk];
      acc += col;
    }
    float s = 0.f;
    for (int f = 0; f < F; ++f) s += lin[load_row(idx, b * F + f, V, err)];
    const float zz = (bias[0] + s) + acc;
    z[b] = zz;
    if (labels) {
      float pp, ll, gg;
      bce_sigmoid_head(zz, labels[b], mean_div, pp, ll, gg);
      if (p) p[b] = pp;
      loss[b] = ll;
      gz[b] = gg;
    } else if (p) {
      p[b] = sigmoidf_ref(zz);
    }
  }
}

// one thread per (position, column): position = (b*F + f)*(F-1) + t'
template <typename IdxT>
__global__ __launch_bounds__(256) void ffm_backward_kernel(
    const IdxT* __restrict__ idx, int64_t B, int F, int K, int64_t V,
    const float* const* __restrict__ tabs, const float* __restrict__ gz,
    int32_t* __restrict__ keys, float* __restrict__ vals) {
  const int64_t per_ex = (int64_t)F * (F - 1);
  const int64_t total = B * per_ex * K;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t pos = e / K;
    const int k = (int)(e - pos * K);
    const int64_t b = pos / per_ex;
    const int r = (int)(pos - b * per_ex);
    const int f = r / (F - 1), tp = r - f * (F - 1);
    const int t = tp < f ? tp : tp + 1;
    const int64_t xf = load_row(idx, b * F + f, V, nullptr);
    const int64_t xt = load_row(idx, b * F + t, V, nullptr);
    vals[e] = gz[b] * tabs[f][xt * K + k];
    if (k == 0) keys[pos] = (int32_t)(t * V + xf);
  }
}

// the keys alone (the fused trainer's catch-up runs before the forward): same positions
template <typename IdxT>
__global__ __launch_bounds__(256) void ffm_keys_kernel(const IdxT* __restrict__ idx, int64_t B,
                                                       int F, int64_t V,
                                                       int32_t* __restrict__ keys,
                                                       int32_t* err) {
  const int64_t per_ex = (int64_t)F * (F - 1);
  const int64_t total = B * per_ex;
  for (int64_t pos = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; pos < total;
       pos += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = pos / per_ex;
    const int r = (int)(pos - b * per_ex);
    const int f = r / (F - 1), tp = r - f * (F - 1);
    const int t = tp < f ? tp : tp + 1;
    keys[pos] = (int32_t)(t * V + load_row(idx, b * F + f, V, err));
  }
}

}  // namespace ctr

using namespace ctr;

static int ffm_check(const void* idx, int idx_type, int64_t B, int F, int K, int64_t V,
                     const float* const* tabs) {
  CTR_REQUIRE(idx && tabs, "ffm: null pointer");
  CTR_REQUIRE(B >= 0 && F > 1 && V > 0, "ffm: bad sizes");
  CTR_REQUIRE(K >= 1 && K <= kWave, "ffm: K must be in [1, 64]");
  CTR_REQUIRE((int64_t)F * V < (int64_t(1) << 31), "ffm: F*V must fit int32 keys");
  CTR_REQUIRE(idx_type == CTR_IDX_I32 || idx_type == CTR_IDX_I64, "bad idx_type %d", idx_type);
  return CTR_OK;
}

extern "C" int ctr_ffm_forward(const void* idx, int idx_type, int64_t B, int F, int K, int64_t V,
                               const float* const* tables, const float* lin, const float* bias,
                               float* z, const float* labels, float mean_div, float* p,
                               float* loss_elem, float* gz, int32_t* err_flag,
                               ctr_stream_t stream) {
  int rc = ffm_check(idx, idx_type, B, F, K, V, tables);
  if (rc != CTR_OK) return rc;
  CTR_REQUIRE(lin && bias && z, "ctr_ffm_forward: null pointer");
  CTR_REQUIRE(!labels || (loss_elem && gz && mean_div > 0.f), "ctr_ffm_forward: labels need "
              "loss_elem, gz and mean_div > 0");
  if (B == 0) return CTR_OK;
  const unsigned grid = (unsigned)ceil_div(B, 4);
  hipStream_t st = as_stream(stream);
  if (idx_type == CTR_IDX_I64)
    hipLaunchKernelGGL(ffm_forward_kernel<int64_t>, grid, 256, 0, st,
                       static_cast<const int64_t*>(idx), B, F, K, V, tables, lin, bias, z, labels,
                       mean_div, p, loss_elem, gz, err_flag);
  else
    hipLaunchKernelGGL(ffm_forward_kernel<int32_t>, grid, 256, 0, st,
                       static_cast<const int32_t*>(idx), B, F, K, V, tables, lin, bias, z, labels,
                       mean_div, p, loss_elem, gz, err_flag);
  CTR_LAUNCH_CHECK("ctr_ffm_forward");
  return CTR_OK;
}

extern "C" int ctr_ffm_backward(const void* idx, int idx_type, int64_t B, int F, int K,
                                int64_t V, const float* const* tables, const float* gz,
                                int32_t* keys, float* vals, ctr_stream_t stream) {
  int rc = ffm_check(idx, idx_type, B, F, K, V, tables);
  if (rc != CTR_OK) return rc;
  CTR_REQUIRE(gz && keys && vals, "ctr_ffm_backward: null pointer");
  if (B == 0) return CTR_OK;
  const int64_t total = B * F * (int64_t)(F - 1) * K;
  const unsigned grid = (unsigned)std::min<int64_t>(ceil_div(total, 256), 16384);
  hipStream_t st = as_stream(stream);
  if (idx_type == CTR_IDX_I64)
    hipLaunchKernelGGL(ffm_backward_kernel<int64_t>, grid, 256, 0, st,
                       static_cast<const int64_t*>(idx), B, F, K, V, tables, gz, keys, vals);
  else
    hipLaunchKernelGGL(ffm_backward_kernel<int32_t>, grid, 256, 0, st,
                       static_cast<const int32_t*>(idx), B, F, K, V, tables, gz, keys, vals);
  CTR_LAUNCH_CHECK("ctr_ffm_backward");
  return CTR_OK;
}

extern "C" int ctr_ffm_keys(const void* idx, int idx_type, int64_t B, int F, int64_t V,
                            int32_t* keys, int32_t* err_flag, ctr_stream_t stream) {
  CTR_REQUIRE(idx && keys && B >= 0 && F > 1 && V > 0, "ctr_ffm_keys: bad arguments");
  CTR_REQUIRE((int64_t)F * V < (int64_t(1) << 31), "ctr_ffm_keys: F*V must fit int32 keys");
  CTR_REQUIRE(idx_type == CTR_IDX_I32 || idx_type == CTR_IDX_I64, "bad idx_type %d", idx_type);
  if (B == 0) return CTR_OK;
  const int64_t total = B * F * (int64_t)(F - 1);
  const unsigned grid = (unsigned)std::min<int64_t>(ceil_div(total, 256), 16384);
  hipStream_t st = as_stream(stream);
  if (idx_type == CTR_IDX_I64)
    hipLaunchKernelGGL(ffm_keys_kernel<int64_t>, grid, 256, 0, st,
                       static_cast<const int64_t*>(idx), B, F, V, keys, err_flag);
  else
    hipLaunchKernelGGL(ffm_keys_kernel<int32_t>, grid, 256, 0, st,
                       static_cast<const int32_t*>(idx), B, F, V, keys, err_flag);
  CTR_LAUNCH_CHECK("ctr_ffm_keys");
  return CTR_OK;
}

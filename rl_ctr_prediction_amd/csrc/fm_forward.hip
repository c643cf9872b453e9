// Forward kernels of the CTR hot path.
//
// Layout: the embedding table E is [V,K] fp32 row-major (the `feature_embedding.weight`
// parameter itself, no repacking), the linear table w is [V] (`linear.weight` [V,1]),
// a batch is idx [B,F] (int64 from the reference's LongTensor, or int32).
//
// One wave per example. For K % 4 == 0 with (K/4) | 64 a lane owns one float4 column
// c = lane % (K/4) of rows f = lane / (K/4) + j * (64 / (K/4)): a K=64 row is 16 lanes x
// 16 B (one 256-B line), a wave fetches 4 rows per global_load_dwordx4; K=16 fetches 16
// rows per instruction. All F row loads of an example are issued before the first use
// (register staging), the per-k sums over fields are xor-butterflies (ds_bpermute/DPP).
#include "ctr_common.h"

namespace ctr {

// --------------------------------------------------------------------- gather -------
template <typename IdxT>
__global__ __launch_bounds__(256) void gather_rows_vec4(const float4* __restrict__ table,
                                                        int64_t V, int K4,
                                                        const IdxT* __restrict__ idx,
                                                        int64_t n, float4* __restrict__ out,
                                                        int32_t* err) {
  const int64_t total = n * K4;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = t / K4;
    const int c = (int)(t - i * K4);
    const int64_t r = load_row(idx, i, V, err);
    out[t] = table[r * K4 + c];
  }
}

template <typename IdxT>
__global__ __launch_bounds__(256) void gather_rows_scalar(const float* __restrict__ table,
                                                          int64_t V, int K,
                                                          const IdxT* __restrict__ idx,
                                                          int64_t n, float* __restrict__ out,
                                                          int32_t* err) {
  const int64_t total = n * K;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = t / K;
    const int c = (int)(t - i * K);
    const int64_t r = load_row(idx, i, V, err);
    out[t] = table[r * K + c];
  }
}

// ------------------------------------------------------------- FM forward (vec) -----
// K4 = K/4 float4 columns per row, RPI = 64/K4 rows per wave-instruction, MAXIT =
// ceil(FMAX/RPI) register-staged row loads per lane (F <= FMAX).
template <typename IdxT, int K4, int FMAX>
__global__ __launch_bounds__(256) void fm_forward_vec(
    const IdxT* __restrict__ idx, int64_t B, int F, int64_t V, const float4* __restrict__ emb,
    const float* __restrict__ lin, const float* __restrict__ bias, float* __restrict__ z_out,
    float4* __restrict__ sum_out, float4* __restrict__ emb_out, const float* __restrict__ labels,
    float mean_div, float* __restrict__ p_out, float* __restrict__ loss_out,
    float* __restrict__ gz_out, int32_t* err, uint16_t* __restrict__ xpl, int64_t xpl_ld,
    int64_t xpl_ps) {
  constexpr int RPI = kWave / K4;
  constexpr int MAXIT = (FMAX + RPI - 1) / RPI;
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t b = (int64_t)blockIdx.x * (blockDim.x / kWave) + (threadIdx.x / kWave);
  if (b >= B) return;  // wave-uniform
  const int c = lane % K4;
  const int r0 = lane / K4;
  const float yb = labels ? labels[b] : 0.f;  // in flight with the id loads

  // One id per lane (lane f < F), range-checked once, then broadcast by ds_bpermute.
  int my_row = 0;
  float my_w = 0.f;
  if (lane < F) {
    my_row = (int)load_row(idx, b * F + lane, V, err);
    my_w = lin[my_row];
  }

  float4 e[MAXIT];
#pragma unroll
  for (int it = 0; it < MAXIT; ++it) {
    const int f = r0 + it * RPI;
    const int row = __shfl(my_row, f < F ? f : 0, kWave);
    e[it] = (f < F) ? emb[(int64_t)row * K4 + c] : make_float4(0.f, 0.f, 0.f, 0.f);
  }

  float4 s = make_float4(0.f, 0.f, 0.f, 0.f), q = s;
#pragma unroll
  for (int it = 0; it < MAXIT; ++it) {
    const int f = r0 + it * RPI;
    if (f < F) {
      s.x += e[it].x; s.y += e[it].y; s.z += e[it].z; s.w += e[it].w;
      q.x += e[it].x * e[it].x; q.y += e[it].y * e[it].y;
      q.z += e[it].z * e[it].z; q.w += e[it].w * e[it].w;
      if (emb_out) emb_out[(b * F + f) * K4 + c] = e[it];
      // DeepFM's MLP input as its three bf16 planes (csrc/gemm_planes.hip's operand)
      if (xpl) store_planes4_at(xpl + b * xpl_ld + (int64_t)f * (4 * K4) + 4 * c, xpl_ps, e[it]);
    }
  }
  // Sum over the RPI lanes that share column c (lanes c, c+K4, c+2*K4, ...).
  s.x = xor_reduce_from<K4>(s.x); s.y = xor_reduce_from<K4>(s.y);
  s.z = xor_reduce_from<K4>(s.z); s.w = xor_reduce_from<K4>(s.w);
  q.x = xor_reduce_from<K4>(q.x); q.y = xor_reduce_from<K4>(q.y);
  q.z = xor_reduce_from<K4>(q.z); q.w = xor_reduce_from<K4>(q.w);

  if (sum_out && lane < K4) sum_out[b * K4 + c] = s;

  // ix = sum_k (square_of_sum_k - sum_of_square_k), p_model.py:49-52.
  float t = (s.x * s.x - q.x) + (s.y * s.y - q.y) + (s.z * s.z - q.z) + (s.w * s.w - q.w);
#pragma unroll
  for (int o = 1; o < K4; o <<= 1) t += __shfl_xor(t, o, kWave);
  const float lin_sum = wave_sum(my_w);

  if (lane == 0) {
    const float z = (bias[0] + lin_sum) + t * 0.5f;  // p_model.py:54
    if (z_out) z_out[b] = z;
    if (labels) {
      float p, l, g;
      bce_sigmoid_head(z, yb, mean_div, p, l, g);
      if (p_out) p_out[b] = p;
      if (loss_out) loss_out[b] = l;
      if (gz_out) gz_out[b] = g;
    } else if (p_out) {
      p_out[b] = sigmoidf_ref(z);
    }
  }
}

// ---------------------------------------------------------- FM forward (generic) ----
// Any K, any F (e.g. the driver's default latent_dims=10): lanes over k, loop over f.
template <typename IdxT>
__global__ __launch_bounds__(256) void fm_forward_generic(
    const IdxT* __restrict__ idx, int64_t B, int F, int K, int64_t V,
    const float* __restrict__ emb, const float* __restrict__ lin, const float* __restrict__ bias,
    float* __restrict__ z_out, float* __restrict__ sum_out, float* __restrict__ emb_out,
    const float* __restrict__ labels, float mean_div, float* __restrict__ p_out,
    float* __restrict__ loss_out, float* __restrict__ gz_out, int32_t* err) {
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t b = (int64_t)blockIdx.x * (blockDim.x / kWave) + (threadIdx.x / kWave);
  if (b >= B) return;
  float ix_part = 0.f;
  for (int k0 = 0; k0 < K; k0 += kWave) {
    const int k = k0 + lane;
    float s = 0.f, q = 0.f;
    for (int f = 0; f < F; ++f) {
      const int64_t row = load_row(idx, b * F + f, V, err);
      if (k < K) {
        const float e = emb[row * K + k];
        s += e;
        q += e * e;
        if (emb_out) emb_out[(b * F + f) * K + k] = e;
      }
    }
    if (k < K) {
      ix_part += s * s - q;
      if (sum_out) sum_out[b * K + k] = s;
    }
  }
  const float ix = wave_sum(ix_part);
  float w = 0.f;
  for (int f = lane; f < F; f += kWave) w += lin[load_row(idx, b * F + f, V, err)];
  const float lin_sum = wave_sum(w);
  if (lane == 0) {
    const float z = (bias[0] + lin_sum) + ix * 0.5f;
    if (z_out) z_out[b] = z;
    if (labels) {
      float p, l, g;
      bce_sigmoid_head(z, labels[b], mean_div, p, l, g);
      if (p_out) p_out[b] = p;
      if (loss_out) loss_out[b] = l;
      if (gz_out) gz_out[b] = g;
    } else if (p_out) {
      p_out[b] = sigmoidf_ref(z);
    }
  }
}

// ------------------------------------------------------------------ BCE head -------
__global__ __launch_bounds__(256) void bce_sigmoid_kernel(const float* __restrict__ z,
                                                          const float* __restrict__ y, int64_t B,
                                                          float mean_div, float* p_out,
                                                          float* loss_out, float* gz_out) {
  for (int64_t b = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; b < B;
       b += (int64_t)gridDim.x * blockDim.x) {
    float p, l, g;
    bce_sigmoid_head(z[b], y[b], mean_div, p, l, g);
    if (p_out) p_out[b] = p;
    if (loss_out) loss_out[b] = l;
    if (gz_out) gz_out[b] = g;
  }
}

// ------------------------------------------------------------- DeepFM out head ------
// One wave per example: the 200-wide Linear(200,1) dot, the sum with the FM logit, the
// BCE head, and the gradient into the last hidden layer through Dropout and ReLU.
__global__ __launch_bounds__(256) void deepfm_head_kernel(
    const float* __restrict__ h, int64_t B, int H, const float* __restrict__ w,
    const float* __restrict__ bo, const float* __restrict__ z_fm, const float* __restrict__ y,
    float mean_div, float drop_scale, float* z_out, float* p_out, float* loss_out,
    float* gz_out, float* __restrict__ dh_pre, uint16_t* __restrict__ dpl, int64_t dpl_ld,
    int64_t dpl_ps) {
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t b = (int64_t)blockIdx.x * (blockDim.x / kWave) + (threadIdx.x / kWave);
  if (b >= B) return;
  const float* hb = h + b * H;
  const float zfm = z_fm[b], yb = y ? y[b] : 0.f;  // in flight with the row loads
  // H <= 256 (the reference's 200): the lane's <= 4 h / w values loaded together and kept for
  // the gradient below (a loop with a load -> use chain per 64 columns was ~4 dependent
  // memory round trips per example: 11.4 us at C3 for 6.5 MB); the same sums in the same order
  constexpr int kMaxJ = 4;
  const bool held = H <= kMaxJ * kWave;
  float hv[kMaxJ], wv[kMaxJ];
  float part = 0.f;
  if (held) {
#pragma unroll
    for (int q = 0; q < kMaxJ; ++q) {
      const int j = lane + q * kWave;
      hv[q] = j < H ? hb[j] : 0.f;
      wv[q] = j < H ? w[j] : 0.f;
    }
#pragma unroll
    for (int q = 0; q < kMaxJ; ++q)
      if (lane + q * kWave < H) part += hv[q] * wv[q];
  } else {
    for (int j = lane; j < H; j += kWave) part += hb[j] * w[j];
  }
  const float dot = wave_sum(part);
  const float z = zfm + (dot + bo[0]);  // p_model.py:322 (to_fm(x) + mlp(...))
  float p, l, g;
  if (y) {
    bce_sigmoid_head(z, yb, mean_div, p, l, g);
  } else {
    p = sigmoidf_ref(z);
    l = 0.f;
    g = 0.f;
  }
  if (lane == 0) {
    if (z_out) z_out[b] = z;
    if (p_out) p_out[b] = p;
    if (loss_out && y) loss_out[b] = l;
    if (gz_out && y) gz_out[b] = g;
  }
  if ((dh_pre || dpl) && y) {  // dh_pre NULL: the planes only (no reader of the fp32 copy)
    float* d = dh_pre ? dh_pre + b * H : nullptr;
    auto put = [&](int j, float hj, float wj) {
      const float v = hj > 0.f ? (g * wj) * drop_scale : 0.f;
      if (d) d[j] = v;
      if (dpl) {  // dH2's planes for the dH1 / dW1 GEMMs (csrc/gemm_planes.hip)
        uint16_t h3[3];
        psplit1(v, h3);
#pragma unroll
        for (int p = 0; p < 3; ++p) dpl[p * dpl_ps + b * dpl_ld + j] = h3[p];
      }
    };
    if (held) {
#pragma unroll
      for (int q = 0; q < kMaxJ; ++q)
        if (lane + q * kWave < H) put(lane + q * kWave, hv[q], wv[q]);
    } else {
      for (int j = lane; j < H; j += kWave) put(j, hb[j], w[j]);
    }
  }
}

// --------------------------------------------------------- Feature_Embedding (A7) ---
// Wave per example; the F rows are staged in LDS (stage_rows_wave: all F*K loads in
// flight at once) with a +1 float row pad so that the 64 lanes (each on a different (i,j)
// pair) reading column k of rows i and j hit different banks; the flat rows go straight
// to the output.
template <typename IdxT>
__global__ __launch_bounds__(256) void feature_embedding_kernel(
    const IdxT* __restrict__ idx, int64_t B, int F, int K, int64_t V,
    const float* __restrict__ emb, float* __restrict__ out, int32_t* err,
    uint16_t* __restrict__ xpl = nullptr, int64_t xpl_ld = 0, int64_t xpl_ps = 0) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int wave = threadIdx.x / kWave;
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t b = (int64_t)blockIdx.x * (blockDim.x / kWave) + wave;
  if (b >= B) return;  // wave-uniform; the tile is wave-private (no block barrier)
  const int ld = K + 1;
  float* tile = lds + (int64_t)wave * F * ld;
  const int P = F * (F - 1) / 2;
  const int64_t width = (int64_t)P + (int64_t)F * K;
  float* ob = out + b * width;
  stage_rows_wave(idx, b, F, K, V, emb, tile, ld, ob + P, err, lane);
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS stores are done
  __builtin_amdgcn_wave_barrier();
  // row-major pair order of Feature_embedding.py:40-43: (0,1),(0,2)...(0,F-1),(1,2)...;
  // lane -> pairs p = lane, lane + 64, ...; (i, j) walked incrementally
  int i = 0, rem = lane;
  for (int p = lane; p < P; p += kWave, rem += kWave) {
    while (rem >= F - 1 - i) {
      rem -= F - 1 - i;
      ++i;
    }
    const int j = i + 1 + rem;
    const float* ei = tile + i * ld;
    const float* ej = tile + j * ld;
    float acc = 0.f;
    for (int k = 0; k < K; ++k) acc += ei[k] * ej[k];
    ob[p] = acc;
    if (xpl) {
      uint16_t h3[3];
      psplit1(acc, h3);
#pragma unroll
      for (int q = 0; q < 3; ++q) xpl[q * xpl_ps + b * xpl_ld + p] = h3[q];
    }
  }
  if (xpl) {  // the flat part's planes (columns P ..), from the staged tile
    for (int t = lane; t < F * K; t += kWave) {
      const int f = t / K, k = t - f * K;
      uint16_t h3[3];
      psplit1(tile[f * ld + k], h3);
#pragma unroll
      for (int q = 0; q < 3; ++q) xpl[q * xpl_ps + b * xpl_ld + P + t] = h3[q];
    }
  }
}

template <typename IdxT>
static int launch_fm_forward(const IdxT* idx, int64_t B, int F, int K, int64_t V,
                             const float* emb, const float* lin, const float* bias, float* z,
                             float* sum_e, float* emb_out, const float* labels, float mean_div,
                             float* p, float* loss, float* gz, int32_t* err, hipStream_t st,
                             const ctr_planes* xpl = nullptr) {
  const int waves_per_block = 4;
  const dim3 grid((unsigned)ceil_div(B, waves_per_block)), block(256);
  const bool vec_ok = (K % 4 == 0) && (kWave % (K / 4) == 0) && F <= 64 &&
                      (reinterpret_cast<uintptr_t>(emb) % 16 == 0) &&
                      (!sum_e || reinterpret_cast<uintptr_t>(sum_e) % 16 == 0) &&
                      (!emb_out || reinterpret_cast<uintptr_t>(emb_out) % 16 == 0);
#define CTR_FM_VEC(K4_, FMAX_)                                                              \
  hipLaunchKernelGGL((fm_forward_vec<IdxT, K4_, FMAX_>), grid, block, 0, st, idx, B, F, V,  \
                     reinterpret_cast<const float4*>(emb), lin, bias, z,                    \
                     reinterpret_cast<float4*>(sum_e), reinterpret_cast<float4*>(emb_out),  \
                     labels, mean_div, p, loss, gz, err,                                    \
                     xpl ? static_cast<uint16_t*>(xpl->data) : nullptr, xpl ? xpl->ld : 0,  \
                     xpl ? xpl->plane_stride : 0)
  if (vec_ok) {
    const int K4 = K / 4;
    const bool f32 = F <= 32;
    switch (K4) {
      case 1: if (f32) CTR_FM_VEC(1, 32); else CTR_FM_VEC(1, 64); break;
      case 2: if (f32) CTR_FM_VEC(2, 32); else CTR_FM_VEC(2, 64); break;
      case 4: if (f32) CTR_FM_VEC(4, 32); else CTR_FM_VEC(4, 64); break;
      case 8: if (f32) CTR_FM_VEC(8, 32); else CTR_FM_VEC(8, 64); break;
      case 16: if (f32) CTR_FM_VEC(16, 32); else CTR_FM_VEC(16, 64); break;
      case 32: if (f32) CTR_FM_VEC(32, 32); else CTR_FM_VEC(32, 64); break;
      case 64: if (f32) CTR_FM_VEC(64, 32); else CTR_FM_VEC(64, 64); break;
      default: goto generic;
    }
#undef CTR_FM_VEC
    CTR_LAUNCH_CHECK("fm_forward_vec");
    return CTR_OK;
  }
generic:
  CTR_REQUIRE(!xpl, "ctr_fm_forward_planes: needs K %% 4 == 0, (K/4) | 64, F <= 64, 16-B rows");
  hipLaunchKernelGGL((fm_forward_generic<IdxT>), grid, block, 0, st, idx, B, F, K, V, emb, lin,
                     bias, z, sum_e, emb_out, labels, mean_div, p, loss, gz, err);
  CTR_LAUNCH_CHECK("fm_forward_generic");
  return CTR_OK;
}

}  // namespace ctr

using namespace ctr;

extern "C" int ctr_embedding_gather(const float* table, int64_t V, int K, const void* idx,
                                    int idx_type, int64_t n, float* out, int32_t* err_flag,
                                    ctr_stream_t stream) {
  CTR_REQUIRE(table && idx && out, "ctr_embedding_gather: null pointer");
  CTR_REQUIRE(V > 0 && K > 0 && n >= 0, "ctr_embedding_gather: bad sizes V=%lld K=%d n=%lld",
              (long long)V, K, (long long)n);
  CTR_REQUIRE(idx_type == CTR_IDX_I32 || idx_type == CTR_IDX_I64, "bad idx_type %d", idx_type);
  if (n == 0) return CTR_OK;
  hipStream_t st = as_stream(stream);
  const bool vec = K % 4 == 0 && reinterpret_cast<uintptr_t>(table) % 16 == 0 &&
                   reinterpret_cast<uintptr_t>(out) % 16 == 0;
  const int64_t total = vec ? n * (K / 4) : n * K;
  const unsigned grid = (unsigned)std::min<int64_t>(ceil_div(total, 256), 8192);
  if (vec) {
    if (idx_type == CTR_IDX_I64)
      hipLaunchKernelGGL(gather_rows_vec4<int64_t>, grid, 256, 0, st,
                         reinterpret_cast<const float4*>(table), V, K / 4,
                         static_cast<const int64_t*>(idx), n, reinterpret_cast<float4*>(out),
                         err_flag);
    else
      hipLaunchKernelGGL(gather_rows_vec4<int32_t>, grid, 256, 0, st,
                         reinterpret_cast<const float4*>(table), V, K / 4,
                         static_cast<const int32_t*>(idx), n, reinterpret_cast<float4*>(out),
                         err_flag);
  } else {
    if (idx_type == CTR_IDX_I64)
      hipLaunchKernelGGL(gather_rows_scalar<int64_t>, grid, 256, 0, st, table, V, K,
                         static_cast<const int64_t*>(idx), n, out, err_flag);
    else
      hipLaunchKernelGGL(gather_rows_scalar<int32_t>, grid, 256, 0, st, table, V, K,
                         static_cast<const int32_t*>(idx), n, out, err_flag);
  }
  CTR_LAUNCH_CHECK("ctr_embedding_gather");
  return CTR_OK;
}

extern "C" int ctr_fm_forward(const void* idx, int idx_type, int64_t B, int F, int K, int64_t V,
                              const float* emb, const float* lin, const float* bias, float* z,
                              float* sum_e, float* emb_out, const float* labels, float mean_div,
                              float* p, float* loss_elem, float* gz, int32_t* err_flag,
                              ctr_stream_t stream) {
  CTR_REQUIRE(idx && emb && lin && bias, "ctr_fm_forward: null input pointer");
  CTR_REQUIRE(B >= 0 && F > 0 && K > 0 && V > 0 && V < (int64_t(1) << 31),
              "ctr_fm_forward: bad sizes B=%lld F=%d K=%d V=%lld", (long long)B, F, K,
              (long long)V);
  CTR_REQUIRE(idx_type == CTR_IDX_I32 || idx_type == CTR_IDX_I64, "bad idx_type %d", idx_type);
  CTR_REQUIRE(!labels || mean_div > 0.f, "ctr_fm_forward: mean_div must be > 0");
  if (B == 0) return CTR_OK;
  hipStream_t st = as_stream(stream);
  if (idx_type == CTR_IDX_I64)
    return launch_fm_forward(static_cast<const int64_t*>(idx), B, F, K, V, emb, lin, bias, z,
                             sum_e, emb_out, labels, mean_div, p, loss_elem, gz, err_flag, st);
  return launch_fm_forward(static_cast<const int32_t*>(idx), B, F, K, V, emb, lin, bias, z,
                           sum_e, emb_out, labels, mean_div, p, loss_elem, gz, err_flag, st);
}

extern "C" int ctr_fm_forward_planes(const void* idx, int idx_type, int64_t B, int F, int K,
                                     int64_t V, const float* emb, const float* lin,
                                     const float* bias, float* z, float* sum_e,
                                     const ctr_planes* emb_planes, int32_t* err_flag,
                                     ctr_stream_t stream) {
  CTR_REQUIRE(idx && emb && lin && bias && emb_planes && emb_planes->data,
              "ctr_fm_forward_planes: null pointer");
  CTR_REQUIRE(B >= 0 && F > 0 && K > 0 && V > 0 && V < (int64_t(1) << 31),
              "ctr_fm_forward_planes: bad sizes");
  CTR_REQUIRE(idx_type == CTR_IDX_I32 || idx_type == CTR_IDX_I64, "bad idx_type %d", idx_type);
  CTR_REQUIRE(emb_planes->rows >= B && emb_planes->cols >= (int64_t)F * K &&
                  emb_planes->ld % 4 == 0 && (uintptr_t)emb_planes->data % 8 == 0,
              "ctr_fm_forward_planes: planes must hold [B, F*K] with 8-B aligned rows");
  if (B == 0) return CTR_OK;
  hipStream_t st = as_stream(stream);
  if (idx_type == CTR_IDX_I64)
    return launch_fm_forward(static_cast<const int64_t*>(idx), B, F, K, V, emb, lin, bias, z,
                             sum_e, nullptr, nullptr, 1.f, nullptr, nullptr, nullptr, err_flag, st,
                             emb_planes);
  return launch_fm_forward(static_cast<const int32_t*>(idx), B, F, K, V, emb, lin, bias, z, sum_e,
                           nullptr, nullptr, 1.f, nullptr, nullptr, nullptr, err_flag, st,
                           emb_planes);
}

extern "C" int ctr_bce_sigmoid(const float* z, const float* labels, int64_t B, float mean_div,
                               float* p, float* loss_elem, float* gz, ctr_stream_t stream) {
  CTR_REQUIRE(z && labels, "ctr_bce_sigmoid: null pointer");
  CTR_REQUIRE(B >= 0 && mean_div > 0.f, "ctr_bce_sigmoid: bad sizes");
  if (B == 0) return CTR_OK;
  const unsigned grid = (unsigned)std::min<int64_t>(ceil_div(B, 256), 4096);
  hipLaunchKernelGGL(bce_sigmoid_kernel, grid, 256, 0, as_stream(stream), z, labels, B, mean_div,
                     p, loss_elem, gz);
  CTR_LAUNCH_CHECK("ctr_bce_sigmoid");
  return CTR_OK;
}

extern "C" int ctr_deepfm_head(const float* h, int64_t B, int H, const float* w_out,
                               const float* b_out, const float* z_fm, const float* labels,
                               float mean_div, float drop_scale, float* z, float* p,
                               float* loss_elem, float* gz, float* dh_pre, ctr_stream_t stream) {
  CTR_REQUIRE(h && w_out && b_out && z_fm, "ctr_deepfm_head: null input pointer");
  CTR_REQUIRE(B >= 0 && H > 0, "ctr_deepfm_head: bad sizes");
  CTR_REQUIRE(!labels || mean_div > 0.f, "ctr_deepfm_head: mean_div must be > 0");
  if (B == 0) return CTR_OK;
  hipLaunchKernelGGL(deepfm_head_kernel, (unsigned)ceil_div(B, 4), 256, 0, as_stream(stream), h,
                     B, H, w_out, b_out, z_fm, labels, mean_div, drop_scale, z, p, loss_elem, gz,
                     dh_pre, nullptr, 0, 0);
  CTR_LAUNCH_CHECK("ctr_deepfm_head");
  return CTR_OK;
}

extern "C" int ctr_deepfm_head_planes(const float* h, int64_t B, int H, const float* w_out,
                                      const float* b_out, const float* z_fm, const float* labels,
                                      float mean_div, float drop_scale, float* z, float* p,
                                      float* loss_elem, float* gz, float* dh_pre,
                                      const ctr_planes* dh_planes, ctr_stream_t stream) {
  CTR_REQUIRE(h && w_out && b_out && z_fm && labels && dh_planes && dh_planes->data,
              "ctr_deepfm_head_planes: null pointer");
  CTR_REQUIRE(B >= 0 && H > 0 && mean_div > 0.f, "ctr_deepfm_head_planes: bad sizes");
  CTR_REQUIRE(dh_planes->rows >= B && dh_planes->cols >= H && dh_planes->ld >= H,
              "ctr_deepfm_head_planes: planes smaller than dh [B, H]");
  if (B == 0) return CTR_OK;
  hipLaunchKernelGGL(deepfm_head_kernel, (unsigned)ceil_div(B, 4), 256, 0, as_stream(stream), h,
                     B, H, w_out, b_out, z_fm, labels, mean_div, drop_scale, z, p, loss_elem, gz,
                     dh_pre, static_cast<uint16_t*>(dh_planes->data), dh_planes->ld,
                     dh_planes->plane_stride);
  CTR_LAUNCH_CHECK("ctr_deepfm_head_planes");
  return CTR_OK;
}

extern "C" int ctr_feature_embedding_forward_planes(const void* idx, int idx_type, int64_t B,
                                                    int F, int K, int64_t V, const float* emb,
                                                    float* out, const ctr_planes* out_planes,
                                                    int32_t* err_flag, ctr_stream_t stream) {
  CTR_REQUIRE(idx && emb && out, "ctr_feature_embedding_forward: null pointer");
  const int64_t W = (int64_t)F * (F - 1) / 2 + (int64_t)F * K;
  CTR_REQUIRE(!out_planes || (out_planes->data && out_planes->rows >= B &&
                              out_planes->cols >= W && out_planes->ld >= W &&
                              out_planes->plane_stride >= out_planes->rows * out_planes->ld),
              "ctr_feature_embedding_forward_planes: planes smaller than the state [B, %lld]",
              (long long)W);
  CTR_REQUIRE(B >= 0 && F > 1 && K > 0 && V > 0, "ctr_feature_embedding_forward: bad sizes");
  CTR_REQUIRE(idx_type == CTR_IDX_I32 || idx_type == CTR_IDX_I64, "bad idx_type %d", idx_type);
  const size_t lds = (size_t)4 * F * (K + 1) * sizeof(float);
  CTR_REQUIRE(lds <= 160 * 1024, "ctr_feature_embedding_forward: F*K too large for LDS");
  if (B == 0) return CTR_OK;
  hipStream_t st = as_stream(stream);
  const unsigned grid = (unsigned)ceil_div(B, 4);
  uint16_t* xpl = out_planes ? static_cast<uint16_t*>(out_planes->data) : nullptr;
  const int64_t xld = out_planes ? out_planes->ld : 0;
  const int64_t xps = out_planes ? out_planes->plane_stride : 0;
  if (idx_type == CTR_IDX_I64)
    hipLaunchKernelGGL(feature_embedding_kernel<int64_t>, grid, 256, lds, st,
                       static_cast<const int64_t*>(idx), B, F, K, V, emb, out, err_flag, xpl,
                       xld, xps);
  else
    hipLaunchKernelGGL(feature_embedding_kernel<int32_t>, grid, 256, lds, st,
                       static_cast<const int32_t*>(idx), B, F, K, V, emb, out, err_flag, xpl,
                       xld, xps);
  CTR_LAUNCH_CHECK("ctr_feature_embedding_forward");
  return CTR_OK;
}

extern "C" int ctr_feature_embedding_forward(const void* idx, int idx_type, int64_t B, int F,
                                             int K, int64_t V, const float* emb, float* out,
                                             int32_t* err_flag, ctr_stream_t stream) {
  return ctr_feature_embedding_forward_planes(idx, idx_type, B, F, K, V, emb, out, nullptr,
                                              err_flag, stream);
}

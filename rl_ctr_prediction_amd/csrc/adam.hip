// Adam with coupled L2 (torch.optim.Adam(lr, weight_decay)) — dense
// semantics: every element of every parameter moves every step, as in the reference
// (nn.Embedding(sparse=False) + Adam). This is the dominant HBM stream of the step:
// per element it reads p, m, v and writes p, m, v (24 B); the embedding gradient is not
// materialised densely — a row's gradient is read from the compact per-row sums only
// when rowmap[row] >= 0, so the dense pass costs 24 B/elem + 4 B/row, not 32 B/elem.
//
// Arithmetic follows torch's single-tensor CPU Adam (torch/optim/adam.py), checked
// against torch 2.10: m and v bit-exact with the FMA forms below; p to <=1 ulp of the
// update (torch's vectorised CPU sqrt is not correctly rounded; ours is).
#include "ctr_common.h"

namespace ctr {

struct AdamHP {
  float neg_step_size;  // -lr / (1 - beta1^t)
  float bc2_sqrt;       // sqrt(1 - beta2^t)
  float w1;             // 1 - beta1   (lerp weight)
  float beta2;
  float w2;             // 1 - beta2   (addcmul value)
  float eps;
  float wd;
};

__device__ __forceinline__ void adam_elem(float& p, float g, float& m, float& v,
                                          const AdamHP& h) {
#pragma clang fp contract(off)
  g = __builtin_fmaf(h.wd, p, g);                 // grad.add(param, alpha=wd)
  m = __builtin_fmaf(h.w1, g - m, m);             // exp_avg.lerp_(grad, 1-beta1)
  v = __builtin_fmaf(h.w2 * g, g, v * h.beta2);   // exp_avg_sq.mul_(b2).addcmul_(g, g, 1-b2)
  const float denom = sqrtf(v) / h.bc2_sqrt + h.eps;  // (v.sqrt() / bc2_sqrt).add_(eps)
  p = p + (h.neg_step_size * m) / denom;          // param.addcdiv_(m, denom, value=-ss)
}

__device__ __forceinline__ void adam_vec(float4& p, float4 g, float4& m, float4& v,
                                         const AdamHP& h) {
  adam_elem(p.x, g.x, m.x, v.x, h);
  adam_elem(p.y, g.y, m.y, v.y, h);
  adam_elem(p.z, g.z, m.z, v.z, h);
  adam_elem(p.w, g.w, m.w, v.w, h);
}

// ------------------------------------------------------------------ dense -----------
__global__ __launch_bounds__(256) void adam_dense_vec(float4* __restrict__ p,
                                                      const float4* __restrict__ g,
                                                      float4* __restrict__ m,
                                                      float4* __restrict__ v, int64_t n4,
                                                      AdamHP h) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4;
       i += (int64_t)gridDim.x * blockDim.x) {
    float4 pp = p[i], mm = m[i], vv = v[i];
    adam_vec(pp, g[i], mm, vv, h);
    p[i] = pp;
    m[i] = mm;
    v[i] = vv;
  }
}

__global__ __launch_bounds__(256) void adam_dense_scalar(float* __restrict__ p,
                                                         const float* __restrict__ g,
                                                         float* __restrict__ m,
                                                         float* __restrict__ v, int64_t lo,
                                                         int64_t n, AdamHP h) {
  for (int64_t i = lo + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    float pp = p[i], mm = m[i], vv = v[i];
    adam_elem(pp, g[i], mm, vv, h);
    p[i] = pp;
    m[i] = mm;
    v[i] = vv;
  }
}

// -------------------------------------------------------- embedding + linear --------
// A wave owns a tile of 64 consecutive rows: lane l reads rowmap / w / m_w / v_w of row
// base+l (one coalesced 256-B access each), then the [64, K] slab of E, m_E, v_E streams
// through in float4 columns (K4 = K/4 lanes per row, 64/K4 rows per wave-instruction; a
// K=64 row is one 256-B line). The touched-row check is a ds_bpermute of the lane's
// rowmap entry; the entry is reset to -1 once both the row and its linear weight used it.
template <int K4>
__global__ __launch_bounds__(256) void adam_embedding_vec(
    float4* __restrict__ E, float4* __restrict__ mE, float4* __restrict__ vE,
    float* __restrict__ w, float* __restrict__ mw, float* __restrict__ vw, int64_t V,
    int32_t* __restrict__ rowmap, const float4* __restrict__ grows,
    const float* __restrict__ glin, AdamHP h) {
  constexpr int RPI = kWave / K4;  // rows per wave-instruction
  constexpr int ITERS = kWave / RPI;
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t waves = (int64_t)gridDim.x * (blockDim.x / kWave);
  const int64_t n_tiles = (V + kWave - 1) / kWave;
  const int c = lane % K4;
  const int r_in = lane / K4;
  for (int64_t tile = (int64_t)blockIdx.x * (blockDim.x / kWave) + threadIdx.x / kWave;
       tile < n_tiles; tile += waves) {
    const int64_t base = tile * kWave;
    const int64_t my_row = base + lane;
    const bool row_ok = my_row < V;
    const int32_t rm = row_ok ? rowmap[my_row] : -1;

    if (w && row_ok) {
      float pp = w[my_row], mm = mw[my_row], vv = vw[my_row];
      adam_elem(pp, rm >= 0 ? glin[rm] : 0.f, mm, vv, h);
      w[my_row] = pp;
      mw[my_row] = mm;
      vw[my_row] = vv;
    }
#pragma unroll 4
    for (int it = 0; it < ITERS; ++it) {
      const int r = it * RPI + r_in;  // row within tile
      const int32_t u = __shfl(rm, r, kWave);
      const int64_t row = base + r;
      if (row < V) {
        const int64_t e = row * K4 + c;
        float4 pp = E[e], mm = mE[e], vv = vE[e];
        const float4 g = u >= 0 ? grows[(int64_t)u * K4 + c] : make_float4(0.f, 0.f, 0.f, 0.f);
        adam_vec(pp, g, mm, vv, h);
        E[e] = pp;
        mE[e] = mm;
        vE[e] = vv;
      }
    }
    if (rm >= 0) rowmap[my_row] = -1;
  }
}

// Any K (e.g. the driver default latent_dims=10): a thread per row.
__global__ __launch_bounds__(256) void adam_embedding_scalar(
    float* __restrict__ E, float* __restrict__ mE, float* __restrict__ vE, float* __restrict__ w,
    float* __restrict__ mw, float* __restrict__ vw, int64_t V, int K,
    int32_t* __restrict__ rowmap, const float* __restrict__ grows,
    const float* __restrict__ glin, AdamHP h) {
  for (int64_t row = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; row < V;
       row += (int64_t)gridDim.x * blockDim.x) {
    const int32_t u = rowmap[row];
    for (int k = 0; k < K; ++k) {
      const int64_t e = row * K + k;
      float pp = E[e], mm = mE[e], vv = vE[e];
      adam_elem(pp, u >= 0 ? grows[(int64_t)u * K + k] : 0.f, mm, vv, h);
      E[e] = pp;
      mE[e] = mm;
      vE[e] = vv;
    }
    if (w) {
      float pp = w[row], mm = mw[row], vv = vw[row];
      adam_elem(pp, u >= 0 ? glin[u] : 0.f, mm, vv, h);
      w[row] = pp;
      mw[row] = mm;
      vw[row] = vv;
    }
    if (u >= 0) rowmap[row] = -1;
  }
}

// Hyper-parameters arrive as doubles, exactly as torch's python code holds them; each is
// rounded to float once, where ATen casts the python scalar for the fp32 kernel.
static AdamHP make_hp(double step_size, double bc2_sqrt, double beta1, double beta2, double eps,
                      double wd) {
  AdamHP h;
  h.neg_step_size = (float)(-step_size);
  h.bc2_sqrt = (float)bc2_sqrt;
  h.w1 = (float)(1.0 - beta1);
  h.beta2 = (float)beta2;
  h.w2 = (float)(1.0 - beta2);
  h.eps = (float)eps;
  h.wd = (float)wd;
  return h;
}

}  // namespace ctr

using namespace ctr;

extern "C" int ctr_adam_dense(float* p, const float* g, float* m, float* v, int64_t n,
                              double step_size, double bc2_sqrt, double beta1, double beta2,
                              double eps, double weight_decay, ctr_stream_t stream) {
  CTR_REQUIRE(n >= 0, "ctr_adam_dense: n < 0");
  if (n == 0) return CTR_OK;
  CTR_REQUIRE(p && g && m && v, "ctr_adam_dense: null pointer");
  CTR_REQUIRE(bc2_sqrt > 0.0, "ctr_adam_dense: bc2_sqrt must be > 0");
  const AdamHP h = make_hp(step_size, bc2_sqrt, beta1, beta2, eps, weight_decay);
  hipStream_t st = as_stream(stream);
  const bool al = ((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) % 16 == 0;
  int64_t done = 0;
  if (al && n >= 4) {
    const int64_t n4 = n / 4;
    const unsigned grid = (unsigned)std::min<int64_t>(ceil_div(n4, 256), 4096);
    hipLaunchKernelGGL(adam_dense_vec, grid, 256, 0, st, reinterpret_cast<float4*>(p),
                       reinterpret_cast<const float4*>(g), reinterpret_cast<float4*>(m),
                       reinterpret_cast<float4*>(v), n4, h);
    CTR_LAUNCH_CHECK("adam_dense_vec");
    done = n4 * 4;
  }
  if (done < n) {
    const unsigned grid = (unsigned)std::min<int64_t>(ceil_div(n - done, 256), 4096);
    hipLaunchKernelGGL(adam_dense_scalar, grid, 256, 0, st, p, g, m, v, done, n, h);
    CTR_LAUNCH_CHECK("adam_dense_scalar");
  }
  return CTR_OK;
}

extern "C" int ctr_adam_embedding(float* emb, float* m_emb, float* v_emb, float* lin, float* m_lin,
                                  float* v_lin, int64_t V, int K, int32_t* rowmap,
                                  const float* grad_rows, const float* grad_lin,
                                  double step_size, double bc2_sqrt, double beta1, double beta2,
                                  double eps, double weight_decay, ctr_stream_t stream) {
  CTR_REQUIRE(emb && m_emb && v_emb && rowmap && grad_rows, "ctr_adam_embedding: null pointer");
  CTR_REQUIRE(V > 0 && K > 0, "ctr_adam_embedding: bad sizes");
  CTR_REQUIRE((lin && m_lin && v_lin && grad_lin) || (!lin && !m_lin && !v_lin),
              "ctr_adam_embedding: linear table pointers must be all set or all NULL");
  CTR_REQUIRE(bc2_sqrt > 0.0, "ctr_adam_embedding: bc2_sqrt must be > 0");
  const AdamHP h = make_hp(step_size, bc2_sqrt, beta1, beta2, eps, weight_decay);
  hipStream_t st = as_stream(stream);
  const bool al =
      ((uintptr_t)emb | (uintptr_t)m_emb | (uintptr_t)v_emb | (uintptr_t)grad_rows) % 16 == 0;
  const int K4 = K / 4;
  if (K % 4 == 0 && al && K4 <= 64 && (kWave % K4) == 0) {
    const int64_t n_tiles = ceil_div(V, kWave);
    const unsigned grid = (unsigned)std::min<int64_t>(ceil_div(n_tiles, 4), 8192);
#define CTR_ADAM_VEC(K4_)                                                                     \
  hipLaunchKernelGGL((adam_embedding_vec<K4_>), grid, 256, 0, st,                             \
                     reinterpret_cast<float4*>(emb), reinterpret_cast<float4*>(m_emb),        \
                     reinterpret_cast<float4*>(v_emb), lin, m_lin, v_lin, V, rowmap,          \
                     reinterpret_cast<const float4*>(grad_rows), grad_lin, h)
    switch (K4) {
      case 1: CTR_ADAM_VEC(1); break;
      case 2: CTR_ADAM_VEC(2); break;
      case 4: CTR_ADAM_VEC(4); break;
      case 8: CTR_ADAM_VEC(8); break;
      case 16: CTR_ADAM_VEC(16); break;
      case 32: CTR_ADAM_VEC(32); break;
      case 64: CTR_ADAM_VEC(64); break;
    }
#undef CTR_ADAM_VEC
    CTR_LAUNCH_CHECK("adam_embedding_vec");
    return CTR_OK;
  }
  const unsigned grid = (unsigned)std::min<int64_t>(ceil_div(V, 256), 8192);
  hipLaunchKernelGGL(adam_embedding_scalar, grid, 256, 0, st, emb, m_emb, v_emb, lin, m_lin, v_lin,
                     V, K, rowmap, grad_rows, grad_lin, h);
  CTR_LAUNCH_CHECK("adam_embedding_scalar");
  return CTR_OK;
}

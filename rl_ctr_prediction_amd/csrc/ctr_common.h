// Shared device/host helpers for libctr_hip.so (gfx950 only: wave64, CDNA4).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "../../include/ctr_hip.h"

namespace ctr {

constexpr int kWave = 64;  // CDNA wavefront; never 32

// ---------------------------------------------------------------- error plumbing ------
void set_error(const char* fmt, ...);

#define CTR_REQUIRE(cond, ...)                       \
  do {                                               \
    if (!(cond)) {                                   \
      ::ctr::set_error(__VA_ARGS__);                 \
      return CTR_ERR_INVALID;                        \
    }                                                \
  } while (0)

#define CTR_LAUNCH_CHECK(what)                                                   \
  do {                                                                           \
    hipError_t e_ = hipGetLastError();                                           \
    if (e_ != hipSuccess) {                                                      \
      ::ctr::set_error("%s: %s", what, hipGetErrorString(e_));                   \
      return CTR_ERR_HIP;                                                        \
    }                                                                            \
  } while (0)

#define CTR_HIP_CHECK(expr)                                                      \
  do {                                                                           \
    hipError_t e_ = (expr);                                                      \
    if (e_ != hipSuccess) {                                                      \
      ::ctr::set_error("%s: %s", #expr, hipGetErrorString(e_));                  \
      return CTR_ERR_HIP;                                                        \
    }                                                                            \
  } while (0)

inline hipStream_t as_stream(ctr_stream_t s) { return reinterpret_cast<hipStream_t>(s); }

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }
inline int64_t align_up(int64_t a, int64_t b) { return ceil_div(a, b) * b; }

// ------------------------------------------------------------------ index loads ------
// Feature ids arrive as int64 (the reference's LongTensor) or int32. An id outside
// [0, V) reads row 0 and raises CTR_EFLAG_INDEX instead of faulting.
template <typename IdxT>
__device__ __forceinline__ int64_t load_row(const IdxT* idx, int64_t i, int64_t V,
                                            int32_t* err) {
  int64_t r = static_cast<int64_t>(idx[i]);
  if (r < 0 || r >= V) {
    if (err) atomicOr(err, (int32_t)CTR_EFLAG_INDEX);
    r = 0;
  }
  return r;
}

// One example's F embedding rows [K] staged by one wave into a wave-private LDS tile (row
// stride ld) and, when `flat` is given, copied to flat[f*K + k]. Lane f loads id f once;
// the F*K elements are then dealt over all 64 lanes with the row broadcast by a shuffle, so
// every element load is independent (a loop over f with a dependent id -> row load per
// field serialised F memory round trips: ~40 us for 4096 x 26 x 16). The shuffles run
// with every lane active (uniform trip count); only the loads and stores are predicated.
template <typename IdxT>
__device__ __forceinline__ void stage_rows_wave(const IdxT* __restrict__ idx, int64_t b, int F,
                                                int K, int64_t V,
                                                const float* __restrict__ emb, float* tile,
                                                int ld, float* __restrict__ flat,
                                                int32_t* err, int lane) {
  // F <= 64, K % 4 == 0, F*K <= 2048 (the CTR shapes: 26 x 64, 22 x 64 ...): float4 pieces,
  // all of a lane's (<= 8) loads in flight before the first LDS store — the loop below, not
  // unrolled, waits for each load before its store (one memory round trip per 64 elements)
  constexpr int kMaxV4 = 8;
  if (F <= 64 && (K & 3) == 0 && F * K <= 4 * 64 * kMaxV4) {
    const int K4 = K >> 2, n4 = F * K4;
    const long long my_row = lane < F ? (long long)load_row(idx, b * F + lane, V, err) : 0ll;
    const bool fvec = flat && (reinterpret_cast<uintptr_t>(flat) & 15) == 0;
    float4 v[kMaxV4];
#pragma unroll
    for (int it = 0; it < kMaxV4; ++it) {
      const int t = lane + 64 * it;  // float4 piece
      int f = t / K4;
      f = f < F ? f : F - 1;
      const long long row = __shfl(my_row, f, 64);
      if (t < n4) v[it] = *reinterpret_cast<const float4*>(emb + row * K + 4 * (t - f * K4));
    }
#pragma unroll
    for (int it = 0; it < kMaxV4; ++it) {
      const int t = lane + 64 * it;
      if (t < n4) {
        const int f = t / K4, k = 4 * (t - f * K4);
        float* tr = tile + f * ld + k;
        if ((ld & 3) == 0) {
          *reinterpret_cast<float4*>(tr) = v[it];
        } else {
          tr[0] = v[it].x;
          tr[1] = v[it].y;
          tr[2] = v[it].z;
          tr[3] = v[it].w;
        }
        if (fvec) {
          *reinterpret_cast<float4*>(flat + 4 * t) = v[it];
        } else if (flat) {
          flat[4 * t] = v[it].x;
          flat[4 * t + 1] = v[it].y;
          flat[4 * t + 2] = v[it].z;
          flat[4 * t + 3] = v[it].w;
        }
      }
    }
    return;
  }
  for (int f0 = 0; f0 < F; f0 += 64) {
    const int nf = F - f0 < 64 ? F - f0 : 64;
    long long my_row = 0;
    if (lane < nf) my_row = (long long)load_row(idx, b * F + f0 + lane, V, err);
    const int n = nf * K, iters = (n + 63) / 64;
    for (int it = 0; it < iters; ++it) {
      const int t = lane + 64 * it;
      int f = t / K;
      f = f < nf ? f : nf - 1;
      const long long row = __shfl(my_row, f, 64);
      if (t < n) {
        const int k = t - f * K;
        const float e = emb[(int64_t)row * K + k];
        tile[(f0 + f) * ld + k] = e;
        if (flat) flat[(int64_t)f0 * K + t] = e;
      }
    }
  }
}

// ------------------------------------------------------------ wave reductions -------
// Butterfly over lanes that differ only in bits >= log2(stride): sums the `group`
// lanes l, l+stride, l+2*stride, ... (stride*group == 64). __shfl_xor lowers to
// ds_bpermute / DPP on gfx950.
template <int STRIDE>
__device__ __forceinline__ float xor_reduce_from(float v) {
#pragma unroll
  for (int o = STRIDE; o < kWave; o <<= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

__device__ __forceinline__ int32_t wave_sum_i32(int32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

__device__ __forceinline__ double wave_sum_f64(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

// ------------------------------------------- exact three-plane bf16 split (MLP) -----
// x = x0 + x1 + x2, x0 = bf16_rne(x), x1 = bf16_rne(x - x0), x2 = x - x0 - x1 (exact: the
// residuals have <= 16 and <= 8 significant bits); x0 + (x1 + x2) == x in fp32. The planes
// feed the split-bf16 MLP GEMM (csrc/gemm_planes.hip); producers write them directly.
typedef float pf32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 pbf16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t psplit_pair(float x, float y, float& rx, float& ry) {
  const pbf16x2 hv = __builtin_convertvector((pf32x2){x, y}, pbf16x2);
  const pf32x2 hf = __builtin_convertvector(hv, pf32x2);
  rx = x - hf.x;
  ry = y - hf.y;
  return __builtin_bit_cast(uint32_t, hv);
}

__device__ __forceinline__ uint32_t ppack_pair(float x, float y) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((pf32x2){x, y}, pbf16x2));
}

// four consecutive elements -> their 8-byte piece of each plane
__device__ __forceinline__ void psplit4(float4 v, uint2 (&o)[3]) {
  float r0, r1, r2, r3, q0, q1, q2, q3;
  o[0].x = psplit_pair(v.x, v.y, r0, r1);
  o[0].y = psplit_pair(v.z, v.w, r2, r3);
  o[1].x = psplit_pair(r0, r1, q0, q1);
  o[1].y = psplit_pair(r2, r3, q2, q3);
  o[2].x = ppack_pair(q0, q1);
  o[2].y = ppack_pair(q2, q3);
}

__device__ __forceinline__ void psplit1(float v, uint16_t (&o)[3]) {
  const __bf16 h0 = (__bf16)v;
  const float r = v - (float)h0;
  const __bf16 h1 = (__bf16)r;
  const __bf16 h2 = (__bf16)(r - (float)h1);
  o[0] = __builtin_bit_cast(uint16_t, h0);
  o[1] = __builtin_bit_cast(uint16_t, h1);
  o[2] = __builtin_bit_cast(uint16_t, h2);
}

// store the planes of 4 consecutive elements at (row base) + p * ps
__device__ __forceinline__ void store_planes4_at(uint16_t* base, int64_t ps, float4 v) {
  uint2 pl[3];
  psplit4(v, pl);
#pragma unroll
  for (int p = 0; p < 3; ++p) *reinterpret_cast<uint2*>(base + p * ps) = pl[p];
}

// -------------------------------------------- BCE after sigmoid (reference exact) ---
// torch.sigmoid then nn.BCELoss(mean) then autograd, UNFUSED, in
// ATen's own operation order (checked bit-exact on CPU, tests/test_oracle.py):
//   loss   = (y-1)*max(log1p(-p),-100) - y*max(log p,-100)
//   g_p    = ((p - y) / max((1-p)*p, 1e-12)) / mean_div        (mean_div = numel)
//   g_z    = (g_p * (1-p)) * p          (exactly 0 when p rounds to 0 or 1)
__device__ __forceinline__ float sigmoidf_ref(float z) { return 1.0f / (1.0f + expf(-z)); }

__device__ __forceinline__ void bce_sigmoid_head(float z, float y, float mean_div,
                                                 float& p, float& loss, float& gz) {
#pragma clang fp contract(off)
  p = sigmoidf_ref(z);
  const float lp = fmaxf(logf(p), -100.0f);
  const float l1p = fmaxf(log1pf(-p), -100.0f);
  loss = (y - 1.0f) * l1p - y * lp;
  const float denom = fmaxf((1.0f - p) * p, 1e-12f);
  const float gp = ((p - y) / denom) / mean_div;
  gz = gp * (1.0f - p) * p;
}

// ------------------------------------------------------ counter-based dropout RNG ---
// splitmix64 finaliser of (seed, counter): a stateless hash, so the backward can
// recompute (or, here, never needs) the mask; statistically uniform 32-bit output.
__device__ __forceinline__ uint32_t hash_u32(uint64_t seed, uint64_t ctr) {
  uint64_t z = seed + 0x9E3779B97F4A7C15ull * (ctr + 1);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return static_cast<uint32_t>(z >> 32);
}

}  // namespace ctr

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

// Micro-benchmark of the deferred-Adam replay arithmetic (adam_common.h adam_elem with
// g = 0): no HBM traffic, only the per-element-step VALU work the flush is bound by.
// Reports ns and SIMD cycles per wave-element-step for the variants below, so the flush's
// floor can be priced against the issue costs in MI355X_MICROARCH.md.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/replay_ubench.hip -o /tmp/replay_ubench
//   (add -fno-slp-vectorize for the scalar-only build)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#include "../rl_ctr_prediction_amd/csrc/adam_common.h"

using namespace ctr;

// VAR 0: adam_elem as shipped. VAR 1: the same with the square root and reciprocal replaced
// by multiplies (prices the transcendentals). VAR 2: adam_elem's arithmetic written out with
// g folded to wd * p (what the compiler should make of VAR 0 anyway).
template <int VAR>
__device__ __forceinline__ void replay1(float& p, float& m, float& v, const AdamHP& h) {
#pragma clang fp contract(off)
  if (VAR == 0) {
    adam_elem(p, 0.f, m, v, h);
  } else if (VAR == 1) {
    const float g = h.wd * p;
    m = __builtin_fmaf(h.w1, g - m, m);
    v = __builtin_fmaf(h.w2 * g, g, v * h.beta2);
    const float denom = __builtin_fmaf(v * 1.0001f, h.inv_bc2_sqrt, h.eps);
    p = __builtin_fmaf(h.neg_step_size * m, denom * 0.999f, p);
  } else {
    const float g = h.wd * p;
    m = __builtin_fmaf(h.w1, g - m, m);
    v = __builtin_fmaf(h.w2 * g, g, v * h.beta2);
    const float denom = __builtin_fmaf(__builtin_amdgcn_sqrtf(v), h.inv_bc2_sqrt, h.eps);
    p = __builtin_fmaf(h.neg_step_size * m, __builtin_amdgcn_rcpf(denom), p);
  }
}

typedef float f2v __attribute__((ext_vector_type(2)));

// VAR 3: two elements at a time with every non-transcendental op packed, the denominator's
// fma included (adam_elem leaves it scalar: the square roots arrive as two scalars).
__device__ __forceinline__ void replay2(float& p0, float& p1, float& m0, float& m1, float& v0,
                                        float& v1, const AdamHP& h) {
#pragma clang fp contract(off)
  const f2v p = {p0, p1}, m = {m0, m1}, v = {v0, v1};
  const f2v wd = {h.wd, h.wd}, w1 = {h.w1, h.w1}, w2 = {h.w2, h.w2}, b2 = {h.beta2, h.beta2};
  const f2v ib = {h.inv_bc2_sqrt, h.inv_bc2_sqrt}, ep = {h.eps, h.eps};
  const f2v ns = {h.neg_step_size, h.neg_step_size}, z = {0.f, 0.f};
  const f2v g = __builtin_elementwise_fma(wd, p, z);
  const f2v mn = __builtin_elementwise_fma(w1, g - m, m);
  const f2v vn = __builtin_elementwise_fma(w2 * g, g, v * b2);
  const f2v sq = {__builtin_amdgcn_sqrtf(vn.x), __builtin_amdgcn_sqrtf(vn.y)};
  const f2v d = __builtin_elementwise_fma(sq, ib, ep);
  const f2v rc = {__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
  const f2v pn = __builtin_elementwise_fma(ns * mn, rc, p);
  p0 = pn.x; p1 = pn.y; m0 = mn.x; m1 = mn.y; v0 = vn.x; v1 = vn.y;
}

template <int VAR, int NCH>
__global__ __launch_bounds__(256) void replay_kernel(float* __restrict__ out, int steps,
                                                     const float2* __restrict__ tab, AdamHP h) {
  __shared__ float2 s_tab[4096];
  for (int i = threadIdx.x; i < steps + 1 && i < 4096; i += blockDim.x) s_tab[i] = tab[i];
  __syncthreads();
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  float p[NCH], m[NCH], v[NCH];
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    p[i] = 0.01f * (tid % 97 + i);
    m[i] = 1e-3f * (i + 1);
    v[i] = 1e-6f * (i + 3);
  }
  for (int s = 1; s <= steps; ++s) {
    const float2 t = s_tab[s];
    h.neg_step_size = t.x;
    h.inv_bc2_sqrt = t.y;
    if constexpr (VAR == 3) {
#pragma unroll
      for (int i = 0; i < NCH; i += 2)
        replay2(p[i], p[i + 1], m[i], m[i + 1], v[i], v[i + 1], h);
    } else {
#pragma unroll
      for (int i = 0; i < NCH; ++i) replay1<VAR>(p[i], m[i], v[i], h);
    }
  }
  float acc = 0.f;
#pragma unroll
  for (int i = 0; i < NCH; ++i) acc += p[i] + m[i] + v[i];
  out[tid] = acc;
}

template <int VAR, int NCH>
static void run(const char* name, float* out, const float2* tab, AdamHP h, int blocks,
                int steps) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  replay_kernel<VAR, NCH><<<blocks, 256>>>(out, steps, tab, h);  // warm
  hipEventRecord(a);
  const int reps = 5;
  for (int r = 0; r < reps; ++r) replay_kernel<VAR, NCH><<<blocks, 256>>>(out, steps, tab, h);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0.f;
  hipEventElapsedTime(&ms, a, b);
  ms /= reps;
  const double elem_steps = (double)blocks * 256 * NCH * steps;
  const double wave_elem_steps = elem_steps / 64;
  const double simd_cycles = ms * 1e-3 * 2.4e9 * 1024;  // 256 CUs x 4 SIMDs at 2.4 GHz
  printf("%-28s NCH=%2d blocks=%5d: %.3f ms  %.4f ps/elem-step  %.1f SIMD-cyc/wave-elem-step\n",
         name, NCH, blocks, ms, ms * 1e9 / elem_steps, simd_cycles / wave_elem_steps);
}

int main() {
  const int steps = 200;
  std::vector<float2> htab(steps + 1);
  for (int s = 0; s <= steps; ++s)
    htab[s] = make_float2(-1e-3f / (1.f - __builtin_powf(0.9f, s + 1)),
                          1.f / __builtin_sqrtf(1.f - __builtin_powf(0.999f, s + 1)));
  float2* tab;
  hipMalloc(&tab, sizeof(float2) * (steps + 1));
  hipMemcpy(tab, htab.data(), sizeof(float2) * (steps + 1), hipMemcpyHostToDevice);
  AdamHP h = make_hp(1e-3, 1.0, 0.9, 0.999, 1e-8, 1e-5);
  const int blocks = 256 * 8;  // every launch below uses at most this many blocks
  float* out;
  hipMalloc(&out, sizeof(float) * blocks * 256);
  run<0, 16>("shipped adam_elem", out, tab, h, blocks, steps);
  run<0, 8>("shipped adam_elem", out, tab, h, blocks, steps);
  run<0, 32>("shipped adam_elem", out, tab, h, blocks, steps);
  run<1, 16>("no transcendentals", out, tab, h, blocks, steps);
  run<2, 16>("same, explicit", out, tab, h, blocks, steps);
  run<0, 16>("shipped, 4 blk/CU", out, tab, h, 256 * 4, steps);
  run<3, 16>("packed denominator", out, tab, h, blocks, steps);
  run<3, 8>("packed denominator", out, tab, h, blocks, steps);
  hipFree(out);
  hipFree(tab);
  return 0;
}

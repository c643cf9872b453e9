// The Adam element update shared by every optimizer kernel (csrc/adam.hip) and the fused
// scatter + Adam apply (csrc/sparse_grad.hip): one definition, so the dense pass, the
// deferred replay and the fused apply produce bitwise identical tables.
#pragma once

#include "ctr_common.h"

namespace ctr {

struct AdamHP {
  float neg_step_size;  // -lr / (1 - beta1^t)
  float inv_bc2_sqrt;   // 1 / sqrt(1 - beta2^t)
  float w1;             // 1 - beta1   (lerp weight)
  float beta2;
  float w2;             // 1 - beta2   (addcmul value)
  float eps;
  float wd;
};

// One Adam element update. m and v use torch's own FMA forms (bit-identical to its CPU
// single-tensor Adam, pinned by tests); the parameter step uses the hardware square root
// and reciprocal (v_sqrt_f32 / v_rcp_f32, ~1 ulp) instead of IEEE-exact sequences: torch's
// own CPU sqrt is not correctly rounded either, the step differs by a few ulps of the
// step (~1e-10 absolute at lr 1e-3), and the replayed (deferred) path stays ~3x cheaper.
// Every Adam kernel below calls this one function, so the dense and the deferred-exact
// paths produce bitwise identical tables.
__device__ __forceinline__ void adam_elem(float& p, float g, float& m, float& v,
                                          const AdamHP& h) {
#pragma clang fp contract(off)
  g = __builtin_fmaf(h.wd, p, g);                 // grad.add(param, alpha=wd)
  m = __builtin_fmaf(h.w1, g - m, m);             // exp_avg.lerp_(grad, 1-beta1)
  v = __builtin_fmaf(h.w2 * g, g, v * h.beta2);   // exp_avg_sq.mul_(b2).addcmul_(g, g, 1-b2)
  const float denom = __builtin_fmaf(__builtin_amdgcn_sqrtf(v), h.inv_bc2_sqrt, h.eps);
  p = __builtin_fmaf(h.neg_step_size * m, __builtin_amdgcn_rcpf(denom), p);  // addcdiv_
}

// Four elements (a float4 column). Scalar ops on purpose: a packed-fp32 form
// (v_pk_fma_f32 / v_pk_mul_f32, bitwise the same results) measured slower on MI355X — the
// apply pass 2-4x (deferred_rows_vec<APPLY>: 7.3 -> 32.6 us at C2, 33.5 -> 59.7 us at C3)
// and within a few % on the VALU-bound flush (packed fp32 issues at about the scalar rate on
// gfx950).
__device__ __forceinline__ void adam_vec(float4& p, float4 g, float4& m, float4& v,
                                         const AdamHP& h) {
  adam_elem(p.x, g.x, m.x, v.x, h);
  adam_elem(p.y, g.y, m.y, v.y, h);
  adam_elem(p.z, g.z, m.z, v.z, h);
  adam_elem(p.w, g.w, m.w, v.w, h);
}

// The replay step of an absent row (g = 0 before weight decay) on four elements: adam_elem's
// arithmetic exactly (same IEEE operations in the same order, so bitwise adam_vec with a zero
// gradient), written on float pairs so that every non-transcendental operation is one
// v_pk_* instruction — the denominator's fma included, which hipcc's SLP pass leaves scalar
// in adam_vec because the square roots arrive as two scalars. The replay is the flush's
// bound (VALU at ~90 % of SIMD cycles at 20 replayed steps, r02_flush_pmc.txt):
// tools/replay_ubench.hip measured 37.3 vs 43.3 SIMD cycles per wave-element-step.
typedef float ctr_f2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void adam_replay_pair(float& p0, float& p1, float& m0, float& m1,
                                                 float& v0, float& v1, const AdamHP& h) {
#pragma clang fp contract(off)
  const ctr_f2 p = {p0, p1}, m = {m0, m1}, v = {v0, v1};
  const ctr_f2 wd = {h.wd, h.wd}, w1 = {h.w1, h.w1}, w2 = {h.w2, h.w2};
  const ctr_f2 b2 = {h.beta2, h.beta2}, ib = {h.inv_bc2_sqrt, h.inv_bc2_sqrt};
  const ctr_f2 ep = {h.eps, h.eps}, ns = {h.neg_step_size, h.neg_step_size}, z = {0.f, 0.f};
  const ctr_f2 g = __builtin_elementwise_fma(wd, p, z);             // grad.add(param, alpha=wd)
  const ctr_f2 mn = __builtin_elementwise_fma(w1, g - m, m);        // lerp_
  const ctr_f2 vn = __builtin_elementwise_fma(w2 * g, g, v * b2);   // mul_(b2).addcmul_
  const ctr_f2 sq = {__builtin_amdgcn_sqrtf(vn.x), __builtin_amdgcn_sqrtf(vn.y)};
  const ctr_f2 d = __builtin_elementwise_fma(sq, ib, ep);
  const ctr_f2 rc = {__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
  const ctr_f2 pn = __builtin_elementwise_fma(ns * mn, rc, p);      // addcdiv_
  p0 = pn.x; p1 = pn.y;
  m0 = mn.x; m1 = mn.y;
  v0 = vn.x; v1 = vn.y;
}

__device__ __forceinline__ void adam_replay_vec(float4& p, float4& m, float4& v, const AdamHP& h) {
  adam_replay_pair(p.x, p.y, m.x, m.y, v.x, v.y, h);
  adam_replay_pair(p.z, p.w, m.z, m.w, v.z, v.w, h);
}

// step_tab[2t] = -lr/(1-beta1^t), step_tab[2t+1] = 1/sqrt(1-beta2^t)  (host doubles -> f32)
__device__ __forceinline__ void load_step(AdamHP& h, const float* __restrict__ tab, int s) {
  const float2 v = reinterpret_cast<const float2*>(tab)[s];
  h.neg_step_size = v.x;
  h.inv_bc2_sqrt = v.y;
}

// Hyper-parameters arrive as doubles, exactly as torch's python code holds them; each is
// rounded to float once, where ATen casts the python scalar for the fp32 kernel.
static inline AdamHP make_hp(double step_size, double bc2_sqrt, double beta1, double beta2,
                             double eps, double wd) {
  AdamHP h;
  h.neg_step_size = (float)(-step_size);
  h.inv_bc2_sqrt = (float)(1.0 / bc2_sqrt);
  h.w1 = (float)(1.0 - beta1);
  h.beta2 = (float)beta2;
  h.w2 = (float)(1.0 - beta2);
  h.eps = (float)eps;
  h.wd = (float)wd;
  return h;
}

// One row of a deferred table whose state (p, m, v of the float4 column c, and of the
// linear weight on lane c == 0) and last[] are already in registers: replay the steps it
// missed up to step-1, then step `step` with its gradient, and store it back.
__device__ __forceinline__ void deferred_apply_loaded(
    float4* __restrict__ E, float4* __restrict__ mE, float4* __restrict__ vE,
    float* __restrict__ w, float* __restrict__ mw, float* __restrict__ vw,
    int32_t* __restrict__ last, int64_t r, int KV, int c, bool col, float4 g, float glin,
    int step, const float* __restrict__ tab, AdamHP h, int from, float4 pp, float4 mm,
    float4 vv, float pw, float mws, float vws) {
  const int64_t e = r * KV + c;
  const bool own_lin = w && c == 0;
  for (int s = from + 1; s < step; ++s) {
    load_step(h, tab, s);
    if (col) adam_replay_vec(pp, mm, vv, h);
    if (own_lin) adam_elem(pw, 0.f, mws, vws, h);
  }
  load_step(h, tab, step);
  if (col) {
    adam_vec(pp, g, mm, vv, h);
    E[e] = pp; mE[e] = mm; vE[e] = vv;
  }
  if (own_lin) {
    adam_elem(pw, glin, mws, vws, h);
    w[r] = pw; mw[r] = mws; vw[r] = vws;
  }
  if (c == 0) last[r] = step;
}

// The same with the row's state loaded here (the body of deferred_rows_vec<APPLY=true>).
__device__ __forceinline__ void deferred_apply_row(
    float4* __restrict__ E, float4* __restrict__ mE, float4* __restrict__ vE,
    float* __restrict__ w, float* __restrict__ mw, float* __restrict__ vw,
    int32_t* __restrict__ last, int64_t r, int KV, int c, bool col, float4 g, float glin,
    int step, const float* __restrict__ tab, AdamHP h) {
  const int from = last[r];
  const int64_t e = r * KV + c;
  float4 pp, mm, vv;
  if (col) {
    pp = E[e]; mm = mE[e]; vv = vE[e];
  }
  const bool own_lin = w && c == 0;
  float pw = 0.f, mws = 0.f, vws = 0.f;
  if (own_lin) {
    pw = w[r]; mws = mw[r]; vws = vw[r];
  }
  deferred_apply_loaded(E, mE, vE, w, mw, vw, last, r, KV, c, col, g, glin, step, tab, h, from,
                        pp, mm, vv, pw, mws, vws);
}

}  // namespace ctr

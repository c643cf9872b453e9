// Ensemble prediction + sign reward of the RL drivers:
// `generate_preds` (reference src/all_main/hybrid_td3_main_per_v10.py:54-164, the same
// function in every hybrid_* / PA_DDPG / RL_average driver). For every example b with
// pretrained pCTRs preds[b, 0..M-1], an ensemble size a = actions[b] in 1..M, model
// weights pw[b, :] and continuous actions ca[b, :]:
//
//   a == M:  y = sum_m pw[b,m] * preds[b,m]                    (lines 89-96)
//            ret_c[b, :] = ca[b, :]
//   a <  M:  models   = the a largest pw[b, :] (descending, ties by lower index: a stable
//                       sort of -pw, line 62)
//            w        = softmax(the a largest ca[b, :])          (lines 111-113)
//            y        = sum_m w[m] * preds[b, models[m]]         (lines 118-131)
//            ret_c[b, models[m]] = m-th largest of ca[j, :], where j is b's ORDINAL among
//                       the batch's examples with the same action — the reference indexes
//                       the full-batch `sort_c_actions` with positions local to the action
//                       group (line 127); kept, it is what the drivers store as transitions
//   reward:  label 1: y > mean_m preds[b,m] ? 1 : 0; label 0: y < mean ? 1 : 0 (137-157)
//   actions outside 1..M: y = 1, reward = 1, ret_c = 0 (the tensors' initial values)
//
// The per-action ordinals come from one 1024-thread block walking the batch in order with
// wave ballots (stable by construction); the rest is one thread per example with M <= 32
// values in registers (top-a by repeated arg-max: a <= M <= 32, no sort needed).
#include "ctr_common.h"

namespace ctr {

constexpr int kMaxModels = 32;

template <typename AT>
__global__ __launch_bounds__(1024) void action_rank_kernel(const AT* __restrict__ act, int64_t B,
                                                           int M, int32_t* __restrict__ rank) {
  __shared__ int32_t s_cnt[16][kMaxModels + 1];
  __shared__ int32_t s_run[kMaxModels + 1];
  const int t = threadIdx.x, lane = t & (kWave - 1), w = t / kWave;
  if (t <= M) s_run[t] = 0;
  __syncthreads();
  const uint64_t below = lane ? (~0ull >> (kWave - lane)) : 0ull;
  for (int64_t base = 0; base < B; base += 1024) {
    const int64_t b = base + t;
    const int64_t a64 = b < B ? (int64_t)act[b] : 0;
    const int a = (a64 >= 1 && a64 <= M) ? (int)a64 : 0;
    int prefix = 0;
    for (int v = 1; v <= M; ++v) {
      const uint64_t mask = __ballot(a == v);
      if (a == v) prefix = __popcll(mask & below);
      if (lane == 0) s_cnt[w][v] = __popcll(mask);
    }
    __syncthreads();
    if (b < B) {
      int r = -1;
      if (a) {
        r = s_run[a] + prefix;
        for (int ww = 0; ww < w; ++ww) r += s_cnt[ww][a];
      }
      rank[b] = r;
    }
    __syncthreads();
    if (t >= 1 && t <= M) {
      int s = 0;
      for (int ww = 0; ww < 16; ++ww) s += s_cnt[ww][t];
      s_run[t] += s;
    }
    __syncthreads();
  }
}

template <typename AT, typename LT>
__global__ __launch_bounds__(256) void ensemble_preds_kernel(
    const float* __restrict__ preds, int64_t ldp, const AT* __restrict__ act,
    const float* __restrict__ pw, const float* __restrict__ ca, const LT* __restrict__ labels,
    const int32_t* __restrict__ rank, int64_t B, int M, float* __restrict__ y_out,
    float* __restrict__ r_out, float* __restrict__ rc_out) {
#pragma clang fp contract(off)  // the reference's separate torch.mul / torch.sum roundings
  for (int64_t b = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; b < B;
       b += (int64_t)gridDim.x * blockDim.x) {
    float pr[kMaxModels], rc[kMaxModels];
    float s = 0.f;
#pragma unroll
    for (int m = 0; m < kMaxModels; ++m) {
      pr[m] = m < M ? preds[b * ldp + m] : 0.f;
      rc[m] = 0.f;
      if (m < M) s += pr[m];
    }
    const float mean = s / (float)M;  // current_pretrain_y_preds.mean(dim=1)
    const int64_t a64 = (int64_t)act[b];
    float y = 1.f, reward = 1.f;
    if (a64 >= 1 && a64 <= M) {
      const int a = (int)a64;
      const float* pwb = pw + b * M;
      const float* cab = ca + b * M;
      if (a == M) {
        y = 0.f;
#pragma unroll
        for (int m = 0; m < kMaxModels; ++m)
          if (m < M) {
            y += pwb[m] * pr[m];
            rc[m] = cab[m];
          }
      } else {
        const float* caj = ca + (int64_t)rank[b] * M;  // the reference's local-index row
        uint32_t used_p = 0, used_c = 0, used_j = 0;
        float top_c[kMaxModels], row_p[kMaxModels];
        for (int m = 0; m < a; ++m) {
          // m-th model by descending pw (ties: lower index first)
          int bp = -1, bc = -1, bj = -1;
          float vp = 0.f, vc = 0.f, vj = 0.f;
          for (int k = 0; k < M; ++k) {
            const float p = pwb[k], c = cab[k], cj = caj[k];
            if (!(used_p >> k & 1) && (bp < 0 || p > vp)) { bp = k; vp = p; }
            if (!(used_c >> k & 1) && (bc < 0 || c > vc)) { bc = k; vc = c; }
            if (!(used_j >> k & 1) && (bj < 0 || cj > vj)) { bj = k; vj = cj; }
          }
          used_p |= 1u << bp;
          used_c |= 1u << bc;
          used_j |= 1u << bj;
          top_c[m] = vc;
          row_p[m] = pr[bp];
          rc[bp] = vj;  // return_c_actions[.., k] = sort_c_actions[j, m] * -1
        }
        // softmax over the a largest c values (torch.softmax: max-shifted exp, then / sum)
        const float mx = top_c[0];
        float e[kMaxModels], den = 0.f;
        for (int m = 0; m < a; ++m) {
          e[m] = expf(top_c[m] - mx);
          den += e[m];
        }
        y = 0.f;
        for (int m = 0; m < a; ++m) y += (e[m] / den) * row_p[m];
      }
      const int64_t lab = (int64_t)labels[b];
      if (lab == 1) reward = y > mean ? 1.f : 0.f;
      else if (lab == 0) reward = y < mean ? 1.f : 0.f;
    }
    y_out[b] = y;
    r_out[b] = reward;
#pragma unroll
    for (int m = 0; m < kMaxModels; ++m)
      if (m < M) rc_out[b * M + m] = rc[m];
  }
}

template <typename AT, typename LT>
static int launch_ensemble(const float* preds, int64_t ldp, const void* act, const float* pw,
                           const float* ca, const void* labels, int32_t* rank, int64_t B, int M,
                           float* y, float* r, float* rc, hipStream_t st) {
  hipLaunchKernelGGL(action_rank_kernel<AT>, 1, 1024, 0, st, static_cast<const AT*>(act), B, M,
                     rank);
  CTR_LAUNCH_CHECK("action_rank_kernel");
  const unsigned grid = (unsigned)std::min<int64_t>(ceil_div(B, 256), 4096);
  hipLaunchKernelGGL((ensemble_preds_kernel<AT, LT>), grid, 256, 0, st, preds, ldp,
                     static_cast<const AT*>(act), pw, ca, static_cast<const LT*>(labels), rank,
                     B, M, y, r, rc);
  CTR_LAUNCH_CHECK("ensemble_preds_kernel");
  return CTR_OK;
}

}  // namespace ctr

using namespace ctr;

extern "C" int ctr_ensemble_preds(const float* preds, int64_t B, int M, int64_t ld_preds,
                                  const void* actions, int action_type, const float* prob_weights,
                                  const float* c_actions, const void* labels, int label_type,
                                  float* y_preds, float* rewards, float* return_c_actions,
                                  int32_t* rank_ws, ctr_stream_t stream) {
  CTR_REQUIRE(B >= 0 && M >= 1 && M <= kMaxModels && ld_preds >= M,
              "ctr_ensemble_preds: need 1 <= M <= %d models and ld_preds >= M", kMaxModels);
  CTR_REQUIRE(action_type == CTR_IDX_I32 || action_type == CTR_IDX_I64, "bad action_type %d",
              action_type);
  CTR_REQUIRE(label_type == CTR_IDX_I32 || label_type == CTR_IDX_I64, "bad label_type %d",
              label_type);
  if (B == 0) return CTR_OK;
  CTR_REQUIRE(preds && actions && prob_weights && c_actions && labels && y_preds && rewards &&
                  return_c_actions && rank_ws,
              "ctr_ensemble_preds: null pointer");
  hipStream_t st = as_stream(stream);
  const bool a64 = action_type == CTR_IDX_I64, l64 = label_type == CTR_IDX_I64;
  if (a64 && l64)
    return launch_ensemble<int64_t, int64_t>(preds, ld_preds, actions, prob_weights, c_actions,
                                             labels, rank_ws, B, M, y_preds, rewards,
                                             return_c_actions, st);
  if (a64)
    return launch_ensemble<int64_t, int32_t>(preds, ld_preds, actions, prob_weights, c_actions,
                                             labels, rank_ws, B, M, y_preds, rewards,
                                             return_c_actions, st);
  if (l64)
    return launch_ensemble<int32_t, int64_t>(preds, ld_preds, actions, prob_weights, c_actions,
                                             labels, rank_ws, B, M, y_preds, rewards,
                                             return_c_actions, st);
  return launch_ensemble<int32_t, int32_t>(preds, ld_preds, actions, prob_weights, c_actions,
                                           labels, rank_ws, B, M, y_preds, rewards,
                                           return_c_actions, st);
}

// Op-level C interface: one POD argument struct per `ctr::<op>` PyTorch op
// (rl_ctr_prediction_amd/torch_ops.py), for bindings without torch (ctypes, cgo, JNI). Each
// ctr_op_<op> composes the flat entry points of include/ctr_hip.h in the order the torch op
// does, so the results are the same bits; ctr_workspace_bytes(op, dims) sizes the scratch
// the composite carves (plans, row partials, row maps).
#include <cmath>

#include "ctr_common.h"

namespace ctr {

// rowmap[rows[u]] = u (rows distinct, in [0, V)); an out-of-range row is skipped and flagged
template <typename I>
__global__ __launch_bounds__(256) void rowmap_set_kernel(const I* __restrict__ rows, int64_t n,
                                                         int64_t V, int32_t* __restrict__ rowmap,
                                                         int32_t* __restrict__ err_flag) {
  const int64_t u = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (u >= n) return;
  const int64_t r = (int64_t)rows[u];
  if (r < 0 || r >= V) {
    if (err_flag) atomicOr(err_flag, (int32_t)CTR_EFLAG_INDEX);
    return;
  }
  rowmap[r] = (int32_t)u;
}

// The plan a composite op builds in its workspace: S-entry arrays + seg_offsets (S+1) +
// num_unique, then the radix scratch.
struct PlanCarve {
  ctr_sparse_plan plan;
  void* plan_ws;
  int64_t plan_ws_bytes;
  char* rest;
};

static int64_t plan_arrays_bytes(int64_t S) {
  return 4 * align_up(S * 4, 256) + align_up((S + 1) * 4, 256) + 256;
}

static int64_t plan_total_bytes(int64_t S, int64_t V) {
  return plan_arrays_bytes(S) + align_up(ctr_sparse_plan_workspace_bytes(S, V), 256);
}

static PlanCarve carve_plan(void* ws, int64_t S, int64_t V) {
  PlanCarve c{};
  char* p = static_cast<char*>(ws);
  auto take = [&](int64_t bytes) {
    char* q = p;
    p += align_up(bytes, 256);
    return q;
  };
  c.plan.S = S;
  c.plan.sorted_slots = reinterpret_cast<int32_t*>(take(S * 4));
  c.plan.sorted_rows = reinterpret_cast<int32_t*>(take(S * 4));
  c.plan.pos_seg = reinterpret_cast<int32_t*>(take(S * 4));
  c.plan.unique_rows = reinterpret_cast<int32_t*>(take(S * 4));
  c.plan.seg_offsets = reinterpret_cast<int32_t*>(take((S + 1) * 4));
  c.plan.num_unique = reinterpret_cast<int32_t*>(take(4));
  c.plan_ws_bytes = align_up(ctr_sparse_plan_workspace_bytes(S, V), 256);
  c.plan_ws = take(c.plan_ws_bytes);
  c.rest = p;
  return c;
}

// torch/optim/adam.py's step scalars (python doubles: 1 - beta ** step, lr / bc1, bc2 ** 0.5)
static void adam_scalars(int64_t step, double lr, double beta1, double beta2, double* step_size,
                         double* bc2_sqrt) {
  const double t = (double)(step < 1 ? 1 : step);
  *step_size = lr / (1.0 - std::pow(beta1, t));
  *bc2_sqrt = std::pow(1.0 - std::pow(beta2, t), 0.5);
}

static int64_t fm_bwd_bytes(int64_t B, int64_t F, int64_t K, int64_t V) {
  const int64_t S = B * F;
  return plan_total_bytes(S, V) + align_up(ctr_segment_workspace_bytes(S, (int)K), 256) +
         align_up(S * K * 4, 256) + align_up(S * 4, 256) +
         align_up(ctr_reduce_workspace_bytes(B, 1), 256);
}

static int64_t scatter_bytes(int64_t S, int64_t K, int64_t V) {
  return plan_total_bytes(S, V) + align_up(ctr_segment_workspace_bytes(S, (int)K), 256) +
         align_up(S * K * 4, 256);
}

}  // namespace ctr

using namespace ctr;

extern "C" int64_t ctr_workspace_bytes(int op, const int64_t* dims, int n_dims) {
  auto need = [&](int n) {
    if (n_dims < n || (n > 0 && !dims)) return false;
    for (int i = 0; i < n; ++i)
      if (dims[i] < 0) return false;
    return true;
  };
  switch (op) {
    case CTR_OP_FM_FWD:
    case CTR_OP_DEEPFM_GATHER_CONCAT:
    case CTR_OP_ADAM_DENSE:
    case CTR_OP_PAIRWISE_FE:
      return 0;
    case CTR_OP_FM_BWD:  // {B, F, K, V}
      return need(4) ? fm_bwd_bytes(dims[0], dims[1], dims[2], dims[3]) : -1;
    case CTR_OP_EMB_SCATTER_ADD:  // {n_slots, K, V}
      return need(3) ? scatter_bytes(dims[0], dims[1], dims[2]) : -1;
    case CTR_OP_ADAM_ROWWISE:  // {V}
      return need(1) ? align_up(dims[0] * 4, 256) : -1;
    case CTR_OP_PG_RETURNS:  // {n}
      return need(1) ? align_up(ctr_pg_workspace_bytes(dims[0]), 256) + 256 : -1;
  }
  return -1;
}

#define CTR_OP_WS(a_, need_)                                                          \
  CTR_REQUIRE((need_) >= 0 && (a_)->ws_bytes >= (need_) && ((need_) == 0 || (a_)->ws), \
              "%s: workspace smaller than ctr_workspace_bytes()", __func__)

extern "C" int ctr_op_fm_fwd(const ctr_fm_fwd_args* a, ctr_stream_t stream) {
  CTR_REQUIRE(a, "ctr_op_fm_fwd: null args");
  return ctr_fm_forward(a->idx, a->idx_type, a->B, a->F, a->K, a->V, a->emb, a->lin, a->bias,
                        a->z, a->sum_e, nullptr, nullptr, 1.f, nullptr, nullptr, nullptr,
                        a->err_flag, stream);
}

extern "C" int ctr_op_fm_bwd(const ctr_fm_bwd_args* a, ctr_stream_t stream) {
  CTR_REQUIRE(a, "ctr_op_fm_bwd: null args");
  CTR_REQUIRE(a->B >= 0 && a->F > 0 && a->K > 0 && a->V > 0, "ctr_op_fm_bwd: bad sizes");
  CTR_REQUIRE(a->g_emb && a->g_lin && a->g_bias && a->emb && a->sum_e && a->gz && a->idx,
              "ctr_op_fm_bwd: null pointer");
  const int64_t S = a->B * a->F, K = a->K;
  const int64_t need = fm_bwd_bytes(a->B, a->F, K, a->V);
  CTR_OP_WS(a, need);
  hipStream_t st = as_stream(stream);
  CTR_HIP_CHECK(hipMemsetAsync(a->g_emb, 0, (size_t)(a->V * K * 4), st));
  CTR_HIP_CHECK(hipMemsetAsync(a->g_lin, 0, (size_t)(a->V * 4), st));
  PlanCarve c = carve_plan(a->ws, S, a->V);
  char* p = c.rest;
  const int64_t seg_bytes = align_up(ctr_segment_workspace_bytes(S, (int)K), 256);
  void* seg_ws = p;
  p += seg_bytes;
  float* rows = reinterpret_cast<float*>(p);
  p += align_up(S * K * 4, 256);
  float* rows_lin = reinterpret_cast<float*>(p);
  p += align_up(S * 4, 256);
  void* red_ws = p;
  const int64_t red_bytes = align_up(ctr_reduce_workspace_bytes(a->B, 1), 256);
  int rc = ctr_sparse_plan_build(a->idx, a->idx_type, a->V, &c.plan, c.plan_ws, c.plan_ws_bytes,
                                 a->err_flag, stream);
  if (rc != CTR_OK) return rc;
  rc = ctr_fm_embedding_grad(&c.plan, (int)a->F, (int)K, a->emb, a->gz, a->sum_e, nullptr, rows,
                             rows_lin, nullptr, seg_ws, seg_bytes, stream);
  if (rc != CTR_OK) return rc;
  rc = ctr_rows_to_dense(&c.plan, (int)K, rows, rows_lin, a->g_emb, a->g_lin, stream);
  if (rc != CTR_OK) return rc;
  return ctr_sum_f32(a->gz, a->B, 1.f, a->g_bias, red_ws, red_bytes, stream);
}

extern "C" int ctr_op_deepfm_gather_concat(const ctr_deepfm_gather_concat_args* a,
                                           ctr_stream_t stream) {
  CTR_REQUIRE(a, "ctr_op_deepfm_gather_concat: null args");
  CTR_REQUIRE(a->B >= 0 && a->F > 0, "ctr_op_deepfm_gather_concat: bad sizes");
  return ctr_embedding_gather(a->emb, a->V, a->K, a->idx, a->idx_type, a->B * a->F, a->out,
                              a->err_flag, stream);
}

extern "C" int ctr_op_emb_scatter_add(const ctr_emb_scatter_add_args* a, ctr_stream_t stream) {
  CTR_REQUIRE(a, "ctr_op_emb_scatter_add: null args");
  CTR_REQUIRE(a->n_slots >= 0 && a->K > 0 && a->V > 0, "ctr_op_emb_scatter_add: bad sizes");
  CTR_REQUIRE(a->dense && (a->n_slots == 0 || (a->idx && a->grad_slots)),
              "ctr_op_emb_scatter_add: null pointer");
  const int64_t S = a->n_slots, K = a->K;
  const int64_t need = scatter_bytes(S, K, a->V);
  CTR_OP_WS(a, need);
  hipStream_t st = as_stream(stream);
  CTR_HIP_CHECK(hipMemsetAsync(a->dense, 0, (size_t)(a->V * K * 4), st));
  if (S == 0) return CTR_OK;
  PlanCarve c = carve_plan(a->ws, S, a->V);
  char* p = c.rest;
  const int64_t seg_bytes = align_up(ctr_segment_workspace_bytes(S, (int)K), 256);
  void* seg_ws = p;
  p += seg_bytes;
  float* rows = reinterpret_cast<float*>(p);
  int rc = ctr_sparse_plan_build(a->idx, a->idx_type, a->V, &c.plan, c.plan_ws, c.plan_ws_bytes,
                                 a->err_flag, stream);
  if (rc != CTR_OK) return rc;
  rc = ctr_segment_sum_rows(&c.plan, (int)K, a->grad_slots, nullptr, rows, nullptr, nullptr,
                            seg_ws, seg_bytes, stream);
  if (rc != CTR_OK) return rc;
  return ctr_rows_to_dense(&c.plan, (int)K, rows, nullptr, a->dense, nullptr, stream);
}

extern "C" int ctr_op_adam_dense(const ctr_adam_dense_args* a, ctr_stream_t stream) {
  CTR_REQUIRE(a, "ctr_op_adam_dense: null args");
  double ss, bc2s;
  adam_scalars(a->step, a->lr, a->beta1, a->beta2, &ss, &bc2s);
  return ctr_adam_dense(a->p, a->g, a->m, a->v, a->n, ss, bc2s, nullptr, nullptr, a->beta1,
                        a->beta2, a->eps, a->weight_decay, stream);
}

extern "C" int ctr_op_adam_rowwise(const ctr_adam_rowwise_args* a, ctr_stream_t stream) {
  CTR_REQUIRE(a, "ctr_op_adam_rowwise: null args");
  CTR_REQUIRE(a->V > 0 && a->K > 0 && a->n_rows >= 0, "ctr_op_adam_rowwise: bad sizes");
  CTR_REQUIRE(a->rows_type == CTR_IDX_I32 || a->rows_type == CTR_IDX_I64,
              "ctr_op_adam_rowwise: bad rows_type");
  CTR_REQUIRE(a->n_rows == 0 || (a->rows && a->grad_rows), "ctr_op_adam_rowwise: null pointer");
  const int64_t need = align_up(a->V * 4, 256);
  CTR_OP_WS(a, need);
  hipStream_t st = as_stream(stream);
  int32_t* rowmap = static_cast<int32_t*>(a->ws);
  CTR_HIP_CHECK(hipMemsetAsync(rowmap, 0xFF, (size_t)(a->V * 4), st));  // -1: no gradient
  if (a->n_rows > 0) {
    const unsigned g = (unsigned)ceil_div(a->n_rows, 256);
    if (a->rows_type == CTR_IDX_I64)
      hipLaunchKernelGGL(rowmap_set_kernel<int64_t>, g, 256, 0, st,
                         static_cast<const int64_t*>(a->rows), a->n_rows, a->V, rowmap, a->err_flag);
    else
      hipLaunchKernelGGL(rowmap_set_kernel<int32_t>, g, 256, 0, st,
                         static_cast<const int32_t*>(a->rows), a->n_rows, a->V, rowmap, a->err_flag);
    CTR_LAUNCH_CHECK("rowmap_set_kernel");
  }
  double ss, bc2s;
  adam_scalars(a->step, a->lr, a->beta1, a->beta2, &ss, &bc2s);
  return ctr_adam_embedding(a->emb, a->m, a->v, nullptr, nullptr, nullptr, a->V, a->K, rowmap,
                            a->grad_rows, nullptr, ss, bc2s, nullptr, nullptr, a->beta1,
                            a->beta2, a->eps, a->weight_decay, stream);
}

extern "C" int ctr_op_pairwise_fe(const ctr_pairwise_fe_args* a, ctr_stream_t stream) {
  CTR_REQUIRE(a, "ctr_op_pairwise_fe: null args");
  return ctr_feature_embedding_forward(a->idx, a->idx_type, a->B, a->F, a->K, a->V, a->emb,
                                       a->out, a->err_flag, stream);
}

extern "C" int ctr_op_pg_returns(const ctr_pg_returns_args* a, ctr_stream_t stream) {
  CTR_REQUIRE(a, "ctr_op_pg_returns: null args");
  CTR_REQUIRE(a->n >= 0, "ctr_op_pg_returns: bad size");
  const int64_t pg = align_up(ctr_pg_workspace_bytes(a->n), 256);
  const int64_t need = pg + 256;
  CTR_OP_WS(a, need);
  double* stats = reinterpret_cast<double*>(static_cast<char*>(a->ws) + pg);
  return ctr_pg_discount_norm(a->r, a->n, a->gamma, a->vt, a->vt_f32, stats, a->ws, pg, stream);
}

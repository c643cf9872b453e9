// Deterministic reductions (loss mean, bias / 1-row-Linear gradients) and the REINFORCE
// kernels of PG_model.PolicyGradient.
//
// Every reduction here has a fixed, size-determined order (grid sizes depend only on the
// problem size; partials are added in block order), so results are identical bits run to
// run and on every data-parallel rank.
#include "ctr_common.h"

namespace ctr {

constexpr int kSumBlocks = 256;  // stage-1 blocks of ctr_sum_f32 (fixed => deterministic)

__device__ __forceinline__ float block_sum_256(float v, float* sh) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) sh[wave] = v;
  __syncthreads();
  float r = 0.f;
  if (threadIdx.x == 0) r = (sh[0] + sh[1]) + (sh[2] + sh[3]);
  __syncthreads();
  return r;  // valid in thread 0
}

__global__ __launch_bounds__(256) void sum_stage1(const float* __restrict__ x, int64_t n,
                                                  int64_t per_block, float* __restrict__ part) {
  __shared__ float sh[4];
  const int64_t lo = blockIdx.x * per_block;
  const int64_t hi = min(n, lo + per_block);
  float acc = 0.f;
#pragma unroll 32
  for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) acc += x[i];
  const float r = block_sum_256(acc, sh);
  if (threadIdx.x == 0) part[blockIdx.x] = r;
}

// One launch for n <= kSmallSum (batch-sized vectors): 1024 threads, fixed order.
constexpr int64_t kSmallSum = 1 << 16;
__global__ __launch_bounds__(1024) void sum_small(const float* __restrict__ x, int64_t n,
                                                  float scale, float* __restrict__ out) {
  __shared__ float sh[16];
  float acc = 0.f;
#pragma unroll 32
  for (int64_t i = threadIdx.x; i < n; i += 1024) acc += x[i];
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float r = 0.f;
    for (int w2 = 0; w2 < 16; ++w2) r += sh[w2];
    out[0] = r * scale;
  }
}

__global__ __launch_bounds__(256) void sum_stage2(const float* __restrict__ part, int nparts,
                                                  float scale, float* __restrict__ out) {
  __shared__ float sh[4];
  float acc = 0.f;
  for (int i = threadIdx.x; i < nparts; i += blockDim.x) acc += part[i];
  const float r = block_sum_256(acc, sh);
  if (threadIdx.x == 0) out[0] = r * scale;
}

// colsum: grid (ceil(N/64), RS); block = 64 columns x 4 row lanes.
__global__ __launch_bounds__(256) void colsum_stage1(const float* __restrict__ X, int64_t M,
                                                     int64_t N, int64_t ldx,
                                                     const float* __restrict__ w,
                                                     int64_t rows_per_split,
                                                     float* __restrict__ part) {
  __shared__ float sh[4][64];
  const int cx = threadIdx.x & 63, ry = threadIdx.x >> 6;
  const int64_t n = (int64_t)blockIdx.x * 64 + cx;
  const int64_t lo = (int64_t)blockIdx.y * rows_per_split;
  const int64_t hi = min(M, lo + rows_per_split);
  float acc = 0.f;
  // unrolled so the loads of 8 rows are in flight together (a rolled loop waits one
  // memory round trip per row); the additions stay in row order (deterministic)
  if (n < N) {
    if (w) {
#pragma unroll 32
      for (int64_t m = lo + ry; m < hi; m += 4) acc += w[m] * X[m * ldx + n];
    } else {
#pragma unroll 32
      for (int64_t m = lo + ry; m < hi; m += 4) acc += X[m * ldx + n];
    }
  }
  sh[ry][cx] = acc;
  __syncthreads();
  if (ry == 0 && n < N) part[blockIdx.y * N + n] = (sh[0][cx] + sh[1][cx]) + (sh[2][cx] + sh[3][cx]);
}

__global__ __launch_bounds__(256) void colsum_stage2(const float* __restrict__ part, int rs,
                                                     int64_t N, float scale,
                                                     float* __restrict__ out) {
  for (int64_t n = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; n < N;
       n += (int64_t)gridDim.x * blockDim.x) {
    float s = 0.f;
#pragma unroll 32
    for (int r = 0; r < rs; ++r) s += part[(int64_t)r * N + n];
    out[n] = s * scale;
  }
}

// Several column sums in ONE launch pair (the DeepFM step's bias / last-layer weight
// gradients): each job keeps exactly colsum_stage1/2's row partition and order, so every
// output is bitwise what ctr_colsum_f32 gives; blocks enumerate (job, 64-column block).
constexpr int kMaxColsumJobs = 8;
struct ColsumJobs {
  int n;
  const float* X[kMaxColsumJobs];
  int64_t M[kMaxColsumJobs], N[kMaxColsumJobs], ldx[kMaxColsumJobs], rps[kMaxColsumJobs];
  const float* w[kMaxColsumJobs];
  float scale[kMaxColsumJobs];
  float* out[kMaxColsumJobs];
  int rs[kMaxColsumJobs];
  int64_t cb0[kMaxColsumJobs + 1];  // first 64-column block of each job
  int64_t part0[kMaxColsumJobs];    // offset of each job's partials
  int64_t col0[kMaxColsumJobs + 1]; // first output column of each job (all jobs flattened)
};

__global__ __launch_bounds__(256) void colsum_multi_stage1(ColsumJobs J, float* __restrict__ part) {
  __shared__ float sh[4][64];
  int j = 0;
  while (j + 1 < J.n && (int64_t)blockIdx.x >= J.cb0[j + 1]) ++j;
  if ((int)blockIdx.y >= J.rs[j]) return;  // block-uniform
  const int cx = threadIdx.x & 63, ry = threadIdx.x >> 6;
  const int64_t n = ((int64_t)blockIdx.x - J.cb0[j]) * 64 + cx;
  const int64_t N = J.N[j], ldx = J.ldx[j];
  const int64_t lo = (int64_t)blockIdx.y * J.rps[j];
  const int64_t hi = min(J.M[j], lo + J.rps[j]);
  const float* X = J.X[j];
  const float* w = J.w[j];
  float acc = 0.f;
  if (n < N) {
    if (w) {
#pragma unroll 32
      for (int64_t m = lo + ry; m < hi; m += 4) acc += w[m] * X[m * ldx + n];
    } else {
#pragma unroll 32
      for (int64_t m = lo + ry; m < hi; m += 4) acc += X[m * ldx + n];
    }
  }
  sh[ry][cx] = acc;
  __syncthreads();
  if (ry == 0 && n < N)
    part[J.part0[j] + blockIdx.y * N + n] = (sh[0][cx] + sh[1][cx]) + (sh[2][cx] + sh[3][cx]);
}

// one thread per output column of every job (all jobs' columns flattened, so the partial
// loads of all of them are in flight at once: a loop over the jobs put each job's load round
// trip after the previous one's, 21 us for the policy net's five bias gradients); the
// partials summed in split order as before
__global__ __launch_bounds__(256) void colsum_multi_stage2(ColsumJobs J,
                                                           const float* __restrict__ part) {
  const int64_t g = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (g >= J.col0[J.n]) return;
  int j = 0;
  while (j + 1 < J.n && g >= J.col0[j + 1]) ++j;
  const int64_t N = J.N[j], n = g - J.col0[j];
  const float* pj = part + J.part0[j];
  float s = 0.f;
#pragma unroll 32
  for (int r = 0; r < J.rs[j]; ++r) s += pj[(int64_t)r * N + n];
  J.out[j][n] = s * J.scale[j];
}

static int colsum_splits(int64_t M) {
  return (int)std::max<int64_t>(1, std::min<int64_t>(ceil_div(M, 256), 64));
}

// ----------------------------------------------------------------- REINFORCE --------
// torch.softmax(x, dim=1) for narrow rows (A = number of actions).
__global__ __launch_bounds__(256) void softmax_rows_kernel(const float* __restrict__ x, int64_t B,
                                                           int A, float* __restrict__ out) {
  for (int64_t b = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; b < B;
       b += (int64_t)gridDim.x * blockDim.x) {
    const float* xb = x + b * A;
    float mx = xb[0];
    for (int j = 1; j < A; ++j) mx = fmaxf(mx, xb[j]);
    float s = 0.f;
    for (int j = 0; j < A; ++j) s += expf(xb[j] - mx);
    for (int j = 0; j < A; ++j) out[b * A + j] = expf(xb[j] - mx) / s;
  }
}

// PG_model.discount_and_norm_rewards (139-154), fp64 like the reference's numpy buffer:
// d[i] = r[i] + gamma*d[i+1] (reverse), then d -= mean(d); d /= std(d) (population).
// One block of 1024 threads: each thread owns a contiguous chunk whose backward walk is the
// affine map d(lo) = S + P * d(hi). The maps compose right to left, (S1,P1)∘(S2,P2) =
// (S1 + P1*S2, P1*P2), so each thread's carry d(hi) comes from a suffix scan of the maps:
// 6 shuffle steps inside the wave, then the 16 wave totals (log-depth instead of a
// 1024-long serial chain on one thread: 34 -> ~6 us at C4's 4096 transitions). Each chunk
// is then re-walked from its carry.
__global__ __launch_bounds__(1024) void pg_discount_norm_kernel(const float* __restrict__ r,
                                                                int64_t n, double gamma,
                                                                double* __restrict__ out,
                                                                float* __restrict__ out_f32,
                                                                double* __restrict__ stats) {
  __shared__ double s_wsum[16];
  __shared__ double s_wpow[16];
  __shared__ double s_red[16];
  const int t = threadIdx.x, T = blockDim.x;
  const int lane = t & 63, wv = t >> 6, nw = T >> 6;
  const int64_t cs = (n + T - 1) / T;
  const int64_t lo = min(n, (int64_t)t * cs), hi = min(n, lo + cs);
  double acc = 0.0, pw = 1.0;
  for (int64_t i = hi - 1; i >= lo; --i) {
    acc = acc * gamma + (double)r[i];
    pw *= gamma;
  }
  // inclusive suffix scan over the wave's lanes: lane l ends with lanes l..63 composed
  double S = acc, P = pw;
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const double S2 = __shfl_down(S, o, kWave), P2 = __shfl_down(P, o, kWave);
    if (lane + o < kWave) {
      S = S + P * S2;
      P = P * P2;
    }
  }
  if (lane == 0) {
    s_wsum[wv] = S;
    s_wpow[wv] = P;
  }
  // lanes l+1..63 of this wave (identity for the last lane)
  double Sx = __shfl_down(S, 1, kWave), Px = __shfl_down(P, 1, kWave);
  if (lane == kWave - 1) {
    Sx = 0.0;
    Px = 1.0;
  }
  __syncthreads();
  double after = 0.0;  // d at the start of wave wv+1 = waves wv+1..nw-1 applied to 0
  for (int w = nw - 1; w > wv; --w) after = s_wsum[w] + s_wpow[w] * after;
  double run = Sx + Px * after;
  double part = 0.0;
  for (int64_t i = hi - 1; i >= lo; --i) {
    run = run * gamma + (double)r[i];
    out[i] = run;
    part += run;
  }
  // mean
  auto block_sum = [&](double v) -> double {
    v = wave_sum_f64(v);
    if ((t & 63) == 0) s_red[t >> 6] = v;
    __syncthreads();
    double tot = 0.0;
    for (int w = 0; w < T / 64; ++w) tot += s_red[w];
    __syncthreads();
    return tot;
  };
  const double mean = block_sum(part) / (double)n;
  double part2 = 0.0;
  for (int64_t i = lo; i < hi; ++i) {
    out[i] -= mean;
    part2 += out[i];
  }
  // np.std of the centred buffer: its own mean, then sqrt(mean(|x - mean|^2))
  const double mean2 = block_sum(part2) / (double)n;
  double part3 = 0.0;
  for (int64_t i = lo; i < hi; ++i) {
    const double dv = out[i] - mean2;
    part3 += dv * dv;
  }
  const double stdv = sqrt(block_sum(part3) / (double)n);
  for (int64_t i = lo; i < hi; ++i) {
    out[i] /= stdv;
    if (out_f32) out_f32[i] = (float)out[i];
  }
  if (t == 0 && stats) {
    stats[0] = mean;
    stats[1] = stdv;
  }
}

// PG_model.loss_func (104-107) + autograd through gather/log/softmax, one block:
//   nlp = sum_b -log(p[b, a_b - 1]);  loss = mean(nlp * vt) ;
//   c = d loss / d nlp = sum_i vt_i / n;  g[b,a] = -c / p[b,a];
//   dlogit[b,j] = p[b,j] * (g[b,j] - g[b,a] * p[b,a])     (softmax backward)
// vt_mean != NULL (data-parallel episode split over ranks): c = vt_mean[0] * grad_scale
// with the episode-wide mean from pg_vt_mean_kernel, and loss = nlp * vt_mean[0] — this
// rank's share of the global loss (the shares are summed by the caller's all-reduce).
__device__ __forceinline__ float block_sum_1024(float v, float* s_red) {
  const int t = threadIdx.x, T = blockDim.x;
  v = wave_sum(v);
  if ((t & 63) == 0) s_red[t >> 6] = v;
  __syncthreads();
  float tot = 0.f;
  for (int w = 0; w < T / 64; ++w) tot += s_red[w];
  __syncthreads();
  return tot;
}

__global__ __launch_bounds__(1024) void pg_loss_grad_kernel(const float* __restrict__ p,
                                                            const int64_t* __restrict__ acts,
                                                            const float* __restrict__ vt,
                                                            const float* __restrict__ vt_mean,
                                                            int64_t B, int A, float grad_scale,
                                                            float* __restrict__ loss_out,
                                                            float* __restrict__ dlogits) {
  __shared__ float s_red[16];
  const int t = threadIdx.x, T = blockDim.x;
  float nl = 0.f, sv = 0.f;
  for (int64_t b = t; b < B; b += T) {
    int64_t a = acts[b] - 1;
    a = a < 0 ? 0 : (a >= A ? A - 1 : a);
    nl += -logf(p[b * A + a]);
    if (!vt_mean) sv += vt[b];
  }
  const float nlp = block_sum_1024(nl, s_red);
  float c;
  if (vt_mean) {
    if (t == 0 && loss_out) loss_out[0] = nlp * vt_mean[0];
    c = vt_mean[0] * grad_scale;
  } else {
    const float svt = block_sum_1024(sv, s_red);
    float lv = 0.f;
    for (int64_t b = t; b < B; b += T) lv += nlp * vt[b];
    const float loss = block_sum_1024(lv, s_red) / (float)B;
    if (t == 0 && loss_out) loss_out[0] = loss;
    c = (svt / (float)B) * grad_scale;
  }
  if (!dlogits) return;
  for (int64_t b = t; b < B; b += T) {
    int64_t a = acts[b] - 1;
    a = a < 0 ? 0 : (a >= A ? A - 1 : a);
    const float pa = p[b * A + a];
    const float ga = -c / pa;
    const float dot = ga * pa;
    for (int j = 0; j < A; ++j) {
      const float gj = (j == a) ? ga : 0.f;
      dlogits[b * A + j] = p[b * A + j] * (gj - dot);
    }
  }
}

// mean(vt) over a whole episode in exactly the order pg_loss_grad_kernel sums it, so a
// data-parallel step uses the bit-identical c of the single-process step.
__global__ __launch_bounds__(1024) void pg_vt_mean_kernel(const float* __restrict__ vt, int64_t n,
                                                          float* __restrict__ out) {
  __shared__ float s_red[16];
  float sv = 0.f;
  for (int64_t b = threadIdx.x; b < n; b += blockDim.x) sv += vt[b];
  const float svt = block_sum_1024(sv, s_red);
  if (threadIdx.x == 0) out[0] = svt / (float)n;
}

}  // namespace ctr

using namespace ctr;

extern "C" int64_t ctr_reduce_workspace_bytes(int64_t M, int64_t N) {
  if (M < 0 || N < 0) return -1;
  const int64_t a = (int64_t)kSumBlocks * 4;
  const int64_t b = (int64_t)colsum_splits(M) * std::max<int64_t>(N, 1) * 4;
  return align_up(std::max(a, b), 256);
}

extern "C" int ctr_sum_f32(const float* x, int64_t n, float scale, float* out, void* ws,
                           int64_t ws_bytes, ctr_stream_t stream) {
  CTR_REQUIRE(out && n >= 0 && (x || n == 0), "ctr_sum_f32: bad arguments");
  CTR_REQUIRE(ws && ws_bytes >= (int64_t)kSumBlocks * 4, "ctr_sum_f32: workspace too small");
  hipStream_t st = as_stream(stream);
  if (n <= kSmallSum) {
    hipLaunchKernelGGL(sum_small, 1, 1024, 0, st, x, n, scale, out);
    CTR_LAUNCH_CHECK("sum_small");
    return CTR_OK;
  }
  const int64_t per = std::max<int64_t>(1, ceil_div(n, kSumBlocks));
  float* part = static_cast<float*>(ws);
  hipLaunchKernelGGL(sum_stage1, kSumBlocks, 256, 0, st, x, n, per, part);
  CTR_LAUNCH_CHECK("sum_stage1");
  hipLaunchKernelGGL(sum_stage2, 1, 256, 0, st, part, kSumBlocks, scale, out);
  CTR_LAUNCH_CHECK("sum_stage2");
  return CTR_OK;
}

extern "C" int ctr_colsum_f32(const float* X, int64_t M, int64_t N, int64_t ldx, const float* row_w,
                              float scale, float* out, void* ws, int64_t ws_bytes,
                              ctr_stream_t stream) {
  CTR_REQUIRE(M >= 0 && N >= 0 && ldx >= N, "ctr_colsum_f32: bad sizes");
  if (N == 0) return CTR_OK;
  CTR_REQUIRE(out && (X || M == 0), "ctr_colsum_f32: null pointer");
  const int rs = colsum_splits(M);
  CTR_REQUIRE(ws && ws_bytes >= (int64_t)rs * N * 4, "ctr_colsum_f32: workspace too small");
  hipStream_t st = as_stream(stream);
  float* part = static_cast<float*>(ws);
  const int64_t rps = std::max<int64_t>(1, ceil_div(M, rs));
  hipLaunchKernelGGL(colsum_stage1, dim3((unsigned)ceil_div(N, 64), (unsigned)rs), 256, 0, st, X,
                     M, N, ldx, row_w, rps, part);
  CTR_LAUNCH_CHECK("colsum_stage1");
  hipLaunchKernelGGL(colsum_stage2, (unsigned)std::min<int64_t>(ceil_div(N, 256), 1024), 256, 0,
                     st, part, rs, N, scale, out);
  CTR_LAUNCH_CHECK("colsum_stage2");
  return CTR_OK;
}

static int colsum_multi_plan(int n, const ctr_colsum_job* jobs, ColsumJobs& J, int64_t& need) {
  CTR_REQUIRE(n >= 1 && n <= kMaxColsumJobs && jobs, "ctr_colsum_multi_f32: 1..%d jobs",
              kMaxColsumJobs);
  memset(&J, 0, sizeof(J));
  J.n = n;
  need = 0;
  for (int j = 0; j < n; ++j) {
    const ctr_colsum_job& c = jobs[j];
    CTR_REQUIRE(c.M >= 0 && c.N >= 1 && c.ldx >= c.N && c.out && (c.X || c.M == 0),
                "ctr_colsum_multi_f32: bad job %d", j);
    J.X[j] = c.X; J.M[j] = c.M; J.N[j] = c.N; J.ldx[j] = c.ldx; J.w[j] = c.row_w;
    J.scale[j] = c.scale; J.out[j] = c.out;
    J.rs[j] = colsum_splits(c.M);
    J.rps[j] = std::max<int64_t>(1, ceil_div(c.M, J.rs[j]));
    J.cb0[j + 1] = J.cb0[j] + ceil_div(c.N, 64);
    J.col0[j + 1] = J.col0[j] + c.N;
    J.part0[j] = need;
    need += (int64_t)J.rs[j] * c.N;
  }
  need *= 4;
  return CTR_OK;
}

extern "C" int64_t ctr_colsum_multi_workspace_bytes(int n_jobs, const ctr_colsum_job* jobs) {
  ColsumJobs J;
  int64_t need = 0;
  if (colsum_multi_plan(n_jobs, jobs, J, need) != CTR_OK) return -1;
  return align_up(std::max<int64_t>(need, 4), 256);
}

extern "C" int ctr_colsum_multi_f32(int n_jobs, const ctr_colsum_job* jobs, void* ws,
                                    int64_t ws_bytes, ctr_stream_t stream) {
  ColsumJobs J;
  int64_t need = 0;
  int rc = colsum_multi_plan(n_jobs, jobs, J, need);
  if (rc != CTR_OK) return rc;
  CTR_REQUIRE(ws && ws_bytes >= need, "ctr_colsum_multi_f32: workspace too small");
  int rs_max = 1;
  for (int j = 0; j < n_jobs; ++j) rs_max = std::max(rs_max, J.rs[j]);
  hipStream_t st = as_stream(stream);
  float* part = static_cast<float*>(ws);
  hipLaunchKernelGGL(colsum_multi_stage1, dim3((unsigned)J.cb0[n_jobs], (unsigned)rs_max), 256, 0,
                     st, J, part);
  CTR_LAUNCH_CHECK("colsum_multi_stage1");
  hipLaunchKernelGGL(colsum_multi_stage2, (unsigned)ceil_div(J.col0[n_jobs], 256), 256, 0, st, J,
                     static_cast<const float*>(part));
  CTR_LAUNCH_CHECK("colsum_multi_stage2");
  return CTR_OK;
}

extern "C" int ctr_softmax_rows(const float* x, int64_t B, int A, float* out, ctr_stream_t stream) {
  CTR_REQUIRE(B >= 0 && A > 0 && (B == 0 || (x && out)), "ctr_softmax_rows: bad arguments");
  if (B == 0) return CTR_OK;
  hipLaunchKernelGGL(softmax_rows_kernel, (unsigned)std::min<int64_t>(ceil_div(B, 256), 4096), 256,
                     0, as_stream(stream), x, B, A, out);
  CTR_LAUNCH_CHECK("ctr_softmax_rows");
  return CTR_OK;
}

extern "C" int64_t ctr_pg_workspace_bytes(int64_t n) { return n < 0 ? -1 : 0; }

extern "C" int ctr_pg_discount_norm(const float* r, int64_t n, double gamma, double* out,
                                    float* out_f32, double* stats, void* ws, int64_t ws_bytes,
                                    ctr_stream_t stream) {
  (void)ws;
  (void)ws_bytes;
  CTR_REQUIRE(n > 0 && r && out, "ctr_pg_discount_norm: bad arguments");
  hipLaunchKernelGGL(pg_discount_norm_kernel, 1, 1024, 0, as_stream(stream), r, n, gamma, out,
                     out_f32, stats);
  CTR_LAUNCH_CHECK("ctr_pg_discount_norm");
  return CTR_OK;
}

extern "C" int ctr_pg_loss_grad(const float* probs, const int64_t* acts, const float* vt,
                                int64_t B, int A, float grad_scale, float* loss_out,
                                float* dlogits, void* ws, int64_t ws_bytes, ctr_stream_t stream) {
  (void)ws;
  (void)ws_bytes;
  CTR_REQUIRE(B > 0 && A > 0 && probs && acts && vt, "ctr_pg_loss_grad: bad arguments");
  hipLaunchKernelGGL(pg_loss_grad_kernel, 1, 1024, 0, as_stream(stream), probs, acts, vt,
                     (const float*)nullptr, B, A, grad_scale, loss_out, dlogits);
  CTR_LAUNCH_CHECK("ctr_pg_loss_grad");
  return CTR_OK;
}

extern "C" int ctr_pg_vt_mean(const float* vt, int64_t n, float* out, ctr_stream_t stream) {
  CTR_REQUIRE(n > 0 && vt && out, "ctr_pg_vt_mean: bad arguments");
  hipLaunchKernelGGL(pg_vt_mean_kernel, 1, 1024, 0, as_stream(stream), vt, n, out);
  CTR_LAUNCH_CHECK("ctr_pg_vt_mean");
  return CTR_OK;
}

extern "C" int ctr_pg_loss_grad_global(const float* probs, const int64_t* acts, int64_t B, int A,
                                       const float* vt_mean, float grad_scale, float* loss_out,
                                       float* dlogits, ctr_stream_t stream) {
  CTR_REQUIRE(B >= 0 && A > 0 && vt_mean && (B == 0 || (probs && acts)),
              "ctr_pg_loss_grad_global: bad arguments");
  hipLaunchKernelGGL(pg_loss_grad_kernel, 1, 1024, 0, as_stream(stream), probs, acts,
                     (const float*)nullptr, vt_mean, B, A, grad_scale, loss_out, dlogits);
  CTR_LAUNCH_CHECK("ctr_pg_loss_grad_global");
  return CTR_OK;
}

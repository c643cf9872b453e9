// Adam with coupled L2 (torch.optim.Adam(lr, weight_decay)) — dense
// semantics: every element of every parameter moves every step, as in the reference
// (nn.Embedding(sparse=False) + Adam). This is the dominant HBM stream of the step:
// per element it reads p, m, v and writes p, m, v (24 B); the embedding gradient is not
// materialised densely — a row's gradient is read from the compact per-row sums only
// when rowmap[row] >= 0, so the dense pass costs 24 B/elem + 4 B/row, not 32 B/elem.
//
// Arithmetic follows torch's single-tensor CPU Adam (torch/optim/adam.py), checked
// against torch 2.10: m and v bit-exact with the FMA forms below; the parameter step to a
// few ulps of the step (see adam_elem).
//
// Deferred-exact mode (temporal blocking). A row absent from a batch gets g = wd*p — a
// function of its own state only — so its per-step update needs no information from the
// step it skipped. Instead of streaming all V rows through HBM every step, each row keeps
// last[r] = the step it is current to; a row is brought forward by replaying the missed
// steps in registers with the SAME adam_elem and the SAME per-step scalars, (1) before a
// batch reads it (catch-up, unique rows of the batch), (2) when its gradient is applied
// (apply), (3) for every row at a flush (epoch end, checkpoint, eval). Every element still
// receives every step's arithmetic, in order; only the HBM round trips of untouched rows
// between two uses disappear. Results are bitwise identical to the dense pass
// (tests/test_gpu_deferred.py).
#include "adam_common.h"

#include <cstdlib>

namespace ctr {

// (adam_replay_vec, the replay step of an absent row, is in adam_common.h. Measured and
// rejected on MI355X before it: an inline-asm packed form (4.32 vs 4.42 ms at 20 replayed
// steps, 3.06 vs 2.64 at 1 step), and one reciprocal per element pair (1/d0 = d1 *
// rcp(d0*d1): the flush 33.3-34.1 ms either way at C5 — the extra multiplies cancel the
// saved reciprocal).)

// ------------------------------------------------------------------ dense -----------
// step_ptr != NULL: the step's scalars come from the device step table (HIP-graph replay)

// Up to two row-major [rows, cols] sub-matrices of the flat parameter vector (the MLP
// weights the GEMMs read as bf16 planes) whose planes are rewritten with the updated values,
// so the next step's GEMMs need no split pass. off and cols are multiples of 4: a float4
// never straddles two rows.
constexpr int kMaxPlaneViews = 3;
struct PlaneViews {
  int n;
  int64_t off[kMaxPlaneViews], len[kMaxPlaneViews], cols[kMaxPlaneViews];
  int64_t ld[kMaxPlaneViews], ps[kMaxPlaneViews];
  uint16_t* d[kMaxPlaneViews];
};

__global__ __launch_bounds__(256) void adam_dense_vec(float4* __restrict__ p,
                                                      const float4* __restrict__ g,
                                                      float4* __restrict__ m,
                                                      float4* __restrict__ v, int64_t n4,
                                                      AdamHP h, const float* __restrict__ tab,
                                                      const int32_t* __restrict__ step_ptr,
                                                      PlaneViews pv) {
  if (step_ptr) load_step(h, tab, *step_ptr);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4;
       i += (int64_t)gridDim.x * blockDim.x) {
    float4 pp = p[i], mm = m[i], vv = v[i];
    adam_vec(pp, g[i], mm, vv, h);
    p[i] = pp;
    m[i] = mm;
    v[i] = vv;
#pragma unroll
    for (int j = 0; j < kMaxPlaneViews; ++j) {
      const int64_t e = 4 * i - pv.off[j];
      if (j < pv.n && e >= 0 && e < pv.len[j]) {
        if (pv.cols[j] % 4 == 0) {  // the four elements share a row
          const int64_t r = e / pv.cols[j], c = e - r * pv.cols[j];
          store_planes4_at(pv.d[j] + r * pv.ld[j] + c, pv.ps[j], pp);
        } else {  // rows of any width (PG's 741-wide first layer): element by element
          const float pe[4] = {pp.x, pp.y, pp.z, pp.w};
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int64_t eq = e + q;
            if (eq < pv.len[j]) {
              const int64_t r = eq / pv.cols[j], c = eq - r * pv.cols[j];
              uint16_t h3[3];
              psplit1(pe[q], h3);
#pragma unroll
              for (int pl = 0; pl < 3; ++pl) pv.d[j][pl * pv.ps[j] + r * pv.ld[j] + c] = h3[pl];
            }
          }
        }
      }
    }
  }
}

__global__ __launch_bounds__(256) void adam_dense_scalar(float* __restrict__ p,
                                                         const float* __restrict__ g,
                                                         float* __restrict__ m,
                                                         float* __restrict__ v, int64_t lo,
                                                         int64_t n, AdamHP h,
                                                         const float* __restrict__ tab,
                                                         const int32_t* __restrict__ step_ptr) {
  if (step_ptr) load_step(h, tab, *step_ptr);
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
    const float* __restrict__ glin, AdamHP h, const float* __restrict__ tab,
    const int32_t* __restrict__ step_ptr) {
  if (step_ptr) load_step(h, tab, *step_ptr);
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
    const float* __restrict__ glin, AdamHP h, const float* __restrict__ tab,
    const int32_t* __restrict__ step_ptr) {
  if (step_ptr) load_step(h, tab, *step_ptr);
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

// ------------------------------------------------------------ deferred-exact --------

// A/B builds only (tools/build_variant.py): 0 = every replayed step's scalars from the
// global table
#ifndef CTR_ROWS_TAB_WIN
#define CTR_ROWS_TAB_WIN 64
#endif

// Rows of a sparse plan (unique rows of a batch). One lane group of K4 lanes per row
// (float4 columns), 64/K4 rows per wave. APPLY=false: replay to `step` (catch-up before
// the forward reads the rows). APPLY=true: replay to step-1, then step `step` with the
// row's gradient. Lane 0 of the group also owns the row's linear weight.
template <int K4, bool APPLY>
__global__ __launch_bounds__(256) void deferred_rows_vec(
    float4* __restrict__ E, float4* __restrict__ mE, float4* __restrict__ vE,
    float* __restrict__ w, float* __restrict__ mw, float* __restrict__ vw,
    int32_t* __restrict__ last, const int32_t* __restrict__ rows,
    const int32_t* __restrict__ num_unique, const float4* __restrict__ grows,
    const float* __restrict__ glin, int step_val, const int32_t* __restrict__ step_ptr,
    const float* __restrict__ tab, AdamHP h) {
  // the step table's last kTabWin entries (steps target-kTabWin+1 .. target) staged in LDS
  // once per block: a replayed step reads its scalars from LDS instead of a dependent
  // global load per step (older steps, past a longer gap than the flush period, still read
  // the global table)
  constexpr int kTabWin = CTR_ROWS_TAB_WIN > 0 ? CTR_ROWS_TAB_WIN : 1;
  __shared__ float2 s_tab[kTabWin];
  const int c = threadIdx.x % K4;
  const int64_t groups = (int64_t)gridDim.x * (blockDim.x / K4);
  const int U = *num_unique;
  const int step = step_ptr ? *step_ptr : step_val;
  const int target = APPLY ? step - 1 : step;
  const int win0 = CTR_ROWS_TAB_WIN > 0 ? max(0, target - kTabWin + 1) : target + 1;
  if (threadIdx.x < kTabWin && win0 + (int)threadIdx.x <= target)
    s_tab[threadIdx.x] = reinterpret_cast<const float2*>(tab)[win0 + threadIdx.x];
  __syncthreads();
  // (measured: two rows per lane group with all their loads issued first, 30.3 vs 30.6 us
  // at C3 with one replayed step — the random 256-B row traffic, ~3 TB/s, is the floor)
  for (int64_t u = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) / K4; u < U; u += groups) {
    const int64_t r = rows[u];
    // the row's state is loaded beside last[r], not behind the staleness test: one dependent
    // round trip less per row (a current row's loads are wasted, and with the periodic
    // flush few rows of a batch are current)
    const int64_t e = r * K4 + c;
    const int from = last[r];
    float4 pp = E[e], mm = mE[e], vv = vE[e];
    float pw = 0.f, mws = 0.f, vws = 0.f;
    const bool own_lin = w && c == 0;
    if (own_lin) {
      pw = w[r]; mws = mw[r]; vws = vw[r];
    }
    if (!APPLY && from >= target) continue;
    for (int s = from + 1; s <= target; ++s) {
      if (s >= win0) {
        const float2 v = s_tab[s - win0];
        h.neg_step_size = v.x;
        h.inv_bc2_sqrt = v.y;
      } else {
        load_step(h, tab, s);
      }
      adam_replay_vec(pp, mm, vv, h);
      if (own_lin) adam_elem(pw, 0.f, mws, vws, h);
    }
    if (APPLY) {
      load_step(h, tab, step);
      adam_vec(pp, grows[u * K4 + c], mm, vv, h);
      if (own_lin) adam_elem(pw, glin[u], mws, vws, h);
    }
    E[e] = pp; mE[e] = mm; vE[e] = vv;
    if (own_lin) {
      w[r] = pw; mw[r] = mws; vw[r] = vws;
    }
    if (c == 0) last[r] = APPLY ? step : target;
  }
}

// Catch-up straight from a batch's feature ids, without the sparse plan (so the plan can be
// built on another stream while the forward runs). Duplicate ids are resolved through a
// V-sized owner scratch: every slot stores its index at owner[row] (plain stores, one of
// them survives), then the slot whose index survived replays the row. Who replays is
// arbitrary; what is computed is not (same adam_elem chain as every other path).
template <typename IdxT>
__global__ __launch_bounds__(256) void deferred_mark_kernel(const IdxT* __restrict__ idx,
                                                            int64_t S, int64_t V,
                                                            int32_t* __restrict__ owner) {
  for (int64_t s = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; s < S;
       s += (int64_t)gridDim.x * blockDim.x)
    owner[load_row(idx, s, V, nullptr)] = (int32_t)s;
}

// The same catch-up with one LANE per slot for the ownership / staleness test and the
// replay done by lane groups over a compacted per-wave list: the test for all 64 slots of a
// wave issues together (idx -> owner -> last, three dependent loads for 64 slots at once
// instead of for one slot per K4-lane group), then the wave's stale owned rows — a fraction
// of its slots — are dealt to its 64/K4 lane groups, UNR rows per group at a time with
// every load of the batch issued before the replay. Same adam_elem chain: bitwise the
// per-slot kernel above.
template <typename IdxT, int K4, int UNR>
__global__ __launch_bounds__(256) void deferred_catchup_wave(
    float4* __restrict__ E, float4* __restrict__ mE, float4* __restrict__ vE,
    float* __restrict__ w, float* __restrict__ mw, float* __restrict__ vw,
    int32_t* __restrict__ last, const IdxT* __restrict__ idx, int64_t S, int64_t V,
    const int32_t* __restrict__ owner, const int32_t* __restrict__ step_ptr,
    const float* __restrict__ tab, AdamHP h) {
  constexpr int RPI = kWave / K4;  // lane groups (rows in flight per batch step) per wave
  __shared__ int32_t s_row[4][kWave];
  __shared__ int32_t s_from[4][kWave];
  const int lane = threadIdx.x & (kWave - 1);
  const int wib = threadIdx.x / kWave;
  const int g = lane / K4, c = lane % K4;
  const int step = *step_ptr;
  const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x / kWave);
  for (int64_t base = ((int64_t)blockIdx.x * (blockDim.x / kWave) + wib) * kWave; base < S;
       base += nwaves * kWave) {
    const int64_t s = base + lane;
    bool need = false;
    int32_t r = 0, from = 0;
    if (s < S) {
      r = (int32_t)load_row(idx, s, V, nullptr);
      if (owner[r] == (int32_t)s) {
        from = last[r];
        need = from < step;
      }
    }
    const uint64_t mask = __ballot(need);
    const int n = __popcll(mask);
    if (need) {
      const int pos = __popcll(mask & ((1ull << lane) - 1));
      s_row[wib][pos] = r;
      s_from[wib][pos] = from;
    }
    __builtin_amdgcn_wave_barrier();
    for (int j0 = 0; j0 < n; j0 += RPI * UNR) {
      float4 pp[UNR], mm[UNR], vv[UNR];
      int32_t rr[UNR], ff[UNR];
      int fmin = step;
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const int j = j0 + u * RPI + g;
        rr[u] = j < n ? s_row[wib][j] : -1;
        ff[u] = j < n ? s_from[wib][j] : step;
        fmin = min(fmin, ff[u]);
        if (rr[u] >= 0) {
          const int64_t e = (int64_t)rr[u] * K4 + c;
          pp[u] = E[e]; mm[u] = mE[e]; vv[u] = vE[e];
        }
      }
      for (int t = fmin + 1; t <= step; ++t) {
        load_step(h, tab, t);
#pragma unroll
        for (int u = 0; u < UNR; ++u)
          if (t > ff[u]) adam_replay_vec(pp[u], mm[u], vv[u], h);
      }
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        if (rr[u] < 0) continue;
        const int64_t e = (int64_t)rr[u] * K4 + c;
        E[e] = pp[u]; mE[e] = mm[u]; vE[e] = vv[u];
        if (c == 0) {
          if (w) {
            float pw = w[rr[u]], mws = mw[rr[u]], vws = vw[rr[u]];
            for (int t = ff[u] + 1; t <= step; ++t) {
              load_step(h, tab, t);
              adam_elem(pw, 0.f, mws, vws, h);
            }
            w[rr[u]] = pw; mw[rr[u]] = mws; vw[rr[u]] = vws;
          }
          last[rr[u]] = step;
        }
      }
    }
    __builtin_amdgcn_wave_barrier();  // the list is re-filled by the next iteration
  }
}

// Device step counters of a trainer: ctr[0] = completed steps, ctr[1] = the step in flight.
// Within a step, ctr[0] stays at t-1 (catch-up and dropout read it) and ctr[1] = t
// (the Adam apply reads it), so work on several streams never sees the counter move.
__global__ void step_begin_kernel(int32_t* ctr) { ctr[1] = ctr[0] + 1; }
// loss_sum (optional): the driver's epoch loss, accumulated on the device in double —
// adding the fp32 batch loss widened exactly, in step order, is bitwise the reference's
// Python `total_loss += loss.item()` (all_main/pretrain_main.py:79)
__global__ void step_end_kernel(int32_t* ctr, const float* loss, double* loss_sum) {
  const int32_t t = ctr[1];
  ctr[0] = t;
  ctr[1] = t + 1;  // the next step's: ctr_step_begin is then a no-op
  if (loss_sum) loss_sum[0] += (double)loss[0];
}

// The FM step's dense tail in one launch (single process): the batch loss and the FM
// bias gradient summed exactly as sum_small does (same per-thread order, wave butterfly,
// 16 wave partials in order: bitwise ctr_sum_f32), the flat dense parameters' Adam step at
// ctr[1] (adam_elem, bitwise adam_dense_vec), then ctr_step_end — four launches of the C2
// step graph (2 x sum_small, adam_dense_vec, step_end_kernel) become one.
__global__ __launch_bounds__(1024) void fm_step_tail_kernel(
    const float* __restrict__ loss_elem, const float* __restrict__ gz, int64_t B,
    float loss_scale, float* __restrict__ loss_out, float* bias_grad, float* __restrict__ p,
    const float* g, float* __restrict__ m, float* __restrict__ v, int64_t n, AdamHP h,
    const float* __restrict__ tab, int32_t* ctr, double* loss_sum) {
  __shared__ float sh[2][16];
  const int t = threadIdx.x;
  float al = 0.f, ag = 0.f;
#pragma unroll 8
  for (int64_t i = t; i < B; i += 1024) {
    al += loss_elem[i];
    ag += gz[i];
  }
  al = wave_sum(al);
  ag = wave_sum(ag);
  if ((t & 63) == 0) {
    sh[0][t >> 6] = al;
    sh[1][t >> 6] = ag;
  }
  load_step(h, tab, ctr[1]);
  __syncthreads();
  if (t == 0) {
    float rl = 0.f, rg = 0.f;
    for (int w2 = 0; w2 < 16; ++w2) {
      rl += sh[0][w2];
      rg += sh[1][w2];
    }
    const float L = rl * loss_scale;
    loss_out[0] = L;
    if (loss_sum) loss_sum[0] += (double)L;
    bias_grad[0] = rg * 1.0f;
  }
  __syncthreads();  // the bias gradient (an element of g) is visible to the block
  for (int64_t i = t; i < n; i += 1024) {
    float pp = p[i], mm = m[i], vv = v[i];
    adam_elem(pp, g[i], mm, vv, h);
    p[i] = pp;
    m[i] = mm;
    v[i] = vv;
  }
  __syncthreads();  // every thread has read ctr[1]
  if (t == 0) {
    const int32_t s = ctr[1];
    ctr[0] = s;
    ctr[1] = s + 1;
  }
}

// Every row to `step` (epoch end / checkpoint / eval; deferred_flush_tile below). Rows
// already current cost 4 B. The per-step scalars of steps 1..step are staged once per block
// in LDS (one ds_read_b64 per replayed step instead of a dependent global load).
constexpr int kMaxLdsSteps = 8192;  // 64 KiB of float2

// tiled flush tuning (tools/build_variant.py): rows per batch = CTR_FLUSH_UNR wave-
// instructions (4 measured best: 2.59 ms at 1 replayed step, 4.46 ms at 20, C3 table)
#ifndef CTR_FLUSH_UNR
#define CTR_FLUSH_UNR 4
#endif

// The flush, tiled (what ctr_adam_deferred_flush launches): a wave owns 64 consecutive
// rows. Lane l holds last[base + l] and the linear weight's (p, m, v) of row base + l —
// coalesced 256-B accesses, replayed in-lane — and the [64, K] slabs of E, m_E, v_E stream
// through in float4 columns, UNR wave-instructions' worth of rows per batch: every load of
// a batch is issued before its replay, so each wave keeps 3 x UNR KiB in flight, and the
// replay of the batch's rows runs as one step loop over all of them (4 x UNR independent
// chains per lane). Tiles whose rows are all current are skipped on one vote; last[] is
// written back coalesced. Same adam_elem, same per-step scalars: bitwise the old pass.
template <int K4, int UNR, bool LDS_TAB>
__global__ __launch_bounds__(256) void deferred_flush_tile(
    float4* __restrict__ E, float4* __restrict__ mE, float4* __restrict__ vE,
    float* __restrict__ w, float* __restrict__ mw, float* __restrict__ vw, int64_t V,
    int32_t* __restrict__ last, int step, const float* __restrict__ tab, AdamHP h) {
  extern __shared__ __attribute__((aligned(16))) float2 s_tab[];
  if (LDS_TAB) {
    for (int i = threadIdx.x; i <= step; i += blockDim.x)
      s_tab[i] = reinterpret_cast<const float2*>(tab)[i];
    __syncthreads();
  }
  constexpr int RPI = kWave / K4;  // rows per wave-instruction
  constexpr int ITERS = K4;        // wave-instructions per 64-row tile
  static_assert(ITERS % UNR == 0, "batches of UNR instructions");
  const int lane = threadIdx.x & (kWave - 1);
  const int c = lane % K4, r_in = lane / K4;
  const int64_t waves = (int64_t)gridDim.x * (blockDim.x / kWave);
  const int64_t n_tiles = (V + kWave - 1) / kWave;
  auto set_step = [&](int t) {
    if (LDS_TAB) {
      const float2 v = s_tab[t];
      h.neg_step_size = v.x;
      h.inv_bc2_sqrt = v.y;
    } else {
      load_step(h, tab, t);
    }
  };
  for (int64_t tile = (int64_t)blockIdx.x * (blockDim.x / kWave) + threadIdx.x / kWave;
       tile < n_tiles; tile += waves) {
    const int64_t base = tile * kWave;
    const int64_t my = base + lane;
    const bool ok = my < V;
    const int from_l = ok ? last[my] : step;
    if (__all(from_l >= step)) continue;  // every row of the tile is current
    if (w && from_l < step) {
      float pp = w[my], mm = mw[my], vv = vw[my];
      for (int s = from_l + 1; s <= step; ++s) {
        set_step(s);
        adam_elem(pp, 0.f, mm, vv, h);
      }
      w[my] = pp; mw[my] = mm; vw[my] = vv;
    }
    // (measured: issuing batch b+1's loads before batch b's replay, through a second
    // register buffer, made the 20-step flush 12 % slower; the unprefetched batch loop is
    // kept — tools/_run_flush2.sh variants)
#pragma unroll 1
    for (int it0 = 0; it0 < ITERS; it0 += UNR) {
      float4 pp[UNR], mm[UNR], vv[UNR];
      int from[UNR];
      int64_t e[UNR];
      int f0 = step;
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const int r = (it0 + u) * RPI + r_in;
        from[u] = __shfl(from_l, r, kWave);  // lanes past V hold `step`: skipped
        e[u] = (base + r) * K4 + c;
        f0 = min(f0, from[u]);
        if (from[u] < step) {
          pp[u] = E[e[u]]; mm[u] = mE[e[u]]; vv[u] = vE[e[u]];
        }
      }
      for (int s = f0 + 1; s <= step; ++s) {
        set_step(s);
#pragma unroll
        for (int u = 0; u < UNR; ++u)
          if (s > from[u]) adam_replay_vec(pp[u], mm[u], vv[u], h);
      }
#pragma unroll
      for (int u = 0; u < UNR; ++u)
        if (from[u] < step) {
          E[e[u]] = pp[u]; mE[e[u]] = mm[u]; vE[e[u]] = vv[u];
        }
    }
    if (from_l < step) last[my] = step;
  }
}

// The flush, software-pipelined (build option CTR_FLUSH_PIPE=1, K4 >= 8; measured slower,
// kept for the record). The tile kernel's waves each load a batch, replay it, store it;
// at 20 replayed steps the flush measured close to the SUM of its row traffic and its replay
// (C3 table: 3.09 ms at 1 step, 4.33 at 20, 7.22 at 40), which suggested waves of a SIMD
// falling into step. Here each wave keeps the NEXT batch's loads in flight while it replays
// the current one: two register buffers of UNR float4 rows (UNR = 2 keeps four waves per
// SIMD at K = 64). Loads are unconditional — a row already current reads row 0's cached
// columns instead — so the compiler's in-order vmcnt counting waits for the current buffer
// only; stores stay predicated. A tile's NB batches are unrolled, the first batch of the
// next tile (and its rows' last[] / linear state, one tile ahead) is issued under the
// current tile's last batch; the linear weight's chain rides in the replay loop of a
// tile's first batch. Bitwise the tile kernel (tests/test_gpu_deferred.py), but slower:
// C3 table 4.62-4.68 vs 4.28-4.32 ms at 20 steps, 8.14-8.29 vs 7.26-7.50 at 40 (grids
// 512-4096 no better) — the replay per step costs more at UNR = 2, and the flush's
// counters (r02_flush_pmc.txt: VALU busy ~95 % of SIMD cycles at 20 steps, at ~1.8 GHz)
// say it is arithmetic-bound there, not waiting on its loads.
#ifndef CTR_FLUSH_PIPE
#define CTR_FLUSH_PIPE 0
#endif
#ifndef CTR_FLUSH_PIPE_UNR
#define CTR_FLUSH_PIPE_UNR 2
#endif

template <int UNR>
struct FlushBatch {
  float4 p[UNR], m[UNR], v[UNR];
  int from[UNR];
  int64_t e[UNR];
};

struct FlushTileMeta {  // the lane's own row of a tile: last[] and the linear weight's state
  int fl;
  float lp, lm, lv;
};

template <int K4, int UNR, bool LDS_TAB>
__global__ __launch_bounds__(256) void deferred_flush_pipe(
    float4* __restrict__ E, float4* __restrict__ mE, float4* __restrict__ vE,
    float* __restrict__ w, float* __restrict__ mw, float* __restrict__ vw, int64_t V,
    int32_t* __restrict__ last, int step, const float* __restrict__ tab, AdamHP h) {
  extern __shared__ __attribute__((aligned(16))) float2 s_tab[];
  if (LDS_TAB) {
    for (int i = threadIdx.x; i <= step; i += blockDim.x)
      s_tab[i] = reinterpret_cast<const float2*>(tab)[i];
    __syncthreads();
  }
  constexpr int RPI = kWave / K4;  // rows per wave-instruction
  constexpr int NB = K4 / UNR;     // batches per 64-row tile
  static_assert(K4 % UNR == 0 && NB % 2 == 0, "an even number of batches per tile");
  const int lane = threadIdx.x & (kWave - 1);
  const int c = lane % K4, r_in = lane / K4;
  const int64_t waves = (int64_t)gridDim.x * (blockDim.x / kWave);
  const int64_t n_tiles = (V + kWave - 1) / kWave;
  const int64_t t_first = (int64_t)blockIdx.x * (blockDim.x / kWave) + threadIdx.x / kWave;
  if (t_first >= n_tiles) return;  // wave-uniform, after the block's only barrier
  const int64_t t_last = t_first + (n_tiles - 1 - t_first) / waves * waves;
  auto set_step = [&](int t) {
    if (LDS_TAB) {
      const float2 v = s_tab[t];
      h.neg_step_size = v.x;
      h.inv_bc2_sqrt = v.y;
    } else {
      load_step(h, tab, t);
    }
  };
  auto load_meta = [&](int64_t tile, FlushTileMeta& M) {
    const int64_t my = tile * kWave + lane;
    const bool ok = my < V;
    const int64_t ms = ok ? my : 0;  // clamped: every lane loads a valid address
    const int f = last[ms];
    M.fl = ok ? f : step;            // lanes past V read as current
    if (w) {
      M.lp = w[ms];
      M.lm = mw[ms];
      M.lv = vw[ms];
    }
  };
  auto issue = [&](int64_t tile, int bi, const FlushTileMeta& M, FlushBatch<UNR>& X) {
    const int64_t base = tile * kWave;
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int r = (bi * UNR + u) * RPI + r_in;
      X.from[u] = __shfl(M.fl, r, kWave);
      X.e[u] = (base + r) * K4 + c;
      const int64_t el = X.from[u] < step ? X.e[u] : c;  // current rows: row 0, cached
      X.p[u] = E[el];
      X.m[u] = mE[el];
      X.v[u] = vE[el];
    }
  };
  auto replay_store = [&](int64_t tile, bool first, FlushTileMeta& M, FlushBatch<UNR>& X) {
    int f0 = step;
#pragma unroll
    for (int u = 0; u < UNR; ++u) f0 = min(f0, X.from[u]);
    const int fl_lin = (first && w) ? M.fl : step;
    f0 = min(f0, fl_lin);
    for (int s = f0 + 1; s <= step; ++s) {
      set_step(s);
      if (s > fl_lin) adam_elem(M.lp, 0.f, M.lm, M.lv, h);
#pragma unroll
      for (int u = 0; u < UNR; ++u)
        if (s > X.from[u]) adam_replay_vec(X.p[u], X.m[u], X.v[u], h);
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u)
      if (X.from[u] < step) {
        E[X.e[u]] = X.p[u];
        mE[X.e[u]] = X.m[u];
        vE[X.e[u]] = X.v[u];
      }
    if (first && M.fl < step) {  // fl < step only for rows below V
      const int64_t my = tile * kWave + lane;
      if (w) {
        w[my] = M.lp;
        mw[my] = M.lm;
        vw[my] = M.lv;
      }
      last[my] = step;
    }
  };
  FlushBatch<UNR> X0, X1;
  FlushTileMeta cur, nxt;
  load_meta(t_first, cur);
  load_meta(t_first + waves <= t_last ? t_first + waves : t_last, nxt);
  issue(t_first, 0, cur, X0);
  for (int64_t tile = t_first; tile <= t_last; tile += waves) {
    const int64_t nt = tile + waves <= t_last ? tile + waves : t_last;  // clamped: the last
    // tile's prefetch re-reads a batch it never replays
#pragma unroll
    for (int bi = 0; bi < NB; ++bi) {
      FlushBatch<UNR>& now = (bi & 1) ? X1 : X0;
      FlushBatch<UNR>& ahead = (bi & 1) ? X0 : X1;
      if (bi + 1 < NB)
        issue(tile, bi + 1, cur, ahead);
      else
        issue(nt, 0, nxt, ahead);
      replay_store(tile, bi == 0, cur, now);
    }
    cur = nxt;
    load_meta(nt + waves <= t_last ? nt + waves : t_last, nxt);
  }
}

// Any K: a thread per row (rows list, or all rows when rows == NULL).
template <bool APPLY>
__global__ __launch_bounds__(256) void deferred_scalar(
    float* __restrict__ E, float* __restrict__ mE, float* __restrict__ vE, float* __restrict__ w,
    float* __restrict__ mw, float* __restrict__ vw, int64_t n_rows, int K,
    int32_t* __restrict__ last, const int32_t* __restrict__ rows,
    const int32_t* __restrict__ num_unique, const float* __restrict__ grows,
    const float* __restrict__ glin, int step_val, const int32_t* __restrict__ step_ptr,
    const float* __restrict__ tab, AdamHP h) {
  const int step = step_ptr ? *step_ptr : step_val;
  const int64_t n = rows ? (int64_t)*num_unique : n_rows;
  const int target = APPLY ? step - 1 : step;
  for (int64_t u = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; u < n;
       u += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = rows ? (int64_t)rows[u] : u;
    const int from = last[r];
    if (!APPLY && from >= target) continue;
    for (int k = 0; k < K; ++k) {
      const int64_t e = r * K + k;
      float pp = E[e], mm = mE[e], vv = vE[e];
      for (int s = from + 1; s <= target; ++s) {
        load_step(h, tab, s);
        adam_elem(pp, 0.f, mm, vv, h);
      }
      if (APPLY) {
        load_step(h, tab, step);
        adam_elem(pp, grows[u * K + k], mm, vv, h);
      }
      E[e] = pp; mE[e] = mm; vE[e] = vv;
    }
    if (w) {
      float pp = w[r], mm = mw[r], vv = vw[r];
      for (int s = from + 1; s <= target; ++s) {
        load_step(h, tab, s);
        adam_elem(pp, 0.f, mm, vv, h);
      }
      if (APPLY) {
        load_step(h, tab, step);
        adam_elem(pp, glin[u], mm, vv, h);
      }
      w[r] = pp; mw[r] = mm; vw[r] = vv;
    }
    last[r] = APPLY ? step : target;
  }
}


}  // namespace ctr

using namespace ctr;

static int adam_dense_impl(float* p, const float* g, float* m, float* v, int64_t n,
                           double step_size, double bc2_sqrt, const float* step_table,
                           const int32_t* step_ptr, double beta1, double beta2, double eps,
                           double weight_decay, const PlaneViews& pv, ctr_stream_t stream) {
  CTR_REQUIRE(n >= 0, "ctr_adam_dense: n < 0");
  if (n == 0) return CTR_OK;
  CTR_REQUIRE(p && g && m && v, "ctr_adam_dense: null pointer");
  CTR_REQUIRE(step_ptr ? step_table != nullptr : bc2_sqrt > 0.0,
              "ctr_adam_dense: bc2_sqrt must be > 0 (or step_table given with step_ptr)");
  const AdamHP h = make_hp(step_ptr ? 1.0 : step_size, step_ptr ? 1.0 : bc2_sqrt, beta1, beta2,
                           eps, weight_decay);
  hipStream_t st = as_stream(stream);
  const bool al = ((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) % 16 == 0;
  CTR_REQUIRE(pv.n == 0 || (al && n % 4 == 0),
              "ctr_adam_dense_planes: needs 16-B aligned vectors and n %% 4 == 0");
  int64_t done = 0;
  if (al && n >= 4) {
    const int64_t n4 = n / 4;
    const unsigned grid = (unsigned)std::min<int64_t>(ceil_div(n4, 256), 4096);
    hipLaunchKernelGGL(adam_dense_vec, grid, 256, 0, st, reinterpret_cast<float4*>(p),
                       reinterpret_cast<const float4*>(g), reinterpret_cast<float4*>(m),
                       reinterpret_cast<float4*>(v), n4, h, step_table, step_ptr, pv);
    CTR_LAUNCH_CHECK("adam_dense_vec");
    done = n4 * 4;
  }
  if (done < n) {
    const unsigned grid = (unsigned)std::min<int64_t>(ceil_div(n - done, 256), 4096);
    hipLaunchKernelGGL(adam_dense_scalar, grid, 256, 0, st, p, g, m, v, done, n, h, step_table,
                       step_ptr);
    CTR_LAUNCH_CHECK("adam_dense_scalar");
  }
  return CTR_OK;
}

extern "C" int ctr_adam_dense(float* p, const float* g, float* m, float* v, int64_t n,
                              double step_size, double bc2_sqrt, const float* step_table,
                              const int32_t* step_ptr, double beta1, double beta2, double eps,
                              double weight_decay, ctr_stream_t stream) {
  PlaneViews pv{};
  return adam_dense_impl(p, g, m, v, n, step_size, bc2_sqrt, step_table, step_ptr, beta1, beta2,
                         eps, weight_decay, pv, stream);
}

extern "C" int ctr_adam_dense_planes(float* p, const float* g, float* m, float* v, int64_t n,
                                     double step_size, double bc2_sqrt, const float* step_table,
                                     const int32_t* step_ptr, double beta1, double beta2,
                                     double eps, double weight_decay, const ctr_plane_view* views,
                                     int n_views, ctr_stream_t stream) {
  CTR_REQUIRE(n_views >= 0 && n_views <= kMaxPlaneViews && (n_views == 0 || views),
              "ctr_adam_dense_planes: 0..%d plane views", kMaxPlaneViews);
  PlaneViews pv{};
  pv.n = n_views;
  for (int j = 0; j < n_views; ++j) {
    const ctr_plane_view& w = views[j];
    const ctr_planes& q = w.planes;
    CTR_REQUIRE(w.offset >= 0 && w.offset % 4 == 0 && w.rows > 0 && w.cols > 0 &&
                    w.offset + w.rows * w.cols <= n,
                "ctr_adam_dense_planes: view %d outside the vector or not float4-aligned", j);
    CTR_REQUIRE(q.data && (uintptr_t)q.data % 16 == 0 && q.ld % 4 == 0 && q.ld >= w.cols &&
                    q.rows >= w.rows && q.plane_stride >= q.rows * q.ld,
                "ctr_adam_dense_planes: view %d: bad plane layout", j);
    pv.off[j] = w.offset;
    pv.len[j] = w.rows * w.cols;
    pv.cols[j] = w.cols;
    pv.ld[j] = q.ld;
    pv.ps[j] = q.plane_stride;
    pv.d[j] = static_cast<uint16_t*>(q.data);
  }
  return adam_dense_impl(p, g, m, v, n, step_size, bc2_sqrt, step_table, step_ptr, beta1, beta2,
                         eps, weight_decay, pv, stream);
}

extern "C" int ctr_adam_embedding(float* emb, float* m_emb, float* v_emb, float* lin, float* m_lin,
                                  float* v_lin, int64_t V, int K, int32_t* rowmap,
                                  const float* grad_rows, const float* grad_lin,
                                  double step_size, double bc2_sqrt, const float* step_table,
                                  const int32_t* step_ptr, double beta1, double beta2,
                                  double eps, double weight_decay, ctr_stream_t stream) {
  CTR_REQUIRE(emb && m_emb && v_emb && rowmap && grad_rows, "ctr_adam_embedding: null pointer");
  CTR_REQUIRE(V > 0 && K > 0, "ctr_adam_embedding: bad sizes");
  CTR_REQUIRE((lin && m_lin && v_lin && grad_lin) || (!lin && !m_lin && !v_lin),
              "ctr_adam_embedding: linear table pointers must be all set or all NULL");
  CTR_REQUIRE(step_ptr ? step_table != nullptr : bc2_sqrt > 0.0,
              "ctr_adam_embedding: bc2_sqrt must be > 0 (or step_table given with step_ptr)");
  const AdamHP h = make_hp(step_ptr ? 1.0 : step_size, step_ptr ? 1.0 : bc2_sqrt, beta1, beta2,
                           eps, weight_decay);
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
                     reinterpret_cast<const float4*>(grad_rows), grad_lin, h, step_table,      \
                     step_ptr)
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
                     V, K, rowmap, grad_rows, grad_lin, h, step_table, step_ptr);
  CTR_LAUNCH_CHECK("adam_embedding_scalar");
  return CTR_OK;
}

// The owner side of a row-sharded step: each unique row's gradient is the sum of its few
// received entries (at most one per requester: a requester sends each row once), summed in
// plan order — source rank, then position — straight in the lane group that then replays
// the row's missed steps and applies this one (deferred_rows_vec<APPLY>'s update, the same
// adam_vec chain). One launch instead of the chunked segmented sums + fused apply, whose
// chunk machinery pays off for long segments (a batch's hot rows), not for runs of <= N.
// skip_row (the owner's spare row, the target of every padding entry: a long segment whose
// value is never used) is left alone. out / out_lin (optional): the sums.
template <int K4>
__global__ __launch_bounds__(256) void deferred_entries_vec(
    float4* __restrict__ E, float4* __restrict__ mE, float4* __restrict__ vE,
    float* __restrict__ w, float* __restrict__ mw, float* __restrict__ vw,
    int32_t* __restrict__ last, const int32_t* __restrict__ rows,
    const int32_t* __restrict__ num_unique, const int32_t* __restrict__ seg_offsets,
    const int32_t* __restrict__ sorted_entries, const float4* __restrict__ vals,
    const float* __restrict__ vals_lin, int64_t run_len, int64_t chunk, int64_t skip_row,
    int step_val,
    const int32_t* __restrict__ step_ptr, const float* __restrict__ tab, AdamHP h,
    float4* __restrict__ out, float* __restrict__ out_lin) {
  constexpr int kTabWin = CTR_ROWS_TAB_WIN > 0 ? CTR_ROWS_TAB_WIN : 1;
  __shared__ float2 s_tab[kTabWin];
  const int c = threadIdx.x % K4;
  const int64_t groups = (int64_t)gridDim.x * (blockDim.x / K4);
  const int U = *num_unique;
  const int step = step_ptr ? *step_ptr : step_val;
  const int target = step - 1;
  const int win0 = CTR_ROWS_TAB_WIN > 0 ? max(0, target - kTabWin + 1) : target + 1;
  if (threadIdx.x < kTabWin && win0 + (int)threadIdx.x <= target)
    s_tab[threadIdx.x] = reinterpret_cast<const float2*>(tab)[win0 + threadIdx.x];
  __syncthreads();
  for (int64_t u = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) / K4; u < U; u += groups) {
    const int64_t r = rows[u];
    if (r == skip_row) continue;
    const int64_t e = r * K4 + c;
    const int from = last[r];
    float4 pp = E[e], mm = mE[e], vv = vE[e];
    float pw = 0.f, mws = 0.f, vws = 0.f;
    const bool own_lin = w && c == 0;
    if (own_lin) {
      pw = w[r]; mws = mw[r]; vws = vw[r];
    }
    // entry s: row s of vals [entries][K] and vals_lin[s]; chunked (run_len > 0): row
    // s % run_len of chunk s / run_len (chunk floats each: run_len rows, then their linear
    // values — the exchange's receive buffer as it arrived)
    auto row_of = [&](int64_t s) -> const float4* {
      if (run_len == 0) return vals + s * K4;
      const int64_t j = s / run_len;
      return reinterpret_cast<const float4*>(reinterpret_cast<const float*>(vals) + j * chunk) +
             (s - j * run_len) * K4;
    };
    auto lin_of = [&](int64_t s) -> float {
      if (run_len == 0) return vals_lin[s];
      const int64_t j = s / run_len;
      return reinterpret_cast<const float*>(vals)[j * chunk + run_len * 4 * K4 + (s - j * run_len)];
    };
    const int p0 = seg_offsets[u], p1 = seg_offsets[u + 1];
    int64_t s = sorted_entries[p0];
    float4 g = row_of(s)[c];
    float gl = own_lin ? lin_of(s) : 0.f;
    for (int p = p0 + 1; p < p1; ++p) {
      s = sorted_entries[p];
      const float4 x = row_of(s)[c];
      g.x += x.x; g.y += x.y; g.z += x.z; g.w += x.w;
      if (own_lin) gl += lin_of(s);
    }
    if (out) out[u * K4 + c] = g;
    if (out_lin && c == 0) out_lin[u] = gl;
    for (int t = from + 1; t <= target; ++t) {
      if (t >= win0) {
        const float2 v = s_tab[t - win0];
        h.neg_step_size = v.x;
        h.inv_bc2_sqrt = v.y;
      } else {
        load_step(h, tab, t);
      }
      adam_replay_vec(pp, mm, vv, h);
      if (own_lin) adam_elem(pw, 0.f, mws, vws, h);
    }
    load_step(h, tab, step);
    adam_vec(pp, g, mm, vv, h);
    if (own_lin) adam_elem(pw, gl, mws, vws, h);
    E[e] = pp; mE[e] = mm; vE[e] = vv;
    if (own_lin) {
      w[r] = pw; mw[r] = mws; vw[r] = vws;
    }
    if (c == 0) last[r] = step;
  }
}

static bool deferred_vec_ok(int K, const void* a, const void* b, const void* c, const void* g) {
  return K % 4 == 0 && K / 4 <= 64 && (kWave % (K / 4)) == 0 &&
         ((uintptr_t)a | (uintptr_t)b | (uintptr_t)c | (uintptr_t)g) % 16 == 0;
}

extern "C" int ctr_adam_deferred_rows(float* emb, float* m_emb, float* v_emb, float* lin,
                                      float* m_lin, float* v_lin, int64_t V, int K, int32_t* last,
                                      const ctr_sparse_plan* plan, const float* grad_rows,
                                      const float* grad_lin, int64_t step, const int32_t* step_ptr,
                                      const float* step_table, double beta1, double beta2,
                                      double eps, double weight_decay, ctr_stream_t stream) {
  CTR_REQUIRE(emb && m_emb && v_emb && last && step_table, "ctr_adam_deferred_rows: null pointer");
  CTR_REQUIRE(plan && plan->unique_rows && plan->num_unique, "ctr_adam_deferred_rows: bad plan");
  CTR_REQUIRE(V > 0 && K > 0 && (step_ptr || (step >= 1 && step < (int64_t(1) << 31))),
              "ctr_adam_deferred_rows: bad sizes");
  CTR_REQUIRE((lin && m_lin && v_lin) || (!lin && !m_lin && !v_lin),
              "ctr_adam_deferred_rows: linear table pointers must be all set or all NULL");
  CTR_REQUIRE(!grad_rows || !lin || grad_lin, "ctr_adam_deferred_rows: grad_lin missing");
  if (plan->S == 0) return CTR_OK;
  const AdamHP h = make_hp(1.0, 1.0, beta1, beta2, eps, weight_decay);
  hipStream_t st = as_stream(stream);
  const bool apply = grad_rows != nullptr;
  const int64_t n = plan->S;  // upper bound on unique rows
  if (deferred_vec_ok(K, emb, m_emb, v_emb, grad_rows)) {
    const int K4 = K / 4;
    const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>(ceil_div(n * K4, 256), 8192));
#define CTR_DEF_ROWS(K4_)                                                                        \
  if (apply)                                                                                     \
    hipLaunchKernelGGL((deferred_rows_vec<K4_, true>), grid, 256, 0, st,                         \
                       reinterpret_cast<float4*>(emb), reinterpret_cast<float4*>(m_emb),         \
                       reinterpret_cast<float4*>(v_emb), lin, m_lin, v_lin, last,                \
                       plan->unique_rows, plan->num_unique,                                      \
                       reinterpret_cast<const float4*>(grad_rows), grad_lin, (int)step,          \
                       step_ptr, step_table, h);                                                 \
  else                                                                                           \
    hipLaunchKernelGGL((deferred_rows_vec<K4_, false>), grid, 256, 0, st,                        \
                       reinterpret_cast<float4*>(emb), reinterpret_cast<float4*>(m_emb),         \
                       reinterpret_cast<float4*>(v_emb), lin, m_lin, v_lin, last,                \
                       plan->unique_rows, plan->num_unique, nullptr, nullptr, (int)step,         \
                       step_ptr, step_table, h)
    switch (K4) {
      case 1: CTR_DEF_ROWS(1); break;
      case 2: CTR_DEF_ROWS(2); break;
      case 4: CTR_DEF_ROWS(4); break;
      case 8: CTR_DEF_ROWS(8); break;
      case 16: CTR_DEF_ROWS(16); break;
      case 32: CTR_DEF_ROWS(32); break;
      case 64: CTR_DEF_ROWS(64); break;
    }
#undef CTR_DEF_ROWS
    CTR_LAUNCH_CHECK("deferred_rows_vec");
    return CTR_OK;
  }
  const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>(ceil_div(n, 256), 8192));
  if (apply)
    hipLaunchKernelGGL(deferred_scalar<true>, grid, 256, 0, st, emb, m_emb, v_emb, lin, m_lin,
                       v_lin, n, K, last, plan->unique_rows, plan->num_unique, grad_rows, grad_lin,
                       (int)step, step_ptr, step_table, h);
  else
    hipLaunchKernelGGL(deferred_scalar<false>, grid, 256, 0, st, emb, m_emb, v_emb, lin, m_lin,
                       v_lin, n, K, last, plan->unique_rows, plan->num_unique, nullptr, nullptr,
                       (int)step, step_ptr, step_table, h);
  CTR_LAUNCH_CHECK("deferred_scalar");
  return CTR_OK;
}

extern "C" int ctr_adam_deferred_entries(float* emb, float* m_emb, float* v_emb, float* lin,
                                         float* m_lin, float* v_lin, int64_t V, int K,
                                         int32_t* last, const ctr_sparse_plan* plan,
                                         const float* vals, const float* vals_lin,
                                         int64_t run_len, int64_t chunk, int64_t skip_row,
                                         int64_t step, const int32_t* step_ptr,
                                         const float* step_table, double beta1, double beta2,
                                         double eps, double weight_decay, float* out,
                                         float* out_lin, ctr_stream_t stream) {
  CTR_REQUIRE(emb && m_emb && v_emb && last && step_table && vals,
              "ctr_adam_deferred_entries: null pointer");
  CTR_REQUIRE(plan && plan->unique_rows && plan->num_unique && plan->seg_offsets &&
                  plan->sorted_slots,
              "ctr_adam_deferred_entries: bad plan");
  CTR_REQUIRE(V > 0 && K > 0 && (step_ptr || (step >= 1 && step < (int64_t(1) << 31))),
              "ctr_adam_deferred_entries: bad sizes");
  CTR_REQUIRE((lin && m_lin && v_lin && (vals_lin || run_len > 0)) || (!lin && !m_lin && !v_lin),
              "ctr_adam_deferred_entries: linear table pointers (and vals_lin) all set or all NULL");
  CTR_REQUIRE(run_len >= 0 && (run_len == 0 || (chunk % 4 == 0 &&
                                                 chunk >= run_len * K + (lin ? run_len : 0))),
              "ctr_adam_deferred_entries: chunk must hold run_len rows (+ their linear values)");
  CTR_REQUIRE(deferred_vec_ok(K, emb, m_emb, v_emb, vals) && (!out || (uintptr_t)out % 16 == 0),
              "ctr_adam_deferred_entries: needs K %% 4 == 0, (K/4) | 64 and 16-B aligned rows");
  if (plan->S == 0) return CTR_OK;
  const AdamHP h = make_hp(1.0, 1.0, beta1, beta2, eps, weight_decay);
  const int K4 = K / 4;
  const int64_t n = plan->S;  // upper bound on unique rows
  const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>(ceil_div(n * K4, 256), 8192));
#define CTR_DEF_ENTRIES(K4_)                                                                    \
  hipLaunchKernelGGL((deferred_entries_vec<K4_>), grid, 256, 0, as_stream(stream),              \
                     reinterpret_cast<float4*>(emb), reinterpret_cast<float4*>(m_emb),          \
                     reinterpret_cast<float4*>(v_emb), lin, m_lin, v_lin, last,                 \
                     plan->unique_rows, plan->num_unique, plan->seg_offsets, plan->sorted_slots, \
                     reinterpret_cast<const float4*>(vals), vals_lin, run_len, chunk, skip_row, \
                     (int)step,                                                                  \
                     step_ptr, step_table, h, reinterpret_cast<float4*>(out), out_lin)
  switch (K4) {
    case 1: CTR_DEF_ENTRIES(1); break;
    case 2: CTR_DEF_ENTRIES(2); break;
    case 4: CTR_DEF_ENTRIES(4); break;
    case 8: CTR_DEF_ENTRIES(8); break;
    case 16: CTR_DEF_ENTRIES(16); break;
    case 32: CTR_DEF_ENTRIES(32); break;
    case 64: CTR_DEF_ENTRIES(64); break;
  }
#undef CTR_DEF_ENTRIES
  CTR_LAUNCH_CHECK("deferred_entries_vec");
  return CTR_OK;
}

extern "C" int ctr_adam_deferred_flush(float* emb, float* m_emb, float* v_emb, float* lin,
                                       float* m_lin, float* v_lin, int64_t V, int K, int32_t* last,
                                       int64_t step, const float* step_table, double beta1,
                                       double beta2, double eps, double weight_decay,
                                       ctr_stream_t stream) {
  CTR_REQUIRE(emb && m_emb && v_emb && last && step_table, "ctr_adam_deferred_flush: null pointer");
  CTR_REQUIRE(V > 0 && K > 0 && step >= 0 && step < (int64_t(1) << 31),
              "ctr_adam_deferred_flush: bad sizes");
  CTR_REQUIRE((lin && m_lin && v_lin) || (!lin && !m_lin && !v_lin),
              "ctr_adam_deferred_flush: linear table pointers must be all set or all NULL");
  if (step == 0) return CTR_OK;
  const AdamHP h = make_hp(1.0, 1.0, beta1, beta2, eps, weight_decay);
  hipStream_t st = as_stream(stream);
  if (deferred_vec_ok(K, emb, m_emb, v_emb, nullptr)) {
    const int K4 = K / 4;
    const int64_t n_tiles = ceil_div(V, kWave);
    const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>(ceil_div(n_tiles, 4), 8192));
    const bool lds = step < kMaxLdsSteps;
    const size_t lds_bytes = lds ? (size_t)(step + 1) * sizeof(float2) : 0;
    if (CTR_FLUSH_PIPE && K4 >= 8) {
      // one generation of resident waves less a little (a wave's first batch is its only
      // unhidden load): 256 CUs x 4 blocks of 4 waves at <= 128 VGPRs; CTR_FLUSH_GRID tunes
      static const int64_t pipe_grid = [] {
        const char* s = std::getenv("CTR_FLUSH_GRID");
        return s ? std::max<int64_t>(1, std::atoll(s)) : int64_t(1024);
      }();
      const unsigned pgrid = (unsigned)std::max<int64_t>(1, std::min<int64_t>(ceil_div(n_tiles, 4), pipe_grid));
#define CTR_DEF_PIPE(K4_)                                                                     \
  if (lds)                                                                                    \
    hipLaunchKernelGGL((deferred_flush_pipe<K4_, CTR_FLUSH_PIPE_UNR, true>), pgrid, 256,      \
                       lds_bytes, st, reinterpret_cast<float4*>(emb),                         \
                       reinterpret_cast<float4*>(m_emb), reinterpret_cast<float4*>(v_emb), lin, \
                       m_lin, v_lin, V, last, (int)step, step_table, h);                      \
  else                                                                                        \
    hipLaunchKernelGGL((deferred_flush_pipe<K4_, CTR_FLUSH_PIPE_UNR, false>), pgrid, 256, 0,  \
                       st, reinterpret_cast<float4*>(emb), reinterpret_cast<float4*>(m_emb),  \
                       reinterpret_cast<float4*>(v_emb), lin, m_lin, v_lin, V, last,          \
                       (int)step, step_table, h)
      switch (K4) {
        case 8: CTR_DEF_PIPE(8); break;
        case 16: CTR_DEF_PIPE(16); break;
        case 32: CTR_DEF_PIPE(32); break;
        case 64: CTR_DEF_PIPE(64); break;
      }
#undef CTR_DEF_PIPE
      CTR_LAUNCH_CHECK("deferred_flush_pipe");
      return CTR_OK;
    }
#define CTR_DEF_FLUSH(K4_, UNR_)                                                           \
  if (lds)                                                                                      \
    hipLaunchKernelGGL((deferred_flush_tile<K4_, UNR_, true>), grid, 256, lds_bytes, st,        \
                       reinterpret_cast<float4*>(emb), reinterpret_cast<float4*>(m_emb),        \
                       reinterpret_cast<float4*>(v_emb), lin, m_lin, v_lin, V, last, (int)step, \
                       step_table, h);                                                          \
  else                                                                                          \
    hipLaunchKernelGGL((deferred_flush_tile<K4_, UNR_, false>), grid, 256, 0, st,               \
                       reinterpret_cast<float4*>(emb), reinterpret_cast<float4*>(m_emb),        \
                       reinterpret_cast<float4*>(v_emb), lin, m_lin, v_lin, V, last, (int)step, \
                       step_table, h)
    switch (K4) {
      case 1: CTR_DEF_FLUSH(1, 1); break;
      case 2: CTR_DEF_FLUSH(2, 2); break;
      case 4: CTR_DEF_FLUSH(4, 4); break;
      case 8: CTR_DEF_FLUSH(8, CTR_FLUSH_UNR); break;
      case 16: CTR_DEF_FLUSH(16, CTR_FLUSH_UNR); break;
      case 32: CTR_DEF_FLUSH(32, CTR_FLUSH_UNR); break;
      case 64: CTR_DEF_FLUSH(64, CTR_FLUSH_UNR); break;
    }
#undef CTR_DEF_FLUSH
    CTR_LAUNCH_CHECK("deferred_flush_tile");
    return CTR_OK;
  }
  const unsigned grid = (unsigned)std::min<int64_t>(ceil_div(V, 256), 8192);
  hipLaunchKernelGGL(deferred_scalar<false>, grid, 256, 0, st, emb, m_emb, v_emb, lin, m_lin,
                     v_lin, V, K, last, nullptr, nullptr, nullptr, nullptr, (int)step, nullptr,
                     step_table, h);
  CTR_LAUNCH_CHECK("deferred_flush_scalar");
  return CTR_OK;
}

static int launch_catchup_wave(float* emb, float* m_emb, float* v_emb, float* lin, float* m_lin,
                               float* v_lin, int64_t V, int K, int32_t* last, const void* idx,
                               int idx_type, int64_t S, const int32_t* owner,
                               const int32_t* step_ptr, const float* step_table, AdamHP h,
                               hipStream_t st, int64_t max_blocks = 8192);

extern "C" int ctr_adam_deferred_catchup_ids(float* emb, float* m_emb, float* v_emb, float* lin,
                                             float* m_lin, float* v_lin, int64_t V, int K,
                                             int32_t* last, const void* idx, int idx_type,
                                             int64_t S, int32_t* owner, const int32_t* step_ptr,
                                             const float* step_table, double beta1, double beta2,
                                             double eps, double weight_decay,
                                             ctr_stream_t stream) {
  CTR_REQUIRE(emb && m_emb && v_emb && last && owner && step_ptr && step_table,
              "ctr_adam_deferred_catchup_ids: null pointer");
  CTR_REQUIRE(V > 0 && V < (int64_t(1) << 31) && K > 0 && S >= 0 && S < (int64_t(1) << 31),
              "ctr_adam_deferred_catchup_ids: bad sizes");
  CTR_REQUIRE((lin && m_lin && v_lin) || (!lin && !m_lin && !v_lin),
              "ctr_adam_deferred_catchup_ids: linear table pointers must be all set or all NULL");
  CTR_REQUIRE(idx_type == CTR_IDX_I32 || idx_type == CTR_IDX_I64, "bad idx_type %d", idx_type);
  CTR_REQUIRE(deferred_vec_ok(K, emb, m_emb, v_emb, nullptr),
              "ctr_adam_deferred_catchup_ids: needs K %% 4 == 0, (K/4) | 64 and 16-B rows");
  if (S == 0) return CTR_OK;
  const AdamHP h = make_hp(1.0, 1.0, beta1, beta2, eps, weight_decay);
  hipStream_t st = as_stream(stream);
  const unsigned gm = (unsigned)std::min<int64_t>(ceil_div(S, 256), 4096);
  if (idx_type == CTR_IDX_I64)
    hipLaunchKernelGGL(deferred_mark_kernel<int64_t>, gm, 256, 0, st,
                       static_cast<const int64_t*>(idx), S, V, owner);
  else
    hipLaunchKernelGGL(deferred_mark_kernel<int32_t>, gm, 256, 0, st,
                       static_cast<const int32_t*>(idx), S, V, owner);
  CTR_LAUNCH_CHECK("deferred_mark_kernel");
  return launch_catchup_wave(emb, m_emb, v_emb, lin, m_lin, v_lin, V, K, last, idx, idx_type, S,
                             owner, step_ptr, step_table, h, st);
}

static int launch_catchup_wave(float* emb, float* m_emb, float* v_emb, float* lin, float* m_lin,
                               float* v_lin, int64_t V, int K, int32_t* last, const void* idx,
                               int idx_type, int64_t S, const int32_t* owner,
                               const int32_t* step_ptr, const float* step_table, AdamHP h,
                               hipStream_t st, int64_t max_blocks) {
  const int K4 = K / 4;
  // one lane per slot: S / 256 blocks of 4 waves (a wave re-loops when S exceeds the grid)
  const unsigned grid =
      (unsigned)std::max<int64_t>(1, std::min<int64_t>(ceil_div(S, 256), max_blocks));
#define CTR_CATCHUP(IT, K4_)                                                                   \
  hipLaunchKernelGGL((deferred_catchup_wave<IT, K4_, 2>), grid, 256, 0, st,                    \
                     reinterpret_cast<float4*>(emb), reinterpret_cast<float4*>(m_emb),         \
                     reinterpret_cast<float4*>(v_emb), lin, m_lin, v_lin, last,                \
                     static_cast<const IT*>(idx), S, V, owner, step_ptr, step_table, h)
#define CTR_CATCHUP_K(IT)                  \
  switch (K4) {                            \
    case 1: CTR_CATCHUP(IT, 1); break;     \
    case 2: CTR_CATCHUP(IT, 2); break;     \
    case 4: CTR_CATCHUP(IT, 4); break;     \
    case 8: CTR_CATCHUP(IT, 8); break;     \
    case 16: CTR_CATCHUP(IT, 16); break;   \
    case 32: CTR_CATCHUP(IT, 32); break;   \
    case 64: CTR_CATCHUP(IT, 64); break;   \
  }
  if (idx_type == CTR_IDX_I64) {
    CTR_CATCHUP_K(int64_t)
  } else {
    CTR_CATCHUP_K(int32_t)
  }
#undef CTR_CATCHUP_K
#undef CTR_CATCHUP
  CTR_LAUNCH_CHECK("deferred_catchup_wave");
  return CTR_OK;
}

extern "C" int ctr_step_begin(int32_t* step_ctr, ctr_stream_t stream) {
  CTR_REQUIRE(step_ctr, "ctr_step_begin: null pointer");
  hipLaunchKernelGGL(step_begin_kernel, 1, 1, 0, as_stream(stream), step_ctr);
  CTR_LAUNCH_CHECK("step_begin_kernel");
  return CTR_OK;
}

extern "C" int ctr_step_end(int32_t* step_ctr, ctr_stream_t stream) {
  CTR_REQUIRE(step_ctr, "ctr_step_end: null pointer");
  hipLaunchKernelGGL(step_end_kernel, 1, 1, 0, as_stream(stream), step_ctr, nullptr, nullptr);
  CTR_LAUNCH_CHECK("step_end_kernel");
  return CTR_OK;
}

extern "C" int ctr_step_end_loss(int32_t* step_ctr, const float* loss, double* loss_sum,
                                 ctr_stream_t stream) {
  CTR_REQUIRE(step_ctr && loss && loss_sum, "ctr_step_end_loss: null pointer");
  hipLaunchKernelGGL(step_end_kernel, 1, 1, 0, as_stream(stream), step_ctr, loss, loss_sum);
  CTR_LAUNCH_CHECK("step_end_kernel");
  return CTR_OK;
}

extern "C" int ctr_fm_step_tail(const float* loss_elem, const float* gz, int64_t B,
                                float loss_scale, float* loss_out, float* bias_grad, float* p,
                                const float* g, float* m, float* v, int64_t n,
                                const float* step_table, int32_t* step_ctr, double beta1,
                                double beta2, double eps, double weight_decay,
                                double* loss_sum, ctr_stream_t stream) {
  CTR_REQUIRE(loss_elem && gz && loss_out && bias_grad && step_table && step_ctr && B >= 0,
              "ctr_fm_step_tail: bad arguments");
  CTR_REQUIRE(n >= 0 && (n == 0 || (p && g && m && v)), "ctr_fm_step_tail: bad dense vector");
  const AdamHP h = make_hp(0.0, 1.0, beta1, beta2, eps, weight_decay);
  hipLaunchKernelGGL(fm_step_tail_kernel, 1, 1024, 0, as_stream(stream), loss_elem, gz, B,
                     loss_scale, loss_out, bias_grad, p, g, m, v, n, h, step_table, step_ctr,
                     loss_sum);
  CTR_LAUNCH_CHECK("fm_step_tail_kernel");
  return CTR_OK;
}

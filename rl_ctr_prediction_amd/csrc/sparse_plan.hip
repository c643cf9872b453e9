// Sparse plan of a batch: the stable grouping of the S = B*F slots by
// embedding row that embedding_dense_backward performs implicitly. Output (ctr_sparse_plan):
// slots sorted by (row, slot), the sorted rows, each position's segment ordinal, the unique
// rows in ascending order and their segment offsets — bit-identical to numpy's stable
// argsort + unique (tests/test_gpu_kernels.py).
//
// Two builds, the same plan bit for bit: the column plan (ctr_sparse_plan_build_cols, below:
// a batch's [B][F] ids sorted per column in LDS, then merged — what the trainers use) and the
// flat LSD plan (ctr_sparse_plan_build: any id vector). The flat plan is an
// LSD radix sort, 8-bit digits (kPlanBits), two launches per pass and no
// inter-workgroup hand-off inside a launch (a cross-XCD look-back chain costs ~1 us per hop
// on gfx950; a kernel boundary ~1.5 us):
//   radix_hist:    per tile (256 threads x IPT keys) the 256-bin digit histogram, LDS
//                  integer atomics (order-free, so deterministic counts) -> hist[tile][256]
//   radix_scatter: each block scans the tile histograms itself (coalesced 1-KB rows, one
//                  digit per thread) for its global digit bases, ranks its keys stably with
//                  wave ballots (8 ballots give the lanes holding the same digit; popcount
//                  below the lane = rank), and scatters (key, slot).
// Keys of a tile are striped (item i of thread t = tile + i*256 + t), so (item, wave,
// lane) order is input order and the ranking is stable. Pass 0 reads the feature ids
// directly (int64 or int32; the slot index is the value), the last pass writes the plan.
// Then two launches turn the sorted rows into segments (head counts per tile, then a
// block scan that writes pos_seg / unique_rows / seg_offsets / num_unique).
#include "ctr_common.h"

namespace ctr {

constexpr int kSortThreads = 256;
constexpr int kSortWaves = kSortThreads / kWave;

// Digit width (8 bits = 256 bins: kPlanBits below).
template <int BITS>
struct Radix {
  static constexpr int kBins = 1 << BITS;
  static constexpr int kDPT = kBins / kSortThreads;  // digits owned per thread (1 or 8)
};

struct RadixPass {
  const void* idx;     // pass 0: feature ids
  int idx_type;
  int64_t V;
  const uint32_t* keys_in;
  const int32_t* vals_in;
  uint32_t* keys_out;
  int32_t* vals_out;
  int32_t* hist;       // [n_tiles][bins]
  int64_t S;
  int n_tiles;
  int shift;
  int32_t* err;
};

template <bool FIRST>
__device__ __forceinline__ uint32_t radix_key(const RadixPass& a, int64_t i, int32_t* err) {
  if (FIRST) {
    return a.idx_type == CTR_IDX_I64
               ? (uint32_t)load_row(static_cast<const int64_t*>(a.idx), i, a.V, err)
               : (uint32_t)load_row(static_cast<const int32_t*>(a.idx), i, a.V, err);
  }
  return a.keys_in[i];
}

template <int IPT, bool FIRST, int BITS>
__global__ __launch_bounds__(kSortThreads) void radix_hist_kernel(RadixPass a) {
  constexpr int R = Radix<BITS>::kBins;
  __shared__ int32_t h[R];
  const int t = threadIdx.x;
  for (int d = t; d < R; d += kSortThreads) h[d] = 0;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * (kSortThreads * IPT);
#pragma unroll
  for (int i = 0; i < IPT; ++i) {
    const int64_t e = base + i * kSortThreads + t;
    if (e < a.S) atomicAdd(&h[(radix_key<FIRST>(a, e, a.err) >> a.shift) & (R - 1)], 1);
  }
  __syncthreads();
  for (int d = t; d < R; d += kSortThreads) a.hist[(int64_t)blockIdx.x * R + d] = h[d];
}

// Exclusive scan of one value per thread over the 256-thread block (4 waves).
__device__ __forceinline__ int32_t block_exclusive_scan(int32_t v, int32_t* wave_tot) {
  const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
  int32_t x = v;
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const int32_t y = __shfl_up(x, o, kWave);
    if (lane >= o) x += y;
  }
  if (lane == kWave - 1) wave_tot[w] = x;
  __syncthreads();
  int32_t off = 0;
#pragma unroll
  for (int j = 0; j < kSortWaves; ++j) off += j < w ? wave_tot[j] : 0;
  __syncthreads();
  return off + x - v;
}

// One pass of the stable LSD sort over one tile: the block scans the per-tile digit
// histograms for its global digit bases (thread t owns the DPT consecutive digits
// [t*DPT, (t+1)*DPT); the tile rows are read 8 at a time, independent loads in flight
// together), ranks its keys stably with wave ballots (BITS ballots give the lanes holding
// the same digit; popcount below the lane = rank within the wave) and scatters (key, value).
// Ranking works on groups of G item rows: every (row, wave) leader records its digit
// count, ONE barrier, each thread turns its digits' counts into exclusive prefixes over
// (row, wave) order carried across groups, one barrier, and every key reads its offset —
// 2 barriers per group instead of 3 per row (8-bit digits: G = 8 rows, 2 x 32 KB LDS).
template <int IPT, bool FIRST, bool LAST, int BITS>
__global__ __launch_bounds__(kSortThreads) void radix_scatter_kernel(RadixPass a) {
  constexpr int R = Radix<BITS>::kBins, DPT = Radix<BITS>::kDPT;
  // item rows ranked together (the two LDS count arrays stay <= 32 KB each)
  constexpr int G = (R <= 256) ? (IPT < 8 ? IPT : 8) : (R <= 1024 ? 2 : 1);
  static_assert(IPT % G == 0, "IPT must be a multiple of the ranking group");
  __shared__ int32_t s_base[R];                   // global base of each digit for this tile
  __shared__ int32_t s_run[R];                    // digits ranked in earlier groups
  __shared__ int32_t s_cnt[G][kSortWaves][R];     // (row, wave) digit counts of a group
  __shared__ int32_t s_pre[G][kSortWaves][R];     // their exclusive prefixes (+ s_run)
  __shared__ int32_t s_wtot[kSortWaves];
  const int t = threadIdx.x;
  const int lane = t & (kWave - 1), w = t / kWave;
  const int tile = blockIdx.x;

  // keys of this tile, striped (loads first: they overlap the histogram scan below)
  const int64_t base = (int64_t)tile * (kSortThreads * IPT);
  uint32_t key[IPT];
  int32_t val[IPT];
#pragma unroll
  for (int i = 0; i < IPT; ++i) {
    const int64_t e = base + i * kSortThreads + t;
    key[i] = 0;
    val[i] = 0;
    if (e < a.S) {
      key[i] = radix_key<FIRST>(a, e, nullptr);
      val[i] = FIRST ? (int32_t)e : a.vals_in[e];
    }
  }

  // digits [t*DPT, (t+1)*DPT): totals over all tiles and the part of the tiles before this one
  int32_t tot[DPT], before[DPT];
#pragma unroll
  for (int k = 0; k < DPT; ++k) tot[k] = before[k] = 0;
  {
    const int32_t* hcol = a.hist + t * DPT;
    constexpr int U = 8;  // tile rows loaded together
    for (int j0 = 0; j0 < a.n_tiles; j0 += U) {
      int32_t hv[U][DPT];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int j = j0 + u;
        if constexpr (DPT % 4 == 0) {
#pragma unroll
          for (int k = 0; k < DPT; k += 4) {
            int4 q = make_int4(0, 0, 0, 0);
            if (j < a.n_tiles) q = *reinterpret_cast<const int4*>(hcol + (int64_t)j * R + k);
            hv[u][k] = q.x; hv[u][k + 1] = q.y; hv[u][k + 2] = q.z; hv[u][k + 3] = q.w;
          }
        } else {
#pragma unroll
          for (int k = 0; k < DPT; ++k) hv[u][k] = j < a.n_tiles ? hcol[(int64_t)j * R + k] : 0;
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int k = 0; k < DPT; ++k) {
          tot[k] += hv[u][k];
          before[k] += j0 + u < tile ? hv[u][k] : 0;
        }
    }
  }
  int32_t mine = 0;
#pragma unroll
  for (int k = 0; k < DPT; ++k) mine += tot[k];
  int32_t start = block_exclusive_scan(mine, s_wtot);
#pragma unroll
  for (int k = 0; k < DPT; ++k) {
    s_base[t * DPT + k] = start + before[k];
    s_run[t * DPT + k] = 0;
    start += tot[k];
  }
  for (int d = t; d < R; d += kSortThreads)
#pragma unroll
    for (int i = 0; i < G; ++i)
#pragma unroll
      for (int j = 0; j < kSortWaves; ++j) s_cnt[i][j][d] = 0;
  __syncthreads();

  const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (kWave - lane));
  int32_t pos[IPT];
#pragma unroll
  for (int g0 = 0; g0 < IPT; g0 += G) {
    int rank[G];
#pragma unroll
    for (int i = 0; i < G; ++i) {
      const int64_t e = base + (g0 + i) * kSortThreads + t;
      const bool ok = e < a.S;
      const uint32_t d = (key[g0 + i] >> a.shift) & (R - 1);
      uint64_t peers = __ballot(ok);
#pragma unroll
      for (int b = 0; b < BITS; ++b) {
        const uint64_t m = __ballot((d >> b) & 1u);
        peers &= ((d >> b) & 1u) ? m : ~m;
      }
      rank[i] = __popcll(peers & lt);
      if (ok && rank[i] == 0) s_cnt[i][w][d] = __popcll(peers);
    }
    __syncthreads();
    // per owned digit: exclusive prefix over (row, wave) of this group, after s_run
#pragma unroll
    for (int k = 0; k < DPT; ++k) {
      const int dd = t * DPT + k;
      int32_t run = s_run[dd];
#pragma unroll
      for (int i = 0; i < G; ++i)
#pragma unroll
        for (int j = 0; j < kSortWaves; ++j) {
          const int32_t c = s_cnt[i][j][dd];
          s_pre[i][j][dd] = run;
          s_cnt[i][j][dd] = 0;
          run += c;
        }
      s_run[dd] = run;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < G; ++i) {
      const int64_t e = base + (g0 + i) * kSortThreads + t;
      const bool ok = e < a.S;
      const uint32_t d = (key[g0 + i] >> a.shift) & (R - 1);
      pos[g0 + i] = ok ? s_base[d] + s_pre[i][w][d] + rank[i] : -1;
    }
  }
#pragma unroll
  for (int i = 0; i < IPT; ++i) {
    if (pos[i] >= 0) {
      a.keys_out[pos[i]] = key[i];
      a.vals_out[pos[i]] = val[i];
    }
  }
}

// ------------------------------------------------------------------- segments --------
constexpr int kSegIPT = 8;
constexpr int kSegTile = kSortThreads * kSegIPT;

__global__ __launch_bounds__(kSortThreads) void seg_count_kernel(const int32_t* __restrict__ rows,
                                                                 int64_t S,
                                                                 int32_t* __restrict__ tile_heads,
                                                                 const int32_t* __restrict__ skip) {
  __shared__ int32_t s_w[kSortWaves];
  if (skip && *skip == 0) return;  // the column plan's merge wrote the segments
  const int64_t base = (int64_t)blockIdx.x * kSegTile;
  int32_t c = 0;
#pragma unroll
  for (int i = 0; i < kSegIPT; ++i) {
    const int64_t s = base + i * kSortThreads + threadIdx.x;
    if (s < S) c += (s == 0 || rows[s] != rows[s - 1]) ? 1 : 0;
  }
  c = wave_sum_i32(c);
  if ((threadIdx.x & (kWave - 1)) == 0) s_w[threadIdx.x / kWave] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    int32_t tot = 0;
    for (int j = 0; j < kSortWaves; ++j) tot += s_w[j];
    tile_heads[blockIdx.x] = tot;
  }
}

__global__ __launch_bounds__(kSortThreads) void seg_write_kernel(
    const int32_t* __restrict__ rows, int64_t S, const int32_t* __restrict__ tile_heads,
    int n_tiles, int32_t* __restrict__ pos_seg, int32_t* __restrict__ unique_rows,
    int32_t* __restrict__ seg_offsets, int32_t* __restrict__ num_unique,
    const int32_t* __restrict__ skip) {
  __shared__ int32_t s_w[kSortWaves];
  if (skip && *skip == 0) return;
  const int t = threadIdx.x;
  // heads in the tiles before this one
  int32_t before = 0;
  for (int j = t; j < (int)blockIdx.x; j += kSortThreads) before += tile_heads[j];
  before = wave_sum_i32(before);
  if ((t & (kWave - 1)) == 0) s_w[t / kWave] = before;
  __syncthreads();
  int32_t tile_base = 0;
  for (int j = 0; j < kSortWaves; ++j) tile_base += s_w[j];
  __syncthreads();
  // blocked: thread t owns kSegIPT consecutive positions
  const int64_t s0 = (int64_t)blockIdx.x * kSegTile + (int64_t)t * kSegIPT;
  int32_t r[kSegIPT];
  bool head[kSegIPT];
  int32_t cnt = 0;
  int32_t prev = (s0 > 0 && s0 - 1 < S) ? rows[s0 - 1] : -1;
#pragma unroll
  for (int i = 0; i < kSegIPT; ++i) {
    const int64_t s = s0 + i;
    r[i] = s < S ? rows[s] : -1;
    head[i] = s < S && (s == 0 || r[i] != prev);
    prev = r[i];
    cnt += head[i] ? 1 : 0;
  }
  int32_t u = tile_base + block_exclusive_scan(cnt, s_w) - 1;
#pragma unroll
  for (int i = 0; i < kSegIPT; ++i) {
    const int64_t s = s0 + i;
    if (s < S) {
      if (head[i]) {
        ++u;
        unique_rows[u] = r[i];
        seg_offsets[u] = (int32_t)s;
      }
      pos_seg[s] = u;
      if (s == S - 1) {
        *num_unique = u + 1;
        seg_offsets[u + 1] = (int32_t)S;
      }
    }
  }
}

// ------------------------------------------- column plan: 2 launches (+1 that idles) -------
// The ids of a batch are a [B][F] matrix (slot s = b*F + f) whose columns are the feature
// fields, and in every CTR layout (the reference's creat_data.py feature offsets, Criteo /
// Avazu field ranges) each column's ids lie in a range of their own. The stable (row, slot)
// order of the whole batch is then the concatenation of each column's own stable order, and
// a column of B <= 8192 ids sorts inside one workgroup's LDS. So:
//   colplan_sort  one block per run (a column of B <= 8192 ids; 256 / 512 / 1024 threads x 8):
//                 the run's ids sorted by a stable LSD radix on (row - run min) in LDS —
//                 8-bit digits, only as many passes as the run's row range needs, each
//                 ranked with wave ballots, the ids blocked by wave — and written out with
//                 each position's ordinal among the run's distinct rows;
//                 run_info = {min, max, length, distinct rows}.
//   colplan_merge one thread per slot: its sorted position is its position in its run plus,
//                 for every other run, how many of that run's (row, slot) keys are smaller —
//                 the whole run when its max row is below the slot's row, none when its min
//                 is above, a binary search otherwise (runs whose ranges overlap: any layout
//                 stays exact). When no two runs' ranges overlap (checked by every block
//                 from run_info) the segment of a slot is the distinct rows of the runs below
//                 plus its ordinal in its run, and this launch writes the whole plan;
//                 otherwise it counts every row's first position into its sorted tile's
//                 head count (the binary searches tell whether another run holds the row
//                 at a smaller slot) and leaves flags[0] = 1 for seg_write (which returns at
//                 once on flags[0] == 0) to turn those counts into the segments.
// Bit-identical to the LSD plan (tests/test_gpu_kernels.py), no inter-workgroup hand-off.
constexpr int kColMaxRuns = 256;
constexpr int kColIPT = 8;  // ids per thread of a column sort (blocks of 256 / 512 / 1024)

struct ColArgs {
  const void* idx;
  int idx_type;
  int64_t V, S, B;
  int F, RM, nc, n_runs;  // run r = (column r / nc, chunk r % nc) of RM rows
  int32_t* run_rows;      // [S] runs back to back, run r at f*B + c*RM
  int32_t* run_slots;
  int32_t* run_seg;
  int32_t* run_info;      // [n_runs][4]
  int32_t* tile_heads;    // [ceil(S / kSegTile)]: zeroed by the sort, counted by the merge
  int32_t* flags;
  int32_t* err;
  ctr_sparse_plan plan;
};

// block-wide helpers for NW waves (s_w: NW ints)
template <int NW>
__device__ __forceinline__ int32_t col_block_reduce(int32_t v, bool is_max, int32_t* s_w) {
#pragma unroll
  for (int o = kWave / 2; o > 0; o >>= 1) {
    const int32_t y = __shfl_xor(v, o, kWave);
    v = is_max ? max(v, y) : min(v, y);
  }
  const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
  if (lane == 0) s_w[w] = v;
  __syncthreads();
  int32_t r = s_w[0];
#pragma unroll
  for (int j = 1; j < NW; ++j) r = is_max ? max(r, s_w[j]) : min(r, s_w[j]);
  __syncthreads();
  return r;
}

template <int NW>
__device__ __forceinline__ int32_t col_block_exscan(int32_t v, int32_t* s_w) {
  const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
  int32_t x = v;
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const int32_t y = __shfl_up(x, o, kWave);
    if (lane >= o) x += y;
  }
  if (lane == kWave - 1) s_w[w] = x;
  __syncthreads();
  int32_t off = 0;
#pragma unroll
  for (int j = 0; j < NW; ++j) off += j < w ? s_w[j] : 0;
  __syncthreads();
  return off + x - v;
}

#ifndef CTR_COLPLAN_TRACE
#define CTR_COLPLAN_TRACE 0
#endif
#if CTR_COLPLAN_TRACE
// tuning builds only: per sort block wall_clock64 at [start, bits known, end of passes 1..3,
// end], then bits and n
__device__ unsigned long long g_colplan_trace[kColMaxRuns * 8];
#define COLPLAN_MARK(slot, v) \
  if (t == 0) g_colplan_trace[r * 8 + (slot)] = (v)
#else
#define COLPLAN_MARK(slot, v)
#endif

// ids q0 + i*64 (i < IPT) of column f, rows b0.. (q >= n: a clamped load, value unused)
template <int IPT, typename IdxT>
__device__ __forceinline__ void col_load_ids(const IdxT* __restrict__ idx, int64_t b0, int F,
                                             int f, int n, int q0, int64_t (&raw)[IPT]) {
#pragma unroll
  for (int i = 0; i < IPT; ++i) {
    const int q = min(q0 + i * kWave, n - 1);
    raw[i] = static_cast<int64_t>(idx[(b0 + q) * F + f]);
  }
}

// One run per block of NT threads x IPT ids, BLOCKED by wave: wave w holds the run's ids
// [w*IPT*64, (w+1)*IPT*64), item i of lane l being id w*IPT*64 + i*64 + l — so (wave, item,
// lane) order is slot order. Per 8-bit pass each wave ranks its items in order with no
// barrier: 8 ballots give an item's equal-digit peers in its wave-instruction, its place
// is the wave's running count of that digit (a wave-private LDS histogram) plus its rank
// among the peers, and the peer group's lowest lane adds the group to the histogram. Then
// one barrier, the digit bases (a scan of the digit totals) and per digit the waves'
// exclusive prefix, one barrier, the scatter into LDS. 4 barriers per pass. Measured and not
// kept (profiles/r04_colplan_trace{2,3}.txt, sort phase trace): ceil(bits/11) equal-width
// passes on 16-bit wave counters (C2 13.2 us, C3 25.7: an 11-bit pass costs 1.7x an 8-bit
// one) and ceil(bits/8) equal-width passes <= 8 bits (C2 15.0, C3 23.3) against this
// kernel's 13.9 / 23.0.
template <int NT, int IPT>
__global__ __launch_bounds__(NT) void colplan_sort_kernel(ColArgs a) {
  constexpr int NW = NT / kWave;
  constexpr int RM = NT * IPT;
  constexpr int WR = IPT * kWave;  // ids per wave
  constexpr int R = 256;
  __shared__ uint32_t sk[RM];
  __shared__ int32_t sv[RM];
  __shared__ int32_t s_wh[NW][R];  // per wave: running digit counts, then its bases
  __shared__ int32_t s_w[NW];
  const int t = threadIdx.x;
  const int lane = t & (kWave - 1), w = t / kWave;
  const int r = blockIdx.x;
  const int f = r / a.nc, c = r - f * a.nc;
  const int64_t b0 = (int64_t)c * RM;
  const int n = (int)min<int64_t>(RM, a.B - b0);
  COLPLAN_MARK(0, wall_clock64());
  const int64_t n_seg = (a.S + kSegTile - 1) / kSegTile;
  for (int64_t j = (int64_t)r * NT + t; j < n_seg; j += (int64_t)a.n_runs * NT)
    a.tile_heads[j] = 0;
  uint32_t key[IPT];
  int32_t val[IPT];
  int32_t lo = INT32_MAX, hi = 0;
  // all IPT loads in flight before the first range check: one index type per loop and no
  // branch per item (a per-item type branch, or a check's error atomic that may alias idx,
  // serialises the loads on their full latency)
  int64_t raw[IPT];
  if (a.idx_type == CTR_IDX_I64)
    col_load_ids<IPT>(static_cast<const int64_t*>(a.idx), b0, a.F, f, n, w * WR + lane, raw);
  else
    col_load_ids<IPT>(static_cast<const int32_t*>(a.idx), b0, a.F, f, n, w * WR + lane, raw);
#pragma unroll
  for (int i = 0; i < IPT; ++i) {
    const int q = w * WR + i * kWave + lane;
    key[i] = 0;
    val[i] = 0;
    if (q < n) {
      int64_t row = raw[i];
      if (row < 0 || row >= a.V) {
        if (a.err) atomicOr(a.err, (int32_t)CTR_EFLAG_INDEX);
        row = 0;
      }
      key[i] = (uint32_t)row;
      val[i] = (int32_t)((b0 + q) * a.F + f);
      lo = min(lo, (int32_t)row);
      hi = max(hi, (int32_t)row);
    }
  }
  lo = col_block_reduce<NW>(lo, false, s_w);
  hi = col_block_reduce<NW>(hi, true, s_w);
  const uint32_t span = (uint32_t)(hi - lo);
  const int bits = span == 0 ? 0 : 32 - __builtin_clz(span);
  int32_t* wh = s_wh[w];
  COLPLAN_MARK(1, wall_clock64());
  COLPLAN_MARK(6, bits);
  COLPLAN_MARK(7, n);
  for (int shift = 0; shift < bits; shift += 8) {
    for (int d = lane; d < R; d += kWave) wh[d] = 0;  // wave-private: no barrier
    int32_t loc[IPT];
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
      const bool ok = w * WR + i * kWave + lane < n;
      const uint32_t d = ((key[i] - (uint32_t)lo) >> shift) & (R - 1);
      const uint64_t okm = __ballot(ok);
      uint32_t plo = (uint32_t)okm, phi = (uint32_t)(okm >> 32);
#pragma unroll
      for (int bb = 0; bb < 8; ++bb) {
        // bit set: keep the lanes whose bit is set (m), else those whose bit is clear (~m)
        const int32_t sb = (int32_t)(d << (31 - bb)) >> 31;  // v_bfe_i32: 0 / all ones
        const uint32_t bm = (uint32_t)sb;
        const uint64_t m = __ballot(sb < 0);
        plo &= ~((uint32_t)m ^ bm);
        phi &= ~((uint32_t)(m >> 32) ^ bm);
      }
      const int rank = (int)__builtin_amdgcn_mbcnt_hi(phi, __builtin_amdgcn_mbcnt_lo(plo, 0u));
      const int32_t before = ok ? wh[d] : 0;
      loc[i] = before + rank;
      __builtin_amdgcn_wave_barrier();
      if (ok && rank == 0) wh[d] = before + __popc(plo) + __popc(phi);
      __builtin_amdgcn_wave_barrier();
    }
    __syncthreads();
    // digit d: its total over the waves -> base of the digit (scan of the totals), then
    // each wave's base = digit base + the earlier waves' counts
    {
      int32_t tot = 0;
      if (t < R)
#pragma unroll
        for (int j = 0; j < NW; ++j) tot += s_wh[j][t];
      const int32_t base = col_block_exscan<NW>(tot, s_w);  // (barriers inside)
      if (t < R) {
        int32_t run = base;
#pragma unroll
        for (int j = 0; j < NW; ++j) {
          const int32_t cn = s_wh[j][t];
          s_wh[j][t] = run;
          run += cn;
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < IPT; ++i)
      if (w * WR + i * kWave + lane < n) {
        const uint32_t d = ((key[i] - (uint32_t)lo) >> shift) & (R - 1);
        const int p = wh[d] + loc[i];
        sk[p] = key[i];
        sv[p] = val[i];
      }
    __syncthreads();
    if (shift + 8 < bits) {  // the next pass ranks in the new order (the last leaves it in LDS)
#pragma unroll
      for (int i = 0; i < IPT; ++i) {
        const int q = w * WR + i * kWave + lane;
        if (q < n) {
          key[i] = sk[q];
          val[i] = sv[q];
        }
      }
      __syncthreads();
    }
    COLPLAN_MARK(2 + min(shift / 8, 2), wall_clock64());
  }
  if (bits == 0) {  // one row value: already in slot order
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
      const int q = w * WR + i * kWave + lane;
      if (q < n) {
        sk[q] = key[i];
        sv[q] = val[i];
      }
    }
    __syncthreads();
  }
  // blocked: thread t writes positions [t*IPT, (t+1)*IPT) with their distinct-row ordinals
  const int q0 = t * IPT;
  int32_t cnt = 0;
#pragma unroll
  for (int i = 0; i < IPT; ++i) {
    const int q = q0 + i;
    cnt += (q < n && (q == 0 || sk[q] != sk[q - 1])) ? 1 : 0;
  }
  const int32_t ex = col_block_exscan<NW>(cnt, s_w);
  int32_t u = ex - 1;
  const int64_t off = (int64_t)f * a.B + b0;
  const bool al = ((reinterpret_cast<uintptr_t>(a.run_rows + off) |
                    reinterpret_cast<uintptr_t>(a.run_slots + off) |
                    reinterpret_cast<uintptr_t>(a.run_seg + off)) & 15) == 0;
  if (IPT % 4 == 0 && al && q0 + IPT <= n) {  // 16-B LDS reads and stores
#pragma unroll
    for (int i = 0; i < IPT; i += 4) {
      const uint4 k4 = *reinterpret_cast<const uint4*>(sk + q0 + i);
      const int4 v4 = *reinterpret_cast<const int4*>(sv + q0 + i);
      const uint32_t kp = (q0 + i == 0) ? ~k4.x : sk[q0 + i - 1];
      int4 u4;
      u4.x = u += k4.x != kp ? 1 : 0;
      u4.y = u += k4.y != k4.x ? 1 : 0;
      u4.z = u += k4.z != k4.y ? 1 : 0;
      u4.w = u += k4.w != k4.z ? 1 : 0;
      *reinterpret_cast<int4*>(a.run_rows + off + q0 + i) =
          make_int4((int32_t)k4.x, (int32_t)k4.y, (int32_t)k4.z, (int32_t)k4.w);
      *reinterpret_cast<int4*>(a.run_slots + off + q0 + i) = v4;
      *reinterpret_cast<int4*>(a.run_seg + off + q0 + i) = u4;
    }
  } else {
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
      const int q = q0 + i;
      if (q < n) {
        const uint32_t k = sk[q];
        u += (q == 0 || k != sk[q - 1]) ? 1 : 0;
        a.run_rows[off + q] = (int32_t)k;
        a.run_slots[off + q] = sv[q];
        a.run_seg[off + q] = u;
      }
    }
  }
  if (t == NT - 1) reinterpret_cast<int4*>(a.run_info)[r] = make_int4(lo, hi, n, ex + cnt);
  COLPLAN_MARK(5, wall_clock64());
}

// the (row, slot) keys of run [o, o + len) smaller than (row, slot): binary search
__device__ __forceinline__ int32_t colplan_rank_in(const ColArgs& a, int64_t o, int32_t len,
                                                   int32_t row, int32_t slot) {
  int32_t lo = 0, hi = len;
  while (lo < hi) {
    const int32_t mid = (lo + hi) >> 1;
    const int32_t rm = a.run_rows[o + mid];
    const bool less = rm < row || (rm == row && a.run_slots[o + mid] < slot);
    if (less) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

__global__ __launch_bounds__(kSortThreads) void colplan_merge_kernel(ColArgs a) {
  __shared__ int4 s_info[kColMaxRuns];
  __shared__ int s_overlap;
  const int t = threadIdx.x;
  const int nr = a.n_runs;
  // this slot's run entries, loaded with the run table (one memory round trip for both)
  const int64_t e = (int64_t)blockIdx.x * kSortThreads + t;
  const bool live = e < a.S;
  const int f = (int)((live ? e : 0) / a.B);
  const int64_t wi = (live ? e : 0) - (int64_t)f * a.B;
  const int c = (int)(wi / a.RM);
  const int p = (int)(wi - (int64_t)c * a.RM);
  const int32_t row = live ? a.run_rows[e] : 0, slot = live ? a.run_slots[e] : 0;
  const int32_t lseg = live ? a.run_seg[e] : 0;
  const int32_t prev_row = live && p > 0 ? a.run_rows[e - 1] : -1;
  if (t == 0) s_overlap = 0;
  for (int g = t; g < nr; g += kSortThreads) s_info[g] = reinterpret_cast<const int4*>(a.run_info)[g];
  __syncthreads();
  {
    bool ov = false;
    for (int g = t; g < nr; g += kSortThreads) {
      const int4 x = s_info[g];
      for (int h = g + 1; h < nr; ++h) {
        const int4 y = s_info[h];
        ov |= !(x.y < y.x || y.y < x.x);
      }
    }
    if (ov) s_overlap = 1;  // benign race: every writer stores 1
  }
  __syncthreads();
  const bool disjoint = s_overlap == 0;
  if (blockIdx.x == 0 && t == 0) {
    a.flags[0] = disjoint ? 0 : 1;
    if (disjoint) {
      int32_t U = 0;
      for (int g = 0; g < nr; ++g) U += s_info[g].w;
      *a.plan.num_unique = U;
      a.plan.seg_offsets[U] = (int32_t)a.S;
    }
  }
  if (!live) return;
  const int r = f * a.nc + c;
  int64_t pos = p;
  int32_t segb = 0;
  bool first_elsewhere = false;  // another run holds this row at a smaller slot
  for (int g = 0; g < nr; ++g) {
    if (g == r) continue;
    const int4 x = s_info[g];
    if (x.y < row) {
      pos += x.z;
      segb += x.w;
    } else if (x.x <= row) {
      const int gf = g / a.nc, gc = g - gf * a.nc;
      const int64_t o = (int64_t)gf * a.B + (int64_t)gc * a.RM;
      const int32_t below = colplan_rank_in(a, o, x.z, row, slot);
      pos += below;
      first_elsewhere |= below > 0 && a.run_rows[o + below - 1] == row;
    }
  }
  a.plan.sorted_rows[pos] = row;
  a.plan.sorted_slots[pos] = slot;
  const bool local_head = p == 0 || prev_row != row;
  if (disjoint) {
    const int32_t seg = segb + lseg;
    a.plan.pos_seg[pos] = seg;
    if (local_head) {
      a.plan.unique_rows[seg] = row;
      a.plan.seg_offsets[seg] = (int32_t)pos;
    }
  } else if (local_head && !first_elsewhere) {
    // the first position of its row over every run: count it in its sorted tile (integer
    // adds, order-free), seg_write turns the tile counts into the segments
    atomicAdd(&a.tile_heads[pos / kSegTile], 1);
  }
}

// ------------------------------------------------------------ row sharding -------------
// slot -> unique-row ordinal (the inverse of the plan's grouping): the forward of a
// row-sharded step reads the rows it received, compacted in unique order.
__global__ __launch_bounds__(256) void slot_to_unique_kernel(const int32_t* __restrict__ sorted_slots,
                                                             const int32_t* __restrict__ pos_seg,
                                                             int64_t S, int32_t* __restrict__ out) {
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < S;
       p += (int64_t)gridDim.x * blockDim.x)
    out[sorted_slots[p]] = pos_seg[p];
}

__global__ __launch_bounds__(256) void ids_add_kernel(int32_t* __restrict__ ids, int64_t n,
                                                      int32_t delta) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    ids[i] += delta;
}

// Unique rows are ascending, so the rows of shard j (ids in [j*shard_rows, (j+1)*shard_rows))
// are one contiguous run: counts[j] = its length, found by binary search (one thread per shard).
__global__ void shard_counts_kernel(const int32_t* __restrict__ unique_rows,
                                    const int32_t* __restrict__ num_unique, int64_t shard_rows,
                                    int n_shards, int64_t* __restrict__ counts) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n_shards) return;
  const int U = *num_unique;
  auto lower = [&](int64_t v) {  // first position with unique_rows[pos] >= v
    int lo = 0, hi = U;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if ((int64_t)unique_rows[mid] < v) lo = mid + 1;
      else hi = mid;
    }
    return lo;
  };
  counts[j] = lower((int64_t)(j + 1) * shard_rows) - lower((int64_t)j * shard_rows);
}

// The same counts for up to kCountsMaxShards shards in ONE block, and their maximum (the
// step's largest run, what the capacity agreement reads): wave w finds the run boundary
// lower_bound(w * shard_rows) by a 64-ary search — 64 probes per round, a ballot picks the
// sub-range — so the chain is ~3 dependent loads at U = 61k instead of a binary search's 16
// (the thread-per-shard kernel above ran 24 us at C3, plus a separate max launch).
constexpr int kCountsMaxShards = 15;

__device__ __forceinline__ int wave_lower_bound(const int32_t* __restrict__ rows, int U, int64_t v,
                                                int lane) {
  int lo = 0, hi = U;  // the answer lies in [lo, hi]
  while (hi - lo > kWave) {
    const int step = (hi - lo + kWave - 1) / kWave;
    const int q = lo + lane * step;
    const bool below = q < hi && (int64_t)rows[q] < v;
    const int c = __popcll(__ballot(below));  // probes below v (a prefix of the lanes)
    if (c == 0) return lo;                    // rows[lo] >= v
    const int nlo = lo + (c - 1) * step + 1;
    hi = min(hi, lo + c * step);
    lo = nlo;
  }
  const int q = lo + lane;
  const bool below = q < hi && (int64_t)rows[q] < v;
  return lo + __popcll(__ballot(below));
}

__global__ __launch_bounds__(1024) void shard_counts_max_kernel(
    const int32_t* __restrict__ unique_rows, const int32_t* __restrict__ num_unique,
    int64_t shard_rows, int n_shards, int64_t* __restrict__ counts, int64_t* __restrict__ max_out) {
  __shared__ int bound[kCountsMaxShards + 1];
  const int w = threadIdx.x / kWave, lane = threadIdx.x % kWave;
  const int U = *num_unique;
  if (w <= n_shards) {
    const int b = w == 0 ? 0 : wave_lower_bound(unique_rows, U, (int64_t)w * shard_rows, lane);
    if (lane == 0) bound[w] = b;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t mx = 0;
    for (int j = 0; j < n_shards; ++j) {
      const int64_t c = bound[j + 1] - bound[j];
      counts[j] = c;
      mx = c > mx ? c : mx;
    }
    if (max_out) max_out[0] = mx;
  }
}

// Fixed-capacity exchange of a row-sharded step: every (requester, owner) pair moves C rows
// (equal-split all-to-alls whose sizes depend on C alone, so a step is graph-capturable).
// The plan's unique rows owned by shard j are the run [lo_j, hi_j) of unique_rows (ascending);
// slot i of destination j carries run entry lo_j + i as an owner-local id, or, past the run,
// the owner's dummy row id (its row count: owners keep one spare row that padding entries
// read and update, never a real one). counts[j] / offsets[j] (int32) describe the runs; a
// run longer than C raises CTR_EFLAG_CAPACITY.
__global__ __launch_bounds__(256) void shard_pack_ids_kernel(
    const int32_t* __restrict__ unique_rows, const int32_t* __restrict__ num_unique,
    int64_t shard_rows, int64_t V, int64_t C, int32_t* __restrict__ send,
    int32_t* __restrict__ counts, int32_t* __restrict__ offsets, int32_t* err, int cyc) {
  const int j = blockIdx.y;
  const int U = *num_unique;
  const int64_t base = (int64_t)j * shard_rows;
  // the run's bounds by two waves' 64-ary searches (~3 dependent loads each, not a binary
  // search's 16 in every thread), shared through LDS
  __shared__ int bounds[2];
  const int wave = threadIdx.x / kWave;
  if (wave < 2) {
    const int b = wave_lower_bound(unique_rows, U, base + (wave ? shard_rows : 0), threadIdx.x % kWave);
    if (threadIdx.x % kWave == 0) bounds[wave] = b;
  }
  __syncthreads();
  const int lo = bounds[0], hi = bounds[1];
  // the owner's spare row = its row count: blocks min(shard_rows, V - j*shard_rows),
  // cyclic (n_shards < 0 passed as cyc) ceil((V - j) / n)
  const int32_t dummy = cyc > 0 ? (int32_t)max<int64_t>(0, (V - j + cyc - 1) / cyc)
                                : (int32_t)max<int64_t>(0, min<int64_t>(shard_rows, V - base));
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < C;
       i += (int64_t)gridDim.x * blockDim.x)
    send[(int64_t)j * C + i] = lo + i < hi ? (int32_t)(unique_rows[lo + i] - base) : dummy;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    counts[j] = hi - lo;
    offsets[j] = lo;
    if (hi - lo > C && err) atomicOr(err, (int32_t)CTR_EFLAG_CAPACITY);
  }
}

// Cyclic row sharding: global row r is owned by shard r % n, as its local row r / n. The
// batch's ids are mapped in place to r' = (r % n) * shard_rows + r / n, a space in which every
// shard's rows are one contiguous block again (shard j: [j*shard_rows, j*shard_rows + n_j),
// n_j = ceil((V - j) / n)), so the plan's ascending unique rows come out grouped by owner and
// the exchange below runs unchanged. An id outside [0, V) raises CTR_EFLAG_INDEX and maps
// to row 0 (nn.Embedding's IndexError, raised by the host's check_errors).
template <typename T>
__global__ __launch_bounds__(256) void shard_permute_ids_kernel(T* __restrict__ ids, int64_t count,
                                                                int64_t V, int64_t n,
                                                                int64_t shard_rows,
                                                                int32_t* err) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < count;
       i += (int64_t)gridDim.x * blockDim.x) {
    int64_t r = (int64_t)ids[i];
    if (r < 0 || r >= V) {
      if (err) atomicOr(err, (int32_t)CTR_EFLAG_INDEX);
      r = 0;
    }
    ids[i] = (T)((r % n) * shard_rows + r / n);
  }
}

// Row runs between the compact order (run j at offsets[j], counts[j] rows) and the padded
// exchange layout (run j at j*C, C rows): PACK writes every padded slot (zeros past a run),
// UNPACK writes the runs only. W floats per row (float4 when W % 4 == 0).
template <typename VT, bool PACK>
__global__ __launch_bounds__(256) void shard_runs_copy_kernel(
    const VT* __restrict__ src, VT* __restrict__ dst, int64_t W, int64_t C,
    const int32_t* __restrict__ counts, const int32_t* __restrict__ offsets) {
  const int j = blockIdx.y;
  // a run longer than the capacity (CTR_EFLAG_CAPACITY raised by the pack) is cut to C
  // rows both ways: never a read past run j's padded block
  const int64_t cnt = min<int64_t>(counts[j], C), off = offsets[j];
  const int64_t n = (PACK ? C : cnt) * W;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < n;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = t / W, k = t - i * W;
    const int64_t padded = ((int64_t)j * C + i) * W + k, compact = (off + i) * W + k;
    if (PACK) {
      VT v;
      if (i < cnt) v = src[compact];
      else memset(&v, 0, sizeof(v));
      dst[padded] = v;
    } else {
      dst[compact] = src[padded];
    }
  }
}

// The row-sharded exchange's rows WITH their linear weight in one message per (requester,
// owner) pair: chunk j of the padded buffer = [C rows of K floats][C linear weights][pad to a
// multiple of 4] (`chunk` floats), so a step moves the embedding rows and the linear weights
// (and their gradients) in one equal-split all-to-all each instead of two. One thread per
// float4 of a row; the thread of the row's first float4 also moves its linear weight.
//   GATHER: chunked[j][i] = (E[ids[jC+i]], lin[ids[jC+i]])           (owner, rows out)
//   PACK:   chunked[j][i] = (rows[off_j+i], lin[off_j+i]), zeros past counts[j]
//   UNPACK: (rows[off_j+i], lin[off_j+i]) = chunked[j][i] for i < counts[j]
enum { kRowsGather = 0, kRowsPack = 1, kRowsUnpack = 2 };
template <int MODE>
__global__ __launch_bounds__(256) void shard_rows_lin_kernel(
    const float4* __restrict__ src, const float* __restrict__ src_lin, float4* __restrict__ dst,
    float* __restrict__ dst_lin, const int32_t* __restrict__ ids, int64_t K4, int64_t C,
    int64_t chunk, const int32_t* __restrict__ counts, const int32_t* __restrict__ offsets) {
  const int j = blockIdx.y;
  const int64_t cnt = MODE == kRowsGather ? C : min<int64_t>(counts[j], C);
  const int64_t off = MODE == kRowsGather ? 0 : offsets[j];
  const int64_t n = (MODE == kRowsUnpack ? cnt : C) * K4;
  const int64_t cbase = (int64_t)j * chunk;  // floats
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < n;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = t / K4, k = t - i * K4;
    if (MODE == kRowsUnpack) {
      const float* cs = reinterpret_cast<const float*>(src) + cbase;  // chunk j
      dst[(off + i) * K4 + k] = reinterpret_cast<const float4*>(cs + i * 4 * K4)[k];
      if (k == 0 && dst_lin) dst_lin[off + i] = cs[C * 4 * K4 + i];
    } else {
      float* const cf = reinterpret_cast<float*>(dst) + cbase;  // chunk j
      float4* const crow = reinterpret_cast<float4*>(cf + i * 4 * K4);
      if (MODE == kRowsGather) {
        const int64_t r = ids[(int64_t)j * C + i];
        crow[k] = src[r * K4 + k];
        if (k == 0 && src_lin) cf[C * 4 * K4 + i] = src_lin[r];
      } else {
        const bool live = i < cnt;
        crow[k] = live ? src[(off + i) * K4 + k] : make_float4(0.f, 0.f, 0.f, 0.f);
        if (k == 0 && src_lin) cf[C * 4 * K4 + i] = live ? src_lin[off + i] : 0.f;
      }
    }
  }
}

// ------------------------------------------------------------------ host side --------
static int key_bits(int64_t V) {
  int bits = 1;
  while (bits < 32 && (int64_t(1) << bits) < V) ++bits;
  return bits;
}

// Items per thread: 8 (2048-key tiles) while that keeps the per-block histogram scan short
// (<= 256 tiles); larger batches (data-parallel gathered plans) use 32 (8192-key tiles).
static int plan_ipt(int64_t S) { return S <= 256 * 2048 ? 8 : 32; }

// Digits of 8 bits: measured on MI355X (tools/plan_ab2.sh, us per plan, round 2), wider
// digits save a pass but each pass costs more than the pass saved — 10 bits: C2 (V = 1M, 2
// vs 3 passes) 53.7 vs 55.0, C5 (V = 40M, 3 vs 4 passes) 85.0 vs 75.6; 11 bits: C2 69
constexpr int kPlanBits = 8;

struct PlanLayout {
  uint32_t* keys[2];
  int32_t* vals[2];
  int32_t* hist;
  int32_t* tile_heads;
  int32_t* run_info;  // column plan: [n_runs][4] {min row, max row, length, unique rows}
  int32_t* flags;     // column plan: [0] = 1 while the segment launches still have work
  size_t total;
};

static size_t plan_layout(int64_t S, char* base, PlanLayout* L) {
  const int ipt = plan_ipt(S);
  const int64_t n_tiles = ceil_div(std::max<int64_t>(S, 1), kSortThreads * ipt);
  const int64_t n_seg = ceil_div(std::max<int64_t>(S, 1), kSegTile);
  size_t off = 0;
  auto take = [&](size_t bytes) {
    const size_t o = off;
    off += (size_t)align_up((int64_t)bytes, 256);
    return base ? base + o : nullptr;
  };
  for (int j = 0; j < 2; ++j) {
    L->keys[j] = reinterpret_cast<uint32_t*>(take(sizeof(uint32_t) * S));
    L->vals[j] = reinterpret_cast<int32_t*>(take(sizeof(int32_t) * S));
  }
  L->hist = reinterpret_cast<int32_t*>(take(sizeof(int32_t) * Radix<kPlanBits>::kBins * n_tiles));
  L->tile_heads = reinterpret_cast<int32_t*>(take(sizeof(int32_t) * n_seg));
  // column plan: a run per (column, chunk of <= 8192 rows), at most kColMaxRuns
  L->run_info = reinterpret_cast<int32_t*>(take(sizeof(int32_t) * 4 * kColMaxRuns));
  L->flags = reinterpret_cast<int32_t*>(take(sizeof(int32_t) * 64));
  L->total = off;
  return off;
}

template <int NT>
static int run_colplan(ColArgs& a, const PlanLayout& L, hipStream_t st) {
  hipLaunchKernelGGL((colplan_sort_kernel<NT, kColIPT>), (unsigned)a.n_runs, NT, 0, st, a);
  CTR_LAUNCH_CHECK("colplan_sort_kernel");
  hipLaunchKernelGGL(colplan_merge_kernel, (unsigned)ceil_div(a.S, kSortThreads), kSortThreads, 0,
                     st, a);
  CTR_LAUNCH_CHECK("colplan_merge_kernel");
  const unsigned gs = (unsigned)ceil_div(a.S, kSegTile);
  hipLaunchKernelGGL(seg_write_kernel, gs, kSortThreads, 0, st, a.plan.sorted_rows, a.S,
                     L.tile_heads, (int)gs, a.plan.pos_seg, a.plan.unique_rows,
                     a.plan.seg_offsets, a.plan.num_unique, a.flags);
  CTR_LAUNCH_CHECK("seg_write_kernel");
  return CTR_OK;
}

template <int IPT, int BITS>
static int run_passes(RadixPass a, int passes, const ctr_sparse_plan* plan, PlanLayout& L,
                      hipStream_t st) {
  const unsigned grid = (unsigned)a.n_tiles;
  constexpr int R = Radix<BITS>::kBins;
  for (int p = 0; p < passes; ++p) {
    const bool first = p == 0, last = p == passes - 1;
    a.shift = p * BITS;
    a.hist = L.hist;
    a.keys_in = first ? nullptr : L.keys[(p - 1) & 1];
    a.vals_in = first ? nullptr : L.vals[(p - 1) & 1];
    a.keys_out = last ? reinterpret_cast<uint32_t*>(plan->sorted_rows) : L.keys[p & 1];
    a.vals_out = last ? plan->sorted_slots : L.vals[p & 1];
    if (first)
      hipLaunchKernelGGL((radix_hist_kernel<IPT, true, BITS>), grid, kSortThreads, 0, st, a);
    else
      hipLaunchKernelGGL((radix_hist_kernel<IPT, false, BITS>), grid, kSortThreads, 0, st, a);
    CTR_LAUNCH_CHECK("radix_hist_kernel");
    if (first && last)
      hipLaunchKernelGGL((radix_scatter_kernel<IPT, true, true, BITS>), grid, kSortThreads, 0, st, a);
    else if (first)
      hipLaunchKernelGGL((radix_scatter_kernel<IPT, true, false, BITS>), grid, kSortThreads, 0, st, a);
    else if (last)
      hipLaunchKernelGGL((radix_scatter_kernel<IPT, false, true, BITS>), grid, kSortThreads, 0, st, a);
    else
      hipLaunchKernelGGL((radix_scatter_kernel<IPT, false, false, BITS>), grid, kSortThreads, 0, st, a);
    CTR_LAUNCH_CHECK("radix_scatter_kernel");
  }
  return CTR_OK;
}

}  // namespace ctr

using namespace ctr;

static bool plan_ok(const ctr_sparse_plan* p) {
  return p && p->S >= 0 && p->sorted_slots && p->sorted_rows && p->pos_seg && p->unique_rows &&
         p->seg_offsets && p->num_unique;
}

extern "C" int64_t ctr_sparse_plan_workspace_bytes(int64_t S, int64_t V) {
  if (S < 0 || V <= 0 || S >= (int64_t(1) << 24)) {
    set_error("ctr_sparse_plan_workspace_bytes: bad sizes (need 0 <= S < 2^24, V > 0)");
    return -1;
  }
  PlanLayout L;
  return (int64_t)plan_layout(S, nullptr, &L);
}

extern "C" int ctr_sparse_plan_build(const void* idx, int idx_type, int64_t V,
                                     const ctr_sparse_plan* plan, void* ws, int64_t ws_bytes,
                                     int32_t* err_flag, ctr_stream_t stream) {
  CTR_REQUIRE(plan_ok(plan), "ctr_sparse_plan_build: incomplete plan");
  CTR_REQUIRE(idx || plan->S == 0, "ctr_sparse_plan_build: null idx");
  CTR_REQUIRE(V > 0 && V < (int64_t(1) << 31) && plan->S < (int64_t(1) << 24),
              "ctr_sparse_plan_build: bad sizes (need V < 2^31, S < 2^24)");
  CTR_REQUIRE(idx_type == CTR_IDX_I32 || idx_type == CTR_IDX_I64, "bad idx_type %d", idx_type);
  hipStream_t st = as_stream(stream);
  const int64_t S = plan->S;
  if (S == 0) {
    CTR_HIP_CHECK(hipMemsetAsync(plan->num_unique, 0, sizeof(int32_t), st));
    CTR_HIP_CHECK(hipMemsetAsync(plan->seg_offsets, 0, sizeof(int32_t), st));
    return CTR_OK;
  }
  PlanLayout L;
  const size_t need = plan_layout(S, static_cast<char*>(ws), &L);
  if (!ws || ws_bytes < (int64_t)need) {
    set_error("ctr_sparse_plan_build: workspace %lld < %lld bytes", (long long)ws_bytes,
              (long long)need);
    return CTR_ERR_WORKSPACE;
  }
  const int ipt = plan_ipt(S);
  RadixPass a;
  memset(&a, 0, sizeof(a));
  a.idx = idx;
  a.idx_type = idx_type;
  a.V = V;
  a.hist = L.hist;
  a.S = S;
  a.n_tiles = (int)ceil_div(S, kSortThreads * ipt);
  a.err = err_flag;
  const int passes = (int)ceil_div(key_bits(V), kPlanBits);
  const int rc = ipt == 8 ? run_passes<8, kPlanBits>(a, passes, plan, L, st)
                          : run_passes<32, kPlanBits>(a, passes, plan, L, st);
  if (rc != CTR_OK) return rc;
  const unsigned gs = (unsigned)ceil_div(S, kSegTile);
  hipLaunchKernelGGL(seg_count_kernel, gs, kSortThreads, 0, st, plan->sorted_rows, S,
                     L.tile_heads, nullptr);
  CTR_LAUNCH_CHECK("seg_count_kernel");
  hipLaunchKernelGGL(seg_write_kernel, gs, kSortThreads, 0, st, plan->sorted_rows, S,
                     L.tile_heads, (int)gs, plan->pos_seg, plan->unique_rows, plan->seg_offsets,
                     plan->num_unique, nullptr);
  CTR_LAUNCH_CHECK("seg_write_kernel");
  return CTR_OK;
}

#if CTR_COLPLAN_TRACE
extern "C" int ctr_debug_colplan_trace(unsigned long long* host, int n_blocks) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_colplan_trace),
                                  sizeof(unsigned long long) * 8 * std::min(n_blocks, kColMaxRuns));
}
#endif

extern "C" int ctr_sparse_plan_build_cols(const void* idx, int idx_type, int64_t V, int64_t F,
                                          const ctr_sparse_plan* plan, void* ws, int64_t ws_bytes,
                                          int32_t* err_flag, ctr_stream_t stream) {
  CTR_REQUIRE(plan_ok(plan), "ctr_sparse_plan_build_cols: incomplete plan");
  CTR_REQUIRE(F > 0 && plan->S % F == 0, "ctr_sparse_plan_build_cols: S %% F != 0");
  const int64_t S = plan->S, B = S / std::max<int64_t>(F, 1);
  const int nt = B <= 2048 ? 256 : B <= 4096 ? 512 : 1024;  // threads of a run's block
  const int RM = nt * kColIPT;
  const int64_t nc = S == 0 ? 0 : ceil_div(B, (int64_t)RM);
  // one run per column (a column of <= 8192 ids sorts in one block; chunks of a longer
  // column would overlap, and the merge's binary searches grow with the overlapping runs),
  // the run table in one block's LDS: otherwise the LSD plan
  if (S == 0 || nc > 1 || F > kColMaxRuns)
    return ctr_sparse_plan_build(idx, idx_type, V, plan, ws, ws_bytes, err_flag, stream);
  CTR_REQUIRE(idx, "ctr_sparse_plan_build_cols: null idx");
  CTR_REQUIRE(V > 0 && V < (int64_t(1) << 31) && S < (int64_t(1) << 24),
              "ctr_sparse_plan_build_cols: bad sizes (need V < 2^31, S < 2^24)");
  CTR_REQUIRE(idx_type == CTR_IDX_I32 || idx_type == CTR_IDX_I64, "bad idx_type %d", idx_type);
  PlanLayout L;
  const size_t need = plan_layout(S, static_cast<char*>(ws), &L);
  if (!ws || ws_bytes < (int64_t)need) {
    set_error("ctr_sparse_plan_build_cols: workspace %lld < %lld bytes", (long long)ws_bytes,
              (long long)need);
    return CTR_ERR_WORKSPACE;
  }
  ColArgs a;
  memset(&a, 0, sizeof(a));
  a.idx = idx;
  a.idx_type = idx_type;
  a.V = V;
  a.S = S;
  a.B = B;
  a.F = (int)F;
  a.RM = RM;
  a.nc = (int)nc;
  a.n_runs = (int)(F * nc);
  a.run_rows = reinterpret_cast<int32_t*>(L.keys[0]);
  a.run_slots = L.vals[0];
  a.run_seg = reinterpret_cast<int32_t*>(L.keys[1]);
  a.run_info = L.run_info;
  a.tile_heads = L.tile_heads;
  a.flags = L.flags;
  a.err = err_flag;
  a.plan = *plan;
  hipStream_t st = as_stream(stream);
  switch (nt) {
    case 256: return run_colplan<256>(a, L, st);
    case 512: return run_colplan<512>(a, L, st);
    default: return run_colplan<1024>(a, L, st);
  }
}

// ------------------------------------------- owner plan over sorted runs (row sharding) -----
// The owner of a row shard receives, per step, one run of C ids from each of the N <= 8
// requesters (send[j*C + i]): run j holds requester j's rows of this shard in ascending order,
// each once, then padding up to C with the shard's spare row (its largest id). The plan of
// that vector — the stable (row, position) grouping ctr_sparse_plan_build computes by a full
// LSD sort — follows from a per-row bitmask of the requesting runs: a row's entries come from
// distinct runs, in run order, so its position in the sorted vector is (entries of smaller
// rows) + (its runs below this one), and its segment is (distinct smaller rows); the padding
// forms the last segment in position order. 5 launches over N*C entries and the shard's
// n_rows/4 mask words (mark, two scan launches, scatter, clear) instead of 8 over 3 radix
// passes; bit-identical to the LSD plan (tests/test_gpu_kernels.py).
constexpr int kRunWordsPerBlock = 1024;  // 256 threads x 4 mask words

__global__ __launch_bounds__(256) void runs_mark_kernel(const int32_t* __restrict__ ids,
                                                        int64_t C, int64_t S, int32_t spare,
                                                        uint32_t* __restrict__ mask,
                                                        int32_t* __restrict__ run_len) {
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < S;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int j = (int)(e / C);
    const int64_t i = e - (int64_t)j * C;
    const int32_t r = ids[e];
    if (r != spare) {
      atomicOr(&mask[r >> 2], 1u << (((r & 3) << 3) + j));
      if (i == C - 1 || ids[e + 1] == spare) run_len[j] = (int32_t)(i + 1);
    } else if (i == 0) {
      run_len[j] = 0;
    }
  }
}

__device__ __forceinline__ int32_t nz_bytes(uint32_t w) {
  return ((w & 0xffu) != 0) + ((w & 0xff00u) != 0) + ((w & 0xff0000u) != 0) + ((w >> 24) != 0);
}

// per mask word: (entries, distinct rows) exclusive within its block; per block the totals
__global__ __launch_bounds__(256) void runs_scan_words_kernel(const uint32_t* __restrict__ mask,
                                                              int64_t n_words,
                                                              int2* __restrict__ word_pre,
                                                              int2* __restrict__ block_tot) {
  __shared__ int2 s_w[4];
  const int t = threadIdx.x, lane = t & (kWave - 1), w = t / kWave;
  const int64_t w0 = (int64_t)blockIdx.x * kRunWordsPerBlock + (int64_t)t * 4;
  uint32_t m[4];
  int2 tot = make_int2(0, 0);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    m[q] = w0 + q < n_words ? mask[w0 + q] : 0u;
    tot.x += __popc(m[q]);
    tot.y += nz_bytes(m[q]);
  }
  int2 x = tot;  // inclusive wave scan
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const int yx = __shfl_up(x.x, o, kWave), yy = __shfl_up(x.y, o, kWave);
    if (lane >= o) { x.x += yx; x.y += yy; }
  }
  if (lane == kWave - 1) s_w[w] = x;
  __syncthreads();
  int2 off = make_int2(0, 0);
#pragma unroll
  for (int j = 0; j < 4; ++j)
    if (j < w) { off.x += s_w[j].x; off.y += s_w[j].y; }
  int2 run = make_int2(off.x + x.x - tot.x, off.y + x.y - tot.y);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    if (w0 + q < n_words) word_pre[w0 + q] = run;
    run.x += __popc(m[q]);
    run.y += nz_bytes(m[q]);
  }
  if (t == 255) block_tot[blockIdx.x] = make_int2(off.x + x.x, off.y + x.y);
}

// one block: exclusive scan of the block totals in place; hdr = {entries, distinct rows}
__global__ __launch_bounds__(1024) void runs_scan_blocks_kernel(int2* __restrict__ block_tot,
                                                                int64_t n_blocks,
                                                                int32_t* __restrict__ hdr) {
  __shared__ int2 s_w[16];
  __shared__ int2 s_carry;
  const int t = threadIdx.x, lane = t & (kWave - 1), w = t / kWave;
  if (t == 0) s_carry = make_int2(0, 0);
  __syncthreads();
  for (int64_t b0 = 0; b0 < n_blocks; b0 += 1024) {
    const int64_t b = b0 + t;
    const int2 v = b < n_blocks ? block_tot[b] : make_int2(0, 0);
    int2 x = v;
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
      const int yx = __shfl_up(x.x, o, kWave), yy = __shfl_up(x.y, o, kWave);
      if (lane >= o) { x.x += yx; x.y += yy; }
    }
    if (lane == kWave - 1) s_w[w] = x;
    __syncthreads();
    int2 off = s_carry;
    for (int j = 0; j < w; ++j) { off.x += s_w[j].x; off.y += s_w[j].y; }
    if (b < n_blocks) block_tot[b] = make_int2(off.x + x.x - v.x, off.y + x.y - v.y);
    __syncthreads();
    if (t == 1023) s_carry = make_int2(off.x + x.x, off.y + x.y);
    __syncthreads();
  }
  if (t == 0) { hdr[0] = s_carry.x; hdr[1] = s_carry.y; }
}

__global__ __launch_bounds__(256) void runs_scatter_kernel(
    const int32_t* __restrict__ ids, int64_t C, int64_t S, int32_t spare,
    const uint32_t* __restrict__ mask, const int2* __restrict__ word_pre,
    const int2* __restrict__ block_pre, const int32_t* __restrict__ hdr,
    const int32_t* __restrict__ run_len, ctr_sparse_plan plan) {
  const int32_t T = hdr[0], UR = hdr[1];
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < S;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int j = (int)(e / C);
    const int64_t i = e - (int64_t)j * C;
    const int32_t r = ids[e];
    if (r != spare) {
      const int64_t wi = r >> 2;
      const uint32_t m = mask[wi];
      const int sh = (r & 3) << 3;
      const uint32_t below = sh ? (m & ((1u << sh) - 1u)) : 0u;  // the word's smaller rows
      const uint32_t mine = (m >> sh) & 0xffu;
      const int2 wp = word_pre[wi], bp = block_pre[wi / kRunWordsPerBlock];
      const int32_t base = bp.x + wp.x + __popc(below);
      const int32_t seg = bp.y + wp.y + nz_bytes(below);
      const uint32_t before = mine & ((1u << j) - 1u);  // runs below this one holding r
      const int32_t pos = base + __popc(before);
      plan.sorted_rows[pos] = r;
      plan.sorted_slots[pos] = (int32_t)e;
      plan.pos_seg[pos] = seg;
      if (before == 0) {
        plan.unique_rows[seg] = r;
        plan.seg_offsets[seg] = base;
      }
    } else {
      int32_t pad_before = 0;  // padding entries of the runs below
      for (int q = 0; q < j; ++q) pad_before += (int32_t)C - run_len[q];
      const int32_t pos = T + pad_before + (int32_t)(i - run_len[j]);
      plan.sorted_rows[pos] = spare;
      plan.sorted_slots[pos] = (int32_t)e;
      plan.pos_seg[pos] = UR;
      if (pos == T) {
        plan.unique_rows[UR] = spare;
        plan.seg_offsets[UR] = T;
      }
    }
    if (e == 0) {
      const int32_t U = UR + (T < (int32_t)S ? 1 : 0);
      *plan.num_unique = U;
      plan.seg_offsets[U] = (int32_t)S;
    }
  }
}

__global__ __launch_bounds__(256) void runs_clear_kernel(const int32_t* __restrict__ ids,
                                                         int64_t S, int32_t spare,
                                                         uint32_t* __restrict__ mask) {
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < S;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int32_t r = ids[e];
    if (r != spare) mask[r >> 2] = 0u;  // every writer of a word stores 0
  }
}

extern "C" int ctr_plan_slot_to_unique(const ctr_sparse_plan* plan, int32_t* slot_to_unique,
                                       ctr_stream_t stream) {
  CTR_REQUIRE(plan_ok(plan) && slot_to_unique, "ctr_plan_slot_to_unique: bad arguments");
  if (plan->S == 0) return CTR_OK;
  const unsigned grid = (unsigned)std::min<int64_t>(ceil_div(plan->S, 256), 4096);
  hipLaunchKernelGGL(slot_to_unique_kernel, grid, 256, 0, as_stream(stream), plan->sorted_slots,
                     plan->pos_seg, plan->S, slot_to_unique);
  CTR_LAUNCH_CHECK("slot_to_unique_kernel");
  return CTR_OK;
}

extern "C" int ctr_plan_shard_counts(const ctr_sparse_plan* plan, int64_t shard_rows,
                                     int n_shards, int64_t* counts, ctr_stream_t stream) {
  return ctr_plan_shard_counts_max(plan, shard_rows, n_shards, counts, nullptr, stream);
}

extern "C" int ctr_plan_shard_counts_max(const ctr_sparse_plan* plan, int64_t shard_rows,
                                         int n_shards, int64_t* counts, int64_t* max_out,
                                         ctr_stream_t stream) {
  CTR_REQUIRE(plan_ok(plan) && counts && shard_rows > 0 && n_shards > 0,
              "ctr_plan_shard_counts: bad arguments");
  // the last boundary is lower_bound(n_shards * shard_rows): int32 ids stay below it
  if (n_shards <= kCountsMaxShards) {
    hipLaunchKernelGGL(shard_counts_max_kernel, 1, kWave * (n_shards + 1), 0, as_stream(stream),
                       plan->unique_rows, plan->num_unique, shard_rows, n_shards, counts, max_out);
    CTR_LAUNCH_CHECK("shard_counts_max_kernel");
    return CTR_OK;
  }
  CTR_REQUIRE(max_out == nullptr, "ctr_plan_shard_counts_max: the maximum needs <= %d shards",
              kCountsMaxShards);
  hipLaunchKernelGGL(shard_counts_kernel, (unsigned)ceil_div(n_shards, 64), 64, 0,
                     as_stream(stream), plan->unique_rows, plan->num_unique, shard_rows, n_shards,
                     counts);
  CTR_LAUNCH_CHECK("shard_counts_kernel");
  return CTR_OK;
}

extern "C" int ctr_ids_add(int32_t* ids, int64_t n, int32_t delta, ctr_stream_t stream) {
  CTR_REQUIRE(n >= 0 && (ids || n == 0), "ctr_ids_add: bad arguments");
  if (n == 0) return CTR_OK;
  const unsigned grid = (unsigned)std::min<int64_t>(ceil_div(n, 256), 4096);
  hipLaunchKernelGGL(ids_add_kernel, grid, 256, 0, as_stream(stream), ids, n, delta);
  CTR_LAUNCH_CHECK("ids_add_kernel");
  return CTR_OK;
}

static int shard_pack_ids_impl(const ctr_sparse_plan* plan, int64_t shard_rows, int64_t V,
                               int n_shards, int cyclic, int64_t capacity, int32_t* send,
                               int32_t* counts, int32_t* offsets, int32_t* err_flag,
                               ctr_stream_t stream) {
  CTR_REQUIRE(plan_ok(plan) && send && counts && offsets && shard_rows > 0 && n_shards > 0 &&
                  capacity > 0 && V > 0 && shard_rows * n_shards >= V,
              "ctr_shard_pack_ids: bad arguments");
  CTR_REQUIRE(shard_rows < (int64_t(1) << 31), "ctr_shard_pack_ids: shard too large");
  const dim3 grid((unsigned)std::min<int64_t>(ceil_div(capacity, 256), 1024), (unsigned)n_shards);
  hipLaunchKernelGGL(shard_pack_ids_kernel, grid, 256, 0, as_stream(stream), plan->unique_rows,
                     plan->num_unique, shard_rows, V, capacity, send, counts, offsets, err_flag,
                     cyclic ? n_shards : 0);
  CTR_LAUNCH_CHECK("shard_pack_ids_kernel");
  return CTR_OK;
}

extern "C" int ctr_shard_pack_ids(const ctr_sparse_plan* plan, int64_t shard_rows, int64_t V,
                                  int n_shards, int64_t capacity, int32_t* send, int32_t* counts,
                                  int32_t* offsets, int32_t* err_flag, ctr_stream_t stream) {
  return shard_pack_ids_impl(plan, shard_rows, V, n_shards, 0, capacity, send, counts, offsets,
                             err_flag, stream);
}

extern "C" int ctr_shard_pack_ids_layout(const ctr_sparse_plan* plan, int64_t shard_rows,
                                         int64_t V, int n_shards, int cyclic, int64_t capacity,
                                         int32_t* send, int32_t* counts, int32_t* offsets,
                                         int32_t* err_flag, ctr_stream_t stream) {
  return shard_pack_ids_impl(plan, shard_rows, V, n_shards, cyclic, capacity, send, counts,
                             offsets, err_flag, stream);
}

extern "C" int ctr_shard_permute_ids(void* ids, int ids_is_64, int64_t count, int64_t V,
                                     int n_shards, int64_t shard_rows, int32_t* err_flag,
                                     ctr_stream_t stream) {
  CTR_REQUIRE(count >= 0 && (ids || count == 0) && V > 0 && n_shards > 0 && shard_rows > 0 &&
                  shard_rows * n_shards >= V,
              "ctr_shard_permute_ids: bad arguments");
  CTR_REQUIRE(ids_is_64 || shard_rows * n_shards < (int64_t(1) << 31),
              "ctr_shard_permute_ids: int32 ids cannot address the permuted space");
  if (count == 0) return CTR_OK;
  const unsigned grid = (unsigned)std::min<int64_t>(ceil_div(count, 256), 4096);
  if (ids_is_64)
    hipLaunchKernelGGL(shard_permute_ids_kernel<int64_t>, grid, 256, 0, as_stream(stream),
                       static_cast<int64_t*>(ids), count, V, (int64_t)n_shards, shard_rows, err_flag);
  else
    hipLaunchKernelGGL(shard_permute_ids_kernel<int32_t>, grid, 256, 0, as_stream(stream),
                       static_cast<int32_t*>(ids), count, V, (int64_t)n_shards, shard_rows, err_flag);
  CTR_LAUNCH_CHECK("shard_permute_ids_kernel");
  return CTR_OK;
}

extern "C" int ctr_shard_runs_copy(const float* src, float* dst, int64_t width, int64_t capacity,
                                   int n_shards, const int32_t* counts, const int32_t* offsets,
                                   int pack, ctr_stream_t stream) {
  CTR_REQUIRE(src && dst && counts && offsets && width > 0 && capacity > 0 && n_shards > 0,
              "ctr_shard_runs_copy: bad arguments");
  hipStream_t st = as_stream(stream);
  const bool vec = width % 4 == 0 && ((uintptr_t)src | (uintptr_t)dst) % 16 == 0;
  const int64_t W = vec ? width / 4 : width;
  const dim3 grid((unsigned)std::min<int64_t>(ceil_div(capacity * W, 256), 2048), (unsigned)n_shards);
  if (vec) {
    const float4* s4 = reinterpret_cast<const float4*>(src);
    float4* d4 = reinterpret_cast<float4*>(dst);
    if (pack) hipLaunchKernelGGL((shard_runs_copy_kernel<float4, true>), grid, 256, 0, st, s4, d4, W, capacity, counts, offsets);
    else hipLaunchKernelGGL((shard_runs_copy_kernel<float4, false>), grid, 256, 0, st, s4, d4, W, capacity, counts, offsets);
  } else {
    if (pack) hipLaunchKernelGGL((shard_runs_copy_kernel<float, true>), grid, 256, 0, st, src, dst, W, capacity, counts, offsets);
    else hipLaunchKernelGGL((shard_runs_copy_kernel<float, false>), grid, 256, 0, st, src, dst, W, capacity, counts, offsets);
  }
  CTR_LAUNCH_CHECK("shard_runs_copy_kernel");
  return CTR_OK;
}

// chunked E + linear rows (shard_rows_lin_kernel): chunk >= C*K (+ C with a linear table),
// a multiple of 4; K % 4 == 0; 16-B aligned buffers
static bool rows_lin_ok(const void* a, const void* b, int K, int64_t C, int64_t chunk, bool lin) {
  return a && b && K > 0 && K % 4 == 0 && C > 0 && chunk % 4 == 0 &&
         chunk >= C * K + (lin ? C : 0) && ((uintptr_t)a | (uintptr_t)b) % 16 == 0;
}

template <int MODE>
static int rows_lin_launch(const float* src, const float* src_lin, float* dst, float* dst_lin,
                           const int32_t* ids, int K, int64_t C, int64_t chunk, int n_shards,
                           const int32_t* counts, const int32_t* offsets, ctr_stream_t stream) {
  const int64_t K4 = K / 4;
  const dim3 grid((unsigned)std::min<int64_t>(ceil_div(C * K4, 256), 2048), (unsigned)n_shards);
  hipLaunchKernelGGL(shard_rows_lin_kernel<MODE>, grid, 256, 0, as_stream(stream),
                     reinterpret_cast<const float4*>(src), src_lin, reinterpret_cast<float4*>(dst),
                     dst_lin, ids, K4, C, chunk, counts, offsets);
  CTR_LAUNCH_CHECK("shard_rows_lin_kernel");
  return CTR_OK;
}

extern "C" int ctr_shard_gather_rows(const float* emb, const float* lin, int K, const int32_t* ids,
                                     int n_shards, int64_t capacity, int64_t chunk, float* out,
                                     ctr_stream_t stream) {
  CTR_REQUIRE(ids && n_shards > 0 && rows_lin_ok(emb, out, K, capacity, chunk, lin != nullptr),
              "ctr_shard_gather_rows: bad arguments");
  return rows_lin_launch<kRowsGather>(emb, lin, out, nullptr, ids, K, capacity, chunk, n_shards,
                                      nullptr, nullptr, stream);
}

extern "C" int ctr_shard_rows_pack(const float* rows, const float* lin, int K, int64_t capacity,
                                   int64_t chunk, int n_shards, const int32_t* counts,
                                   const int32_t* offsets, float* out, ctr_stream_t stream) {
  CTR_REQUIRE(counts && offsets && n_shards > 0 &&
                  rows_lin_ok(rows, out, K, capacity, chunk, lin != nullptr),
              "ctr_shard_rows_pack: bad arguments");
  return rows_lin_launch<kRowsPack>(rows, lin, out, nullptr, nullptr, K, capacity, chunk, n_shards,
                                    counts, offsets, stream);
}

extern "C" int ctr_shard_rows_unpack(const float* in, int K, int64_t capacity, int64_t chunk,
                                     int n_shards, const int32_t* counts, const int32_t* offsets,
                                     float* rows, float* lin, ctr_stream_t stream) {
  CTR_REQUIRE(counts && offsets && n_shards > 0 &&
                  rows_lin_ok(in, rows, K, capacity, chunk, lin != nullptr),
              "ctr_shard_rows_unpack: bad arguments");
  return rows_lin_launch<kRowsUnpack>(in, nullptr, rows, lin, nullptr, K, capacity, chunk,
                                      n_shards, counts, offsets, stream);
}

static int64_t runs_ws_layout(int64_t n_rows, int64_t n_runs, int64_t* off_word, int64_t* off_block,
                              int64_t* off_hdr) {
  const int64_t n_words = ceil_div(std::max<int64_t>(n_rows, 1), 4);
  const int64_t n_blocks = ceil_div(n_words, kRunWordsPerBlock);
  *off_word = 0;
  *off_block = align_up(n_words * 8, 256);
  *off_hdr = *off_block + align_up(n_blocks * 8, 256);
  return *off_hdr + align_up((2 + n_runs) * 4, 256);
}

extern "C" int64_t ctr_sparse_plan_runs_workspace_bytes(int n_runs, int64_t run_len,
                                                        int64_t n_rows) {
  if (n_runs < 1 || n_runs > 8 || run_len < 1 || n_rows < 1) {
    set_error("ctr_sparse_plan_runs_workspace_bytes: need 1 <= n_runs <= 8, run_len >= 1, "
              "n_rows >= 1");
    return -1;
  }
  int64_t a, b, c;
  return runs_ws_layout(n_rows, n_runs, &a, &b, &c);
}

extern "C" int ctr_sparse_plan_build_runs(const int32_t* ids, int n_runs, int64_t run_len,
                                          int64_t n_rows, const ctr_sparse_plan* plan,
                                          uint32_t* mask, void* ws, int64_t ws_bytes,
                                          ctr_stream_t stream) {
  CTR_REQUIRE(plan_ok(plan) && ids && mask, "ctr_sparse_plan_build_runs: bad arguments");
  CTR_REQUIRE(n_runs >= 1 && n_runs <= 8 && run_len >= 1 && n_rows >= 1 &&
                  n_rows < (int64_t(1) << 31) && plan->S == n_runs * run_len &&
                  plan->S < (int64_t(1) << 31),
              "ctr_sparse_plan_build_runs: need 1 <= n_runs <= 8, S = n_runs * run_len");
  int64_t ow, ob, oh;
  const int64_t need = runs_ws_layout(n_rows, n_runs, &ow, &ob, &oh);
  CTR_REQUIRE(ws && ws_bytes >= need, "ctr_sparse_plan_build_runs: workspace too small");
  char* base = static_cast<char*>(ws);
  int2* word_pre = reinterpret_cast<int2*>(base + ow);
  int2* block_tot = reinterpret_cast<int2*>(base + ob);
  int32_t* hdr = reinterpret_cast<int32_t*>(base + oh);
  int32_t* run_len_d = hdr + 2;
  const int64_t S = plan->S, n_words = ceil_div(n_rows, 4);
  const int64_t n_blocks = ceil_div(n_words, kRunWordsPerBlock);
  const int32_t spare = (int32_t)(n_rows - 1);
  hipStream_t st = as_stream(stream);
  const unsigned g = (unsigned)std::max<int64_t>(1, std::min<int64_t>(ceil_div(S, 256), 4096));
  hipLaunchKernelGGL(runs_mark_kernel, g, 256, 0, st, ids, run_len, S, spare, mask, run_len_d);
  CTR_LAUNCH_CHECK("runs_mark_kernel");
  hipLaunchKernelGGL(runs_scan_words_kernel, (unsigned)n_blocks, 256, 0, st, mask, n_words,
                     word_pre, block_tot);
  CTR_LAUNCH_CHECK("runs_scan_words_kernel");
  hipLaunchKernelGGL(runs_scan_blocks_kernel, 1, 1024, 0, st, block_tot, n_blocks, hdr);
  CTR_LAUNCH_CHECK("runs_scan_blocks_kernel");
  hipLaunchKernelGGL(runs_scatter_kernel, g, 256, 0, st, ids, run_len, S, spare, mask,
                     word_pre, block_tot, hdr, run_len_d, *plan);
  CTR_LAUNCH_CHECK("runs_scatter_kernel");
  hipLaunchKernelGGL(runs_clear_kernel, g, 256, 0, st, ids, S, spare, mask);
  CTR_LAUNCH_CHECK("runs_clear_kernel");
  return CTR_OK;
}

// Embedding scatter-add of the CTR hot path, deterministic.
//
// The reference's autograd writes a DENSE [V,K] gradient (embedding_dense_backward
// accumulates the slots of each row in slot order). Here a batch's S = B*F slots are
// grouped once per step into a sparse plan (csrc/sparse_plan.hip: a stable radix sort of
// (row, slot) pairs, then segment heads) and each row's contributions are summed in slot
// order.
// Hot rows (Zipf ids: one row can own >1000 slots of a batch) are split into fixed
// 16-position chunks so every lane group does equal work; chunk partials of rows that
// span chunks are added in chunk order by a second pass. No float atomics anywhere: the
// result is bitwise reproducible, which is what keeps data-parallel replicas identical.
#include "adam_common.h"

// FM rows: the per-slot term without the row's own embedding (g*s + d), the row term
// -(sum g) * e added once per row where its sum completes — the embedding row is then read
// once per unique row (the apply pass holds it anyway) instead of once per slot (at C3 the
// 54 MB of random row reads in seg_chunk). The sums differ from the per-slot form by fp32
// association only, within the oracle's gradient bar (tests/conftest.py: both terms are in
// grad_condition). CTR_SEG_FM_DEFER=0 builds the per-slot form.
#ifndef CTR_SEG_FM_DEFER
#define CTR_SEG_FM_DEFER 1
#endif

namespace ctr {

// Sorted positions per lane group: 16 when a row is >= 16 lane columns (K >= 64), else 4
// (small K: more, shorter chunks keep enough waves in flight to hide the gather latency).
constexpr int kMinChunk = 4;
template <int LPR>
constexpr int seg_chunk() { return LPR >= 16 ? 16 : 4; }

// ------------------------------------------------------- segmented row sums ----------
// Vector width VT (float4 when K % 4 == 0, else float), KV = K / width columns, LPR lanes
// per row (power of two >= KV), one lane group per chunk of CHUNK sorted positions.
template <typename VT>
struct VOps;
template <>
struct VOps<float> {
  __device__ static float zero() { return 0.f; }
  __device__ static void add(float& a, float b) { a += b; }
  __device__ static float shfl_xor(float v, int o) { return __shfl_xor(v, o, kWave); }
  // (g*s - g*e) + d, each product rounded (the reference's two autograd terms)
  __device__ static float fm(float g, float s, float e, float d) {
#pragma clang fp contract(off)
    return (g * s - g * e) + d;
  }
  // the slot's term without its row: g*s + d (the row's -e * sum(g) is added once per row)
  __device__ static float fm2(float g, float s, float d) {
#pragma clang fp contract(off)
    return g * s + d;
  }
  // a row's sum of fm2 terms A and its sum of g, c: A - c*e (the product rounded)
  __device__ static float fin(float acc, float c, float e) {
#pragma clang fp contract(off)
    return acc - c * e;
  }
};
template <>
struct VOps<float4> {
  __device__ static float4 zero() { return make_float4(0.f, 0.f, 0.f, 0.f); }
  __device__ static float4 shfl_xor(float4 v, int o) {
    return make_float4(__shfl_xor(v.x, o, kWave), __shfl_xor(v.y, o, kWave),
                       __shfl_xor(v.z, o, kWave), __shfl_xor(v.w, o, kWave));
  }
  __device__ static void add(float4& a, float4 b) {
    a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
  }
  __device__ static float4 fm(float g, float4 s, float4 e, float4 d) {
    return make_float4(VOps<float>::fm(g, s.x, e.x, d.x), VOps<float>::fm(g, s.y, e.y, d.y),
                       VOps<float>::fm(g, s.z, e.z, d.z), VOps<float>::fm(g, s.w, e.w, d.w));
  }
  __device__ static float4 fm2(float g, float4 s, float4 d) {
    return make_float4(VOps<float>::fm2(g, s.x, d.x), VOps<float>::fm2(g, s.y, d.y),
                       VOps<float>::fm2(g, s.z, d.z), VOps<float>::fm2(g, s.w, d.w));
  }
  __device__ static float4 fin(float4 acc, float c, float4 e) {
    return make_float4(VOps<float>::fin(acc.x, c, e.x), VOps<float>::fin(acc.y, c, e.y),
                       VOps<float>::fin(acc.z, c, e.z), VOps<float>::fin(acc.w, c, e.w));
  }
};

struct SegArgs {
  int64_t S;
  int KV;
  const int32_t* sorted_slots;
  const int32_t* sorted_rows;
  const int32_t* pos_seg;
  const int32_t* unique_rows;
  const int32_t* seg_offsets;
  const int32_t* num_unique;
  // FM contribution (MODE_FM)
  int F;
  const float* gz;
  const void* sum_e;
  const void* dx;
  const void* emb;
  // FM with the row term deferred (CTR_SEG_FM_DEFER): per slot g*s + d, per row
  // sum - (sum g) * e, e read once per row (emb by unique row, or by segment ordinal for a
  // table compacted in unique order: emb_by_seg)
  bool fm_defer;
  bool emb_by_seg;
  // generic contribution (MODE_VALS)
  const void* vals;
  const float* vals_lin;
  // outputs
  void* out;
  float* out_lin;
  int32_t* rowmap;
  void* part;       // [n_chunks, 2, KV]  chunk partials: [0] run holding the chunk's first
  float* part_lin;  // [n_chunks, 2]      position, [1] the chunk's last (open) run
  // fused deferred-Adam apply (float4 path, seg_combine_apply_kernel): every row's final
  // sum is applied to the table by the pass that finishes the spanning rows
  bool apply;
  bool out_keep;  // apply mode: also write the spanning rows' sums to out / out_lin
  float4 *E, *mE, *vE;
  float *w, *mw, *vw;
  int32_t* last;
  const int32_t* step_ptr;
  const float* tab;
  AdamHP hp;
  // row-sharded requester (map_n > 0): row u's sum goes straight into its owner's exchange
  // chunk — run j = the last with map_off[j] <= u, row u - map_off[j] of chunk j (map_chunk
  // floats from out), its linear sum after the chunk's map_C rows (map_lin)
  int map_n;
  bool map_lin;
  const int32_t* map_off;
  int64_t map_C, map_chunk;
};

// a completed row sum: written out (and the rowmap entry of the dense-mode optimizer)
template <typename VT>
__device__ __forceinline__ void seg_emit(const SegArgs& a, int64_t u, int c, bool col,
                                         const VT& acc, float accl) {
  if (a.map_n > 0) {
    int j = 0;
    while (j + 1 < a.map_n && u >= a.map_off[j + 1]) ++j;
    const int64_t i = u - a.map_off[j];
    // a run longer than the capacity (flagged CTR_EFLAG_CAPACITY by shard_pack_ids, raised
    // by the host's check) must not spill into the next owner's chunk: its rows past C are
    // dropped here, as the pack / unpack kernels clamp to min(count, C)
    if (i >= a.map_C) return;
    float* const base = static_cast<float*>(a.out) + j * a.map_chunk;
    if (col) reinterpret_cast<VT*>(base)[i * a.KV + c] = acc;
    if (c == 0 && a.map_lin)
      base[a.map_C * a.KV * (int64_t)(sizeof(VT) / sizeof(float)) + i] = accl;
    return;
  }
  if (col) static_cast<VT*>(a.out)[u * a.KV + c] = acc;
  if (c == 0) {
    if (a.out_lin) a.out_lin[u] = accl;
    if (a.rowmap) a.rowmap[a.unique_rows[u]] = (int32_t)u;
  }
}

// a completed row sum of the deferred FM form: its row term, then written out
template <typename VT>
__device__ __forceinline__ void seg_final(const SegArgs& a, int64_t u, int c, bool col, VT acc,
                                          float accl) {
  if (a.fm_defer && col) {
    const int64_t r = a.emb_by_seg ? u : (int64_t)a.unique_rows[u];
    acc = VOps<VT>::fin(acc, accl, static_cast<const VT*>(a.emb)[r * a.KV + c]);
  }
  seg_emit<VT>(a, u, c, col, acc, accl);
}

enum { MODE_FM = 0, MODE_VALS = 1 };

template <typename VT, int LPR, int MODE>
__global__ __launch_bounds__(256) void seg_chunk_kernel(SegArgs a) {
  constexpr int kChunk = seg_chunk<LPR>();
  const int64_t gid = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) / LPR;
  const int c = threadIdx.x % LPR;
  const int64_t start = gid * kChunk;
  if (start >= a.S) return;
  const bool col = c < a.KV;
  const int n = (int)min<int64_t>(kChunk, a.S - start);

  // Stage every load of the chunk first (ILP), then walk the runs in slot order.
  int seg[kChunk];
  VT val[kChunk];
  float gl[kChunk];
#pragma unroll
  for (int i = 0; i < kChunk; ++i) {
    seg[i] = -1;
    val[i] = VOps<VT>::zero();
    gl[i] = 0.f;
    if (i < n) {
      const int64_t pos = start + i;
      const int32_t slot = a.sorted_slots[pos];
      seg[i] = a.pos_seg[pos];
      if (MODE == MODE_FM) {
        const int64_t b = slot / a.F;
        const float g = a.gz[b];
        gl[i] = g;
        if (col) {
          const VT s = static_cast<const VT*>(a.sum_e)[b * a.KV + c];
          const VT d = a.dx ? static_cast<const VT*>(a.dx)[(int64_t)slot * a.KV + c]
                            : VOps<VT>::zero();
          if (a.fm_defer) {  // the row's own term once per row (seg_final / the apply)
            val[i] = VOps<VT>::fm2(g, s, d);
          } else {
            const int32_t row = a.sorted_rows[pos];
            const VT e = static_cast<const VT*>(a.emb)[(int64_t)row * a.KV + c];
            val[i] = VOps<VT>::fm(g, s, e, d);
          }
        }
      } else {
        if (a.vals_lin) gl[i] = a.vals_lin[slot];
        if (col) val[i] = static_cast<const VT*>(a.vals)[(int64_t)slot * a.KV + c];
      }
    }
  }

  auto flush = [&](int u, const VT& acc, float accl, bool first_run) {
    const int32_t off0 = a.seg_offsets[u];
    const int32_t off1 = a.seg_offsets[u + 1];
    if (off0 / kChunk == (off1 - 1) / kChunk) {  // whole row inside this chunk: final
      if (a.apply)  // the apply pass adds the deferred row term (it holds the row)
        seg_emit<VT>(a, u, c, col, acc, accl);
      else
        seg_final<VT>(a, u, c, col, acc, accl);
    } else {
      const int64_t k = gid * 2 + (first_run ? 0 : 1);
      if (col) static_cast<VT*>(a.part)[k * a.KV + c] = acc;
      if (c == 0) a.part_lin[k] = accl;
    }
  };

  VT acc = VOps<VT>::zero();
  float accl = 0.f;
  int cur = seg[0];
  bool first_run = true;
#pragma unroll
  for (int i = 0; i < kChunk; ++i) {
    if (i < n) {
      if (seg[i] != cur) {
        flush(cur, acc, accl, first_run);
        acc = VOps<VT>::zero();
        accl = 0.f;
        cur = seg[i];
        first_run = false;
      }
      VOps<VT>::add(acc, val[i]);
      accl += gl[i];
    }
  }
  flush(cur, acc, accl, first_run);
}

// Rows that span chunks, one wave per row: the row's P chunk partials (the first chunk's
// open run — slot [0] if the row starts the chunk, else [1] — then slot [0] of every later
// chunk) are dealt round-robin to the wave's 64/LPR lane groups, each sums its share in
// chunk order, and the group sums meet in a fixed xor butterfly: a fixed summation tree for
// a given P, so bitwise reproducible, and a hot Zipf row of thousands of slots is no longer
// one lane group's serial walk.
template <typename VT, int LPR>
__global__ __launch_bounds__(256) void seg_combine_kernel(SegArgs a) {
  constexpr int kChunk = seg_chunk<LPR>();
  constexpr int G = kWave / LPR;
  const int lane = threadIdx.x & (kWave - 1);
  const int g = lane / LPR, c = lane % LPR;
  const bool col = c < a.KV;
  const int64_t waves = (int64_t)gridDim.x * (blockDim.x / kWave);
  const int U = *a.num_unique;
  for (int64_t u = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) / kWave; u < U; u += waves) {
    const int32_t off0 = a.seg_offsets[u];
    const int32_t off1 = a.seg_offsets[u + 1];
    const int64_t fs = off0 / kChunk, ls = (off1 - 1) / kChunk;
    if (fs == ls) continue;  // wave-uniform
    const int64_t P = ls - fs + 1;
    VT acc = VOps<VT>::zero();
    float accl = 0.f;
    for (int64_t i = g; i < P; i += G) {
      const int64_t k = i == 0 ? fs * 2 + ((off0 % kChunk) == 0 ? 0 : 1) : (fs + i) * 2;
      if (col) VOps<VT>::add(acc, static_cast<const VT*>(a.part)[k * a.KV + c]);
      accl += a.part_lin[k];
    }
#pragma unroll
    for (int o = LPR; o < kWave; o <<= 1) {
      VOps<VT>::add(acc, VOps<VT>::shfl_xor(acc, o));
      accl += __shfl_xor(accl, o, kWave);
    }
    if (g == 0) seg_final<VT>(a, u, c, col, acc, accl);
  }
}

// The combine pass with the deferred Adam apply fused in (float4): a wave takes G = 64/LPR
// consecutive unique rows, lane group g row u0 + g, and every lane group applies its own
// row — the sum from seg_chunk's `out` for a row inside one chunk — so the G applies (the
// memory-heavy part) run side by side. One launch for what the combine and
// ctr_adam_deferred_rows did in two, and the spanning rows' sums never make the round trip
// through `out`.
// A spanning row's sum is seg_combine_kernel's, bit for bit: G accumulators, accumulator s
// the running sum (from zero) of pieces s, s+G, s+2G ... in chunk order, then the pairwise
// tree over the G accumulators in index order that the xor butterfly forms. A row of at
// most T pieces (the common case: a few chunks) is summed that way by its own lane group,
// every piece load in flight at once and all G rows side by side; a row of more pieces (hot
// Zipf rows) by the whole wave — lane group g accumulator g, then the butterfly — into a
// wave-private LDS slot, one such row after another. (The whole-wave walk over every
// spanning row cost a dependent segment-bounds + partials round trip per row, serially.)
template <int LPR>
__global__ __launch_bounds__(256) void seg_combine_apply_kernel(SegArgs a) {
  using VT = float4;
  constexpr int kChunk = seg_chunk<LPR>();
  constexpr int G = kWave / LPR;
  // most pieces one lane group sums alone (accumulators past T stay zero, still in the tree)
  constexpr int T = G < 8 ? 8 : (G > 16 ? 16 : G);
  __shared__ VT s_sum[4][kWave];      // [wave][row of the G * lane group column]
  __shared__ float s_lin[4][G];
  const int lane = threadIdx.x & (kWave - 1);
  const int wib = threadIdx.x / kWave;
  const int g = lane / LPR, c = lane % LPR;
  const bool col = c < a.KV;
  const int64_t waves = (int64_t)gridDim.x * (blockDim.x / kWave);
  const int U = *a.num_unique;
  const int step = *a.step_ptr;
  const VT* __restrict__ part = static_cast<const VT*>(a.part);
  for (int64_t u0 = ((blockIdx.x * (int64_t)blockDim.x + threadIdx.x) / kWave) * G; u0 < U;
       u0 += waves * G) {
    const int64_t u = u0 + g;
    const bool valid = u < U;
    int32_t off0 = 0, off1 = 1;
    if (valid) {
      off0 = a.seg_offsets[u];
      off1 = a.seg_offsets[u + 1];
    }
    const int64_t fs = off0 / kChunk, ls = (off1 - 1) / kChunk;
    const int P = (int)(ls - fs + 1);  // pieces: 1 = inside one chunk
    const int64_t k0 = fs * 2 + ((off0 % kChunk) == 0 ? 0 : 1);  // piece 0's partial slot
    // rows of more than T pieces: the whole wave, one row after another
    uint64_t big = __ballot(valid && P > T && c == 0);
    while (big) {
      const int src = __builtin_ctzll(big);
      big &= big - 1;
      const int j = src / LPR;
      const int Pj = __shfl(P, src, kWave);
      const int64_t fsj = __shfl((int)fs, src, kWave);
      const int64_t k0j = __shfl((int)k0, src, kWave);
      VT acc = VOps<VT>::zero();
      float accl = 0.f;
      for (int i = g; i < Pj; i += G) {
        const int64_t k = i == 0 ? k0j : (fsj + i) * 2;
        if (col) VOps<VT>::add(acc, part[k * a.KV + c]);
        accl += a.part_lin[k];
      }
#pragma unroll
      for (int o = LPR; o < kWave; o <<= 1) {
        VOps<VT>::add(acc, VOps<VT>::shfl_xor(acc, o));
        accl += __shfl_xor(accl, o, kWave);
      }
      if (g == 0) {
        s_sum[wib][j * LPR + c] = acc;
        if (c == 0) s_lin[wib][j] = accl;
      }
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the wave-private slots are written
    __builtin_amdgcn_wave_barrier();
    if (valid) {
      VT gr;
      float gl;
      if (P == 1) {
        gr = col ? static_cast<const VT*>(a.out)[u * a.KV + c] : VOps<VT>::zero();
        gl = a.out_lin ? a.out_lin[u] : 0.f;
      } else if (P <= T) {
        VT acc[G];
        float accl[G];
#pragma unroll
        for (int s = 0; s < G; ++s) {
          acc[s] = VOps<VT>::zero();
          accl[s] = 0.f;
        }
#pragma unroll
        for (int i = 0; i < T; ++i) {
          if (i < P) {
            const int64_t k = i == 0 ? k0 : (fs + i) * 2;
            if (col) VOps<VT>::add(acc[i % G], part[k * a.KV + c]);
            accl[i % G] += a.part_lin[k];
          }
        }
#pragma unroll
        for (int w2 = 1; w2 < G; w2 <<= 1)
#pragma unroll
          for (int s = 0; s + w2 < G; s += 2 * w2) {
            VOps<VT>::add(acc[s], acc[s + w2]);
            accl[s] += accl[s + w2];
          }
        gr = acc[0];
        gl = accl[0];
      } else {
        gr = s_sum[wib][g * LPR + c];
        gl = s_lin[wib][g];
      }
      const int64_t r = a.unique_rows[u];
      if (a.fm_defer && col)  // the row's term: e = the row as the forward read it (step-1)
        gr = VOps<VT>::fin(gr, gl, a.E[r * a.KV + c]);
      if ((P > 1 || a.fm_defer) && a.out_keep) seg_emit<VT>(a, u, c, col, gr, gl);
      deferred_apply_row(a.E, a.mE, a.vE, a.w, a.mw, a.vw, a.last, r, a.KV, c,
                         col, gr, gl, step, a.tab, a.hp);
    }
    __builtin_amdgcn_wave_barrier();  // the slots are re-filled by the next iteration
  }
}

template <typename VT, int LPR>
static int launch_seg_lpr(SegArgs& a, int mode, hipStream_t st) {
  const int64_t n_chunks = ceil_div(a.S, seg_chunk<LPR>());
  const int groups_per_block = 256 / LPR;
  const unsigned g1 = (unsigned)ceil_div(n_chunks, groups_per_block);
  if (mode == MODE_FM)
    hipLaunchKernelGGL((seg_chunk_kernel<VT, LPR, MODE_FM>), g1, 256, 0, st, a);
  else
    hipLaunchKernelGGL((seg_chunk_kernel<VT, LPR, MODE_VALS>), g1, 256, 0, st, a);
  CTR_LAUNCH_CHECK("seg_chunk_kernel");
  // one wave per unique row (rows are at most S): up to 2048 blocks of 4 waves
  const unsigned g2 = (unsigned)std::max<int64_t>(1, std::min<int64_t>(ceil_div(a.S, 4), 2048));
  if constexpr (std::is_same<VT, float4>::value) {
    if (a.apply) {
      hipLaunchKernelGGL((seg_combine_apply_kernel<LPR>), g2, 256, 0, st, a);
      CTR_LAUNCH_CHECK("seg_combine_apply_kernel");
      return CTR_OK;
    }
  }
  hipLaunchKernelGGL((seg_combine_kernel<VT, LPR>), g2, 256, 0, st, a);
  CTR_LAUNCH_CHECK("seg_combine_kernel");
  return CTR_OK;
}

static int pow2_at_least(int x) {
  int p = 1;
  while (p < x) p <<= 1;
  return p;
}

static int launch_seg(SegArgs& a, int K, int mode, hipStream_t st, bool aligned16) {
  const bool vec = (K % 4 == 0) && aligned16 && K / 4 <= 64;
  const int KV = vec ? K / 4 : K;
  a.KV = KV;
  const int lpr = pow2_at_least(KV);
  if (vec) {
    switch (lpr) {
      case 1: return launch_seg_lpr<float4, 1>(a, mode, st);
      case 2: return launch_seg_lpr<float4, 2>(a, mode, st);
      case 4: return launch_seg_lpr<float4, 4>(a, mode, st);
      case 8: return launch_seg_lpr<float4, 8>(a, mode, st);
      case 16: return launch_seg_lpr<float4, 16>(a, mode, st);
      case 32: return launch_seg_lpr<float4, 32>(a, mode, st);
      case 64: return launch_seg_lpr<float4, 64>(a, mode, st);
    }
  } else {
    switch (lpr) {
      case 1: return launch_seg_lpr<float, 1>(a, mode, st);
      case 2: return launch_seg_lpr<float, 2>(a, mode, st);
      case 4: return launch_seg_lpr<float, 4>(a, mode, st);
      case 8: return launch_seg_lpr<float, 8>(a, mode, st);
      case 16: return launch_seg_lpr<float, 16>(a, mode, st);
      case 32: return launch_seg_lpr<float, 32>(a, mode, st);
      case 64: return launch_seg_lpr<float, 64>(a, mode, st);
    }
  }
  set_error("segmented row sum: K=%d unsupported (K<=64, or K%%4==0 and K<=256)", K);
  return CTR_ERR_UNSUPPORTED;
}

static int64_t seg_ws_bytes(int64_t S, int K) {
  const int64_t n_chunks = ceil_div(S, kMinChunk);
  return align_up(n_chunks * 2 * (int64_t)K * 4, 256) + align_up(n_chunks * 2 * 4, 256);
}

// ------------------------------------------------------------------ to dense -------
__global__ __launch_bounds__(256) void rows_to_dense_kernel(const int32_t* __restrict__ unique_rows,
                                                            const int32_t* __restrict__ num_unique,
                                                            int K, const float* __restrict__ grad,
                                                            const float* __restrict__ grad_lin,
                                                            float* __restrict__ dense,
                                                            float* __restrict__ dense_lin) {
  const int64_t U = *num_unique;
  const int64_t total = U * K;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t u = t / K;
    const int k = (int)(t - u * K);
    const int64_t row = unique_rows[u];
    dense[row * K + k] = grad[t];
    if (k == 0 && dense_lin && grad_lin) dense_lin[row] = grad_lin[u];
  }
}

static bool plan_ok(const ctr_sparse_plan* p) {
  return p && p->S >= 0 && p->sorted_slots && p->sorted_rows && p->pos_seg && p->unique_rows &&
         p->seg_offsets && p->num_unique;
}

}  // namespace ctr

using namespace ctr;

extern "C" int64_t ctr_segment_workspace_bytes(int64_t S, int K) {
  if (S < 0 || K <= 0) return -1;
  return seg_ws_bytes(S, K);
}

static int seg_prepare(SegArgs& a, const ctr_sparse_plan* plan, int K, void* out, float* out_lin,
                       int32_t* rowmap, void* ws, int64_t ws_bytes) {
  memset(&a, 0, sizeof(a));
  a.S = plan->S;
  a.sorted_slots = plan->sorted_slots;
  a.sorted_rows = plan->sorted_rows;
  a.pos_seg = plan->pos_seg;
  a.unique_rows = plan->unique_rows;
  a.seg_offsets = plan->seg_offsets;
  a.num_unique = plan->num_unique;
  a.out = out;
  a.out_lin = out_lin;
  a.rowmap = rowmap;
  const int64_t need = seg_ws_bytes(plan->S, K);
  if (!ws || ws_bytes < need) {
    set_error("segmented row sum: workspace %lld < %lld bytes", (long long)ws_bytes,
              (long long)need);
    return CTR_ERR_WORKSPACE;
  }
  const int64_t n_chunks = ceil_div(plan->S, kMinChunk);
  a.part = ws;
  a.part_lin = reinterpret_cast<float*>(static_cast<char*>(ws) +
                                        align_up(n_chunks * 2 * (int64_t)K * 4, 256));
  return CTR_OK;
}

extern "C" int ctr_fm_embedding_grad(const ctr_sparse_plan* plan, int F, int K, const float* emb,
                                     const float* gz, const float* sum_e, const float* dx,
                                     float* grad_rows, float* grad_lin, int32_t* rowmap, void* ws,
                                     int64_t ws_bytes, ctr_stream_t stream) {
  CTR_REQUIRE(plan_ok(plan), "ctr_fm_embedding_grad: incomplete plan");
  CTR_REQUIRE(F > 0 && K > 0, "ctr_fm_embedding_grad: bad sizes");
  CTR_REQUIRE(emb && gz && sum_e && grad_rows && grad_lin, "ctr_fm_embedding_grad: null pointer");
  if (plan->S == 0) return CTR_OK;
  SegArgs a;
  int rc = seg_prepare(a, plan, K, grad_rows, grad_lin, rowmap, ws, ws_bytes);
  if (rc != CTR_OK) return rc;
  a.F = F;
  a.gz = gz;
  a.sum_e = sum_e;
  a.dx = dx;
  a.emb = emb;
  a.fm_defer = CTR_SEG_FM_DEFER;
  a.emb_by_seg = plan->sorted_rows == plan->pos_seg;
  const bool al = ((uintptr_t)emb | (uintptr_t)sum_e | (uintptr_t)dx | (uintptr_t)grad_rows |
                   (uintptr_t)ws) % 16 == 0;
  return launch_seg(a, K, MODE_FM, as_stream(stream), al);
}

static int seg_set_apply(SegArgs& a, int K, const ctr_deferred_table* t, const int32_t* step_ptr,
                         const float* step_table, double beta1, double beta2, double eps,
                         double weight_decay) {
  CTR_REQUIRE(t && t->emb && t->m_emb && t->v_emb && t->last && step_ptr && step_table,
              "segment sum + Adam: null table / step pointer");
  CTR_REQUIRE((t->lin && t->m_lin && t->v_lin) || (!t->lin && !t->m_lin && !t->v_lin),
              "segment sum + Adam: linear table pointers must be all set or all NULL");
  CTR_REQUIRE(K % 4 == 0 && K / 4 <= 64 &&
                  ((uintptr_t)t->emb | (uintptr_t)t->m_emb | (uintptr_t)t->v_emb) % 16 == 0,
              "segment sum + Adam: needs K %% 4 == 0, K <= 256 and 16-B aligned rows");
  a.apply = true;
  a.E = reinterpret_cast<float4*>(t->emb);
  a.mE = reinterpret_cast<float4*>(t->m_emb);
  a.vE = reinterpret_cast<float4*>(t->v_emb);
  a.w = t->lin;
  a.mw = t->m_lin;
  a.vw = t->v_lin;
  a.last = t->last;
  a.step_ptr = step_ptr;
  a.tab = step_table;
  a.hp = make_hp(1.0, 1.0, beta1, beta2, eps, weight_decay);
  return CTR_OK;
}

extern "C" int ctr_fm_embedding_grad_adam(const ctr_sparse_plan* plan, int F, int K,
                                          const float* gz, const float* sum_e, const float* dx,
                                          const ctr_deferred_table* table,
                                          const int32_t* step_ptr, const float* step_table,
                                          double beta1, double beta2, double eps,
                                          double weight_decay, float* grad_rows,
                                          float* grad_lin, int keep_sums, void* ws,
                                          int64_t ws_bytes, ctr_stream_t stream) {
  CTR_REQUIRE(plan_ok(plan), "ctr_fm_embedding_grad_adam: incomplete plan");
  CTR_REQUIRE(F > 0 && K > 0 && gz && sum_e, "ctr_fm_embedding_grad_adam: bad arguments");
  if (plan->S == 0) return CTR_OK;
  CTR_REQUIRE(grad_rows && grad_lin, "ctr_fm_embedding_grad_adam: grad_rows / grad_lin needed");
  SegArgs a;
  int rc = seg_prepare(a, plan, K, grad_rows, grad_lin, nullptr, ws, ws_bytes);
  if (rc != CTR_OK) return rc;
  rc = seg_set_apply(a, K, table, step_ptr, step_table, beta1, beta2, eps, weight_decay);
  if (rc != CTR_OK) return rc;
  a.out_keep = keep_sums != 0;
  a.F = F;
  a.gz = gz;
  a.sum_e = sum_e;
  a.dx = dx;
  a.emb = table->emb;
  a.fm_defer = CTR_SEG_FM_DEFER;
  a.emb_by_seg = plan->sorted_rows == plan->pos_seg;
  CTR_REQUIRE(((uintptr_t)sum_e | (uintptr_t)dx | (uintptr_t)grad_rows | (uintptr_t)ws) % 16 == 0,
              "ctr_fm_embedding_grad_adam: 16-B aligned buffers required");
  return launch_seg(a, K, MODE_FM, as_stream(stream), true);
}

extern "C" int ctr_segment_sum_rows_adam(const ctr_sparse_plan* plan, int K, const float* vals,
                                         const float* vals_lin, const ctr_deferred_table* table,
                                         const int32_t* step_ptr, const float* step_table,
                                         double beta1, double beta2, double eps,
                                         double weight_decay, float* out, float* out_lin,
                                         int keep_sums, void* ws, int64_t ws_bytes,
                                         ctr_stream_t stream) {
  CTR_REQUIRE(plan_ok(plan), "ctr_segment_sum_rows_adam: incomplete plan");
  CTR_REQUIRE(K > 0 && vals, "ctr_segment_sum_rows_adam: bad arguments");
  if (plan->S == 0) return CTR_OK;
  CTR_REQUIRE(out && !vals_lin == !out_lin, "ctr_segment_sum_rows_adam: out (and out_lin) needed");
  SegArgs a;
  int rc = seg_prepare(a, plan, K, out, out_lin, nullptr, ws, ws_bytes);
  if (rc != CTR_OK) return rc;
  rc = seg_set_apply(a, K, table, step_ptr, step_table, beta1, beta2, eps, weight_decay);
  if (rc != CTR_OK) return rc;
  a.out_keep = keep_sums != 0;
  a.vals = vals;
  a.vals_lin = vals_lin;
  CTR_REQUIRE(((uintptr_t)vals | (uintptr_t)out | (uintptr_t)ws) % 16 == 0,
              "ctr_segment_sum_rows_adam: 16-B aligned buffers required");
  return launch_seg(a, K, MODE_VALS, as_stream(stream), true);
}

extern "C" int ctr_segment_sum_rows(const ctr_sparse_plan* plan, int K, const float* vals,
                                    const float* vals_lin, float* out, float* out_lin,
                                    int32_t* rowmap, void* ws, int64_t ws_bytes,
                                    ctr_stream_t stream) {
  CTR_REQUIRE(plan_ok(plan), "ctr_segment_sum_rows: incomplete plan");
  CTR_REQUIRE(K > 0 && vals && out, "ctr_segment_sum_rows: bad arguments");
  CTR_REQUIRE(!vals_lin == !out_lin, "ctr_segment_sum_rows: vals_lin and out_lin go together");
  if (plan->S == 0) return CTR_OK;
  SegArgs a;
  int rc = seg_prepare(a, plan, K, out, out_lin, rowmap, ws, ws_bytes);
  if (rc != CTR_OK) return rc;
  a.vals = vals;
  a.vals_lin = vals_lin;
  const bool al = ((uintptr_t)vals | (uintptr_t)out | (uintptr_t)ws) % 16 == 0;
  return launch_seg(a, K, MODE_VALS, as_stream(stream), al);
}

extern "C" int ctr_shard_row_grads(const ctr_sparse_plan* plan, int F, int K, const float* emb,
                                   const float* gz, const float* sum_e, const float* dx,
                                   const float* vals, int lin, int n_runs,
                                   const int32_t* run_offsets, int64_t run_len, int64_t chunk,
                                   float* out_chunks, void* ws, int64_t ws_bytes,
                                   ctr_stream_t stream) {
  CTR_REQUIRE(plan_ok(plan), "ctr_shard_row_grads: incomplete plan");
  CTR_REQUIRE(K > 0 && K % 4 == 0 && out_chunks && run_offsets && n_runs > 0 && run_len > 0,
              "ctr_shard_row_grads: bad arguments");
  CTR_REQUIRE(chunk % 4 == 0 && chunk >= run_len * K + (lin ? run_len : 0),
              "ctr_shard_row_grads: chunk must hold run_len rows (+ their linear sums)");
  CTR_REQUIRE(gz ? (F > 0 && emb && sum_e) : (vals && !lin),
              "ctr_shard_row_grads: FM mode needs emb / gz / sum_e; vals mode has no linear sums");
  if (plan->S == 0) return CTR_OK;
  SegArgs a;
  int rc = seg_prepare(a, plan, K, out_chunks, nullptr, nullptr, ws, ws_bytes);
  if (rc != CTR_OK) return rc;
  a.map_n = n_runs;
  a.map_lin = lin != 0;
  a.map_off = run_offsets;
  a.map_C = run_len;
  a.map_chunk = chunk;
  const bool al = ((uintptr_t)emb | (uintptr_t)sum_e | (uintptr_t)dx | (uintptr_t)vals |
                   (uintptr_t)out_chunks | (uintptr_t)ws) % 16 == 0;
  CTR_REQUIRE(al, "ctr_shard_row_grads: 16-B aligned buffers required");
  if (gz) {
    a.F = F;
    a.gz = gz;
    a.sum_e = sum_e;
    a.dx = dx;
    a.emb = emb;
    a.fm_defer = CTR_SEG_FM_DEFER;
    a.emb_by_seg = plan->sorted_rows == plan->pos_seg;
    return launch_seg(a, K, MODE_FM, as_stream(stream), true);
  }
  a.vals = vals;
  return launch_seg(a, K, MODE_VALS, as_stream(stream), true);
}

extern "C" int ctr_rows_to_dense(const ctr_sparse_plan* plan, int K, const float* grad_rows,
                                 const float* grad_lin, float* dense, float* dense_lin,
                                 ctr_stream_t stream) {
  CTR_REQUIRE(plan_ok(plan) && K > 0 && grad_rows && dense, "ctr_rows_to_dense: bad arguments");
  if (plan->S == 0) return CTR_OK;
  const unsigned grid = (unsigned)std::min<int64_t>(ceil_div(plan->S * (int64_t)K, 256), 4096);
  hipLaunchKernelGGL(rows_to_dense_kernel, grid, 256, 0, as_stream(stream), plan->unique_rows,
                     plan->num_unique, K, grad_rows, grad_lin, dense, dense_lin);
  CTR_LAUNCH_CHECK("ctr_rows_to_dense");
  return CTR_OK;
}

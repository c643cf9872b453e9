// Shared pieces of the two MLP GEMM kernels (csrc/gemm.hip: exact-f32 MFMA;
// csrc/gemm_sb16.hip: split-bf16 MFMA): arguments, fused epilogues, the accumulator
// write-out, and the split-bf16 tile chooser/launcher used by ctr_gemm_f32_ex.
#pragma once

#include "ctr_common.h"

namespace ctr {

typedef float floatx16 __attribute__((ext_vector_type(16)));

struct GemmArgs {
  int64_t M, N, K;
  const float* A;
  int64_t lda;
  const float* B;
  int64_t ldb;
  float* C;
  int64_t ldc;
  int epi;
  const float* bias;
  const float* aux;
  int64_t ldaux;
  float scale;        // GRAD_MASK multiplier
  uint32_t drop_thr;  // keep iff hash >= drop_thr
  float drop_scale;   // 1/(1-p)
  uint64_t seed, offset;
  const int32_t* step_ptr;  // dropout stream of step *step_ptr: offset += step << 32
  int64_t k_per_split;
  int64_t slab_stride;  // elements between split-K slabs (0: no split)
  bool vec_a, vec_b;
  bool vec_c;  // C rows 16-B aligned (float4 epilogue stores)
};

__device__ __forceinline__ float apply_epi(const GemmArgs& a, int epi, float acc, int64_t m,
                                           int64_t n) {
  switch (epi) {
    case CTR_EPI_BIAS:
      return acc + a.bias[n];
    case CTR_EPI_BIAS_RELU: {
      const float v = acc + a.bias[n];
      return v > 0.f ? v : 0.f;
    }
    case CTR_EPI_BIAS_RELU_DROP: {
      float v = acc + a.bias[n];
      v = v > 0.f ? v : 0.f;
      const uint32_t hsh = hash_u32(a.seed, a.offset + (uint64_t)(m * a.N + n));
      return hsh >= a.drop_thr ? v * a.drop_scale : 0.f;
    }
    case CTR_EPI_GRAD_MASK:
      return a.aux[m * a.ldaux + n] > 0.f ? acc * a.scale : 0.f;
    default:
      return acc;
  }
}

// Write a wave's TM x TN 32x32 accumulators (C/D map of every 32x32 MFMA on gfx950:
// col = lane & 31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)) through a wave-private 32x36
// LDS tile `et`, then in row order through the epilogue: each store instruction covers
// 8 rows x 128 B (float4 per lane). Split-K blocks (slab_stride != 0) write their raw
// partial sums into slab blockIdx.z. Keeps the accumulator indexing static (a per-element
// epilogue over all TM*TN*16 values put the accumulators in scratch).
template <int TM, int TN>
__device__ __forceinline__ void gemm_store_tiles(GemmArgs a, floatx16 (&acc)[TM][TN], float* et,
                                                 int64_t mb, int64_t nb, int lane) {
  float* C = a.C + (int64_t)blockIdx.z * a.slab_stride;
  const int epi = a.slab_stride ? (int)CTR_EPI_NONE : a.epi;
  if (epi == CTR_EPI_BIAS_RELU_DROP && a.step_ptr) a.offset += (uint64_t)(*a.step_ptr) << 32;
  const int h = lane >> 5, il = lane & 31;
  const int er = lane >> 3, ec = 4 * (lane & 7);
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) {
#pragma unroll
      for (int r = 0; r < 16; ++r) et[((r & 3) + 8 * (r >> 2) + 4 * h) * 36 + il] = acc[i][tn][r];
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): wave-private tile, no barrier
      __builtin_amdgcn_wave_barrier();
      const int64_t n = nb + tn * 32 + ec;
      for (int j = 0; j < 4; ++j) {
        const int row = er + 8 * j;
        const int64_t m = mb + i * 32 + row;
        if (m >= a.M) continue;
        const float4 v = *reinterpret_cast<const float4*>(et + row * 36 + ec);
        float* crow = C + m * a.ldc;
        if (a.vec_c && n + 3 < a.N) {
          float4 o;
          o.x = apply_epi(a, epi, v.x, m, n + 0);
          o.y = apply_epi(a, epi, v.y, m, n + 1);
          o.z = apply_epi(a, epi, v.z, m, n + 2);
          o.w = apply_epi(a, epi, v.w, m, n + 3);
          *reinterpret_cast<float4*>(crow + n) = o;
        } else {
          if (n + 0 < a.N) crow[n + 0] = apply_epi(a, epi, v.x, m, n + 0);
          if (n + 1 < a.N) crow[n + 1] = apply_epi(a, epi, v.y, m, n + 1);
          if (n + 2 < a.N) crow[n + 2] = apply_epi(a, epi, v.z, m, n + 2);
          if (n + 3 < a.N) crow[n + 3] = apply_epi(a, epi, v.w, m, n + 3);
        }
      }
      __builtin_amdgcn_wave_barrier();
    }
}

// Block -> output tile: tiles sharing A rows are consecutive, and consecutive tiles are
// kept on one XCD (blocks b, b+8, b+16... share an XCD under round-robin dispatch).
__device__ __forceinline__ int64_t xcd_tile_index() {
  const int64_t T = gridDim.x;
  int64_t tix = blockIdx.x;
  if (T % 8 == 0) tix = (tix % 8) * (T / 8) + tix / 8;
  return tix;
}

// ---------------------------------------------------- split-bf16 host interface -----
struct Sb16Cfg {
  int tile;     // index into the split-bf16 tilings (csrc/gemm_sb16.hip)
  int splits;   // split-K over blockIdx.z (fp32 slabs + splitk_reduce_kernel)
  int64_t kps;  // k per split
  int bm, bn;   // the tiling's block tile
};
Sb16Cfg sb16_choose(int64_t M, int64_t N, int64_t K);
int sb16_num_tiles();
void sb16_tile_dims(int tile, int& bm, int& bn);
void sb16_launch(const Sb16Cfg& c, const GemmArgs& a, bool ta, bool tb, dim3 grid, hipStream_t st);

}  // namespace ctr

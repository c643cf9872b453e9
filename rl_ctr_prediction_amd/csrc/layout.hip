// Layout change for the weight-gradient GEMM of DeepFM / IPNN's first Linear (SURVEY.md
// §8a A2): dW0 = dH1^T X sums over the batch, which is the row index of both operands as
// they are produced ([B, 300] and [B, F*K], k = batch strided). The split-bf16 GEMM stages
// k-contiguous operands as float4 runs and rows-contiguous ones as 4x4 register transposes
// (four loads and four splits per unit): with dH1^T and X^T written once per step, the
// same product runs k-contiguous on both sides (98 -> 68 us at the C3 shape,
// profiles/r01_gemm_tuning_sb16.txt). The transposes run on the weight-gradient stream
// beside the dH1 / dX GEMMs (HBM-bound work beside MFMA-bound work).
//
// ctr_transpose_f32: dst[c * ld_dst + r] = src[r * ld_src + c] for r < rows, c < cols.
// 64 x 64 tiles through LDS (row stride 65: the column reads of the write phase are
// conflict-free); reads coalesced along c, writes along r. Pure copies: bit-exact.
#include "ctr_common.h"

namespace ctr {

// ctr_batch_stage_copy: a batch's ids and labels into its input slot in ONE launch (the
// runtime's D2D copies are one copy kernel each, ~2.5-5 us apiece on the plan stream at
// C2 / C3). Both segments walk one grid-stride index space of 16-B units (or bytes where a
// segment is not 16-B aligned and sized): pure copies, bit-exact.
__global__ __launch_bounds__(256) void batch_stage_copy_kernel(char* __restrict__ d0,
                                                               const char* __restrict__ s0,
                                                               int64_t u0, bool v0,
                                                               char* __restrict__ d1,
                                                               const char* __restrict__ s1,
                                                               int64_t u1, bool v1) {
  const int64_t total = u0 + u1;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const bool first = t < u0;
    const int64_t i = first ? t : t - u0;
    char* d = first ? d0 : d1;
    const char* s = first ? s0 : s1;
    if (first ? v0 : v1)
      reinterpret_cast<uint4*>(d)[i] = reinterpret_cast<const uint4*>(s)[i];
    else
      d[i] = s[i];
  }
}

constexpr int kTT = 64;

__global__ __launch_bounds__(256) void transpose_f32_kernel(const float* __restrict__ src,
                                                            int64_t rows, int64_t cols,
                                                            int64_t ld_src, float* __restrict__ dst,
                                                            int64_t ld_dst, int64_t row_tiles) {
  __shared__ float tile[kTT][kTT + 1];
  const int tx = threadIdx.x & (kTT - 1), ty = threadIdx.x >> 6;  // 64 x 4 threads
  const int64_t c0 = (int64_t)blockIdx.x * kTT;
  for (int64_t rt = blockIdx.y; rt < row_tiles; rt += gridDim.y) {
    const int64_t r0 = rt * kTT;
    const int64_t c = c0 + tx;
#pragma unroll
    for (int i = 0; i < kTT / 4; ++i) {
      const int64_t r = r0 + ty + 4 * i;
      if (r < rows && c < cols) tile[ty + 4 * i][tx] = src[r * ld_src + c];
    }
    __syncthreads();
    const int64_t r = r0 + tx;
#pragma unroll
    for (int i = 0; i < kTT / 4; ++i) {
      const int64_t cc = c0 + ty + 4 * i;
      if (r < rows && cc < cols) dst[cc * ld_dst + r] = tile[tx][ty + 4 * i];
    }
    __syncthreads();  // the tile is reused by the next row tile
  }
}

// float4 form (rows, cols, both lds multiples of 4, 16-B aligned bases): a thread reads 4
// consecutive c of one row and writes 4 consecutive r of one output row; 16 threads cover a
// 64-float run on both sides.
__global__ __launch_bounds__(256) void transpose_f32x4_kernel(const float* __restrict__ src,
                                                              int64_t rows, int64_t cols,
                                                              int64_t ld_src,
                                                              float* __restrict__ dst,
                                                              int64_t ld_dst, int64_t row_tiles) {
  __shared__ float tile[kTT][kTT + 1];
  const int q = threadIdx.x & 15, p = threadIdx.x >> 4;  // 16 quads x 16 lines
  const int64_t c0 = (int64_t)blockIdx.x * kTT;
  for (int64_t rt = blockIdx.y; rt < row_tiles; rt += gridDim.y) {
    const int64_t r0 = rt * kTT;
    const int64_t c = c0 + 4 * q;
#pragma unroll
    for (int i = 0; i < kTT / 16; ++i) {
      const int rr = p + 16 * i;
      const int64_t r = r0 + rr;
      if (r < rows && c < cols) {
        const float4 v = *reinterpret_cast<const float4*>(src + r * ld_src + c);
        tile[rr][4 * q + 0] = v.x;
        tile[rr][4 * q + 1] = v.y;
        tile[rr][4 * q + 2] = v.z;
        tile[rr][4 * q + 3] = v.w;
      }
    }
    __syncthreads();
    const int64_t r = r0 + 4 * q;
#pragma unroll
    for (int i = 0; i < kTT / 16; ++i) {
      const int cc = p + 16 * i;
      if (r < rows && c0 + cc < cols) {
        const float4 v = make_float4(tile[4 * q + 0][cc], tile[4 * q + 1][cc],
                                     tile[4 * q + 2][cc], tile[4 * q + 3][cc]);
        *reinterpret_cast<float4*>(dst + (c0 + cc) * ld_dst + r) = v;
      }
    }
    __syncthreads();
  }
}

}  // namespace ctr

using namespace ctr;

extern "C" int ctr_transpose_f32(const float* src, int64_t rows, int64_t cols, int64_t ld_src,
                                 float* dst, int64_t ld_dst, ctr_stream_t stream) {
  CTR_REQUIRE(rows >= 0 && cols >= 0, "ctr_transpose_f32: bad sizes");
  if (rows == 0 || cols == 0) return CTR_OK;
  CTR_REQUIRE(src && dst, "ctr_transpose_f32: null pointer");
  CTR_REQUIRE(ld_src >= cols && ld_dst >= rows, "ctr_transpose_f32: need ld_src >= cols and "
              "ld_dst >= rows");
  const int64_t col_tiles = ceil_div(cols, kTT), row_tiles = ceil_div(rows, kTT);
  // gridDim.x * blockDim.x must fit 32 bits
  CTR_REQUIRE(col_tiles <= (int64_t)(UINT32_MAX / 256), "ctr_transpose_f32: too many columns");
  const dim3 grid((unsigned)col_tiles, (unsigned)std::min<int64_t>(row_tiles, 65535));
  const bool vec = rows % 4 == 0 && cols % 4 == 0 && ld_src % 4 == 0 && ld_dst % 4 == 0 &&
                  reinterpret_cast<uintptr_t>(src) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(dst) % 16 == 0;
  if (vec)
    hipLaunchKernelGGL(transpose_f32x4_kernel, grid, 256, 0, as_stream(stream), src, rows, cols,
                       ld_src, dst, ld_dst, row_tiles);
  else
    hipLaunchKernelGGL(transpose_f32_kernel, grid, 256, 0, as_stream(stream), src, rows, cols,
                       ld_src, dst, ld_dst, row_tiles);
  CTR_LAUNCH_CHECK("ctr_transpose_f32");
  return CTR_OK;
}

extern "C" int ctr_batch_stage_copy(void* dst0, const void* src0, int64_t n0, void* dst1,
                                    const void* src1, int64_t n1, ctr_stream_t stream) {
  CTR_REQUIRE(n0 >= 0 && n1 >= 0 && (n0 == 0 || (dst0 && src0)) && (n1 == 0 || (dst1 && src1)),
              "ctr_batch_stage_copy: bad arguments");
  if (n0 + n1 == 0) return CTR_OK;
  auto vec = [](const void* d, const void* s, int64_t n) {
    return n % 16 == 0 && ((uintptr_t)d | (uintptr_t)s) % 16 == 0;
  };
  const bool v0 = vec(dst0, src0, n0), v1 = vec(dst1, src1, n1);
  const int64_t u0 = v0 ? n0 / 16 : n0, u1 = v1 ? n1 / 16 : n1;
  const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>(ceil_div(u0 + u1, 256), 4096));
  hipLaunchKernelGGL(batch_stage_copy_kernel, grid, 256, 0, as_stream(stream),
                     static_cast<char*>(dst0), static_cast<const char*>(src0), u0, v0,
                     static_cast<char*>(dst1), static_cast<const char*>(src1), u1, v1);
  CTR_LAUNCH_CHECK("batch_stage_copy_kernel");
  return CTR_OK;
}

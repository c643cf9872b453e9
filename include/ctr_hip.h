/*
 * ctr_hip.h — C ABI of libctr_hip.so, the MI355X (gfx950) hot path of
 * jqsl2012/RL_CTR_Prediction's CTR training step.
 *
 * Scope: the multi-field sparse->embedding gather, the FM
 * interaction (sum-square trick) and linear term, the DeepFM MLP head, the log-loss
 * (BCE after sigmoid) backward, the embedding scatter-add, the coupled-L2 Adam step,
 * Feature_Embedding's pairwise inner products and the REINFORCE loss of PG_model.
 *
 * Conventions (every entry point):
 *   - plain device pointers and sizes, row-major, fp32 unless stated; index arrays are
 *     int32 (CTR_IDX_I32) or int64 (CTR_IDX_I64, what the reference's LongTensor holds);
 *   - all work is enqueued on `stream` (a hipStream_t; NULL = legacy default stream);
 *     nothing synchronises, nothing allocates; scratch is caller-owned and sized by the
 *     matching *_workspace_bytes() query;
 *   - return CTR_OK (0) or a CTR_ERR_* code; ctr_last_error() then holds a thread-local
 *     message. Out-of-range feature ids never fault: the kernel reads row 0 instead and
 *     ORs CTR_EFLAG_INDEX into *err_flag (optional device int32), the analogue of
 *     nn.Embedding's "index out of range" error, checked by the host when it chooses.
 */
#ifndef CTR_HIP_H
#define CTR_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* ctr_stream_t; /* hipStream_t */

enum ctr_status {
  CTR_OK = 0,
  CTR_ERR_INVALID = 1,     /* argument out of contract */
  CTR_ERR_HIP = 2,         /* HIP runtime / launch error */
  CTR_ERR_WORKSPACE = 3,   /* scratch smaller than the *_workspace_bytes() answer */
  CTR_ERR_UNSUPPORTED = 4  /* shape this build does not handle */
};

enum ctr_idx_type { CTR_IDX_I32 = 0, CTR_IDX_I64 = 1 };

enum ctr_err_flag {
  CTR_EFLAG_INDEX = 1,    /* a feature id outside [0, V) */
  CTR_EFLAG_CAPACITY = 2  /* a row-sharded exchange run longer than its capacity */
};

/* GEMM epilogues (ctr_gemm_f32). */
enum ctr_epilogue {
  CTR_EPI_NONE = 0,            /* C = A.B                                                  */
  CTR_EPI_BIAS = 1,            /* C = A.B + bias[n]                                        */
  CTR_EPI_BIAS_RELU = 2,       /* C = relu(A.B + bias[n])                                  */
  CTR_EPI_BIAS_RELU_DROP = 3,  /* C = dropout(relu(A.B + bias[n]); p, seed, offset)        */
  CTR_EPI_GRAD_MASK = 4        /* C = aux[m,n] > 0 ? (A.B) * scale : 0  (relu+dropout bwd) */
};

int ctr_abi_version(void);
const char* ctr_last_error(void);
/* Number of visible HIP devices (0 on a host without a GPU); never initialises a context
 * beyond hipGetDeviceCount. */
int ctr_device_count(void);
/* A stream whose kernels run only on the CUs set in mask[0 .. n_words) (bit c % 32 of word
 * c / 32 = CU c in the driver's numbering; hipExtStreamCreateWithCUMask), and its release.
 * The mask holds for launches on that stream, eager or as the root of a graph launched on
 * it, not for a graph branch forked onto it (tools/cumask_probe.hip). Used by the
 * weight-gradient side stream experiment (CTR_WGRAD_CU_FRAC); no reference
 * counterpart. */
int ctr_stream_create_cu_masked(const uint32_t* mask, int n_words, ctr_stream_t* out);
int ctr_stream_destroy(ctr_stream_t stream);

/* ---------------------------------------------------------------- A3: gather ---------
 * out[i, :] = table[idx[i], :]  — nn.Embedding.forward.
 * Replaces: p_model.py:47,303,320 and Feature_embedding.py:52 (self.feature_embedding(x)). */
int ctr_embedding_gather(const float* table, int64_t V, int K, const void* idx, int idx_type,
                         int64_t n, float* out, int32_t* err_flag, ctr_stream_t stream);

/* ------------------------------------------------------ A1/A2/A4: FM forward ---------
 * Fused gather + FM second order + linear term for B examples of F fields:
 *   z[b]      = bias[0] + sum_f lin[x_bf] + 0.5 * sum_k ((sum_f E[x_bf,k])^2 - sum_f E[x_bf,k]^2)
 *   sum_e     [B,K]   sum_f E[x_bf,:]      (optional; the backward needs it)
 *   emb_out   [B,F*K] E[x_bf,:] flattened  (optional; DeepFM's MLP input)
 * If labels != NULL the BCE-after-sigmoid head is fused (FM model):
 *   p[b] = sigmoid(z[b]); loss_elem[b] = BCE(p, y) (log clamped at -100);
 *   gz[b] = d(mean BCE)/dz with the reference's UNFUSED formula in ATen's operation order,
 *           mean_div = the batch the mean runs over (B, or B_global under data parallel):
 *           g_p = ((p-y)/max((1-p)p, 1e-12))/mean_div; gz = (g_p*(1-p))*p.
 *   p, loss_elem, gz may then be non-NULL individually.
 * Replaces: p_model.py:40-57 (FM.forward), 296-313 (DeepFM.to_fm), nn.BCELoss at
 * all_main/pretrain_main.py:74,139. */
int ctr_fm_forward(const void* idx, int idx_type, int64_t B, int F, int K, int64_t V,
                   const float* emb, const float* lin, const float* bias,
                   float* z, float* sum_e, float* emb_out,
                   const float* labels, float mean_div,
                   float* p, float* loss_elem, float* gz,
                   int32_t* err_flag, ctr_stream_t stream);

/* BCE after sigmoid on precomputed logits (same formulas as the fused FM head).
 * Replaces: torch.sigmoid (p_model.py:55,324) + nn.BCELoss (pretrain_main.py:74). */
int ctr_bce_sigmoid(const float* z, const float* labels, int64_t B, float mean_div,
                    float* p, float* loss_elem, float* gz, ctr_stream_t stream);

/* DeepFM output head: z[b] = z_fm[b] + h[b,:].w_out + b_out[0]; then the BCE head as above.
 * dh_pre[b,j] = h[b,j] > 0 ? gz[b]*w_out[j]*drop_scale : 0  (grad through the last
 * Linear, the Dropout and the ReLU that produced h; drop_scale = 1/(1-p) or 1 in eval).
 * Replaces: p_model.py:322-324 (mlp[6] Linear(200,1) + sum + sigmoid), pretrain_main.py:74. */
int ctr_deepfm_head(const float* h, int64_t B, int H, const float* w_out, const float* b_out,
                    const float* z_fm, const float* labels, float mean_div, float drop_scale,
                    float* z, float* p, float* loss_elem, float* gz, float* dh_pre,
                    ctr_stream_t stream);

/* -------------------------------------------------------- MLP: fp32 MFMA GEMM ---------
 * C[M,N] = op(A)[M,K] . op(B)[K,N] with epilogue `epi` (enum ctr_epilogue).
 * trans_a = 0: A stored [M,K] (lda >= K); 1: A stored [K,M] (lda >= M).
 * trans_b = 0: B stored [K,N] (ldb >= N); 1: B stored [N,K] (ldb >= K)  (nn.Linear weight).
 * Dropout keeps element (m,n) iff hash(seed, offset + m*N + n) >= p*2^32 and scales by
 * 1/(1-p), where offset += (*step_ptr) << 32 when step_ptr != NULL (a per-step mask read
 * on the device, for HIP-graph replay). `scale` is used by CTR_EPI_GRAD_MASK. Split-K
 * (long K, few tiles) uses `ws`.
 * Replaces: nn.Linear / ReLU / Dropout of DeepFM.mlp (p_model.py:276-293) and of
 * PG_model.Net.mlp (PG_model.py:41-51), forward and autograd backward (dX and dW). */
int64_t ctr_gemm_f32_workspace_bytes(int trans_a, int trans_b, int64_t M, int64_t N, int64_t K);
/* ctr_gemm_f32 = ctr_gemm_f32_ex(CTR_GEMM_AUTO, ...). */
int ctr_gemm_f32(int trans_a, int trans_b, int64_t M, int64_t N, int64_t K,
                 const float* A, int64_t lda, const float* B, int64_t ldb,
                 float* C, int64_t ldc, int epi, const float* bias,
                 const float* aux, int64_t ldaux, float scale,
                 float drop_p, uint64_t seed, uint64_t offset, const int32_t* step_ptr,
                 void* ws, int64_t ws_bytes, ctr_stream_t stream);

/* GEMM algorithms (same contract, same fp32 operands and outputs):
 *  CTR_GEMM_EXACT_F32  v_mfma_f32_32x32x2_f32: exact fp32 products, fp32 accumulation.
 *  CTR_GEMM_SPLIT_BF16 each fp32 operand split exactly into three bf16 planes
 *                      (x = x0 + x1 + x2, RNE); the six partial products with
 *                      i + j <= 2 on v_mfma_f32_32x32x16_bf16, fp32 accumulation. The
 *                      dropped terms are <= 2^-23 |a*b| per product (one fp32 multiply's
 *                      rounding); 2.7x the fp32 matrix rate.
 *  CTR_GEMM_AUTO       SPLIT_BF16 unless the environment sets CTR_GEMM_ALGO=exact. */
enum ctr_gemm_algo { CTR_GEMM_AUTO = 0, CTR_GEMM_EXACT_F32 = 1, CTR_GEMM_SPLIT_BF16 = 2 };
int64_t ctr_gemm_f32_ex_workspace_bytes(int algo, int trans_a, int trans_b, int64_t M, int64_t N,
                                        int64_t K);
int ctr_gemm_f32_ex(int algo, int trans_a, int trans_b, int64_t M, int64_t N, int64_t K,
                    const float* A, int64_t lda, const float* B, int64_t ldb,
                    float* C, int64_t ldc, int epi, const float* bias,
                    const float* aux, int64_t ldaux, float scale,
                    float drop_p, uint64_t seed, uint64_t offset, const int32_t* step_ptr,
                    void* ws, int64_t ws_bytes, ctr_stream_t stream);
/* The algorithm CTR_GEMM_AUTO (or any value) resolves to in this process. */
int ctr_gemm_resolved_algo(int algo);

/* ------------------------------------------- A2: MLP GEMM on pre-split planes -------
 * The fused trainer's MLP GEMMs (the six products of DeepFM's / InnerPNN's MLP per step,
 * p_model.py:276-293,322 forward and backward). An fp32 matrix travels as its exact
 * three-plane bf16 split x = x0 + x1 + x2 (CTR_GEMM_SPLIT_BF16's numerics), written once
 * by its producer, so the GEMM stages operands by LDS-DMA without any split work.
 *
 * ctr_planes: bf16 bits [3][rows][cols] with row stride `ld` and plane stride
 * `plane_stride` (elements); `rows`/`cols` = the allocated storage extents. CONTRACT: the
 * storage beyond the matrix's logical extent is ZERO and stays zero (the GEMM reads whole
 * 32-deep k tiles), ld % 8 == 0, data 16-B aligned.
 *
 * ctr_split_planes: planes of src [rows, cols] (row stride ld); writes the valid region.
 *
 * ctr_gemm_planes: C[M,N] = A.B with the ctr_gemm_f32 epilogues. Orientation per operand:
 *   a_rc = 0: A stored [M][K] (k contiguous)     a_rc = 1: A stored [K][M] (A^T product)
 *   b_rc = 0: B stored [N][K] (nn.Linear weight) b_rc = 1: B stored [K][N]
 * Storage must cover align_up(K, 32) along k, zero-padded. Outputs: C (fp32, ldc) and/or Cp
 * (the planes of the epilogue's result, for the next GEMM). Split-K scratch is sized by
 * ctr_gemm_planes_workspace_bytes. ctr_gemm_planes_config reports the tiling chosen
 * (tuning and tests). */
typedef struct ctr_planes {
  void* data;
  int64_t ld;
  int64_t plane_stride;
  int64_t rows;
  int64_t cols;
} ctr_planes;
int ctr_split_planes(const float* src, int64_t rows, int64_t cols, int64_t ld,
                     const ctr_planes* dst, ctr_stream_t stream);
int64_t ctr_gemm_planes_workspace_bytes(int a_rc, int b_rc, int64_t M, int64_t N, int64_t K);
int ctr_gemm_planes(int a_rc, int b_rc, int64_t M, int64_t N, int64_t K,
                    const ctr_planes* A, const ctr_planes* B, float* C, int64_t ldc,
                    const ctr_planes* Cp, int epi, const float* bias, const float* aux,
                    int64_t ldaux, float scale, float drop_p, uint64_t seed, uint64_t offset,
                    const int32_t* step_ptr, void* ws, int64_t ws_bytes, ctr_stream_t stream);
int ctr_gemm_planes_config(int a_rc, int b_rc, int64_t M, int64_t N, int64_t K, int* tile,
                           int* splits, int* bm, int* bn);
/* ctr_gemm_planes_lastcol: ctr_gemm_planes whose result column N-1 is written to
 * last_col[m] (m < M) instead of C, which then holds N-1 columns (ldc >= N-1). With a B
 * operand whose column N-1 is all ones (a ones column in the planes' zero padding), a weight
 * gradient dW = G^T X and its bias gradient db = colsum(G) come out of ONE GEMM.
 * Replaces: the mlp.0 / mlp.3 weight AND bias gradients of p_model.py:276-293 backward. */
int ctr_gemm_planes_lastcol(int a_rc, int b_rc, int64_t M, int64_t N, int64_t K,
                            const ctr_planes* A, const ctr_planes* B, float* C, int64_t ldc,
                            const ctr_planes* Cp, int epi, const float* bias, const float* aux,
                            int64_t ldaux, float scale, float drop_p, uint64_t seed,
                            uint64_t offset, const int32_t* step_ptr, float* last_col, void* ws,
                            int64_t ws_bytes, ctr_stream_t stream);

/* The producers of the MLP's GEMM operands writing planes directly (no fp32 round trip):
 * ctr_fm_forward_planes: ctr_fm_forward (no BCE head; DeepFM's FM part) whose flattened
 *   embeddings (emb_out [B, F*K]) are written as planes; needs K % 4 == 0, (K/4) | 64,
 *   F <= 64. Replaces: p_model.py:303,320 (the two gathers of DeepFM.forward).
 * ctr_deepfm_head_planes: ctr_deepfm_head with labels, writing dh_pre [B, H] in fp32 (dh_pre
 *   may be NULL: the planes only) and as planes (the dH1 / dW1 GEMM operand). Replaces:
 *   p_model.py:290-293,322 backward. */
int ctr_fm_forward_planes(const void* idx, int idx_type, int64_t B, int F, int K, int64_t V,
                          const float* emb, const float* lin, const float* bias, float* z,
                          float* sum_e, const ctr_planes* emb_planes, int32_t* err_flag,
                          ctr_stream_t stream);
int ctr_deepfm_head_planes(const float* h, int64_t B, int H, const float* w_out,
                           const float* b_out, const float* z_fm, const float* labels,
                           float mean_div, float drop_scale, float* z, float* p, float* loss_elem,
                           float* gz, float* dh_pre, const ctr_planes* dh_planes,
                           ctr_stream_t stream);

/* Deterministic reductions (fixed order; identical bits run to run).
 * ctr_sum_f32:    out[0] = scale * sum_i x[i]
 * ctr_colsum_f32: out[n] = scale * sum_m (row_w ? row_w[m] : 1) * X[m,n]   (bias / dW of
 *                 a 1-row Linear). */
int64_t ctr_reduce_workspace_bytes(int64_t M, int64_t N);
int ctr_sum_f32(const float* x, int64_t n, float scale, float* out, void* ws, int64_t ws_bytes,
                ctr_stream_t stream);
int ctr_colsum_f32(const float* X, int64_t M, int64_t N, int64_t ldx, const float* row_w,
                   float scale, float* out, void* ws, int64_t ws_bytes, ctr_stream_t stream);
/* Up to 8 ctr_colsum_f32 jobs in one launch pair, each output bitwise ctr_colsum_f32's
 * (same row partition and order): the DeepFM step's bias gradients (colsum dH1, dH2), the
 * last layer's weight gradient (gz-weighted colsum of H2) and its bias (colsum of gz). */
typedef struct ctr_colsum_job {
  const float* X;
  int64_t M, N, ldx;
  const float* row_w;
  float scale;
  float* out;
} ctr_colsum_job;
int64_t ctr_colsum_multi_workspace_bytes(int n_jobs, const ctr_colsum_job* jobs);
int ctr_colsum_multi_f32(int n_jobs, const ctr_colsum_job* jobs, void* ws, int64_t ws_bytes,
                         ctr_stream_t stream);

/* dst[c * ld_dst + r] = src[r * ld_src + c] (r < rows, c < cols), bit-exact copy: dH1^T and
 * X^T for the k-contiguous dW0 = dH1^T X GEMM of DeepFM / IPNN (p_model.py:279-293, the
 * weight gradient autograd forms for mlp.0). */
int ctr_transpose_f32(const float* src, int64_t rows, int64_t cols, int64_t ld_src, float* dst,
                      int64_t ld_dst, ctr_stream_t stream);

/* ------------------------------------------------ A3: embedding scatter-add -----------
 * A sparse plan groups the S = B*F slots (slot s = b*F + f) of a batch by feature id.
 * All arrays are caller-owned device buffers of S int32 (seg_offsets: S+1, num_unique: 1):
 *   sorted_slots  slot ids ordered by (row, slot) — a STABLE sort, so each row's slots keep
 *                 the order embedding_dense_backward accumulates them in;
 *   sorted_rows   the row of each sorted position;
 *   pos_seg       the segment (unique-row ordinal) of each sorted position;
 *   unique_rows   the distinct rows ascending, first *num_unique valid;
 *   seg_offsets   row u owns sorted positions [seg_offsets[u], seg_offsets[u+1]).
 * Index work: bit-exact (tests compare with numpy.unique). Replaces the grouping inside
 * embedding_dense_backward (autograd through p_model.py:47,54,303,311,320). */
typedef struct ctr_sparse_plan {
  int64_t S;
  int32_t* sorted_slots;
  int32_t* sorted_rows;
  int32_t* pos_seg;
  int32_t* unique_rows;
  int32_t* seg_offsets;
  int32_t* num_unique;
} ctr_sparse_plan;

int64_t ctr_sparse_plan_workspace_bytes(int64_t S, int64_t V);
/* Row sharding: rank j owns ids [j*shard_rows, (j+1)*shard_rows).
 * ctr_plan_slot_to_unique: slot_to_unique[s] = the unique-row ordinal of slot s (int32[S]);
 *   a forward over the rows received from their owners (compacted in unique order) reads
 *   them with these ids.
 * ctr_plan_shard_counts: counts[j] (int64[n_shards]) = how many of the plan's unique rows
 *   shard j owns; the unique rows are ascending, so they leave grouped by owner. */
int ctr_plan_slot_to_unique(const ctr_sparse_plan* plan, int32_t* slot_to_unique,
                            ctr_stream_t stream);
int ctr_plan_shard_counts(const ctr_sparse_plan* plan, int64_t shard_rows, int n_shards,
                          int64_t* counts, ctr_stream_t stream);
/* ctr_plan_shard_counts_max: the same counts and, in max_out[0] (int64, may be NULL), their
 * maximum — the step's largest per-owner run, which sizes the row-sharded exchange (one
 * launch; max_out needs n_shards <= 15). */
int ctr_plan_shard_counts_max(const ctr_sparse_plan* plan, int64_t shard_rows, int n_shards,
                              int64_t* counts, int64_t* max_out, ctr_stream_t stream);
/* ctr_sparse_plan_build_runs: the plan (bit-identical to ctr_sparse_plan_build's) of the ids an
 * owner shard receives in a row-sharded step: n_runs <= 8 runs of run_len int32 ids
 * (ids[j*run_len + i]), each run ascending with every row at most once, padded at its end with
 * the spare row n_rows - 1 (repeated); rows in [0, n_rows). mask: uint32[ceil(n_rows/4)], zero
 * on entry and left zero (a per-row bitmask of the requesting runs); ws: caller scratch of
 * ctr_sparse_plan_runs_workspace_bytes bytes. plan->S must be n_runs * run_len. */
int64_t ctr_sparse_plan_runs_workspace_bytes(int n_runs, int64_t run_len, int64_t n_rows);
int ctr_sparse_plan_build_runs(const int32_t* ids, int n_runs, int64_t run_len, int64_t n_rows,
                               const ctr_sparse_plan* plan, uint32_t* mask, void* ws,
                               int64_t ws_bytes, ctr_stream_t stream);
/* ids[i] += delta (global row ids <-> shard-local row ids). */
int ctr_ids_add(int32_t* ids, int64_t n, int32_t delta, ctr_stream_t stream);
/* Fixed-capacity exchange of a row-sharded step (no reference counterpart: the reference
 * runs on one device, all_main/pretrain_main.py:232; this is the exchange SURVEY.md §8e
 * adds around nn.Embedding's gather / embedding_dense_backward, p_model.py:47,303,311,320).
 * Every (requester, owner j) pair moves `capacity` rows, so the all-to-alls are equal-split
 * and their sizes depend on the capacity alone (a step is capturable in a HIP graph).
 * ctr_shard_pack_ids: send[j*capacity + i] (int32) = the i-th unique row of the plan owned by
 *   shard j as an owner-local id, or past that run the owner's spare row (its row count,
 *   min(shard_rows, V - j*shard_rows)); counts[j] / offsets[j] (int32[n_shards]) = the run's
 *   length and start in the plan's unique rows; a run longer than capacity ORs
 *   CTR_EFLAG_CAPACITY into *err_flag.
 * ctr_shard_runs_copy: rows of `width` floats between the compact order (run j at offsets[j])
 *   and the padded layout (run j at j*capacity): pack = 1 writes every padded row (zeros past
 *   a run), pack = 0 writes the runs back to their compact places. */
/* ctr_batch_stage_copy: one launch copying a batch into its fixed input slot — n0 bytes src0 ->
 * dst0 (the ids) and n1 bytes src1 -> dst1 (the labels; n1 = 0: none); device pointers, bitwise
 * copies. The staging of the reference's per-iteration batch (all_main/pretrain_main.py:71-74,
 * `for x, y in loader: x.to(device)`) ahead of the step that trains on it. */
int ctr_batch_stage_copy(void* dst0, const void* src0, int64_t n0, void* dst1, const void* src1,
                         int64_t n1, ctr_stream_t stream);
int ctr_shard_pack_ids(const ctr_sparse_plan* plan, int64_t shard_rows, int64_t V, int n_shards,
                       int64_t capacity, int32_t* send, int32_t* counts, int32_t* offsets,
                       int32_t* err_flag, ctr_stream_t stream);
int ctr_shard_runs_copy(const float* src, float* dst, int64_t width, int64_t capacity,
                        int n_shards, const int32_t* counts, const int32_t* offsets, int pack,
                        ctr_stream_t stream);
/* Cyclic row sharding (ABI v12): global row r belongs to shard r % n_shards as its local row
 * r / n_shards, so every shard owns rows of every feature field (the field-ordered vocabulary
 * of the reference's encoders, creat_data.py / data_.py, puts the high-cardinality fields in
 * the last row blocks: contiguous blocks leave one owner most of every batch's rows).
 * ctr_shard_permute_ids: in place, ids[i] = (r % n_shards) * shard_rows + r / n_shards — the
 *   space in which each shard's rows are one contiguous block [j*shard_rows, j*shard_rows+n_j),
 *   n_j = ceil((V - j) / n_shards); ids outside [0, V) raise CTR_EFLAG_INDEX and map to
 *   row 0. int64 or int32 ids (ids_is_64); the plan and the exchange then run on these ids.
 * ctr_shard_pack_ids_layout: ctr_shard_pack_ids over permuted ids; cyclic != 0: each owner's
 *   spare row is its cyclic row count n_j (blocks: as ctr_shard_pack_ids). */
int ctr_shard_permute_ids(void* ids, int ids_is_64, int64_t count, int64_t V, int n_shards,
                          int64_t shard_rows, int32_t* err_flag, ctr_stream_t stream);
int ctr_shard_pack_ids_layout(const ctr_sparse_plan* plan, int64_t shard_rows, int64_t V,
                              int n_shards, int cyclic, int64_t capacity, int32_t* send,
                              int32_t* counts, int32_t* offsets, int32_t* err_flag,
                              ctr_stream_t stream);
/* The same exchange with each row's linear weight in the same message: the padded buffer is
 * n_shards chunks of `chunk` floats (chunk >= capacity*K + capacity, a multiple of 4), chunk j
 * = [capacity rows of K floats][capacity linear weights][padding]; lin == NULL: rows only.
 * One equal-split all-to-all then moves rows and weights (and their gradients) together.
 * ctr_shard_gather_rows (owner): chunk j row i = (emb[ids[j*capacity+i]], lin[...]).
 * ctr_shard_rows_pack: chunk j row i = (rows[offsets[j]+i], lin[...]) for i < counts[j],
 *   zeros past it.  ctr_shard_rows_unpack: the reverse, for i < counts[j].
 * K % 4 == 0, 16-B aligned buffers. */
int ctr_shard_gather_rows(const float* emb, const float* lin, int K, const int32_t* ids,
                          int n_shards, int64_t capacity, int64_t chunk, float* out,
                          ctr_stream_t stream);
int ctr_shard_rows_pack(const float* rows, const float* lin, int K, int64_t capacity,
                        int64_t chunk, int n_shards, const int32_t* counts,
                        const int32_t* offsets, float* out, ctr_stream_t stream);
int ctr_shard_rows_unpack(const float* in, int K, int64_t capacity, int64_t chunk, int n_shards,
                          const int32_t* counts, const int32_t* offsets, float* rows, float* lin,
                          ctr_stream_t stream);
/* ctr_shard_row_grads: a row-sharded requester's per-row gradient sums (ctr_fm_embedding_grad
 * when gz != NULL, else ctr_segment_sum_rows over vals without linear sums) written straight
 * into the exchange chunks of ctr_shard_rows_pack's layout: unique row u of run j (the last
 * run with run_offsets[j] <= u) goes to row u - run_offsets[j] of chunk j, its linear sum
 * after the chunk's run_len rows (lin != 0). Rows past a run's count are not written (the
 * owner's spare row takes them). K % 4 == 0, 16-B aligned buffers. */
int ctr_shard_row_grads(const ctr_sparse_plan* plan, int F, int K, const float* emb,
                        const float* gz, const float* sum_e, const float* dx, const float* vals,
                        int lin, int n_runs, const int32_t* run_offsets, int64_t run_len,
                        int64_t chunk, float* out_chunks, void* ws, int64_t ws_bytes,
                        ctr_stream_t stream);
int ctr_sparse_plan_build(const void* idx, int idx_type, int64_t V, const ctr_sparse_plan* plan,
                          void* ws, int64_t ws_bytes, int32_t* err_flag, ctr_stream_t stream);
/* The same plan (bit-identical) for ids laid out as a [S/F][F] matrix (slot s = b*F + f: the
 * batch's feature fields as columns): each column sorted inside one workgroup, then merged —
 * 2 launches of work where a column's ids occupy a range of their own (the CTR layouts), and
 * exact for any ids. Falls back to ctr_sparse_plan_build for S/F > 8192 or F > 256. */
int ctr_sparse_plan_build_cols(const void* idx, int idx_type, int64_t V, int64_t F,
                               const ctr_sparse_plan* plan, void* ws, int64_t ws_bytes,
                               int32_t* err_flag, ctr_stream_t stream);

/* Segmented row sums over a plan, deterministic: each row's slots are summed in slot
 * order in chunks of 16 positions, chunk partials are then added in chunk order (hot
 * rows spread over many waves; identical bits run to run and rank to rank).
 *   ctr_fm_embedding_grad (FM / DeepFM backward, slot s = b*F + f):
 *     grad_rows[u,:] = sum_{s in row u} ((gz[b]*sum_e[b,:] - gz[b]*E[row,:]) + dx[s,:])
 *     grad_lin[u]    = sum_{s in row u} gz[b]
 *     dx (the MLP input gradient, [B, F*K]) is NULL for FM.
 *   ctr_segment_sum_rows (generic; multi-GPU exchange): out[u,:] = sum vals[s,:],
 *     out_lin[u] = sum vals_lin[s] (both optional-lin).
 * If rowmap != NULL also rowmap[row_u] = u (ctr_adam_embedding consumes and resets it).
 * Replaces: FM/DeepFM backward through p_model.py:47-54 / 303-311 / 320-322 and
 * embedding_dense_backward. */
int64_t ctr_segment_workspace_bytes(int64_t S, int K);
int ctr_fm_embedding_grad(const ctr_sparse_plan* plan, int F, int K, const float* emb,
                          const float* gz, const float* sum_e, const float* dx,
                          float* grad_rows, float* grad_lin, int32_t* rowmap, void* ws,
                          int64_t ws_bytes, ctr_stream_t stream);
int ctr_segment_sum_rows(const ctr_sparse_plan* plan, int K, const float* vals,
                         const float* vals_lin, float* out, float* out_lin, int32_t* rowmap,
                         void* ws, int64_t ws_bytes, ctr_stream_t stream);

/* Dense gradient for the autograd (drop-in) path: dense[V,K] (and dense_lin[V], optional)
 * must be zero on entry; dense[row_u,:] = grad_rows[u,:]. */
int ctr_rows_to_dense(const ctr_sparse_plan* plan, int K, const float* grad_rows,
                      const float* grad_lin, float* dense, float* dense_lin,
                      ctr_stream_t stream);

/* ---------------------------------------------------------------- A5: Adam -----------
 * torch.optim.Adam(lr, betas, eps, weight_decay) with coupled L2, one step, for EVERY
 * element (dense semantics). Host-computed step scalars (as torch computes them):
 *   step_size = lr / (1 - beta1^t),  bc2_sqrt = sqrt(1 - beta2^t).
 * Per element: g += wd*p; m += (1-beta1)*(g-m); v = v*beta2 + (1-beta2)*g*g;
 *              p += -step_size * (m / (sqrt(v)/bc2_sqrt + eps))
 * (m, v bit-identical to torch's CPU Adam; the p step uses ~1-ulp hardware sqrt/rcp).
 * ctr_adam_dense:     g is a dense gradient (MLP, bias).
 * ctr_adam_embedding: the embedding table E[V,K] and the linear table w[V] in one pass;
 *   the gradient of row r is grad_rows[rowmap[r]] when rowmap[r] >= 0, else 0; rowmap
 *   entries read >= 0 are reset to -1. lin/m_lin/v_lin may be NULL (Feature tables w/o
 *   a linear term).
 * Device step (HIP-graph replay): with step_ptr != NULL the step t = *step_ptr is read on
 * the device and the scalars come from step_table (layout of ctr_adam_deferred_rows
 * below); step_size / bc2_sqrt are then ignored.
 * Replaces: torch.optim.Adam.step at all_main/pretrain_main.py:78,153. */
int ctr_adam_dense(float* p, const float* g, float* m, float* v, int64_t n, double step_size,
                   double bc2_sqrt, const float* step_table, const int32_t* step_ptr,
                   double beta1, double beta2, double eps, double weight_decay,
                   ctr_stream_t stream);
/* ctr_adam_dense_planes: ctr_adam_dense that also rewrites the bf16 planes (ctr_planes) of
 *   up to three row-major [rows, cols] sub-matrices of p (the MLP weights: p[offset + r*cols
 *   + c]) with the updated values, so the next step's plane GEMMs need no ctr_split_planes.
 *   offset % 4 == 0, n % 4 == 0, 16-B aligned vectors; any cols (a multiple of 4 is faster).
 *   Replaces: the same optimizer.step; the planes are this framework's GEMM operand format. */
typedef struct ctr_plane_view {
  int64_t offset;
  int64_t rows;
  int64_t cols;
  ctr_planes planes;
} ctr_plane_view;
int ctr_adam_dense_planes(float* p, const float* g, float* m, float* v, int64_t n,
                          double step_size, double bc2_sqrt, const float* step_table,
                          const int32_t* step_ptr, double beta1, double beta2, double eps,
                          double weight_decay, const ctr_plane_view* views, int n_views,
                          ctr_stream_t stream);
int ctr_adam_embedding(float* emb, float* m_emb, float* v_emb, float* lin, float* m_lin,
                       float* v_lin, int64_t V, int K, int32_t* rowmap,
                       const float* grad_rows, const float* grad_lin, double step_size,
                       double bc2_sqrt, const float* step_table, const int32_t* step_ptr,
                       double beta1, double beta2, double eps, double weight_decay,
                       ctr_stream_t stream);

/* Deferred-exact dense Adam (temporal blocking) — same results as ctr_adam_embedding,
 * bitwise. A row absent from a batch is updated with g = wd*p, a function of its own state;
 * last[r] (int32 [V], 0 at optimizer creation) records the step row r is current to, and
 * missed steps are replayed in registers with the same per-element arithmetic and the same
 * per-step scalars step_table[2t] = -lr/(1-beta1^t), step_table[2t+1] = 1/sqrt(1-beta2^t)
 * (fp32, host-computed in double as torch does; entries 0..step valid):
 *   ctr_adam_deferred_rows, grad_rows == NULL: bring the plan's unique rows to `step`
 *     (call before a forward pass reads them; catch-up to the last completed step);
 *   ctr_adam_deferred_rows, grad_rows != NULL: bring them to step-1 and apply step `step`
 *     with their gradient (grad_rows[u], grad_lin[u] for unique row u);
 *   ctr_adam_deferred_flush: bring every row to `step` (before anything else reads the
 *     tables: epoch end, checkpoint, evaluation).
 * ctr_adam_deferred_rows reads the step from *step_ptr on the device when step_ptr != NULL.
 * Replaces: torch.optim.Adam.step at all_main/pretrain_main.py:78 over nn.Embedding weights. */
int ctr_adam_deferred_rows(float* emb, float* m_emb, float* v_emb, float* lin, float* m_lin,
                           float* v_lin, int64_t V, int K, int32_t* last,
                           const ctr_sparse_plan* plan, const float* grad_rows,
                           const float* grad_lin, int64_t step, const int32_t* step_ptr,
                           const float* step_table, double beta1, double beta2, double eps,
                           double weight_decay, ctr_stream_t stream);
/* ctr_adam_deferred_entries: the owner side of a row-sharded step — for each unique row u of
 * `plan` (built over the received entries), g_u = the sum of vals[e] (and vals_lin[e]) over
 * its entries e in plan order (source rank, then position: sequential fp32 adds), then the
 * row replayed to step-1 and stepped with g_u (ctr_adam_deferred_rows with grad_rows = the
 * sums, in one launch). skip_row (e.g. the shard's spare row, the padding target) is left
 * untouched (-1: none). out [U][K] / out_lin [U] (optional): the sums. K % 4 == 0, (K/4) | 64.
 * run_len = 0: vals [entries][K], vals_lin [entries]; run_len > 0: vals is the chunked
 * exchange layout of ctr_shard_rows_pack (entry e = row e % run_len of chunk e / run_len,
 * chunk floats per chunk, the linear values after the rows; vals_lin unused). */
int ctr_adam_deferred_entries(float* emb, float* m_emb, float* v_emb, float* lin, float* m_lin,
                              float* v_lin, int64_t V, int K, int32_t* last,
                              const ctr_sparse_plan* plan, const float* vals,
                              const float* vals_lin, int64_t run_len, int64_t chunk,
                              int64_t skip_row, int64_t step,
                              const int32_t* step_ptr, const float* step_table, double beta1,
                              double beta2, double eps, double weight_decay, float* out,
                              float* out_lin, ctr_stream_t stream);
int ctr_adam_deferred_flush(float* emb, float* m_emb, float* v_emb, float* lin, float* m_lin,
                            float* v_lin, int64_t V, int K, int32_t* last, int64_t step,
                            const float* step_table, double beta1, double beta2, double eps,
                            double weight_decay, ctr_stream_t stream);
/* The catch-up of ctr_adam_deferred_rows (grad_rows == NULL) taken straight from a batch's
 * S feature ids, no sparse plan needed (the plan can then be built concurrently on another
 * stream): duplicates are resolved through `owner`, a caller-owned int32[V] scratch (no
 * initialisation needed); the target step is read from device memory (*step_ptr), so the
 * call can be captured in a HIP graph. Needs K % 4 == 0 and (K/4) | 64. */
int ctr_adam_deferred_catchup_ids(float* emb, float* m_emb, float* v_emb, float* lin,
                                  float* m_lin, float* v_lin, int64_t V, int K, int32_t* last,
                                  const void* idx, int idx_type, int64_t S, int32_t* owner,
                                  const int32_t* step_ptr, const float* step_table, double beta1,
                                  double beta2, double eps, double weight_decay,
                                  ctr_stream_t stream);
/* Fused scatter + deferred Adam (ws == 1, deferred mode): the segmented row sums of
 * ctr_fm_embedding_grad / ctr_segment_sum_rows with ctr_adam_deferred_rows(the sums,
 * step = *step_ptr) folded into the pass that finishes the rows spanning several chunks —
 * bitwise the same tables, one launch fewer, and the spanning rows' sums never round-trip
 * through memory. grad_rows / grad_lin (out / out_lin) are required scratch; with
 * keep_sums != 0 they hold every row's sum afterwards (else only the rows inside one
 * chunk). Needs K % 4 == 0, K <= 256.
 * Replaces: embedding_dense_backward + optimizer.step of all_main/pretrain_main.py:77-78. */
typedef struct ctr_deferred_table {
  float* emb;
  float* m_emb;
  float* v_emb;
  float* lin;    /* the linear table w[V] and its moments, or all NULL */
  float* m_lin;
  float* v_lin;
  int32_t* last; /* step each row is current to */
} ctr_deferred_table;
int ctr_fm_embedding_grad_adam(const ctr_sparse_plan* plan, int F, int K, const float* gz,
                               const float* sum_e, const float* dx,
                               const ctr_deferred_table* table, const int32_t* step_ptr,
                               const float* step_table, double beta1, double beta2, double eps,
                               double weight_decay, float* grad_rows, float* grad_lin,
                               int keep_sums, void* ws, int64_t ws_bytes, ctr_stream_t stream);
int ctr_segment_sum_rows_adam(const ctr_sparse_plan* plan, int K, const float* vals,
                              const float* vals_lin, const ctr_deferred_table* table,
                              const int32_t* step_ptr, const float* step_table, double beta1,
                              double beta2, double eps, double weight_decay, float* out,
                              float* out_lin, int keep_sums, void* ws, int64_t ws_bytes,
                              ctr_stream_t stream);

/* Device step counters (int32[2]): ctr[0] = completed steps, ctr[1] = the step in flight.
 * ctr_step_begin: ctr[1] = ctr[0] + 1;  ctr_step_end: ctr[0] = ctr[1], ctr[1] += 1. A
 * counter initialised to {0, 1} therefore needs no ctr_step_begin (one launch less per
 * step); within a step both values are constant, so kernels on several streams can read
 * them: the catch-up and the dropout stream read ctr[0], the Adam apply ctr[1]. */
int ctr_step_begin(int32_t* step_ctr, ctr_stream_t stream);
int ctr_step_end(int32_t* step_ctr, ctr_stream_t stream);
/* ctr_step_end_loss: ctr_step_end, and loss_sum[0] += (double)loss[0] — the driver's epoch
 *   loss accumulated on the device (fp64, in step order: bitwise the reference's Python
 *   `total_loss += train_loss.item()`, all_main/pretrain_main.py:79, with no host sync per
 *   step). */
int ctr_step_end_loss(int32_t* step_ctr, const float* loss, double* loss_sum,
                      ctr_stream_t stream);
/* ctr_fm_step_tail: the FM step's dense tail (one process) in one launch —
 *   loss_out[0] = loss_scale * sum(loss_elem[:B]), bias_grad[0] = sum(gz[:B]) (bitwise
 *   ctr_sum_f32), Adam on the flat dense vector (p, g, m, v)[:n] at step ctr[1] (bitwise
 *   ctr_adam_dense; bias_grad may point into g), then ctr_step_end(step_ctr); loss_sum
 *   (may be NULL): loss_sum[0] += (double)loss_out[0], as ctr_step_end_loss.
 *   Replaces: all_main/pretrain_main.py:74-78 (loss.backward's bias gradient, the batch
 *   loss, optimizer.step() on the FM bias) at the end of a step. */
int ctr_fm_step_tail(const float* loss_elem, const float* gz, int64_t B, float loss_scale,
                     float* loss_out, float* bias_grad, float* p, const float* g, float* m,
                     float* v, int64_t n, const float* step_table, int32_t* step_ctr,
                     double beta1, double beta2, double eps, double weight_decay,
                     double* loss_sum, ctr_stream_t stream);

/* ------------------------------------------------ A7: Feature_Embedding -------------
 * out[b] = [ <E[x_bi],E[x_bj]> for i<j in row-major pair order ] ++ flat(E[x_b]),
 * out is [B, F(F-1)/2 + F*K]. Replaces: Feature_embedding.py:51-59. */
int ctr_feature_embedding_forward(const void* idx, int idx_type, int64_t B, int F, int K,
                                  int64_t V, const float* emb, float* out, int32_t* err_flag,
                                  ctr_stream_t stream);
/* ctr_feature_embedding_forward_planes: the same, and the state's three exact bf16 planes
 *   (ctr_planes, >= [B, F(F-1)/2 + F*K]) for the planes GEMM of the policy's first layer
 *   (out_planes NULL: the plain call). Replaces: Feature_embedding.py:51-59 feeding
 *   PG_model.py:52 (the first nn.Linear of Net). */
int ctr_feature_embedding_forward_planes(const void* idx, int idx_type, int64_t B, int F,
                                         int K, int64_t V, const float* emb, float* out,
                                         const ctr_planes* out_planes, int32_t* err_flag,
                                         ctr_stream_t stream);

/* ------------------------------------------ §8f: binary on-disk batches (host) -----
 * ctr_csv_to_bin: the reference's encoded CSV (`label,idx_1..idx_F` per line,
 *   src/encode/data_.py:85; parsed by pd.read_csv at all_main/pretrain_main.py:50-53) ->
 *   a "CTRBIN01" file: 64-byte header (rows, cols = 1+F, max feature id) + int32
 *   [rows][cols] (label, ids), memory-mappable. Streams in constant memory; ragged rows
 *   or non-integer fields fail with the line number. Host code, no GPU needed.
 * ctr_bin_info: header fields of such a file (validates magic and size). */
int ctr_csv_to_bin(const char* csv_path, const char* bin_path, int64_t* rows, int32_t* cols,
                   int64_t* max_id);
int ctr_bin_info(const char* bin_path, int64_t* rows, int32_t* cols, int64_t* max_id,
                 int64_t* data_offset);

/* ------------------------------------- §8f: ensemble prediction + sign reward -------
 * generate_preds of the RL drivers (hybrid_td3_main_per_v10.py:54-164): preds [B, M] (row
 * stride ld_preds; the M pretrained models' pCTRs), actions [B] (ensemble size, 1-based),
 * prob_weights / c_actions [B, M], labels [B] (0/1) -> y_preds [B], rewards [B],
 * return_c_actions [B, M]; M <= 32. Keeps the reference's indexing of the sorted
 * c_actions by the example's ordinal within its action group (line 127). rank_ws:
 * int32[B] scratch. action_type / label_type: CTR_IDX_I32 or CTR_IDX_I64. */
int ctr_ensemble_preds(const float* preds, int64_t B, int M, int64_t ld_preds,
                       const void* actions, int action_type, const float* prob_weights,
                       const float* c_actions, const void* labels, int label_type,
                       float* y_preds, float* rewards, float* return_c_actions, int32_t* rank_ws,
                       ctr_stream_t stream);

/* ------------------------------------------------ §8f: FFM (field-aware FM) ---------
 * tables: a DEVICE array of F pointers, table t = field t's embedding [V, K] (K <= 64,
 * F*V < 2^31). ctr_ffm_forward: z = bias + sum_f lin[x_f] + sum_{i<j} sum_k
 * E_j[x_i,k] * E_i[x_j,k] (p_model.FFM.forward, p_model.py:82-100), with the fused BCE head
 * when labels != NULL (as ctr_fm_forward). ctr_ffm_backward: the F(F-1) row gradients of
 * every example, vals[pos, :] = gz[b] * E_f[x_bt, :] for table t's row x_bf, key[pos] =
 * t*V + x_bf, pos = (b*F + f)*(F-1) + (t < f ? t : t-1) ([B*F*(F-1)] keys, [.., K] vals):
 * a sparse plan over the keys (key range F*V) + ctr_segment_sum_rows give every table's
 * row sums in slot order. */
int ctr_ffm_forward(const void* idx, int idx_type, int64_t B, int F, int K, int64_t V,
                    const float* const* tables, const float* lin, const float* bias, float* z,
                    const float* labels, float mean_div, float* p, float* loss_elem, float* gz,
                    int32_t* err_flag, ctr_stream_t stream);
int ctr_ffm_backward(const void* idx, int idx_type, int64_t B, int F, int K, int64_t V,
                     const float* const* tables, const float* gz, int32_t* keys, float* vals,
                     ctr_stream_t stream);
/* ctr_ffm_keys: the keys of ctr_ffm_backward alone (same positions): the table rows an FFM
 * step reads and updates, for the fused trainer's catch-up before the forward. */
int ctr_ffm_keys(const void* idx, int idx_type, int64_t B, int F, int64_t V, int32_t* keys,
                 int32_t* err_flag, ctr_stream_t stream);

/* ------------------------------------------------ §8f: IPNN (InnerPNN) --------------
 * ctr_ipnn_forward: cat[b] = flat(E[x_b]) (F*K) ++ [ <E[x_bi],E[x_bj]> for i<j, row-major ]
 *   (P = F(F-1)/2), cat is [B, >= F*K + P] with row stride ldc: the MLP input of
 *   p_model.InnerPNN.forward (p_model.py:187-195).
 * ctr_ipnn_backward: dslot[b*F+f, :] (slot order, [B*F, K]) = dcat[b, f*K:(f+1)*K]
 *   + sum_{j != f} dcat[b, F*K + pair(f,j)] * E[x_bj, :] — the gradient of every slot's
 *   embedding through the view and the two pair index ops; per-row sums then go through
 *   ctr_segment_sum_rows (embedding_dense_backward of p_model.py:187). */
int ctr_ipnn_forward(const void* idx, int idx_type, int64_t B, int F, int K, int64_t V,
                     const float* emb, float* cat, int64_t ldc, int32_t* err_flag,
                     ctr_stream_t stream);
/* ctr_ipnn_forward_planes: ctr_ipnn_forward writing cat as its three bf16 planes (the
 *   split-bf16 MLP GEMMs' operand) — cat itself may then be NULL (no fp32 copy, no split
 *   pass); with both, both are written. */
int ctr_ipnn_forward_planes(const void* idx, int idx_type, int64_t B, int F, int K, int64_t V,
                            const float* emb, float* cat, int64_t ldc,
                            const ctr_planes* cat_planes, int32_t* err_flag,
                            ctr_stream_t stream);
int ctr_ipnn_backward(const void* idx, int idx_type, int64_t B, int F, int K, int64_t V,
                      const float* emb, const float* dcat, int64_t ldd, float* dslot,
                      ctr_stream_t stream);

/* ------------------------------------------------------ A8: REINFORCE (PG) -----------
 * ctr_softmax_rows: out[b,:] = softmax(x[b,:]) (PG_model.py:56).
 * ctr_pg_discount_norm: discounted return of an episode, reverse recurrence
 *   d[i] = r[i] + gamma*d[i+1] in fp64, then (d - mean)/std (population std), written as
 *   fp64 `out` and fp32 `out_f32`; stats[0..1] = mean, std (fp64, std before division).
 *   Replaces PG_model.py:139-154.
 * ctr_pg_loss_grad: loss = sum_b(-log probs[b, act_b - 1]) * mean(vt) (PG_model.py:104-107,
 *   actions 1-based) and the gradient w.r.t. the softmax LOGITS (softmax backward fused),
 *   scaled by grad_scale. loss_out is a device scalar.
 * ctr_pg_vt_mean: out[0] = mean(vt[0..n)) summed in the order ctr_pg_loss_grad uses.
 * ctr_pg_loss_grad_global: ctr_pg_loss_grad for one rank's slice of an episode that is
 *   split over data-parallel ranks: c = vt_mean[0] (the episode-wide mean, device scalar)
 *   and loss_out = sum_b(-log probs[b, act_b - 1]) * vt_mean[0], this rank's share of the
 *   episode loss (the shares sum to it). Same reference lines as ctr_pg_loss_grad. */
int ctr_softmax_rows(const float* x, int64_t B, int A, float* out, ctr_stream_t stream);
int64_t ctr_pg_workspace_bytes(int64_t n);
int ctr_pg_discount_norm(const float* r, int64_t n, double gamma, double* out, float* out_f32,
                         double* stats, void* ws, int64_t ws_bytes, ctr_stream_t stream);
int ctr_pg_loss_grad(const float* probs, const int64_t* acts, const float* vt, int64_t B,
                     int A, float grad_scale, float* loss_out, float* dlogits, void* ws,
                     int64_t ws_bytes, ctr_stream_t stream);
int ctr_pg_vt_mean(const float* vt, int64_t n, float* out, ctr_stream_t stream);
int ctr_pg_loss_grad_global(const float* probs, const int64_t* acts, int64_t B, int A,
                            const float* vt_mean, float grad_scale, float* loss_out,
                            float* dlogits, ctr_stream_t stream);


/* ==== Op-level interface: one POD argument struct per torch.library op ====
 * ctr_op_<op>(const ctr_<op>_args* a, stream) is the C form of the `ctr::<op>` PyTorch op
 * (rl_ctr_prediction_amd/torch_ops.py) — what a binding without torch (ctypes, cgo, JNI)
 * calls. Each composes the entry points above with the same results, bit for bit. (The
 * `ctr_op_` prefix keeps the names apart from the flat entry points: C has no overloads.)
 * Scratch: ctr_workspace_bytes(op, dims, n_dims) with the op's dims listed below; the op
 * carves its plan / partials / row map out of `ws`. Outputs that the reference returns as
 * fresh tensors (dense gradients) are caller-owned buffers the op zero-fills itself.
 * `flags`: CTR_OPF_DETERMINISTIC (every op here is deterministic: sums in a fixed order, no
 * float atomics; the flag is accepted and always honoured). */
enum ctr_op {
  CTR_OP_FM_FWD = 1,               /* dims: none                     */
  CTR_OP_FM_BWD = 2,               /* dims: {B, F, K, V}             */
  CTR_OP_DEEPFM_GATHER_CONCAT = 3, /* dims: none                     */
  CTR_OP_EMB_SCATTER_ADD = 4,      /* dims: {n_slots, K, V}          */
  CTR_OP_ADAM_DENSE = 5,           /* dims: none                     */
  CTR_OP_ADAM_ROWWISE = 6,         /* dims: {V}                      */
  CTR_OP_PAIRWISE_FE = 7,          /* dims: none                     */
  CTR_OP_PG_RETURNS = 8            /* dims: {n}                      */
};
enum ctr_op_flags { CTR_OPF_DETERMINISTIC = 1 };
/* Scratch bytes of op `op` for `dims` (see enum ctr_op); -1 for an unknown op or bad dims. */
int64_t ctr_workspace_bytes(int op, const int64_t* dims, int n_dims);

/* ctr::fm_fwd — FM.forward logit and the per-example embedding sums its backward needs:
 * z[B] (the [B,1] logit), sum_e[B,K]. Replaces p_model.py:40-57. */
typedef struct ctr_fm_fwd_args {
  const void* idx; int idx_type; int64_t B; int F; int K; int64_t V;
  const float* emb; const float* lin; const float* bias;
  float* z; float* sum_e; int32_t* err_flag; int flags;
} ctr_fm_fwd_args;
int ctr_op_fm_fwd(const ctr_fm_fwd_args* a, ctr_stream_t stream);

/* ctr::fm_bwd — FM's parameter gradients from dL/dz: dense g_emb[V,K], g_lin[V] (both
 * zero-filled here, then the batch's rows written: embedding_dense_backward) and g_bias[1]
 * = sum gz. Replaces autograd through p_model.py:40-57 (all_main/pretrain_main.py:77). */
typedef struct ctr_fm_bwd_args {
  const void* idx; int idx_type; int64_t B; int F; int K; int64_t V;
  const float* emb; const float* sum_e; const float* gz;
  float* g_emb; float* g_lin; float* g_bias;
  void* ws; int64_t ws_bytes; int32_t* err_flag; int flags;
} ctr_fm_bwd_args;
int ctr_op_fm_bwd(const ctr_fm_bwd_args* a, ctr_stream_t stream);

/* ctr::deepfm_gather_concat — out[B, F*K] = E[x] flattened (DeepFM's MLP input,
 * p_model.py:320-321). */
typedef struct ctr_deepfm_gather_concat_args {
  const void* idx; int idx_type; int64_t B; int F; int K; int64_t V;
  const float* emb; float* out; int32_t* err_flag; int flags;
} ctr_deepfm_gather_concat_args;
int ctr_op_deepfm_gather_concat(const ctr_deepfm_gather_concat_args* a, ctr_stream_t stream);

/* ctr::emb_scatter_add — dense[V,K] (zero-filled here) = embedding_dense_backward of
 * per-slot gradients grad_slots[n_slots, K] at ids idx[n_slots] (slot order kept per row). */
typedef struct ctr_emb_scatter_add_args {
  const void* idx; int idx_type; int64_t n_slots; int K; int64_t V;
  const float* grad_slots; float* dense;
  void* ws; int64_t ws_bytes; int32_t* err_flag; int flags;
} ctr_emb_scatter_add_args;
int ctr_op_emb_scatter_add(const ctr_emb_scatter_add_args* a, ctr_stream_t stream);

/* ctr::adam_dense — one torch.optim.Adam step (coupled L2) of n elements at step `step`
 * (1-based; the bias corrections are computed here in double as torch does). Replaces
 * all_main/pretrain_main.py:78 (optimizer.step) for dense parameters. */
typedef struct ctr_adam_dense_args {
  float* p; const float* g; float* m; float* v; int64_t n; int64_t step;
  double lr; double beta1; double beta2; double eps; double weight_decay; int flags;
} ctr_adam_dense_args;
int ctr_op_adam_dense(const ctr_adam_dense_args* a, ctr_stream_t stream);

/* ctr::adam_rowwise — the same Adam step for EVERY row of emb[V,K] (dense semantics), the
 * gradient of row rows[u] being grad_rows[u,:] and 0 for rows not listed (rows distinct).
 * A listed row outside [0, V) is not applied and raises CTR_EFLAG_INDEX in *err_flag (may
 * be NULL: then such a row is dropped silently), as the torch op's index_copy_ raises. */
typedef struct ctr_adam_rowwise_args {
  float* emb; float* m; float* v; int64_t V; int K;
  const void* rows; int rows_type; int64_t n_rows; const float* grad_rows; int64_t step;
  double lr; double beta1; double beta2; double eps; double weight_decay;
  void* ws; int64_t ws_bytes; int32_t* err_flag; int flags;
} ctr_adam_rowwise_args;
int ctr_op_adam_rowwise(const ctr_adam_rowwise_args* a, ctr_stream_t stream);

/* ctr::pairwise_fe — Feature_Embedding.forward: [B, F(F-1)/2 + F*K]
 * (Feature_embedding.py:51-59). */
typedef struct ctr_pairwise_fe_args {
  const void* idx; int idx_type; int64_t B; int F; int K; int64_t V;
  const float* emb; float* out; int32_t* err_flag; int flags;
} ctr_pairwise_fe_args;
int ctr_op_pairwise_fe(const ctr_pairwise_fe_args* a, ctr_stream_t stream);

/* ctr::pg_returns — discount_and_norm_rewards: vt (fp64) and its fp32 copy
 * (PG_model.py:139-154). */
typedef struct ctr_pg_returns_args {
  const float* r; int64_t n; double gamma; double* vt; float* vt_f32;
  void* ws; int64_t ws_bytes; int flags;
} ctr_pg_returns_args;
int ctr_op_pg_returns(const ctr_pg_returns_args* a, ctr_stream_t stream);

#ifdef __cplusplus
}
#endif

#endif /* CTR_HIP_H */

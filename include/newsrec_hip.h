/* newsrec_hip.h — C ABI of libnewsrec_hip.so, the MI355X (gfx950) kernels of the two-tower
 * news-recommendation train/score path of tyh666/News-Recommendation-MIND.
 *
 * The reference is 100 % Python/PyTorch: it has no FFI of its own.  Each entry point below
 * replaces the aten ops that one reference function launches (cited per entry); the Python
 * shim (news-recommendation-mind_amd/newsrec_amd/_lib.py) binds them with ctypes and keeps
 * the reference's nn.Module contracts.
 *
 * Conventions (all entries):
 *   - every pointer is a DEVICE pointer; the caller owns all memory (inputs, outputs and
 *     workspace).  The library never allocates, frees or synchronises.
 *   - calls are stream-ordered on `stream` and may be captured into a hipGraph.
 *   - return 0 on success, a negative hipError_t on a launch failure, or
 *     -1000 - k for an invalid argument k.
 *   - fp32 storage and fp32 arithmetic (the reference has no autocast anywhere).
 */
#ifndef NEWSREC_HIP_H
#define NEWSREC_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ihipStream_t* hipStream_t;

/* Hash of the sources this library was built from (build.py source_hash: csrc, include, flags);
 * the Python binding refuses a library whose hash differs from the tree next to it. */
const char* nr_build_hash(void);

/* ------------------------------------------------------------------ GEMM operands */

/* How the stored row index of an operand is found. */
enum nr_rows_map {
  NR_ROWS_PLAIN = 0,  /* row r  -> data + r * ld                                          */
  NR_ROWS_GATHER = 1, /* row r  -> data + rows[r] * ld   (word-embedding gather, BERT.py:39) */
  NR_ROWS_CONV3 = 2   /* row r = (news n, pos t), tap j in {0,1,2} of a k=3, pad=1 Conv1d:
                         data + rows[n*seq_len + t+j-1] * ld, zeros when t+j-1 is outside
                         [0, seq_len) (CNN.py:12-17).  Column c of tap j is c - j*seg.    */
};

enum nr_layout {
  NR_KCONTIG = 0, /* stored rows are the M (or N) index, k contiguous: A[M][K], B[N][K]   */
  NR_MNCONTIG = 1 /* stored rows are the k index, M (or N) contiguous: A[K][M], B[K][N]   */
};

typedef struct nr_operand {
  const float* data;
  int64_t ld;          /* elements between stored rows (GATHER/CONV3 tables: multiple of 4,
                          16-B aligned; plain operands take float4 loads when aligned)   */
  const int64_t* rows; /* row table for GATHER / CONV3 (token ids), else NULL             */
  int32_t map;         /* enum nr_rows_map                                                 */
  int32_t seq_len;     /* CONV3: tokens per news (L)                                       */
  int32_t seg;         /* CONV3: columns per tap (E)                                       */
  int32_t layout;      /* enum nr_layout                                                   */
} nr_operand;

enum nr_epilogue {
  NR_EPI_STORE = 0,      /* C[m][n] = acc + bias[n]                                          */
  NR_EPI_STORE_RELU = 1, /* C[m][n] = max(acc + bias[n], 0)                 (CNN.py:41-42)   */
  NR_EPI_ATOMIC = 2,     /* C[m][n] += acc  (split-K weight gradients; C pre-zeroed)          */
  NR_EPI_SCATTER = 3,    /* C[c_rows(m)][n'] += acc, rows equal to pad_row skipped: the
                            embedding backward (nn.Embedding padding_idx) fused into dgrad  */
  NR_EPI_STORE_TANH = 4, /* C[m][n] = tanh(acc + bias[n])                   (CNN.py:46)      */
  NR_EPI_ACCUM_GATE = 5, /* C[m][n] = aux[m][n] > 0 ? C[m][n] + acc : 0, aux = c_rows->data
                            (ld c_rows->ld): adds a second gradient path, then ReLU's mask   */
  NR_EPI_ACCUM = 6,      /* C[m][n] += acc + bias[n]  (row tiles are block-exclusive)         */
  NR_EPI_SCATTER_STORE = 7, /* C[c_rows(m)][n] = acc for DISTINCT GATHER rows (pad_row skipped):
                            the table gradient over nr_unique_rows' ids, plain vector stores */
  NR_EPI_STORE_GELU = 8, /* aux[m][n] = acc + bias[n]; C[m][n] = gelu(aux[m][n]) (exact erf GELU,
                            BertIntermediate); aux = c_rows->data, ld c_rows->ld               */
  NR_EPI_GELU_GRAD = 9,  /* C[m][n] = acc * gelu'(aux[m][n]), aux = c_rows->data (ld c_rows->ld):
                            the dgrad of the intermediate dense through its GELU               */
  NR_EPI_SCATTER_ZEROED = 10 /* NR_EPI_SCATTER_STORE whose destination rows are ZERO on entry (the
                            zero-filled table gradient): the large-tile kernel may split K over the
                            last partial round of its tiles and add those pieces atomically   */
};

/* GEMM arithmetic, chosen PER CALL (the `prec` argument of nr_gemm_f32 / nr_gemm_f32_dyn; the
 * library holds no precision state, so calls are re-entrant across threads and streams):
 *   NR_GEMM_F32     v_mfma_f32_32x32x2_f32: exact fp32 products, fp32 accumulation.
 *   NR_GEMM_BF16X6  each fp32 operand split into three bf16 terms (x = h + m + l to 2^-24 |x|) and
 *                   the six products of order >= 2^-16 (hh, hm, mh, hl, mm, lh) accumulated in fp32 on
 *                   v_mfma_f32_32x32x16_bf16 (16x the f32 MFMA rate): fp32-class accuracy (dropped
 *                   terms <= 3 * 2^-24 |a b|), 6 bf16 MFMAs per f32-equivalent.  128x128-tile fast
 *                   path (problems under 400 such tiles and ineligible operands run NR_GEMM_F32).
 *   NR_GEMM_BF16    bf16 arithmetic (autocast-style): fp32 operands rounded to bf16 (RNE) on their way
 *                   to LDS, ONE v_mfma_f32_32x32x16_bf16 product per tile and k-step, fp32
 *                   accumulation and fp32 outputs.  Ineligible operands run NR_GEMM_F32.
 * Storage stays fp32 in every mode (fp32 master weights). */
enum nr_gemm_precision { NR_GEMM_F32 = 0, NR_GEMM_BF16X6 = 1, NR_GEMM_BF16 = 2 };

/* C (op)= A(m,k) * B(k,n) over k in [0,K) in the arithmetic `prec` (enum nr_gemm_precision).
 * Replaces: nn.Linear / F.linear of models/Modules/Attention.py:107-108 (keyProject,
 * valueProject), CNN.py:23 (wordQueryProject is done in nr_attn_pool), the Conv1d of
 * CNN.py:12-17 (as a K = 3E GEMM over CONV3 rows) and their autograd backward.
 * split_k > 1 requires NR_EPI_ATOMIC or NR_EPI_SCATTER. */
int nr_gemm_f32(int64_t M, int64_t N, int64_t K, const nr_operand* A, const nr_operand* B,
                float* C, int64_t ldc, const float* bias, int32_t epilogue,
                const nr_operand* c_rows, int64_t pad_row, int32_t split_k, int32_t prec,
                hipStream_t stream);

/* nr_gemm_f32 with device-resident extents: M and K are host upper bounds (grid sizing) and
 * the kernel reads the actual values from m_dev / k_dev (either may be NULL), so a row count
 * produced on the GPU (nr_unique_rows) sizes the GEMM without a host synchronisation.
 * Fast-path operands only (16-B aligned, ld % 4 == 0); K and *k_dev multiples of 32. */
int nr_gemm_f32_dyn(int64_t M, int64_t N, int64_t K, const nr_operand* A, const nr_operand* B,
                    float* C, int64_t ldc, const float* bias, int32_t epilogue,
                    const nr_operand* c_rows, int64_t pad_row, int32_t split_k,
                    const int32_t* m_dev, const int32_t* k_dev, int32_t prec,
                    hipStream_t stream);

/* nr_gemm_f32_dyn whose persistent grid occupies at most max_cus CUs (0 = every CU), so that a
 * collective issued on another stream just before it (the data-parallel word-table all-reduce,
 * twotower.py:49-50's DDP bucket reduction) finds CUs to run on while the GEMM computes. */
int nr_gemm_f32_dyn_cus(int64_t M, int64_t N, int64_t K, const nr_operand* A, const nr_operand* B,
                        float* C, int64_t ldc, const float* bias, int32_t epilogue,
                        const nr_operand* c_rows, int64_t pad_row, int32_t split_k,
                        const int32_t* m_dev, const int32_t* k_dev, int32_t prec, int32_t max_cus,
                        hipStream_t stream);

/* nr_gemm_f32 / nr_gemm_f32_dyn_cus with a caller-owned workspace (m_dev, k_dev NULL and max_cus 0:
 * the static form).  When a split-K NR_EPI_ATOMIC contraction runs on the 256 x 256 kernel and
 * `work` (16-B aligned, work_elems floats) holds its partial tiles, every split stores its partial
 * tile with plain stores and one reduction launch adds the splits into C in split order
 * (deterministic) -- instead of fp32 atomics.  Likewise an NR_EPI_SCATTER_ZEROED bf16x6 contraction
 * on that kernel (the distinct-row table dgrad, nn.Embedding's backward through BERT.py:39): the K
 * pieces of its last partial round of tiles (the stream-K tail) store plain partial tiles there and
 * one reduction adds each tile's pieces in piece order into its destination rows, instead of fp32
 * atomics into the zeroed rows.  Any other call ignores `work`.
 * nr_gemm_splitk_workspace() elements always suffice.  Measured: without colsum this path is
 * slower than the atomic epilogue on the NRMS weight gradient (292-301 vs 277 µs) and equal on
 * BERT's; it pays when it also carries the bias gradient (below).
 * colsum (device, [M], may be NULL; then colsum_folded may be NULL too): a weight gradient's bias
 * gradient, colsum[m] += Σ_k A[k][m] for an MN-contiguous A (A = dY stored [K][M]).  On that path
 * the units of the first column tile sum the A tiles they load anyway and the reduction adds the
 * per-split sums: *colsum_folded (host) = 1.  Otherwise *colsum_folded = 0 and colsum is left
 * alone -- the caller reduces it (nr_colsum). */
int nr_gemm_f32_ws(int64_t M, int64_t N, int64_t K, const nr_operand* A, const nr_operand* B, float* C,
                   int64_t ldc, const float* bias, int32_t epilogue, const nr_operand* c_rows,
                   int64_t pad_row, int32_t split_k, const int32_t* m_dev, const int32_t* k_dev,
                   int32_t prec, int32_t max_cus, float* work, int64_t work_elems, float* colsum,
                   int32_t* colsum_folded, hipStream_t stream);
/* floats of split-K workspace that serve any nr_gemm_f32_ws call on the current device */
int64_t nr_gemm_splitk_workspace(void);

/* ------------------------------------------------------------------ distinct token rows */

/* Distinct ids of a token batch (the news tower projects each word-table row once, not once
 * per token: BERT.py:39 + Attention.py:107-108 commute with the gather).  Outputs:
 *   uids[U_pad]      distinct ids ascending, padded with fill_row up to U_pad = ceil32(U)
 *   inv[T]           uids[inv[t]] == ids[t]
 *   seg_off[U_pad+1], seg_tok[T], seg_of[T]   CSR of the tokens of each distinct id whose
 *                    grad_mask is nonzero (grad_mask NULL: every token); seg_of[p] = the
 *                    distinct row owning CSR position p.  Leave a token out only when its
 *                    gradient row is zero (masked tokens of nr_mha_pool_bwd: exactly zero).
 *   counts[4]        {U, U_pad, bad, T_csr} (bad = 1 if an id fell outside [0, V))
 * Equal ids are aggregated per workgroup (LDS hash) before the global atomics; three launches
 * (count, scan, fill), four above 65,536 ids (the scan's tile totals in a pass of their own).
 * work: nr_unique_rows_workspace(V) int32 (4 + 4*ceil4(V) + 2*ceil(V/4096)), 16-B aligned, all zero
 * before the first call; every call leaves its flag word and counters zero again (the fill pass
 * clears them: no zero-fill launch), so one buffer serves every call on a stream, one call at a time.
 * Capacity: uids / seg_off hold ceil32(min(T, V)) (+1) entries. */
int nr_unique_rows(const int64_t* ids, int64_t T, int64_t V, int64_t fill_row,
                   const void* grad_mask, int32_t mask_dtype, int32_t* work, int64_t* uids,
                   int64_t* inv, int32_t* seg_off, int32_t* seg_tok, int32_t* seg_of,
                   int32_t* counts, hipStream_t stream);
/* int32 elements of nr_unique_rows' work buffer for a vocabulary of V ids */
int64_t nr_unique_rows_workspace(int64_t V);

/* Bytes of `work` nr_segment_rows_sum needs for T tokens of `width` floats. */
int64_t nr_segment_rows_sum_workspace(int64_t T, int64_t width);

/* dst[u][:] = Σ_{t in segment u} src[t][:]  for u < counts[0] (zero for an empty segment),
 * zero rows up to counts[1]; the CSR holds counts[3] <= T positions.
 * The per-distinct-row gradient of the projection (what embedding_dense_backward sums after
 * the dgrad, summed before it).  No atomics.  width, lds, ldd multiples of 4; rows_max >=
 * counts[1]; src, dst, work 16-B aligned. */
int nr_segment_rows_sum(const float* src, int64_t lds, int64_t width, int64_t T,
                        const int32_t* seg_off, const int32_t* seg_tok, const int32_t* seg_of,
                        const int32_t* counts, int64_t rows_max, float* work, float* dst,
                        int64_t ldd, hipStream_t stream);

/* dst rows [V, width] whose id is absent from the batch of the last nr_unique_rows call on `work`
 * (and the pad row) set to zero; the present rows are left for the distinct-row scatter GEMM that
 * writes every one of them (nr_gemm_f32_ws NR_EPI_SCATTER_ZEROED with a workspace, bf16x6): the word
 * table's dense gradient (nn.Embedding backward, BERT.py:39) without a full zero fill.  counts: that
 * call's counts.  width % 4 == 0, dst 16-B aligned.  flags (nullable, uint8 [V]): 1 for a present row,
 * 0 for a zeroed one -- the per-row flags nr_adam_multi's row_touched reads to skip zero rows. */
int nr_unique_rows_zero_absent(const int32_t* work, const int32_t* counts, int64_t V, int64_t pad_row, float* dst,
                               int64_t ldd, int64_t width, uint8_t* flags, hipStream_t stream);

/* nr_segment_rows_sum for the segments of two or more tokens only: a one-token segment's dst row is
 * left as it is (its producer wrote it there: nr_mha_pool_bwd with seg_off).  Same arguments,
 * workspace and alignment rules as nr_segment_rows_sum. */
int nr_segment_rows_sum_multi(const float* src, int64_t lds, int64_t width, int64_t T, const int32_t* seg_off,
                              const int32_t* seg_tok, const int32_t* seg_of, const int32_t* counts,
                              int64_t rows_max, float* work, float* dst, int64_t ldd, hipStream_t stream);

/* The CNN encoder's k = 3 convolution per distinct row (CNN.py:41, Conv1d(E -> H, k = 3, pad = 1)).
 * nr_segment_rows_sum_conv3: dst[u][tap*tap_width + c] = sum over the CSR tokens t of distinct row u
 * of src[t + 1 - tap][c] for tap in {0, 1, 2}, zero when t + 1 - tap leaves t's title of L tokens
 * (the CSR must hold every token: nr_unique_rows with grad_mask NULL).  The per-distinct-row input of
 * both the table dgrad (dtable[u] = dst[u] . W3) and the conv wgrad (dW3 = dstᵀ table[uids]).
 * Workspace: nr_segment_rows_sum_workspace(T, 3 * tap_width).  Same alignment rules as above. */
int nr_segment_rows_sum_conv3(const float* src, int64_t lds, int64_t tap_width, int32_t L, int64_t T,
                              const int32_t* seg_off, const int32_t* seg_tok, const int32_t* seg_of,
                              const int32_t* counts, int64_t rows_max, float* work, float* dst,
                              int64_t ldd, hipStream_t stream);

/* out[t][h] = act(bias[h] + sum_{tap} P[inv[t + tap - 1]][tap*tap_width + h]) for h < H (taps outside
 * t's title of L tokens skipped; act = ReLU when relu != 0), out[t][h] = 0 for H <= h < tap_width.
 * P = the per-distinct-row tap projections [U][3 * tap_width] (one GEMM over distinct rows).
 * tap_width, ldp, ldo multiples of 4; P, out 16-B aligned. */
int nr_conv3_rows_fwd(const float* P, int64_t ldp, int32_t tap_width, int32_t H, const int64_t* inv,
                      int64_t T, int32_t L, const float* bias, int32_t relu, float* out, int64_t ldo,
                      hipStream_t stream);

/* The distinct-row CNN encoder's weight operands in one launch: w3t [3*Hp][E] (row tap*Hp + h =
 * conv_w[h][:][tap], the Conv1d weight [H][E][3]; rows h >= H zero), wqp [Hp][Hp] and bqp [Hp] (the
 * key projection zero-padded); optional w3tt [E][3*Hp] = w3t transposed (the K-contiguous weight
 * operand of the table dgrad; NULL: not written).  nr_cnn_unpack_grads maps the gradients of those
 * operands back to the parameters' layouts (dconv_w [H][E][3], dwq [H][H], dbq [H]; stored, not
 * accumulated). */
int nr_cnn_pack_weights(const float* conv_w, const float* wq, const float* bq, int32_t H, int32_t E,
                        int32_t Hp, float* w3t, float* wqp, float* bqp, float* w3tt, hipStream_t stream);
int nr_cnn_unpack_grads(const float* dw3t, const float* dwqp, const float* dbqp, int32_t H, int32_t E,
                        int32_t Hp, float* dconv_w, float* dwq, float* dbq, hipStream_t stream);

/* CNN_Encoder's word attention head fused per title (models/Encoders/CNN.py:44-46 with
 * scaled_dp_attention, Modules/Attention.py:5-30, over the conv output C of CNN.py:41-42):
 * K = tanh(C wqᵀ + bq), s_l = scale q·K_l, p = XSoftmax(s, mask), news = Σ_l p_l C_l.  The key
 * projection reaches HBM only through kout.  C [nseq*L][Hp] (ldc % 4 == 0, 16-B aligned, exactly zero past the
 * valid width), wq [Hp][Hp] / bq [Hp] zero-padded (nr_cnn_pack_weights), q [qn]; Hp a multiple of
 * 32 up to 160, L <= 32.  prec: enum nr_gemm_precision of the key products.  news [nseq][Hp]
 * (ldn >= Hp), probs [nseq*L].  kout (optional, [nseq*L][ldk >= Hp], ldk % 4 == 0, 16-B aligned,
 * L * ldk * 4 < 2^31): K
 * stored for the backward (which then skips the key recompute); NULL keeps the key projection on chip. */
int nr_cnn_keypool_fwd(const float* C, int64_t ldc, const float* wq, const float* bq, const float* q, int32_t qn,
                       const void* mask, int32_t mask_dtype, int64_t nseq, int32_t L, int32_t Hp, float scale,
                       int32_t prec, float* news, int64_t ldn, float* probs, float* kout, int64_t ldk,
                       hipStream_t stream);
/* Backward of nr_cnn_keypool_fwd in one pass over C (the key projection read from kin or recomputed): dc [nseq*L][Hp] =
 * ReLU'(C) ⊙ (p dnews + dK wq + dz) (the conv pre-activation gradient; dz optional, [T][>= H]),
 * dK = ds q ⊙ (1 - K²); dwq [Hp][Hp] = Σ dKᵀ C, dbq [Hp] = Σ dK, dq [qn] = Σ ds K, dconv_b [H] =
 * Σ_t dc[t] -- all STORED (not accumulated), summed deterministically over per-workgroup partials in
 * ws (nr_cnn_keypool_workspace(nseq, Hp) floats).  kin (optional): the forward's kout -- K is read
 * instead of recomputed.  Replaces the reference's autograd through CNN.py:46 + Attention.py:22-29
 * and the ReLU of CNN.py:42. */
int64_t nr_cnn_keypool_workspace(int64_t nseq, int32_t Hp);
int nr_cnn_keypool_bwd(const float* C, int64_t ldc, const float* wq, const float* bq, const float* q, int32_t qn,
                       int64_t nseq, int32_t L, int32_t Hp, int32_t H, float scale, int32_t prec,
                       const float* probs, const float* dnews, int64_t lddn, const float* dz, int64_t lddz,
                       float* dc, int64_t lddc, float* dwq, float* dbq, float* dq, float* dconv_b, float* ws,
                       int64_t ws_floats, const float* kin, int64_t ldk, hipStream_t stream);

/* ------------------------------------------------------------------ attention */

/* Tied-QK multi-head self attention core, one sequence of L <= 64 tokens per (seq, head):
 * out[s*L+i][h*dv:(h+1)*dv] = Σ_j XSoftmax(qk_i·qk_j * scale, m_i m_j) v_j.
 * Replaces MultiheadAttention.forward after the projections (models/Modules/Attention.py:
 * 125-147), get_attn_mask (:33-53) and XSoftmax.forward (:66-74).  (dk, dv) in
 * {(64,32),(32,32),(64,64),(64,16),(16,16)} for L <= 32, {(32,32),(64,64),(16,16),(64,32)}
 * for L <= 64.  mask: [nseq, L] of enum nr_mask_dtype (0=u8, 1=i64, 2=f64, 3=f32).
 * rows (optional): token s*L+j reads qk / v row rows[s*L+j] (projections computed once per
 * distinct row, e.g. the fast-eval news table, and gathered inside the kernel). */
int nr_mha_attn_fwd(const float* qk, int64_t ld_qk, const float* v, int64_t ld_v,
                    const int64_t* rows, const void* mask, int32_t mask_dtype, int64_t nseq, int32_t L,
                    int32_t heads, int32_t dk, int32_t dv, float scale, float* out,
                    int64_t ld_out, hipStream_t stream);

/* Eval-time MHA user encoder + its pooling in one launch (MHA_User_Encoder.forward, models/Encoders/
 * MHA.py:58-75, with Attention_Pooling, Pooling.py:12-25), for the fast eval's history read through
 * per-news projections (TwoTowerBaseModel.predict_fast :78-83 over Manager._eval_fast's news table):
 *   O_s = MultiheadAttention core of sequence s (as nr_mha_attn_fwd: tied key, pairwise mask,
 *         heads concatenated) over rows y[yrows[s*L + j]] = [key proj (heads*dk) | value proj (heads*dv)],
 *   out[s] = Σ_l XSoftmax(q · O_{s,l} / sqrt(heads*dv), m)_l O_{s,l}.
 * One workgroup per sequence, the attention products on the matrix cores in `prec` (nr_gemm_precision
 * values; bf16x6 = fp32-class).  L <= 64; (dk, dv, heads*dv) in {(32,32,384), (64,32,384), (64,64,768)};
 * y_rows = rows of y (y_rows * ldy * 4 < 2^32); yrows NULL = identity.  No autograd (eval only). */
int nr_mha_user_pool_fwd(const float* y, int64_t ldy, int64_t y_rows, const int64_t* yrows, const void* mask,
                         int32_t mask_dtype, int64_t nseq, int32_t L, int32_t heads, int32_t dk, int32_t dv,
                         const float* q, float* out, int64_t ldo, int32_t prec, hipStream_t stream);

/* Backward of nr_mha_attn_fwd (XSoftmax.backward, Attention.py:77-80, and the two matmuls);
 * recomputes P.  dqk receives the gradient of the shared key projection (both roles).
 * dbias_k [heads*dk] / dbias_v [heads*dv] (both or neither; device): the projection bias gradient
 * (keyProject / valueProject bias, Attention.py:107-108) ATOMICALLY ACCUMULATED as the column sums of
 * dqk / dv_out over the nseq*L rows (caller zeroes) -- the separate column-sum pass folded in. */
int nr_mha_attn_bwd(const float* qk, int64_t ld_qk, const float* v, int64_t ld_v,
                    const void* mask, int32_t mask_dtype, int64_t nseq, int32_t L,
                    int32_t heads, int32_t dk, int32_t dv, float scale, const float* dout,
                    int64_t ld_dout, float* dqk, int64_t ld_dqk, float* dv_out, int64_t ld_dv,
                    float* dbias_k, float* dbias_v, hipStream_t stream);

/* Fused MHA news-encoder tail, one workgroup per title (L <= 32): for each head the tied-QK
 * attention on the f32 MFMA (S = Kp Kpᵀ / sqrt(dk), XSoftmax with m_i m_j, O = P Vp), then
 * LayerNorm (eps) -> dropout(p, counter RNG) -> learned-query pooling, all in LDS.
 * y = [T][heads*dk | heads*dv] projections.  (dk, dv, heads*dv) in {(64,32,384), (64,64,768),
 * (64,32,256), (32,32,384)}.  Replaces MultiheadAttention.forward :125-147 + MHA.py:37-38.
 * Saves stats [T][2] and probs [T]; zout (optional) receives Z = the encoder's token output;
 * oout (optional, ldo >= heads*dv) receives O, the attention output before the LayerNorm
 * (training: lets nr_mha_pool_bwd skip the attention recompute).
 * yrows (optional): token t reads projection row yrows[t] (distinct-row projections).
 * rng (optional, all dropout entries): the dropout key comes from the device pair
 * (rng[0], rng[1] + offset) instead of (seed, offset), so a replayed graph draws new masks.
 * prec (enum nr_gemm_precision, fwd and bwd): the arithmetic of the attention products (S = K Kᵀ,
 * O = P V and their backward) -- NR_GEMM_F32 exact fp32 MFMA products, NR_GEMM_BF16X6 the
 * fp32-class six-product bf16 form in the forward and exact fp32 products in the backward (faster
 * there), NR_GEMM_BF16 one bf16 product; softmax, LayerNorm and pooling stay fp32 in every mode. */
int nr_mha_pool_fwd(const float* y, int64_t ldy, const int64_t* yrows, const void* mask,
                    int32_t mask_dtype, int64_t nseq,
                    int32_t L, int32_t heads, int32_t dk, int32_t dv, const float* gamma,
                    const float* beta, float eps, float p_drop, uint64_t seed, uint64_t offset,
                    const uint64_t* rng, const float* q, float* news, int64_t ldn, float* zout,
                    int64_t ldz, float* oout, int64_t ldo, float* stats, float* probs,
                    int32_t prec, hipStream_t stream);

/* Backward of nr_mha_pool_fwd: writes dy [T][heads*(dk+dv)] and ATOMICALLY ACCUMULATES dbias
 * (= column sums of dy), dq, dgamma, dbeta (caller zeroes).  dy stays per token (row t) when
 * yrows is given; rows of masked tokens are exactly zero.  With o (the forward's oout) and dob the
 * backward runs split: a per-title pooling/LN pass writes each token's LayerNorm-backward row terms
 * into dob [T][lddob >= 8] (caller's workspace, 16-B aligned, lddob % 4 == 0), then a per-(title, head)
 * attention pass at high occupancy rebuilds its head's slice of dO from o and those terms (dO never
 * goes through HBM); with o and dob NULL one
 * fused kernel per title loads the saved O, keeps dO in LDS and runs every head's attention
 * backward; without o the fused kernel recomputes the attention.
 * ws (optional, forms with o only): ws_copies x ceil4(3*heads*dv + heads*(dk+dv)) floats, ZERO on entry
 * and left zero on return -- workgroups spread their dgamma / dbeta / dq / dbias atomics over the
 * copies (one address per title would serialise them at L2) and a last kernel adds the copy sums
 * into the outputs.
 * dy rows are addressed by 32-bit byte offsets: dy_rows (rows of the dy buffer, >= nseq*L) *
 * lddy * 4 < 2^32.  seg_off (optional; with yrows): the CSR offsets of nr_unique_rows over the
 * gradient-carrying tokens -- a token alone in its distinct row's segment writes its gradient row
 * straight to dy row dyu_row0 + yrows[t] (the per-distinct-row sum, which nr_segment_rows_sum_multi
 * then skips), a masked token writes nothing; dsto: [nseq*L] uint32 scratch (the split form's LN
 * pass stores each token's row offset there for the attention pass). */
int nr_mha_pool_bwd(const float* y, int64_t ldy, const int64_t* yrows, const void* mask,
                    int32_t mask_dtype, int64_t nseq,
                    int32_t L, int32_t heads, int32_t dk, int32_t dv, const float* gamma,
                    const float* beta, float p_drop, uint64_t seed, uint64_t offset,
                    const uint64_t* rng, const float* q, const float* stats, const float* probs,
                    const float* dnews,
                    int64_t ldn, const float* dz, int64_t lddz, const float* o, int64_t ldo,
                    float* dob, int64_t lddob, float* dy, int64_t lddy,
                    float* dbias, float* dq, float* dgamma, float* dbeta, float* ws,
                    int32_t ws_copies, const int32_t* seg_off, int64_t dyu_row0, int64_t dy_rows,
                    uint32_t* dsto, int32_t prec, hipStream_t stream);

/* ------------------------------------------------------------------ pooling */

/* Learned-query attention pooling of nseq sequences of L <= 64 rows of D features:
 *   Z = Dropout_p(LayerNorm(X))  (gamma == NULL: no LN; p_drop == 0: no dropout)
 *   out[s] = Σ_l XSoftmax(scale * q·K_l, mask)_l Z_l,   K = key rows, or Z when key == NULL
 * Replaces MHA_Encoder.forward :37-38 (LN eps, dropout with a stateless (seed, offset)
 * counter RNG), MHA_User_Encoder :72, Attention_Pooling.forward (Pooling.py:22-24) and the
 * pooling of CNN_Encoder (CNN.py:46, key = tanh(W c + b) from nr_gemm_f32).
 * Saves stats [nseq*L][2] (mean, rstd; LN only) and probs [nseq*L] for the backward;
 * zout (optional) receives Z, the encoder's per-token output. */
int nr_attn_pool_fwd(const float* x, int64_t ldx, const float* key, int64_t ldk, const float* q,
                     const void* mask, int32_t mask_dtype, const float* gamma, const float* beta,
                     float eps, float p_drop, uint64_t seed, uint64_t offset, const uint64_t* rng,
                     int64_t nseq, int32_t L, int32_t D, float scale, float* out, int64_t ldo,
                     float* zout,
                     int64_t ldz, float* stats, float* probs, hipStream_t stream);

/* Backward of nr_attn_pool_fwd (dz: optional upstream grad of Z, added to the pooling's):
 * writes dx (through dropout and LN) and dk (key != NULL;
 * multiplied by 1 - K² when key_tanh), and ATOMICALLY ACCUMULATES dq[D], dgamma[D],
 * dbeta[D] (caller zeroes them). */
int nr_attn_pool_bwd(const float* x, int64_t ldx, const float* key, int64_t ldk, const float* q,
                     const void* mask, int32_t mask_dtype, const float* gamma, const float* beta,
                     float p_drop, uint64_t seed, uint64_t offset, const uint64_t* rng,
                     int64_t nseq, int32_t L, int32_t D, float scale, const float* stats,
                     const float* probs,
                     const float* dout, int64_t lddo, const float* dz, int64_t lddz, float* dx,
                     int64_t lddx, float* dk, int64_t lddk, int32_t key_tanh, float* dq,
                     float* dgamma, float* dbeta, hipStream_t stream);

/* Learned-query pooling without LayerNorm / dropout, one wave per sequence (rows as coalesced float4
 * segments, per-row dot products as wave reductions, no LDS staging), or one workgroup per sequence
 * (rows split over its 8 waves) for D > 256 or fewer than 1024 sequences:
 *   out[s] = Σ_l XSoftmax(scale * q·K_l, mask)_l X_l,  K = key rows, or X when key == NULL.
 * Replaces CNN_Encoder's pooling (CNN.py:46, key = tanh(W c + b)) and Attention_Pooling
 * (Pooling.py:22-24).  D <= 1024, L <= 64; the row matrices (x, key, out, dx, dk, dz) 16-B aligned with
 * ld % 4 == 0 and ld >= D; q (and each dout row) hold qn <= D valid floats, any alignment, features
 * past qn taken as zero (a zero-padded row width D > qn then pools exact zeros there).  Saves
 * probs [nseq*L]. */
int nr_seq_pool_fwd(const float* x, int64_t ldx, const float* key, int64_t ldk, const float* q, int32_t qn,
                    const void* mask, int32_t mask_dtype, int64_t nseq, int32_t L, int32_t D, float scale,
                    float* out, int64_t ldo, float* probs, hipStream_t stream);

/* Backward of nr_seq_pool_fwd: dx = p dout (+ ds q when tied) (+ dz), dk = ds q (* (1 - K²) when
 * key_tanh) for a separate key; ATOMICALLY ACCUMULATES dq[0 .. qn) (one add per feature per
 * workgroup). */
int nr_seq_pool_bwd(const float* x, int64_t ldx, const float* key, int64_t ldk, const float* q, int32_t qn,
                    const void* mask, int32_t mask_dtype, int64_t nseq, int32_t L, int32_t D, float scale,
                    const float* probs, const float* dout, int64_t lddo, const float* dz, int64_t lddz,
                    float* dx, int64_t lddx, float* dk, int64_t lddk, int32_t key_tanh, float* dq,
                    hipStream_t stream);

/* ------------------------------------------------------------------ recurrent user encoders */

enum nr_cell { NR_CELL_LSTM = 0, NR_CELL_GRU = 1 };

/* Sequential part of a one-layer LSTM/GRU over B sequences of N steps (RNN.py:50-73 with
 * pack_padded_sequence semantics: len = count of nonzero mask[b, :], output h at step
 * len-1; mask == NULL: len = N, as LSTUR, RNN.py:100-104).  gx = x W_ihᵀ + b_ih for all
 * steps [B*N][G*H] (G = 4 LSTM, 3 GRU), whh_t = W_hhᵀ [H][G*H].  reverse: step t reads row
 * N-1-t (flip(dims=[1])).  h0 rows: h0[h0_idx[b]] (or h0[b]; NULL = zeros), c0 = 0.
 * Saves gates [B*N][4H] (LSTM i,f,g,o / GRU r,z,n,W_hn h+b_hn), hprev, cprev (LSTM). */
int nr_rnn_fwd(int32_t cell, const float* gx, int64_t ldgx, const float* whh_t, const float* bhh,
               const float* h0, int64_t ldh0, const int64_t* h0_idx, const void* mask,
               int32_t mask_dtype, int32_t reverse, int64_t B, int32_t N, int32_t H,
               float* gates, float* hprev, float* cprev, float* hout, int64_t ldho,
               hipStream_t stream);

/* BPTT of nr_rnn_fwd.  Writes the pre-activation gate gradients of the input path dgi and
 * of the recurrent path dgh ([B*N][G*H]; equal for LSTM, dgh may be NULL then) and dh0. */
int nr_rnn_bwd(int32_t cell, const float* whh, const float* gates, const float* hprev,
               const float* cprev, const void* mask, int32_t mask_dtype, int32_t reverse,
               int64_t B, int32_t N, int32_t H, const float* dhout, int64_t lddho, float* dgi,
               float* dgh, int64_t lddg, float* dh0, int64_t lddh0, hipStream_t stream);

/* ------------------------------------------------------------------ scorer, optimizer, misc */

enum nr_score_mode { NR_SCORE_RAW = 0, NR_SCORE_LOG_SOFTMAX = 1, NR_SCORE_SIGMOID = 2 };

/* logits[b][c] = head(cdd_row(b,c) · user[b] / sqrt(H)); cdd_row = cdd[cdd_idx[b*C+c]]
 * (predict_fast's news-table gather, TwoTowerBaseModel.py:80) or cdd[b*C+c].
 * Replaces compute_score + log_softmax / sigmoid (TwoTowerBaseModel.py:51-75). */
int nr_score_fwd(const float* cdd, int64_t ldc, const int64_t* cdd_idx, const float* user,
                 int64_t ldu, int64_t B, int32_t C, int32_t H, int32_t mode, float* logits,
                 hipStream_t stream);

/* The training head with its loss: logits = log_softmax(cdd_row(b,c) · user[b] / sqrt(H)) as
 * nr_score_fwd (NR_SCORE_LOG_SOFTMAX) AND loss[0] = mean_b -logits[b][label[b]] -- Manager.py:641's
 * NLLLoss (torch.nn.NLLLoss() defaults: reduction 'mean', ignore_index -100) on
 * TwoTowerBaseModel.forward's output, in one launch (no separate loss kernels, no zero fill): one
 * workgroup per impression, the last to finish forms the mean over the labels in [0, C) in a fixed
 * order (labels -100 are ignored: no term, not counted; all ignored -> NaN, torch's 0/0).  A label
 * outside [0, C) other than -100 (torch raises) makes the loss NaN and sets work[1] to 1 -- a sticky
 * status the caller reads and clears itself.  work: nr_score_nll_workspace(B) int32,
 * all zero before the first call; every call leaves work[0] zero again (work[1] is the status, the
 * rest scratch), so one buffer serves every call on a stream.  Calls on one buffer must not run
 * concurrently. */
int nr_score_nll_fwd(const float* cdd, int64_t ldc, const float* user, int64_t ldu,
                     const int64_t* label, int64_t B, int32_t C, int32_t H, float* logits, float* loss,
                     int32_t* work, hipStream_t stream);
/* int32 elements of nr_score_nll_fwd's work buffer for B impressions */
int64_t nr_score_nll_workspace(int64_t B);

/* Backward of nr_score_nll_fwd: the gradient of the loss (dloss, a device scalar, or NULL; spread
 * over the labels in [0, C) as 1/count each) plus an optional gradient of the logits themselves
 * (dlogits [B][C] or NULL). */
int nr_score_nll_bwd(const float* cdd, int64_t ldc, const float* user, int64_t ldu,
                     const float* logits, const int64_t* label, const float* dloss,
                     const float* dlogits, int64_t B, int32_t C, int32_t H, float* dcdd, int64_t lddc,
                     float* duser, int64_t lddu, hipStream_t stream);

/* Backward of nr_score_fwd (cdd_idx == NULL form) given dlogits [B][C]. */
int nr_score_bwd(const float* cdd, int64_t ldc, const float* user, int64_t ldu,
                 const float* logits, const float* dlogits, int64_t B, int32_t C, int32_t H,
                 int32_t mode, float* dcdd, int64_t lddc, float* duser, int64_t lddu,
                 hipStream_t stream);

/* One torch.optim.Adam step (amsgrad=False) on n contiguous fp32 elements; `step` is the
 * 1-based step count after increment (bias corrections as torch).  The gradient is read as
 * grad * grad_scale (1/world_size folds the data-parallel mean into the update).  step_dev
 * (optional): the step count read on the device instead (graph replays).
 * Manager.py:404-413,647. */
int nr_adam(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n,
            float lr, float beta1, float beta2, float eps, float weight_decay, int64_t step,
            const int64_t* step_dev, float grad_scale, hipStream_t stream);

/* One torch.optim.Adam step over many tensors in as few launches as possible (<= 40 tensors per
 * launch, descriptors passed by value: graph-capturable).  Per tensor: contiguous fp32 param /
 * grad / exp_avg / exp_avg_sq of n elements, its group's lr (host `lr`, or `lr_dev` read on the
 * device: a replayed graph follows a learning-rate scheduler, Manager.py:415-420), and the step
 * count after increment (host `step`, or `step_dev` on the device).  Same arithmetic as nr_adam. */
typedef struct nr_adam_tensor {
  float* param;
  const float* grad;
  float* exp_avg;
  float* exp_avg_sq;
  int64_t n;
  float lr;
  int64_t step;
  const int64_t* step_dev;
  const float* lr_dev;
  /* optional: one byte per row of row_len elements, 0 = the row's gradient is all zero (a row-sparse
   * table gradient, e.g. LSTUR's user table): its gradient is not read (the update uses g = 0, the
   * same arithmetic as reading the zeros).  NULL: every element's gradient is read. */
  const uint8_t* row_touched;
  int64_t row_len;
} nr_adam_tensor;
int nr_adam_multi(const nr_adam_tensor* tensors, int32_t count, float beta1, float beta2, float eps,
                  float weight_decay, float grad_scale, hipStream_t stream);
/* nr_adam_multi whose launches also advance the device step counts (tensors with step_dev): each
 * tensor's bias correction uses *step_dev + 1 and the workgroup that finishes last adds 1 to every
 * step_dev of its launch (torch's `state_steps += 1` without a launch of its own).  ticket: one
 * int32, zero before the first call and left zero by every call. */
int nr_adam_multi_step(const nr_adam_tensor* tensors, int32_t count, float beta1, float beta2, float eps,
                       float weight_decay, float grad_scale, int32_t* ticket, hipStream_t stream);

/* out[i] = table[idx[i]] rows of E floats (E % 4 == 0).  BERT_Embedding.forward, BERT.py:39. */
int nr_embedding_fwd(const float* table, int64_t V, int64_t E, const int64_t* idx, int64_t n,
                     float* out, hipStream_t stream);

/* dtable[idx[i]] += dout[i] for idx[i] != padding_idx (atomic; dtable pre-zeroed):
 * embedding_dense_backward with nn.Embedding(padding_idx=0). */
int nr_embedding_bwd(const float* dout, int64_t V, int64_t E, const int64_t* idx, int64_t n,
                     int64_t padding_idx, float* dtable, hipStream_t stream);

/* dtable[idx[i]] += dout[i] (rows of E floats, leading dimensions ldo / ldt) for idx[i] != padding_idx,
 * the rows of each id summed in ascending i by one wave and added once: deterministic with duplicate
 * ids (no atomics).  For row-sparse gradients of few rows (n <= 2^20; O(n^2) id reads): LSTUR's user
 * table (embedding_dense_backward of userEmbedding, models/Encoders/RNN.py:100-104) on one process and
 * in the data-parallel row-sparse exchange (the DDP mean of twotower.py:49-50), so every rank forms
 * the same bits. */
int nr_rows_add_ordered(const float* dout, int64_t ldo, int64_t V, int64_t E, const int64_t* idx, int64_t n,
                        int64_t padding_idx, float* dtable, int64_t ldt, hipStream_t stream);

/* XSoftmax (models/Modules/Attention.py:56-80) over the last dimension: out = softmax of x's rows
 * with the entries whose mask (same [rows, cols] shape, enum nr_mask_dtype) is zero excluded, those
 * entries exactly 0, a fully masked row all 0.  Backward (_softmax_backward_data, Attention.py:77-80):
 * dx = y (dy - Σ_row dy y).  Contiguous [rows, cols] tensors, one wave per row. */
int nr_xsoftmax_fwd(const float* x, const void* mask, int32_t mask_dtype, int64_t rows, int64_t cols,
                    float* out, hipStream_t stream);
int nr_xsoftmax_bwd(const float* y, const float* dy, int64_t rows, int64_t cols, float* dx, hipStream_t stream);

/* dst[i][:] = src[idx[i]][:] for rows of `cols` floats (any width; leading dimensions lds / ldd): the
 * news-table rows of the fast-eval history slots (predict_fast's encode_user over the cached table,
 * TwoTowerBaseModel.py:78-83 / Manager.py:516). */
int nr_gather_rows_f32(const float* src, int64_t lds, int64_t V, const int64_t* idx, int64_t n, int64_t cols,
                       float* dst, int64_t ldd, hipStream_t stream);

/* dst[c][r] = src[r][c] for a [rows, cols] fp32 matrix (leading dimensions lds >= cols, ldd >= rows):
 * the NRMS table-gradient GEMM's k-contiguous copy of the joint [keyProject; valueProject] weight
 * (models/Modules/Attention.py:107-108), so both of its operands take the K-contiguous loaders. */
int nr_transpose_f32(const float* src, int64_t lds, int64_t rows, int64_t cols, float* dst, int64_t ldd,
                     hipStream_t stream);

/* out[c] += Σ_r x[r][c]  (bias gradients; out pre-zeroed or accumulated).  Deterministic two-pass
 * reduction (no atomics) through `work` of nr_colsum_workspace(rows, cols) bytes. */
int64_t nr_colsum_workspace(int64_t rows, int64_t cols);
int nr_colsum(const float* x, int64_t ldx, int64_t rows, int64_t cols, float* out, float* work,
              hipStream_t stream);
/* nr_colsum in one launch: the last workgroup to finish each 64-column chunk sums that chunk's
 * partial rows (fixed order: the same result as nr_colsum).  tick: ceil(cols / 64) int32 arrival
 * counters, zero before the first call and left zero by every call. */
int nr_colsum_ws(const float* x, int64_t ldx, int64_t rows, int64_t cols, float* out, float* work,
                 int32_t* tick, hipStream_t stream);

/* ---------------------------------------------------------------- device-side MIND data path
 * (csrc/mind_batch.hip).  The dataset lives in HBM as CSR arrays:
 *   tok, attn    [n_news, L] int32   encoded_news / attn_mask truncated to L columns with the
 *                                    last column forced to [SEP] (utils/MIND.py:103-108)
 *   his_off/ids  CSR of every impression's click history (behaviors.pkl "histories")
 *   neg_off/ids  CSR of every train impression's unclicked news ("negatives")
 *   imprs        [P, 2] int32 (impression index, clicked news) train samples ("imprs")
 *   uindex       [I] int32 user index per impression ("uindexes")
 * status: int32 word OR-ed with 1 (sample index out of range), 2 (news id out of range),
 * 4 (candidate row / user row out of range); the caller zeroes it and checks it when it wants. */
enum nr_batch_flags { NR_BATCH_REVERSE_HISTORY = 1, NR_BATCH_SHUFFLE_POS = 2, NR_BATCH_CURSOR = 4 };

/* One collated train batch of B impressions: MIND.__getitem__ train branch
 * (utils/MIND.py:311-365) with newsample (utils/utils.py:83-98) for every sample_idx[b] in [0, P),
 * then the DataLoader default collate.  Negatives: a uniform npratio-subset in uniform random
 * order drawn from the counter RNG (seed, offset [+ b * 4C + d]); or, when rng is non-null, from
 * the device words rng = {seed, offset, ticket, cursor, n_order}: the launch draws from (rng[0],
 * rng[1]) and advances rng[1] by B * 4C itself (the workgroup that finishes last, counted on
 * rng[2], which is zero on entry and left zero), so a replayed graph forms fresh batches with no
 * extra launch.  NR_BATCH_CURSOR (rng required): sample_idx is a whole epoch order of rng[4]
 * entries and batch b takes sample_idx[(rng[3] mod (rng[4] / B)) * B + b] (the sampler's
 * DistributedSampler order walked on the device); the last workgroup also adds 1 to rng[3].
 * Outputs (C = npratio + 1): cdd_id [B,C] i64, his_id [B,his_size]
 * i64, cdd_tok/cdd_attn [B,C,L] i64, his_tok/his_attn [B,his_size,L] i64, cdd_mask [B,C] f64,
 * his_mask [B,his_size] f64, user_id [B] i64, label [B] i64.  Replaces the Python
 * `random.sample` / `np.random.shuffle` streams (parity: structure exact, draws from this RNG). */
int nr_form_train_batch(const int64_t* sample_idx, int64_t B, const int32_t* imprs, int64_t P,
                        const int64_t* his_off, const int32_t* his_ids, const int64_t* neg_off,
                        const int32_t* neg_ids, const int32_t* uindex, const int32_t* tok,
                        const int32_t* attn, int64_t n_news, int32_t L, int32_t npratio,
                        int32_t his_size, int32_t flags, uint64_t seed, uint64_t offset,
                        uint64_t* rng, int64_t* cdd_id, int64_t* his_id, int64_t* cdd_tok,
                        int64_t* cdd_attn, int64_t* his_tok, int64_t* his_attn, double* cdd_mask,
                        double* his_mask, int64_t* user_id, int64_t* label, int32_t* status,
                        hipStream_t stream);

/* Device RNG pair bookkeeping for graph-replayed steps: snap = state (the (seed, offset) pair the
 * kernels of this forward/backward read), then state[1] += n (the elements the step's dropout
 * draws -- nn.Dropout's RNG consumption in MHA_Encoder / CNN_Encoder, models/Encoders/MHA.py:38,
 * CNN.py:44), in ONE launch (torch clone + add cost two).  snap may be null (advance only). */
int nr_rng_take(uint64_t* state, uint64_t* snap, uint64_t n, hipStream_t stream);

/* History side of B consecutive dev/test impression chunks chunk0 .. chunk0+B-1
 * (utils/MIND.py:367-449; chunk_impr[c] = impression of chunk c).  his_tok/his_attn may be null
 * (fast eval reads history representations from the news table instead).  impr_index[b] =
 * impression + 1 as the reference returns it. */
int nr_form_eval_batch(int64_t chunk0, int64_t B, const int32_t* chunk_impr, int64_t n_chunks,
                       const int64_t* his_off, const int32_t* his_ids, const int32_t* uindex,
                       const int32_t* tok, const int32_t* attn, int64_t n_news, int32_t L,
                       int32_t his_size, int32_t flags, int64_t* his_id, int64_t* his_tok,
                       int64_t* his_attn, double* his_mask, int64_t* user_id, int64_t* impr_index,
                       int32_t* status, hipStream_t stream);

/* out_tok[i, :] = tok[ids[i], :], out_attn likewise (int32 table -> int64 rows). */
int nr_gather_news_rows(const int64_t* ids, int64_t n, const int32_t* tok, const int32_t* attn,
                        int64_t n_news, int32_t L, int64_t* out_tok, int64_t* out_attn,
                        int32_t* status, hipStream_t stream);

/* predict_fast over a packed ragged candidate list (models/TwoTowerBaseModel.py:78-83):
 * out[c] = f(table[cand_ids[c]] . user[cand_seg[c] - seg_base] / sqrt(H)), f = sigmoid
 * (NR_SCORE_SIGMOID) or identity (NR_SCORE_RAW). */
int nr_score_ragged(const float* table, int64_t ldt, int64_t n_rows, const int64_t* cand_ids,
                    const int32_t* cand_seg, int64_t seg_base, int64_t n, const float* user,
                    int64_t ldu, int64_t n_users, int32_t H, int32_t mode, float* out,
                    int32_t* status, hipStream_t stream);

/* Per-impression ranking metrics of cal_metric (utils/Manager.py:1205-1273, 1276-1345) for G
 * groups preds/labels[grp_off[g] .. grp_off[g+1]): out [G, 2 + 2*nk] f64 =
 * {roc_auc, mrr, ndcg@ks[0..nk), hit@ks[0..nk)}; nk <= 8.  Ties in the score order follow a
 * stable argsort reversed (the later index ranks first).  flags[g]: NR_METRIC_ONE_CLASS (auc
 * undefined: sklearn raises), NR_METRIC_NONBINARY (labels outside {0,1}: auc undefined). */
enum nr_metric_flags { NR_METRIC_ONE_CLASS = 1, NR_METRIC_NONBINARY = 2 };
int nr_impression_metrics(const float* preds, const int32_t* labels, const int64_t* grp_off,
                          int64_t G, const int32_t* ks, int32_t nk, double* out, int32_t* flags,
                          hipStream_t stream);

/* ---------------------------------------------------------------- BERT towers (XFormer / PLM)
 * transformers BertModel as models/XFormer.py:68,94 and models/PLM.py:102,121 call it (token
 * type ids never passed: every token takes token_type_embeddings row 0).  The dense layers are
 * nr_gemm_f32 calls (QKV, attention output, intermediate with NR_EPI_STORE_GELU, output, pooler
 * with NR_EPI_STORE_TANH over the [CLS] rows); the entries below are the code between them.
 * H % 4 == 0, H <= 1024; rows are float4-aligned.  Dropout uses the counter RNG of the other
 * fused kernels ((seed, offset), or the device pair rng with offset added). */

/* out[s*L+l] = Dropout_p(LayerNorm_eps(word[ids[s*L+l]] + pos[l] + type0)); saves stats [T][2]
 * = (mean, rstd).  BertEmbeddings.forward.  status (optional): |= 2 on an id outside [0, V). */
int nr_bert_embed_fwd(const float* word, int64_t V, const float* pos, int64_t P, const float* type0,
                      const int64_t* ids, int64_t nseq, int32_t L, int32_t H, const float* gamma,
                      const float* beta, float eps, float p_drop, uint64_t seed, uint64_t offset,
                      const uint64_t* rng, float* out, int64_t ldo, float* stats, int32_t* status,
                      hipStream_t stream);

/* Backward of nr_bert_embed_fwd up to the LayerNorm input: ds [T][H] = dL/d(word+pos+type) (the
 * table gradients are then nr_embedding_bwd / nr_colsum of ds); ATOMICALLY ACCUMULATES dgamma,
 * dbeta (caller zeroes). */
int nr_bert_embed_bwd(const float* word, int64_t V, const float* pos, const float* type0,
                      const int64_t* ids, int64_t nseq, int32_t L, int32_t H, const float* gamma,
                      float p_drop, uint64_t seed, uint64_t offset, const uint64_t* rng,
                      const float* stats, const float* dout, int64_t ldd, float* ds, int64_t ldds,
                      float* dgamma, float* dbeta, hipStream_t stream);

/* out = LayerNorm_eps(Dropout_p(x) + res): BertSelfOutput / BertOutput (x = the dense output with
 * its bias).  Saves stats [T][2]. */
int nr_bert_add_ln_fwd(const float* x, int64_t ldx, const float* res, int64_t ldr, int64_t T, int32_t H,
                       const float* gamma, const float* beta, float eps, float p_drop, uint64_t seed,
                       uint64_t offset, const uint64_t* rng, float* out, int64_t ldo, float* stats,
                       hipStream_t stream);

/* Backward of nr_bert_add_ln_fwd (recomputes the LayerNorm input): dres = dL/dres (STORED),
 * dx = dL/dx (stored), dgamma / dbeta ATOMICALLY ACCUMULATED. */
int nr_bert_add_ln_bwd(const float* x, int64_t ldx, const float* res, int64_t ldr, int64_t T, int32_t H,
                       const float* gamma, float p_drop, uint64_t seed, uint64_t offset,
                       const uint64_t* rng, const float* stats, const float* dout, int64_t ldd,
                       float* dres, int64_t lddr, float* dx, int64_t lddx, float* dgamma, float* dbeta,
                       hipStream_t stream);

/* BertSelfAttention core for nseq sequences of L tokens (any L), heads of 64 dims:
 *   ctx[s*L+i][h*64:] = Σ_j Dropout_p(softmax_j(q_i·k_j / 8 + (1 - m_j) * FLT_MIN_NEG)) v_j
 * with q / k / v at columns h*64, koff + h*64, voff + h*64 of qkv rows (ld ldq).  Fully masked
 * rows are uniform over the L keys (the additive-mask arithmetic).  Saves ml [T][heads][2] =
 * (row max, 1 / row sum) for the backward.  mask: [nseq, L] of enum nr_mask_dtype.  prec (enum
 * nr_gemm_precision): the arithmetic of the four products (Q Kᵀ, P V and their backward) --
 * NR_GEMM_F32 the f32 MFMA, NR_GEMM_BF16X6 the fp32-class bf16 split form, NR_GEMM_BF16 one bf16
 * product; the softmax, its statistics and the dropout stay fp32.  Replaces the self-attention core
 * of transformers' BertSelfAttention.forward as models/XFormer.py:68,94 call it. */
int nr_bert_attn_fwd(const float* qkv, int64_t ldq, int64_t koff, int64_t voff, const void* mask,
                     int32_t mask_dtype, int64_t nseq, int32_t L, int32_t heads, float p_drop,
                     uint64_t seed, uint64_t offset, const uint64_t* rng, float* ctx, int64_t ldc,
                     float* ml, uint32_t* keep, int32_t prec, hipStream_t stream);

/* Words of the optional `keep` buffer of nr_bert_attn_fwd / _bwd: one 32-bit word per (sequence, head,
 * query, 32-key tile) holding the dropout keep bits of that query's probabilities (ceil(L / 32) words
 * per query).  The bf16-MFMA forward (prec != NR_GEMM_F32) with p_drop > 0 stores them; the backward
 * reads them instead of re-deriving each element's counter hash (the attention-probability dropout of
 * BertSelfAttention, models/XFormer.py:68,94).  NULL: the backward re-hashes (same masks). */
int64_t nr_bert_attn_keep_words(int64_t nseq, int32_t L, int32_t heads);

/* Bytes of `work` nr_bert_attn_bwd needs (16-B aligned): D = rowsum(dctx * ctx) per (query, head),
 * and for L > 96 (four-wave launches) the dS tiles the dK/dV kernel stores and the dQ kernel reads
 * (4096 * nseq * heads * ceil(L / 32)^2 bytes; unused by prec = NR_GEMM_F32). */
int64_t nr_bert_attn_bwd_workspace(int64_t nseq, int32_t L, int32_t heads);

/* Backward of nr_bert_attn_fwd: writes dQ, dK, dV into dqkv at the columns of qkv (every column
 * of the 3 * heads * 64 block is stored).  Deterministic (no atomics).  prec as in the forward
 * (the two may differ; ml is the forward's either way). */
int nr_bert_attn_bwd(const float* qkv, int64_t ldq, int64_t koff, int64_t voff, const void* mask,
                     int32_t mask_dtype, int64_t nseq, int32_t L, int32_t heads, float p_drop,
                     uint64_t seed, uint64_t offset, const uint64_t* rng, const float* ctx, int64_t ldc,
                     const float* ml, const uint32_t* keep, const float* dctx, int64_t ldd, float* work,
                     float* dqkv, int64_t lddq, int32_t prec, hipStream_t stream);

/* dx = dy * (1 - y^2): the pooler's tanh backward (BertPooler). */
int nr_tanh_bwd(const float* y, int64_t ldy, const float* dy, int64_t lddy, int64_t rows, int32_t cols,
                float* dx, int64_t lddx, hipStream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* NEWSREC_HIP_H */

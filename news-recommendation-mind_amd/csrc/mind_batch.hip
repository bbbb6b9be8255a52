// Device-side data path around the train/score step:
//   nr_form_train_batch    MIND.__getitem__ train branch (utils/MIND.py:311-365) + newsample
//                          (utils/utils.py:83-98) + the DataLoader's default collate, for a whole
//                          batch of impressions in one launch: news-id -> token-row gather from a
//                          device-resident token table, negative sampling on the device
//   nr_form_eval_batch     the history side of the dev/test branches (utils/MIND.py:367-449) for a
//                          contiguous range of impression chunks (the candidates of such a range
//                          are a contiguous slice of the packed candidate list: no gather needed)
//   nr_gather_news_rows    encoded_news[ids] / attn_mask[ids] (utils/MIND.py:340-343, 397-400)
//   nr_score_ragged        predict_fast (models/TwoTowerBaseModel.py:78-83) over a packed ragged
//                          candidate list: table row . user row / sqrt(H), sigmoid
//   nr_impression_metrics  cal_metric's per-impression terms (utils/Manager.py:1205-1273):
//                          roc_auc_score, mrr_score, ndcg_score@k, hit_score@k
//
// All of these are HBM/latency-bound integer and gather work: no MFMA, coalesced row copies,
// one workgroup per impression.
#include "common.h"
#include "../../include/newsrec_hip.h"

namespace {

// ---------------------------------------------------------------- counter-based sampling RNG
// draw d of impression slot b: a 32-bit splitmix64 output of (seed, offset + b * stride + d);
// uniform integer in [0, m) by the multiply-shift map (bias <= m / 2^32)
__device__ __forceinline__ uint32_t draw_below(uint64_t seed, uint64_t ctr, uint32_t m) {
  return (uint32_t)(((uint64_t)nr_dropout_key(seed, ctr) * (uint64_t)m) >> 32);
}

// history ids of impression `imp` into s_ids[0..his_size): the first his_size clicks
// (utils/MIND.py:327), reversed when `reverse` (descend_history, :339-342; the test branch
// inverts the flag, :433-436), right-padded with news 0; his_mask[:len] = 1, his_mask[0] = 1
// when the history is empty (:330-337)
// (threads t0, t0 + nt, ... of the workgroup take part)
__device__ void history_ids(const int64_t* his_off, const int32_t* his_ids, int64_t imp, int his_size,
                            bool reverse, int32_t* s_ids, double* his_mask_row, int t0 = 0, int nt = 0) {
  if (nt == 0) nt = blockDim.x;
  const int64_t h0 = his_off[imp];
  const int64_t full = his_off[imp + 1] - h0;
  const int hl = full < his_size ? (int)full : his_size;
  for (int j = (int)threadIdx.x - t0; j < his_size; j += nt) {
    int32_t id = 0;
    if (j < hl) id = his_ids[h0 + (reverse ? hl - 1 - j : j)];
    s_ids[j] = id;
    if (his_mask_row) his_mask_row[j] = (j < hl || (hl == 0 && j == 0)) ? 1.0 : 0.0;
  }
}

// token rows of the news in s_ids[0..rows) -> out_tok / out_attn (int64, [rows, L]); ids
// outside [0, n_news) read row 0 and set *status bit 1 (the table was validated on upload,
// so this only guards memory safety)
__device__ void gather_rows(const int32_t* s_ids, int rows, const int32_t* tok, const int32_t* attn,
                            int64_t n_news, int L, int64_t* out_tok, int64_t* out_attn, int32_t* status) {
  const int total = rows * L;
  for (int e = threadIdx.x; e < total; e += blockDim.x) {
    const int r = e / L, l = e - r * L;
    int64_t id = s_ids[r];
    if (id < 0 || id >= n_news) {
      if (status) atomicOr(status, 2);
      id = 0;
    }
    const int64_t src = id * L + l;
    out_tok[e] = tok[src];
    if (out_attn) out_attn[e] = attn[src];
  }
}

struct TrainArgs {
  const int64_t* sample_idx; int64_t B;
  const int32_t* imprs; int64_t P;
  const int64_t* his_off; const int32_t* his_ids;
  const int64_t* neg_off; const int32_t* neg_ids;
  const int32_t* uindex;
  const int32_t* tok; const int32_t* attn; int64_t n_news; int L;
  int npratio, his_size, flags;
  uint64_t seed, offset; uint64_t* rng;
  int64_t *cdd_id, *his_id, *cdd_tok, *cdd_attn, *his_tok, *his_attn;
  double *cdd_mask, *his_mask;
  int64_t *user_id, *label;
  int32_t* status;
};

// History rows per workgroup of form_train_kernel: an impression's 50 history titles go to five
// workgroups beside the one that samples its candidates, so no workgroup walks more than a short
// chain of dependent loads (sample index -> impression -> history offsets -> ids -> token rows) and one
// pass of its token-row gather (one workgroup per impression, every title in it: 15.6 us per B = 32
// batch, most of it the serial gather loop behind the sampling chain)
constexpr int FT_HIS_ROWS = 10;

__global__ __launch_bounds__(256) void form_train_kernel(TrainArgs a) {
  extern __shared__ int32_t s_mem[];
  const int C = a.npratio + 1, NH = a.his_size;
  int32_t* s_ids = s_mem;                 // [C] candidates, or this part's history rows
  int32_t* s_pick = s_mem + C + NH;       // [npratio] sampled negative positions
  int32_t* s_perm = s_pick + a.npratio;   // [C] shuffle_pos permutation
  int32_t* s_tmp = s_perm + C;            // [C]
  __shared__ int64_t s_imp;
  __shared__ int32_t s_neg_num, s_label, s_cand0;
  const int64_t b = blockIdx.x;
  const int part = (int)blockIdx.y;       // 0: candidates (+ user id, label); 1..: history rows
  uint64_t seed = a.seed, off = a.offset;
  if (a.rng) { seed = a.rng[0]; off = a.rng[1]; }
  const uint64_t ctr0 = off + (uint64_t)b * (uint64_t)(4 * C);

  if (threadIdx.x == 0) {
    int64_t sb = b;
    if (a.flags & NR_BATCH_CURSOR) {   // this launch's batch of the epoch order
      const uint64_t nb = a.rng[4] / (uint64_t)gridDim.x;
      sb += (int64_t)((nb > 0 ? a.rng[3] % nb : 0) * (uint64_t)gridDim.x);
    }
    int64_t idx = a.sample_idx[sb];
    if (idx < 0 || idx >= a.P) { if (part == 0) atomicOr(a.status, 1); idx = 0; }
    s_imp = a.imprs[2 * idx];
    s_cand0 = a.imprs[2 * idx + 1];
  }
  __syncthreads();
  if (part > 0) {
    // history rows [j0, j1) (utils/MIND.py:327-345)
    const int j0 = (part - 1) * FT_HIS_ROWS, j1 = j0 + FT_HIS_ROWS < NH ? j0 + FT_HIS_ROWS : NH;
    if (j0 < j1) {
      const int64_t imp = s_imp;
      const int64_t h0 = a.his_off[imp];
      const int64_t full = a.his_off[imp + 1] - h0;
      const int hl = full < NH ? (int)full : NH;
      const bool reverse = (a.flags & NR_BATCH_REVERSE_HISTORY) != 0;
      for (int j = j0 + (int)threadIdx.x; j < j1; j += blockDim.x) {
        int32_t id = 0;
        if (j < hl) id = a.his_ids[h0 + (reverse ? hl - 1 - j : j)];
        s_ids[j - j0] = id;
        a.his_mask[b * NH + j] = (j < hl || (hl == 0 && j == 0)) ? 1.0 : 0.0;
        a.his_id[b * NH + j] = id;
      }
      __syncthreads();
      gather_rows(s_ids, j1 - j0, a.tok, a.attn, a.n_news, a.L, a.his_tok + (b * NH + j0) * a.L,
                  a.his_attn ? a.his_attn + (b * NH + j0) * a.L : nullptr, a.status);
    }
  } else {
    if (threadIdx.x == 0) {
      s_ids[0] = s_cand0;
      const int64_t imp = s_imp;
      const int64_t nb = a.neg_off[imp];
      const int n = (int)(a.neg_off[imp + 1] - nb);
      const int k = a.npratio;
      if (k > n) {
        // newsample: fewer negatives than npratio -> all of them in order, then news 0 (utils.py:95-96)
        for (int i = 0; i < k; ++i) s_ids[1 + i] = i < n ? a.neg_ids[nb + i] : 0;
        s_neg_num = n;
      } else {
        // random.sample(negs, k): a uniform k-subset (Floyd), in uniform random order (Fisher-Yates)
        int d = 0;
        for (int j = n - k, m = 0; j < n; ++j, ++m) {
          const int t = (int)draw_below(seed, ctr0 + d++, (uint32_t)(j + 1));
          bool seen = false;
          for (int q = 0; q < m; ++q) seen |= s_pick[q] == t;
          s_pick[m] = seen ? j : t;
        }
        for (int i = k - 1; i > 0; --i) {
          const int r = (int)draw_below(seed, ctr0 + d++, (uint32_t)(i + 1));
          const int32_t tmp = s_pick[i]; s_pick[i] = s_pick[r]; s_pick[r] = tmp;
        }
        for (int i = 0; i < k; ++i) s_ids[1 + i] = a.neg_ids[nb + s_pick[i]];
        s_neg_num = k;
      }
      int lab = 0;
      if (a.flags & NR_BATCH_SHUFFLE_POS) {
        // np.random.shuffle(arange(C)); cdd_ids = cdd_ids[s]; label = position of the positive
        // (utils/MIND.py:319-324)
        for (int i = 0; i < C; ++i) s_perm[i] = i;
        for (int i = C - 1; i > 0; --i) {
          const int r = (int)draw_below(seed, ctr0 + 2 * k + (C - 1 - i), (uint32_t)(i + 1));
          const int32_t tmp = s_perm[i]; s_perm[i] = s_perm[r]; s_perm[r] = tmp;
        }
        for (int i = 0; i < C; ++i) s_tmp[i] = s_ids[i];
        for (int i = 0; i < C; ++i) s_ids[i] = s_tmp[s_perm[i]];
        for (int i = 0; i < C; ++i) if (s_perm[i] == 0) lab = i;
      }
      s_label = lab;
      a.user_id[b] = a.uindex[imp];
    }
    __syncthreads();
    for (int i = threadIdx.x; i < C; i += blockDim.x) {
      a.cdd_id[b * C + i] = s_ids[i];
      a.cdd_mask[b * C + i] = i < s_neg_num + 1 ? 1.0 : 0.0;
    }
    if (threadIdx.x == 0) a.label[b] = s_label;
    gather_rows(s_ids, C, a.tok, a.attn, a.n_news, a.L, a.cdd_tok + b * C * a.L,
                a.cdd_attn ? a.cdd_attn + b * C * a.L : nullptr, a.status);
  }
  if (a.rng) {
    // every workgroup has read (rng[0], rng[1], rng[3]) above; the last one to get here advances the
    // offset (and the cursor) for the next launch and resets the ticket
    __syncthreads();
    if (threadIdx.x == 0) {
      const unsigned long long t = atomicAdd(reinterpret_cast<unsigned long long*>(a.rng + 2), 1ull);
      if (t == (unsigned long long)gridDim.x * gridDim.y - 1) {
        atomicAdd(reinterpret_cast<unsigned long long*>(a.rng + 1), (unsigned long long)(4 * C) * gridDim.x);
        if (a.flags & NR_BATCH_CURSOR) atomicAdd(reinterpret_cast<unsigned long long*>(a.rng + 3), 1ull);
        __hip_atomic_store(a.rng + 2, (uint64_t)0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
}

struct EvalArgs {
  int64_t chunk0, B;
  const int32_t* chunk_impr; int64_t n_chunks;
  const int64_t* his_off; const int32_t* his_ids;
  const int32_t* uindex;
  const int32_t* tok; const int32_t* attn; int64_t n_news; int L;
  int his_size, flags;
  int64_t *his_id, *his_tok, *his_attn;
  double* his_mask;
  int64_t *user_id, *impr_index;
  int32_t* status;
};

__global__ __launch_bounds__(256) void form_eval_kernel(EvalArgs a) {
  extern __shared__ int32_t s_mem[];
  const int64_t b = blockIdx.x;
  const int NH = a.his_size;
  int64_t c = a.chunk0 + b;
  if (c >= a.n_chunks) {
    if (threadIdx.x == 0) atomicOr(a.status, 1);
    c = 0;
  }
  const int64_t imp = a.chunk_impr[c];
  history_ids(a.his_off, a.his_ids, imp, NH, (a.flags & NR_BATCH_REVERSE_HISTORY) != 0, s_mem,
              a.his_mask + b * NH);
  __syncthreads();
  for (int j = threadIdx.x; j < NH; j += blockDim.x) a.his_id[b * NH + j] = s_mem[j];
  if (threadIdx.x == 0) {
    a.user_id[b] = a.uindex[imp];
    a.impr_index[b] = imp + 1;   // "impr_index": impr_index + 1 (utils/MIND.py:403)
  }
  if (a.his_tok)
    gather_rows(s_mem, NH, a.tok, a.attn, a.n_news, a.L, a.his_tok + b * NH * a.L,
                a.his_attn ? a.his_attn + b * NH * a.L : nullptr, a.status);
}

// one workgroup per 256 / L rows (at least one row): ids -> int64 token / mask rows
__global__ __launch_bounds__(256) void gather_news_kernel(const int64_t* ids, int64_t n, const int32_t* tok,
                                                          const int32_t* attn, int64_t n_news, int L,
                                                          int64_t* out_tok, int64_t* out_attn, int32_t* status) {
  const int64_t total = n * L;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = e / L, l = e - r * L;
    int64_t id = ids[r];
    if (id < 0 || id >= n_news) {
      atomicOr(status, 2);
      id = 0;
    }
    out_tok[e] = tok[id * L + l];
    if (out_attn) out_attn[e] = attn[id * L + l];
  }
}

// one wave per candidate: float4 row loads, DPP wave sum; out = s / sqrt(H) (raw) or sigmoid
__global__ __launch_bounds__(256) void score_ragged_kernel(const float* table, int64_t ldt, int64_t n_rows,
                                                           const int64_t* cand_ids, const int32_t* cand_seg,
                                                           int64_t seg_base, int64_t n, const float* user,
                                                           int64_t ldu, int64_t n_users, int H, bool vec4,
                                                           float scale, int mode, float* out, int32_t* status) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t c = wave; c < n; c += nwaves) {
    int64_t row = cand_ids[c];
    int64_t u = (int64_t)cand_seg[c] - seg_base;
    if (row < 0 || row >= n_rows || u < 0 || u >= n_users) {
      if (lane == 0) atomicOr(status, 4);
      row = row < 0 || row >= n_rows ? 0 : row;
      u = u < 0 || u >= n_users ? 0 : u;
    }
    const float* x = table + row * ldt;
    const float* y = user + u * ldu;
    float s = 0.f;
    if (vec4) {
      for (int d = lane * 4; d < H; d += 256) {
        const float4 xv = *reinterpret_cast<const float4*>(x + d);
        const float4 yv = *reinterpret_cast<const float4*>(y + d);
        s = fmaf(xv.x, yv.x, s); s = fmaf(xv.y, yv.y, s); s = fmaf(xv.z, yv.z, s); s = fmaf(xv.w, yv.w, s);
      }
    } else {
      for (int d = lane; d < H; d += 64) s = fmaf(x[d], y[d], s);
    }
    s = nr_wave_sum(s) * scale;
    if (lane == 0) out[c] = mode == NR_SCORE_SIGMOID ? 1.f / (1.f + __expf(-s)) : s;
  }
}

// ---------------------------------------------------------------- per-impression metrics
#define NR_METRIC_MAX_K 8

template <typename T>
__device__ __forceinline__ T wave_sum_t(T v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// One WAVE per impression group (MIND dev impressions average ~37 candidates: a 256-thread
// block per group left most lanes idle and paid a block barrier per group).  Lane l owns
// candidates l, l+64, ...; the O(n^2) rank counts read the group's scores / labels straight
// from global memory (wave-uniform addresses: one broadcast load per j, L1/L2 resident).
// Ranks follow np.argsort(score)[::-1] with a stable ascending sort: descending score, ties
// broken toward the LATER index (numpy's default sort kind is not stable on SIMD builds, so the
// reference's own tie order is machine-dependent).
__global__ __launch_bounds__(256) void metrics_kernel(const float* preds, const int32_t* labels,
                                                      const int64_t* grp_off, int64_t G, const int32_t* ks,
                                                      int nk, double* out, int32_t* flags) {
  const int lane = threadIdx.x & 63;
  const int64_t g = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (g >= G) return;
  const int64_t o0 = grp_off[g];
  const int n = (int)(grp_off[g + 1] - o0);
  const float* P = preds + o0;
  const int32_t* Y = labels + o0;
  int kk[NR_METRIC_MAX_K];
  for (int q = 0; q < nk; ++q) kk[q] = ks[q] < n ? ks[q] : n;
  double mrr = 0.0, ysum = 0.0;
  double dcg[NR_METRIC_MAX_K], idcg[NR_METRIC_MAX_K], hit[NR_METRIC_MAX_K];
  for (int q = 0; q < NR_METRIC_MAX_K; ++q) { dcg[q] = 0.0; idcg[q] = 0.0; hit[q] = 0.0; }
  unsigned long long auc2 = 0, npos = 0, nneg = 0, nonbin = 0;
  for (int i0 = 0; i0 < n; i0 += 64) {
    const int i = i0 + lane;
    const bool live = i < n;
    const float pi = live ? P[i] : 0.f;
    const int32_t yi = live ? Y[i] : 0;
    int rs = 0, ry = 0;
    unsigned long long a2 = 0;
    for (int j = 0; j < n; ++j) {
      const float pj = P[j];
      const int32_t yj = Y[j];
      rs += (pj > pi) | ((pj == pi) & (j > i));
      ry += (yj > yi) | ((yj == yi) & (j > i));
      a2 += (yi == 1 && yj == 0) ? ((pi > pj) ? 2u : (pi == pj ? 1u : 0u)) : 0u;
    }
    if (!live) continue;
    auc2 += a2;
    npos += yi == 1;
    nneg += yi == 0;
    nonbin += (yi != 0 && yi != 1);
    ysum += (double)yi;
    mrr += (double)yi / (double)(rs + 1);
    const double gain = exp2((double)yi) - 1.0;
    for (int q = 0; q < nk; ++q) {
      if (rs < kk[q]) dcg[q] += gain / log2((double)(rs + 2));
      if (ry < kk[q]) idcg[q] += gain / log2((double)(ry + 2));
      if (yi == 1 && rs < ks[q]) hit[q] = 1.0;
    }
  }
  mrr = wave_sum_t(mrr); ysum = wave_sum_t(ysum);
  auc2 = wave_sum_t(auc2); npos = wave_sum_t(npos); nneg = wave_sum_t(nneg); nonbin = wave_sum_t(nonbin);
  for (int q = 0; q < nk; ++q) { dcg[q] = wave_sum_t(dcg[q]); idcg[q] = wave_sum_t(idcg[q]); hit[q] = wave_sum_t(hit[q]); }
  if (lane == 0) {
    const int W = 2 + 2 * nk;
    double* o = out + g * W;
    int32_t f = 0;
    const double nanv = __builtin_nan("");
    if (nonbin) f |= NR_METRIC_NONBINARY;
    if (npos == 0 || nneg == 0) f |= NR_METRIC_ONE_CLASS;
    o[0] = (f & (NR_METRIC_NONBINARY | NR_METRIC_ONE_CLASS)) ? nanv
           : (double)auc2 / (2.0 * (double)npos * (double)nneg);
    o[1] = mrr / ysum;                                    // 0 / 0 -> nan as numpy
    for (int q = 0; q < nk; ++q) {
      o[2 + q] = dcg[q] / idcg[q];
      o[2 + nk + q] = hit[q] > 0.0 ? 1.0 : 0.0;
    }
    flags[g] = f;
  }
}

}  // namespace

extern "C" int nr_form_train_batch(const int64_t* sample_idx, int64_t B, const int32_t* imprs, int64_t P,
                                   const int64_t* his_off, const int32_t* his_ids, const int64_t* neg_off,
                                   const int32_t* neg_ids, const int32_t* uindex, const int32_t* tok,
                                   const int32_t* attn, int64_t n_news, int32_t L, int32_t npratio,
                                   int32_t his_size, int32_t flags, uint64_t seed, uint64_t offset,
                                   uint64_t* rng, int64_t* cdd_id, int64_t* his_id, int64_t* cdd_tok,
                                   int64_t* cdd_attn, int64_t* his_tok, int64_t* his_attn, double* cdd_mask,
                                   double* his_mask, int64_t* user_id, int64_t* label, int32_t* status,
                                   hipStream_t stream) {
  if (B < 0 || P < 1 || n_news < 1 || L < 1 || npratio < 0 || his_size < 1) return NR_EINVAL(0);
  if (!sample_idx || !imprs || !his_off || !his_ids || !neg_off || !uindex || !tok || !status) return NR_EINVAL(1);
  if (!cdd_id || !his_id || !cdd_tok || !his_tok || !cdd_mask || !his_mask || !user_id || !label)
    return NR_EINVAL(2);
  if (npratio > 0 && !neg_ids) return NR_EINVAL(3);
  if ((flags & NR_BATCH_CURSOR) && !rng) return NR_EINVAL(5);
  if (B == 0) return NR_OK;
  TrainArgs a{sample_idx, B, imprs, P, his_off, his_ids, neg_off, neg_ids, uindex, tok, attn, n_news, L,
              npratio, his_size, flags, seed, offset, rng, cdd_id, his_id, cdd_tok, cdd_attn, his_tok,
              his_attn, cdd_mask, his_mask, user_id, label, status};
  const int C = npratio + 1;
  const size_t smem = (size_t)(C + his_size + npratio + 2 * C) * sizeof(int32_t);
  if (smem > 60 * 1024) return NR_EINVAL(4);
  const unsigned parts = 1u + (unsigned)((his_size + FT_HIS_ROWS - 1) / FT_HIS_ROWS);
  hipLaunchKernelGGL(form_train_kernel, dim3((unsigned)B, parts), dim3(256), smem, stream, a);
  NR_LAUNCH_CHECK();
  return NR_OK;
}

extern "C" int nr_form_eval_batch(int64_t chunk0, int64_t B, const int32_t* chunk_impr, int64_t n_chunks,
                                  const int64_t* his_off, const int32_t* his_ids, const int32_t* uindex,
                                  const int32_t* tok, const int32_t* attn, int64_t n_news, int32_t L,
                                  int32_t his_size, int32_t flags, int64_t* his_id, int64_t* his_tok,
                                  int64_t* his_attn, double* his_mask, int64_t* user_id, int64_t* impr_index,
                                  int32_t* status, hipStream_t stream) {
  if (B < 0 || chunk0 < 0 || n_chunks < 0 || n_news < 1 || L < 1 || his_size < 1) return NR_EINVAL(0);
  if (!chunk_impr || !his_off || !his_ids || !uindex || !status) return NR_EINVAL(1);
  if (!his_id || !his_mask || !user_id || !impr_index) return NR_EINVAL(2);
  if (his_tok && !tok) return NR_EINVAL(3);
  if (chunk0 + B > n_chunks) return NR_EINVAL(4);
  if (B == 0) return NR_OK;
  EvalArgs a{chunk0, B, chunk_impr, n_chunks, his_off, his_ids, uindex, tok, attn, n_news, L, his_size, flags,
             his_id, his_tok, his_attn, his_mask, user_id, impr_index, status};
  hipLaunchKernelGGL(form_eval_kernel, dim3((unsigned)B), dim3(256), (size_t)his_size * sizeof(int32_t), stream, a);
  NR_LAUNCH_CHECK();
  return NR_OK;
}

extern "C" int nr_gather_news_rows(const int64_t* ids, int64_t n, const int32_t* tok, const int32_t* attn,
                                   int64_t n_news, int32_t L, int64_t* out_tok, int64_t* out_attn,
                                   int32_t* status, hipStream_t stream) {
  if (n < 0 || n_news < 1 || L < 1) return NR_EINVAL(0);
  if (!ids || !tok || !out_tok || !status || (out_attn && !attn)) return NR_EINVAL(1);
  if (n == 0) return NR_OK;
  const int64_t total = n * L;
  const int64_t blocks = (total + 255) / 256 < 65536 ? (total + 255) / 256 : 65536;
  hipLaunchKernelGGL(gather_news_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, ids, n, tok, attn, n_news,
                     L, out_tok, out_attn, status);
  NR_LAUNCH_CHECK();
  return NR_OK;
}

extern "C" int nr_score_ragged(const float* table, int64_t ldt, int64_t n_rows, const int64_t* cand_ids,
                               const int32_t* cand_seg, int64_t seg_base, int64_t n, const float* user,
                               int64_t ldu, int64_t n_users, int32_t H, int32_t mode, float* out, int32_t* status,
                               hipStream_t stream) {
  if (n < 0 || n_rows < 1 || n_users < 1 || H < 1 || ldt < H || ldu < H) return NR_EINVAL(0);
  if (mode != NR_SCORE_RAW && mode != NR_SCORE_SIGMOID) return NR_EINVAL(1);
  if (!table || !cand_ids || !cand_seg || !user || !out || !status) return NR_EINVAL(2);
  if (n == 0) return NR_OK;
  const bool vec4 = (H % 4 == 0) && (ldt % 4 == 0) && (ldu % 4 == 0) && ((uintptr_t)table % 16 == 0) &&
                    ((uintptr_t)user % 16 == 0);
  const int64_t waves = n < 8192 * 4 ? n : 8192 * 4;
  const unsigned blocks = (unsigned)((waves + 3) / 4);
  hipLaunchKernelGGL(score_ragged_kernel, dim3(blocks), dim3(256), 0, stream, table, ldt, n_rows, cand_ids,
                     cand_seg, seg_base, n, user, ldu, n_users, H, vec4, 1.0f / sqrtf((float)H), mode, out,
                     status);
  NR_LAUNCH_CHECK();
  return NR_OK;
}

extern "C" int nr_impression_metrics(const float* preds, const int32_t* labels, const int64_t* grp_off, int64_t G,
                                     const int32_t* ks, int32_t nk, double* out, int32_t* flags,
                                     hipStream_t stream) {
  if (G < 0 || nk < 0 || nk > NR_METRIC_MAX_K) return NR_EINVAL(0);
  if (!preds || !labels || !grp_off || !out || !flags || (nk > 0 && !ks)) return NR_EINVAL(1);
  if (G == 0) return NR_OK;
  if ((G + 3) / 4 > 0x7FFFFFFF) return NR_EINVAL(2);
  hipLaunchKernelGGL(metrics_kernel, dim3((unsigned)((G + 3) / 4)), dim3(256), 0, stream, preds, labels, grp_off, G, ks, nk,
                     out, flags);
  NR_LAUNCH_CHECK();
  return NR_OK;
}

namespace {
__global__ void rng_take_kernel(uint64_t* state, uint64_t* snap, uint64_t n) {
  if (threadIdx.x != 0) return;
  const uint64_t seed = state[0], off = state[1];
  if (snap) {
    snap[0] = seed;
    snap[1] = off;
  }
  state[1] = off + n;
}
}  // namespace

extern "C" int nr_rng_take(uint64_t* state, uint64_t* snap, uint64_t n, hipStream_t stream) {
  if (!state) return NR_EINVAL(0);
  hipLaunchKernelGGL(rng_take_kernel, dim3(1), dim3(64), 0, stream, state, snap, n);
  NR_LAUNCH_CHECK();
  return NR_OK;
}

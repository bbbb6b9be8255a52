// Distinct-row compaction of a token batch, and the matching segment sum.
//
// The news tower's first layer is a per-token linear map of word-table rows, so it only has
// to run once per DISTINCT token id of the batch: Y[t] = (table[u] Wᵀ + b) at u = id[t].  A
// MIND batch holds far fewer distinct ids than tokens (padding and frequent words repeat), so
// the projection GEMM, its table-gradient GEMM and its weight-gradient GEMM all shrink from T
// rows to U (U <= min(T, V)).  The backward needs dY summed per distinct id (the segment sum
// below) — the same sums embedding_dense_backward forms (reference: BERT.py:39 through
// nn.Embedding), taken before the GEMM instead of after it.
//
// nr_unique_rows  : ids[T] -> uids[U_pad] (ascending), inv[T] (uids[inv[t]] == ids[t]),
//                   CSR seg_off[U_pad + 1] / seg_tok[T] of the tokens of each distinct id,
//                   counts = {U, U_pad}; U_pad = U rounded up to 32 (pad entries = fill_row,
//                   empty segments).  Sizes stay on the device: no host synchronisation.
// nr_segment_rows_sum : dst[u] = sum over t in segment u of src[t]   (zero for pad rows);
//                   two passes over the CSR, no atomics: ranges of 64 positions, then the
//                   segments cut by a range boundary (a long padding segment spans many).
#include "common.h"
#include "../../include/newsrec_hip.h"

namespace {

constexpr int SCAN_THREADS = 1024;
constexpr int SEG_RANGE = 64;   // CSR positions per segment-sum workgroup

// Tokens equal to the hot id (the padding row: most of a padded title batch) are counted per
// workgroup (ballot popcounts into LDS, one global atomic per block) — same-address global
// atomics serialise at one L2 channel, ~825 of them took ~25 us.
constexpr int CNT_THREADS = 1024;

__global__ __launch_bounds__(CNT_THREADS) void count_kernel(const int64_t* __restrict__ ids, int64_t T, int64_t V,
                                                            int64_t hot, int32_t* __restrict__ cnt,
                                                            int32_t* __restrict__ counts) {
  __shared__ int32_t hot_n;
  if (threadIdx.x == 0) hot_n = 0;
  __syncthreads();
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t v = t < T ? ids[t] : -1;
  const bool bad = t < T && (v < 0 || v >= V);
  if (bad) counts[2] = 1;   // out-of-range id: flagged, token dropped
  const uint64_t hb = __ballot(t < T && v == hot);
  if (hb && (threadIdx.x & 63) == __builtin_ctzll(hb)) atomicAdd(&hot_n, __builtin_popcountll(hb));
  if (t < T && !bad && v != hot) atomicAdd(&cnt[v], 1);
  __syncthreads();
  if (threadIdx.x == 0 && hot_n) atomicAdd(&cnt[hot], hot_n);
}

// Inclusive wave scan (Hillis-Steele over the 64 lanes).
__device__ __forceinline__ int32_t wave_scan_incl(int32_t x) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int32_t y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  return x;
}

// One workgroup walks the vocabulary in coalesced tiles of 4 x 1024 entries (4 consecutive per
// thread): exclusive scans of (cnt[v] > 0) -> pos[v] and of cnt[v] -> off[v], and the
// compaction uids[pos[v]] = v, seg_off[pos[v]] = off[v].
__global__ __launch_bounds__(SCAN_THREADS) void scan_kernel(const int32_t* __restrict__ cnt, int64_t V,
                                                            int32_t* __restrict__ pos, int32_t* __restrict__ off,
                                                            int64_t* __restrict__ uids, int32_t* __restrict__ seg_off,
                                                            int32_t* __restrict__ counts, int64_t fill_row) {
  __shared__ int32_t wu[SCAN_THREADS / 64], wc[SCAN_THREADS / 64];
  __shared__ int32_t carry[2];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  if (tid == 0) carry[0] = carry[1] = 0;
  __syncthreads();
  for (int64_t base = 0; base < V; base += 4 * SCAN_THREADS) {
    const int64_t v0 = base + 4 * tid;
    int32_t c[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) c[k] = v0 + k < V ? cnt[v0 + k] : 0;
    int32_t fu = 0, fc = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) { fu += c[k] > 0; fc += c[k]; }
    const int32_t iu = wave_scan_incl(fu), ic = wave_scan_incl(fc);
    if (lane == 63) { wu[w] = iu; wc[w] = ic; }
    __syncthreads();
    int32_t pu = carry[0], pc = carry[1];
    for (int k = 0; k < w; ++k) { pu += wu[k]; pc += wc[k]; }
    pu += iu - fu;   // exclusive
    pc += ic - fc;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int64_t v = v0 + k;
      if (v < V) {
        pos[v] = pu;
        off[v] = pc;
        if (c[k] > 0) {
          uids[pu] = v;
          seg_off[pu] = pc;
        }
      }
      pu += c[k] > 0;
      pc += c[k];
    }
    __syncthreads();
    if (tid == SCAN_THREADS - 1) { carry[0] = pu; carry[1] = pc; }
    __syncthreads();
  }
  if (tid == 0) {
    const int32_t U = carry[0], Tv = carry[1];
    const int32_t Up = (U + 31) / 32 * 32;
    counts[0] = U;
    counts[1] = Up;
    for (int32_t u = U; u < Up; ++u) {
      uids[u] = fill_row;
      seg_off[u] = Tv;
    }
    seg_off[Up] = Tv;
  }
}

// CSR fill: token t goes to a slot of its id's segment; seg_of[p] = the distinct row of CSR
// position p.  Hot-id tokens take consecutive slots: wave offsets from an LDS scan, one global
// atomic per workgroup.
__global__ __launch_bounds__(CNT_THREADS) void fill_kernel(const int64_t* __restrict__ ids, int64_t T, int64_t V,
                                                           int64_t hot, const int32_t* __restrict__ pos,
                                                           const int32_t* __restrict__ off,
                                                           int32_t* __restrict__ cursor, int64_t* __restrict__ inv,
                                                           int32_t* __restrict__ seg_tok,
                                                           int32_t* __restrict__ seg_of) {
  __shared__ int32_t wn[CNT_THREADS / 64];
  __shared__ int32_t hot_base;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t v = t < T ? ids[t] : -1;
  const bool ok = t < T && v >= 0 && v < V;
  if (t < T && !ok) inv[t] = 0;
  const uint64_t hb = __ballot(ok && v == hot);
  if (lane == 0) wn[w] = __builtin_popcountll(hb);
  __syncthreads();
  if (threadIdx.x == 0) {
    int32_t n = 0;
    for (int k = 0; k < CNT_THREADS / 64; ++k) n += wn[k];
    hot_base = n ? atomicAdd(&cursor[hot], n) : 0;
  }
  __syncthreads();
  int32_t slot = 0;
  if (ok && v == hot) {
    int32_t before = 0;
    for (int k = 0; k < w; ++k) before += wn[k];
    slot = hot_base + before + __builtin_popcountll(hb & ((1ull << lane) - 1));
  }
  if (!ok) return;
  if (v != hot) slot = atomicAdd(&cursor[v], 1);
  const int32_t u = pos[v];
  const int32_t p = off[v] + slot;
  inv[t] = u;
  seg_tok[p] = (int32_t)t;
  seg_of[p] = u;
}

// Segment sum, pass 1: workgroup b sums the CSR positions [b*R, (b+1)*R) piece by piece (a
// piece = the part of one segment inside the range).  Whole segments are stored to dst; a
// segment cut by a range boundary leaves its pieces in part[b][slot] (slot 0: the block's
// first piece, slot 1: a later one) for pass 2.  The piece table is built once in LDS; the
// sum loop per (piece, float4 column) has no branches and 4 loads in flight.
__global__ __launch_bounds__(256) void segsum_pieces_kernel(const float* __restrict__ src, int64_t lds, int64_t w4,
                                                            const int32_t* __restrict__ seg_off,
                                                            const int32_t* __restrict__ seg_tok,
                                                            const int32_t* __restrict__ seg_of, int64_t T,
                                                            float4* __restrict__ part, float* __restrict__ dst,
                                                            int64_t ldd) {
  const int64_t b = blockIdx.x, p0 = b * SEG_RANGE;
  const int64_t p1 = p0 + SEG_RANGE < T ? p0 + SEG_RANGE : T;
  const int n = (int)(p1 - p0);
  __shared__ int32_t s_tok[SEG_RANGE], s_seg[SEG_RANGE];
  __shared__ int32_t pc_beg[SEG_RANGE + 1], pc_u[SEG_RANGE];
  __shared__ int64_t pc_dst[SEG_RANGE];   // float4 index of the piece's destination
  __shared__ int32_t npieces;
  const int tid = threadIdx.x;
  if (tid < n) {
    s_tok[tid] = seg_tok[p0 + tid];
    s_seg[tid] = seg_of[p0 + tid];
  }
  __syncthreads();
  if (tid < 64) {   // one wave: piece starts = positions whose segment differs from the previous
    const bool start = tid < n && (tid == 0 || s_seg[tid] != s_seg[tid - 1]);
    const uint64_t sb = __ballot(start);
    if (start) {
      const int k = __builtin_popcountll(sb & ((1ull << tid) - 1));
      const int32_t u = s_seg[tid];
      const int64_t gb = seg_off[u], ge = seg_off[u + 1];
      int64_t d;
      if (gb >= p0 && ge <= p1) d = u * (ldd / 4);                    // whole segment -> dst row
      else d = -1 - ((b * 2 + (gb > p0 ? 1 : 0)) * w4);               // cut -> part slot (encoded)
      pc_beg[k] = tid;
      pc_u[k] = u;
      pc_dst[k] = d;
    }
    if (tid == 0) {
      const int np = __builtin_popcountll(sb);
      npieces = np;
      pc_beg[np] = n;
    }
  }
  __syncthreads();
  const int np = npieces;
  float4* dst4 = reinterpret_cast<float4*>(dst);
  for (int k = 0; k < np; ++k) {
    const int i0 = pc_beg[k], i1 = pc_beg[k + 1];
    const int64_t d = pc_dst[k];
    float4* out = d >= 0 ? dst4 + d : part + (-1 - d);
    for (int64_t j = tid; j < w4; j += blockDim.x) {
      float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
      int i = i0;
      for (; i + 4 <= i1; i += 4) {
        const float4 x0 = reinterpret_cast<const float4*>(src + (int64_t)s_tok[i] * lds)[j];
        const float4 x1 = reinterpret_cast<const float4*>(src + (int64_t)s_tok[i + 1] * lds)[j];
        const float4 x2 = reinterpret_cast<const float4*>(src + (int64_t)s_tok[i + 2] * lds)[j];
        const float4 x3 = reinterpret_cast<const float4*>(src + (int64_t)s_tok[i + 3] * lds)[j];
        s.x += x0.x; s.y += x0.y; s.z += x0.z; s.w += x0.w;
        s.x += x1.x; s.y += x1.y; s.z += x1.z; s.w += x1.w;
        s.x += x2.x; s.y += x2.y; s.z += x2.z; s.w += x2.w;
        s.x += x3.x; s.y += x3.y; s.z += x3.z; s.w += x3.w;
      }
      for (; i < i1; ++i) {
        const float4 x = reinterpret_cast<const float4*>(src + (int64_t)s_tok[i] * lds)[j];
        s.x += x.x; s.y += x.y; s.z += x.z; s.w += x.w;
      }
      out[j] = s;
    }
  }
}

// Pass 2, one workgroup per distinct row: a cut segment sums its pieces in range order (the
// long padding segment: hundreds of pieces, split over thread groups then combined in LDS);
// pad rows [U, U_pad) are zeroed; whole segments were written by pass 1.
constexpr int FIX_THREADS = 1024;

__global__ __launch_bounds__(FIX_THREADS) void segsum_fix_kernel(int64_t w4, const int32_t* __restrict__ seg_off,
                                                                 const int32_t* __restrict__ counts,
                                                                 const float4* __restrict__ part,
                                                                 float* __restrict__ dst, int64_t ldd) {
  __shared__ float4 acc_s[FIX_THREADS];
  const int64_t u = blockIdx.x;
  const int32_t U = counts[0], Up = counts[1];
  if (u >= Up) return;
  float4* drow = reinterpret_cast<float4*>(dst + u * ldd);
  if (u >= U) {
    for (int64_t j = threadIdx.x; j < w4; j += blockDim.x) drow[j] = make_float4(0.f, 0.f, 0.f, 0.f);
    return;
  }
  const int64_t sb = seg_off[u], se = seg_off[u + 1];
  const int64_t b0 = sb / SEG_RANGE, b1 = (se - 1) / SEG_RANGE;
  if (b0 == b1) return;
  // groups of w4 threads each take every G-th piece; w4 > FIX_THREADS: one group, column loop
  const int G = w4 <= FIX_THREADS ? (int)(FIX_THREADS / w4) : 1;
  const int g = (int)(threadIdx.x / (w4 < FIX_THREADS ? w4 : FIX_THREADS));
  const int64_t j0 = threadIdx.x - (int64_t)g * (w4 < FIX_THREADS ? w4 : FIX_THREADS);
  for (int64_t jb = 0; jb < w4; jb += FIX_THREADS) {
    const int64_t j = jb + j0;
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    if (g < G && j < w4) {
      for (int64_t b = b0 + g; b <= b1; b += G) {
        const int slot = (b == b0 && sb > b0 * SEG_RANGE) ? 1 : 0;
        const float4 x = part[(b * 2 + slot) * w4 + j];
        s.x += x.x; s.y += x.y; s.z += x.z; s.w += x.w;
      }
    }
    if (G > 1) {
      acc_s[threadIdx.x] = s;
      __syncthreads();
      if (g == 0 && j < w4) {
        for (int k = 1; k < G; ++k) {
          const float4 x = acc_s[k * w4 + j0];
          s.x += x.x; s.y += x.y; s.z += x.z; s.w += x.w;
        }
        drow[j] = s;
      }
      __syncthreads();
    } else if (j < w4) {
      drow[j] = s;
    }
  }
}

}  // namespace

extern "C" int nr_unique_rows(const int64_t* ids, int64_t T, int64_t V, int64_t fill_row, int32_t* work,
                              int64_t* uids, int64_t* inv, int32_t* seg_off, int32_t* seg_tok, int32_t* seg_of,
                              int32_t* counts, hipStream_t stream) {
  if (T < 0 || V < 1 || V > 0x7fffffff || T > 0x7fffffff) return NR_EINVAL(0);
  if (!ids || !work || !uids || !inv || !seg_off || !seg_tok || !seg_of || !counts) return NR_EINVAL(1);
  if (fill_row < 0 || fill_row >= V) return NR_EINVAL(2);
  int32_t* cnt = work;
  int32_t* cursor = work + V;
  int32_t* pos = work + 2 * V;
  int32_t* off = work + 3 * V;
  hipError_t e = hipMemsetAsync(work, 0, sizeof(int32_t) * 2 * V, stream);
  if (e != hipSuccess) return -(int)e;
  e = hipMemsetAsync(counts, 0, sizeof(int32_t) * 3, stream);
  if (e != hipSuccess) return -(int)e;
  const unsigned gb = (unsigned)((T + CNT_THREADS - 1) / CNT_THREADS);
  if (T > 0)
    hipLaunchKernelGGL(count_kernel, dim3(gb), dim3(CNT_THREADS), 0, stream, ids, T, V, fill_row, cnt, counts);
  hipLaunchKernelGGL(scan_kernel, dim3(1), dim3(SCAN_THREADS), 0, stream, cnt, V, pos, off, uids, seg_off, counts,
                     fill_row);
  if (T > 0)
    hipLaunchKernelGGL(fill_kernel, dim3(gb), dim3(CNT_THREADS), 0, stream, ids, T, V, fill_row, pos, off, cursor,
                       inv, seg_tok, seg_of);
  NR_LAUNCH_CHECK();
  return NR_OK;
}

extern "C" int64_t nr_segment_rows_sum_workspace(int64_t T, int64_t width) {
  return ((T + SEG_RANGE - 1) / SEG_RANGE) * 2 * width * (int64_t)sizeof(float);
}

extern "C" int nr_segment_rows_sum(const float* src, int64_t lds, int64_t width, int64_t T, const int32_t* seg_off,
                                   const int32_t* seg_tok, const int32_t* seg_of, const int32_t* counts,
                                   int64_t rows_max, float* work, float* dst, int64_t ldd, hipStream_t stream) {
  if (width < 0 || (width & 3) || (lds & 3) || (ldd & 3) || rows_max < 0 || T < 0) return NR_EINVAL(0);
  if (!src || !seg_off || !seg_tok || !seg_of || !counts || !dst || (T > 0 && !work)) return NR_EINVAL(1);
  if ((reinterpret_cast<uintptr_t>(src) & 15) || (reinterpret_cast<uintptr_t>(dst) & 15) ||
      (reinterpret_cast<uintptr_t>(work) & 15))
    return NR_EINVAL(2);
  if (rows_max == 0 || width == 0) return NR_OK;
  const int64_t w4 = width / 4;
  if (T > 0)
    hipLaunchKernelGGL(segsum_pieces_kernel, dim3((unsigned)((T + SEG_RANGE - 1) / SEG_RANGE)), dim3(256), 0, stream,
                       src, lds, w4, seg_off, seg_tok, seg_of, T, reinterpret_cast<float4*>(work), dst, ldd);
  hipLaunchKernelGGL(segsum_fix_kernel, dim3((unsigned)rows_max), dim3(FIX_THREADS), 0, stream, w4, seg_off, counts,
                     reinterpret_cast<const float4*>(work), dst, ldd);
  NR_LAUNCH_CHECK();
  return NR_OK;
}

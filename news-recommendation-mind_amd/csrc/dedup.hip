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
//                   CSR seg_off[U_pad + 1] / seg_tok / seg_of of the tokens of each distinct
//                   id whose grad_mask is set (all tokens without a mask: masked-out tokens of
//                   the fused MHA tail receive an exactly-zero dY, so leaving them out of the
//                   sums changes nothing and drops the long padding segment),
//                   counts = {U, U_pad, bad, T_csr}; U_pad = U rounded up to 32 (pad entries =
//                   fill_row, empty segments).  Sizes stay on the device: no host sync.
// nr_segment_rows_sum : dst[u] = sum over t in segment u of src[t]   (zero for empty / pad
//                   rows); two passes over the CSR, no atomics: ranges of 64 positions, then
//                   the segments cut by a range boundary.
#include "common.h"
#include "../../include/newsrec_hip.h"

namespace {

constexpr int SEG_RANGE = 64;   // CSR positions per segment-sum workgroup
constexpr int SEG_BATCH = 8;   // row loads in flight per thread (16 measured equal: 1.4273 vs 1.4259 ms per NRMS step)
// tokens per count / fill workgroup: 512 -> 7.7 + 8.3 us for the bench batch, 1024: 8.4 + 8.9, 256: 9.0 +
// 9.8 (profiles/r05_ag_ab_count_fill_threads.json)
constexpr int CNT_THREADS = 512;
constexpr int HASH_BITS = 10;   // 2 slots per token
constexpr int HASH_SLOTS = 1 << HASH_BITS;
static_assert(HASH_SLOTS == 2 * CNT_THREADS, "hash table: two slots per token of the workgroup");

// Per-workgroup aggregation of equal ids: an open-addressing hash table in LDS (512 tokens ->
// 1024 slots) collects (id, count); one global atomic per distinct id of the block.  Frequent
// ids (padding, [CLS], [SEP]: once per title) would otherwise serialise thousands of
// same-address atomics at one L2 channel.  Returns the slot; `rank` = the token's arrival
// order among the block's tokens of that id counted in `hcnt` (unique, order not fixed).
__device__ __forceinline__ int hash_slot(int32_t* hkey, int32_t v) {
  uint32_t h = ((uint32_t)v * 0x9E3779B1u) >> (32 - HASH_BITS);
  for (;;) {
    const int32_t old = atomicCAS(&hkey[h], -1, v);
    if (old == -1 || old == v) return (int)h;
    h = (h + 1) & (HASH_SLOTS - 1);
  }
}

__device__ __forceinline__ bool grad_on(const void* gm, int dt, int64_t t) {
  return gm == nullptr || nr_mask_at(gm, dt, t);
}

// Workspace (nr_unique_rows_workspace): ctrl[4] | cnt_all[V] | cnt_csr[V] | cursor[V] | pos[V] | tot[2 nb].
// ctrl, cnt_all, cnt_csr and tot are zero on entry and left zero on return (fill_kernel, the last
// pass, clears the counters, the tile totals and the flag), so a call needs no zero-fill launch;
// cursor / pos are rewritten every call.
constexpr int CTRL_BAD = 1;    // an id fell outside [0, V)
constexpr int CTRL_WORDS = 4;

// Vocabulary scan over tiles of SCAN_PER x NT entries: coalesced loads into LDS, each thread
// scans SCAN_PER consecutive entries read back with a 1-word row pad, wave scans of the thread
// sums; writes pos[v] (exclusive scan of "id present"),
// cursor[v] (exclusive scan of the segment lengths: each segment's first CSR slot, advanced by
// fill_kernel's atomics), the compaction uids[pos[v]] = v and seg_off[pos[v]] = cursor[v], all
// leaving through LDS with coalesced stores.  Totals of the tile -> tile_u / tile_c.
constexpr int SCAN_PER = 16;
template <int NT> constexpr int scan_tile_n() { return SCAN_PER * NT; }
template <int NT> constexpr int scan_lds_words() { return scan_tile_n<NT>() + scan_tile_n<NT>() / SCAN_PER; }

__device__ __forceinline__ int scan_lds_index(int v) { return v + v / SCAN_PER; }

template <int NT>
__device__ __forceinline__ void scan_load(int32_t* tile, const int32_t* __restrict__ src, int64_t base, int nv) {
  const int tid = threadIdx.x;
  int32_t ld[SCAN_PER];   // all loads in flight before the first LDS store
#pragma unroll
  for (int k = 0; k < SCAN_PER; ++k) {
    const int i = tid + k * NT;
    ld[k] = i < nv ? src[base + i] : 0;
  }
#pragma unroll
  for (int k = 0; k < SCAN_PER; ++k) tile[scan_lds_index(tid + k * NT)] = ld[k];
}

template <int NT>
__device__ void scan_tile(int32_t* tile, int32_t* wu, int32_t* wc, const int32_t* __restrict__ cnt_all,
                          const int32_t* __restrict__ cnt_csr, int64_t base, int nv, int32_t ubase, int32_t cbase,
                          int32_t* __restrict__ pos, int32_t* __restrict__ cursor, int64_t* __restrict__ uids,
                          int32_t* __restrict__ seg_off, int32_t& tile_u, int32_t& tile_c) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  int32_t f[SCAN_PER], c[SCAN_PER];   // f: id present, c: segment length
  scan_load<NT>(tile, cnt_all, base, nv);
  __syncthreads();
#pragma unroll
  for (int k = 0; k < SCAN_PER; ++k) f[k] = tile[scan_lds_index(SCAN_PER * tid + k)] > 0 ? 1 : 0;
  __syncthreads();
  scan_load<NT>(tile, cnt_csr, base, nv);
  __syncthreads();
  int32_t fu = 0, fc = 0;
#pragma unroll
  for (int k = 0; k < SCAN_PER; ++k) {
    c[k] = tile[scan_lds_index(SCAN_PER * tid + k)];
    fu += f[k];
    fc += c[k];
  }
  int32_t iu = fu, ic = fc;   // inclusive wave scans
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int32_t yu = __shfl_up(iu, d, 64), yc = __shfl_up(ic, d, 64);
    if (lane >= d) { iu += yu; ic += yc; }
  }
  if (lane == 63) { wu[w] = iu; wc[w] = ic; }
  __syncthreads();
  int32_t pu = ubase, pc = cbase;
  for (int k = 0; k < w; ++k) { pu += wu[k]; pc += wc[k]; }
  pu += iu - fu;   // exclusive
  pc += ic - fc;
  const int32_t pu0 = pu, pc0 = pc;
  tile_u = 0;
  tile_c = 0;
#pragma unroll
  for (int k = 0; k < NT / 64; ++k) { tile_u += wu[k]; tile_c += wc[k]; }
#pragma unroll
  for (int k = 0; k < SCAN_PER; ++k) {
    tile[scan_lds_index(SCAN_PER * tid + k)] = pu;
    pu += f[k];
  }
  __syncthreads();
  for (int i = tid; i < nv; i += NT) pos[base + i] = tile[scan_lds_index(i)];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < SCAN_PER; ++k) {
    tile[scan_lds_index(SCAN_PER * tid + k)] = pc;
    pc += c[k];
  }
  __syncthreads();
  for (int i = tid; i < nv; i += NT) cursor[base + i] = tile[scan_lds_index(i)];
  __syncthreads();
  pu = pu0;
#pragma unroll
  for (int k = 0; k < SCAN_PER; ++k) {   // compacted ids (tile-local positions)
    if (f[k]) tile[pu - ubase] = SCAN_PER * tid + k;
    pu += f[k];
  }
  __syncthreads();
  for (int i = tid; i < tile_u; i += NT) uids[ubase + i] = base + tile[i];
  __syncthreads();
  pu = pu0;
  pc = pc0;
#pragma unroll
  for (int k = 0; k < SCAN_PER; ++k) {
    if (f[k]) tile[pu - ubase] = pc;
    pu += f[k];
    pc += c[k];
  }
  __syncthreads();
  for (int i = tid; i < tile_u; i += NT) seg_off[ubase + i] = tile[i];
  __syncthreads();   // tile / wu / wc free for the next tile
}

// counts = {U, U_pad, bad, T_csr} and the pad entries of uids / seg_off (one workgroup)
__device__ __forceinline__ void scan_finish(int32_t U, int32_t Tv, const int32_t* __restrict__ ctrl,
                                            int64_t* __restrict__ uids, int32_t* __restrict__ seg_off,
                                            int32_t* __restrict__ counts, int64_t fill_row) {
  const int tid = threadIdx.x;
  const int32_t Up = (U + 31) / 32 * 32;
  if (tid == 0) {
    counts[0] = U;
    counts[1] = Up;
    counts[2] = ctrl[CTRL_BAD];
    counts[3] = Tv;
    seg_off[Up] = Tv;
  }
  if (tid < Up - U) {
    uids[U + tid] = fill_row;
    seg_off[U + tid] = Tv;
  }
}

// cnt_all[v]: tokens of id v (distinctness), cnt_csr[v]: those with grad_mask set (segments);
// tot[2 b], tot[2 b + 1]: the distinct ids and the segment positions of vocabulary tile b (the first
// block to count an id sees it at zero), per block collected in LDS up to COUNT_TILES_LDS tiles, so the
// scan reads the totals of the tiles before its own instead of re-reading their counters.
constexpr int COUNT_TILES_LDS = 256;
__global__ __launch_bounds__(CNT_THREADS) void count_kernel(const int64_t* __restrict__ ids, int64_t T, int64_t V,
                                                            const void* gm, int gm_dt, int32_t* __restrict__ ctrl,
                                                            int32_t* __restrict__ cnt_all,
                                                            int32_t* __restrict__ cnt_csr, int32_t* __restrict__ tot,
                                                            int nb, int tile_n) {
  __shared__ int32_t hkey[HASH_SLOTS], hall[HASH_SLOTS], hcsr[HASH_SLOTS];
  __shared__ int32_t th[2 * COUNT_TILES_LDS];
  const bool lds_tiles = nb <= COUNT_TILES_LDS;
  for (int i = threadIdx.x; i < HASH_SLOTS; i += blockDim.x) { hkey[i] = -1; hall[i] = 0; hcsr[i] = 0; }
  if (lds_tiles)
    for (int i = threadIdx.x; i < 2 * nb; i += blockDim.x) th[i] = 0;
  __syncthreads();
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < T) {
    const int64_t v = ids[t];
    if (v < 0 || v >= V) {
      ctrl[CTRL_BAD] = 1;   // out-of-range id: flagged, token dropped
    } else {
      const int h = hash_slot(hkey, (int32_t)v);
      atomicAdd(&hall[h], 1);
      if (grad_on(gm, gm_dt, t)) atomicAdd(&hcsr[h], 1);
    }
  }
  __syncthreads();
  int32_t* tt = lds_tiles ? th : tot;
  for (int i = threadIdx.x; i < HASH_SLOTS; i += blockDim.x)
    if (hkey[i] >= 0) {
      const int32_t k = hkey[i], b = k / tile_n;
      if (atomicAdd(&cnt_all[k], hall[i]) == 0) atomicAdd(&tt[2 * b], 1);
      if (hcsr[i]) {
        atomicAdd(&cnt_csr[k], hcsr[i]);
        atomicAdd(&tt[2 * b + 1], hcsr[i]);
      }
    }
  if (lds_tiles) {
    __syncthreads();
    for (int i = threadIdx.x; i < 2 * nb; i += blockDim.x)
      if (th[i]) atomicAdd(&tot[i], th[i]);
  }
}

// The scan over tiles of 16 x 256 entries, one workgroup per tile (ceil(V / 4096) CUs): each tile
// adds up the totals count_kernel left for the tiles before it and runs scan_tile; the last tile
// writes counts and the pad entries.
constexpr int SCAN_THREADS = 256;

// block-wide sums of two values (every thread gets both)
__device__ __forceinline__ void block_sum2(int32_t& a, int32_t& b, int32_t* red) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    a += __shfl_xor(a, d, 64);
    b += __shfl_xor(b, d, 64);
  }
  if (lane == 0) { red[2 * w] = a; red[2 * w + 1] = b; }
  __syncthreads();
  a = 0; b = 0;
#pragma unroll
  for (int k = 0; k < SCAN_THREADS / 64; ++k) { a += red[2 * k]; b += red[2 * k + 1]; }
  __syncthreads();
}

__global__ __launch_bounds__(SCAN_THREADS) void scan_down_kernel(const int32_t* __restrict__ ctrl,
                                                                 const int32_t* __restrict__ cnt_all,
                                                                 const int32_t* __restrict__ cnt_csr, int64_t V,
                                                                 const int32_t* __restrict__ tot,
                                                                 int32_t* __restrict__ pos, int32_t* __restrict__ cursor,
                                                                 int64_t* __restrict__ uids,
                                                                 int32_t* __restrict__ seg_off,
                                                                 int32_t* __restrict__ counts, int64_t fill_row) {
  __shared__ int32_t tile[scan_lds_words<SCAN_THREADS>()];
  __shared__ int32_t wu[SCAN_THREADS / 64], wc[SCAN_THREADS / 64], red[2 * SCAN_THREADS / 64];
  constexpr int TILE = scan_tile_n<SCAN_THREADS>();
  const int b = blockIdx.x;
  const int64_t base = (int64_t)b * TILE;
  const int nv = (int)(V - base < TILE ? V - base : TILE);
  int32_t ubase = 0, cbase = 0;   // totals of the tiles before this one
  for (int j = threadIdx.x; j < b; j += SCAN_THREADS) { ubase += tot[2 * j]; cbase += tot[2 * j + 1]; }
  block_sum2(ubase, cbase, red);
  int32_t tu, tc;
  scan_tile<SCAN_THREADS>(tile, wu, wc, cnt_all, cnt_csr, base, nv, ubase, cbase, pos, cursor, uids, seg_off, tu, tc);
  if (b == (int)gridDim.x - 1) scan_finish(ubase + tu, cbase + tc, ctrl, uids, seg_off, counts, fill_row);
}

// inv[t] for every token; CSR slots for the tokens with grad_mask set: slot = (block base of its
// id, an atomic on the segment cursor the scan left at the segment's first slot) + (its rank in
// the block), one global atomic per distinct id of the block.  seg_of[p] = the distinct row of CSR
// position p.
__global__ __launch_bounds__(CNT_THREADS) void fill_kernel(const int64_t* __restrict__ ids, int64_t T, int64_t V,
                                                           const void* gm, int gm_dt,
                                                           const int32_t* __restrict__ pos,
                                                           int32_t* __restrict__ cursor, int64_t* __restrict__ inv,
                                                           int32_t* __restrict__ seg_tok,
                                                           int32_t* __restrict__ seg_of, int32_t* __restrict__ ctrl,
                                                           int4* __restrict__ counters, int64_t n_counter4,
                                                           int32_t* __restrict__ tot, int64_t n_tot) {
  // the call's last pass: both counters (2 x ceil4(V) int32, contiguous), the tile totals and the
  // flag back to zero
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n_counter4; q += (int64_t)gridDim.x * blockDim.x)
    counters[q] = make_int4(0, 0, 0, 0);
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n_tot; q += (int64_t)gridDim.x * blockDim.x)
    tot[q] = 0;
  if (blockIdx.x == 0 && threadIdx.x == 0) ctrl[CTRL_BAD] = 0;
  __shared__ int32_t hkey[HASH_SLOTS], hcnt[HASH_SLOTS];
  for (int i = threadIdx.x; i < HASH_SLOTS; i += blockDim.x) { hkey[i] = -1; hcnt[i] = 0; }
  __syncthreads();
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t v = t < T ? ids[t] : -1;
  const bool ok = t < T && v >= 0 && v < V;
  const bool seg = ok && grad_on(gm, gm_dt, t);
  if (t < T) inv[t] = ok ? pos[v] : 0;
  int h = -1;
  int32_t rank = 0;
  if (seg) {
    h = hash_slot(hkey, (int32_t)v);
    rank = atomicAdd(&hcnt[h], 1);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < HASH_SLOTS; i += blockDim.x)   // counts -> block bases (in place)
    if (hkey[i] >= 0) hcnt[i] = atomicAdd(&cursor[hkey[i]], hcnt[i]);
  __syncthreads();
  if (!seg) return;
  const int32_t p = hcnt[h] + rank;
  seg_tok[p] = (int32_t)t;
  seg_of[p] = pos[v];
}

// Segment sum, pass 1: workgroup b sums the CSR positions [b*R, (b+1)*R) piece by piece (a
// piece = the part of one segment inside the range).  Whole segments are stored to dst; a
// segment cut by a range boundary leaves its pieces in part[b][slot] (slot 0: the block's
// first piece, slot 1: a later one) for pass 2.  A table in LDS marks each piece's last
// position and destination; one thread per float4 column streams the range SEG_BATCH rows at a
// time (that many independent loads in flight), flushing at piece ends (block-uniform branches).
// TAPS (the k = 3 convolution's per-distinct-row sums, nr_segment_rows_sum_conv3): output column
// block `tap` (wt4 float4 wide) of token t's contribution is src row t + 1 - tap of the same title
// of L tokens, zero when that row is outside the title.
template <bool TAPS>
__global__ __launch_bounds__(1024) void segsum_pieces_kernel(const float* __restrict__ src, int64_t lds, int64_t w4,
                                                             int64_t wt4, int L,
                                                             const int32_t* __restrict__ seg_off,
                                                             const int32_t* __restrict__ seg_tok,
                                                             const int32_t* __restrict__ seg_of,
                                                             const int32_t* __restrict__ counts,
                                                             float4* __restrict__ part, float* __restrict__ dst,
                                                             int64_t ldd, int skip_single) {
  const int64_t T = counts[3];   // positions in the CSR
  const int64_t b = blockIdx.x, p0 = b * SEG_RANGE;
  if (p0 >= T) return;
  const int64_t p1 = p0 + SEG_RANGE < T ? p0 + SEG_RANGE : T;
  int n = (int)(p1 - p0);
  __shared__ int32_t s_tok[SEG_RANGE], s_seg[SEG_RANGE + 1];
  __shared__ uint8_t s_ok[TAPS ? SEG_RANGE : 1];   // TAPS: bit j = src row t + 1 - j inside the title
  __shared__ int64_t s_dst[SEG_RANGE];   // at a piece's last position: its float4 destination
  __shared__ int s_n;
  const int tid = threadIdx.x;
  if (tid < SEG_RANGE) {   // wave 0 (SEG_RANGE = 64 = one wave): the range's positions, compacted
    int32_t t = 0, u = -1;
    bool keep = tid < n;
    if (keep) {
      t = seg_tok[p0 + tid];
      u = seg_of[p0 + tid];
      // skip_single: a one-token segment's row was written by the producer itself (nr_mha_pool_bwd
      // with seg_off): its position is dropped (a segment of one token is never cut by a range)
      if (skip_single) keep = seg_off[u + 1] - seg_off[u] != 1;
    }
    const uint64_t kb = __ballot(keep);
    const int at = __popcll(kb & ((1ull << tid) - 1ull));
    if (keep) {
      s_tok[at] = t;
      s_seg[at] = u;
      if (TAPS) {
        const int pos = t % L;
        s_ok[at] = (uint8_t)((pos + 1 < L ? 1 : 0) | 2 | (pos > 0 ? 4 : 0));
      }
    }
    if (tid == 0) {
      s_n = __popcll(kb);
      s_seg[__popcll(kb)] = -1;
    }
  }
  __syncthreads();
  n = s_n;
  if (tid < n && s_seg[tid + 1] != s_seg[tid]) {   // last position of a piece
    const int32_t u = s_seg[tid];
    const int64_t gb = seg_off[u], ge = seg_off[u + 1];
    int64_t d;
    if (gb >= p0 && ge <= p1) d = u * (ldd / 4);                    // whole segment -> dst row
    else d = -1 - ((b * 2 + (gb > p0 ? 1 : 0)) * w4);               // cut -> part slot (encoded)
    s_dst[tid] = d;
  }
  __syncthreads();
  float4* dst4 = reinterpret_cast<float4*>(dst);
  for (int64_t j = tid; j < w4; j += blockDim.x) {
    int tap = 0;
    int64_t jc = j;
    if (TAPS) {
      tap = (int)(j / wt4);
      jc = j - tap * wt4;
    }
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int i0 = 0; i0 < n; i0 += SEG_BATCH) {
      float4 x[SEG_BATCH];
#pragma unroll
      for (int k = 0; k < SEG_BATCH; ++k) {
        const int i = i0 + k < n ? i0 + k : n - 1;
        if (TAPS) {
          const bool ok = (s_ok[i] >> tap) & 1;
          const int64_t r = ok ? (int64_t)s_tok[i] + 1 - tap : (int64_t)s_tok[i];
          const float4 v = reinterpret_cast<const float4*>(src + r * lds)[jc];
          x[k] = ok ? v : make_float4(0.f, 0.f, 0.f, 0.f);
        } else {
          x[k] = reinterpret_cast<const float4*>(src + (int64_t)s_tok[i] * lds)[j];
        }
      }
#pragma unroll
      for (int k = 0; k < SEG_BATCH; ++k) {
        const int i = i0 + k;
        if (i < n) {
          s.x += x[k].x; s.y += x[k].y; s.z += x[k].z; s.w += x[k].w;
          if (s_seg[i + 1] != s_seg[i]) {
            const int64_t d = s_dst[i];
            (d >= 0 ? dst4 + d : part + (-1 - d))[j] = s;
            s = make_float4(0.f, 0.f, 0.f, 0.f);
          }
        }
      }
    }
  }
}

// Pass 2: workgroup b takes the distinct rows u = b (mod grid) -- rows of neighbouring ids, e.g. the
// [CLS] / [SEP] of every title, land on different workgroups -- and compacts the rows that need
// work into LDS: segments cut by a range boundary (sum their pieces in range order), empty
// segments and pad rows [U, U_pad) (zero).  Whole segments were written by pass 1.  One wave per
// row for short cuts; a cut with many pieces (a long segment) takes the whole workgroup, pieces
// split over thread groups and combined in LDS.
constexpr int FIX_THREADS = 1024;
constexpr int FIX_BLOCKS = 256;
constexpr int FIX_WAVE_PIECES = 8;

__device__ __forceinline__ float4 f4add(float4 a, float4 b) {
  return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}

__global__ __launch_bounds__(FIX_THREADS) void segsum_fix_kernel(int64_t w4, const int32_t* __restrict__ seg_off,
                                                                 const int32_t* __restrict__ counts,
                                                                 const float4* __restrict__ part,
                                                                 float* __restrict__ dst, int64_t ldd) {
  __shared__ float4 acc_s[FIX_THREADS];
  __shared__ int32_t todo_w[FIX_THREADS], todo_b[FIX_THREADS];
  __shared__ int32_t nw_todo, nb_todo;
  const int32_t U = counts[0], Up = counts[1];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, nwv = FIX_THREADS / 64;
  const int G = w4 <= FIX_THREADS ? (int)(FIX_THREADS / w4) : 1;
  const int64_t gw = w4 < FIX_THREADS ? w4 : FIX_THREADS;
  const int g = (int)(tid / gw);
  const int64_t j0 = tid - (int64_t)g * gw;
  for (int64_t c0 = 0; c0 < Up; c0 += (int64_t)gridDim.x * FIX_THREADS) {
    if (tid == 0) nw_todo = nb_todo = 0;
    __syncthreads();
    {
      const int64_t u = c0 + (int64_t)tid * gridDim.x + blockIdx.x;
      if (u < Up) {
        bool wave_item = false, block_item = false;
        if (u >= U) {
          wave_item = true;   // pad row: zero
        } else {
          const int64_t sb = seg_off[u], se = seg_off[u + 1];
          if (se == sb) {
            wave_item = true;   // no token with a gradient: zero
          } else {
            const int64_t b0 = sb / SEG_RANGE, b1 = (se - 1) / SEG_RANGE;
            if (b0 != b1) (b1 - b0 + 1 > FIX_WAVE_PIECES ? block_item : wave_item) = true;
          }
        }
        if (wave_item) todo_w[atomicAdd(&nw_todo, 1)] = (int32_t)u;
        if (block_item) todo_b[atomicAdd(&nb_todo, 1)] = (int32_t)u;
      }
    }
    __syncthreads();
    const int nw = nw_todo, nb = nb_todo;
    for (int k = wv; k < nw; k += nwv) {   // one wave per row
      const int64_t u = todo_w[k];
      float4* drow = reinterpret_cast<float4*>(dst + u * ldd);
      int64_t sb = 0, se = 0;
      if (u < U) { sb = seg_off[u]; se = seg_off[u + 1]; }
      for (int64_t j = lane; j < w4; j += 64) {
        float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
        if (se > sb) {
          const int64_t b0 = sb / SEG_RANGE, b1 = (se - 1) / SEG_RANGE;
          s = part[(b0 * 2 + (sb > b0 * SEG_RANGE ? 1 : 0)) * w4 + j];
          for (int64_t b = b0 + 1; b <= b1; ++b) s = f4add(s, part[(b * 2) * w4 + j]);
        }
        drow[j] = s;
      }
    }
    for (int k = 0; k < nb; ++k) {   // long segments: the whole workgroup
      const int64_t u = todo_b[k];
      float4* drow = reinterpret_cast<float4*>(dst + u * ldd);
      const int64_t sb = seg_off[u], se = seg_off[u + 1];
      const int64_t b0 = sb / SEG_RANGE, b1 = (se - 1) / SEG_RANGE;
      for (int64_t jb = 0; jb < w4; jb += FIX_THREADS) {
        const int64_t j = jb + j0;
        float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
        if (g < G && j < w4) {
          int64_t b = b0 + g;
          if (b == b0) {   // the first piece may sit in slot 1
            s = part[(b * 2 + (sb > b0 * SEG_RANGE ? 1 : 0)) * w4 + j];
            b += G;
          }
          for (; b + 7 * G <= b1; b += 8 * G) {   // later pieces: slot 0, eight loads in flight
            float4 x[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) x[q] = part[((b + q * G) * 2) * w4 + j];
#pragma unroll
            for (int q = 0; q < 8; ++q) s = f4add(s, x[q]);
          }
          for (; b <= b1; b += G) s = f4add(s, part[(b * 2) * w4 + j]);
        }
        if (G > 1) {
          acc_s[tid] = s;
          __syncthreads();
          if (g == 0 && j < w4) {
            for (int q = 1; q < G; ++q) s = f4add(s, acc_s[q * w4 + j0]);
            drow[j] = s;
          }
          __syncthreads();
        } else if (j < w4) {
          drow[j] = s;
        }
      }
    }
    __syncthreads();
  }
}

}  // namespace

extern "C" int nr_unique_rows(const int64_t* ids, int64_t T, int64_t V, int64_t fill_row, const void* grad_mask,
                              int32_t mask_dtype, int32_t* work, int64_t* uids, int64_t* inv, int32_t* seg_off,
                              int32_t* seg_tok, int32_t* seg_of, int32_t* counts, hipStream_t stream) {
  if (T < 0 || V < 1 || V > 0x7fffffff || T > 0x7fffffff) return NR_EINVAL(0);
  if ((T > 0 && (!ids || !inv || !seg_tok || !seg_of)) || !work || !uids || !seg_off || !counts) return NR_EINVAL(1);
  if (fill_row < 0 || fill_row >= V) return NR_EINVAL(2);
  if (grad_mask && (mask_dtype < NR_MASK_U8 || mask_dtype > NR_MASK_F32)) return NR_EINVAL(5);
  if (reinterpret_cast<uintptr_t>(work) & 15) return NR_EINVAL(6);
  const int64_t V4 = (V + 3) & ~int64_t(3);   // every array 16-B aligned
  int32_t* ctrl = work;
  int32_t* cnt_all = work + CTRL_WORDS;
  int32_t* cnt_csr = cnt_all + V4;
  int32_t* cursor = cnt_csr + V4;
  int32_t* pos = cursor + V4;
  int32_t* tot = pos + V4;   // [nb][2] tile totals (count_kernel; zero on entry, cleared by fill_kernel)
  const int64_t nb = (V + scan_tile_n<SCAN_THREADS>() - 1) / scan_tile_n<SCAN_THREADS>();
  // at least one count workgroup
  const unsigned gb = (unsigned)(T > 0 ? (T + CNT_THREADS - 1) / CNT_THREADS : 1);
  constexpr int TILE = scan_tile_n<SCAN_THREADS>();
  hipLaunchKernelGGL(count_kernel, dim3(gb), dim3(CNT_THREADS), 0, stream, ids, T, V, grad_mask, mask_dtype, ctrl,
                     cnt_all, cnt_csr, tot, (int)nb, TILE);
  hipLaunchKernelGGL(scan_down_kernel, dim3((unsigned)nb), dim3(SCAN_THREADS), 0, stream, ctrl, cnt_all, cnt_csr, V,
                     tot, pos, cursor, uids, seg_off, counts, fill_row);
  // fill runs even for T = 0: it is the pass that clears the counters, the tile totals and the flag
  hipLaunchKernelGGL(fill_kernel, dim3(gb), dim3(CNT_THREADS), 0, stream, ids, T, V, grad_mask, mask_dtype, pos,
                     cursor, inv, seg_tok, seg_of, ctrl, reinterpret_cast<int4*>(cnt_all), 2 * V4 / 4, tot, 2 * nb);
  NR_LAUNCH_CHECK();
  return NR_OK;
}

namespace {
// Rows of a [V, width] matrix whose id is absent from the last nr_unique_rows call on `work` (its
// presence scan pos[] is left there), and the pad row, set to zero; present rows are left alone.
// rows per workgroup: 16 -> 7.5 us for the bench batch's word-table gradient, 11.6 us at 64 (8: 7.7, 32:
// 7.7; profiles/r05_af_ab_zero_absent_rows.json)
constexpr int ZA_ROWS = 16;
__global__ __launch_bounds__(256) void zero_absent_kernel(const int32_t* __restrict__ pos, const int32_t* __restrict__ counts,
                                                          int64_t V, int64_t pad_row, float* __restrict__ dst, int64_t ldd,
                                                          int64_t w4, uint8_t* __restrict__ flags) {
  // flags (optional): 1 for a row the dgrad stores, 0 for one zeroed here (Adam's per-row
  // "gradient may be non-zero" flags)
  // ZA_ROWS rows per workgroup: the first ZA_ROWS lanes test them (coalesced scan reads) and list the
  // absent ones in LDS, then the workgroup zeroes the listed rows together
  __shared__ int32_t rows[ZA_ROWS];
  __shared__ int nrow;
  const int64_t v0 = (int64_t)blockIdx.x * ZA_ROWS;
  if (threadIdx.x < 64) {
    const int64_t v = v0 + threadIdx.x;
    bool absent = false;
    if (threadIdx.x < ZA_ROWS && v < V) {
      const int32_t next = v + 1 < V ? pos[v + 1] : counts[0];
      absent = !(next > pos[v]) || v == pad_row;
      if (flags) flags[v] = absent ? 0 : 1;
    }
    const uint64_t bl = __ballot(absent);
    if (absent) rows[__popcll(bl & ((1ull << threadIdx.x) - 1ull))] = (int32_t)(v - v0);
    if (threadIdx.x == 0) nrow = __popcll(bl);
  }
  __syncthreads();
  const int n = nrow, n4 = (int)w4;
  for (int e = threadIdx.x; e < n * n4; e += 256) {
    const int r = e / n4;
    reinterpret_cast<float4*>(dst + (v0 + rows[r]) * ldd)[e - r * n4] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
}
}  // namespace

extern "C" int nr_unique_rows_zero_absent(const int32_t* work, const int32_t* counts, int64_t V, int64_t pad_row,
                                          float* dst, int64_t ldd, int64_t width, uint8_t* flags,
                                          hipStream_t stream) {
  if (V < 1 || V > 0x7fffffff || width < 0 || width > (int64_t)(0x7fffffff / 64) * 4 || (width & 3) || (ldd & 3) ||
      ldd < width)
    return NR_EINVAL(0);
  if (!work || !counts || !dst) return NR_EINVAL(1);
  if (reinterpret_cast<uintptr_t>(dst) & 15) return NR_EINVAL(2);
  if (width == 0 && !flags) return NR_OK;
  const int64_t V4 = (V + 3) & ~int64_t(3);
  const int32_t* pos = work + CTRL_WORDS + 3 * V4;
  hipLaunchKernelGGL(zero_absent_kernel, dim3((unsigned)((V + ZA_ROWS - 1) / ZA_ROWS)), dim3(256), 0, stream, pos, counts, V, pad_row,
                     dst, ldd, width / 4, flags);
  NR_LAUNCH_CHECK();
  return NR_OK;
}

extern "C" int64_t nr_unique_rows_workspace(int64_t V) {
  const int64_t V4 = (V + 3) & ~int64_t(3);
  return CTRL_WORDS + 4 * V4 + 2 * ((V + scan_tile_n<SCAN_THREADS>() - 1) / scan_tile_n<SCAN_THREADS>());
}

extern "C" int64_t nr_segment_rows_sum_workspace(int64_t T, int64_t width) {
  return ((T + SEG_RANGE - 1) / SEG_RANGE) * 2 * width * (int64_t)sizeof(float);
}

namespace {
int segsum_launch(bool taps, const float* src, int64_t lds, int64_t width, int64_t wt4, int L, int64_t T,
                  const int32_t* seg_off, const int32_t* seg_tok, const int32_t* seg_of, const int32_t* counts,
                  int64_t rows_max, float* work, float* dst, int64_t ldd, hipStream_t stream, int skip_single = 0) {
  if (rows_max == 0 || width == 0) return NR_OK;
  const int64_t w4 = width / 4;
  if (T > 0) {
    const dim3 grid((unsigned)((T + SEG_RANGE - 1) / SEG_RANGE));
    const dim3 block((unsigned)(w4 >= 1024 ? 1024 : (w4 < SEG_RANGE ? SEG_RANGE : (w4 + 63) / 64 * 64)));
    if (taps)
      hipLaunchKernelGGL(segsum_pieces_kernel<true>, grid, block, 0, stream, src, lds, w4, wt4, L, seg_off, seg_tok,
                         seg_of, counts, reinterpret_cast<float4*>(work), dst, ldd, skip_single);
    else
      hipLaunchKernelGGL(segsum_pieces_kernel<false>, grid, block, 0, stream, src, lds, w4, wt4, L, seg_off, seg_tok,
                         seg_of, counts, reinterpret_cast<float4*>(work), dst, ldd, skip_single);
  }
  const int64_t fb = (rows_max + 255) / 256;   // a quarter of each workgroup's threads hold a row
  hipLaunchKernelGGL(segsum_fix_kernel, dim3((unsigned)(fb < FIX_BLOCKS ? fb : FIX_BLOCKS)), dim3(FIX_THREADS), 0,
                     stream, w4, seg_off, counts, reinterpret_cast<const float4*>(work), dst, ldd);
  NR_LAUNCH_CHECK();
  return NR_OK;
}

bool misaligned(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) != 0; }
}  // namespace

extern "C" int nr_segment_rows_sum(const float* src, int64_t lds, int64_t width, int64_t T, const int32_t* seg_off,
                                   const int32_t* seg_tok, const int32_t* seg_of, const int32_t* counts,
                                   int64_t rows_max, float* work, float* dst, int64_t ldd, hipStream_t stream) {
  if (width < 0 || (width & 3) || (lds & 3) || (ldd & 3) || rows_max < 0 || T < 0) return NR_EINVAL(0);
  if (!src || !seg_off || !seg_tok || !seg_of || !counts || !dst || (T > 0 && !work)) return NR_EINVAL(1);
  if (misaligned(src) || misaligned(dst) || misaligned(work)) return NR_EINVAL(2);
  return segsum_launch(false, src, lds, width, 0, 1, T, seg_off, seg_tok, seg_of, counts, rows_max, work, dst, ldd,
                       stream);
}

extern "C" int nr_segment_rows_sum_multi(const float* src, int64_t lds, int64_t width, int64_t T,
                                         const int32_t* seg_off, const int32_t* seg_tok, const int32_t* seg_of,
                                         const int32_t* counts, int64_t rows_max, float* work, float* dst,
                                         int64_t ldd, hipStream_t stream) {
  if (width < 0 || (width & 3) || (lds & 3) || (ldd & 3) || rows_max < 0 || T < 0) return NR_EINVAL(0);
  if (!src || !seg_off || !seg_tok || !seg_of || !counts || !dst || (T > 0 && !work)) return NR_EINVAL(1);
  if (misaligned(src) || misaligned(dst) || misaligned(work)) return NR_EINVAL(2);
  return segsum_launch(false, src, lds, width, 0, 1, T, seg_off, seg_tok, seg_of, counts, rows_max, work, dst, ldd,
                       stream, 1);
}

extern "C" int nr_segment_rows_sum_conv3(const float* src, int64_t lds, int64_t tap_width, int32_t L, int64_t T,
                                         const int32_t* seg_off, const int32_t* seg_tok, const int32_t* seg_of,
                                         const int32_t* counts, int64_t rows_max, float* work, float* dst,
                                         int64_t ldd, hipStream_t stream) {
  if (tap_width < 0 || (tap_width & 3) || (lds & 3) || (ldd & 3) || rows_max < 0 || T < 0 || L < 1 ||
      (T % L) || ldd < 3 * tap_width || lds < tap_width)
    return NR_EINVAL(0);
  if (!src || !seg_off || !seg_tok || !seg_of || !counts || !dst || (T > 0 && !work)) return NR_EINVAL(1);
  if (misaligned(src) || misaligned(dst) || misaligned(work)) return NR_EINVAL(2);
  return segsum_launch(true, src, lds, 3 * tap_width, tap_width / 4, L, T, seg_off, seg_tok, seg_of, counts, rows_max,
                       work, dst, ldd, stream);
}

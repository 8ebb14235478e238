// Config-5 candidate generation (model/retrieve.py:138-232, 244-290, 477-595; candidate
// columns only) and the retrieval recall of model/eval_retrieved.py:45-118.
//
//   k_cand_aids   (R3)  one wave per session: distinct aids, per-type counts / last ts, the six
//                       ordinal ranks, the keep filter (:199-206), best order and the trim
//                       threshold of R5 (:490-503) -> kept (aid, ts_order_aid, type mask, th)
//   k_cand_build  (R4-R6, R8) one wave per session: for every kept aid its self pair and its
//                       list entries (5 co-count top-N lists, 2 kNN lists) are merged per aid_next
//                       in a small LDS hash (pair level: min rank <= th or aid_next == aid), kept
//                       pairs are folded per (session, aid_next) in the session's LDS hash (OR of
//                       sources and type masks, min ts_order_aid), the session's cl50 popularity
//                       list is added (:571-585), and the result is sorted by (ts_order_aid,
//                       aid_next) (:647, with aid_next as the deterministic tie-break)
//   k_cand_recall (R9)  one wave per session and type: filtered rank of each label, hit@k
//
// Ordinal-rank ties are broken by aid ascending (polars leaves them to groupby row order).
#include <algorithm>
#include <cstdlib>
#include "prims.h"
#include "table.h"

namespace ottohip {

constexpr int CS_MAXE = 512;      // events per session handled by k_cand_aids
constexpr int CS_SRC = 7;         // 5 co-count lists + 2 kNN lists
constexpr int CS_NLAST = 99;      // RETRIEVE_N_LAST_* / RETRIEVE_N_MOST_FREQUENT (config.py:76-79)
constexpr uint32_t CS_EMPTY = 0xFFFFFFFFu;
constexpr uint64_t CS_OVF_BIT = 1ull << 63;  // pool offset flag: the region lies in the overflow pool

struct CandLists {
  const uint32_t* off[CS_SRC];   // per source: [n_items + 1] offsets into nxt / rank (by aid)
  const int32_t* nxt[CS_SRC];
  const int16_t* rank[CS_SRC];
  int32_t n_items;
  const uint32_t* pop_off;       // [n_clusters + 1]
  const int32_t* pop_aid;
  int32_t n_clusters;
};

// kept aid record: aid, info = ts_order_aid (16 b) | type mask << 16 (3 b) | th << 19 (5 b)
struct KeptAid { int32_t aid; uint32_t info; };

__device__ __forceinline__ bool rank_before(int ka, int32_t aa, int kb, int32_t ab) {  // desc key, asc aid
  return ka > kb || (ka == kb && aa < ab);
}

__global__ __launch_bounds__(64) void k_cand_aids(const int64_t* __restrict__ off, int64_t S,
                                                  const int32_t* __restrict__ aid, const int32_t* __restrict__ ts,
                                                  const int8_t* __restrict__ type, KeptAid* __restrict__ kept,
                                                  uint32_t* __restrict__ n_kept, int* __restrict__ err) {
  __shared__ int32_t ea[CS_MAXE], et[CS_MAXE];
  __shared__ int8_t ey[CS_MAXE];
  __shared__ int32_t ua[CS_MAXE], un[4][CS_MAXE], ut[4][CS_MAXE];  // n / max ts: [all, clicks, carts, orders]
  __shared__ uint32_t m_sh;
  const int l = threadIdx.x;
  const int64_t s = blockIdx.x;
  if (s >= S) return;
  const int64_t e0 = off[s];
  const int n = (int)(off[s + 1] - e0);
  if (n > CS_MAXE) {
    if (l == 0) { atomicOr(err, 1); n_kept[s] = 0; }
    return;
  }
  for (int i = l; i < n; i += 64) { ea[i] = aid[e0 + i]; et[i] = ts[e0 + i]; ey[i] = type[e0 + i]; }
  if (l == 0) m_sh = 0;
  __syncthreads();
  // distinct aids (first occurrence), compacted in event order
  int base = 0;
  for (int i0 = 0; i0 < n; i0 += 64) {
    const int i = i0 + l;
    bool first = i < n;
    if (first) {
      const int32_t a = ea[i];
      for (int j = 0; j < i; ++j)
        if (ea[j] == a) { first = false; break; }
    }
    const uint64_t b = __ballot(first);
    if (first) ua[base + (int)mbcnt(b)] = ea[i];
    base += (int)__popcll(b);
  }
  const int m = base;
  __syncthreads();
  for (int u = l; u < m; u += 64) {
    const int32_t a = ua[u];
    int cnt[4] = {0, 0, 0, 0}, mt[4] = {INT32_MIN, INT32_MIN, INT32_MIN, INT32_MIN};
    for (int i = 0; i < n; ++i) {
      if (ea[i] != a) continue;
      const int y = ey[i] + 1;
      const int32_t t = et[i];
      cnt[0]++; mt[0] = max(mt[0], t);
#pragma unroll
      for (int q = 1; q < 4; ++q)
        if (q == y) { cnt[q]++; mt[q] = max(mt[q], t); }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) { un[q][u] = cnt[q]; ut[q][u] = mt[q]; }
  }
  __syncthreads();
  for (int u = l; u < m; u += 64) {
    const int32_t a = ua[u];
    int r_ts = 1, r_n = 1, r_nc = 1, r_no = 1, r_t[3] = {1, 1, 1};
    const bool has[3] = {un[1][u] > 0, un[2][u] > 0, un[3][u] > 0};
    for (int v = 0; v < m; ++v) {
      const int32_t b = ua[v];
      r_ts += rank_before(ut[0][v], b, ut[0][u], a);
      r_n += rank_before(un[0][v], b, un[0][u], a);
      r_nc += rank_before(un[2][v], b, un[2][u], a);
      r_no += rank_before(un[3][v], b, un[3][u], a);
#pragma unroll
      for (int q = 0; q < 3; ++q)
        if (un[q + 1][v] > 0) r_t[q] += rank_before(ut[q + 1][v], b, ut[q + 1][u], a);
    }
    // :199-206 keep filter (null ranks never pass)
    const bool keep = (has[0] && r_t[0] <= CS_NLAST) || (has[1] && r_t[1] <= CS_NLAST) ||
                      (has[2] && r_t[2] <= CS_NLAST) || r_n <= CS_NLAST || r_nc <= CS_NLAST || r_no <= CS_NLAST;
    // :496-503 best order (min ignores nulls) and th = max(3, 20 - 17/19 (best - 1)) (f64 as polars)
    int best = min(r_n, r_ts);
#pragma unroll
    for (int q = 0; q < 3; ++q)
      if (has[q]) best = min(best, r_t[q]);
    double th = 20.0 - (17.0 / 19.0) * (double)(best - 1);
    if (th < 3.0) th = 3.0;
    const uint32_t thi = (uint32_t)floor(th);  // integer rank <= th  <=>  rank <= floor(th)
    const uint32_t tm = (has[0] ? 1u : 0u) | (has[1] ? 2u : 0u) | (has[2] ? 4u : 0u);
    if (keep) {
      const uint32_t k = atomicAdd(&m_sh, 1u);
      KeptAid r;
      r.aid = a;
      r.info = (uint32_t)min(r_ts, 0xFFFF) | (tm << 16) | (thi << 19);
      kept[e0 + k] = r;
    }
  }
  __syncthreads();
  if (l == 0) n_kept[s] = m_sh;
}

// Per-aid union of the 7 source lists (SURVEY.md §8(a) R4-R5 are pair-level: a pair (aid, aid_next)
// carries every source that lists it and is kept if its best rank passes). One wave per aid:
// elements (x, source bit, rank) of all lists in LDS, duplicates of x folded (OR of bits, min rank).
// A kept aid's trim threshold th is at most 31 (5 bits) and R5 keeps an entry iff x == aid or its rank
// <= th, so the unique entries are written ordered by that test: the self entry (x == aid) first, then by
// rank 0..31 (entries ranked above 31 can never be kept and are dropped); ucnt[a] = entries written and
// pc[a][th] = the entries a kept aid with threshold th takes (a prefix of the list): k_cand_build scans
// only those instead of every entry (the long sessions' lists were mostly entries above their th).
constexpr int ML_MAX = 256;  // elements per aid across the 7 lists
constexpr int ML_TH = 32;    // trim thresholds 0..31
__global__ __launch_bounds__(256) void k_ml_build(CandLists L, const uint32_t* __restrict__ eoff,
                                                  int32_t* __restrict__ mx, uint16_t* __restrict__ mbr,
                                                  uint32_t* __restrict__ ucnt, uint16_t* __restrict__ pc,
                                                  int* __restrict__ err) {
  __shared__ uint32_t ex[4][ML_MAX];
  __shared__ uint16_t eb[4][ML_MAX], uk[4][ML_MAX];
  __shared__ uint32_t hs[4][ML_TH + 1];
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int64_t a = (int64_t)blockIdx.x * 4 + w;
  if (a >= L.n_items) return;
  uint32_t beg[CS_SRC], len[CS_SRC], tot = 0;
#pragma unroll
  for (int q = 0; q < CS_SRC; ++q) {
    if (L.off[q]) { beg[q] = L.off[q][a]; len[q] = L.off[q][a + 1] - beg[q]; } else { beg[q] = 0; len[q] = 0; }
    tot += len[q];
  }
  if (tot > ML_MAX) {
    if (l == 0) { atomicOr(err, 4); ucnt[a] = 0; }
    if (l < ML_TH) pc[a * ML_TH + l] = 0;
    return;
  }
  if (l <= ML_TH) hs[w][l] = 0;
  for (uint32_t e = l; e < tot; e += 64) {
    uint32_t j = e;
    int q = 0;
#pragma unroll
    for (int z = 0; z < CS_SRC; ++z)
      if (q == z && j >= len[z]) { j -= len[z]; q = z + 1; }
    const int32_t* np = L.nxt[0];
    const int16_t* rp = L.rank[0];
    uint32_t b0 = beg[0];
#pragma unroll
    for (int z = 1; z < CS_SRC; ++z)
      if (q == z) { np = L.nxt[z]; rp = L.rank[z]; b0 = beg[z]; }
    const int r = rp[b0 + j];
    ex[w][e] = (uint32_t)np[b0 + j];
    eb[w][e] = (uint16_t)((2u << q) << 8 | (uint32_t)(r < 0 ? 0 : (r > 255 ? 255 : r)));
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  const uint32_t o = eoff[a];
  // unique entries (the first occurrence of each x) with their folded bits and rank, counted per bucket
  // (0: x == aid, 1 + r: rank r <= 31); the others marked 0xFFFF
  for (uint32_t e0 = 0; e0 < tot; e0 += 64) {
    const uint32_t e = e0 + l;
    if (e < tot) {
      const uint32_t x = ex[w][e];
      bool first = true;
      uint32_t bits = 0, rk = 255;
      for (uint32_t f = 0; f < tot; ++f) {
        if (ex[w][f] != x) continue;
        if (f < e) { first = false; break; }
        bits |= eb[w][f] >> 8;
        rk = min(rk, (uint32_t)(eb[w][f] & 0xFFu));
      }
      const int key = x == (uint32_t)a ? 0 : (rk < (uint32_t)ML_TH ? 1 + (int)rk : -1);
      uk[w][e] = first && key >= 0 ? (uint16_t)(bits << 8 | rk) : (uint16_t)0xFFFFu;
      if (first && key >= 0) atomicAdd(&hs[w][key], 1u);
    }
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  const uint32_t c = l <= ML_TH ? hs[w][l] : 0u;
  const uint32_t incl = wave_incl_scan(c);
  if (l >= 1 && l <= ML_TH) pc[a * ML_TH + l - 1] = (uint16_t)incl;  // entries of the self bucket and ranks <= l - 1
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  if (l <= ML_TH) hs[w][l] = incl - c;  // bucket starts
  if (l == ML_TH) ucnt[a] = incl;
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  for (uint32_t e0 = 0; e0 < tot; e0 += 64) {
    const uint32_t e = e0 + l;
    const uint16_t v = e < tot ? uk[w][e] : (uint16_t)0xFFFFu;
    if (v != 0xFFFFu) {
      const uint32_t x = ex[w][e];
      const int key = x == (uint32_t)a ? 0 : 1 + (int)(v & 0xFFu);
      const uint32_t p = atomicAdd(&hs[w][key], 1u);  // order within a bucket: any (the folds commute)
      mx[o + p] = (int32_t)x;
      mbr[o + p] = v;
    }
  }
}

__global__ void k_ml_total(CandLists L, uint32_t* __restrict__ tot) {
  const int64_t a = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (a >= L.n_items) return;
  uint32_t t = 0;
#pragma unroll
  for (int q = 0; q < CS_SRC; ++q)
    if (L.off[q]) t += L.off[q][a + 1] - L.off[q][a];
  tot[a] = t;
}

struct MergedLists {
  const uint32_t* eoff;   // [n_items] element offset of the aid
  const uint32_t* ucnt;   // [n_items] entries kept in the list (self entry, ranks <= 31)
  const uint16_t* pc;     // [n_items][32] entries a kept aid with trim threshold th takes
  const int32_t* mx;
  const uint16_t* mbr;    // source bits << 8 | min rank
  int32_t n_items;
  const uint32_t* pop_off;
  const int32_t* pop_aid;
  int32_t n_clusters;
};

__device__ __forceinline__ uint32_t cs_hash(uint32_t x, uint32_t mask) { return (x * 0x9E3779B1u >> 9) & mask; }

__device__ __forceinline__ uint64_t shfl_xor_u64(uint64_t v, int m) {
  const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, m), hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), m);
  return ((uint64_t)hi << 32) | lo;
}
// Ascending bitonic sort of a wave's 64 R keys in registers: lane l holds positions l R .. l R + R - 1 (keys
// past n read as ~0). Stages whose partner lies in another lane exchange through __shfl_xor; the last log2 R
// stages of every merge are in-register compare-exchanges. Then the first n sorted keys go to out(p, key).
template <int R, class OUT>
__device__ __forceinline__ void wave_sort_u64(const uint64_t* __restrict__ SK, int n, OUT out) {
  const int l = (int)lane_id();
  uint64_t v[R];
#pragma unroll
  for (int q = 0; q < R; ++q) v[q] = l * R + q < n ? SK[l * R + q] : ~0ull;
#pragma unroll 1
  for (int k = 2; k <= 64 * R; k <<= 1) {
#pragma unroll 1
    for (int j = k >> 1; j >= R; j >>= 1) {  // partner lane l ^ (j / R), same slot
      const int lj = j / R;
      const bool lower = (l & lj) == 0;
#pragma unroll
      for (int q = 0; q < R; ++q) {
        const uint64_t w = shfl_xor_u64(v[q], lj);
        const bool up = ((l * R + q) & k) == 0;
        const bool mn = lower == up;  // this position keeps the smaller key
        const bool lt = w < v[q];
        v[q] = (lt == mn) ? w : v[q];
      }
    }
#pragma unroll
    for (int j = R / 2; j >= 1; j >>= 1) {  // partner slot q ^ j in this lane
      if (j <= (k >> 1)) {
#pragma unroll
        for (int q = 0; q < R; ++q) {
          if ((q & j) == 0) {
            const bool up = ((l * R + q) & k) == 0;
            const uint64_t a = v[q], b = v[q | j];
            const bool sw = (a > b) == up;
            v[q] = sw ? b : a;
            v[q | j] = sw ? a : b;
          }
        }
      }
    }
  }
#pragma unroll
  for (int q = 0; q < R; ++q)
    if (l * R + q < n) out(l * R + q, v[q]);
}

// one wave per session (WAVES sessions per block); pass 0 counts, pass 1 writes at cand_off
template <int HC, int WAVES>
__global__ __launch_bounds__(64 * WAVES) void k_cand_build(const int64_t* __restrict__ off,
                                                          const int64_t* __restrict__ sess, int64_t n_sess,
                                                          const KeptAid* __restrict__ kept,
                                                          const uint32_t* __restrict__ n_kept,
                                                          const int32_t* __restrict__ session_cl, MergedLists L,
                                                          int pass, uint32_t* __restrict__ n_cand,
                                                          const uint64_t* __restrict__ cand_off,
                                                          int32_t* __restrict__ o_next, int16_t* __restrict__ o_ord,
                                                          uint16_t* __restrict__ o_flags,
                                                          int32_t* __restrict__ overflow,
                                                          uint32_t* __restrict__ n_overflow, int dbg) {
  // OVL: the sort keys overlay the key / mask arrays once the table has been read into registers,
  // which halves the wave's LDS (more waves per CU for this latency-bound kernel)
  constexpr bool OVL = true;
  __shared__ uint64_t hkm64[WAVES][HC];  // keys [0, HC) and masks [HC, 2 HC) as u32; sort keys (OVL)
  __shared__ uint32_t ho[WAVES][HC];
  __shared__ uint64_t sk[OVL ? 1 : WAVES][OVL ? 1 : HC];
  __shared__ uint32_t flg[WAVES][64];  // chunk tags of the kept aids' first elements
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int64_t gi = (int64_t)blockIdx.x * WAVES + w;
  if (gi >= n_sess) return;
  const int64_t s = sess ? sess[gi] : gi;
  uint32_t* K = reinterpret_cast<uint32_t*>(hkm64[w]);
  uint32_t* Mk = K + HC;
  uint32_t* Ord = ho[w];
  for (int i = l; i < HC; i += 64) { K[i] = CS_EMPTY; Mk[i] = 0; Ord[i] = 0xFFFFFFFFu; }
  flg[w][l] = 0u;
  uint32_t tag = 0;
  __builtin_amdgcn_wave_barrier();
  bool full = false;
  auto insert = [&](uint32_t x, uint32_t bits, uint32_t ord) {
    uint32_t h = cs_hash(x, HC - 1);
    for (int p = 0; p < HC; ++p) {
      const uint32_t prev = atomicCAS(&K[h], CS_EMPTY, x);  // claim or find in one LDS round trip
      if (prev == CS_EMPTY || prev == x) { atomicOr(&Mk[h], bits); atomicMin(&Ord[h], ord); return; }
      h = (h + 1) & (HC - 1);
    }
    full = true;
  };
  const int64_t e0 = off[s];
  const uint32_t nk = n_kept[s];
  // kept aids 64 at a time: lane k owns kept aid k of the batch; the batch's merged-list entries
  // (+ one self entry per aid) are flattened and spread over the lanes
  for (uint32_t k0 = 0; k0 < nk; k0 += 64) {
    const uint32_t kb = min(64u, nk - k0);
    uint32_t cnt = 0, lo = 0;
    KeptAid r;
    r.aid = 0; r.info = 0;
    if ((uint32_t)l < kb) {
      r = kept[e0 + k0 + l];
      if (r.aid < L.n_items) { lo = L.eoff[r.aid]; cnt = L.pc[(int64_t)r.aid * ML_TH + (r.info >> 19)]; }
      cnt += 1;  // the self pair (aid, aid)
    }
    const uint32_t incl = wave_incl_scan(cnt);
    const uint32_t start = incl - cnt;  // the lane's first element
    const uint32_t aid_l = (uint32_t)r.aid, info_l = r.info;
    const uint32_t T = (dbg & 4) ? 0u : __shfl(incl, 63);
    // the elements of chunk [c0, c0 + 64), one per lane: the owner of element c0 + l is the kept aid of the
    // last start at or before it: the chunk's first owner (starts <= c0) plus the starts in (c0, c0 + l],
    // found by a ballot over the chunk's start flags (a fresh tag per chunk: no clearing). The next chunk's
    // global loads are issued before the current one is inserted (the loop is latency-bound).
    auto fetch = [&](uint32_t c0, uint32_t& a, uint32_t& info, uint32_t& j, uint32_t& x, uint32_t& br) {
      ++tag;
      if ((uint32_t)l < kb && start > c0 && start < c0 + 64) flg[w][start - c0] = tag;
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      const uint64_t M = __ballot(flg[w][l] == tag);
      const uint32_t kb0 = (uint32_t)__popcll(__ballot((uint32_t)l < kb && start <= c0)) - 1u;
      const uint32_t own = kb0 + (uint32_t)mbcnt(M) + (uint32_t)((M >> l) & 1ull);
      a = (uint32_t)__shfl((int)aid_l, (int)own);
      info = (uint32_t)__shfl((int)info_l, (int)own);
      const uint32_t st = (uint32_t)__shfl((int)start, (int)own), lo_o = (uint32_t)__shfl((int)lo, (int)own);
      const uint32_t e = c0 + (uint32_t)l;
      j = e - st;
      x = a; br = 0;
      if (e < T && j > 0) {
        x = (uint32_t)L.mx[lo_o + j - 1];
        br = L.mbr[lo_o + j - 1];
      }
    };
    uint32_t a0 = 0, i0 = 0, j0 = 0, x0 = 0, b0 = 0;
    if (T > 0) fetch(0u, a0, i0, j0, x0, b0);
    for (uint32_t c0 = 0; c0 < T; c0 += 64) {
      uint32_t a1 = 0, i1 = 0, j1 = 0, x1 = 0, b1 = 0;
      if (c0 + 64 < T) fetch(c0 + 64, a1, i1, j1, x1, b1);
      if (c0 + (uint32_t)l < T) {
        const uint32_t ord = i0 & 0xFFFFu, tm = (i0 >> 16) & 7u, th = i0 >> 19;
        if (j0 == 0) {
          insert(a0, 1u | (tm << 8), ord);
        } else if (x0 == a0 || (b0 & 0xFFu) <= th) {
          // R5 (:512-516) pair kept iff aid_next == aid or its best co-count / w2v rank <= th
          insert(x0, (b0 >> 8) | (x0 == a0 ? 1u : 0u) | (tm << 8), ord);
        }
      }
      a0 = a1; i0 = i1; j0 = j1; x0 = x1; b0 = b1;
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  }
  // R6 (:571-585) the cl50 popularity list of the session's cluster; new rows get ts_order 999
  const int32_t c = session_cl ? session_cl[s] : -1;
  if (c >= 0 && c < L.n_clusters && !(dbg & 2)) {
    const uint32_t pb = L.pop_off[c], pe = L.pop_off[c + 1];
    for (uint32_t j = pb + l; j < pe; j += 64) insert((uint32_t)L.pop_aid[j], 1u << 11, 999u);
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  if (__ballot(full)) {  // the session does not fit this tier: retried with a larger table
    if (l == 0) {
      if (overflow) overflow[atomicAdd(n_overflow, 1u)] = (int32_t)s;
      n_cand[s] = 0;
    }
    return;
  }
  // compact (ts_order, aid_next, flags) sort keys
  uint64_t* SK = OVL ? hkm64[w] : sk[OVL ? 0 : w];
  int cnt = 0;
  constexpr int NR = OVL ? HC / 64 : 1;
  uint64_t rk[NR];  // OVL: the lane's table entries (key or ~0), written after the whole table was read
#pragma unroll
  for (int c0 = 0; c0 < HC / 64; ++c0) {
    const int i = c0 * 64 + l;
    const bool occ = K[i] != CS_EMPTY;
    const uint64_t b = __ballot(occ);
    if (OVL) {
#pragma unroll
      for (int q = 0; q < NR; ++q) if (q == c0) rk[q] = ~0ull;
    }
    if (occ && pass == 1) {
      const uint32_t mk_ = Mk[i];
      const uint32_t click = (mk_ >> 8) & 1u, cart = (mk_ >> 9) & 1u, order = (mk_ >> 10) & 1u;
      // flags in SRC order: self, c2c, c2cob, cart2cart, cart2buy, buy2buy, w2v_all, w2v_1_2, pop_cl50
      uint32_t f = (mk_ & 1u);
      f |= (((mk_ >> 1) & 1u) & click) << 1;
      f |= (((mk_ >> 2) & 1u) & click) << 2;
      f |= (((mk_ >> 3) & 1u) & cart) << 3;
      f |= (((mk_ >> 4) & 1u) & cart) << 4;
      f |= (((mk_ >> 5) & 1u) & order) << 5;
      f |= ((mk_ >> 6) & 3u) << 6;
      f |= ((mk_ >> 11) & 1u) << 8;
      const uint64_t key = ((uint64_t)Ord[i] << 48) | ((uint64_t)K[i] << 16) | f;
      if (OVL) {
#pragma unroll
        for (int q = 0; q < NR; ++q) if (q == c0) rk[q] = key;
      } else {
        SK[cnt + (int)mbcnt(b)] = key;
      }
    }
    cnt += (int)__popcll(b);
  }
  if (OVL && pass == 1) {  // every lane has read its entries: the table's memory becomes the key array
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    int c = 0;
#pragma unroll
    for (int q = 0; q < NR; ++q) {
      const bool occ = rk[q] != ~0ull;
      const uint64_t b = __ballot(occ);
      if (occ) SK[c + (int)mbcnt(b)] = rk[q];
      c += (int)__popcll(b);
    }
  }
  if (pass == 0) {
    if (l == 0) n_cand[s] = (uint32_t)cnt;
    return;
  }
  const uint64_t o = cand_off[s] & ~CS_OVF_BIT;
  if (l == 0) n_cand[s] = (uint32_t)cnt;
  auto emit = [&](int i, uint64_t v) __attribute__((always_inline)) {
    o_next[o + i] = (int32_t)(uint32_t)(v >> 16);
    o_ord[o + i] = (int16_t)(v >> 48);
    o_flags[o + i] = (uint16_t)(v & 0x1FFu);
  };
  constexpr int RMAX = HC / 64 < 64 ? HC / 64 : 64;
  if (!(dbg & 1) && cnt <= 64 * RMAX) {  // in registers: 64 R >= cnt keys (cnt <= HC bounds R by the tier)
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    if (cnt <= 64) wave_sort_u64<1>(SK, cnt, emit);
    else if (cnt <= 128) wave_sort_u64<2>(SK, cnt, emit);
    else if (HC <= 256 || cnt <= 256) wave_sort_u64<4>(SK, cnt, emit);
    else if constexpr (HC >= 512) {
      if (HC <= 512 || cnt <= 512) wave_sort_u64<8>(SK, cnt, emit);
      else if constexpr (HC >= 1024) {
        if (HC <= 1024 || cnt <= 1024) wave_sort_u64<16>(SK, cnt, emit);
        else if constexpr (HC >= 2048) {
          if (HC <= 2048 || cnt <= 2048) wave_sort_u64<32>(SK, cnt, emit);
          else if constexpr (HC >= 4096) wave_sort_u64<64>(SK, cnt, emit);
        }
      }
    }
    return;
  }
  int P2 = 1;
  while (P2 < cnt) P2 <<= 1;
  if (dbg & 1) P2 = 1;  // (profiling) skip the sort
  for (int i = cnt + l; i < P2; i += 64) SK[i] = ~0ull;
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  for (int k = 2; k <= P2; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = l; i < P2; i += 64) {
        const int p = i ^ j;
        if (p > i) {
          const uint64_t x = SK[i], y = SK[p];
          const bool up = (i & k) == 0;
          if ((x > y) == up) { SK[i] = y; SK[p] = x; }
        }
      }
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    }
  }
  for (int i = l; i < cnt; i += 64) emit(i, SK[i]);
}

// Single-pass layout: an upper bound of every session's candidates (its kept aids' merged-list
// entries + self pairs + its cluster's popularity list, capped at the tier's table size) gives
// each session a region of a pool; the build pass writes its sorted candidates there and its
// count, and a compaction copies the regions into the session-ordered CSR (no count pass).
__global__ void k_cand_bound(const int64_t* __restrict__ off, int64_t S, const KeptAid* __restrict__ kept,
                             const uint32_t* __restrict__ n_kept, const int32_t* __restrict__ session_cl,
                             MergedLists L, uint32_t cap, uint32_t* __restrict__ ub,
                             uint32_t* __restrict__ ubx = nullptr, uint32_t capx = 0) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= S) return;
  const int64_t e0 = off[s];
  const uint32_t nk = n_kept[s];
  uint64_t t = 0;
  const uint32_t cm = ubx ? capx : cap;  // ubx: the bound capped at capx (tier routing), ub at cap (pool regions)
  for (uint32_t k = 0; k < nk && t < cm; ++k) {
    const KeptAid r = kept[e0 + k];
    t += 1u + (r.aid < L.n_items ? L.pc[(int64_t)r.aid * ML_TH + (r.info >> 19)] : 0u);
  }
  const int32_t c = session_cl ? session_cl[s] : -1;
  if (c >= 0 && c < L.n_clusters) t += L.pop_off[c + 1] - L.pop_off[c];
  ub[s] = (uint32_t)(t < cap ? t : cap);
  if (ubx) ubx[s] = (uint32_t)(t < capx ? t : capx);
}

// one wave per session: pool region [src_off, + n) -> CSR [dst_off, + n)
__global__ __launch_bounds__(256) void k_cand_compact(const uint64_t* __restrict__ src_off,
                                                      const uint64_t* __restrict__ dst_off, int64_t S,
                                                      const int32_t* __restrict__ p_next, const int16_t* __restrict__ p_ord,
                                                      const uint16_t* __restrict__ p_flags,
                                                      const int32_t* __restrict__ q_next, const int16_t* __restrict__ q_ord,
                                                      const uint16_t* __restrict__ q_flags,
                                                      int32_t* __restrict__ o_next, int16_t* __restrict__ o_ord,
                                                      uint16_t* __restrict__ o_flags) {
  const int64_t s = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (s >= S) return;
  const int l = threadIdx.x & 63;
  const uint64_t so = src_off[s], d0 = dst_off[s], n = dst_off[s + 1] - d0;
  const bool ovf = (so & CS_OVF_BIT) != 0;
  const uint64_t b = so & ~CS_OVF_BIT;
  const int32_t* xn = ovf ? q_next : p_next;
  const int16_t* xo = ovf ? q_ord : p_ord;
  const uint16_t* xf = ovf ? q_flags : p_flags;
  for (uint64_t i = l; i < n; i += 64) {
    o_next[d0 + i] = xn[b + i];
    o_ord[d0 + i] = xo[b + i];
    o_flags[d0 + i] = xf[b + i];
  }
}

// sessions by their candidate bound (tables at a load <= 3/4): tier 0 (ub <= 192: 256-slot tables), tier 1
// (<= 384: 512 slots), tier 2 (<= 1536: 1024 slots, then the overflow tier); lists[t * S ..] and cnt3[t]. A
// bound above 1536 goes straight to the overflow list (on config 5 every such session holds > 1024 candidates)
__global__ __launch_bounds__(256) void k_cand_tier(const uint32_t* __restrict__ ub, int64_t S, int64_t* __restrict__ lists,
                                                   uint32_t* __restrict__ cnt3, int32_t* __restrict__ ovf,
                                                   uint32_t* __restrict__ n_ovf) {
  __shared__ uint32_t c[3], b[3];
  if (threadIdx.x < 3) c[threadIdx.x] = 0;
  __syncthreads();
  const int64_t s = (int64_t)blockIdx.x * 256 + threadIdx.x;
  int t = -1;
  uint32_t p = 0;
  if (s < S) {
    const uint32_t u = ub[s];
    t = u <= 192 ? 0 : (u <= 384 ? 1 : 2);
    if (u > 1536) ovf[atomicAdd(n_ovf, 1u)] = (int32_t)s;
    else p = atomicAdd(&c[t], 1u);
    if (u > 1536) t = -1;
  }
  __syncthreads();
  if (threadIdx.x < 3) b[threadIdx.x] = c[threadIdx.x] ? atomicAdd(&cnt3[threadIdx.x], c[threadIdx.x]) : 0u;
  __syncthreads();
  if (t >= 0) lists[t * S + b[t] + p] = s;
}

__global__ void k_cand_ovf_src(const int32_t* __restrict__ ovf_sess, int64_t n, uint32_t cap,
                               uint64_t* __restrict__ src_off) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) src_off[ovf_sess[i]] = CS_OVF_BIT | ((uint64_t)i * cap);
}

// R9: one wave per session; per type: filtered rank of each label in the candidate order
constexpr int RC_MAX = 4096;
__global__ __launch_bounds__(64) void k_cand_recall(const uint64_t* __restrict__ cand_off,
                                                    const int32_t* __restrict__ cnext,
                                                    const uint16_t* __restrict__ cflags, int64_t S,
                                                    const int64_t* __restrict__ lab_off,  // [3][S + 1]
                                                    const int32_t* __restrict__ lab_aid, uint32_t fmask,
                                                    int max_k, unsigned long long* __restrict__ sums,
                                                    int* __restrict__ err) {
  __shared__ uint16_t frank[RC_MAX];
  const int l = threadIdx.x;
  const int64_t s = blockIdx.x;
  if (s >= S) return;
  const uint64_t c0 = cand_off[s], c1 = cand_off[s + 1];
  const int n = (int)(c1 - c0);
  if (n > RC_MAX) { if (l == 0) atomicOr(err, 2); return; }
  // filtered rank (1-based) of every candidate; 0 = filtered out
  int base = 0;
  for (int i0 = 0; i0 < n; i0 += 64) {
    const int i = i0 + l;
    const bool in = i < n && (fmask == 0 || (cflags[c0 + i] & fmask) != 0);
    const uint64_t b = __ballot(in);
    if (i < n) frank[i] = in ? (uint16_t)(base + (int)mbcnt(b) + 1) : 0;
    base += (int)__popcll(b);
  }
  __syncthreads();
  for (int t = 0; t < 3; ++t) {
    const int64_t lb = lab_off[t * (S + 1) + s], le = lab_off[t * (S + 1) + s + 1];
    // one label at a time, the wave's lanes over the candidates (a label is at most once in the session's
    // deduplicated list; one lane per label scanning the list serially was latency-bound: 42 ms per step)
    uint32_t h20 = 0, h100 = 0, h200 = 0, hall = 0, tru = 0;
    for (int64_t j = lb; j < le; ++j) {
      const int32_t y = lab_aid[j];
      int r = 0;
      for (int i0 = 0; i0 < n; i0 += 64) {
        const int i = i0 + l;
        const uint64_t b = __ballot(i < n && cnext[c0 + i] == y);
        if (b) {
          r = frank[i0 + __builtin_ctzll(b)];
          break;
        }
      }
      tru += 1;
      if (r > 0) { hall += 1; h20 += r <= 20; h100 += r <= 100; h200 += r <= 200; }
    }
    if (l == 0 && tru) {
      const uint32_t K = (uint32_t)max_k;
      unsigned long long* o = sums + (size_t)(s & 255) * 16 + t * 5;  // striped: 256 copies of [3][5]
      atomicAdd(&o[0], (unsigned long long)min(h20, K));
      atomicAdd(&o[1], (unsigned long long)min(h100, K));
      atomicAdd(&o[2], (unsigned long long)min(h200, K));
      atomicAdd(&o[3], (unsigned long long)min(hall, K));
      atomicAdd(&o[4], (unsigned long long)min(tru, K));
    }
  }
}

// ---- per-source lists: rows (key, nxt, rank) -> CSR by key (stable in row order)
__global__ void k_cl_keys(const int32_t* __restrict__ key, int64_t n, uint32_t n_keys, uint32_t* __restrict__ k,
                          uint32_t* __restrict__ v, uint32_t* __restrict__ cnt, int* __restrict__ err) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int32_t a = key[i];
  if (a < 0 || (uint32_t)a >= n_keys) { atomicOr(err, 1); k[i] = 0; v[i] = (uint32_t)i; return; }
  k[i] = (uint32_t)a;
  v[i] = (uint32_t)i;
  atomicAdd(&cnt[a], 1u);
}
__global__ void k_cl_gather(const uint32_t* __restrict__ v, int64_t n, const int32_t* __restrict__ nxt,
                            const int16_t* __restrict__ rank, int32_t* __restrict__ o_nxt,
                            int16_t* __restrict__ o_rank) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  o_nxt[i] = nxt[v[i]];
  if (rank) o_rank[i] = rank[v[i]];
}
__global__ void k_u64_to_u32(const uint64_t* __restrict__ a, int64_t n, uint32_t* __restrict__ b) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) b[i] = (uint32_t)a[i];
}

}  // namespace ottohip

namespace ottohip {
// ---- label CSR for R9 (model/eval_retrieved.py:45-118): (type, session index, aid) unique
// session ids sorted with their positions; each label row finds its session by binary search
__global__ void k_lab_sid_keys(const int32_t* __restrict__ sid, int64_t S, uint32_t* __restrict__ k,
                               uint32_t* __restrict__ v) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= S) return;
  k[i] = (uint32_t)sid[i] ^ 0x80000000u;  // signed order
  v[i] = (uint32_t)i;
}
// key of a label row after its aid pass: type << sb | session index, or all ones (dropped)
__global__ void k_lab_group(const uint32_t* __restrict__ perm, int64_t n, const int32_t* __restrict__ sess,
                            const int8_t* __restrict__ type, const uint32_t* __restrict__ sk,
                            const uint32_t* __restrict__ sv, int64_t S, int sb, uint32_t* __restrict__ key) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t j = perm[i];
  const int t = type[j];
  const uint32_t x = (uint32_t)sess[j] ^ 0x80000000u;
  int64_t lo = 0, hi = S;  // first sorted id >= x
  while (lo < hi) {
    const int64_t m = (lo + hi) >> 1;
    if (sk[m] < x) lo = m + 1; else hi = m;
  }
  const bool ok = t >= 0 && t <= 2 && lo < S && sk[lo] == x;
  key[i] = ok ? (((uint32_t)t << sb) | sv[lo]) : 0xFFFFFFFFu;
}
// kept = valid and not an equal (group, aid) duplicate of its predecessor
__global__ void k_lab_keep(const uint32_t* __restrict__ g, const uint32_t* __restrict__ perm, int64_t n,
                           const int32_t* __restrict__ aid, uint32_t* __restrict__ keep) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const bool valid = g[i] != 0xFFFFFFFFu;
  keep[i] = valid && (i == 0 || g[i - 1] != g[i] || aid[perm[i - 1]] != aid[perm[i]]) ? 1u : 0u;
}
__global__ void k_lab_compact(const uint32_t* __restrict__ g, const uint32_t* __restrict__ perm,
                              const uint32_t* __restrict__ keep, const uint64_t* __restrict__ pos, int64_t n,
                              const int32_t* __restrict__ aid, int sb, int64_t S, int32_t* __restrict__ out_aid,
                              uint64_t* __restrict__ out_grp) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || !keep[i]) return;
  out_aid[pos[i]] = aid[perm[i]];
  out_grp[pos[i]] = (uint64_t)(g[i] >> sb) * (uint64_t)S + (g[i] & ((1u << sb) - 1u));
}
// lab_off[t * (S + 1) + s] = first kept label of group >= t * S + s
__global__ void k_lab_off(const uint64_t* __restrict__ grp, int64_t m, int64_t S, int64_t* __restrict__ off) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 3 * (S + 1)) return;
  const int64_t t = i / (S + 1), s = i % (S + 1);
  const uint64_t x = (uint64_t)t * (uint64_t)S + (uint64_t)s;
  int64_t lo = 0, hi = m;
  while (lo < hi) {
    const int64_t md = (lo + hi) >> 1;
    if (grp[md] < x) lo = md + 1; else hi = md;
  }
  off[i] = lo;
}
}  // namespace ottohip

using namespace ottohip;

extern "C" {

int ottohip_labels_csr(ottohip_ctx* ctx, const int32_t* session_ids, int64_t n_sessions, const int32_t* session,
                       const int32_t* aid, const int8_t* type, int64_t n, int64_t* lab_off, int32_t* lab_aid,
                       int64_t* n_out, void* stream) {
  if (!ctx || n_sessions < 0 || n < 0 || !lab_off || !n_out || (n_sessions > 0 && !session_ids) ||
      (n > 0 && (!session || !aid || !type || !lab_aid))) {
    set_error("labels_csr: bad args"); return OTTOHIP_EINVAL;
  }
  if (n_sessions >= ((int64_t)1 << 29) || n >= ((int64_t)1 << 32)) { set_error("labels_csr: input too large"); return OTTOHIP_ELIMIT; }
  hipStream_t s = S(stream);
  OH_HIP(hipSetDevice(ctx->device));
  *n_out = 0;
  const int64_t S_ = n_sessions;
  Workspace& ws = ctx->ws;
  uint32_t *sk, *sv, *sk2, *sv2, *k, *v, *k2, *v2, *keep;
  uint64_t *pos, *grp, *tot;
  OH_TRY(ws.get("lab_sk", (size_t)std::max<int64_t>(S_, 1), &sk));
  OH_TRY(ws.get("lab_sv", (size_t)std::max<int64_t>(S_, 1), &sv));
  OH_TRY(ws.get("lab_sk2", (size_t)std::max<int64_t>(S_, 1), &sk2));
  OH_TRY(ws.get("lab_sv2", (size_t)std::max<int64_t>(S_, 1), &sv2));
  OH_TRY(ws.get("lab_k", (size_t)std::max<int64_t>(n, 1), &k));
  OH_TRY(ws.get("lab_v", (size_t)std::max<int64_t>(n, 1), &v));
  OH_TRY(ws.get("lab_k2", (size_t)std::max<int64_t>(n, 1), &k2));
  OH_TRY(ws.get("lab_v2", (size_t)std::max<int64_t>(n, 1), &v2));
  OH_TRY(ws.get("lab_keep", (size_t)std::max<int64_t>(n, 1), &keep));
  OH_TRY(ws.get("lab_pos", (size_t)std::max<int64_t>(n, 1), &pos));
  OH_TRY(ws.get("lab_grp", (size_t)std::max<int64_t>(n, 1), &grp));
  OH_TRY(ws.get("lab_tot", 1, &tot));
  uint32_t *ks = sk, *vs = sv;
  if (S_ > 0) {
    k_lab_sid_keys<<<grid_for(S_), 256, 0, s>>>(session_ids, S_, ks, vs);
    OH_TRY(radix_sort_pairs(ctx, ks, vs, sk2, sv2, S_, 32, s));
  }
  uint64_t m = 0;
  if (n > 0 && S_ > 0) {
    // stable LSD: aid, then (type, session index) -> (type, session index, aid)
    uint32_t *kk = k, *vv = v;
    OH_HIP(hipMemcpyAsync(kk, aid, (size_t)n * 4, hipMemcpyDeviceToDevice, s));
    OH_TRY(radix_sort_pairs(ctx, kk, vv, k2, v2, n, 32, s, true));
    const int sb = std::max(1, bits_for((uint64_t)S_));
    uint32_t* kn = kk == k ? k2 : k;
    k_lab_group<<<grid_for(n), 256, 0, s>>>(vv, n, session, type, ks, vs, S_, sb, kn);
    kk = kn;
    uint32_t* vn_alt = vv == v ? v2 : v;
    uint32_t* kn_alt = kk == k ? k2 : k;
    OH_TRY(radix_sort_pairs(ctx, kk, vv, kn_alt, vn_alt, n, 32, s));
    k_lab_keep<<<grid_for(n), 256, 0, s>>>(kk, vv, n, aid, keep);
    OH_TRY(exclusive_scan_u32(ctx, keep, pos, n, tot, s));
    OH_TRY(d2h(&m, tot, 1, s));
    k_lab_compact<<<grid_for(n), 256, 0, s>>>(kk, vv, keep, pos, n, aid, sb, S_, lab_aid, grp);
  }
  k_lab_off<<<grid_for(3 * (S_ + 1)), 256, 0, s>>>(grp, (int64_t)m, S_, lab_off);
  OH_HIP(hipGetLastError());
  *n_out = (int64_t)m;
  return 0;
}


// rows (key, nxt[, rank]) -> CSR: out_off [n_keys + 1] (u32), out_nxt / out_rank [n] in key order
int ottohip_lists_build(ottohip_ctx* ctx, const int32_t* key, const int32_t* nxt, const int16_t* rank, int64_t n,
                        int32_t n_keys, uint32_t* out_off, int32_t* out_nxt, int16_t* out_rank, void* stream) {
  if (!ctx || n < 0 || n_keys < 1 || !out_off || (n > 0 && (!key || !nxt || !out_nxt || (rank && !out_rank)))) {
    set_error("lists_build: bad arguments"); return OTTOHIP_EINVAL;
  }
  if (n >= ((int64_t)1 << 32)) { set_error("lists_build: n >= 2^32"); return OTTOHIP_ELIMIT; }
  hipStream_t s = S(stream);
  OH_HIP(hipSetDevice(ctx->device));
  Workspace& ws = ctx->ws;
  uint32_t *k0, *v0, *k1, *v1, *cnt;
  uint64_t* off64;
  int* err;
  OH_TRY(ws.get("cl_k0", (size_t)std::max<int64_t>(n, 1), &k0));
  OH_TRY(ws.get("cl_v0", (size_t)std::max<int64_t>(n, 1), &v0));
  OH_TRY(ws.get("cl_k1", (size_t)std::max<int64_t>(n, 1), &k1));
  OH_TRY(ws.get("cl_v1", (size_t)std::max<int64_t>(n, 1), &v1));
  OH_TRY(ws.get("cl_cnt", (size_t)n_keys + 1, &cnt));
  OH_TRY(ws.get("cl_off", (size_t)n_keys + 1, &off64));
  OH_TRY(ws.get("cl_err", 1, &err));
  OH_HIP(hipMemsetAsync(cnt, 0, ((size_t)n_keys + 1) * 4, s));
  OH_HIP(hipMemsetAsync(err, 0, sizeof(int), s));
  if (n > 0) {
    k_cl_keys<<<grid_for(n), 256, 0, s>>>(key, n, (uint32_t)n_keys, k0, v0, cnt, err);
    uint32_t *k = k0, *v = v0;
    OH_TRY(radix_sort_pairs(ctx, k, v, k1, v1, n, std::max(1, bits_for((uint64_t)n_keys)), s));
    k_cl_gather<<<grid_for(n), 256, 0, s>>>(v, n, nxt, rank, out_nxt, out_rank);
  }
  OH_TRY(exclusive_scan_u32(ctx, cnt, off64, (int64_t)n_keys + 1, nullptr, s));
  k_u64_to_u32<<<grid_for((int64_t)n_keys + 1), 256, 0, s>>>(off64, (int64_t)n_keys + 1, out_off);
  OH_HIP(hipGetLastError());
  int herr = 0;
  OH_TRY(d2h(&herr, err, 1, s));
  if (herr) { set_error("lists_build: key outside [0, n_keys)"); return OTTOHIP_ERANGE; }
  return 0;
}

struct ottohip_candidates {
  int64_t n_sessions = 0, n_cand = 0;
  uint64_t* off = nullptr;  // [S + 1]
  int32_t* next = nullptr;
  int16_t* ord = nullptr;
  uint16_t* flags = nullptr;
  void release() {
    dev_free(off);
    dev_free(next);
    dev_free(ord);
    dev_free(flags);
    off = nullptr; next = nullptr; ord = nullptr; flags = nullptr;
  }
};

int ottohip_candidates_generate(ottohip_ctx* ctx, const int64_t* session_offsets, int64_t n_sessions,
                                const int32_t* aid, const int32_t* ts, const int8_t* type,
                                const ottohip_cand_lists* lists, const int32_t* session_cl,
                                ottohip_candidates** out, void* stream) {
  if (!ctx || !lists || !out || n_sessions < 0 || (n_sessions > 0 && (!session_offsets || !aid || !ts || !type))) {
    set_error("candidates_generate: bad arguments"); return OTTOHIP_EINVAL;
  }
  *out = nullptr;
  hipStream_t s = S(stream);
  OH_HIP(hipSetDevice(ctx->device));
  CandLists L;
  for (int q = 0; q < CS_SRC; ++q) {
    L.off[q] = lists->off[q]; L.nxt[q] = lists->nxt[q]; L.rank[q] = lists->rank[q];
    if (L.off[q] && (!L.nxt[q] || !L.rank[q])) { set_error("candidates_generate: list %d incomplete", q); return OTTOHIP_EINVAL; }
  }
  L.n_items = lists->n_items;
  L.pop_off = lists->pop_off; L.pop_aid = lists->pop_aid; L.n_clusters = lists->pop_off ? lists->n_clusters : 0;
  ottohip_candidates* C = new ottohip_candidates();
  C->n_sessions = n_sessions;
  auto fail = [&](int rc) { C->release(); delete C; return rc; };
  const int64_t Sn = n_sessions;
  if (dev_alloc(reinterpret_cast<void**>(&C->off), (Sn + 1) * sizeof(uint64_t), "cand_off") != hipSuccess) return fail(OTTOHIP_ENOMEM);
  if (Sn == 0) {
    OH_HIP(hipMemsetAsync(C->off, 0, sizeof(uint64_t), s));
    *out = C;
    return 0;
  }
  int64_t E = 0;
  OH_TRY(d2h(&E, session_offsets + Sn, 1, s));
  Workspace& ws = ctx->ws;
  KeptAid* kept;
  uint32_t *n_kept, *n_cand, *n_ovf;
  int32_t* ovf;
  uint64_t* tot;
  int* err;
  int rc;
  if ((rc = ws.get("cs_kept", (size_t)std::max<int64_t>(E, 1), &kept)) ||
      (rc = ws.get("cs_nkept", (size_t)Sn, &n_kept)) || (rc = ws.get("cs_ncand", (size_t)Sn + 1, &n_cand)) ||
      (rc = ws.get("cs_novf", 1, &n_ovf)) || (rc = ws.get("cs_ovf", (size_t)Sn, &ovf)) ||
      (rc = ws.get("cs_tot", 1, &tot)) || (rc = ws.get("cs_err", 1, &err)))
    return fail(rc);
  hipMemsetAsync(err, 0, sizeof(int), s);
  static const int dbg = getenv("OTTOHIP_CAND_DBG") ? atoi(getenv("OTTOHIP_CAND_DBG")) : 0;  // profiling ablations
  // per-aid merged source lists (once per call)
  MergedLists M;
  M.n_items = L.n_items;
  M.pop_off = L.pop_off; M.pop_aid = L.pop_aid; M.n_clusters = L.n_clusters;
  {
    uint32_t *tot_e, *ucnt, *eoff32;
    uint16_t* pc;
    uint64_t *eoff, *etot;
    int32_t* mx;
    uint16_t* mbr;
    const int64_t NI = std::max<int32_t>(L.n_items, 1);
    if ((rc = ws.get("ml_tot", (size_t)NI + 1, &tot_e)) || (rc = ws.get("ml_eoff", (size_t)NI + 1, &eoff)) ||
        (rc = ws.get("ml_eoff32", (size_t)NI + 1, &eoff32)) || (rc = ws.get("ml_ucnt", (size_t)NI, &ucnt)) ||
        (rc = ws.get("ml_etot", 1, &etot)) || (rc = ws.get("ml_pc", (size_t)NI * ML_TH, &pc)))
      return fail(rc);
    int ph0 = ctx->begin("cand_merge_lists", s, 0);
    hipMemsetAsync(tot_e + NI, 0, 4, s);
    k_ml_total<<<grid_for(NI), 256, 0, s>>>(L, tot_e);
    if ((rc = exclusive_scan_u32(ctx, tot_e, eoff, NI + 1, etot, s))) return fail(rc);
    uint64_t ne = 0;
    if ((rc = d2h(&ne, etot, 1, s))) return fail(rc);
    if (ne >= ((uint64_t)1 << 32)) { set_error("candidates_generate: > 2^32 list entries"); return fail(OTTOHIP_ELIMIT); }
    if ((rc = ws.get("ml_x", (size_t)std::max<uint64_t>(ne, 1), &mx)) ||
        (rc = ws.get("ml_br", (size_t)std::max<uint64_t>(ne, 1), &mbr)))
      return fail(rc);
    k_u64_to_u32<<<grid_for(NI + 1), 256, 0, s>>>(eoff, NI + 1, eoff32);
    k_ml_build<<<(unsigned)ceil_div(NI, 4), 256, 0, s>>>(L, eoff32, mx, mbr, ucnt, pc, err);
    ctx->end(ph0, s);
    M.eoff = eoff32; M.ucnt = ucnt; M.pc = pc; M.mx = mx; M.mbr = mbr;
  }
  int ph = ctx->begin("cand_aids", s, 9.0 * E);
  hipMemsetAsync(n_ovf, 0, sizeof(uint32_t), s);
  hipMemsetAsync(n_cand + Sn, 0, sizeof(uint32_t), s);
  k_cand_aids<<<(unsigned)Sn, 64, 0, s>>>(session_offsets, Sn, aid, ts, type, kept, n_kept, err);
  ctx->end(ph, s);
  ph = ctx->begin("cand_build", s, 0);
  constexpr int W = 2, HC1 = 1024, HC2 = 4096;
  // per-session pool regions from an upper bound (tier-1 table size at most), one build pass
  uint32_t* ub;
  uint64_t *pool_off, *ptot;
  if ((rc = ws.get("cs_ub", (size_t)Sn, &ub)) || (rc = ws.get("cs_pool_off", (size_t)Sn + 1, &pool_off)) ||
      (rc = ws.get("cs_ptot", 1, &ptot)))
    return fail(rc);
  uint32_t* ubx;
  if ((rc = ws.get("cs_ubx", (size_t)Sn, &ubx))) return fail(rc);
  k_cand_bound<<<grid_for(Sn), 256, 0, s>>>(session_offsets, Sn, kept, n_kept, session_cl, M, (uint32_t)HC1, ub, ubx,
                                             (uint32_t)HC2);
  if ((rc = exclusive_scan_u32(ctx, ub, pool_off, Sn, ptot, s))) return fail(rc);
  uint64_t npool = 0;
  if ((rc = d2h(&npool, ptot, 1, s))) return fail(rc);
  int32_t* p_next;
  int16_t* p_ord;
  uint16_t* p_flags;
  const size_t pcap = (size_t)std::max<uint64_t>(npool, 1);
  if ((rc = ws.get("cs_pool_next", pcap, &p_next)) || (rc = ws.get("cs_pool_ord", pcap, &p_ord)) ||
      (rc = ws.get("cs_pool_flags", pcap, &p_flags)))
    return fail(rc);
  // tables sized by the session's bound (OTTOHIP_CAND_TIER=0: every session in a 1024-slot table first): the
  // smaller tables hold more waves per CU (69 % of the config-5 sessions have a bound <= 256, 8 % above 1024)
  static const bool tiers = !(getenv("OTTOHIP_CAND_TIER") && !strcmp(getenv("OTTOHIP_CAND_TIER"), "0"));
  if (tiers) {
    int64_t* tl;
    uint32_t* tc;
    if ((rc = ws.get("cs_tier", (size_t)Sn * 3, &tl)) || (rc = ws.get("cs_tierc", 3, &tc))) return fail(rc);
    OH_HIP(hipMemsetAsync(tc, 0, 3 * sizeof(uint32_t), s));
    k_cand_tier<<<(unsigned)ceil_div(Sn, 256), 256, 0, s>>>(ubx, Sn, tl, tc, ovf, n_ovf);
    uint32_t h3[3];
    if ((rc = d2h(h3, tc, 3, s))) return fail(rc);
    if (h3[0])
      k_cand_build<256, 4><<<(unsigned)ceil_div((int64_t)h3[0], 4), 256, 0, s>>>(
          session_offsets, tl, h3[0], kept, n_kept, session_cl, M, 1, n_cand, pool_off, p_next, p_ord, p_flags, ovf,
          n_ovf, dbg);
    if (h3[1])
      k_cand_build<512, 2><<<(unsigned)ceil_div((int64_t)h3[1], 2), 128, 0, s>>>(
          session_offsets, tl + Sn, h3[1], kept, n_kept, session_cl, M, 1, n_cand, pool_off, p_next, p_ord, p_flags,
          ovf, n_ovf, dbg);
    if (h3[2])
      k_cand_build<HC1, W><<<(unsigned)ceil_div((int64_t)h3[2], W), 64 * W, 0, s>>>(
          session_offsets, tl + 2 * Sn, h3[2], kept, n_kept, session_cl, M, 1, n_cand, pool_off, p_next, p_ord,
          p_flags, ovf, n_ovf, dbg);
  } else {
    k_cand_build<HC1, W><<<(unsigned)ceil_div(Sn, W), 64 * W, 0, s>>>(session_offsets, nullptr, Sn, kept, n_kept,
                                                                       session_cl, M, 1, n_cand, pool_off, p_next, p_ord,
                                                                       p_flags, ovf, n_ovf, dbg);
  }
  uint32_t novf = 0;
  int herr = 0;
  if ((rc = d2h(&novf, n_ovf, 1, s)) || (rc = d2h(&herr, err, 1, s))) return fail(rc);
  if (herr & 1) { set_error("candidates_generate: a session has more than %d events", CS_MAXE); return fail(OTTOHIP_ELIMIT); }
  if (herr & 4) { set_error("candidates_generate: an aid has more than %d list entries", ML_MAX); return fail(OTTOHIP_ELIMIT); }
  int32_t* q_next = p_next;
  int16_t* q_ord = p_ord;
  uint16_t* q_flags = p_flags;
  if (novf) {  // sessions beyond the 1024-slot tier: the 4096-slot tier, regions in an overflow pool
    int64_t* ovf64 = nullptr;
    uint32_t* n_ovf2 = nullptr;
    int32_t* ovf2 = nullptr;
    if ((rc = ws.get("cs_novf2", 1, &n_ovf2)) || (rc = ws.get("cs_ovf2", (size_t)novf, &ovf2)) ||
        (rc = ws.get("cs_ovf64", (size_t)novf, &ovf64)) || (rc = ws.get("cs_q_next", (size_t)novf * HC2, &q_next)) ||
        (rc = ws.get("cs_q_ord", (size_t)novf * HC2, &q_ord)) || (rc = ws.get("cs_q_flags", (size_t)novf * HC2, &q_flags)))
      return fail(rc);
    std::vector<int32_t> ho(novf);
    if ((rc = d2h(ho.data(), ovf, novf, s))) return fail(rc);
    std::sort(ho.begin(), ho.end());
    std::vector<int64_t> ho64(ho.begin(), ho.end());
    OH_HIP(hipMemcpyAsync(ovf, ho.data(), novf * sizeof(int32_t), hipMemcpyHostToDevice, s));
    OH_HIP(hipMemcpyAsync(ovf64, ho64.data(), novf * sizeof(int64_t), hipMemcpyHostToDevice, s));
    OH_HIP(hipMemsetAsync(n_ovf2, 0, sizeof(uint32_t), s));
    k_cand_ovf_src<<<grid_for(novf), 256, 0, s>>>(ovf, novf, (uint32_t)HC2, pool_off);
    k_cand_build<HC2, 1><<<novf, 64, 0, s>>>(session_offsets, ovf64, novf, kept, n_kept, session_cl, M, 1, n_cand,
                                             pool_off, q_next, q_ord, q_flags, ovf2, n_ovf2, dbg);
    uint32_t novf2 = 0;
    if ((rc = d2h(&novf2, n_ovf2, 1, s))) return fail(rc);
    if (novf2) { set_error("candidates_generate: %u sessions exceed 4096 candidates", novf2); return fail(OTTOHIP_ELIMIT); }
  }
  if (dbg & 8) {  // (profiling) per-session candidate count distribution, then the uncapped bound's, then both
    std::vector<uint32_t> hc(Sn), hb(Sn);
    if ((rc = d2h(hc.data(), n_cand, (size_t)Sn, s))) return fail(rc);
    k_cand_bound<<<grid_for(Sn), 256, 0, s>>>(session_offsets, Sn, kept, n_kept, session_cl, M, 1u << 30, ub);
    if ((rc = d2h(hb.data(), ub, (size_t)Sn, s))) return fail(rc);
    int64_t jb[6][4] = {};
    auto bin4 = [](uint32_t v) { return v <= 256 ? 0 : v <= 512 ? 1 : v <= 1024 ? 2 : 3; };
    auto bin6 = [](uint32_t v) { return v <= 256 ? 0 : v <= 512 ? 1 : v <= 1024 ? 2 : v <= 1536 ? 3 : v <= 2048 ? 4 : 5; };
    int64_t sb[6] = {0, 0, 0, 0, 0, 0};
    for (int64_t i = 0; i < Sn; ++i) {
      const uint32_t v = hb[i];
      sb[v <= 128 ? 0 : v <= 256 ? 1 : v <= 384 ? 2 : v <= 512 ? 3 : v <= 1024 ? 4 : 5]++;
      jb[bin6(v)][bin4(hc[i])]++;
    }
    fprintf(stderr, "[ottohip] candidate bound per session: <=128 %lld, <=256 %lld, <=384 %lld, <=512 %lld, <=1024 %lld, "
            "more %lld\n", (long long)sb[0], (long long)sb[1], (long long)sb[2], (long long)sb[3], (long long)sb[4],
            (long long)sb[5]);
    for (int a = 0; a < 6; ++a)
      fprintf(stderr, "[ottohip] bound bin %d -> count bins %lld %lld %lld %lld\n", a, (long long)jb[a][0],
              (long long)jb[a][1], (long long)jb[a][2], (long long)jb[a][3]);
    int64_t nb[6] = {0, 0, 0, 0, 0, 0};
    for (uint32_t v : hc) nb[v <= 128 ? 0 : v <= 256 ? 1 : v <= 384 ? 2 : v <= 512 ? 3 : v <= 1024 ? 4 : 5]++;
    fprintf(stderr, "[ottohip] candidates per session: <=128 %lld, <=256 %lld, <=384 %lld, <=512 %lld, <=1024 %lld, "
            "more %lld\n", (long long)nb[0], (long long)nb[1], (long long)nb[2], (long long)nb[3], (long long)nb[4],
            (long long)nb[5]);
  }
  if ((rc = exclusive_scan_u32(ctx, n_cand, C->off, Sn + 1, tot, s))) return fail(rc);
  uint64_t nc = 0;
  if ((rc = d2h(&nc, tot, 1, s))) return fail(rc);
  C->n_cand = (int64_t)nc;
  const size_t cap = (size_t)std::max<uint64_t>(nc, 1);
  if (dev_alloc(reinterpret_cast<void**>(&C->next), cap * 4, "cand_next") ||
      dev_alloc(reinterpret_cast<void**>(&C->ord), cap * 2, "cand_ord") ||
      dev_alloc(reinterpret_cast<void**>(&C->flags), cap * 2, "cand_flags"))
    return fail(OTTOHIP_ENOMEM);
  k_cand_compact<<<(unsigned)ceil_div(Sn, 4), 256, 0, s>>>(pool_off, C->off, Sn, p_next, p_ord, p_flags, q_next, q_ord,
                                                          q_flags, C->next, C->ord, C->flags);
  if (hipGetLastError() != hipSuccess) { set_error("k_cand_build launch failed"); return fail(OTTOHIP_EHIP); }
  ctx->end(ph, s);
  *out = C;
  return 0;
}

int ottohip_candidates_info(const ottohip_candidates* c, int64_t* n_sessions, int64_t* n_cand) {
  if (!c) { set_error("candidates_info: NULL"); return OTTOHIP_EINVAL; }
  if (n_sessions) *n_sessions = c->n_sessions;
  if (n_cand) *n_cand = c->n_cand;
  return 0;
}

int ottohip_candidates_copy(const ottohip_candidates* c, uint64_t* off, int32_t* aid_next, int16_t* ts_order,
                            uint16_t* flags, void* stream) {
  if (!c) { set_error("candidates_copy: NULL"); return OTTOHIP_EINVAL; }
  hipStream_t s = S(stream);
  if (off) OH_HIP(hipMemcpyAsync(off, c->off, (c->n_sessions + 1) * 8, hipMemcpyDeviceToDevice, s));
  if (c->n_cand > 0) {
    if (aid_next) OH_HIP(hipMemcpyAsync(aid_next, c->next, c->n_cand * 4, hipMemcpyDeviceToDevice, s));
    if (ts_order) OH_HIP(hipMemcpyAsync(ts_order, c->ord, c->n_cand * 2, hipMemcpyDeviceToDevice, s));
    if (flags) OH_HIP(hipMemcpyAsync(flags, c->flags, c->n_cand * 2, hipMemcpyDeviceToDevice, s));
  }
  return 0;
}

int ottohip_candidates_view(const ottohip_candidates* c, const uint64_t** off, const int32_t** aid_next,
                            const int16_t** ts_order, const uint16_t** flags) {
  if (!c) { set_error("candidates_view: NULL"); return OTTOHIP_EINVAL; }
  if (off) *off = c->off;
  if (aid_next) *aid_next = c->next;
  if (ts_order) *ts_order = c->ord;
  if (flags) *flags = c->flags;
  return 0;
}

void ottohip_candidates_free(ottohip_candidates* c) {
  if (!c) return;
  (void)hipDeviceSynchronize();
  c->release();
  delete c;
}

int ottohip_candidates_recall(ottohip_ctx* ctx, const ottohip_candidates* c, const int64_t* lab_off,
                              const int32_t* lab_aid, uint32_t src_mask, int max_k, int64_t* sums_out, void* stream) {
  if (!ctx || !c || !sums_out || (c->n_sessions > 0 && !lab_off)) { set_error("candidates_recall: bad args"); return OTTOHIP_EINVAL; }
  for (int i = 0; i < 15; ++i) sums_out[i] = 0;
  if (c->n_sessions == 0) return 0;
  hipStream_t s = S(stream);
  OH_HIP(hipSetDevice(ctx->device));
  unsigned long long* sums;
  int* err;
  OH_TRY(ctx->ws.get("rc_sums", 256 * 16, &sums));
  OH_TRY(ctx->ws.get("rc_err", 1, &err));
  OH_HIP(hipMemsetAsync(sums, 0, 256 * 16 * 8, s));
  OH_HIP(hipMemsetAsync(err, 0, sizeof(int), s));
  k_cand_recall<<<(unsigned)c->n_sessions, 64, 0, s>>>(c->off, c->next, c->flags, c->n_sessions, lab_off, lab_aid,
                                                       src_mask, max_k, sums, err);
  OH_HIP(hipGetLastError());
  std::vector<unsigned long long> h(256 * 16);
  OH_TRY(d2h(h.data(), sums, h.size(), s));
  int herr = 0;
  OH_TRY(d2h(&herr, err, 1, s));
  if (herr) { set_error("candidates_recall: a session has more than %d candidates", RC_MAX); return OTTOHIP_ELIMIT; }
  for (int k = 0; k < 256; ++k)
    for (int i = 0; i < 15; ++i) sums_out[i] += (int64_t)h[(size_t)k * 16 + i];
  return 0;
}

}  // extern "C"

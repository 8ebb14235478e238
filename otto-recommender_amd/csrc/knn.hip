// Word2Vec top-K neighbour search on gfx950 MFMA (model/w2vec_aids.py:125-173).
//
// The reference searches a faiss IVFFlat index (nlist 100, nprobe 3, METRIC_L2) for the first
// 600k vocabulary rows, k = 20 (w2vec_aids.py:98-110,164). This engine is exact:
//   1. k_knn_pack: items -> bf16 [V x 128]; columns [0, dim) = v, columns dim, dim+1 = hi/lo
//      bf16 split of -|v|^2 / 2, rest 0. Queries -> bf16 [Q x 128] with 1, 1 in those columns.
//      One MFMA product then gives s = q.v - |v|^2/2, and |q - v|^2 = |q|^2 - 2 s ranks like -s.
//   2. k_knn_main<2> (pre-pass, every 16th item tile): a lower bound of each query's KN_C-th
//      best score. k_knn_main<0>: v_mfma_f32_32x32x16_bf16 with items as A (256-item tiles
//      streamed into two LDS slots by LDS-DMA, XOR-swizzled 16-B chunks) and 64 queries per
//      wave held in registers as B; after a lane swap each lane owns one query and keeps its
//      KN_C best (score, item) in a sorted register list, inserting only above the bound.
//   3. k_knn_rerank: one wave per query recomputes |q - v|^2 exactly in fp32 for the KN_C
//      candidates and sorts by (d2, index): the top-k rows and their exact squared distances.
#include <cmath>
#include <cstdlib>
#include "common.h"

namespace ottohip {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int KN_KD = 128;               // padded K (bf16 per row)
constexpr int KN_CH = KN_KD * 2 / 16;    // 16-B chunks per row (16)
constexpr int KN_QW = 64;                // queries per wave (two 32-column MFMA blocks)
constexpr int KN_WAVES = 8;
constexpr int KN_T = 64 * KN_WAVES;      // 512 threads
constexpr int KN_QB = KN_QW * KN_WAVES;  // 256 queries per workgroup
constexpr int KN_IT = 256;               // items per LDS tile (8 row-blocks of 32)
constexpr int KN_C = 24;                 // candidates per query (k = 20 plus a rerank margin)
constexpr int KN_KMAX = KN_C - 4;        // largest k: 4 candidates of margin for the bf16 scores' error
constexpr int KN_CAND = 64;              // rerank width (2 * KN_C candidates, padded)
constexpr int PRE_STRIDE = 16;           // threshold pre-pass: every 16th item tile

__device__ __forceinline__ uint16_t f2bf(float f) {  // round to nearest even
  uint32_t u = __float_as_uint(f);
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}
__device__ __forceinline__ float bf2f(uint16_t b) { return __uint_as_float((uint32_t)b << 16); }

// items (rows of emb) -> packed bf16 with the -|v|^2/2 columns; or queries (rows[q]) with 1, 1
__global__ void k_knn_pack(const float* __restrict__ emb, int64_t n, int dim, const int32_t* __restrict__ rows,
                           int64_t n_items, int is_query, uint16_t* __restrict__ out, int* __restrict__ err) {
  const int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (i >= n) return;
  const int l = threadIdx.x & 63;
  int64_t src = rows ? rows[i] : i;
  if (src < 0 || src >= n_items) {  // never read outside the embedding table
    if (l == 0 && err) atomicOr(err, 1);
    src = 0;
  }
  const float* v = emb + src * dim;
  float ss = 0.f;
  for (int d = l; d < KN_KD; d += 64) {
    float x = d < dim ? v[d] : 0.f;
    ss += x * x;
    out[i * KN_KD + d] = d < dim ? f2bf(x) : 0;
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) ss += __shfl_xor(ss, o);
  if (l == 0) {
    if (is_query) {
      out[i * KN_KD + dim] = f2bf(1.f);
      out[i * KN_KD + dim + 1] = f2bf(1.f);
    } else {
      const float nh = -0.5f * ss;
      const uint16_t hi = f2bf(nh);
      out[i * KN_KD + dim] = hi;
      out[i * KN_KD + dim + 1] = f2bf(nh - bf2f(hi));
    }
  }
}

// 64 queries per wave: two 32x32 output blocks (queries qbase + [0, 32) and qbase + [32, 64))
// share every item fragment; v_permlane32_swap then gives each lane ONE query with all 32 item
// scores of a row-block, so each query keeps a single register list of KN_C candidates.
// Item tiles of 256 items stream into two LDS slots by LDS-DMA (global_load_lds_dwordx4, 8 per
// thread per tile; the next tile is in flight while this one is scored): vmcnt + raw s_barrier,
// one barrier per 256 items.
constexpr int KN_RING = 2;
constexpr int KN_GL = KN_IT * KN_CH / KN_T;  // glds per thread per tile (8)

// MODE 0: full scan with top-KN_C inserts, the list starting at thr_io[q] (if given).
// MODE 1: ablation (scores only).  MODE 3: ablation without the item stream (timing only).
// MODE 2: threshold pre-pass over tiles 0, 16, 32, ... (never the last, partial tile): the
//   KN_C largest 32-item block maxima of the sampled tiles, a sorted list per query; KN_C
//   distinct blocks each hold an item scoring >= their maximum, so the KN_C-th of them is a lower
//   bound of the query's KN_C-th best score -> thr_io[q]. MODE 0 then inserts only items above it.
// KS = k-steps of 16 over the packed row: ceil((dim + 2) / 16) rounded up to 7 or 8 (dim 100 -> 7,
// so the zero padding of columns 112..127 is neither streamed nor multiplied).
// BUF (MODE 0): the register list keeps scores only (one v_med3 per slot per insert instead of a
//   compare, a med3 and two index selects); every inserted (score, item) is appended to the query's
//   buffer cbuf[q * KN_BCAP ..] in insertion order and ncand[q] counts them. The final list is the
//   first KN_C of the inserted candidates by (score desc, insertion order) -- exactly the candidates the
//   index list would hold -- which k_knn_rerank_buf selects before the exact rerank.
typedef short s16x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ s16x4 lo4(const bf16x8& v) {  // the low 4 bf16 of a fragment as the x8 MFMA's operand
  const uint4 u = __builtin_bit_cast(uint4, v);
  return __builtin_bit_cast(s16x4, make_uint2(u.x, u.y));
}
// HALF: the last k-step covers 8 columns with v_mfma_f32_32x32x8_bf16 (dim + 2 <= 16 (KS - 1) + 8: dim 100 -> 104
//   columns instead of 112; the 14th chunk of a row is neither streamed nor multiplied).
constexpr int KN_BCAP = 512;  // inserted candidates kept per query (overflow: the search reruns with index lists)
template <int ABL, int KS, bool BUF = false, bool HALF = false>
__global__ __launch_bounds__(KN_T) void k_knn_main(const uint4* __restrict__ items, int64_t V,
                                                  const uint4* __restrict__ queries, int64_t nq,
                                                  uint32_t* __restrict__ cand, float* __restrict__ thr_io,
                                                  int pre_stride, uint2* __restrict__ cbuf = nullptr,
                                                  uint32_t* __restrict__ ncand = nullptr) {
  __shared__ uint4 ring[KN_RING * KN_IT * KN_CH];  // 2 x 64 KiB, the only LDS object
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, r = l & 31, h = l >> 5;
  const int64_t qbase = (int64_t)blockIdx.x * KN_QB + w * 64;
  const auto probe = __builtin_amdgcn_permlane32_swap((unsigned)l, (unsigned)(l + 64), false, false);
  const bool semA = __builtin_amdgcn_readfirstlane(probe[1]) == 32u;  // vsrc lane 0 received vdst lane 32
  const int64_t q = semA ? qbase + l : qbase + ((l + 32) & 63);
  const int offx = semA ? 0 : 4, offy = 4 - offx;
  static_assert(KS >= 1 && KS <= KN_KD / 16, "k-steps");
  bf16x8 bqa[KS], bqb[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int64_t qa = qbase + r, qb = qbase + 32 + r;
    uint4 ua = make_uint4(0, 0, 0, 0), ub = make_uint4(0, 0, 0, 0);
    const bool tail = HALF && s == KS - 1;  // 8 columns: lane half h holds columns 16 s + 4 h .. + 3
    if (qa < nq) ua = queries[qa * KN_CH + 2 * s + (tail ? 0 : h)];
    if (qb < nq) ub = queries[qb * KN_CH + 2 * s + (tail ? 0 : h)];
    if (tail) {
      ua = h ? make_uint4(ua.z, ua.w, 0u, 0u) : make_uint4(ua.x, ua.y, 0u, 0u);
      ub = h ? make_uint4(ub.z, ub.w, 0u, 0u) : make_uint4(ub.x, ub.y, 0u, 0u);
    }
    bqa[s] = __builtin_bit_cast(bf16x8, ua);
    bqb[s] = __builtin_bit_cast(bf16x8, ub);
  }
  float sc[KN_C];
  uint32_t ix[KN_C];
#pragma unroll
  for (int j = 0; j < KN_C; ++j) { sc[j] = -INFINITY; ix[j] = 0xFFFFFFFFu; }
  float thr = -INFINITY;
  constexpr bool PRE = ABL == 2;
  const int64_t nTall = ceil_div(V, KN_IT);
  const int64_t nT = PRE ? (nTall - 1 + pre_stride - 1) / pre_stride : nTall;  // tiles scanned
  if (ABL == 0 && thr_io) {  // start the list at the pre-pass bound (placeholders with no index)
    const float b = q < nq ? thr_io[q] : -INFINITY;
#pragma unroll
    for (int j = 0; j < KN_C; ++j) sc[j] = b;
    thr = b;
  }
  // LDS chunk p = u*512 + tid holds item row p>>4, source chunk (p & 15) ^ (row & 15);
  // rows past V read row V-1 (valid memory; their scores are masked below); source chunks past
  // the KS k-steps (zero padding) are not fetched and never read
  auto issue = [&](int64_t t) {
    if (ABL == 3 && t >= KN_RING) return;  // ablation: item stream off after the first tiles (timing only)
    uint4* dst = ring + (int)(t % KN_RING) * (KN_IT * KN_CH);
    const int64_t tt = PRE ? t * pre_stride : t;
#pragma unroll
    for (int u = 0; u < KN_GL; ++u) {
      const int p = u * KN_T + tid, row = p >> 4, c = p & 15;
      int64_t item = tt * KN_IT + row;
      if (item >= V) item = V - 1;
      if (KS < KN_KD / 16 && (c ^ (row & 15)) >= 2 * KS - (HALF ? 1 : 0)) continue;
      __builtin_amdgcn_global_load_lds(items + item * KN_CH + (c ^ (row & 15)), dst + u * KN_T + w * 64, 16, 0, 0);
    }
  };
  // the list is kept sorted descending, so the threshold is its last score and an insert is a
  // branch-free shift: slot j takes slot j-1 if s beats it, else s if s beats slot j (score: one
  // v_med3 of (sc[j-1], s, sc[j]); index: two selects). A lane-dependent "replace the minimum"
  // slot becomes a compare/select chain over every slot instead.
  uint32_t nbuf = 0;
  auto insert = [&](float s_, uint32_t item) __attribute__((always_inline)) {
    if constexpr (BUF) {
      if (!PRE) {
        if (q < nq && nbuf < (uint32_t)KN_BCAP)  // padding lanes past nq keep no buffer
          cbuf[(size_t)q * KN_BCAP + nbuf] = make_uint2(__float_as_uint(s_), item);
        ++nbuf;
#pragma unroll
        for (int jj = 0; jj < KN_C - 1; ++jj) {  // scores only: slot j takes max(slot j-1 clipped by s, ...)
          const int j = KN_C - 1 - jj;
          sc[j] = __builtin_amdgcn_fmed3f(sc[j - 1], s_, sc[j]);
        }
        sc[0] = fmaxf(sc[0], s_);
        thr = sc[KN_C - 1];
        return;
      }
    }
    bool cj = s_ > sc[KN_C - 1];
#pragma unroll
    for (int jj = 0; jj < KN_C - 1; ++jj) {  // downwards: slot j - 1 still holds its old value
      const int j = KN_C - 1 - jj;
      const bool cp = s_ > sc[j - 1];
      uint32_t a = ix[j - 1], b = ix[j];
      asm("" : "+v"(a), "+v"(b));  // keeps the selects on values: a select of the two slots' addresses
                                   // would leave ix[] as a memory array (LDS / scratch)
      ix[j] = cp ? a : (cj ? item : b);
      sc[j] = __builtin_amdgcn_fmed3f(sc[j - 1], s_, sc[j]);
      cj = cp;
    }
    ix[0] = cj ? item : ix[0];
    sc[0] = fmaxf(sc[0], s_);
    thr = sc[KN_C - 1];
  };
  // one 32-item row-block's scores (accumulators pA = queries qbase + [0, 32), pB = + [32, 64))
  // into the lists. Per-lane maxima first: swapping the two maxima gives this lane's query maximum
  // over the 32 rows, and the 16-register redistribution runs only when some lane has a candidate.
  auto drain = [&](f32x16& pA, f32x16& pB, int64_t ib) __attribute__((always_inline)) {
    float mA = pA[0], mB = pB[0];
#pragma unroll
    for (int i = 1; i < 16; ++i) { mA = fmaxf(mA, pA[i]); mB = fmaxf(mB, pB[i]); }
    const auto msw = __builtin_amdgcn_permlane32_swap(__float_as_uint(mA), __float_as_uint(mB), false, false);
    const float m = fmaxf(__uint_as_float(msw[0]), __uint_as_float(msw[1]));
    if (ABL == 1 || ABL == 3) { thr = fmaxf(thr, m * 1e-30f); return; }  // ablation builds: no candidate handling
    if (PRE) {  // the sampled blocks' KN_C largest maxima (sorted list, no indices)
      if (m > thr) insert(m, 0u);
      return;
    }
    if (__ballot(m > thr)) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {  // pA -> rows + offx, pB -> rows + offy of this lane's query
        const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(pA[i]), __float_as_uint(pB[i]), false, false);
        pA[i] = __uint_as_float(sw[0]);
        pB[i] = __uint_as_float(sw[1]);
      }
    }
    if (m > thr) {
      // this lane's 32 scores of the block as unique keys: the row slot j (0..31) replaces the
      // 5 low mantissa bits (32 ulp, far below the bf16 inputs' error), so the best remaining
      // candidate is one max over keys below the last one taken, and its key names its row
      // (the keys overwrite the drained accumulators in place)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        pA[i] = __uint_as_float((__float_as_uint(pA[i]) & ~31u) | (uint32_t)i);
        pB[i] = __uint_as_float((__float_as_uint(pB[i]) & ~31u) | (uint32_t)(16 + i));
      }
      // the lane's two best keys in one pass (k2 = med3(k1, k2, x) before k1 = max(k1, x)); a
      // block rarely holds a third candidate for one query, so the general "best key below the
      // last taken" loop runs only after the second was inserted
      float k1 = -INFINITY, k2 = -INFINITY;
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        k2 = __builtin_amdgcn_fmed3f(k1, k2, pA[j]);
        k1 = fmaxf(k1, pA[j]);
        k2 = __builtin_amdgcn_fmed3f(k1, k2, pB[j]);
        k1 = fmaxf(k1, pB[j]);
      }
      float last = INFINITY;
      for (int it = 0;; ++it) {  // it is the same on every lane still looping
        float cur;
        if (it == 0) {
          cur = k1;
        } else if (it == 1) {
          cur = k2;
        } else {
          cur = -INFINITY;
#pragma unroll
          for (int j = 0; j < 16; ++j) {
            cur = fmaxf(cur, pA[j] < last ? pA[j] : -INFINITY);
            cur = fmaxf(cur, pB[j] < last ? pB[j] : -INFINITY);
          }
        }
        if (!(cur > thr)) break;
        const uint32_t j = __float_as_uint(cur) & 31u, i = j & 15u;
        const int64_t item = ib + (i & 3) + 8 * (i >> 2) + (j < 16 ? offx : offy);
        if (item < V) insert(cur, (uint32_t)item);
        last = cur;
      }
    }
  };
  // Row-blocks are software-pipelined over two accumulator sets: block b accumulates in set b & 1
  // while block b - 1 (the other set) is drained, so the drain's VALU work issues between block b's
  // MFMAs instead of after them. A tile holds an even number of blocks, so block 0 of tile t drains
  // block NBLK - 1 of tile t - 1 (set 1, -inf before the first tile).
  constexpr int NBLK = KN_IT / 32;
  static_assert(NBLK % 2 == 0, "even number of row-blocks per tile");
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 16; ++i) { acc[1][0][i] = -INFINITY; acc[1][1][i] = -INFINITY; }
  static_assert(KN_RING == 2, "double-buffered tiles: one tile in flight while the other is scored");
  issue(0);
  for (int64_t t = 0; t < nT; ++t) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's share of tile t has landed
    __builtin_amdgcn_s_barrier();  // tile t visible to all waves; slot (t+1) % 2 = (t-1) % 2 is free
    if (t + 1 < nT) issue(t + 1);
    const uint4* T = ring + (int)(t & 1) * (KN_IT * KN_CH);
    // item fragments (one per (row-block, k-step) step, shared by the two query halves' MFMAs)
    // are read three steps ahead
    constexpr int NSTEP = NBLK * KS;
    constexpr int AHEAD = 3;
    bf16x8 F[NSTEP];
    auto ld = [&](int g) __attribute__((always_inline)) {
      const int row = (g / KS) * 32 + r, s_ = g % KS;
      if (HALF && s_ == KS - 1) {  // the 8-column step: this lane half's 8 bytes of chunk 2 s_
        const uint2 x = reinterpret_cast<const uint2*>(T)[(row * KN_CH + ((2 * s_) ^ (row & 15))) * 2 + h];
        F[g] = __builtin_bit_cast(bf16x8, make_uint4(x.x, x.y, 0u, 0u));
      } else {
        F[g] = __builtin_bit_cast(bf16x8, T[row * KN_CH + ((2 * s_ + h) ^ (row & 15))]);
      }
    };
#pragma unroll
    for (int g = 0; g < AHEAD; ++g) ld(g);
#pragma clang loop unroll(full)
    for (int g = 0; g < NSTEP; ++g) {
      const int b = g / KS, s = g % KS, c = b & 1;
      if (g + AHEAD < NSTEP) ld(g + AHEAD);
      if (s == 0) { acc[c][0] = {}; acc[c][1] = {}; }
      if (HALF && s == KS - 1) {  // v_mfma_f32_32x32x8_bf16 over the last 8 columns
        const s16x4 fa = lo4(F[g]);
        acc[c][0] = __builtin_amdgcn_mfma_f32_32x32x8bf16_1k(fa, lo4(bqa[s]), acc[c][0], 0, 0, 0);
        acc[c][1] = __builtin_amdgcn_mfma_f32_32x32x8bf16_1k(fa, lo4(bqb[s]), acc[c][1], 0, 0, 0);
      } else {
        acc[c][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(F[g], bqa[s], acc[c][0], 0, 0, 0);
        acc[c][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(F[g], bqb[s], acc[c][1], 0, 0, 0);
      }
      if (s == KS - 1) drain(acc[c ^ 1][0], acc[c ^ 1][1], t * KN_IT + (int64_t)(b - 1) * 32);
    }
  }
  drain(acc[1][0], acc[1][1], (nT - 1) * KN_IT + (int64_t)(NBLK - 1) * 32);  // the last block
  if ((ABL == 1 || ABL == 3) && thr == 12345.f) ix[0] = 0;  // keep the ablated scores live
  if (PRE) {  // KN_C distinct blocks hold an item scoring >= their maximum: the KN_C-th largest
              // sampled block maximum is a lower bound of the query's KN_C-th best score
    if (q < nq) thr_io[q] = nextafterf(sc[KN_C - 1], -INFINITY);  // items tying the bound are still inserted
    return;
  }
  if constexpr (BUF) {
    if (q < nq) ncand[q] = nbuf;
    return;
  }
  if (q < nq) {
#pragma unroll
    for (int j = 0; j < KN_CAND; ++j) cand[q * KN_CAND + j] = j < KN_C ? ix[j] : 0xFFFFFFFFu;
  }
}

// BUF search: per query (one wave) the first KN_C inserted candidates by (score desc, insertion order):
// each lane ranks its buffer entries against all of them (keys unique by position), the entries of rank
// < KN_C go to cand[] in rank order; a query with more than KN_BCAP inserts sets *overflow
__global__ __launch_bounds__(256) void k_knn_select_buf(const uint2* __restrict__ cbuf,
                                                        const uint32_t* __restrict__ ncand, int64_t nq,
                                                        uint32_t* __restrict__ cand, int* __restrict__ overflow) {
  __shared__ uint64_t keys[4][KN_BCAP];
  const int64_t q = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int w = threadIdx.x >> 6;
  const uint32_t l = lane_id();
  if (q >= nq) return;
  const uint32_t nc = ncand[q];
  if (nc > (uint32_t)KN_BCAP) { if (l == 0) atomicOr(overflow, 1); return; }
  const uint2* b = cbuf + (size_t)q * KN_BCAP;
  for (uint32_t i = l; i < nc; i += 64) {  // ascending key = (score desc, position asc)
    const uint32_t sb = b[i].x;
    const uint32_t ord = (sb & 0x80000000u) ? ~sb : (sb | 0x80000000u);
    keys[w][i] = ((uint64_t)~ord << 32) | i;
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  for (uint32_t i = l; i < KN_CAND; i += 64) cand[q * KN_CAND + i] = 0xFFFFFFFFu;
  __builtin_amdgcn_wave_barrier();
  for (uint32_t i = l; i < nc; i += 64) {
    const uint64_t ki = keys[w][i];
    uint32_t r = 0;
    for (uint32_t j = 0; j < nc; ++j) r += keys[w][j] < ki ? 1u : 0u;
    if (r < (uint32_t)KN_C) cand[q * KN_CAND + r] = b[i].y;
  }
}

// one wave per query: exact fp32 |q - v|^2 of the 64 candidates, sorted by (d2, index)
__global__ __launch_bounds__(256) void k_knn_rerank(const float* __restrict__ emb, int64_t V, int dim,
                                                    const int32_t* __restrict__ qrows, int64_t nq,
                                                    const uint32_t* __restrict__ cand, int k,
                                                    int32_t* __restrict__ out_idx, float* __restrict__ out_d2) {
  const int64_t q = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (q >= nq) return;
  const uint32_t l = lane_id();
  const uint32_t c = cand[q * KN_CAND + l];
  int64_t qr = qrows ? qrows[q] : q;
  if (qr < 0 || qr >= V) qr = 0;  // flagged by k_knn_pack; the call returns an error
  const float* qv = emb + qr * dim;
  float d2 = INFINITY;
  if (c < (uint32_t)V) {
    const float* v = emb + (int64_t)c * dim;
    float acc = 0.f;
    if ((dim & 3) == 0) {  // rows are 16-B aligned: vector loads
      const float4* q4 = reinterpret_cast<const float4*>(qv);
      const float4* v4 = reinterpret_cast<const float4*>(v);
      for (int d = 0; d < dim / 4; ++d) {
        const float4 a = q4[d], b = v4[d];
        float t = a.x - b.x; acc = fmaf(t, t, acc);
        t = a.y - b.y; acc = fmaf(t, t, acc);
        t = a.z - b.z; acc = fmaf(t, t, acc);
        t = a.w - b.w; acc = fmaf(t, t, acc);
      }
    } else {
      for (int d = 0; d < dim; ++d) {
        const float t = qv[d] - v[d];
        acc = fmaf(t, t, acc);
      }
    }
    d2 = acc;
  }
  // bitonic sort of 64 (d2 bits, index) keys; d2 >= 0 so its bits order like the float
  uint64_t key = ((uint64_t)__float_as_uint(d2) << 32) | c;
#pragma unroll
  for (int kk = 2; kk <= 64; kk <<= 1) {
#pragma unroll
    for (int j = kk >> 1; j > 0; j >>= 1) {
      const uint64_t o = shfl64(key, (int)(l ^ (uint32_t)j));
      const bool up = (l & kk) == 0, lower = (l & j) == 0;
      key = (lower == up) ? (key < o ? key : o) : (key > o ? key : o);
    }
  }
  if ((int)l < k) {
    const uint32_t idx = (uint32_t)key;
    out_idx[q * k + l] = idx < (uint32_t)V ? (int32_t)idx : -1;
    out_d2[q * k + l] = __uint_as_float((uint32_t)(key >> 32));
  }
}

}  // namespace ottohip

using namespace ottohip;

extern "C" {

struct ottohip_knn_index {
  int device;
  int64_t n_items;
  int dim;
  const float* emb;      // caller-owned fp32 [n_items x dim]
  uint16_t* packed;      // bf16 [n_items x 128]
};

int ottohip_knn_index_create(ottohip_ctx* c, const float* emb, int64_t n_items, int dim,
                             ottohip_knn_index** out, void* stream) {
  if (!c || !emb || !out || n_items < 1 || dim < 1 || dim > KN_KD - 2 || n_items >= (int64_t)0xFFFFFFFFu) {
    set_error("knn_index_create: bad arguments (dim must be <= %d)", KN_KD - 2);
    return OTTOHIP_EINVAL;
  }
  Ctx* ctx = ctx_base(c);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  ottohip_knn_index* ix = new ottohip_knn_index();
  ix->device = ctx->device; ix->n_items = n_items; ix->dim = dim; ix->emb = emb;
  if (dev_alloc(reinterpret_cast<void**>(&ix->packed), (size_t)n_items * KN_KD * 2, "knn_packed") != hipSuccess) {
    delete ix; set_error("knn_index_create: allocation failed"); return OTTOHIP_ENOMEM;
  }
  k_knn_pack<<<(unsigned)ceil_div(n_items * 64, 256), 256, 0, s>>>(emb, n_items, dim, nullptr, n_items, 0, ix->packed,
                                                                   nullptr);
  OH_HIP(hipGetLastError());
  *out = ix;
  return 0;
}

void ottohip_knn_index_free(ottohip_knn_index* ix) {
  if (!ix) return;
  (void)hipSetDevice(ix->device);
  (void)hipDeviceSynchronize();
  dev_free(ix->packed);
  delete ix;
}

int ottohip_knn_topk(ottohip_ctx* c, const ottohip_knn_index* ix, const int32_t* query_rows, int64_t n_q, int k,
                     int32_t* out_idx, float* out_d2, void* stream) {
  if (!c || !ix || n_q < 0 || k < 1 || k > KN_KMAX || !out_idx || !out_d2) {
    set_error("knn_topk: bad arguments (1 <= k <= %d)", KN_KMAX);
    return OTTOHIP_EINVAL;
  }
  if (n_q == 0) return 0;
  if (!query_rows && n_q > ix->n_items) {
    set_error("knn_topk: n_q=%lld query rows 0..n_q-1 exceed the index (%lld rows)", (long long)n_q,
              (long long)ix->n_items);
    return OTTOHIP_EINVAL;
  }
  Ctx* ctx = ctx_base(c);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  ctx->reset_timing();
  uint16_t* qp;
  uint32_t* cand;
  int* err;
  OH_TRY(ctx->ws.get("knn_q", (size_t)n_q * KN_KD * 2, reinterpret_cast<void**>(&qp)));
  OH_TRY(ctx->ws.get("knn_cand", (size_t)n_q * KN_CAND, &cand));
  OH_TRY(ctx->ws.get("knn_err", 1, &err));
  OH_HIP(hipMemsetAsync(err, 0, sizeof(int), s));
  int ph = ctx->begin("knn_pack", s, 0);
  k_knn_pack<<<(unsigned)ceil_div(n_q * 64, 256), 256, 0, s>>>(ix->emb, n_q, ix->dim, query_rows, ix->n_items, 1, qp, err);
  ctx->end(ph, s);
  static const int abl = getenv("OTTOHIP_KNN_ABLATE") ? atoi(getenv("OTTOHIP_KNN_ABLATE")) : 0;
  static const int nopre = getenv("OTTOHIP_KNN_NOPRE") ? atoi(getenv("OTTOHIP_KNN_NOPRE")) : 0;
  // pre-pass sampling stride (A/B switch OTTOHIP_KNN_PRE_STRIDE; PRE_STRIDE by default)
  static const int pst = getenv("OTTOHIP_KNN_PRE_STRIDE") ? std::max(2, atoi(getenv("OTTOHIP_KNN_PRE_STRIDE"))) : PRE_STRIDE;
  const unsigned grid = (unsigned)ceil_div(n_q, KN_QB);
  const int64_t nT = ceil_div(ix->n_items, KN_IT);
  float* thr = nullptr;
  const bool k8 = ix->dim + 2 > 7 * 16;
  // the 8-column last k-step (OTTOHIP_KNN_HALF=0: seven 16-column steps; read per call)
  const bool half = !k8 && ix->dim + 2 <= 6 * 16 + 8 && !(getenv("OTTOHIP_KNN_HALF") && !strcmp(getenv("OTTOHIP_KNN_HALF"), "0"));
  if (!abl && !nopre && (nT - 1) / pst >= KN_C) {  // enough sampled tiles for KN_C groups
    OH_TRY(ctx->ws.get("knn_thr", (size_t)n_q, &thr));
    const int64_t nS = (nT - 1 + pst - 1) / pst;
    ph = ctx->begin("knn_pre", s, 2.0 * (double)n_q * (double)(nS * KN_IT) * ix->dim);
    (k8 ? k_knn_main<2, 8> : (half ? k_knn_main<2, 7, false, true> : k_knn_main<2, 7>))<<<grid, KN_T, 0, s>>>(reinterpret_cast<const uint4*>(ix->packed), ix->n_items,
                                          reinterpret_cast<const uint4*>(qp), n_q, cand, thr, pst, nullptr, nullptr);
    ctx->end(ph, s);
  }
  ph = ctx->begin("knn_main", s, 2.0 * (double)n_q * (double)ix->n_items * ix->dim);
  // candidate buffers instead of index lists (OTTOHIP_KNN_BUF=0: index lists; A/B switch)
  const bool use_buf = !(getenv("OTTOHIP_KNN_BUF") && !strcmp(getenv("OTTOHIP_KNN_BUF"), "0"));  // read per call
  bool done = false;
  if (use_buf && !abl) {
    uint2* cbuf;
    uint32_t* ncand;
    int* ovf;
    OH_TRY(ctx->ws.get("knn_cbuf", (size_t)n_q * KN_BCAP, &cbuf));
    OH_TRY(ctx->ws.get("knn_ncand", (size_t)n_q, &ncand));
    OH_TRY(ctx->ws.get("knn_ovf", 1, &ovf));
    OH_HIP(hipMemsetAsync(ovf, 0, sizeof(int), s));
    (k8 ? k_knn_main<0, 8, true> : (half ? k_knn_main<0, 7, true, true> : k_knn_main<0, 7, true>))<<<grid, KN_T, 0, s>>>(
        reinterpret_cast<const uint4*>(ix->packed), ix->n_items, reinterpret_cast<const uint4*>(qp), n_q, cand, thr, pst,
        cbuf, ncand);
    ctx->end(ph, s);
    ph = ctx->begin("knn_select", s, 0);
    k_knn_select_buf<<<(unsigned)ceil_div(n_q * 64, 256), 256, 0, s>>>(cbuf, ncand, n_q, cand, ovf);
    ctx->end(ph, s);
    int hov = 0;
    OH_HIP(hipMemcpyAsync(&hov, ovf, sizeof(int), hipMemcpyDeviceToHost, s));
    OH_HIP(hipStreamSynchronize(s));
    done = hov == 0;  // else: some query inserted more than KN_BCAP candidates -> index lists
    if (!done) ph = ctx->begin("knn_main_lists", s, 2.0 * (double)n_q * (double)ix->n_items * ix->dim);
  }
  if (!done) {
    auto kmain = k8 ? (abl == 3 ? k_knn_main<3, 8> : (abl ? k_knn_main<1, 8> : k_knn_main<0, 8>))
                    : (abl == 3 ? k_knn_main<3, 7> : (abl ? k_knn_main<1, 7> : (half ? k_knn_main<0, 7, false, true> : k_knn_main<0, 7>)));
    kmain<<<grid, KN_T, 0, s>>>(reinterpret_cast<const uint4*>(ix->packed), ix->n_items,
                                reinterpret_cast<const uint4*>(qp), n_q, cand, thr, pst, nullptr, nullptr);
    ctx->end(ph, s);
  }
  ph = ctx->begin("knn_rerank", s, 0);
  k_knn_rerank<<<(unsigned)ceil_div(n_q * 64, 256), 256, 0, s>>>(ix->emb, ix->n_items, ix->dim, query_rows, n_q, cand,
                                                                 k, out_idx, out_d2);
  ctx->end(ph, s);
  OH_HIP(hipGetLastError());
  if (query_rows) {  // explicit rows were range-checked on the device
    int herr = 0;
    OH_HIP(hipMemcpyAsync(&herr, err, sizeof(int), hipMemcpyDeviceToHost, s));
    OH_HIP(hipStreamSynchronize(s));
    if (herr) { set_error("knn_topk: a query row is outside [0, n_items)"); return OTTOHIP_ERANGE; }
  }
  return 0;
}
}  // extern "C"

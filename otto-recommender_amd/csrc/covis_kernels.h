// Co-visitation counting kernels for gfx950 (included once, by abi.hip) (model/count_co_events.py:17-100, :168).
//
// Pipeline (DESIGN.md §3 has the data layout and byte model):
//   S1 prep     wave per block of sessions: pack (ts, aid, type) into u64, sort each session
//               in LDS, drop exact duplicates (df.unique(), :92)
//   S2 count    wave per block of sessions: per event i and rule r, the number of partners j
//               in the session window (binary search on ts + per-type prefix counts in LDS);
//               row key = (type_i, aid_i)
//   S3 rows     stable LSD radix sort of events by row key; exclusive scan of counts gives
//               each event its run of output words: rows (aid-major) are contiguous
//   S4 emit     wave per block of sessions, batches of whole sessions: events re-laid out in
//               LDS as per-type ts-sorted lists, so a (rule, next type) window is one contiguous
//               range; the ranges are expanded 64 pairs per round, one u32 word
//               (rule | aid_next | file) per qualifying pair at its row position
//   S5 reduce   rows <= 1024 words: one wave, register bitonic sort + run-length scans
//               (per-file counts folded over files); larger rows: split 2^k-way by a hash of
//               the word's (rule, aid_next) part; split buckets still above 1024 words go to a
//               workgroup LDS hash (overflow: split again with the next level's hash)
// Output: per (rule, aid, aid_next): count (sum over files), count_ge2 (sum of per-file
// counts >= 2) and per-rule file-row statistics for the merge rule of :131-135.
#pragma once
#include "prims.h"

namespace ottohip {

constexpr int EV_BLOCK = 256;     // events per wave block (sessions starting in it)
constexpr int LCAP = 512;         // sessions up to LCAP events run from LDS
constexpr int SPLIT_MEAN = 420;   // hashed split buckets average at most this many words (register sorts only)
constexpr int LDS_SPLIT_MEAN = 2560;  // the same with the LDS leaf (k_agg_lds takes buckets of <= 4096 words)
__constant__ uint32_t c_split_mean = SPLIT_MEAN;  // OTTOHIP_SPLIT_MEAN overrides it (A/B switch, abi.hip)
__constant__ uint32_t c_split_runs = 0;  // split histograms fold runs of equal digits over lanes (OTTOHIP_SPLIT_RUNS=1; measured
                                          // +0.9 ms reduce: the extra VALU outweighs the few runs)
__constant__ uint32_t c_split_fuse = 1;  // one-chunk split tasks counted inside k_split_scatter (OTTOHIP_SPLIT_FUSE=0: off)
__constant__ uint32_t c_hash_prio = 0;  // OTTOHIP_HASH_PRIO: wave priority of the LDS-hash leaves (A/B switch)
__constant__ uint32_t c_lds_leaf = 0;   // rows / split buckets of (SORT_MAX, LDS_CAP] words go to k_agg_lds (abi.hip)
constexpr uint32_t W_EMPTY = 0xFFFFFFFFu;
constexpr int STAT_STRIPES = 256;            // copies of the per-rule statistics
// u64 per copy: [rule * 4 + {rows, pairs, file_rows, file_rows_ge2}] (a symmetric rule's rows with
// aid != aid_next count twice: the row and its mirror), then STAT_RAW + {0: stored rows, 1: stored
// pairs} over all rules (the reduce's conservation check against the emitted words)
constexpr int STAT_RAW = MAX_RULES * 4;
constexpr int STAT_STRIDE = STAT_RAW + 8;

struct RulesDev {
  int32_t lo[MAX_RULES], hi[MAX_RULES];    // window on dt = ts_j - ts_i, inclusive
  uint32_t mask[MAX_RULES];                // allowed next types
  int32_t n_of_type[4];                    // rules whose this_type == t
  int32_t rule_of_type[4][MAX_RULES];      // global rule id per (t, local index)
  // Symmetric rules (next types == {this type}, window symmetric in dt: click_to_click, cart_to_cart,
  // buy_to_buy): every qualifying ordered pair (i, j) has its mirror (j, i), so count(a, b) ==
  // count(b, a) per session, per file and in total. Only pairs with aid_j >= aid_i are emitted
  // (both orders of equal aids) and only the row (a, b), a <= b, is stored: the table's readers
  // (compaction, digest, owner packing) produce the mirror (b, a) of every stored row with a < b
  // (ottohip_table::sym_mask).
  uint32_t sym_mask;
};

__device__ __forceinline__ bool rule_sym(const RulesDev& R, int r) { return (R.sym_mask >> r) & 1u; }

// partners j in [jb, je) of the same type t with aid_j >= aid (packed low word aid << 2 | type). With x = w - lo,
// the partner qualifies iff x is a non-negative multiple of 4 below 2^(A+2): rotating x right by 2 moves a type
// mismatch (x & 3 != 0) into bits 30-31 and a negative difference (aid_j < aid) to >= 2^30 - 2^A, so one compare
// against 2^29 decides when aid < 2^29 (A <= 29); wider aids take the plain test. Four partners per step (two
// ds_read2 of the keys' low words).
__device__ __forceinline__ uint32_t count_sym_partners(const uint64_t* ev, int jb, int je, uint32_t aid, int t, int A) {
  const uint32_t lo = (aid << 2) | (uint32_t)t;
  uint32_t m = 0;
  if (A > 29) {
    for (int j = jb; j < je; ++j) {
      const uint32_t w = (uint32_t)ev[j];
      m += ((w & 3u) == (uint32_t)t && w >= lo) ? 1u : 0u;
    }
    return m;
  }
  constexpr uint32_t LIM = 1u << 29;
  auto ok = [&](uint32_t w) { return __builtin_amdgcn_alignbit(w - lo, w - lo, 2) < LIM ? 1u : 0u; };
  int j = jb;
  for (; j + 4 <= je; j += 4) m += ok((uint32_t)ev[j]) + ok((uint32_t)ev[j + 1]) + ok((uint32_t)ev[j + 2]) + ok((uint32_t)ev[j + 3]);
  for (; j < je; ++j) m += ok((uint32_t)ev[j]);
  return m;
}

struct Layout {
  int A;      // aid bits
  int F;      // file bits
  int BR;     // local rule bits
  int WB;     // word bits = BR + A + F
  uint32_t amask;
};

struct Task {
  uint64_t begin;
  uint32_t len;
  uint32_t row;
  uint32_t rem;   // key bits not yet used for splitting (from the top)
  uint32_t buf;   // which word buffer holds it
};

struct OutRows {
  uint8_t* rule;
  int32_t* aid;
  int32_t* aid_next;
  uint32_t* count;
  uint32_t* count_ge2;
  uint64_t cap;
  unsigned long long* stats;  // [STAT_STRIPES][STAT_STRIDE]
};

// Per-file options of one rule (ottohip_file_opts; A6 branch (2) by rows, count_co_events.py:136-158):
// a row slice of a boundary file is a key range of its (aid, aid_next)-ordered table, so the words
// of file lo_file with key < lo_key and of file hi_file with key >= hi_key are dropped by the leaf
// tasks before they are counted; hist[f] accumulates file f's rows of the rule (low 32 bits) and
// those with per-file count >= 2 (high 32 bits). Applied to the rule's words only.
constexpr int FO_MAXF = 1024;
constexpr int FO_MAXCUT = 64;
constexpr uint8_t FO_NOCUT = 0xFF;
struct FileOpts {
  int type;              // row type of the rule
  uint32_t q;            // the rule's index among the rules of its type (word bits above aid_next)
  uint32_t lo_file, hi_file;  // 0xFFFFFFFF: no cut
  uint32_t cuts;              // lo_file or hi_file set (else the leaves skip the per-word drop test)
  uint64_t lo_key, hi_key;    // key = aid << 32 | aid_next
  unsigned long long* hist;   // [nf] or null
  uint32_t nf;
  uint32_t sym;               // the rule is stored once per unordered pair (no key cuts): hist counts mirrors
  // part mode (ottohip_covis_count_parts, A6 branch (2) from one count): a word of file f with key k belongs
  // to part part_of[f] + (cut_of[f] != NONE && k >= cut_key[cut_of[f]]); k-runs break where the part
  // changes and a row's output "rule" byte is its part (single-rule counts, aid_next < 2^24)
  uint32_t parts;             // 0: off
  const uint8_t* part_of;     // device [nf]
  const uint8_t* cut_of;      // device [nf]: index into cut_key, FO_NOCUT = none
  uint32_t ncut;
  uint64_t cut_key[FO_MAXCUT];
  // part mode over the retained words of a multi-rule count (ottohip_table_count_parts): the words of the type's
  // other rules are dropped (qonly), and a symmetric rule's stored row (a, b), a <= b, also yields its mirror
  // (b, a) as an explicit row in the slot mirror_off + slot of the (non-symmetric) part table, with the mirror's
  // own part (a cut file's key comparison differs between (a, b) and (b, a))
  uint32_t qonly;
  uint64_t mirror_off;        // 0: no mirror rows
  unsigned long long* dropped;  // words dropped by the cuts (the reduce's conservation check)
  unsigned long long* dbg;      // OTTOHIP_DEBUG: [hash dropped, hash kept, sort dropped, sort kept] or null
  unsigned long long* prof;     // OTTOHIP_HASH_PROF: per hash task {len | rows << 32, wall-clock ticks | full << 63} or null
};
// LDS copy of the part-mode tables (FO kernels)
struct PartLds {
  uint8_t part_of[FO_MAXF];
  uint8_t cut_of[FO_MAXF];
  uint64_t cut_key[FO_MAXCUT];
};
__device__ __forceinline__ void part_lds_load(const FileOpts& fo, PartLds& P) {
  if (!fo.parts) return;
  for (uint32_t i = threadIdx.x; i < fo.nf; i += blockDim.x) { P.part_of[i] = fo.part_of[i]; P.cut_of[i] = fo.cut_of[i]; }
  for (uint32_t i = threadIdx.x; i < fo.ncut; i += blockDim.x) P.cut_key[i] = fo.cut_key[i];
}
// part of word w (valid) of row aid
__device__ __forceinline__ uint32_t word_part(const PartLds& P, uint32_t w, uint32_t aid, const Layout& L) {
  const uint32_t f = w & ((1u << L.F) - 1u);
  const uint32_t ci = P.cut_of[f];
  const uint64_t key = ((uint64_t)aid << 32) | ((w >> L.F) & L.amask);
  return (uint32_t)P.part_of[f] + ((ci != FO_NOCUT && key >= P.cut_key[ci & (FO_MAXCUT - 1)]) ? 1u : 0u);
}
// part of the mirror (aid_next, aid) of word w (valid) of row aid
__device__ __forceinline__ uint32_t word_part_mirror(const PartLds& P, uint32_t w, uint32_t aid, const Layout& L) {
  const uint32_t f = w & ((1u << L.F) - 1u);
  const uint32_t ci = P.cut_of[f];
  const uint64_t key = ((uint64_t)((w >> L.F) & L.amask) << 32) | aid;
  return (uint32_t)P.part_of[f] + ((ci != FO_NOCUT && key >= P.cut_key[ci & (FO_MAXCUT - 1)]) ? 1u : 0u);
}
__device__ __forceinline__ bool fo_drop(const FileOpts& fo, uint32_t w, int32_t aid, const Layout& L) {
  if (w == W_EMPTY) return false;
  if ((w >> (L.A + L.F)) != fo.q) return fo.qonly != 0;
  const uint32_t f = w & ((1u << L.F) - 1u);
  const uint64_t key = ((uint64_t)(uint32_t)aid << 32) | ((w >> L.F) & L.amask);
  return (f == fo.lo_file && key < fo.lo_key) || (f == fo.hi_file && key >= fo.hi_key);
}

// ------------------------------------------------------------------ block maps
__global__ void k_block_first(const int64_t* __restrict__ off, int64_t S, int64_t NB,
                              int64_t* __restrict__ first, int32_t* __restrict__ long_list,
                              int32_t* __restrict__ n_long) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s > S) return;
  const int64_t lo = s == 0 ? 0 : off[s - 1] / EV_BLOCK + 1;
  const int64_t hi = s == S ? NB : off[s] / EV_BLOCK;
  for (int64_t b = lo; b <= hi && b <= NB; ++b) first[b] = s;
  if (s < S && off[s + 1] - off[s] > LCAP) {
    int k = atomicAdd(n_long, 1);
    long_list[k] = (int32_t)s;
  }
}

__device__ __forceinline__ int file_of(const int64_t* fb, int nf, int64_t s) {
  int lo = 0, hi = nf;  // largest f with fb[f] <= s
  while (hi - lo > 1) {
    int m = (lo + hi) >> 1;
    if (fb[m] <= s) lo = m; else hi = m;
  }
  return lo;
}

// ------------------------------------------------------------------ S1 prep
// Sort one session (n events) by packed key and compact distinct keys into out[0..);
// the tail [n_kept, n) is set to EV_INVALID. Executed by one wave.
__device__ __forceinline__ void prep_session(const int32_t* __restrict__ aid, const int32_t* __restrict__ ts,
                                             const int8_t* __restrict__ ty, int64_t e0, int n,
                                             uint64_t* keys, uint64_t* sorted, uint64_t* __restrict__ out,
                                             int n_items, int dedup, int* err) {
  const int l = lane_id();
  for (int k = l; k < n; k += 64) {
    const int32_t a = aid[e0 + k], t = ts[e0 + k], y = ty[e0 + k];
    if (a < 0 || a >= n_items || y < 0 || y > 2) atomicOr(err, 1);
    keys[k] = ev_pack(a < 0 ? 0 : a, t, y & 3);
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  for (int k = l; k < n; k += 64) {
    const uint64_t v = keys[k];
    int r = 0;
    for (int j = 0; j < n; ++j) {
      const uint64_t u = keys[j];
      r += (u < v) | ((u == v) & (j < k));
    }
    sorted[r] = v;
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  int base = 0;
  for (int k0 = 0; k0 < n; k0 += 64) {
    const int k = k0 + l;
    const uint64_t v = k < n ? sorted[k] : EV_INVALID;
    const bool keep = k < n && (!dedup || k == 0 || sorted[k - 1] != v);
    const uint64_t m = __ballot(keep);
    if (keep) out[base + (int)mbcnt(m)] = v;
    base += (int)__popcll(m);
  }
  for (int k = base + l; k < n; k += 64) out[k] = EV_INVALID;
}

__global__ __launch_bounds__(64) void k_prep_long(const int64_t* __restrict__ off, const int32_t* __restrict__ list,
                                                  const int64_t* __restrict__ scratch_off,
                                                  uint64_t* __restrict__ scratch, const int32_t* __restrict__ aid,
                                                  const int32_t* __restrict__ ts, const int8_t* __restrict__ ty,
                                                  uint64_t* __restrict__ ev, int n_items, int dedup, int* err) {
  const int64_t s = list[blockIdx.x];
  const int64_t e0 = off[s];
  const int n = (int)(off[s + 1] - e0);
  uint64_t* keys = scratch + 2 * scratch_off[blockIdx.x];
  prep_session(aid, ts, ty, e0, n, keys, keys + n, ev + e0, n_items, dedup, err);
}

// ------------------------------------------------------------------ S2 count
struct SessView {
  const uint64_t* ev;   // sorted valid events [0, nv)
  int nv;
  const uint32_t* pref; // pref[t * (cap+1) + k]: events of type t among [0, k)
  int pstride;
};

// load a session into LDS/global scratch and build per-type exclusive prefix counts
__device__ __forceinline__ int load_session(const uint64_t* __restrict__ src, int n, uint64_t* evs,
                                            uint32_t* pref, int pstride) {
  const int l = lane_id();
  int nv = 0;
  uint32_t base0 = 0, base1 = 0, base2 = 0;
  for (int k0 = 0; k0 < n; k0 += 64) {
    const int k = k0 + l;
    const uint64_t v = k < n ? src[k] : EV_INVALID;
    if (k < n) evs[k] = v;
    const bool valid = v != EV_INVALID;
    const int t = (int)(v & 3u);
    const uint64_t m0 = __ballot(valid && t == 0), m1 = __ballot(valid && t == 1), m2 = __ballot(valid && t == 2);
    if (k < n && pref) {
      pref[0 * pstride + k] = base0 + mbcnt(m0);
      pref[1 * pstride + k] = base1 + mbcnt(m1);
      pref[2 * pstride + k] = base2 + mbcnt(m2);
    }
    base0 += (uint32_t)__popcll(m0); base1 += (uint32_t)__popcll(m1); base2 += (uint32_t)__popcll(m2);
    nv += (int)__popcll(__ballot(valid));
  }
  if (l == 0 && pref) {  // pref[t][nv] = totals (invalid slots carry no types, so totals at n == at nv)
    pref[0 * pstride + nv] = base0; pref[1 * pstride + nv] = base1; pref[2 * pstride + nv] = base2;
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  return nv;
}

__device__ __forceinline__ int lower_ts(const uint64_t* evs, int nv, int64_t x) {  // first k: ts_k >= x
  int lo = 0, hi = nv;
  while (lo < hi) {
    const int m = (lo + hi) >> 1;
    if ((int64_t)ev_ts(evs[m]) < x) lo = m + 1; else hi = m;
  }
  return lo;
}
__device__ __forceinline__ int upper_ts(const uint64_t* evs, int nv, int64_t x) {  // first k: ts_k > x
  int lo = 0, hi = nv;
  while (lo < hi) {
    const int m = (lo + hi) >> 1;
    if ((int64_t)ev_ts(evs[m]) <= x) lo = m + 1; else hi = m;
  }
  return lo;
}

// number of events identical to evs[i] (adjacent in sorted order); 1 after dedup
__device__ __forceinline__ int equal_run(const uint64_t* evs, int nv, int i) {
  const uint64_t v = evs[i];
  int a = i, b = i + 1;
  while (a > 0 && evs[a - 1] == v) --a;
  while (b < nv && evs[b] == v) ++b;
  return b - a;
}

__device__ __forceinline__ uint32_t count_event(const SessView& S, int i, const RulesDev& R, int A) {
  const uint64_t e = S.ev[i];
  const int t = ev_type(e);
  const int64_t tsi = ev_ts(e);
  uint32_t c = 0;
  int run = -1;
  for (int q = 0; q < R.n_of_type[t]; ++q) {
    const int r = R.rule_of_type[t][q];
    const int jb = lower_ts(S.ev, S.nv, tsi + R.lo[r]);
    const int je = upper_ts(S.ev, S.nv, tsi + R.hi[r]);
    if (je <= jb) continue;
    uint32_t m = 0;
    if (rule_sym(R, r)) {
      m = count_sym_partners(S.ev, jb, je, (uint32_t)ev_aid(e), t, A);
    } else {
      for (int tt = 0; tt < 3; ++tt)
        if ((R.mask[r] >> tt) & 1u) m += S.pref[tt * S.pstride + je] - S.pref[tt * S.pstride + jb];
    }
    if (((R.mask[r] >> t) & 1u) && R.lo[r] <= 0 && R.hi[r] >= 0) {
      if (run < 0) run = equal_run(S.ev, S.nv, i);
      m -= (uint32_t)run;  // the identity row of :23-27 (and exact twins when dedup is off)
    }
    c += m;
  }
  return c;
}

// the row key of an event, with (cshift > 0: the fused row layout of S3) its pair count saturated
// at RK_CSAT in the byte above the sorted key bits
constexpr uint32_t RK_CSAT = 255u;

// Grouped row entries (the fused row layout, S2 -> S3 -> S4). The events of one session with the same (type, aid) and
// a nonzero pair count form one group; only one of them (the group's rep) enters the S3 sort, with the group's total
// count, and the group's words are one run of its row: a member's run starts at the rep's word offset plus its
// prefix gpre inside the group (the order of words inside a row is free: the reduce sorts them). Per event, link[e]:
//   LK_REP | count   the event is its own row entry (a rep: count = the group's total; a long session's event; an event
//                    without pairs, count 0)
//   (delta + 512) << 21 | gpre   a member: its rep is event e + delta (|delta| < 512, same batch), gpre < 2^21
// (gpre < 512 members x MAX_RULES x 511 partners < 2^21)
constexpr uint32_t LK_REP = 0x80000000u;
constexpr int LK_DSHIFT = 21;
constexpr uint32_t LK_GMASK = (1u << LK_DSHIFT) - 1u;
__device__ __forceinline__ uint32_t rk_with_count(uint32_t key, uint32_t c, int cshift) {
  return cshift ? key | ((c < RK_CSAT ? c : RK_CSAT) << cshift) : key;
}

__device__ __forceinline__ void count_session(const SessView& S, int64_t e0, int n, const RulesDev& R, int A,
                                              uint32_t* __restrict__ cnt, uint32_t* __restrict__ rk,
                                              uint32_t* __restrict__ pos, int cshift, uint32_t* __restrict__ link) {
  const uint32_t INV = 3u << A;
  for (int k = lane_id(); k < n; k += 64) {
    uint32_t c = 0, key = INV;
    if (k < S.nv) {
      c = count_event(S, k, R, A);
      if (c) { const uint64_t e = S.ev[k]; key = ((uint32_t)ev_type(e) << A) | (uint32_t)ev_aid(e); }
    }
    cnt[e0 + k] = c;
    rk[e0 + k] = rk_with_count(key, c, cshift);
    if (pos) pos[e0 + k] = (uint32_t)(e0 + k);
    if (link) link[e0 + k] = LK_REP | c;  // a long session's events are not grouped: every event is its own row entry
  }
}

__global__ __launch_bounds__(64) void k_count_long(const int64_t* __restrict__ off, const int32_t* __restrict__ list,
                                                   const int64_t* __restrict__ scratch_off,
                                                   uint64_t* __restrict__ scratch, uint32_t* __restrict__ pscratch,
                                                   const uint64_t* __restrict__ ev, RulesDev R, int A,
                                                   uint32_t* __restrict__ cnt, uint32_t* __restrict__ rk,
                                                   uint32_t* __restrict__ pos, int cshift, uint32_t* __restrict__ link) {
  const int64_t s = list[blockIdx.x];
  const int64_t e0 = off[s];
  const int n = (int)(off[s + 1] - e0);
  const int64_t so = scratch_off[blockIdx.x];
  SessView S;
  uint64_t* evs = scratch + 2 * so;
  uint32_t* pref = pscratch + 3 * (so + blockIdx.x);
  S.ev = evs; S.pref = pref; S.pstride = n + 1;
  S.nv = load_session(ev + e0, n, evs, pref, n + 1);
  count_session(S, e0, n, R, A, cnt, rk, pos, cshift, link);
}

// ------------------------------------------------------------------ S1+S2 fused
__device__ __forceinline__ int lds_lower_ts(const uint64_t* tev, int a, int b, int64_t x) {  // first k: ts >= x
  while (a < b) {
    const int m = (a + b) >> 1;
    if ((int64_t)ev_ts(tev[m]) < x) a = m + 1; else b = m;
  }
  return a;
}
__device__ __forceinline__ int lds_upper_ts(const uint64_t* tev, int a, int b, int64_t x) {  // first k: ts > x
  while (a < b) {
    const int m = (a + b) >> 1;
    if ((int64_t)ev_ts(tev[m]) <= x) a = m + 1; else b = m;
  }
  return a;
}

// One wave per 256-event block, batches of whole sessions (<= PB_CAP events, none longer than
// LCAP: those take k_prep_long / k_count_long). Per batch, all in LDS:
//   load + pack (aid, ts, type) coalesced; sort each session by the packed key (a session whose
//   ts never decreases only reorders within runs of equal ts: rank inside the run; any other
//   session is ranked against all of its events); drop exact duplicates (df.unique(), :92);
//   store the packed events; per-type prefix counts; per event and rule the partner count in
//   the window (binary searches on ts) and the row key.
constexpr int PB_CAP = 512;
struct PrepLds {
  uint64_t key[PB_CAP];   // packed raw events, then the final (sorted, deduplicated) session layout
  union {                 // srt is dead once the deduplicated layout is in key: pref reuses it
    uint64_t srt[PB_CAP];   // sorted events before deduplication
    uint16_t pref[3][PB_CAP + 1];
  };
  uint16_t ss[65];        // session starts in the batch; ss[nsess] = batch size
  uint16_t pst[64], pen[64];
  uint8_t esid[PB_CAP];
  uint8_t uns[64];        // session has a ts decrease: full ranking
};
static_assert((uint64_t)PB_CAP * MAX_RULES * (LCAP - 1) < (1ull << LK_DSHIFT), "group prefixes in link bits");

__global__ __launch_bounds__(64) void k_prep_count(const int64_t* __restrict__ off, const int64_t* __restrict__ first,
                                                   int64_t NB, const int32_t* __restrict__ aid,
                                                   const int32_t* __restrict__ ts, const int8_t* __restrict__ ty,
                                                   uint64_t* __restrict__ ev, int n_items, int dedup, int* err,
                                                   RulesDev R, int A, uint32_t* __restrict__ cnt,
                                                   uint32_t* __restrict__ rk, uint32_t* __restrict__ pos, int cshift,
                                                   uint32_t* __restrict__ link) {
  __shared__ PrepLds S;
  __shared__ RulesDev sR;
  const int l = threadIdx.x;
  if (l == 0) sR = R;
  const int64_t g = blockIdx.x;
  if (g >= NB) return;
  const int64_t s0 = first[g], s1 = first[g + 1];
  __syncthreads();
  const uint32_t INV = 3u << A;
  int64_t b = s0;
  while (b < s1) {
    const int64_t base = off[b];
    const int64_t s = b + l;
    const bool in_s = s < s1;
    const int64_t so = in_s ? off[s] : 0, se = in_s ? off[s + 1] : 0;
    const bool ok = in_s && se - base <= PB_CAP && se - so <= LCAP;
    const uint64_t bad = __ballot(!ok);
    const int nsess = bad ? (int)__builtin_ctzll(bad) : 64;
    if (nsess == 0) { ++b; continue; }  // long session: k_prep_long / k_count_long
    const int nb_ev = __shfl((int)(se - base), nsess - 1);
    const int64_t E0 = base;
    if (l < nsess) { S.ss[l] = (uint16_t)(so - base); S.uns[l] = 0; }
    if (l == 0) S.ss[nsess] = (uint16_t)nb_ev;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    const int nch = (nb_ev + 63) >> 6;
    // ---- load, pack, session of each event
#pragma unroll 1
    for (int c = 0; c < nch; ++c) {
      const int idx = c * 64 + l;
      if (idx >= nb_ev) continue;
      const int32_t a = aid[E0 + idx], t = ts[E0 + idx], y = ty[E0 + idx];
      if (a < 0 || a >= n_items || y < 0 || y > 2) atomicOr(err, 1);
      S.key[idx] = ev_pack(a < 0 ? 0 : a, t, y & 3);
      int k = 0;
#pragma unroll
      for (int st = 32; st >= 1; st >>= 1)
        if (k + st < nsess && (int)S.ss[k + st] <= idx) k += st;
      S.esid[idx] = (uint8_t)k;
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
#pragma unroll 1
    for (int c = 0; c < nch; ++c) {
      const int idx = c * 64 + l;
      if (idx >= nb_ev) continue;
      const int k = S.esid[idx];
      if (idx > (int)S.ss[k] && ev_ts(S.key[idx]) < ev_ts(S.key[idx - 1])) S.uns[k] = 1;
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    // ---- sort each session (stable rank by the packed key)
#pragma unroll 1
    for (int c = 0; c < nch; ++c) {
      const int idx = c * 64 + l;
      if (idx >= nb_ev) continue;
      const int k = S.esid[idx];
      const uint64_t v = S.key[idx];
      int lo = S.ss[k], hi = S.ss[k + 1];
      if (!S.uns[k]) {  // ts non-decreasing: only the run of equal ts can be out of order
        const int32_t t = ev_ts(v);
        int a = idx, e = idx + 1;
        while (a > lo && ev_ts(S.key[a - 1]) == t) --a;
        while (e < hi && ev_ts(S.key[e]) == t) ++e;
        lo = a; hi = e;
      }
      int r = lo;
      for (int j = lo; j < hi; ++j) {
        const uint64_t u = S.key[j];
        r += (u < v) | ((u == v) & (j < idx));
      }
      S.srt[r] = v;
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    // ---- deduplicate: kept events first, EV_INVALID tail (positions stay inside the session)
    uint32_t P = 0;
#pragma unroll 1
    for (int c = 0; c < nch; ++c) {
      const int idx = c * 64 + l;
      const bool in = idx < nb_ev;
      const int k = in ? S.esid[idx] : 0;
      const bool keep = in && (!dedup || idx == (int)S.ss[k] || S.srt[idx - 1] != S.srt[idx]);
      const uint64_t m = __ballot(keep);
      const uint32_t Pi = P + mbcnt(m);
      if (in && idx == (int)S.ss[k]) S.pst[k] = (uint16_t)Pi;
      if (in && idx == (int)S.ss[k + 1] - 1) S.pen[k] = (uint16_t)(Pi + (keep ? 1u : 0u));
      if (in) S.key[idx] = EV_INVALID;
      P += (uint32_t)__popcll(m);
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    P = 0;
#pragma unroll 1
    for (int c = 0; c < nch; ++c) {
      const int idx = c * 64 + l;
      const bool in = idx < nb_ev;
      const int k = in ? S.esid[idx] : 0;
      const bool keep = in && (!dedup || idx == (int)S.ss[k] || S.srt[idx - 1] != S.srt[idx]);
      const uint64_t m = __ballot(keep);
      if (keep) S.key[S.ss[k] + (P + mbcnt(m)) - S.pst[k]] = S.srt[idx];
      P += (uint32_t)__popcll(m);
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    // ---- store; per-type prefix counts over the batch
    uint32_t b0 = 0, b1 = 0, b2 = 0;
#pragma unroll 1
    for (int c = 0; c < nch; ++c) {
      const int idx = c * 64 + l;
      const bool in = idx < nb_ev;
      const uint64_t v = in ? S.key[idx] : EV_INVALID;
      if (in) ev[E0 + idx] = v;
      const int t = ev_type(v);
      const uint64_t m0 = __ballot(t == 0), m1 = __ballot(t == 1), m2 = __ballot(t == 2);
      if (in) {
        S.pref[0][idx] = (uint16_t)(b0 + mbcnt(m0));
        S.pref[1][idx] = (uint16_t)(b1 + mbcnt(m1));
        S.pref[2][idx] = (uint16_t)(b2 + mbcnt(m2));
      }
      b0 += (uint32_t)__popcll(m0); b1 += (uint32_t)__popcll(m1); b2 += (uint32_t)__popcll(m2);
    }
    if (l == 0) { S.pref[0][nb_ev] = (uint16_t)b0; S.pref[1][nb_ev] = (uint16_t)b1; S.pref[2][nb_ev] = (uint16_t)b2; }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    // ---- partner counts and row keys
    constexpr int NCH = PB_CAP / 64;
    uint32_t cv[NCH];  // grouped rows: the counts of the lane's events (c is wave-uniform: a select per chunk)
#pragma unroll
    for (int c = 0; c < NCH; ++c) cv[c] = 0u;
#pragma unroll 1
    for (int c = 0; c < nch; ++c) {
      const int idx = c * 64 + l;
      if (idx >= nb_ev) continue;
      const int k = S.esid[idx];
      const uint64_t e = S.key[idx];
      uint32_t cn = 0, key = INV;
      if (e != EV_INVALID) {
        const int lo = S.ss[k], hi = lo + (S.pen[k] - S.pst[k]);  // valid events of the session
        const int t = ev_type(e);
        const int64_t tsi = ev_ts(e);
        int run = -1;
#if defined(OH_PREP_ABL) && OH_PREP_ABL == 3  // timing ablation: no window counts at all, wrong counts
        cn = 1;
        if (false)
#endif
        int32_t plo = 1, phi = -1;  // the previous rule's window: rules of one type sharing a window share its searches
        int jb = 0, je = 0;
        for (int q = 0; q < sR.n_of_type[t]; ++q) {
          const int r = sR.rule_of_type[t][q];
          // a window around dt = 0 ends at or after the event and starts at or before it (the session is in ts
          // order): each search takes one side of the event
          if (sR.lo[r] != plo || sR.hi[r] != phi) {
            plo = sR.lo[r]; phi = sR.hi[r];
            const bool around = plo <= 0 && phi >= 0;
            jb = lds_lower_ts(S.key, lo, around ? idx : hi, tsi + plo);
            je = lds_upper_ts(S.key, around ? idx + 1 : jb, hi, tsi + phi);
          }
          if (je <= jb) continue;
          uint32_t m = 0;
          if (rule_sym(sR, r)) {
#if defined(OH_PREP_ABL) && OH_PREP_ABL == 1  // timing ablation (tools/prep_probe.py): no window scan, wrong counts
            m = (uint32_t)(je - jb);
#else
            m = count_sym_partners(S.key, jb, je, (uint32_t)ev_aid(e), t, A);
#endif
          } else {
#pragma unroll
            for (int tt = 0; tt < 3; ++tt)
              if ((sR.mask[r] >> tt) & 1u) m += (uint32_t)S.pref[tt][je] - (uint32_t)S.pref[tt][jb];
          }
          if (((sR.mask[r] >> t) & 1u) && sR.lo[r] <= 0 && sR.hi[r] >= 0) {
            if (run < 0) {  // the identity row of :23-27 (and exact twins when dedup is off)
              int a = idx, z = idx + 1;
              while (a > lo && S.key[a - 1] == e) --a;
              while (z < hi && S.key[z] == e) ++z;
              run = z - a;
            }
            m -= (uint32_t)run;
          }
          cn += m;
        }
        if (cn) key = ((uint32_t)t << A) | (uint32_t)ev_aid(e);
      }
      cnt[E0 + idx] = cn;
      if (link) {
#pragma unroll
        for (int j = 0; j < NCH; ++j)
          if (j == c) cv[j] = cn;
      } else {
        rk[E0 + idx] = rk_with_count(key, cn, cshift);
        if (pos) pos[E0 + idx] = (uint32_t)(E0 + idx);
      }
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    if (link) {
      // ---- grouped row entries (LK_REP): events of one session with equal (type, aid) and pairs, found by an LDS
      // hash over (aid, session, type); each member takes its prefix in the group by one LDS atomic add, the
      // member that gets 0 is the rep and publishes its position. The hash overlays the dead prefix counts (keys)
      // and the batch's events (sums: the group keys are read into registers first; the events are stored).
      uint32_t gk[NCH], sg[NCH];  // sg: the pair count, then slot << 22 | prefix
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        const int idx = c * 64 + l;
        gk[c] = 0u;
        sg[c] = 0u;
        if (c < nch && idx < nb_ev) {
          const uint64_t e = S.key[idx];
          sg[c] = cv[c];
          if (e != EV_INVALID && sg[c] != 0)  // aid < 2^23 (the fused layout's bound): the key fits 31 bits
            gk[c] = (((uint32_t)ev_aid(e) << 8) | ((uint32_t)S.esid[idx] << 2) | (uint32_t)ev_type(e)) + 1u;
        }
      }
      int tb = 6;
      while ((1 << tb) < 2 * nb_ev && tb < 10) ++tb;
      const uint32_t TS = 1u << tb;
      uint32_t* hkey = reinterpret_cast<uint32_t*>(&S.srt[0]);
      uint32_t* hval = reinterpret_cast<uint32_t*>(&S.key[0]);
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      for (uint32_t i = l; i < TS; i += 64) { hkey[i] = 0u; hval[i] = 0u; }
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      // the first probes of all chunks go out back to back (a wave's LDS operations complete in order, so a later
      // chunk's probe sees an earlier chunk's insert); the few collisions then walk on, lane by lane. The event whose
      // probe inserted the key is the group's rep: it sets the group's sum to its own count (prefix 0) and replaces the
      // key by its position (the probing is over); the other members add their counts, the returned sum is their prefix
      uint32_t hs[NCH], pv[NCH];
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        hs[c] = (gk[c] * 0x9E3779B1u) >> (32 - tb);
        pv[c] = gk[c] ? atomicCAS(&hkey[hs[c]], 0u, gk[c]) : 1u;
      }
#pragma unroll
      for (int c = 0; c < NCH; ++c)
        while (pv[c] != 0u && pv[c] != gk[c] && gk[c]) {
          hs[c] = (hs[c] + 1u) & (TS - 1u);
          pv[c] = atomicCAS(&hkey[hs[c]], 0u, gk[c]);
        }
#pragma unroll
      for (int c = 0; c < NCH; ++c)
        if (gk[c] && pv[c] == 0u) { hval[hs[c]] = sg[c]; hkey[hs[c]] = (uint32_t)(c * 64 + l); }
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
#pragma unroll
      for (int c = 0; c < NCH; ++c)
        if (gk[c] && pv[c] != 0u) sg[c] = atomicAdd(&hval[hs[c]], sg[c]);
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      // row keys and links: a rep's key carries the group's total (LK_REP | total), a member's link its rep and prefix
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        const int idx = c * 64 + l;
        if (c < nch && idx < nb_ev) {
          uint32_t key = INV, lk = LK_REP, tot = 0u;
          if (gk[c] && pv[c] == 0u) {
            tot = hval[hs[c]];
            const uint32_t g = gk[c] - 1u;
            key = ((g & 3u) << A) | (g >> 8);
            lk = LK_REP | tot;
          } else if (gk[c]) {
            const int delta = (int)hkey[hs[c]] - idx;
            lk = ((uint32_t)(delta + 512) << LK_DSHIFT) | sg[c];
          }
          rk[E0 + idx] = rk_with_count(key, tot, cshift);
          link[E0 + idx] = lk;
        }
      }
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    }
    b += nsess;
  }
}

// ------------------------------------------------------------------ S3 rows
// Per event: the first word of its run (row-major word order). u64, or u32 when every word offset
// fits 32 bits (the one-GPU fused layout).
struct EvOff {
  const uint64_t* p64;
  const uint32_t* p32;
  const uint32_t* link;  // grouped row entries (LK_REP): a member's run follows from its rep's offset; null: none
  __device__ __forceinline__ uint64_t at(int64_t e) const { return p32 ? (uint64_t)p32[e] : p64[e]; }
  // the first word of event e's run (e has pairs)
  __device__ __forceinline__ uint64_t run(int64_t e) const {
    if (!link) return at(e);
    const uint32_t lk = link[e];
    if (lk & LK_REP) return at(e);
    return at(e + (int64_t)(lk >> LK_DSHIFT) - 512) + (lk & LK_GMASK);
  }
};

__global__ void k_gather_counts(const uint32_t* __restrict__ rk, const uint32_t* __restrict__ pos,
                                const uint32_t* __restrict__ cnt, int64_t n, uint32_t INV,
                                uint32_t* __restrict__ c_sorted, uint32_t* __restrict__ row_flag) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const uint32_t key = rk[k];
  const bool valid = key != INV;
  c_sorted[k] = valid ? cnt[pos[k]] : 0u;
  row_flag[k] = valid && (k == 0 || rk[k - 1] != key);
}

__global__ void k_rows(const uint32_t* __restrict__ rk, const uint32_t* __restrict__ pos, int64_t n, uint32_t INV,
                       uint32_t kmask, const uint64_t* __restrict__ woff, const uint32_t* __restrict__ row_flag,
                       const uint64_t* __restrict__ row_idx, uint64_t* __restrict__ poff,
                       uint32_t* __restrict__ row_key, uint64_t* __restrict__ row_begin) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const uint32_t key = rk[k];
  if (key == INV) return;
  poff[pos[k]] = woff[k];
  if (row_flag[k]) {
    const uint64_t r = row_idx[k];
    row_key[r] = key & kmask;  // (type, aid); owner bits (multi-GPU layout) dropped
    row_begin[r] = woff[k];
  }
}

// ---- fused row layout (one GPU, rows < 2^24, A <= 21): the event's pair count rides in the
// row key's spare high bits through the radix sort (saturated at RK_CSAT: larger counts, from
// long sessions, are gathered), then one pass of block sums and one pass of per-block scans
// give every event its word offset and every row its key and first word, with X = cnt << 24 |
// [row start] scanned as one u64: no c_sorted / row_flag arrays, no second scan, no gather.
// (RK_CSAT: the key byte above the sorted digits, LSD passes sort whole bytes; written by S1+S2)
constexpr int RT_T = 256, RT_I = 8, RT_TILE = RT_T * RT_I;

// cnt: per event pair counts, or (grouped rows) the link array, whose rep entries hold LK_REP | the group's total
__device__ __forceinline__ uint64_t rows_x(const uint32_t* __restrict__ rks, const uint32_t* __restrict__ poss,
                                           const uint32_t* __restrict__ cnt, int64_t k, uint32_t kmask, uint32_t INV,
                                           int shift, uint32_t& key, bool& start) {
  const uint32_t kk = rks[k];
  key = kk & kmask;
  if (key == INV) { start = false; return 0; }
  start = k == 0 || (rks[k - 1] & kmask) != key;
  uint32_t c = kk >> shift;
  if (c == RK_CSAT) c = cnt[poss[k]] & ~LK_REP;
  return ((uint64_t)c << 24) | (start ? 1u : 0u);
}

__global__ __launch_bounds__(RT_T) void k_rows_sums(const uint32_t* __restrict__ rks, const uint32_t* __restrict__ poss,
                                                    const uint32_t* __restrict__ cnt, int64_t n, uint32_t kmask,
                                                    uint32_t INV, int shift, uint64_t* __restrict__ sums) {
  const int64_t base = (int64_t)blockIdx.x * RT_TILE + (int64_t)threadIdx.x * RT_I;
  uint64_t s = 0;
#pragma unroll
  for (int i = 0; i < RT_I; ++i) {
    if (base + i >= n) break;
    uint32_t key;
    bool st;
    s += rows_x(rks, poss, cnt, base + i, kmask, INV, shift, key, st);
  }
  __shared__ uint64_t ws[RT_T / 64];
  s = wave_sum64(s);
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) sums[blockIdx.x] = ws[0] + ws[1] + ws[2] + ws[3];
}

// poff32 != null: u32 offsets, only for events with position in [plo, plo + pw) (windows of the event
// range, one launch each, measured slower than one pass: plo = 0, pw = ~0); rows only when write_rows.
__global__ __launch_bounds__(RT_T) void k_rows_tile(const uint32_t* __restrict__ rks, const uint32_t* __restrict__ poss,
                                                    const uint32_t* __restrict__ cnt, int64_t n, uint32_t kmask,
                                                    uint32_t INV, int shift, const uint64_t* __restrict__ offs,
                                                    uint64_t* __restrict__ poff, uint32_t* __restrict__ poff32,
                                                    uint32_t plo, uint32_t pw, int write_rows,
                                                    uint32_t* __restrict__ row_key, uint64_t* __restrict__ row_begin,
                                                    uint32_t* __restrict__ wsorted = nullptr) {
  const int64_t base = (int64_t)blockIdx.x * RT_TILE + (int64_t)threadIdx.x * RT_I;
  uint64_t x[RT_I];
  uint32_t key[RT_I];
  bool st[RT_I];
  uint64_t s = 0;
#pragma unroll
  for (int i = 0; i < RT_I; ++i) {
    x[i] = 0; key[i] = INV; st[i] = false;
    if (base + i < n) x[i] = rows_x(rks, poss, cnt, base + i, kmask, INV, shift, key[i], st[i]);
    s += x[i];
  }
  __shared__ uint64_t ws[RT_T / 64];
  const uint64_t incl = wave_incl_scan64(s);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 63) ws[w] = incl;
  __syncthreads();
  uint64_t run = offs[blockIdx.x] + incl - s;
  for (int k = 0; k < w; ++k) run += ws[k];
#pragma unroll
  for (int i = 0; i < RT_I; ++i) {
    if (wsorted && base + i < n) wsorted[base + i] = key[i] != INV ? (uint32_t)(run >> 24) : 0u;  // sorted order
    if (key[i] != INV) {
      const uint64_t woff = run >> 24;
      const uint32_t ps = poss[base + i];
      if (wsorted) {
      } else if (poff32) {
        if (ps - plo < pw) poff32[ps] = (uint32_t)woff;
      } else {
        poff[ps] = woff;
      }
      if (st[i] && write_rows) {
        const uint64_t r = run & 0xFFFFFFull;
        row_key[r] = key[i];
        row_begin[r] = woff;
      }
    }
    run += x[i];
  }
}

// the word offsets in event order from (position, offset) pairs already partitioned by the positions'
// high bits (k_rows_tile's wsorted + one radix pass): each pass of the grid writes into a few MB of
// the destination at a time, so the 4-B writes merge in the caches instead of one random line each
__global__ void k_poff_scatter(const uint32_t* __restrict__ pos, const uint32_t* __restrict__ woff, int64_t n,
                               uint32_t* __restrict__ poff32) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n) poff32[pos[k]] = woff[k];
}
// grouped row entries: a member's run starts at its rep's word offset plus its prefix in the group (LK_REP); the
// reps' offsets are final, so members read them while other members are written
// LF_PER events per thread (stride blockDim): their link and rep-offset loads are in flight together
constexpr int LF_PER = 8;
__global__ __launch_bounds__(256) void k_link_fix(const uint32_t* __restrict__ link, int64_t n,
                                                  uint32_t* __restrict__ poff32, uint64_t* __restrict__ poff) {
  const int64_t e0 = (int64_t)blockIdx.x * (256 * LF_PER) + threadIdx.x;
  uint32_t lk[LF_PER];
#pragma unroll
  for (int j = 0; j < LF_PER; ++j) lk[j] = e0 + j * 256 < n ? link[e0 + j * 256] : LK_REP;
  uint64_t o[LF_PER];
#pragma unroll
  for (int j = 0; j < LF_PER; ++j) {
    o[j] = 0;
    if (!(lk[j] & LK_REP)) {
      const int64_t r = e0 + j * 256 + (int64_t)(lk[j] >> LK_DSHIFT) - 512;
      o[j] = poff32 ? (uint64_t)poff32[r] : poff[r];
    }
  }
#pragma unroll
  for (int j = 0; j < LF_PER; ++j)
    if (!(lk[j] & LK_REP)) {
      const int64_t e = e0 + j * 256;
      if (poff32) poff32[e] = (uint32_t)(o[j] + (lk[j] & LK_GMASK));
      else poff[e] = o[j] + (lk[j] & LK_GMASK);
    }
}
// XCD-aware form: block b runs on XCD b % 8 (workgroups are dealt round robin) and XCD x writes only the
// slices (position high-bit digits) d = x (mod 8), one after the other, its blocks splitting each slice: a
// destination line is written through ONE L2, where its 4-B writes merge before the line goes to HBM (from
// eight XCDs a line went out in parts: 6.85 GB written per build for 0.88 GB of offsets). dstart[d * ntiles]
// = the first element of slice d (radix_pass' offsets); gridDim.x % 8 == 0.
__global__ __launch_bounds__(256) void k_poff_scatter_xcd(const uint32_t* __restrict__ pos,
                                                          const uint32_t* __restrict__ woff, int64_t n,
                                                          const uint64_t* __restrict__ dstart, int ntiles,
                                                          uint32_t* __restrict__ poff32) {
  const int x = blockIdx.x & 7, j = blockIdx.x >> 3, nj = gridDim.x >> 3;
  for (int d = x; d < 256; d += 8) {
    const int64_t a = (int64_t)dstart[(int64_t)d * ntiles];
    const int64_t b = d + 1 < 256 ? (int64_t)dstart[(int64_t)(d + 1) * ntiles] : n;
    const int64_t per = (b - a + nj - 1) / nj;
    const int64_t s0 = a + (int64_t)j * per, s1 = s0 + per < b ? s0 + per : b;
    for (int64_t k = s0 + threadIdx.x; k < s1; k += 256) poff32[pos[k]] = woff[k];
  }
}

// ---- rows without a sort (OTTOHIP_ROWS=atomic, one GPU): the row of key k is the dense index k of
// (type << A | aid); its words are cut into RA_SUB sub-ranges, one per counter, so the atomics of a hot
// row spread over RA_SUB addresses. Each event takes its run inside its sub-range with one returning
// atomic (word order inside a row is free: the reduce sorts it), one scan over the dense counters gives
// every sub-range its first word, and the event's word offset is that start plus its rank.
constexpr int RA_SUB = 8;
__device__ __forceinline__ uint32_t ra_sub(int64_t e) { return (uint32_t)(e >> 8) & (RA_SUB - 1); }
// RA_PER events per thread (coalesced, stride blockDim): their returning atomics are in flight together
// (one at a time leaves the kernel bound by the atomics' round-trip latency)
constexpr int RA_PER = 8;
__global__ __launch_bounds__(256) void k_rows_atomic(const uint32_t* __restrict__ rk, const uint32_t* __restrict__ cnt,
                                                     int64_t n, uint32_t kmask, uint32_t INV, uint32_t* __restrict__ dcnt,
                                                     uint32_t* __restrict__ rank) {
  const int64_t e0 = (int64_t)blockIdx.x * (256 * RA_PER) + threadIdx.x;
  uint32_t key[RA_PER], c[RA_PER], r[RA_PER];
#pragma unroll
  for (int j = 0; j < RA_PER; ++j) {
    const int64_t e = e0 + j * 256;
    key[j] = e < n ? rk[e] & kmask : INV;
    c[j] = key[j] != INV ? cnt[e] : 0u;
  }
#pragma unroll
  for (int j = 0; j < RA_PER; ++j)
    r[j] = c[j] ? atomicAdd(&dcnt[(uint64_t)key[j] * RA_SUB + ra_sub(e0 + j * 256)], c[j]) : 0u;
#pragma unroll
  for (int j = 0; j < RA_PER; ++j)
    if (e0 + j * 256 < n) rank[e0 + j * 256] = r[j];
}
// word offset of every event (u32 when P < 2^32, else u64) from its sub-range start and rank
__global__ __launch_bounds__(256) void k_rows_atomic_off(const uint32_t* __restrict__ rk, int64_t n, uint32_t kmask,
                                                         uint32_t INV, const uint64_t* __restrict__ doff,
                                                         const uint32_t* __restrict__ rank,
                                                         uint32_t* __restrict__ poff32, uint64_t* __restrict__ poff) {
  const int64_t e0 = (int64_t)blockIdx.x * (256 * RA_PER) + threadIdx.x;
  uint64_t o[RA_PER];
#pragma unroll
  for (int j = 0; j < RA_PER; ++j) {
    const int64_t e = e0 + j * 256;
    const uint32_t key = e < n ? rk[e] & kmask : INV;
    o[j] = key != INV ? doff[(uint64_t)key * RA_SUB + ra_sub(e)] + rank[e] : 0;
  }
#pragma unroll
  for (int j = 0; j < RA_PER; ++j) {
    const int64_t e = e0 + j * 256;
    if (e < n) { if (poff32) poff32[e] = (uint32_t)o[j]; else poff[e] = o[j]; }
  }
}
// dense rows: row r = key r, first word = its first sub-range's start
__global__ void k_rows_dense(const uint64_t* __restrict__ doff, int64_t nk, uint32_t* __restrict__ row_key,
                             uint64_t* __restrict__ row_begin) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= nk) return;
  row_key[r] = (uint32_t)r;
  row_begin[r] = doff[(uint64_t)r * RA_SUB];
}

// multi-GPU layout: row keys become (owner(aid), type, aid) so every owner's rows and words
// are contiguous (the all-to-all send segments); invalid events sort after every owner
__global__ void k_owner_key(uint32_t* __restrict__ rk, int64_t n, uint32_t INV, int A, uint32_t G, uint32_t INV2) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const uint32_t key = rk[k];
  rk[k] = key == INV ? INV2 : ((owner_dev(key & ((1u << A) - 1u), G) << (A + 2)) | key);
}

// the same owner-major order in fewer key bits (the fused row layout): (owner, type, the aid's index among its
// owner's aids), the count byte at cshift kept. Local indices follow aid order, so the sort order is the one of
// (owner, type, aid); k_rows_decode turns the rows' keys back into (type, aid)
__global__ void k_owner_key_local(uint32_t* __restrict__ rk, int64_t n, uint32_t INV, int A, uint32_t G, int LB,
                                  uint32_t INV2, uint32_t kmask, const uint32_t* __restrict__ a2l) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const uint32_t x = rk[k], key = x & kmask, hi = x & ~kmask;
  if (key == INV) { rk[k] = hi | INV2; return; }
  const uint32_t aid = key & ((1u << A) - 1u), t = key >> A;
  rk[k] = hi | (owner_dev(aid, G) << (LB + 2)) | (t << LB) | a2l[aid];
}
__global__ void k_rows_decode(uint32_t* __restrict__ row_key, int64_t R, int A, int LB,
                              const uint32_t* __restrict__ obase, const uint32_t* __restrict__ l2a) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= R) return;
  const uint32_t k = row_key[r], o = k >> (LB + 2), t = (k >> LB) & 3u, loc = k & ((1u << LB) - 1u);
  row_key[r] = (t << A) | l2a[obase[o] + loc];
}

// first row of every owner (rows are owner-major); first_row[G] = R
__global__ void k_part_bounds(const uint32_t* __restrict__ row_key, int64_t R, int A, uint32_t G,
                              uint64_t* __restrict__ first_row) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r > R) return;
  const int64_t prev = r == 0 ? -1 : (int64_t)owner_dev(row_key[r - 1] & ((1u << A) - 1u), G);
  const int64_t cur = r == R ? (int64_t)G : (int64_t)owner_dev(row_key[r] & ((1u << A) - 1u), G);
  for (int64_t o = prev + 1; o <= cur; ++o) first_row[o] = (uint64_t)r;
}

__global__ void k_part_words(const uint64_t* __restrict__ first_row, const uint64_t* __restrict__ row_begin, int64_t R,
                             uint64_t P, uint32_t G, uint64_t* __restrict__ first_word) {
  const uint32_t o = blockIdx.x * blockDim.x + threadIdx.x;
  if (o > G) return;
  const uint64_t r = first_row[o];
  first_word[o] = r < (uint64_t)R ? row_begin[r] : P;
}

// rows of one rank -> piece records (row_key << 32 | n_words), the all-to-all companion of the words
__global__ void k_piece_pack(const uint32_t* __restrict__ row_key, const uint64_t* __restrict__ row_begin, int64_t R,
                             uint64_t P, uint64_t* __restrict__ pieces) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= R) return;
  const uint64_t e = r + 1 < R ? row_begin[r + 1] : P;
  pieces[r] = ((uint64_t)row_key[r] << 32) | (e - row_begin[r]);
}

// ---- received pieces (one per (source, row)) -> one contiguous word range per row
// piece record: u64 (row_key << 32) | n_words
__global__ void k_piece_keys(const uint64_t* __restrict__ pieces, int64_t n, uint32_t* __restrict__ key,
                             uint32_t* __restrict__ val, uint32_t* __restrict__ len, uint32_t kmax,
                             int* __restrict__ err) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t p = pieces[i];
  const uint32_t k = (uint32_t)(p >> 32);
  if (k >= kmax) atomicOr(err, 1);
  key[i] = k;
  val[i] = (uint32_t)i;
  len[i] = (uint32_t)p;
}

__global__ void k_piece_order(const uint32_t* __restrict__ key, const uint32_t* __restrict__ val,
                              const uint32_t* __restrict__ len, int64_t n, uint32_t* __restrict__ len_sorted,
                              uint32_t* __restrict__ head) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  len_sorted[i] = len[val[i]];
  head[i] = (i == 0 || key[i] != key[i - 1]) ? 1u : 0u;
}

__global__ void k_piece_rows(const uint32_t* __restrict__ key, const uint32_t* __restrict__ head,
                             const uint64_t* __restrict__ row_idx, const uint64_t* __restrict__ dst, int64_t n,
                             uint32_t* __restrict__ row_key, uint64_t* __restrict__ row_begin) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || !head[i]) return;
  row_key[row_idx[i]] = key[i];
  row_begin[row_idx[i]] = dst[i];
}

// copies are cut into chunks of PC_CH words so hot rows (millions of words) spread over waves
constexpr uint32_t PC_CH = 2048;
__global__ void k_piece_nchunks(const uint32_t* __restrict__ lsort, int64_t n, uint32_t* __restrict__ nch) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) nch[i] = (lsort[i] + PC_CH - 1) / PC_CH;
}
__global__ void k_chunk_map(const uint32_t* __restrict__ nch, const uint64_t* __restrict__ cb, int64_t n,
                            uint32_t* __restrict__ cmap) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  for (uint32_t j = 0; j < nch[i]; ++j) cmap[cb[i] + j] = (uint32_t)i;
}
// one wave per chunk, 4 independent loads in flight per lane
__global__ __launch_bounds__(256) void k_piece_copy(const uint32_t* __restrict__ cmap, const uint64_t* __restrict__ cb,
                                                    int64_t n_chunks, const uint32_t* __restrict__ val,
                                                    const uint32_t* __restrict__ len,
                                                    const uint64_t* __restrict__ src_off,
                                                    const uint64_t* __restrict__ dst,
                                                    const uint32_t* __restrict__ in, uint32_t* __restrict__ out) {
  const int l = threadIdx.x & 63;
  const int64_t c = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (c >= n_chunks) return;
  const uint32_t i = cmap[c];
  const uint32_t p = val[i];
  const uint32_t o = (uint32_t)(c - (int64_t)cb[i]) * PC_CH;
  const uint32_t m = min(len[p] - o, PC_CH);
  const uint32_t* src = in + src_off[p] + o;
  uint32_t* d = out + dst[i] + o;
  uint32_t k = l;
  for (; k + 192 < m; k += 256) {
    const uint32_t a0 = src[k], a1 = src[k + 64], a2 = src[k + 128], a3 = src[k + 192];
    d[k] = a0; d[k + 64] = a1; d[k + 128] = a2; d[k + 192] = a3;
  }
  for (; k < m; k += 64) d[k] = src[k];
}

// ------------------------------------------------------------------ S4 emit
// cnt / poff are indexed [e0 + i]: global arrays with e0 = the session's first event, or the
// block's LDS copies with e0 = the session's offset inside the block
__device__ __forceinline__ void emit_session(const SessView& S, int64_t e0, const RulesDev& R, const Layout& L,
                                             uint32_t file, const uint32_t* __restrict__ cnt,
                                             EvOff poff, uint32_t* __restrict__ words,
                                             int dbg = 0) {
  const int l = lane_id();
  const int sg = l >> 4, sl = l & 15;
  const int shiftR = L.A + L.F;
  for (int i0 = 0; i0 < S.nv; i0 += 4) {
    const int i = i0 + sg;
    bool active = i < S.nv && cnt[e0 + i] != 0u;
    uint64_t out = active ? poff.run(e0 + i) : 0;
    const uint64_t e = active ? S.ev[i] : 0;
    const int t = ev_type(e);
    const int64_t tsi = ev_ts(e);
    const int nr = active ? R.n_of_type[t] : 0;
    for (int q = 0; q < nr; ++q) {
      const int r = R.rule_of_type[t][q];
      const int jb = lower_ts(S.ev, S.nv, tsi + R.lo[r]);
      const int je = (dbg & 2) ? jb : upper_ts(S.ev, S.nv, tsi + R.hi[r]);
      const uint32_t hi = ((uint32_t)q << shiftR) | file;
      for (int j0 = jb; j0 < je; j0 += 16) {
        const int j = j0 + sl;
        bool match = false;
        uint32_t word = 0;
        if (j < je) {
          const uint64_t ej = S.ev[j];
          match = ej != e && ((R.mask[r] >> ev_type(ej)) & 1u) && (!rule_sym(R, r) || ev_aid(ej) >= ev_aid(e));
          word = hi | ((uint32_t)ev_aid(ej) << L.F);
        }
        const uint32_t bal = (uint32_t)(__ballot(match) >> (sg * 16)) & 0xFFFFu;
        if (match && !(dbg & 1)) words[out + (uint64_t)__popc(bal & ((1u << sl) - 1u))] = word;
        out += (uint64_t)__popc(bal);
      }
    }
  }
}

// One wave per 256-event block (the sessions that start in it), processed in batches of whole
// sessions holding <= EB_CAP events. Per batch:
//   pass 1  events -> registers (coalesced), session of each event, per-type prefix counts
//   pass 2  per session, its events are re-laid out in LDS as three ts-sorted lists, one per
//           event type (a stable partition of the session's (ts, aid, type) order)
//   pass 3  per event and (rule, next type in the rule's mask): the window [jb, je) is a
//           binary search in that type's list, so every entry in it qualifies except the
//           event's own run (the identity of :23-27). These segments become records
//           (flattened start, list position, exclusion, output address); the wave then expands
//           the records 64 pairs at a time: each lane finds its record by binary search and
//           writes one word. Every lane writes a word in every round but the last of a flush,
//           independent of session length or of how selective a rule's type mask is.
// Sessions of more than LCAP events take k_emit_long.
constexpr int EB_CAP = 512;    // events per batch (positions fit 10 bits)
#ifndef OH_EB_RCAP
#define OH_EB_RCAP 64
#endif
#ifndef OH_EMIT_WPE
#define OH_EMIT_WPE
#endif
constexpr int EB_RCAP = OH_EB_RCAP;  // segment records per flush
// 64 <= EB_RCAP: one round of record building adds up to 64 records after a flush;
// EB_RCAP <= 128: the flush keeps two record starts per lane (32 overflowed the record arrays: LDS corruption)
static_assert(EB_RCAP >= 64 && EB_RCAP <= 128, "records per emit flush");
constexpr uint32_t EB_NONE = 1023u;

struct EmitRecs {
  uint4 rec[EB_RCAP];                   // per record: start, list position | exclusion, word high bits,
                                        // smallest partner aid written (symmetric rules: the event's aid)
  uint64_t rout[EB_RCAP];
  uint32_t rpre[EB_RCAP];               // record start in the flattened pair order
};
struct EmitPre {
  uint16_t pst[3][64], pen[3][64];      // per-type prefix counts at session start / end
};
struct EmitLds {
  uint64_t tev[EB_CAP];                 // type-partitioned events of the batch
  // passes 1-2 use the prefix counts, pass 3 and the flushes the records: one LDS range for both
  // (the batch's last flush ends before the next batch's pass 1, behind a wave barrier)
  union {
    EmitRecs r;
    EmitPre p;
  } u;
  uint16_t ss[65];                      // session start (batch-relative); ss[f] = batch size
  uint16_t sb[4][64];                   // per session: start of the type-t list; sb[3] = end of valid
  uint32_t sfile[64];
  uint16_t espos[EB_CAP];               // per batch event: position in tev (EB_NONE: invalid)
  uint8_t esid[EB_CAP];                 // per batch event: session index in the batch
  uint32_t mark[128];                   // flush round id at the window positions where a record starts
};

// expand records [0, nrec) holding tot pairs: lane k of round c writes pair c + k. Record starts
// are strictly increasing (a record holds >= 1 pair). Each lane keeps the starts of records l and
// l + 64 in registers and marks the window position of a start that falls in the round, so a
// lane's record is the last one of earlier rounds plus the marks at or below the lane: one LDS
// write and read per round instead of a binary search per pair.
// A record of a symmetric rule writes only the partners with aid >= its smallest aid (rec.w, the event's
// aid; 0 for other rules): a lane's word goes to the record's output at its rank among the record's
// written words -- those of earlier rounds (only the record spanning the round boundary has any: a
// wave-uniform carry) plus those of the record's lanes below it in this round (one ballot).
// GUARD (OTTOHIP_DEBUG): a lane whose record index falls outside [0, nrec) sets err bit 8 and writes
// nothing (the record arrays hold EB_RCAP entries; an out-of-range index would read stale LDS)
template <bool GUARD>
__device__ __forceinline__ void emit_flush(EmitLds& S, int nrec, uint32_t tot, int F, uint32_t* __restrict__ words,
                                           int dbg, uint32_t& rid, int* __restrict__ err) {
  if (dbg & 2) return;  // profiling ablation: records are built, never expanded
  const uint32_t l = lane_id();
  const uint32_t sa = (int)l < nrec ? S.u.r.rpre[l] : 0xFFFFFFFFu;
  const uint32_t sb = (int)l + 64 < nrec ? S.u.r.rpre[l + 64] : 0xFFFFFFFFu;
  const uint64_t below = (1ull << l) - 1ull, upto = below | (1ull << l);  // lanes < l, <= l
  int ob = -1;        // last record starting before the round's window
  uint32_t cc = 0;    // words written in earlier rounds by the record spanning into this round
  for (uint32_t c = 0; c < tot; c += 64) {
    ++rid;
    if (sa - c < 64u) S.mark[sa - c] = rid;
    if (sb - c < 64u) S.mark[sb - c] = rid;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    const uint64_t mm = __ballot(S.mark[l] == rid);
    const uint64_t mle = mm & upto;
#ifndef OH_EMIT_NOCHECK  // always on, as in emit_flush2: the record index clamped into [0, nrec), marks counted below
    const int o = min(max(ob + (int)__popcll(mle), 0), nrec - 1);
#else
    const int o = ob + (int)__popcll(mle);
#endif
    ob += (int)__popcll(mm);
    const uint32_t p = c + l;
    bool qual = false;
    uint32_t word = 0;
    const bool bad = GUARD && p < tot && (o < 0 || o >= nrec);
    if (bad) atomicOr(err, 8);
    if (p < tot && !bad) {
      const uint4 rc = S.u.r.rec[o];
      uint32_t j = (rc.y & 1023u) + (p - rc.x);
      if (j >= ((rc.y >> 10) & 1023u)) j += rc.y >> 21;
      const uint32_t a = (uint32_t)ev_aid(S.tev[j]);
      qual = a >= rc.w;
      word = rc.z | (a << F);
    }
    const uint64_t Q = __ballot(qual);
    // the record's lanes in this round start at its mark, or at lane 0 for the spanning record
    const uint32_t first = mle ? 63u - (uint32_t)__builtin_clzll(mle) : 0u;
    const uint64_t mine = Q & ~((1ull << first) - 1ull);
    const uint32_t car = mle ? 0u : cc;
    if (qual && !(dbg & 1) && !bad) words[S.u.r.rout[o] + car + (uint32_t)__popcll(mine & below)] = word;
    cc = (uint32_t)__builtin_amdgcn_readlane((int)(car + (uint32_t)__popcll(mine)), 63);
  }
  // every record start falls in exactly one round: the marks seen must number nrec (err bit 8 -> the call fails)
#ifndef OH_EMIT_NOCHECK
  if (tot > 0 && ob != nrec - 1 && l == 0) atomicOr(err, 8);
#endif
}

// emit_flush with two pairs per lane per round (128 pairs: lane k writes pairs c + k and c + 64 + k): one mark
// round (writes, barrier) and one loop trip per 128 pairs, and the two halves' record / list reads in flight
// together. The halves run the same rank logic in order; the spanning record's carry passes from half to half.
template <bool GUARD>
__device__ __forceinline__ void emit_flush2(EmitLds& S, int nrec, uint32_t tot, int F, uint32_t* __restrict__ words,
                                            int dbg, uint32_t& rid, int* __restrict__ err) {
  if (dbg & 2) return;  // profiling ablation: records are built, never expanded
  const uint32_t l = lane_id();
  const uint32_t sa = (int)l < nrec ? S.u.r.rpre[l] : 0xFFFFFFFFu;
  const uint32_t sb = (int)l + 64 < nrec ? S.u.r.rpre[l + 64] : 0xFFFFFFFFu;
  const uint64_t below = (1ull << l) - 1ull, upto = below | (1ull << l);  // lanes < l, <= l
  int ob = -1;        // last record starting before the current half's window
  uint32_t cc = 0;    // words written in earlier halves by the record spanning into the current one
  for (uint32_t c = 0; c < tot; c += 128) {
    ++rid;
    if (sa - c < 128u) S.mark[sa - c] = rid;
    if (sb - c < 128u) S.mark[sb - c] = rid;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    const uint64_t mA = __ballot(S.mark[l] == rid), mB = __ballot(S.mark[64 + l] == rid);
    const uint64_t mleA = mA & upto, mleB = mB & upto;
#ifndef OH_EMIT_NOCHECK  // (a cost A/B build only: tools/build_ab.sh -DOH_EMIT_NOCHECK)
    // always on: a lane's record index is clamped into [0, nrec), so a stale or extra mark (round 4: uninitialised
    // mark[64..127] equal to a later round id) can no longer index past the records and write words at a wild
    // address; the count of marks is checked after the loop (err bit 8) and the call fails
    const int oA = min(max(ob + (int)__popcll(mleA), 0), nrec - 1);
    const int oB = min(max(ob + (int)__popcll(mA) + (int)__popcll(mleB), 0), nrec - 1);
#else
    const int oA = ob + (int)__popcll(mleA);
    const int oB = ob + (int)__popcll(mA) + (int)__popcll(mleB);
#endif
    ob += (int)__popcll(mA) + (int)__popcll(mB);
    const uint32_t pA = c + l, pB = c + 64 + l;
    bool qA = false, qB = false;
    uint32_t wA = 0, wB = 0;
    uint64_t dA = 0, dB = 0;
    const bool badA = GUARD && pA < tot && (oA < 0 || oA >= nrec);
    const bool badB = GUARD && pB < tot && (oB < 0 || oB >= nrec);
    if (badA || badB) atomicOr(err, 8);
    if (pA < tot && !badA) {
      const uint4 rc = S.u.r.rec[oA];
      uint32_t j = (rc.y & 1023u) + (pA - rc.x);
      if (j >= ((rc.y >> 10) & 1023u)) j += rc.y >> 21;
      const uint32_t a = (uint32_t)ev_aid(S.tev[j]);
      qA = a >= rc.w;
      wA = rc.z | (a << F);
      dA = S.u.r.rout[oA];
    }
    if (pB < tot && !badB) {
      const uint4 rc = S.u.r.rec[oB];
      uint32_t j = (rc.y & 1023u) + (pB - rc.x);
      if (j >= ((rc.y >> 10) & 1023u)) j += rc.y >> 21;
      const uint32_t a = (uint32_t)ev_aid(S.tev[j]);
      qB = a >= rc.w;
      wB = rc.z | (a << F);
      dB = S.u.r.rout[oB];
    }
    // half A: the record's lanes start at its mark, or at lane 0 for the record spanning into the half
    const uint64_t QA = __ballot(qA);
    const uint32_t firstA = mleA ? 63u - (uint32_t)__builtin_clzll(mleA) : 0u;
    const uint64_t mineA = QA & ~((1ull << firstA) - 1ull);
    const uint32_t carA = mleA ? 0u : cc;
    if (qA && !(dbg & 1)) words[dA + carA + (uint32_t)__popcll(mineA & below)] = wA;
    cc = (uint32_t)__builtin_amdgcn_readlane((int)(carA + (uint32_t)__popcll(mineA)), 63);
    // half B
    const uint64_t QB = __ballot(qB);
    const uint32_t firstB = mleB ? 63u - (uint32_t)__builtin_clzll(mleB) : 0u;
    const uint64_t mineB = QB & ~((1ull << firstB) - 1ull);
    const uint32_t carB = mleB ? 0u : cc;
    if (qB && !(dbg & 1)) words[dB + carB + (uint32_t)__popcll(mineB & below)] = wB;
    cc = (uint32_t)__builtin_amdgcn_readlane((int)(carB + (uint32_t)__popcll(mineB)), 63);
  }
  // every record start falls in exactly one round: the marks seen must number nrec (always on, wave-uniform)
#ifndef OH_EMIT_NOCHECK
  if (tot > 0 && ob != nrec - 1 && l == 0) atomicOr(err, 8);
#endif
}

// Per event type, the (rule, next type) windows an event of that type writes, as pass 3's task list: entry
// q | tt << 4 | sym << 6, the non-symmetric rules first (a symmetric record's written length is only known to
// S2's count, so it goes last in the event's run)
struct EmitTasks {
  uint8_t e[3][3 * MAX_RULES];
  uint8_t n[4];
};
__device__ inline void emit_tasks_build(const RulesDev& R, EmitTasks& T) {
  for (int t = 0; t < 3; ++t) {
    int n = 0;
    for (int pass = 0; pass < 2; ++pass)
      for (int q = 0; q < R.n_of_type[t]; ++q) {
        const int r = R.rule_of_type[t][q];
        if (rule_sym(R, r) != (pass == 1)) continue;
        for (int tt = 0; tt < 3; ++tt)
          if ((R.mask[r] >> tt) & 1u) T.e[t][n++] = (uint8_t)(q | (tt << 4) | (pass << 6));
      }
    T.n[t] = (uint8_t)n;
  }
  T.n[3] = 0;
}

// GUARD (OTTOHIP_DEBUG): bounds checks of the record arrays (err bit 8). TASKS: pass 3 iterates the per-type
// task lists (lanes of different types search their own lists together); else (OTTOHIP_EMIT_TASKS=0) every
// (rule, next type) of the wave's types in turn
template <bool GUARD, bool TASKS, bool FL2 = true>
__global__ __launch_bounds__(64) OH_EMIT_WPE void k_emit(const int64_t* __restrict__ off, const int64_t* __restrict__ first,
                                             int64_t NB, const uint64_t* __restrict__ ev, RulesDev R, Layout L,
                                             const int64_t* __restrict__ fb, int nf, const uint32_t* __restrict__ fid,
                                             const uint32_t* __restrict__ cnt, EvOff poff,
                                             uint32_t* __restrict__ words, int* __restrict__ err, int dbg) {
  __shared__ EmitLds S;
  __shared__ RulesDev sR;
  __shared__ EmitTasks sT;
  const int l = threadIdx.x;
  if (l == 0) sR = R;
  if (TASKS && l == 0) emit_tasks_build(R, sT);
  const int64_t g = blockIdx.x;
  if (g >= NB) return;
  const int64_t s0 = first[g], s1 = first[g + 1];
  if (s0 >= s1) return;
  const int shiftR = L.A + L.F;
  int maxq = 0;
#pragma unroll
  for (int t = 0; t < 3; ++t) maxq = max(maxq, R.n_of_type[t]);
  S.mark[l] = 0u;  // (both halves: a stale value equal to a later round id would be a false record start)
  S.mark[64 + l] = 0u;
  uint32_t rid = 0;  // flush round id (marks of earlier rounds never match)
  int fcur = file_of(fb, nf, s0);
  int64_t next_b = fcur + 1 < nf ? fb[fcur + 1] : INT64_MAX;
  uint32_t fid_cur = fid[fcur];
  __syncthreads();
  const int maxtask = TASKS ? max((int)sT.n[0], max((int)sT.n[1], (int)sT.n[2])) : 0;

  int64_t b = s0;
  while (b < s1) {
    // ---- batch: sessions [b, b + nsess) with <= EB_CAP events, none longer than LCAP
    const int64_t base = off[b];
    const int64_t s = b + l;
    const bool in_s = s < s1;
    const int64_t so = in_s ? off[s] : 0, se = in_s ? off[s + 1] : 0;
    const bool ok = in_s && se - base <= EB_CAP && se - so <= LCAP;
    const uint64_t bad = __ballot(!ok);
    const int nsess = bad ? (int)__builtin_ctzll(bad) : 64;
    if (nsess == 0) { ++b; continue; }  // session b is long (k_emit_long)
    const int nb_ev = (int)(__shfl((int)(se - base), nsess - 1));
    const int64_t E0 = base;
    if (l < nsess) S.ss[l] = (uint16_t)(so - base);
    if (l == 0) S.ss[nsess] = (uint16_t)nb_ev;
    // file of every session (one file for the whole batch unless a file boundary is crossed)
    const int64_t s_last = b + nsess - 1;
    if (s_last < next_b) {
      if (l < nsess) S.sfile[l] = fid_cur;
    } else {
      int fk = fcur;
      if (l < nsess) {
        while (fk + 1 < nf && fb[fk + 1] <= s) ++fk;
        S.sfile[l] = fid[fk];
      }
      fcur = __shfl(fk, nsess - 1);
      next_b = fcur + 1 < nf ? fb[fcur + 1] : INT64_MAX;
      fid_cur = fid[fcur];
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");

    // ---- pass 1: events, sessions, per-type prefixes
    constexpr int NCH = EB_CAP / 64;
    const int nch = (nb_ev + 63) >> 6;
    uint64_t vv[NCH];
    uint32_t sid[NCH], pr[NCH];
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int idx = c * 64 + l;
      vv[c] = (c < nch && idx < nb_ev) ? ev[E0 + idx] : EV_INVALID;
    }
    uint32_t base0 = 0, base1 = 0, base2 = 0;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      if (c >= nch) break;
      const int idx = c * 64 + l;
      const bool in = idx < nb_ev;
      const int t = in ? ev_type(vv[c]) : 3;
      int k = 0;
#pragma unroll
      for (int st = 32; st >= 1; st >>= 1)
        if (k + st < nsess && (int)S.ss[k + st] <= idx) k += st;
      const uint64_t m0 = __ballot(t == 0), m1 = __ballot(t == 1), m2 = __ballot(t == 2);
      const uint32_t P0 = base0 + mbcnt(m0), P1 = base1 + mbcnt(m1), P2 = base2 + mbcnt(m2);
      if (in && idx == (int)S.ss[k]) { S.u.p.pst[0][k] = P0; S.u.p.pst[1][k] = P1; S.u.p.pst[2][k] = P2; }
      if (in && idx == (int)S.ss[k + 1] - 1) {
        S.u.p.pen[0][k] = P0 + (t == 0); S.u.p.pen[1][k] = P1 + (t == 1); S.u.p.pen[2][k] = P2 + (t == 2);
      }
      base0 += (uint32_t)__popcll(m0); base1 += (uint32_t)__popcll(m1); base2 += (uint32_t)__popcll(m2);
      sid[c] = (uint32_t)k;
      pr[c] = t == 0 ? P0 : (t == 1 ? P1 : P2);
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    if (l < nsess) {
      const uint32_t a = S.ss[l];
      if (S.ss[l + 1] > a) {
        const uint32_t c0 = S.u.p.pen[0][l] - S.u.p.pst[0][l], c1 = S.u.p.pen[1][l] - S.u.p.pst[1][l], c2 = S.u.p.pen[2][l] - S.u.p.pst[2][l];
        S.sb[0][l] = a; S.sb[1][l] = a + c0; S.sb[2][l] = a + c0 + c1; S.sb[3][l] = a + c0 + c1 + c2;
      }
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    // ---- pass 2: type-partitioned lists
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      if (c >= nch) break;
      const int idx = c * 64 + l;
      const int t = ev_type(vv[c]);
      if (idx < nb_ev) {
        uint32_t pos = EB_NONE;
        if (t < 3) {
          const uint32_t k = sid[c];
          pos = S.sb[t][k] + pr[c] - S.u.p.pst[t][k];
          S.tev[pos] = vv[c];
        }
        S.espos[idx] = (uint16_t)pos;
        S.esid[idx] = (uint8_t)sid[c];
      }
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    // ---- pass 3: segments -> records -> words
    int nrec = 0;
    uint32_t tot = 0;
#pragma unroll 1
    for (int c = 0; c < nch; ++c) {
      const int idx = c * 64 + l;
      const bool in = idx < nb_ev;
      const uint32_t sp = in ? S.espos[idx] : EB_NONE;
      const bool valid = sp != EB_NONE;
      const uint64_t v = valid ? S.tev[sp] : EV_INVALID;
      const int t = ev_type(v);
      const uint32_t k = in ? S.esid[idx] : 0u;
      const uint64_t eout = valid && cnt[E0 + idx] ? poff.run(E0 + idx) : 0;
      const uint32_t ecnt = valid ? cnt[E0 + idx] : 0;
      const int64_t tsi = ev_ts(v);
      const uint32_t file = S.sfile[k];
      // the event's own run in its list (exact twins stay adjacent when dedup is off)
      uint32_t rlo = sp, rhi = sp + 1;
      if (valid) {
        const uint32_t lb = S.sb[t][k], ub = S.sb[t + 1][k];
        while (rlo > lb && S.tev[rlo - 1] == v) --rlo;
        while (rhi < ub && S.tev[rhi] == v) ++rhi;
      }
      uint32_t eo = 0;
      bool has_sym = false;
      if constexpr (TASKS) {
        // task kk of the lane's event: the (rule, next type) list window of the kk-th entry of its type's task
        // table (symmetric rules last): lanes of different types search their own lists in one iteration
        const int ntk = valid ? (int)sT.n[t] : 0;
#pragma unroll 1
        for (int kk = 0; kk < maxtask; ++kk) {
          const bool act = kk < ntk;
          if (!__ballot(act)) break;
          const uint32_t te = act ? (uint32_t)sT.e[t][kk] : 0u;
          const int q = (int)(te & 15u), tt = (int)((te >> 4) & 3u);
          const bool sym = act && ((te >> 6) & 1u);
          const int r = act ? sR.rule_of_type[t][q] : 0;
          const int32_t lo = sR.lo[r], hi = sR.hi[r];
          has_sym |= sym;
          uint32_t len = 0, jb = 0, xlo = EB_NONE, xlen = 0;
          if (act) {
            const int a = S.sb[tt][k], e = S.sb[tt + 1][k];
            // own list with a window around dt = 0: the lower bound lies at or before the event's own run and the
            // upper bound at or after it (the list is in ts order), so each search takes half of the list
            const bool own = tt == t && lo <= 0 && hi >= 0;
            jb = (uint32_t)lds_lower_ts(S.tev, a, own ? (int)rlo : e, tsi + lo);
            const uint32_t je = (uint32_t)lds_upper_ts(S.tev, own ? (int)rhi : (int)jb, e, tsi + hi);
            len = je - jb;
            if (own) { xlo = rlo; xlen = rhi - rlo; len -= xlen; }
          }
          const uint64_t m = __ballot(len > 0);
          const int nn = (int)__popcll(m);
          if (nn == 0) continue;
          if (nrec + nn > EB_RCAP) {
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            (FL2 ? emit_flush2<GUARD> : emit_flush<GUARD>)(S, nrec, tot, L.F, words, dbg, rid, err);
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            nrec = 0; tot = 0;
          }
          const uint32_t incl = wave_incl_scan(len);
          if (GUARD && nrec + nn > EB_RCAP) atomicOr(err, 8);  // the record arrays would overflow
          if (len > 0 && !(GUARD && nrec + (int)mbcnt(m) >= EB_RCAP)) {
            const int ri = nrec + (int)mbcnt(m);
            S.u.r.rpre[ri] = tot + incl - len;
            S.u.r.rec[ri] = make_uint4(tot + incl - len, jb | (xlo << 10) | (xlen << 21), ((uint32_t)q << shiftR) | file,
                                   sym ? (uint32_t)ev_aid(v) : 0u);
            S.u.r.rout[ri] = eout + eo;
          }
          if (!sym) eo += len;
          nrec += nn;
          tot += __shfl(incl, 63);
        }
      } else {
        const int nq = valid ? sR.n_of_type[t] : 0;
        // the event's symmetric-rule record comes last: its written length is only known to S2's count
        bool lane_sym = false;
        for (int q = 0; q < nq; ++q) lane_sym |= rule_sym(sR, sR.rule_of_type[t][q]);
        const int nqq = __ballot(lane_sym) ? 2 * maxq : maxq;
#pragma unroll 1
        for (int qq = 0; qq < nqq; ++qq) {
          const int q = qq % maxq, pass = qq / maxq;
          const int r = q < nq ? sR.rule_of_type[t][q] : 0;
          const bool sym = q < nq && rule_sym(sR, r);
          const uint32_t msk = (q < nq && sym == (pass == 1)) ? sR.mask[r] : 0u;
          const int32_t lo = sR.lo[r], hi = sR.hi[r];
          has_sym |= msk != 0u && sym;
#pragma unroll 1
          for (int tt = 0; tt < 3; ++tt) {
            const bool act = (msk >> tt) & 1u;
            if (!__ballot(act)) continue;
            uint32_t len = 0, jb = 0, xlo = EB_NONE, xlen = 0;
            if (act) {
              const int a = S.sb[tt][k], e = S.sb[tt + 1][k];
              jb = (uint32_t)lds_lower_ts(S.tev, a, e, tsi + lo);
              const uint32_t je = (uint32_t)lds_upper_ts(S.tev, (int)jb, e, tsi + hi);
              len = je - jb;
              if (tt == t && lo <= 0 && hi >= 0) { xlo = rlo; xlen = rhi - rlo; len -= xlen; }
            }
            const uint64_t m = __ballot(len > 0);
            const int nn = (int)__popcll(m);
            if (nn == 0) continue;
            if (nrec + nn > EB_RCAP) {
              __builtin_amdgcn_wave_barrier();
              __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
              (FL2 ? emit_flush2<GUARD> : emit_flush<GUARD>)(S, nrec, tot, L.F, words, dbg, rid, err);
              __builtin_amdgcn_wave_barrier();
              __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
              nrec = 0; tot = 0;
            }
            const uint32_t incl = wave_incl_scan(len);
            if (GUARD && nrec + nn > EB_RCAP) atomicOr(err, 8);  // the record arrays would overflow
            if (len > 0 && !(GUARD && nrec + (int)mbcnt(m) >= EB_RCAP)) {
              const int ri = nrec + (int)mbcnt(m);
              S.u.r.rpre[ri] = tot + incl - len;
              S.u.r.rec[ri] = make_uint4(tot + incl - len, jb | (xlo << 10) | (xlen << 21), ((uint32_t)q << shiftR) | file,
                                     sym ? (uint32_t)ev_aid(v) : 0u);
              S.u.r.rout[ri] = eout + eo;
            }
            if (!sym) eo += len;
            nrec += nn;
            tot += __shfl(incl, 63);
          }
        }
      }
      if (valid && (has_sym ? eo > ecnt : eo != ecnt)) atomicOr(err, 4);
    }
    if (nrec > 0) {
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      (FL2 ? emit_flush2<GUARD> : emit_flush<GUARD>)(S, nrec, tot, L.F, words, dbg, rid, err);
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    b += nsess;
  }
}

__global__ __launch_bounds__(64) void k_emit_long(const int64_t* __restrict__ off, const int32_t* __restrict__ list,
                                                  const int64_t* __restrict__ scratch_off,
                                                  uint64_t* __restrict__ scratch, uint32_t* __restrict__ pscratch,
                                                  const uint64_t* __restrict__ ev, RulesDev R, Layout L,
                                                  const int64_t* __restrict__ fb, int nf,
                                                  const uint32_t* __restrict__ fid,
                                                  const uint32_t* __restrict__ cnt, EvOff poff,
                                                  uint32_t* __restrict__ words) {
  const int64_t s = list[blockIdx.x];
  const int64_t e0 = off[s];
  const int n = (int)(off[s + 1] - e0);
  const int64_t so = scratch_off[blockIdx.x];
  SessView S;
  uint64_t* evs = scratch + 2 * so;
  uint32_t* pref = pscratch + 3 * (so + blockIdx.x);
  S.ev = evs; S.pref = pref; S.pstride = n + 1;
  S.nv = load_session(ev + e0, n, evs, pref, n + 1);
  emit_session(S, e0, R, L, fid[file_of(fb, nf, s)], cnt, poff, words);
}

// ------------------------------------------------------------------ S5 reduce
__device__ __forceinline__ uint32_t hslot(uint32_t w, uint32_t mask) { return (w * 0x9E3779B1u >> 7) & mask; }

// row (type, aid) -> global rule id and output fields
struct RowInfo { int type; int32_t aid; };
__device__ __forceinline__ RowInfo row_info(const uint32_t* row_key, uint32_t row, int A) {
  const uint32_t k = row_key[row];
  RowInfo ri; ri.type = (int)(k >> A); ri.aid = (int32_t)(k & ((1u << A) - 1u));
  return ri;
}

__device__ __forceinline__ void put_row(const OutRows& O, uint64_t p, int rule, int32_t aid, int32_t next,
                                        uint32_t c, uint32_t c2) {
  if (p < O.cap) {
    O.rule[p] = (uint8_t)rule; O.aid[p] = aid; O.aid_next[p] = next; O.count[p] = c; O.count_ge2[p] = c2;
  }
}

// per-thread statistics per global rule, indexed statically (no scratch)
struct RuleAcc {
  uint32_t rows[MAX_RULES], nf1[MAX_RULES], nf2[MAX_RULES];
  unsigned long long pairs[MAX_RULES];
  uint32_t raw_rows;
  unsigned long long raw_pairs;
  __device__ void zero() {
#pragma unroll
    for (int r = 0; r < MAX_RULES; ++r) { rows[r] = nf1[r] = nf2[r] = 0; pairs[r] = 0; }
    raw_rows = 0; raw_pairs = 0;
  }
  // mult 2: a symmetric rule's row with aid != aid_next (its mirror row counts too)
  __device__ void add(int rule, uint32_t c, uint32_t nf, uint32_t mult) {
#pragma unroll
    for (int r = 0; r < MAX_RULES; ++r)
      if (r == rule) {
        rows[r] += mult; pairs[r] += (unsigned long long)c * mult; nf1[r] += (nf & 0xFFFFu) * mult;
        nf2[r] += (nf >> 16) * mult;
      }
    raw_rows += 1; raw_pairs += c;
  }
  // wave reduction, then one device atomic per nonzero statistic into this wave's stripe of
  // the striped statistics array (STAT_STRIPES copies: same-address atomics serialise in L2)
  __device__ void flush(unsigned long long* stats_striped, int n_rules) {
    const uint32_t gwave = (blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
    unsigned long long* stats = stats_striped + (size_t)(gwave & (STAT_STRIPES - 1)) * STAT_STRIDE;
    for (int r = 0; r < n_rules; ++r) {
      unsigned long long v[4] = {rows[0], pairs[0], nf1[0], nf2[0]};
#pragma unroll
      for (int q = 0; q < MAX_RULES; ++q)
        if (q == r) { v[0] = rows[q]; v[1] = pairs[q]; v[2] = nf1[q]; v[3] = nf2[q]; }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        unsigned long long x = v[k];
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) {
          const uint32_t lo = __shfl_xor((uint32_t)x, d), hi = __shfl_xor((uint32_t)(x >> 32), d);
          x += ((unsigned long long)hi << 32) | lo;
        }
        if (lane_id() == 0 && x) atomicAdd(&stats[r * 4 + k], x);
      }
    }
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      unsigned long long x = k == 0 ? (unsigned long long)raw_rows : raw_pairs;
#pragma unroll
      for (int d = 32; d >= 1; d >>= 1) {
        const uint32_t lo = __shfl_xor((uint32_t)x, d), hi = __shfl_xor((uint32_t)(x >> 32), d);
        x += ((unsigned long long)hi << 32) | lo;
      }
      if (lane_id() == 0 && x) atomicAdd(&stats[STAT_RAW + k], x);
    }
  }
};

// one workgroup per task: LDS hash of (rule|aid_next|file) counts, then folded over files.
// Phase A slots: u64 (word << 32 | count); phase B: u64 (key2 << 32 | count) + u64 (count_ge2 << 32 | nf2 << 16 | nf1)
constexpr int AGG_T = 256;
constexpr int HCAP = 4096;
constexpr unsigned long long SLOT_EMPTY = 0xFFFFFFFF00000000ull;

__device__ __forceinline__ unsigned long long lds_load(unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
constexpr uint32_t HASH_FULL = 0xFFFFFFFFu;  // hash_insert_batch: table full

// ---- register sort path: one wave per task of <= 64*M words, no LDS, no atomics
__device__ __forceinline__ uint32_t wave_incl_max(uint32_t v) { return dpp_incl_scan<true>(v); }

// median of three: with c = 0 it is min(a, b), with c = ~0 max(a, b). Written in C (the backend
// folds min(max(min(a, b), c), max(a, b)) into one v_med3_u32): an inline-asm med3 is opaque to
// the hazard recognizer, which then padded every following DPP move with s_nop
__device__ __forceinline__ uint32_t umed3(uint32_t a, uint32_t b, uint32_t c) {
  const uint32_t mn = a < b ? a : b, mx = a < b ? b : a;
  const uint32_t t = mn > c ? mn : c;
  return mx < t ? mx : t;
}

// Bitonic sort of 64*M keys held as v[m] = element (lane*M + m), ascending. Every
// compare-exchange is one v_med3_u32 against a sentinel (0: keep the min, ~0: keep the max)
// that depends only on the lane and the stage; partners in other lanes come by DPP / permlane.
template <int M>
__device__ __forceinline__ void wave_bitonic_sort(uint32_t (&v)[M]) {
  constexpr int N = 64 * M;
  uint32_t l = lane_id();
  asm volatile("" : "+v"(l));  // keeps the per-stage sentinels from being hoisted into registers
#pragma unroll
  for (int k = 2; k <= N; k <<= 1) {
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1) {
      // sentinels by arithmetic on the lane bits (no lane-mask registers): 0 = keep the min
      const int kb = __builtin_ctz(k), jb = __builtin_ctz(j);
      if (j >= M && (j / M == 16 || j / M == 32) && M >= 2) {
        // partner 16 / 32 lanes away: one v_permlane16/32_swap of two registers puts every pair's
        // lower element in the first and its upper element in the second at the same lane, an
        // in-lane compare-exchange (two med3) sorts both registers' pairs, a second swap puts
        // them back: 2 VALU per register instead of a swap, a copy, a select and a med3
        const uint32_t lo_lane = l & ~(uint32_t)(j / M);  // lane of the pair's lower element
        const uint32_t smin = 0u - (((lo_lane * M) >> kb) & 1u);  // 0: the lower element takes the min
#pragma unroll
        for (int m = 0; m < M; m += 2) {
          uint32_t x = v[m], y = v[m + 1];
          if (j / M == 16) {
            const auto sw = __builtin_amdgcn_permlane16_swap(x, y, false, false);
            x = sw[0]; y = sw[1];
          } else {
            const auto sw = __builtin_amdgcn_permlane32_swap(x, y, false, false);
            x = sw[0]; y = sw[1];
          }
          const uint32_t lo = umed3(x, y, smin), hi = umed3(x, y, ~smin);
          if (j / M == 16) {
            const auto sw = __builtin_amdgcn_permlane16_swap(lo, hi, false, false);
            v[m] = sw[0]; v[m + 1] = sw[1];
          } else {
            const auto sw = __builtin_amdgcn_permlane32_swap(lo, hi, false, false);
            v[m] = sw[0]; v[m + 1] = sw[1];
          }
        }
      } else if (j >= M) {  // partner in lane l ^ (j / M), same register; direction from lane bits only
        const uint32_t sent = 0u - ((((l * M) >> kb) ^ ((l * M) >> jb)) & 1u);
#pragma unroll
        for (int m = 0; m < M; ++m) v[m] = umed3(v[m], xor_lane_n(v[m], j / M), sent);
      } else {  // partner in this lane
        const uint32_t lane_slo = 0u - (((l * M) >> kb) & 1u);  // used when k >= M
#pragma unroll
        for (int m = 0; m < M; ++m) {
          if (m & j) continue;
          const uint32_t slo = k < M ? ((m & k) ? ~0u : 0u) : lane_slo;
          const uint32_t a = v[m], b = v[m ^ j];
          v[m] = umed3(a, b, slo);
          v[m ^ j] = umed3(a, b, ~slo);
        }
      }
    }
  }
}

// inclusive scan over elements e = lane*M + m (sum or max)
template <int M, bool MAX>
__device__ __forceinline__ void wave_scan_elems(uint32_t (&x)[M]) {
#pragma unroll
  for (int m = 1; m < M; ++m) x[m] = MAX ? (x[m] > x[m - 1] ? x[m] : x[m - 1]) : x[m] + x[m - 1];
  const uint32_t tot = x[M - 1];
  const uint32_t incl = dpp_incl_scan<MAX>(tot);
  const uint32_t excl = lane_prev(incl);
#pragma unroll
  for (int m = 0; m < M; ++m) x[m] = MAX ? (x[m] > excl ? x[m] : excl) : x[m] + excl;
}

// exclusive value before element e = lane*M + m of a per-element inclusive prefix x
template <int M>
__device__ __forceinline__ uint32_t excl_at(const uint32_t (&x)[M], int m, uint32_t lane_prev_tot) {
  return m > 0 ? x[m - 1] : lane_prev_tot;
}

// The fold of one sorted task (k_agg_sort, k_agg_lds): v holds its <= 64*M words (W_EMPTY past the
// end), unsorted; rows go to the slots [obegin, obegin + olen) of the table (the task's own word range),
// the rest of that range is marked empty. stgk / stgb: this wave's staging rows (64*M + 64 each),
// sacc: this wave's statistics accumulator, P / fh: the FO kernels' part tables and per-file rows.
// One run-fold pass over a sorted task (v, with the cross-lane neighbours pl / nl): rows (one per k-run end) are
// staged in this wave's LDS and written to the slots [obegin, obegin + olen). PM: pt holds each element's part
// (pmode), and a k-run is one (key, part). MIRROR: the pass writes the explicit mirror rows (part, aid_next, aid)
// of a symmetric rule's stored rows (pt = the mirrors' parts; the diagonal aid_next == aid has no mirror) and
// takes no statistics; else FO adds the FileOpts rule's per-file rows (fh) and the per-rule statistics go to sacc.
template <int M, bool FO, bool PM, bool MIRROR>
__device__ __forceinline__ uint32_t fold_pass(const uint32_t (&v)[M], uint32_t pl, uint32_t nl, const uint32_t* pt,
                                          uint32_t ppl, uint32_t pnl, bool pmode, uint64_t obegin, uint32_t olen,
                                          uint32_t rk, const RulesDev& sR, const Layout& L, const OutRows& O,
                                          const FileOpts& fo, unsigned long long* fh, uint32_t* stgk, uint32_t* stgb,
                                          unsigned long long* sacc) {
  const uint32_t l = lane_id();
  const int F = L.F, A = L.A;
  // (1) run flags from the neighbours (a w-run = one word = one (rule, aid_next, file)):
  //     X = [w-run end] | [singleton w-run] << 11, summed by one scan (fields <= 1024);
  //     k-run (rule, aid_next) starts and ends as bit masks over the lane's elements
  uint32_t a[M], b[M], c[M];
  uint32_t kst = 0, kend = 0;
#pragma unroll
  for (int m = 0; m < M; ++m) {
    const uint32_t prv = m > 0 ? v[m - 1] : pl, nxt = m < M - 1 ? v[m + 1] : nl;
    const uint32_t valid = v[m] != W_EMPTY ? 1u : 0u;
    const uint32_t ws = valid & (prv != v[m] ? 1u : 0u);
    const uint32_t we = valid & (nxt != v[m] ? 1u : 0u);
    c[m] = we | ((ws & we) << 11);
    b[m] = c[m];
    uint32_t kbs = (prv >> F) != (v[m] >> F) ? 1u : 0u, kbe = (nxt >> F) != (v[m] >> F) ? 1u : 0u;
    if constexpr (PM) {
      if (pmode) {  // a k-run is one (key, part)
        const uint32_t pp = m > 0 ? pt[m - 1] : ppl, pn = m < M - 1 ? pt[m + 1] : pnl;
        kbs |= pp != pt[m] ? 1u : 0u;
        kbe |= pn != pt[m] ? 1u : 0u;
      }
    }
    kst |= (valid & kbs) << m;
    kend |= (valid & kbe) << m;
  }
  if constexpr (FO && !MIRROR) {  // one per-file row per w-run end of the rule; a singleton w-run has count 1
    if (fo.hist && (int)(rk >> A) == fo.type) {
#pragma unroll
      for (int m = 0; m < M; ++m)
        if ((c[m] & 1u) && (v[m] >> (A + F)) == fo.q) {  // a symmetric rule's stored row (a, b), a < b, is
          const unsigned long long mult =                // also the row (b, a) of the file's table
              (fo.sym && ((v[m] >> F) & L.amask) != (rk & L.amask)) ? 2ull : 1ull;
          atomicAdd(&fh[v[m] & ((1u << F) - 1u)], mult * ((c[m] >> 11) ? 1ull : (1ull | (1ull << 32))));
        }
    }
  }
  wave_scan_elems<M, false>(b);
  // (2) at each k-run start: its exclusive X << 10 | position, carried to the k-run's end by one
  //     max scan (strictly increasing over the starts)
#pragma unroll
  for (int m = 0; m < M; ++m) {
    const uint32_t e = l * M + m;
    a[m] = ((kst >> m) & 1u) ? (((b[m] - c[m]) << 10) | e) : 0u;
  }
  wave_scan_elems<M, true>(a);
  // (3) at k-run ends: count = its words, S = its files with one word, nf1 = its files;
  //     count_ge2 = count - S, nf2 = nf1 - S. b = count | count_ge2 << 16, c = nf1 | nf2 << 16
#pragma unroll
  for (int m = 0; m < M; ++m) {
    const uint32_t e = l * M + m;
    const uint32_t d = b[m] - (a[m] >> 10);
    const uint32_t nf1 = d & 2047u, s1 = (d >> 11) & 2047u;
    const uint32_t cnt = e + 1 - (a[m] & 1023u);
    b[m] = cnt | ((cnt - s1) << 16);
    c[m] = nf1 | ((nf1 - s1) << 16);
  }
  // (4) one output row per k-run end: (key2, count | count_ge2 << 16) staged in this wave's LDS
  //     rows at its rank among the k-run ends (other elements write a per-lane dummy slot), then
  //     written out linearly into the task's own word range (coalesced stores on a task-uniform base)
  const int type = (int)(rk >> A);
  const int32_t aid = (int32_t)(rk & ((1u << A) - 1u));
  const uint32_t nmine = (uint32_t)__builtin_popcount(kend);
  const uint32_t incl = wave_incl_scan(nmine);
  const uint32_t nout = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
  // the per-rule statistics come from the registers here (only key2 and the counts are staged)
  const int nq = sR.n_of_type[type];
  const int r0 = sR.rule_of_type[type][0], r1 = sR.rule_of_type[type][1];
  // local rules 0 / 1: rows | nf1 << 16, pairs | nf2 << 16 (a symmetric rule's off-diagonal rows twice);
  // sraw: stored rows | stored pairs << 16
  uint32_t s0a = 0, s0b = 0, s1a = 0, s1b = 0, sraw = 0, q2 = 0;
  const uint32_t sym0 = rule_sym(sR, r0) ? 1u : 0u, sym1 = (nq > 1 && rule_sym(sR, r1)) ? 1u : 0u;
  {
    uint32_t idx = incl - nmine;
#pragma unroll
    for (int m = 0; m < M; ++m) {
      const uint32_t ke = (kend >> m) & 1u;
      const uint32_t k2 = v[m] >> F, q = k2 >> A, cnt = b[m] & 0xFFFFu, cc = c[m];
      const uint32_t slot = ke ? idx : (uint32_t)(64 * M) + l;
      uint32_t k2s = k2;
      if constexpr (PM) {
        if (pmode) k2s = k2 | (pt[m] << 24);  // the part rides above aid_next (< 2^24 in part mode)
      }
      stgk[slot] = k2s;
      stgb[slot] = b[m];
      idx += ke;
      if constexpr (!MIRROR) {
        const uint32_t offd = (k2 & L.amask) != (uint32_t)aid ? 1u : 0u;
        const uint32_t mult = 1u + (offd & (q == 0 ? sym0 : (q == 1 ? sym1 : 0u)));
        const uint32_t ra = (1u | ((cc & 0xFFFFu) << 16)) * mult, rb = (cnt | (cc & 0xFFFF0000u)) * mult;
        sraw += ke ? (1u | (cnt << 16)) : 0u;
        s0a += (ke && q == 0) ? ra : 0u; s0b += (ke && q == 0) ? rb : 0u;
        s1a += (ke && q == 1) ? ra : 0u; s1b += (ke && q == 1) ? rb : 0u;
        q2 |= (ke && q >= 2) ? 1u : 0u;
      }
    }
  }
  if (!MIRROR && __ballot(q2 != 0u)) {  // more than 2 rules of one type (not in the reference's five)
#pragma unroll
    for (int m = 0; m < M; ++m) {
      const uint32_t k2 = v[m] >> F, q = k2 >> A;
      if (((kend >> m) & 1u) && q >= 2) {
        const uint32_t cnt = b[m] & 0xFFFFu, cc = c[m];
        const uint32_t mult = (rule_sym(sR, sR.rule_of_type[type][q]) && (k2 & L.amask) != (uint32_t)aid) ? 2u : 1u;
        unsigned long long* acc = sacc + sR.rule_of_type[type][q] * 4;
        atomicAdd(acc + 0, (unsigned long long)mult); atomicAdd(acc + 1, (unsigned long long)cnt * mult);
        atomicAdd(acc + 2, (unsigned long long)(cc & 0xFFFFu) * mult);
        atomicAdd(acc + 3, (unsigned long long)(cc >> 16) * mult);
      }
    }
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  const bool store = O.cap != 0;
  const uint64_t ob = obegin + (MIRROR ? fo.mirror_off : 0ull);
  uint8_t* o_rule = O.rule + ob;
  int32_t* o_aid = O.aid + ob;
  int32_t* o_next = O.aid_next + ob;
  uint32_t* o_cnt = O.count + ob;
  uint32_t* o_c2 = O.count_ge2 + ob;
  if (store)
    for (uint32_t i = l; i < nout; i += 64) {
      const uint32_t k2 = stgk[i], bb = stgb[i];
      const uint32_t q = k2 >> A;
      const int rule = pmode ? (int)(k2 >> 24) : (q == 0 ? r0 : (q == 1 ? r1 : sR.rule_of_type[type][q]));
      const int32_t next = (int32_t)(k2 & L.amask);
      if (MIRROR && next == aid) { o_rule[i] = 0xFF; continue; }  // the diagonal row is its own mirror
      o_rule[i] = (uint8_t)rule;
      o_aid[i] = MIRROR ? next : aid;
      o_next[i] = MIRROR ? aid : next;
      o_cnt[i] = bb & 0xFFFFu;
      o_c2[i] = bb >> 16;
    }
  if (store)  // the rest of the task's word range holds no row (marked here, no table-wide fill)
    for (uint32_t i = nout + l; i < olen; i += 64) o_rule[i] = 0xFF;
  if constexpr (!MIRROR) {
    for (int q = 0; q < (nq < 2 ? nq : 2); ++q) {
      const uint32_t sa = wave_sum(q == 0 ? s0a : s1a), sb = wave_sum(q == 0 ? s0b : s1b);
      if (l == 0 && sa) {
        unsigned long long* acc = sacc + (q == 0 ? r0 : r1) * 4;
        acc[0] += sa & 0xFFFFu; acc[1] += sb & 0xFFFFu; acc[2] += sa >> 16; acc[3] += sb >> 16;
      }
    }
    {
      const uint32_t sr = wave_sum(sraw);
      if (l == 0) { sacc[STAT_RAW] += sr & 0xFFFFu; sacc[STAT_RAW + 1] += sr >> 16; }
    }
  }
  __builtin_amdgcn_wave_barrier();  // the staging rows are rewritten by the next pass / task
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  return nout;
}

// The fold of one sorted task (k_agg_sort, k_agg_lds): v holds its <= 64*M words (W_EMPTY past the
// end), unsorted; rows go to the slots [obegin, obegin + olen) of the table (the task's own word range),
// the rest of that range is marked empty. stgk / stgb: this wave's staging rows (64*M + 64 each),
// sacc: this wave's statistics accumulator, P / fh: the FO kernels' part tables and per-file rows.
// FO: the FileOpts rule's per-file rows (fh); PM: part mode may be on (fo.parts), else compiled out. In part mode
// with fo.mirror_off (MIR), a second pass writes the explicit mirror rows of the symmetric rule's stored rows.
template <int M, bool FO, bool PM = FO, bool MIR = false>
__device__ __forceinline__ void agg_fold(uint32_t (&v)[M], uint64_t obegin, uint32_t olen, uint32_t rk,
                                         const RulesDev& sR, const Layout& L, const OutRows& O, const FileOpts& fo,
                                         const PartLds* P, unsigned long long* fh, uint32_t* stgk, uint32_t* stgb,
                                         unsigned long long* sacc) {
  wave_bitonic_sort<M>(v);
  // neighbours across lanes; lane 0's predecessor and lane 63's successor are sentinels that differ
  // from the element in every field (so no element needs an index test: words are < W_EMPTY, and the
  // invalid tail is W_EMPTY, sorted last). All flags below are branch-free selects: the former
  // short-circuit tests (e < len && (e == 0 || ...)) compiled to exec-mask branches per element.
  const uint32_t l = lane_id();
  const uint32_t pl0 = lane_prev(v[M - 1]), nl0 = lane_next(v[0]);
  const uint32_t pl = l == 0u ? ~v[0] : pl0, nl = l == 63u ? W_EMPTY : nl0;
  // part mode: parts of the elements and of the cross-lane neighbours (words of one key are in file
  // order, and the part is non-decreasing in the file for a fixed key, so a part's words stay adjacent)
  uint32_t pt[PM ? M : 1];
  uint32_t ppl = 0, pnl = 0;
  const bool pmode = PM && fo.parts;
  if constexpr (PM) {
    if (pmode) {
#pragma unroll
      for (int m = 0; m < M; ++m) pt[m] = v[m] != W_EMPTY ? word_part(*P, v[m], rk & L.amask, L) : 0xFFu;
      ppl = lane_prev(pt[M - 1]);
      pnl = lane_next(pt[0]);
    }
  }
  const uint32_t nout =
      fold_pass<M, FO, PM, false>(v, pl, nl, pt, ppl, pnl, pmode, obegin, olen, rk, sR, L, O, fo, fh, stgk, stgb, sacc);
  if constexpr (PM && MIR) {
    if (pmode && fo.mirror_off) {
      // the mirrors' parts differ from the rows' only for words of a cut file between the two keys
      bool differ = false;
#pragma unroll
      for (int m = 0; m < M; ++m) {
        const uint32_t pm = v[m] != W_EMPTY ? word_part_mirror(*P, v[m], rk & L.amask, L) : 0xFFu;
        differ |= pm != pt[m];
        pt[m] = pm;
      }
      ppl = lane_prev(pt[M - 1]);
      pnl = lane_next(pt[0]);
      if (__ballot(differ)) {
        fold_pass<M, FO, PM, true>(v, pl, nl, pt, ppl, pnl, pmode, obegin, olen, rk, sR, L, O, fo, fh, stgk, stgb,
                                   sacc);
      } else {  // the same runs: the staged rows with (aid, aid_next) swapped
        const int32_t aid = (int32_t)(rk & L.amask);
        const uint64_t ob = obegin + fo.mirror_off;
        if (O.cap != 0)
          for (uint32_t i = l; i < olen; i += 64) {
            const uint32_t k2 = i < nout ? stgk[i] : 0u;
            const int32_t next = (int32_t)(k2 & L.amask);
            if (i >= nout || next == aid) { O.rule[ob + i] = 0xFF; continue; }
            O.rule[ob + i] = (uint8_t)(k2 >> 24);
            O.aid[ob + i] = next;
            O.aid_next[ob + i] = aid;
            O.count[ob + i] = stgb[i] & 0xFFFFu;
            O.count_ge2[ob + i] = stgb[i] >> 16;
          }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      }
    }
  }
}

// One wave per task of <= 64*M words (rows and split buckets): bitonic sort in registers, then
// run-length folding with prefix / max scans only (no LDS, no atomics on the data path).
//   w-runs (equal words = one (rule, aid_next, file)): per-file count cf
//   k-runs (equal rule|aid_next): count = sum cf, count_ge2 = sum of cf >= 2,
//                                 nf1 = w-runs, nf2 = w-runs with cf >= 2
// The next task's words are loaded while the current one is folded. Per-rule statistics go
// through a per-wave LDS accumulator (one lane, after wave sums of packed 16-bit fields: a
// task holds <= 1024 words), so no per-thread accumulator arrays take registers.
// FOM: 0 no FileOpts; 1 FileOpts with key cuts / part mode (static per-file table of FO_MAXF rows + the part
// tables in LDS); 3 part mode with the explicit mirror rows (ottohip_table_count_parts); 2 per-file rows only (the histogram of the call's fo.nf files in dynamic LDS, fo.nf * 8 bytes:
// the main build's statistics cost no occupancy)
extern __shared__ unsigned long long agg_sort_fh_dyn[];
// occupancy: 4 waves per SIMD (<= 128 VGPRs) for the 512- and 1024-word classes, except the part-mode 1024-word
// class (2; its mirror pass would spill heavily at 4)
template <int M, int FOM = 0>
__global__ __launch_bounds__(256, (M >= 16 ? (FOM == 1 ? 2 : (FOM == 3 ? 1 : 4)) : (M == 8 && FOM == 2 ? 4 : 1))) void k_agg_sort(const Task* __restrict__ tasks, int64_t n_tasks,
                                                  const uint32_t* __restrict__ w0, const uint32_t* __restrict__ w1,
                                                  const uint32_t* __restrict__ row_key, RulesDev R, Layout L,
                                                  int n_rules, OutRows O, FileOpts fo) {
  constexpr bool FO = FOM != 0;
  __shared__ unsigned long long sacc[4][STAT_STRIDE];
  __shared__ RulesDev sR;
  __shared__ uint32_t stg[4][2][64 * M + 64];  // per wave: output rows of one task (key2, count | count_ge2 << 16),
                                              // + one dummy slot per lane
  constexpr bool PMODE = FOM == 1 || FOM == 3;
  __shared__ unsigned long long fh_s[PMODE ? FO_MAXF : 1];  // per-file rows of the FileOpts rule
  __shared__ std::conditional_t<PMODE, PartLds, char> sP[1];  // part-mode tables (FOM 1 / 3 only)
  unsigned long long* fh = FOM == 2 ? agg_sort_fh_dyn : fh_s;
  const uint32_t l = lane_id();
  const int wv = threadIdx.x >> 6;
  if (threadIdx.x == 0) sR = R;
  for (int i = (int)l; i < STAT_STRIDE; i += 64) sacc[wv][i] = 0;
  if constexpr (FO) {
    for (uint32_t i = threadIdx.x; i < fo.nf; i += blockDim.x) fh[i] = 0;
    if constexpr (PMODE) part_lds_load(fo, sP[0]);
  }
  __syncthreads();
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  int64_t ti = __builtin_amdgcn_readfirstlane((int)(((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6));
  const int A = L.A;
  uint32_t v[M];
  Task T;
  uint32_t rk = 0, nd = 0;
  auto fetch = [&](int64_t t, Task& TT, uint32_t (&vv)[M], uint32_t& rkk, uint32_t& ndd) {
    TT = tasks[t];
    const uint32_t* W = (TT.buf ? w1 : w0) + TT.begin;
#pragma unroll
    for (int m = 0; m < M; ++m) {  // coalesced load (element m*64 + l), then sorted anyway;
      const uint32_t i = (uint32_t)(m * 64) + l;  // clamped index: no branch around the load
      const uint32_t x = W[i < TT.len ? i : TT.len - 1];
      vv[m] = i < TT.len ? x : W_EMPTY;
    }
    rkk = row_key[TT.row];
    ndd = 0;
    if constexpr (PMODE) {  // the cut words become W_EMPTY (sorted past the task's new end)
      if ((fo.cuts || fo.qonly) && (int)(rkk >> A) == fo.type) {
        const int32_t ad = (int32_t)(rkk & L.amask);
        uint32_t k = 0;
#pragma unroll
        for (int m = 0; m < M; ++m) {  // branch-free (a conditional register write here was miscompiled
          const bool dr = fo_drop(fo, vv[m], ad, L);  // in the hash kernel's load loop: see k_agg_hash)
          k += dr ? 1u : 0u;
          vv[m] = dr ? W_EMPTY : vv[m];
        }
        ndd = wave_sum(k);
      }
    }
  };
  if (ti < n_tasks) fetch(ti, T, v, rk, nd);
  while (ti < n_tasks) {
    const int64_t tn = ti + nw;
    Task Tn;
    uint32_t vn[M];
    uint32_t rkn = 0, ndn = 0;
    if (tn < n_tasks) fetch(tn, Tn, vn, rkn, ndn);
    const uint32_t len = T.len - nd;
    if (FO && nd && l == 0) atomicAdd(fo.dropped, (unsigned long long)nd);
    if (FO && fo.dbg && l == 0) { atomicAdd(fo.dbg + 2, (unsigned long long)nd); atomicAdd(fo.dbg + 3, (unsigned long long)len); }
    agg_fold<M, FO, PMODE, FOM == 3>(v, T.begin, T.len, rk, sR, L, O, fo, reinterpret_cast<const PartLds*>(sP), fh,
                              stg[wv][0], stg[wv][1], sacc[wv]);
    T = Tn;
    rk = rkn;
    nd = ndn;
#pragma unroll
    for (int m = 0; m < M; ++m) v[m] = vn[m];
    ti = tn;
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  const uint32_t gwave = blockIdx.x * (blockDim.x >> 6) + wv;
  unsigned long long* stats = O.stats + (size_t)(gwave & (STAT_STRIPES - 1)) * STAT_STRIDE;
  for (int i = (int)l; i < STAT_STRIDE; i += 64)
    if (sacc[wv][i]) atomicAdd(&stats[i], sacc[wv][i]);
  if constexpr (FO) {
    if (fo.hist) {
      __syncthreads();
      for (uint32_t i = threadIdx.x; i < fo.nf; i += blockDim.x)
        if (fh[i]) atomicAdd(&fo.hist[i], fh[i]);
    }
  }
}

// Task lists filled by classification kernels (wave-aggregated pushes)
// Batched insert of N keys per lane (W_EMPTY = none): the N probe reads are issued together so
// their LDS latency overlaps; returns the number of slots this lane created; slot[j] gets the
// slot index (HASH_FULL if the table was full).
template <int N>
__device__ __forceinline__ uint32_t hash_insert_batch(unsigned long long* slots, const uint32_t (&key)[N],
                                                      const uint32_t (&inc)[N], uint32_t cm, uint32_t (&slot)[N]) {
  uint32_t h[N];
  bool pend[N];
  uint32_t probes[N];
  uint32_t created = 0;
#pragma unroll
  for (int j = 0; j < N; ++j) {
    pend[j] = key[j] != W_EMPTY;
    h[j] = hslot(key[j], cm);
    probes[j] = 0;
    slot[j] = HASH_FULL;
  }
  while (true) {
    bool any = false;
#pragma unroll
    for (int j = 0; j < N; ++j) any |= pend[j];
    if (!any) break;
    unsigned long long v[N];
#pragma unroll
    for (int j = 0; j < N; ++j) v[j] = pend[j] ? lds_load(&slots[h[j]]) : 0ull;
#pragma unroll
    for (int j = 0; j < N; ++j) {
      if (!pend[j]) continue;
      const uint32_t k = (uint32_t)(v[j] >> 32);
      if (k == key[j]) {
        atomicAdd(&slots[h[j]], (unsigned long long)inc[j]);
        slot[j] = h[j];
        pend[j] = false;
      } else if (k == W_EMPTY) {
        const unsigned long long nv = ((unsigned long long)key[j] << 32) | inc[j];
        if (atomicCAS(&slots[h[j]], v[j], nv) == v[j]) { slot[j] = h[j]; pend[j] = false; ++created; }
        // else: retry the same slot with a fresh read
      } else {
        h[j] = (h[j] + 1) & cm;
        if (++probes[j] > cm) pend[j] = false;  // full: slot stays HASH_FULL
      }
    }
  }
  return created;
}

constexpr int N_SORT = 5;  // register-sort classes: 64, 128, 256, 512, 1024 words
constexpr int SORT_MAX = 64 << (N_SORT - 1);
constexpr int LDS_CAP = 4096;  // largest task of the LDS leaf (k_agg_lds)
struct TaskLists {
  Task* sort[N_SORT];     // register sort by size class
  Task* hash;             // workgroup LDS hash (heavy buckets)
  Task* split;            // MSD split
  Task* lds;              // LDS leaf (k_agg_lds)
  unsigned long long* n;  // [N_SORT + 3]: sort classes..., hash, split, lds
  uint64_t cap;           // capacity of every list
};

// FOM as k_agg_sort: 0 no FileOpts, 1 cuts / part mode, 3 part mode with the mirror pass, 2 per-file rows only
template <int FOM = 0>
__global__ __launch_bounds__(AGG_T, 2) void k_agg_hash(const Task* __restrict__ tasks, int64_t n_tasks,
                                                    const uint32_t* __restrict__ w0, const uint32_t* __restrict__ w1,
                                                    const uint32_t* __restrict__ row_key, RulesDev R, Layout L,
                                                    int n_rules, OutRows O, Task* __restrict__ overflow,
                                                    unsigned long long* __restrict__ n_overflow, FileOpts fo) {
  __shared__ unsigned long long lds[2 * HCAP];  // 64 KiB: phase A [0, cap), phase B [0, 2cap)
  __shared__ uint32_t wtot[AGG_T / 64];
  __shared__ uint32_t nocc;
  constexpr bool FO = FOM != 0, PM = FOM == 1 || FOM == 3;
  __shared__ unsigned long long fh[FO ? FO_MAXF : 1];  // per-file rows of the FileOpts rule
  __shared__ std::conditional_t<PM, PartLds, char> sP[1];  // part-mode tables (FOM 1 only)
  const int tid = threadIdx.x;
  // the hash leaves share CUs with the register sorts of the same level (aux stream): a raised wave
  // priority lets their LDS-latency-bound loop issue ahead of the VALU-bound sorts
  if (c_hash_prio == 1) __builtin_amdgcn_s_setprio(1);
  else if (c_hash_prio >= 2) __builtin_amdgcn_s_setprio(3);
  RuleAcc acc;
  acc.zero();
  if constexpr (FO) {
    for (uint32_t i = tid; i < fo.nf; i += AGG_T) fh[i] = 0;
    if constexpr (PM) part_lds_load(fo, sP[0]);
    __syncthreads();
  }
  const bool pmode = PM && fo.parts;
  for (int64_t ti = blockIdx.x; ti < n_tasks; ti += gridDim.x) {
    const Task T = tasks[ti];
    const uint64_t t_start = fo.prof ? wall_clock64() : 0;
    const uint32_t* W = (T.buf ? w1 : w0) + T.begin;
    const RowInfo ri = row_info(row_key, T.row, L.A);
    const bool fo_row = FO && ri.type == fo.type;
    const bool fo_cut = fo_row && (fo.cuts || fo.qonly);
    uint32_t ndrop = 0, dbg_loaded = 0, dbg_ins = 0;
    const uint32_t dbound = T.len;
    // optimistic: more keys possible than fit; give up at 3/4 fill and send the task to a split
    const bool optimistic = 2 * dbound > (uint32_t)HCAP;
    uint32_t cap = 64;
    while (cap < 2 * dbound && cap < (uint32_t)HCAP) cap <<= 1;
    const uint32_t cm = cap - 1, limit = (uint32_t)HCAP / 4;  // + 256 threads x 8 keys stays < HCAP
    unsigned long long* A = lds;
    for (uint32_t i = tid; i < cap; i += AGG_T) A[i] = SLOT_EMPTY;
    if (tid == 0) nocc = 0;
    __syncthreads();
    bool full = false;
    constexpr int PF = 8;  // words per thread loaded ahead of their inserts
    uint32_t wbuf[PF], nbuf[PF];
    const uint32_t l64 = (uint32_t)tid & 63u;
#pragma unroll
    for (int j = 0; j < PF; ++j) {
      const uint32_t i = j * AGG_T + tid;
      nbuf[j] = i < T.len ? W[i] : W_EMPTY;
    }
    for (uint32_t i0 = 0; i0 < T.len && !full; i0 += AGG_T * PF) {
      // the next batch's loads are in flight while this batch is inserted
#pragma unroll
      for (int j = 0; j < PF; ++j) {
        wbuf[j] = nbuf[j];
        const uint32_t i = i0 + (uint32_t)(AGG_T * PF) + j * AGG_T + tid;
        nbuf[j] = i < T.len ? W[i] : W_EMPTY;
      }
#pragma unroll
      for (int j = 0; j < PF; ++j) {
        if (FO && fo.dbg && wbuf[j] != W_EMPTY) ++dbg_loaded;
        if constexpr (PM) {  // branch-free: the cut word becomes W_EMPTY (the if-form lost ~15% of the
                             // W_EMPTY writes under hipcc 7.2 -O3: counted and cut at once, found by the
                             // reduce's conservation check, tests/test_covis_gpu.py::test_file_cuts_hot_rows)
          const bool dr = fo_cut && fo_drop(fo, wbuf[j], ri.aid, L);
          ndrop += dr ? 1u : 0u;
          wbuf[j] = dr ? W_EMPTY : wbuf[j];
        }
      }
      // each thread adds at most PF keys after this check: 256 * 8 < HCAP / 4 keeps the table from filling
      if (optimistic && __hip_atomic_load(&nocc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) > limit) {
        full = true;
        break;
      }
      uint32_t inc[PF], slot[PF];
#pragma unroll
      for (int j = 0; j < PF; ++j) {
        // runs of equal words over the wave's 64 consecutive words (hot keys arrive in long runs:
        // words keep their event order through the splits) become one insert of the run length.
        // Branch-free: a lane that is not a run head carries W_EMPTY.
        const uint32_t w = wbuf[j];
        const bool head = l64 == 0u || lane_prev(w) != w;
        const uint64_t hm = __ballot(head);
        const uint64_t after = l64 == 63u ? 0ull : hm & (~0ull << (l64 + 1u));
        const uint32_t end = after ? (uint32_t)__builtin_ctzll(after) : 64u;
        inc[j] = end - l64;
        wbuf[j] = head ? w : W_EMPTY;
      }
      const uint32_t created = hash_insert_batch<PF>(A, wbuf, inc, cm, slot);
      if (FO && fo.dbg) {
#pragma unroll
        for (int j = 0; j < PF; ++j) dbg_ins += (wbuf[j] != W_EMPTY && slot[j] != HASH_FULL) ? inc[j] : 0u;
      }
#pragma unroll
      for (int j = 0; j < PF; ++j) full |= wbuf[j] != W_EMPTY && slot[j] == HASH_FULL;
      if (optimistic) {
        const uint32_t nc = wave_sum(created);
        if (nc && (tid & 63) == 0) atomicAdd(&nocc, nc);
      }
    }
    full = __syncthreads_or(full);
    if (full) {
      if (tid == 0) {
        const unsigned long long k = atomicAdd(n_overflow, 1ull);
        overflow[k] = T;  // capacity = number of hash tasks
        if (fo.prof) {
          fo.prof[2 * ti] = T.len;
          fo.prof[2 * ti + 1] = (wall_clock64() - t_start) | (1ull << 63);
        }
      }
      __syncthreads();
      continue;
    }
    constexpr int SL = HCAP / AGG_T;  // 16 slots per thread at most
    uint32_t kw[SL], kc[SL];
#pragma unroll
    for (int s = 0; s < SL; ++s) {
      const uint32_t slot = tid + s * AGG_T;
      const unsigned long long v = slot < cap ? A[slot] : SLOT_EMPTY;
      kw[s] = (uint32_t)(v >> 32);
      kc[s] = (uint32_t)v;
    }
    if constexpr (FO) {  // the task completed: its drops count, and every slot is one per-file row
      const uint32_t nd = wave_sum(ndrop);
      if (nd && (tid & 63) == 0) atomicAdd(fo.dropped, (unsigned long long)nd);
      if (fo.dbg) {
        uint32_t kept = 0;
#pragma unroll
        for (int s = 0; s < SL; ++s) kept += kw[s] != W_EMPTY ? kc[s] : 0u;
        kept = wave_sum(kept);
        const uint32_t ld = wave_sum(dbg_loaded), ins = wave_sum(dbg_ins);
        if ((tid & 63) == 0) {
          atomicAdd(fo.dbg + 0, (unsigned long long)nd); atomicAdd(fo.dbg + 1, (unsigned long long)kept);
          atomicAdd(fo.dbg + 4, (unsigned long long)ld); atomicAdd(fo.dbg + 5, (unsigned long long)ins);
        }
      }
      if (fo.hist && fo_row) {
#pragma unroll
        for (int s = 0; s < SL; ++s)
          if (kw[s] != W_EMPTY && (kw[s] >> (L.A + L.F)) == fo.q) {
            const unsigned long long mult = (fo.sym && ((kw[s] >> L.F) & L.amask) != (uint32_t)ri.aid) ? 2ull : 1ull;
            atomicAdd(&fh[kw[s] & ((1u << L.F) - 1u)], mult * (kc[s] >= 2 ? (1ull | (1ull << 32)) : 1ull));
          }
      }
    }
    __syncthreads();
    // pass 0: the rows; pass 1 (part mode with mirror rows): the explicit mirrors (part_m, aid_next, aid) of a
    // symmetric rule's stored rows at mirror_off + slot, no statistics (block-uniform)
    const int npass = (FOM == 3 && pmode && fo.mirror_off) ? 2 : 1;
    uint32_t nout = 0;
#pragma unroll 1
    for (int pass = 0; pass < npass; ++pass) {
    unsigned long long* B = lds;            // key2 << 32 | count
    unsigned long long* B2 = lds + cap;     // count_ge2 << 32 | nf2 << 16 | nf1
    for (uint32_t i = tid; i < cap; i += AGG_T) { B[i] = SLOT_EMPTY; B2[i] = 0; }
    __syncthreads();
#pragma unroll
    for (int s0 = 0; s0 < SL; s0 += 8) {  // <= distinct words: always fits
      if ((uint32_t)(s0 * AGG_T) >= cap) break;
      uint32_t k2[8], c8[8], slot[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        k2[j] = kw[s0 + j] == W_EMPTY ? W_EMPTY : kw[s0 + j] >> L.F;
        if constexpr (PM) {  // part mode: the folded key is (part, aid_next) (pass 1: the mirror's part)
          if (pmode && kw[s0 + j] != W_EMPTY) {
            const uint32_t w = kw[s0 + j], f = w & ((1u << L.F) - 1u), ci = sP[0].cut_of[f];
            const uint64_t ka = (uint64_t)(uint32_t)ri.aid, kb = (uint64_t)((w >> L.F) & L.amask);
            const uint64_t key = pass ? ((kb << 32) | ka) : ((ka << 32) | kb);
            k2[j] |= ((uint32_t)sP[0].part_of[f] +
                      ((ci != FO_NOCUT && key >= sP[0].cut_key[ci & (FO_MAXCUT - 1)]) ? 1u : 0u)) << 24;
          }
        }
        c8[j] = kc[s0 + j];
      }
      hash_insert_batch<8>(B, k2, c8, cm, slot);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (slot[j] == HASH_FULL) continue;
        const uint32_t c = c8[j];
        atomicAdd(&B2[slot[j]], ((unsigned long long)(c >= 2 ? c : 0u) << 32) | 1ull | ((c >= 2 ? 1ull : 0ull) << 16));
      }
    }
    __syncthreads();
    // compact into the task's own word range (outputs <= words); the mirror pass skips the diagonal
    uint32_t mine = 0;
    for (uint32_t i = tid; i < cap; i += AGG_T) {
      const uint32_t k2 = (uint32_t)(B[i] >> 32);
      mine += k2 != W_EMPTY && !(pass && (int32_t)(k2 & L.amask) == ri.aid);
    }
    const uint32_t incl = wave_incl_scan(mine);
    if ((tid & 63) == 63) wtot[tid >> 6] = incl;
    __syncthreads();
    uint32_t pre = 0;
    for (int k = 0; k < (tid >> 6); ++k) pre += wtot[k];
    const uint64_t base = T.begin + (pass ? fo.mirror_off : 0ull);
    uint64_t p = base + pre + incl - mine;
    for (uint32_t i = tid; i < cap; i += AGG_T) {
      const unsigned long long v = B[i];
      const uint32_t k2 = (uint32_t)(v >> 32);
      if (k2 == W_EMPTY) continue;
      const unsigned long long v2 = B2[i];
      const int rule = pmode ? 0 : R.rule_of_type[ri.type][k2 >> L.A];
      const uint32_t c = (uint32_t)v, c2 = (uint32_t)(v2 >> 32), nf = (uint32_t)v2;
      const int32_t next = (int32_t)(k2 & L.amask);
      if (pass) {
        if (next != ri.aid) put_row(O, p++, (int)(k2 >> 24), next, ri.aid, c, c2);
        continue;
      }
      const bool mr = rule_sym(R, rule) && next != ri.aid;
      put_row(O, p++, pmode ? (int)(k2 >> 24) : rule, ri.aid, next, c, c2);  // part mode: the part as "rule"
      acc.add(rule, c, nf, mr ? 2u : 1u);
    }
    // the rest of the task's word range holds no row (no table-wide fill: every word position
    // belongs to exactly one leaf task, sort or hash)
    const uint32_t no = wtot[0] + wtot[1] + wtot[2] + wtot[3];
    for (uint32_t i = no + tid; i < T.len; i += AGG_T) O.rule[base + i] = 0xFF;
    if (pass == 0) nout = no;
    __syncthreads();
    }
    if (fo.prof && tid == 0) {
      fo.prof[2 * ti] = T.len | ((unsigned long long)nout << 32);
      fo.prof[2 * ti + 1] = wall_clock64() - t_start;
    }
  }
  acc.flush(O.stats, n_rules);
  if constexpr (FO) {
    if (fo.hist) {
      __syncthreads();
      for (uint32_t i = tid; i < fo.nf; i += AGG_T)
        if (fh[i]) atomicAdd(&fo.hist[i], fh[i]);
    }
  }
}

// ---- classification of rows and split buckets into task lists

// class of a task: [0, N_SORT) register sort of <= 64 << c words; N_SORT workgroup hash
// (a split bucket that stayed far above its expected size: skewed towards a few hot keys,
// hashed optimistically and sent back to a split on overflow); N_SORT + 1 split (rows, and
// buckets that are large only because the parent needed more than one split's digits);
// N_SORT + 2 the LDS leaf (rows and ordinary buckets of up to LDS_CAP words, when c_lds_leaf).
constexpr int SPLIT_LEVELS = 4;
__device__ __forceinline__ int task_class(uint64_t len, uint32_t level, bool split) {
  for (int c = 0; c < N_SORT; ++c)
    if (len <= (uint64_t)(64 << c)) return c;
  // (the LDS leaf only below SPLIT_LEVELS: its hot-key overflow re-enters the split list, see k_agg_lds)
  if (split && c_lds_leaf && len <= (uint64_t)LDS_CAP && level < (uint32_t)SPLIT_LEVELS) return N_SORT + 2;
  return (split && level < (uint32_t)SPLIT_LEVELS) ? N_SORT + 1 : N_SORT;
}
// Block-aggregated push: every thread of the (256-thread) block must call it once. Per list:
// LDS counter per block, then one device atomic per list per block.
constexpr int N_LISTS = N_SORT + 3;
__device__ __forceinline__ void push_task_block(const TaskLists& TL, bool valid, uint64_t begin, uint64_t len,
                                                uint32_t row, uint32_t rem, uint32_t buf, bool split, int* err) {
  __shared__ uint32_t bcnt[N_LISTS];
  __shared__ unsigned long long bbase[N_LISTS];
  if (valid && len > 0xFFFFFFFFull) { atomicOr(err, 2); valid = false; }
  const int c = valid ? task_class(len, rem, split) : -1;
  if (threadIdx.x < N_LISTS) bcnt[threadIdx.x] = 0;
  __syncthreads();
  uint32_t my = 0;
#pragma unroll
  for (int q = 0; q < N_LISTS; ++q) {
    const uint64_t m = __ballot(c == q);
    if (!m) continue;
    uint32_t wb = 0;
    if (mbcnt(m) == 0 && c == q) wb = atomicAdd(&bcnt[q], (uint32_t)__popcll(m));
    wb = __shfl(wb, __ffsll((long long)m) - 1);
    if (c == q) my = wb + mbcnt(m);
  }
  __syncthreads();
  if (threadIdx.x < N_LISTS && bcnt[threadIdx.x])
    bbase[threadIdx.x] = atomicAdd(&TL.n[threadIdx.x], (unsigned long long)bcnt[threadIdx.x]);
  __syncthreads();
  if (c >= 0) {
    const unsigned long long k = bbase[c] + my;
    Task t; t.begin = begin; t.len = (uint32_t)len; t.row = row; t.rem = rem; t.buf = buf;
    Task* list = c < N_SORT ? TL.sort[c] : (c == N_SORT ? TL.hash : (c == N_SORT + 1 ? TL.split : TL.lds));
    if (k < TL.cap) list[k] = t; else atomicOr(err, 4);
  }
}

__global__ void k_classify_rows(const uint64_t* __restrict__ row_begin, int64_t R, uint64_t P, int WB,
                                TaskLists TL, int* err, uint64_t row_base) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool valid = r < R;
  uint64_t b = 0, e = 0;
  if (valid) { b = row_begin[r] - row_base; e = r + 1 < R ? row_begin[r + 1] - row_base : P; }
  push_task_block(TL, valid && e > b, b, e - b, (uint32_t)r, 0u, 0u, true, err);
}

// split: per task k digit bits, chunks of SPLIT_CH words
constexpr int SPLIT_CH = 16384;
// the split's halves: the first task t with chunk_base[t] >= nchunks / 2 (a task boundary near the middle) ->
// out[0] = t, out[1] = chunk_base[t], out[2] = digit_base[t]
__global__ void k_split_half(const uint64_t* __restrict__ chunk_base, const uint64_t* __restrict__ digit_base, int64_t n,
                             const uint64_t* __restrict__ nchunks_total, uint64_t* __restrict__ out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const uint64_t half = *nchunks_total / 2;
  int64_t lo = 0, hi = n;  // first t with chunk_base[t] >= half
  while (lo < hi) {
    const int64_t m = (lo + hi) >> 1;
    if (chunk_base[m] < half) lo = m + 1; else hi = m;
  }
  out[0] = (uint64_t)lo;
  out[1] = lo < n ? chunk_base[lo] : *nchunks_total;
  out[2] = lo < n ? digit_base[lo] : 0ull;
}
constexpr int SPLIT_T = 256;

// Digits of one split: ceil(len / SPLIT_MEAN), 2..SPLIT_DMAX (any count, not only powers of two), so
// hashed buckets average <= SPLIT_MEAN words and almost all fit the 512-word register sort.
constexpr int SPLIT_DMAX = 512;  // digits per split level (512 vs 256: reduce -1 ms same-box; 1024 was slower)
__device__ __forceinline__ uint32_t split_ndig(const Task& t) {
  const uint64_t d = ((uint64_t)t.len + c_split_mean - 1) / c_split_mean;
  return d < 2 ? 2u : (d > (uint64_t)SPLIT_DMAX ? (uint32_t)SPLIT_DMAX : (uint32_t)d);
}
// Split digit: a hash of the word's (rule, aid_next) part, seeded by the split level, scaled to
// nd digits. Every word of one output row (all its files) lands in the same bucket, buckets are
// balanced whatever the aid_next distribution, and a bucket split again at the next level
// spreads over fresh digits. Row order inside the table is not part of the contract.
__device__ __forceinline__ uint32_t split_digit(uint32_t w, int F, uint32_t level, uint32_t nd) {
  uint32_t x = (w >> F) ^ (level * 0x9E3779B9u);
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return (uint32_t)(((uint64_t)x * nd) >> 32);
}
// Split of one level, no global atomics: per task, chunks of SPLIT_CH words and 2^k digits; a
// (digit-major, chunk-minor) matrix of per-chunk digit counts is scanned once, which gives every
// chunk its exact output offset per digit and every sub-bucket its range.
__global__ void k_split_prepare(const Task* __restrict__ tasks, int64_t n, uint32_t* __restrict__ nchunks,
                                uint32_t* __restrict__ ndigits, uint32_t* __restrict__ nent) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t nch = (uint32_t)ceil_div((int64_t)tasks[i].len, SPLIT_CH), nd = split_ndig(tasks[i]);
  nchunks[i] = nch;
  ndigits[i] = nd;
  nent[i] = nch * nd;
}

__device__ __forceinline__ int64_t find_task(const uint64_t* chunk_base, int64_t n, uint64_t c) {
  int64_t lo = 0, hi = n;  // largest t with chunk_base[t] <= c
  while (hi - lo > 1) {
    const int64_t m = (lo + hi) >> 1;
    if (chunk_base[m] <= c) lo = m; else hi = m;
  }
  return lo;
}

// chunk -> task map of one split level: every hist / scatter block reads its task with one load
// instead of a binary search over the chunk bases (~20 dependent loads at 5e5 tasks)
__global__ void k_split_chunk_task(const uint64_t* __restrict__ chunk_base, const uint32_t* __restrict__ nchunks,
                                   int64_t n, uint32_t* __restrict__ chunk_task) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const uint64_t b = chunk_base[t];
  for (uint32_t c = 0; c < nchunks[t]; ++c) chunk_task[b + c] = (uint32_t)t;
}

__global__ __launch_bounds__(SPLIT_T) void k_split_hist(const Task* __restrict__ tasks, int64_t n,
                                                        const uint64_t* __restrict__ chunk_base,
                                                        const uint32_t* __restrict__ chunk_task,
                                                        const uint64_t* __restrict__ mat_base,
                                                        const uint32_t* __restrict__ w0, const uint32_t* __restrict__ w1,
                                                        int F, uint32_t* __restrict__ hmat) {
  __shared__ uint32_t h[SPLIT_DMAX];
  const int64_t t = chunk_task[blockIdx.x];
  const Task T = tasks[t];
  const uint32_t nd = split_ndig(T), nch = (uint32_t)ceil_div((int64_t)T.len, SPLIT_CH);
  const uint32_t c = (uint32_t)(blockIdx.x - chunk_base[t]);
  if (nch == 1 && c_split_fuse) {  // one-chunk task: k_split_scatter counts it itself (zeros keep the scan exact)
    for (uint32_t d = threadIdx.x; d < nd; d += SPLIT_T) hmat[mat_base[t] + d] = 0u;
    return;
  }
  const uint64_t c0 = (uint64_t)c * SPLIT_CH;
  const uint64_t c1 = c0 + SPLIT_CH < T.len ? c0 + SPLIT_CH : T.len;
  const uint32_t* W = (T.buf ? w1 : w0) + T.begin;
  for (uint32_t i = threadIdx.x; i < nd; i += SPLIT_T) h[i] = 0;
  __syncthreads();
  for (uint64_t i0 = c0; i0 < c1; i0 += 8 * SPLIT_T) {  // 8 loads in flight per thread
    uint32_t wr[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint64_t i = i0 + threadIdx.x + j * SPLIT_T;
      wr[j] = i < c1 ? W[i] : 0u;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (c_split_runs) lds_add_runs(h, split_digit(wr[j], F, T.rem, nd), i0 + threadIdx.x + j * SPLIT_T < c1);
      else if (i0 + threadIdx.x + j * SPLIT_T < c1) atomicAdd(&h[split_digit(wr[j], F, T.rem, nd)], 1u);
  }
  __syncthreads();
  for (uint32_t d = threadIdx.x; d < nd; d += SPLIT_T) hmat[mat_base[t] + (uint64_t)d * nch + c] = h[d];
}

// SUB: scatter sub-tile (staged in LDS in digit order); SUB / SPLIT_T words per thread in registers
template <int SUB>
__global__ __launch_bounds__(SPLIT_T) void k_split_scatter(const Task* __restrict__ tasks, int64_t n,
                                                           const uint64_t* __restrict__ chunk_base,
                                                           const uint32_t* __restrict__ chunk_task,
                                                           const uint64_t* __restrict__ mat_base,
                                                           const uint64_t* __restrict__ hoff,
                                                           uint32_t* __restrict__ w0, uint32_t* __restrict__ w1, int F,
                                                           uint32_t* __restrict__ hmat, uint32_t chunk0 = 0) {
  // chunk0: the first chunk of this launch (a split may run as two launches over chunk ranges)
  constexpr int DPT = SPLIT_DMAX / SPLIT_T;  // digits per thread in the scans
  __shared__ uint32_t h[SPLIT_DMAX], st[SPLIT_DMAX];
  __shared__ uint64_t gb[SPLIT_DMAX];
  __shared__ uint32_t stage[SUB];
  __shared__ uint32_t wsum[SPLIT_T / 64];
  const uint32_t cid = chunk0 + blockIdx.x;
  const int64_t t = chunk_task[cid];
  const Task T = tasks[t];
  const uint32_t nd = split_ndig(T), nch = (uint32_t)ceil_div((int64_t)T.len, SPLIT_CH);
  const uint32_t c = (uint32_t)(cid - chunk_base[t]);
  const uint64_t c0 = (uint64_t)c * SPLIT_CH;
  const uint64_t c1 = c0 + SPLIT_CH < T.len ? c0 + SPLIT_CH : T.len;
  const uint32_t* Win = (T.buf ? w1 : w0) + T.begin;
  uint32_t* Wout = T.buf ? w0 : w1;
  constexpr int SUB_PER_T = SUB / SPLIT_T;
  const int tid = threadIdx.x;
  const uint64_t mb = mat_base[t];
  if (nch == 1 && c_split_fuse) {
    // one-chunk task (<= SPLIT_CH words): its digit counts come from this block (the words are read
    // twice here, the second time from the caches, instead of once by k_split_hist and once here from
    // HBM); they go to hmat for k_split_classify, and the bucket starts are a scan of them
    for (uint32_t d = tid; d < nd; d += SPLIT_T) h[d] = 0;
    __syncthreads();
    for (uint64_t i0 = c0; i0 < c1; i0 += 8 * SPLIT_T) {
      uint32_t wr[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint64_t i = i0 + tid + j * SPLIT_T;
        wr[j] = i < c1 ? Win[i] : 0u;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (c_split_runs) lds_add_runs(h, split_digit(wr[j], F, T.rem, nd), i0 + tid + j * SPLIT_T < c1);
        else if (i0 + tid + j * SPLIT_T < c1) atomicAdd(&h[split_digit(wr[j], F, T.rem, nd)], 1u);
    }
    __syncthreads();
    uint32_t v[DPT], tsum = 0;
#pragma unroll
    for (int q = 0; q < DPT; ++q) {
      const uint32_t d = (uint32_t)(tid * DPT + q);
      v[q] = d < nd ? h[d] : 0u;
      tsum += v[q];
    }
    const uint32_t incl = wave_incl_scan(tsum);
    if ((tid & 63) == 63) wsum[tid >> 6] = incl;
    __syncthreads();
    uint32_t pre = 0;
    for (int q = 0; q < (tid >> 6); ++q) pre += wsum[q];
    uint32_t run = pre + incl - tsum;
#pragma unroll
    for (int q = 0; q < DPT; ++q) {
      const uint32_t d = (uint32_t)(tid * DPT + q);
      if (d < nd) { gb[d] = T.begin + run; hmat[mb + d] = v[q]; }
      run += v[q];
    }
    __syncthreads();  // h / wsum are reused by the sub-tile loop
  } else {
    for (uint32_t d = tid; d < nd; d += SPLIT_T) gb[d] = T.begin + (hoff[mb + (uint64_t)d * nch + c] - hoff[mb]);
  }
  for (uint64_t s0 = c0; s0 < c1; s0 += SUB) {
    const int m = (int)((c1 - s0) < (uint64_t)SUB ? (c1 - s0) : (uint64_t)SUB);
    uint32_t wr[SUB_PER_T], dg[SUB_PER_T];
#pragma unroll
    for (int j = 0; j < SUB_PER_T; ++j) {  // the sub-tile is read once, into registers
      const int i = tid + j * SPLIT_T;
      wr[j] = i < m ? Win[s0 + i] : 0u;
    }
    for (uint32_t d = tid; d < nd; d += SPLIT_T) h[d] = 0;
    __syncthreads();
    // the histogram atomic returns the word's rank among this sub-tile's words of its digit: the
    // staging slot (order inside a bucket is free), no second counter pass
    uint32_t rk[SUB_PER_T];
#pragma unroll
    for (int j = 0; j < SUB_PER_T; ++j) {
      dg[j] = split_digit(wr[j], F, T.rem, nd);
      if (c_split_runs) rk[j] = lds_add_runs(h, dg[j], tid + j * SPLIT_T < m);
      else rk[j] = tid + j * SPLIT_T < m ? atomicAdd(&h[dg[j]], 1u) : 0u;
    }
    __syncthreads();
    {  // exclusive scan of h over the digits -> st (thread t: digits DPT t .. DPT t + DPT - 1)
      uint32_t v[DPT], tsum = 0;
#pragma unroll
      for (int q = 0; q < DPT; ++q) {
        const uint32_t d = (uint32_t)(tid * DPT + q);
        v[q] = d < nd ? h[d] : 0u;
        tsum += v[q];
      }
      const uint32_t incl = wave_incl_scan(tsum);
      if ((tid & 63) == 63) wsum[tid >> 6] = incl;
      __syncthreads();
      uint32_t pre = 0;
      for (int q = 0; q < (tid >> 6); ++q) pre += wsum[q];
      uint32_t run = pre + incl - tsum;
#pragma unroll
      for (int q = 0; q < DPT; ++q) {
        st[tid * DPT + q] = run;
        run += v[q];
      }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < SUB_PER_T; ++j)
      if (tid + j * SPLIT_T < m) stage[st[dg[j]] + rk[j]] = wr[j];
    __syncthreads();
    for (int p = tid; p < m; p += SPLIT_T) {
      const uint32_t w = stage[p];
      const uint32_t d = split_digit(w, F, T.rem, nd);
      Wout[gb[d] + (p - st[d])] = w;
    }
    __syncthreads();
    for (uint32_t d = tid; d < nd; d += SPLIT_T) gb[d] += h[d];  // this chunk's cursor per digit moves past the sub-tile
  }
}

// one thread per (split task, digit): push the non-empty sub-buckets as next-level tasks
__global__ void k_split_classify(const Task* __restrict__ tasks, int64_t n, const uint64_t* __restrict__ digit_base,
                                 const uint64_t* __restrict__ mat_base, const uint64_t* __restrict__ hoff,
                                 int64_t n_digits_total, TaskLists TL, int* err, const uint32_t* __restrict__ hmat,
                                 int64_t d0 = 0) {
  // digits [d0, n_digits_total) (a split may classify its digits in two launches)
  const int64_t i = d0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  Task T;
  T.begin = 0; T.rem = 0; T.row = 0; T.buf = 0; T.len = 0;
  uint64_t b = 0, c = 0;
  if (i < n_digits_total) {
    const int64_t t = find_task(digit_base, n, (uint64_t)i);
    T = tasks[t];
    const uint64_t d = (uint64_t)i - digit_base[t], nch = (uint64_t)ceil_div((int64_t)T.len, SPLIT_CH);
    const uint64_t mb = mat_base[t];
    if (nch == 1 && c_split_fuse) {  // counted by k_split_scatter: hoff holds zeros for this task
      uint64_t lo = 0;
      for (uint64_t e = 0; e < d; ++e) lo += hmat[mb + e];
      c = hmat[mb + d];
      b = T.begin + lo;
    } else {
      const uint64_t lo = hoff[mb + d * nch], hi = hoff[mb + (d + 1) * nch];
      c = hi - lo;
      b = T.begin + (lo - hoff[mb]);
    }
  }
  // a bucket within 4x of its expected size is split again (its parent was too large for one
  // split's 8 bits); one far above it holds a few hot keys and goes to the hash path
  const bool again = c != 0 && (uint64_t)c <= 4 * ((uint64_t)T.len / split_ndig(T) + 1);
  push_task_block(TL, c != 0, b, c, T.row, T.rem + 1u, T.buf ^ 1u, again, err);
}

// ---- LDS leaf: one workgroup per task of (SORT_MAX, LDS_CAP] words (rows, and split buckets of an ordinary
// size). The task is read from HBM once and partitioned in LDS by a second hash of (rule, aid_next) into
// sub-buckets of ~LDS_SUBW words (one LDS atomic per word gives its rank); the sub-buckets starting in one
// LDS_SEG-word window form a segment (a sub-bucket above LDS_BIG words is a segment of its own), so a
// segment holds whole keys and <= 512 words, and each wave sorts and folds segments straight from LDS
// (agg_fold<4 | 8>). A segment above 512 words (hot keys) is written back to its place in the word buffer
// and pushed to this level's split list. Against a split of the bucket in HBM followed by register sorts
// of the sub-buckets, the words are read once instead of three times and written not at all, and the split
// that feeds these tasks needs ~6x fewer digits (longer scatter runs).
constexpr int LDS_T = 256;
constexpr int LDS_WPT = LDS_CAP / LDS_T;           // words per thread
constexpr int LDS_SUBW = 32;                       // mean words per sub-bucket
constexpr int LDS_NSUB = LDS_CAP / LDS_SUBW;       // <= 128 sub-buckets
constexpr int LDS_SEG = 384;
constexpr int LDS_BIG = 128;
static_assert(LDS_SEG + LDS_BIG <= 512, "a grouped segment fits the 512-word fold");
static_assert(LDS_NSUB <= 128, "sub-bucket scan over waves 0 and 1");
template <bool FO = false>
__global__ __launch_bounds__(LDS_T) void k_agg_lds(const Task* __restrict__ tasks, int64_t n_tasks,
                                                   uint32_t* __restrict__ w0, uint32_t* __restrict__ w1,
                                                   const uint32_t* __restrict__ row_key, RulesDev R, Layout L,
                                                   OutRows O, Task* __restrict__ overflow,
                                                   unsigned long long* __restrict__ n_overflow, uint64_t ov_cap,
                                                   int* __restrict__ err, FileOpts fo) {
  __shared__ uint32_t words[LDS_CAP];
  __shared__ uint32_t sh[LDS_NSUB], ss[LDS_NSUB + 1], seg[LDS_NSUB + 1];
  __shared__ uint32_t wtot[LDS_T / 64], nseg;
  __shared__ unsigned long long sacc[LDS_T / 64][STAT_STRIDE];
  __shared__ RulesDev sR;
  __shared__ uint32_t stg[LDS_T / 64][2][64 * 8 + 64];  // per wave: staged output rows (agg_fold)
  __shared__ unsigned long long fh[FO ? FO_MAXF : 1];
  __shared__ std::conditional_t<FO, PartLds, char> sP[1];
  const int tid = threadIdx.x, wv = tid >> 6;
  const uint32_t l = lane_id();
  if (tid == 0) sR = R;
  for (int i = (int)l; i < STAT_STRIDE; i += 64) sacc[wv][i] = 0;
  if constexpr (FO) {
    for (uint32_t i = tid; i < fo.nf; i += LDS_T) fh[i] = 0;
    part_lds_load(fo, sP[0]);
  }
  __syncthreads();
  const PartLds* P = reinterpret_cast<const PartLds*>(sP);
  for (int64_t ti = blockIdx.x; ti < n_tasks; ti += gridDim.x) {
    const Task T = tasks[ti];
    uint32_t* W = (T.buf ? w1 : w0) + T.begin;
    const uint32_t rk = row_key[T.row];
    const uint32_t len = T.len;  // (SORT_MAX, LDS_CAP] by classification
    const uint32_t nsub = (len + LDS_SUBW - 1) / LDS_SUBW;
    uint32_t wr[LDS_WPT];
#pragma unroll
    for (int j = 0; j < LDS_WPT; ++j) {
      const uint32_t i = (uint32_t)(j * LDS_T + tid);
      wr[j] = i < len ? W[i] : W_EMPTY;
    }
    uint32_t ndrop = 0;
    if constexpr (FO) {  // the cut words are dropped before the partition (branch-free, as in k_agg_sort)
      if ((int)(rk >> L.A) == fo.type) {
        const int32_t ad = (int32_t)(rk & L.amask);
#pragma unroll
        for (int j = 0; j < LDS_WPT; ++j) {
          const bool dr = fo_drop(fo, wr[j], ad, L);
          ndrop += dr ? 1u : 0u;
          wr[j] = dr ? W_EMPTY : wr[j];
        }
      }
    }
    if (tid < LDS_NSUB) sh[tid] = 0;
    __syncthreads();
    uint32_t dr[LDS_WPT];
#pragma unroll
    for (int j = 0; j < LDS_WPT; ++j) {  // sub-bucket << 16 | the word's rank in it
      const uint32_t d = split_digit(wr[j], L.F, T.rem + 64u, nsub);
      dr[j] = (d << 16) | (wr[j] != W_EMPTY ? atomicAdd(&sh[d], 1u) : 0u);
    }
    __syncthreads();
    {  // sub-bucket starts ss[0..LDS_NSUB] (exclusive scan over threads 0..127; ss[d >= nsub] = kept words)
      const uint32_t c = tid < (int)nsub ? sh[tid] : 0u;
      const uint32_t incl = wave_incl_scan(c);
      if (l == 63u) wtot[wv] = incl;
      __syncthreads();
      const uint32_t pre = wv == 1 ? wtot[0] : 0u;
      if (tid < LDS_NSUB) ss[tid] = pre + incl - c;
      if (tid == LDS_NSUB - 1) ss[LDS_NSUB] = pre + incl;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < LDS_WPT; ++j)
      if (wr[j] != W_EMPTY) words[ss[dr[j] >> 16] + (dr[j] & 0xFFFFu)] = wr[j];
    // segments: sub-bucket d starts one when its key differs from that of d - 1 (key: the LDS_SEG window
    // of its start, or its own id above LDS_BIG words)
    bool st = false;
    uint64_t sm = 0;
    if (tid < LDS_NSUB) {
      const uint32_t d = (uint32_t)tid;
      auto key = [&](uint32_t e) {
        return ss[e + 1] - ss[e] > (uint32_t)LDS_BIG ? (0x80000000u | e) : ss[e] / (uint32_t)LDS_SEG;
      };
      st = d < nsub && (d == 0 || key(d) != key(d - 1));
      sm = __ballot(st);
      if (l == 0u) wtot[wv] = (uint32_t)__popcll(sm);  // wtot's scan values were read before the last barrier
    }
    __syncthreads();
    if (tid < LDS_NSUB) {
      const uint32_t n0 = wtot[0], n1 = wtot[1];
      if (st) seg[(wv == 1 ? n0 : 0u) + mbcnt(sm)] = (uint32_t)tid;
      if (tid == 0) { nseg = n0 + n1; seg[n0 + n1] = nsub; }
    }
    __syncthreads();
    const uint32_t ns = nseg;
    for (uint32_t j = (uint32_t)wv; j < ns; j += LDS_T / 64) {
      const uint32_t b = __builtin_amdgcn_readfirstlane(ss[seg[j]]), e = __builtin_amdgcn_readfirstlane(ss[seg[j + 1]]);
      const uint32_t n = e - b;
      if (n > 512u) {  // hot keys: back to the word buffer, split at this level (then hashed)
        for (uint32_t i = l; i < n; i += 64) W[b + i] = words[b + i];
        if (l == 0u) {
          const unsigned long long k = atomicAdd(n_overflow, 1ull);
          Task t2;
          // split at the last level that may still split: its sub-buckets (rem SPLIT_LEVELS) are hashed or
          // register-sorted, never sent to an LDS leaf again (a hot key would cycle leaf -> split -> leaf)
          t2.begin = T.begin + b; t2.len = n; t2.row = T.row; t2.buf = T.buf;
          t2.rem = T.rem < (uint32_t)(SPLIT_LEVELS - 1) ? (uint32_t)(SPLIT_LEVELS - 1) : T.rem;
          if (k < ov_cap) overflow[k] = t2; else atomicOr(err, 4);
        }
      } else if (n > 256u) {
        uint32_t v[8];
#pragma unroll
        for (int m = 0; m < 8; ++m) {
          const uint32_t i = (uint32_t)(m * 64) + l;
          v[m] = i < n ? words[b + i] : W_EMPTY;
        }
        agg_fold<8, FO>(v, T.begin + b, n, rk, sR, L, O, fo, P, fh, stg[wv][0], stg[wv][1], sacc[wv]);
      } else if (n > 0u) {
        uint32_t v[4];
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          const uint32_t i = (uint32_t)(m * 64) + l;
          v[m] = i < n ? words[b + i] : W_EMPTY;
        }
        agg_fold<4, FO>(v, T.begin + b, n, rk, sR, L, O, fo, P, fh, stg[wv][0], stg[wv][1], sacc[wv]);
      }
    }
    const uint32_t kept = ss[LDS_NSUB];  // the words cut by the file options leave [kept, len) without rows
    if (O.cap)
      for (uint32_t i = kept + (uint32_t)tid; i < len; i += LDS_T) O.rule[T.begin + i] = 0xFF;
    if constexpr (FO) {
      const uint32_t nd = wave_sum(ndrop);
      if (nd && l == 0u) atomicAdd(fo.dropped, (unsigned long long)nd);
    }
    __syncthreads();  // words / sh / ss / seg are rewritten by the next task
  }
  const uint32_t gwave = blockIdx.x * (LDS_T / 64) + wv;
  unsigned long long* stats = O.stats + (size_t)(gwave & (STAT_STRIPES - 1)) * STAT_STRIDE;
  for (int i = (int)l; i < STAT_STRIDE; i += 64)
    if (sacc[wv][i]) atomicAdd(&stats[i], sacc[wv][i]);
  if constexpr (FO) {
    if (fo.hist) {
      __syncthreads();
      for (uint32_t i = tid; i < fo.nf; i += LDS_T)
        if (fh[i]) atomicAdd(&fo.hist[i], fh[i]);
    }
  }
}

// ------------------------------------------------------------------ per-rule compaction
// One rule's rows of a table, compacted in slot order without per-slot flag / index arrays:
// per 4096-slot block a count (k_blk_count), one scan over the blocks, and a compaction that
// re-evaluates the predicate with wave ballots and block prefixes (k_blk_compact). The predicate is
// rule == r and, with thr > 0, (use_ge2 ? count_ge2 : count) >= thr. sym: the rule's rows are stored
// once (aid <= aid_next); a kept row with aid != aid_next stands for itself and its mirror
// (aid_next, aid), written right after it.
constexpr int FIN_T = 256, FIN_PER = 16, FIN_B = FIN_T * FIN_PER;
// Slot scans read 4 consecutive slots per thread (slot arrays are 16-B aligned and i % 4 == 0): the rule
// bytes as one u32, a u32 column as one uint4 (one-byte / one-word loads per slot ran at a third of HBM
// bandwidth). Past n: rule 0xFF (no row). A block's FIN_B slots are 16 consecutive slots per thread.
__device__ __forceinline__ uint32_t ld_rule4(const uint8_t* __restrict__ rule, int64_t i, int64_t n) {
  if (i + 4 <= n) return *reinterpret_cast<const uint32_t*>(rule + i);
  uint32_t r = 0xFFFFFFFFu;
  for (int j = 0; j < 4; ++j)
    if (i + j < n) r = (r & ~(0xFFu << (8 * j))) | ((uint32_t)rule[i + j] << (8 * j));
  return r;
}
__device__ __forceinline__ uint4 ld_u4(const uint32_t* __restrict__ p, int64_t i, int64_t n) {
  if (i + 4 <= n) return *reinterpret_cast<const uint4*>(p + i);
  uint4 v = make_uint4(0u, 0u, 0u, 0u);
  if (i < n) v.x = p[i];
  if (i + 1 < n) v.y = p[i + 1];
  if (i + 2 < n) v.z = p[i + 2];
  return v;
}
__device__ __forceinline__ uint32_t u4_at(const uint4& v, int j) { return j == 0 ? v.x : (j == 1 ? v.y : (j == 2 ? v.z : v.w)); }
// bit j: byte j of r4 equals r
__device__ __forceinline__ uint32_t rule4_match(uint32_t r4, uint32_t r) {
  uint32_t m = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) m |= (((r4 >> (8 * j)) & 0xFFu) == r ? 1u : 0u) << j;
  return m;
}
// 16 consecutive slots per thread (i % 16 == 0): the rule bytes as one uint4, then the u32 columns of the
// 4-slot groups that hold a candidate as up to 4 independent uint4 loads. Four slots per thread left the
// scans latency-bound (rule -> column -> aid chain per 4 slots: about a fifth of HBM bandwidth).
constexpr int SLOTS_T = 16;
static_assert(FIN_B == FIN_T * SLOTS_T, "a finalize block is one 16-slot run per thread");
__device__ __forceinline__ uint4 ld_rule16(const uint8_t* __restrict__ rule, int64_t i, int64_t n) {
  if (i + 16 <= n) return *reinterpret_cast<const uint4*>(rule + i);
  return make_uint4(ld_rule4(rule, i, n), ld_rule4(rule, i + 4, n), ld_rule4(rule, i + 8, n), ld_rule4(rule, i + 12, n));
}
__device__ __forceinline__ uint32_t rule_at(const uint4& R, int s) { return (u4_at(R, s >> 2) >> (8 * (s & 3))) & 0xFFu; }
struct Slots16 {
  uint4 V[4], A[4], B[4], G[4];
  __device__ __forceinline__ uint32_t v(int s) const { return u4_at(V[s >> 2], s & 3); }
  __device__ __forceinline__ uint32_t a(int s) const { return u4_at(A[s >> 2], s & 3); }
  __device__ __forceinline__ uint32_t b(int s) const { return u4_at(B[s >> 2], s & 3); }
  __device__ __forceinline__ uint32_t g(int s) const { return u4_at(G[s >> 2], s & 3); }
};
// loads column `col` for the 4-slot groups with a bit in mask
__device__ __forceinline__ void ld_groups(const uint32_t* __restrict__ col, int64_t i, int64_t n, uint32_t mask,
                                          uint4 (&X)[4]) {
#pragma unroll
  for (int g = 0; g < 4; ++g) X[g] = ((mask >> (4 * g)) & 15u) ? ld_u4(col, i + 4 * g, n) : make_uint4(0u, 0u, 0u, 0u);
}
// blk_keep over the 16 slots at i: keep / mir bit masks (bit s = slot i + s); V always loaded for kept
// groups when `out`, A / B when `out` or sym (the mirror test), G when want_g
__device__ __forceinline__ void blk_keep16(const uint8_t* __restrict__ rule, const int32_t* __restrict__ a,
                                           const int32_t* __restrict__ b, const uint32_t* __restrict__ c,
                                           const uint32_t* __restrict__ c2, int64_t i, int64_t n, int r, int use_ge2,
                                           uint32_t thr, int sym, bool out, bool want_g, uint32_t& keep,
                                           uint32_t& mir, Slots16& S) {
  const uint4 R = ld_rule16(rule, i, n);
  keep = 0; mir = 0;
#pragma unroll
  for (int g = 0; g < 4; ++g) keep |= rule4_match(u4_at(R, g), (uint32_t)r) << (4 * g);
  if (!keep) return;
  if (thr || out) ld_groups(use_ge2 ? c2 : c, i, n, keep, S.V);
  if (want_g) {
    if (use_ge2) {
#pragma unroll
      for (int g = 0; g < 4; ++g) S.G[g] = S.V[g];
    } else {
      ld_groups(c2, i, n, keep, S.G);
    }
  }
  if (thr) {
#pragma unroll
    for (int s = 0; s < 16; ++s) keep &= ~((S.v(s) < thr ? 1u : 0u) << s);
    if (!keep) return;
  }
  if (out || sym) {
    ld_groups(reinterpret_cast<const uint32_t*>(a), i, n, keep, S.A);
    ld_groups(reinterpret_cast<const uint32_t*>(b), i, n, keep, S.B);
  }
  if (sym) {
#pragma unroll
    for (int s = 0; s < 16; ++s) mir |= (((keep >> s) & 1u) && S.a(s) != S.b(s) ? 1u : 0u) << s;
  }
}
__global__ __launch_bounds__(FIN_T) void k_blk_count(const uint8_t* __restrict__ rule, const int32_t* __restrict__ a,
                                                     const int32_t* __restrict__ b, const uint32_t* __restrict__ c,
                                                     const uint32_t* __restrict__ c2, int64_t n, int r, int use_ge2,
                                                     uint32_t thr, int sym, uint32_t* __restrict__ bcnt, int64_t i0 = 0) {
  __shared__ uint32_t wt[FIN_T / 64];
  const int64_t i = i0 + (int64_t)blockIdx.x * FIN_B + (int64_t)threadIdx.x * SLOTS_T;
  uint32_t k = 0;
  if (i < n) {
    uint32_t keep, mir;
    Slots16 S;
    blk_keep16(rule, a, b, c, c2, i, n, r, use_ge2, thr, sym, false, false, keep, mir, S);
    k = (uint32_t)__popc(keep) + (uint32_t)__popc(mir);
  }
  k = wave_sum(k);
  if ((threadIdx.x & 63) == 0) wt[threadIdx.x >> 6] = k;
  __syncthreads();
  if (threadIdx.x == 0) bcnt[blockIdx.x] = wt[0] + wt[1] + wt[2] + wt[3];
}
// outputs (nullable): o0 = aid, o1 = aid_next, o2 = use_ge2 ? count_ge2 : count, o3 = count_ge2
__global__ __launch_bounds__(FIN_T) void k_blk_compact(const uint8_t* __restrict__ rule, const int32_t* __restrict__ a,
                                                       const int32_t* __restrict__ b, const uint32_t* __restrict__ c,
                                                       const uint32_t* __restrict__ c2, int64_t n, int r, int use_ge2,
                                                       uint32_t thr, int sym, const uint64_t* __restrict__ boff,
                                                       uint32_t* __restrict__ o0, uint32_t* __restrict__ o1,
                                                       uint32_t* __restrict__ o2, uint32_t* __restrict__ o3, int64_t i0 = 0) {
  __shared__ uint32_t wt[FIN_T / 64];
  const int w = threadIdx.x >> 6;
  const int64_t i = i0 + (int64_t)blockIdx.x * FIN_B + (int64_t)threadIdx.x * SLOTS_T;
  uint32_t keep = 0, mir = 0;
  Slots16 S;
  if (i < n) blk_keep16(rule, a, b, c, c2, i, n, r, use_ge2, thr, sym, true, o3 != nullptr, keep, mir, S);
  // block prefix in thread order = slot order (thread t holds slots [16t, 16t + 16) of the block)
  const uint32_t kc = (uint32_t)__popc(keep) + (uint32_t)__popc(mir);
  const uint32_t incl = wave_incl_scan(kc);
  if ((threadIdx.x & 63) == 63) wt[w] = incl;
  __syncthreads();
  uint32_t pre = 0;
#pragma unroll
  for (int k = 0; k < FIN_T / 64; ++k) pre += k < w ? wt[k] : 0u;
  if (!keep) return;
  uint64_t p = boff[blockIdx.x] + pre + incl - kc;
#pragma unroll
  for (int s = 0; s < SLOTS_T; ++s) {
    if (!((keep >> s) & 1u)) continue;
    const uint32_t ai = S.a(s), bi = S.b(s), cv = S.v(s), gv = o3 ? S.g(s) : 0u;
    if (o0) o0[p] = ai;
    if (o1) o1[p] = bi;
    if (o2) o2[p] = cv;
    if (o3) o3[p] = gv;
    ++p;
    if ((mir >> s) & 1u) {
      if (o0) o0[p] = bi;
      if (o1) o1[p] = ai;
      if (o2) o2[p] = cv;
      if (o3) o3[p] = gv;
      ++p;
    }
  }
}
// the rows of every part p < np of a part-mode table (rule byte = part, no mirrors) in one pass: !OUT counts each
// block's rows per part (bcnt[p * nb + block]); OUT writes their (aid, aid_next) to sa / sb at boff[p * nb + block]
// in slot order (use_ge2: rows with count_ge2 >= thr; else count >= thr)
constexpr int KP_MAXP = 16;
template <bool OUT>
__global__ __launch_bounds__(FIN_T) void k_blk_parts(const uint8_t* __restrict__ rule, const int32_t* __restrict__ a,
                                                     const int32_t* __restrict__ b, const uint32_t* __restrict__ c,
                                                     const uint32_t* __restrict__ c2, int64_t n, int np, int use_ge2,
                                                     uint32_t thr, int64_t nb, uint32_t* __restrict__ bcnt,
                                                     const uint64_t* __restrict__ boff, uint32_t* __restrict__ sa,
                                                     uint32_t* __restrict__ sb) {
  __shared__ uint32_t wt[KP_MAXP][FIN_T / 64];
  const int w = threadIdx.x >> 6;
  const int64_t i = (int64_t)blockIdx.x * FIN_B + (int64_t)threadIdx.x * SLOTS_T;
  uint4 R = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu);
  uint32_t kept = 0;
  Slots16 S;
  if (i < n) {
    R = ld_rule16(rule, i, n);
    uint32_t live = 0;
#pragma unroll
    for (int g = 0; g < 4; ++g) live |= (u4_at(R, g) != 0xFFFFFFFFu ? 15u : 0u) << (4 * g);
    if (live) {
      if (thr) ld_groups(use_ge2 ? c2 : c, i, n, live, S.V);
#pragma unroll
      for (int s = 0; s < SLOTS_T; ++s)
        kept |= (rule_at(R, s) < (uint32_t)np && (!thr || S.v(s) >= thr) ? 1u : 0u) << s;
      if (OUT && kept) {
        ld_groups(reinterpret_cast<const uint32_t*>(a), i, n, kept, S.A);
        ld_groups(reinterpret_cast<const uint32_t*>(b), i, n, kept, S.B);
      }
    }
  }
  uint32_t incl[KP_MAXP];
#pragma unroll
  for (int p = 0; p < KP_MAXP; ++p) {
    if (p >= np) break;  // block-uniform
    uint32_t kc = 0;
#pragma unroll
    for (int s = 0; s < SLOTS_T; ++s) kc += ((kept >> s) & 1u) && rule_at(R, s) == (uint32_t)p ? 1u : 0u;
    incl[p] = wave_incl_scan(kc);
    if ((threadIdx.x & 63) == 63) wt[p][w] = incl[p];
  }
  __syncthreads();
  if (!OUT) {
    if ((int)threadIdx.x < np) {
      uint32_t t = 0;
#pragma unroll
      for (int x = 0; x < FIN_T / 64; ++x) t += wt[threadIdx.x][x];
      bcnt[(int64_t)threadIdx.x * nb + blockIdx.x] = t;
    }
    return;
  }
  if (!kept) return;
  uint64_t cur[KP_MAXP];
#pragma unroll
  for (int p = 0; p < KP_MAXP; ++p) {
    if (p >= np) break;
    uint32_t pre = 0, kc = 0;
#pragma unroll
    for (int x = 0; x < FIN_T / 64; ++x) pre += x < w ? wt[p][x] : 0u;
#pragma unroll
    for (int s = 0; s < SLOTS_T; ++s) kc += ((kept >> s) & 1u) && rule_at(R, s) == (uint32_t)p ? 1u : 0u;
    cur[p] = boff[(int64_t)p * nb + blockIdx.x] + pre + incl[p] - kc;
  }
#pragma unroll
  for (int s = 0; s < SLOTS_T; ++s) {
    if (!((kept >> s) & 1u)) continue;
    const uint32_t p = rule_at(R, s);
    uint64_t o = 0;
#pragma unroll
    for (int q = 0; q < KP_MAXP; ++q)
      if ((uint32_t)q == p) o = cur[q]++;
    sa[o] = S.a(s);
    sb[o] = S.b(s);
  }
}
// out[p] = boff[p * nb] (p < np), out[np] = the total
__global__ void k_part_seg(const uint64_t* __restrict__ boff, int64_t nb, int np, uint64_t* __restrict__ out) {
  const int p = threadIdx.x;
  if (p <= np) out[p] = boff[(int64_t)p * nb];
}

// rows and pairs per rule byte (part-mode tables: per part), block histograms in LDS
__global__ __launch_bounds__(256) void k_rule_hist(const uint8_t* __restrict__ rule, const uint32_t* __restrict__ count,
                                                   int64_t n, unsigned long long* __restrict__ rows,
                                                   unsigned long long* __restrict__ pairs) {
  __shared__ unsigned long long hr[256], hp[256];
  hr[threadIdx.x] = 0; hp[threadIdx.x] = 0;
  __syncthreads();
  // 16 consecutive slots per thread; runs of equal rule bytes among them (the common case: one row's slots)
  // take one pair of LDS atomics
  const int64_t stride = (int64_t)gridDim.x * blockDim.x * SLOTS_T;
  for (int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * SLOTS_T; i < n; i += stride) {
    const uint4 R = ld_rule16(rule, i, n);
    uint32_t live = 0;
#pragma unroll
    for (int g = 0; g < 4; ++g) live |= (u4_at(R, g) != 0xFFFFFFFFu ? 15u : 0u) << (4 * g);
    if (!live) continue;
    uint4 C[4];
    ld_groups(count, i, n, live, C);
    uint32_t cur = 0xFFu, nr = 0;
    unsigned long long np = 0;
#pragma unroll
    for (int s = 0; s < SLOTS_T; ++s) {
      const uint32_t r = rule_at(R, s);
      if (r == 0xFFu) continue;
      if (r != cur) {
        if (cur != 0xFFu) { atomicAdd(&hr[cur], (unsigned long long)nr); atomicAdd(&hp[cur], np); }
        cur = r; nr = 0; np = 0;
      }
      ++nr;
      np += u4_at(C[s >> 2], s & 3);
    }
    if (cur != 0xFFu) { atomicAdd(&hr[cur], (unsigned long long)nr); atomicAdd(&hp[cur], np); }
  }
  __syncthreads();
  if (hr[threadIdx.x]) { atomicAdd(&rows[threadIdx.x], hr[threadIdx.x]); atomicAdd(&pairs[threadIdx.x], hp[threadIdx.x]); }
}

// ---- heads of every part of a part-mode table (ottohip_table_part_heads): per part p the first K rows of
// (v desc, aid asc, aid_next asc) among rows with v >= thr (v = count_ge2 or count) are exactly the rows
// with v > c*_p, or v == c*_p and (aid, aid_next) <= (a*_p, n*_p) -- the cut found by histograms over v,
// then over the aids of the tie rows, then over the aid_next of the cut aid (no sort of the part).
constexpr int PH_MAXP = 32;        // parts per call
constexpr uint32_t PH_VBINS = 65536;  // v histogram bins (v >= 65535 share the last: the host falls back)
struct PartCut {
  uint32_t cstar[PH_MAXP];  // 0: keep every row with v >= thr
  uint32_t astar[PH_MAXP];  // 0xFFFFFFFF: no tie cut on aid (every tie row kept)
  uint32_t nstar[PH_MAXP];
  uint32_t stage[PH_MAXP];  // tie histograms: 1 = aids of the v == c* rows, 2 = aid_next of the (c*, a*) rows
};
__global__ __launch_bounds__(256) void k_ph_hist(const uint8_t* __restrict__ rule, const uint32_t* __restrict__ c,
                                                 const uint32_t* __restrict__ c2, int64_t n, int n_parts, int use_ge2,
                                                 uint32_t thr, unsigned long long* __restrict__ hist) {
  __shared__ uint32_t hs[PH_MAXP][256];
  for (int i = threadIdx.x; i < PH_MAXP * 256; i += 256) (&hs[0][0])[i] = 0;
  __syncthreads();
  auto add = [&](uint32_t p, uint32_t v, uint32_t k) {
    if (v < 256u) atomicAdd(&hs[p][v], k);
    else atomicAdd(&hist[(uint64_t)p * PH_VBINS + (v < PH_VBINS ? v : PH_VBINS - 1)], (unsigned long long)k);
  };
  const int l = (int)lane_id();
  // 16 slots per thread; the counts of v in [thr, thr + 8) of the thread's first part are kept in registers
  // (four 16-bit fields per u64) and summed over the wave when its lanes share that part -- the common case:
  // most rows have v near thr, so per-slot LDS atomics on a few bins serialised the wave
  const int64_t stride = (int64_t)gridDim.x * blockDim.x * SLOTS_T;
  for (int64_t i0 = ((int64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63)) * SLOTS_T; i0 < n; i0 += stride) {  // wave-uniform
    const int64_t i = i0 + (int64_t)l * SLOTS_T;
    uint4 R = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu);
    if (i < n) R = ld_rule16(rule, i, n);
    uint32_t live = 0;
#pragma unroll
    for (int g = 0; g < 4; ++g) live |= (u4_at(R, g) != 0xFFFFFFFFu ? 15u : 0u) << (4 * g);
    uint4 V[4];
    ld_groups(use_ge2 ? c2 : c, i, n, live, V);
    uint32_t p0 = 0xFFu;
    unsigned long long lo = 0, hi = 0;
#pragma unroll
    for (int s = 0; s < SLOTS_T; ++s) {
      const uint32_t p = rule_at(R, s), v = u4_at(V[s >> 2], s & 3);
      if (p >= (uint32_t)n_parts || v < thr) continue;
      const uint32_t d = v - thr;
      if (p0 == 0xFFu) p0 = p;
      if (p == p0 && d < 8u) {
        const unsigned long long inc = 1ull << (16 * (d & 3u));
        if (d < 4u) lo += inc; else hi += inc;
      } else {
        add(p, v, 1u);
      }
    }
    const bool has = (lo | hi) != 0ull;
    const uint64_t act = __ballot(has);
    if (!act) continue;
    const uint32_t pf = (uint32_t)__shfl((int)p0, __ffsll((long long)act) - 1);
    if (!__ballot(has && p0 != pf)) {  // one part: wave sums, lane 0 adds
      lo = wave_sum64(lo);
      hi = wave_sum64(hi);
      if (l == 0) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const uint32_t x = (uint32_t)(((k < 4 ? lo : hi) >> (16 * (k & 3))) & 0xFFFFull);
          if (x) add(pf, thr + (uint32_t)k, x);
        }
      }
    } else if (has) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const uint32_t x = (uint32_t)(((k < 4 ? lo : hi) >> (16 * (k & 3))) & 0xFFFFull);
        if (x) add(p0, thr + (uint32_t)k, x);
      }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < n_parts * 256; i += 256) {
    const uint32_t x = (&hs[0][0])[i];
    if (x) atomicAdd(&hist[(uint64_t)(i >> 8) * PH_VBINS + (i & 255)], (unsigned long long)x);
  }
}
// The tie cut. A part's slots sit in aid order (rows sorted by aid; the parts' rows interleave inside an aid's
// range), so the aid of the part's need-th tie row (v == c*) in slot order is a*: stage 1 is a rank search --
// per-block tie counts per part (k_ph_rank_count), one scan, the block holding the rank (k_ph_find_multi), the
// slot inside it (k_ph_tie_pick). Stage 2 histograms the aid_next of the part's (c*, a*) tie rows and counts
// its ties with aid < a* (the rank left for the aid_next cut).
struct PhRank {
  uint64_t need[PH_MAXP];  // per stage-1 part q: the rank (1-based) of the cut tie row
  uint32_t part[PH_MAXP];
};
// stage-1 parts in q order: qx[p] = q, or -1
__device__ __forceinline__ void ph_qindex(const PartCut& pc, int n_parts, int* qx) {
  int q = 0;
  for (int p = 0; p < PH_MAXP; ++p) qx[p] = p < n_parts && pc.stage[p] == 1u ? q++ : -1;
}
// tie rows (v == c*) of the stage-1 parts among the 16 slots at i: bit mask, and the slots' parts in R
__device__ __forceinline__ uint32_t ph_ties16(const uint8_t* __restrict__ rule, const uint32_t* __restrict__ vcol,
                                              int64_t i, int64_t n, int n_parts, const PartCut& pc, uint32_t stage,
                                              uint4& R) {
  R = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu);
  if (i < n) R = ld_rule16(rule, i, n);
  uint32_t live = 0;
#pragma unroll
  for (int g = 0; g < 4; ++g) live |= (u4_at(R, g) != 0xFFFFFFFFu ? 15u : 0u) << (4 * g);
  uint4 V[4];
  ld_groups(vcol, i, n, live, V);
  uint32_t tie = 0;
#pragma unroll
  for (int s = 0; s < SLOTS_T; ++s) {
    const uint32_t p = rule_at(R, s);
    tie |= (p < (uint32_t)n_parts && pc.stage[p] == stage && u4_at(V[s >> 2], s & 3) == pc.cstar[p] ? 1u : 0u) << s;
  }
  return tie;
}
// per FIN_B block: tie rows per stage-1 part -> bcnt[q * nb + block]; with baid, the aids of the block's first and last
// part rows -> baid[2 block], baid[2 block + 1] (an empty block: 0xFFFFFFFF, 0): the slots are in aid order, so the
// blocks that can hold a cut aid's rows form one range (k_ph_aid_range)
__global__ __launch_bounds__(FIN_T) void k_ph_rank_count(const uint8_t* __restrict__ rule, const uint32_t* __restrict__ c,
                                                         const uint32_t* __restrict__ c2, int64_t n, int n_parts,
                                                         int use_ge2, PartCut pc_arg, int64_t nb,
                                                         uint32_t* __restrict__ bcnt, const int32_t* __restrict__ a = nullptr,
                                                         uint32_t* __restrict__ baid = nullptr, uint32_t thr = 1u,
                                                         uint32_t* __restrict__ sure = nullptr) {
  __shared__ PartCut pc;
  __shared__ int qx[PH_MAXP];
  __shared__ uint32_t bc[PH_MAXP];
  __shared__ uint32_t sfirst, slast, ssure;
  if (threadIdx.x == 0) { pc = pc_arg; ph_qindex(pc, n_parts, qx); sfirst = 0xFFFFFFFFu; slast = 0u; ssure = 0u; }
  if (threadIdx.x < PH_MAXP) bc[threadIdx.x] = 0;
  __syncthreads();
  const int64_t i = (int64_t)blockIdx.x * FIN_B + (int64_t)threadIdx.x * SLOTS_T;
  uint4 R;
  const uint32_t tie = ph_ties16(rule, use_ge2 ? c2 : c, i, n, n_parts, pc, 1u, R);
  if (sure) {  // rows kept whatever the tie cut: v > c*, or v == c* of a part without a tie cut (k_ph_count's test)
    uint4 V[4];
    uint32_t live = 0;
#pragma unroll
    for (int g = 0; g < 4; ++g) live |= (u4_at(R, g) != 0xFFFFFFFFu ? 15u : 0u) << (4 * g);
    ld_groups(use_ge2 ? c2 : c, i, n, live, V);
    uint32_t k = 0;
#pragma unroll
    for (int s = 0; s < SLOTS_T; ++s) {
      const uint32_t p = rule_at(R, s), v = u4_at(V[s >> 2], s & 3);
      if (p >= (uint32_t)n_parts || v < thr) continue;
      k += (v > pc.cstar[p] || (v == pc.cstar[p] && pc.stage[p] != 1u)) ? 1u : 0u;
    }
    k = wave_sum(k);
    if (lane_id() == 0 && k) atomicAdd(&ssure, k);
  }
  if (baid) {  // the block's first and last slot holding a part row (slot offsets inside the block, + 1 for the last)
    uint32_t live = 0;
#pragma unroll
    for (int s = 0; s < SLOTS_T; ++s) live |= (rule_at(R, s) < (uint32_t)n_parts ? 1u : 0u) << s;
    // threads hold consecutive slots: the wave's first / last thread with a part row holds its first / last one (one
    // LDS atomic per wave; one per thread serialised 256 atomics on two words per block)
    const uint32_t o = (uint32_t)threadIdx.x * SLOTS_T;
    const uint32_t fs = live ? o + (uint32_t)(__ffs((int)live) - 1) : 0xFFFFFFFFu;
    const uint32_t ls = live ? o + (uint32_t)(32 - __clz((int)live)) : 0u;
    const uint64_t m = __ballot(live != 0u);
    if (m) {
      const int lf = __ffsll((long long)m) - 1, ll = 63 - __clzll((long long)m);
      const uint32_t wf = (uint32_t)__shfl((int)fs, lf), wl = (uint32_t)__shfl((int)ls, ll);
      if (lane_id() == 0) { atomicMin(&sfirst, wf); atomicMax(&slast, wl); }
    }
  }
  uint32_t cp = 0xFFu, cc = 0;
#pragma unroll
  for (int s = 0; s < SLOTS_T; ++s) {  // runs of one part: one LDS atomic each
    if (!((tie >> s) & 1u)) continue;
    const uint32_t p = rule_at(R, s);
    if (p != cp) {
      if (cc) atomicAdd(&bc[qx[cp]], cc);
      cp = p; cc = 0;
    }
    ++cc;
  }
  if (cc) atomicAdd(&bc[qx[cp]], cc);
  __syncthreads();
  if (threadIdx.x < PH_MAXP && qx[threadIdx.x] >= 0)
    bcnt[(int64_t)qx[threadIdx.x] * nb + blockIdx.x] = bc[qx[threadIdx.x]];
  if (sure && threadIdx.x == 0) sure[blockIdx.x] = ssure;
  if (baid && threadIdx.x == 0) {
    const int64_t b0 = (int64_t)blockIdx.x * FIN_B;
    const bool any = sfirst != 0xFFFFFFFFu;
    baid[2 * blockIdx.x] = any ? (uint32_t)a[b0 + sfirst] : 0xFFFFFFFFu;
    baid[2 * blockIdx.x + 1] = any ? (uint32_t)a[b0 + slast - 1] : 0u;
  }
}
// per stage-2 part q (its cut aid astar[q]): the first block whose last aid is >= a* and the last block whose first
// aid is <= a* (empty blocks skipped) -> range[2q] (atomicMin), range[2q + 1] (atomicMax); every slot of aid a* lies in
// between, and no slot before the range holds an aid >= a*
__global__ void k_ph_aid_range(const uint32_t* __restrict__ baid, int64_t nb, int nq, const uint32_t* __restrict__ astar,
                               uint32_t* __restrict__ range) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nb * nq) return;
  const int q = (int)(t / nb);
  const int64_t j = t - (int64_t)q * nb;
  const uint32_t f = baid[2 * j], l = baid[2 * j + 1], as = astar[q];
  if (f == 0xFFFFFFFFu || as == 0xFFFFFFFFu) return;
  // only the blocks at an edge take an atomic (its neighbour on the outside ends below / starts above a*, or is empty);
  // every block past the cut taking one serialised millions of atomics on one word
  const uint32_t lprev = j > 0 ? baid[2 * j - 1] : 0u;               // empty: 0
  const uint32_t fnext = j + 1 < nb ? baid[2 * j + 2] : 0xFFFFFFFFu;  // empty: 0xFFFFFFFF
  if (l >= as && lprev < as) atomicMin(&range[2 * q], (uint32_t)j);
  if (f <= as && fnext > as) atomicMax(&range[2 * q + 1], (uint32_t)j);
}
// per stage-1 part q: the block j whose tie range holds rank need[q] (ex = one exclusive scan over all q's
// blocks), found[2q] = j, found[2q + 1] = the rank inside block j
__global__ void k_ph_find_multi(const uint64_t* __restrict__ ex, const uint32_t* __restrict__ bcnt, int64_t nb, int nq,
                                PhRank rk, uint32_t* __restrict__ found) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nb * nq) return;
  const int q = (int)(t / nb);
  const uint64_t lo = ex[t] - ex[(int64_t)q * nb], hi = lo + bcnt[t], need = rk.need[q];
  if (bcnt[t] && lo < need && need <= hi) { found[2 * q] = (uint32_t)(t - (int64_t)q * nb); found[2 * q + 1] = (uint32_t)(need - lo); }
}
// one block per stage-1 part q: the found[2q + 1]-th tie row of the part in block found[2q] -> its aid
__global__ __launch_bounds__(FIN_T) void k_ph_tie_pick(const uint8_t* __restrict__ rule, const int32_t* __restrict__ a,
                                                       const uint32_t* __restrict__ c, const uint32_t* __restrict__ c2,
                                                       int64_t n, int n_parts, int use_ge2, PartCut pc_arg, PhRank rk,
                                                       const uint32_t* __restrict__ found, uint32_t* __restrict__ astar) {
  __shared__ PartCut pc;
  __shared__ uint32_t wt[FIN_T / 64];
  if (threadIdx.x == 0) pc = pc_arg;
  __syncthreads();
  const int q = blockIdx.x;
  const uint32_t j = found[2 * q], r = found[2 * q + 1], p = rk.part[q];
  if (j == 0xFFFFFFFFu) return;  // block-uniform: the host reports the missing cut
  const int64_t i = (int64_t)j * FIN_B + (int64_t)threadIdx.x * SLOTS_T;
  uint4 R;
  uint32_t tie = ph_ties16(rule, use_ge2 ? c2 : c, i, n, n_parts, pc, 1u, R);
#pragma unroll
  for (int s = 0; s < SLOTS_T; ++s) tie &= ~((rule_at(R, s) != p ? 1u : 0u) << s);
  const uint32_t k = (uint32_t)__popc(tie), incl = wave_incl_scan(k);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 63) wt[w] = incl;
  __syncthreads();
  uint32_t pre = incl - k;
  for (int x = 0; x < w; ++x) pre += wt[x];
  if (pre < r && r <= pre + k) {
    uint32_t m = tie;
    for (uint32_t x = pre + 1; x < r; ++x) m &= m - 1;  // drop the lower set bits
    astar[q] = (uint32_t)a[i + __ffs((int)m) - 1];
  }
}
// stage 1 on a table whose slots are not in aid order (explicit mirror rows, ottohip_table_count_parts): per
// stage-1 part q, a histogram over the aids of its tie rows, h[q * n_items + aid]; a thread's runs of one (part, aid)
// take one atomic each, and a wave whose lanes' last runs share one (part, aid) (a hot aid's rows) takes one for all
__global__ __launch_bounds__(256) void k_ph_tie_aid_hist(const uint8_t* __restrict__ rule, const int32_t* __restrict__ a,
                                                         const uint32_t* __restrict__ c, const uint32_t* __restrict__ c2,
                                                         int64_t n, int n_parts, int use_ge2, PartCut pc_arg,
                                                         int64_t n_items, uint32_t* __restrict__ h) {
  __shared__ PartCut pc;
  __shared__ int qx[PH_MAXP];
  if (threadIdx.x == 0) { pc = pc_arg; ph_qindex(pc, n_parts, qx); }
  __syncthreads();
  const int l = (int)lane_id();
  const int64_t stride = (int64_t)gridDim.x * blockDim.x * SLOTS_T;
  for (int64_t i0 = ((int64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63)) * SLOTS_T; i0 < n; i0 += stride) {  // wave-uniform
    const int64_t i = i0 + (int64_t)l * SLOTS_T;
    uint4 R;
    const uint32_t tie = ph_ties16(rule, use_ge2 ? c2 : c, i, n, n_parts, pc, 1u, R);
    if (!__ballot(tie != 0u)) continue;
    uint4 A[4];
    ld_groups(reinterpret_cast<const uint32_t*>(a), i, n, tie, A);
    uint32_t cp = 0xFFu, ca = 0, cc = 0;
#pragma unroll
    for (int s = 0; s < SLOTS_T; ++s) {
      if (!((tie >> s) & 1u)) continue;
      const uint32_t p = rule_at(R, s), ai = u4_at(A[s >> 2], s & 3);
      if (p != cp || ai != ca) {
        if (cc) atomicAdd(&h[(uint64_t)qx[cp] * n_items + ca], cc);
        cp = p; ca = ai; cc = 0;
      }
      ++cc;
    }
    // the last run of every lane: one atomic for the wave when all of them name the same (part, aid)
    const uint32_t key = cc ? ((cp << 24) | ca) : 0xFFFFFFFFu;
    const uint64_t act = __ballot(cc != 0u);
    const uint32_t k0 = (uint32_t)__shfl((int)key, __ffsll((long long)act) - 1);
    if (!__ballot(cc != 0u && key != k0)) {
      const uint32_t tot = wave_sum(cc);
      if (l == __ffsll((long long)act) - 1) atomicAdd(&h[(uint64_t)qx[cp] * n_items + ca], tot);
    } else if (cc) {
      atomicAdd(&h[(uint64_t)qx[cp] * n_items + ca], cc);
    }
  }
}
// stage 2: aid_next histogram of the (c*, a*) tie rows of the stage-2 parts, and per part the tie rows with
// aid < a* (lt); 16 slots per thread, grid-stride
// kept rows per block from the rank pass (k_ph_count's result without re-reading the table): the sure rows plus, per
// stage-2 part q, all of its tie rows in blocks before its cut aid's range and none after it; blocks inside some
// range [rng[2q], rng[2q + 1]] are left to k_ph_count (flag 1 in inr)
__global__ void k_ph_combine(const uint32_t* __restrict__ sure, const uint32_t* __restrict__ tcnt, int64_t nb, int nq,
                             const uint32_t* __restrict__ rng, uint32_t* __restrict__ bcnt, uint32_t* __restrict__ inr) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= nb) return;
  uint32_t k = sure[j], in = 0;
  for (int q = 0; q < nq; ++q) {
    const uint32_t lo = rng[2 * q], hi = rng[2 * q + 1];
    if ((uint64_t)j < lo) k += tcnt[(int64_t)q * nb + j];
    else if ((uint64_t)j <= hi) in = 1;
  }
  bcnt[j] = k;
  inr[j] = in;
}
// slot range [s0, n) (s0 a multiple of SLOTS_T); only_part >= 0: that part's rows only (the others' stage stays 2
// for their own launches)
__global__ __launch_bounds__(256) void k_ph_tie_hist2(const uint8_t* __restrict__ rule, const int32_t* __restrict__ a,
                                                      const int32_t* __restrict__ b, const uint32_t* __restrict__ c,
                                                      const uint32_t* __restrict__ c2, int64_t n, int n_parts,
                                                      int use_ge2, PartCut pc_arg, int64_t n_items,
                                                      uint32_t* __restrict__ h, unsigned long long* __restrict__ lt,
                                                      int64_t s0 = 0, int only_part = -1) {
  // the cut tables in LDS: indexing the kernel-argument copy by a lane's part went through scratch memory
  __shared__ PartCut pc;
  __shared__ uint32_t lts[PH_MAXP];
  if (threadIdx.x == 0) {
    pc = pc_arg;
    if (only_part >= 0)
      for (int p = 0; p < PH_MAXP; ++p)
        if (p != only_part && pc.stage[p] == 2u) pc.stage[p] = 4u;  // not this launch's part
  }
  if (threadIdx.x < PH_MAXP) lts[threadIdx.x] = 0;
  __syncthreads();
  const int64_t stride = (int64_t)gridDim.x * blockDim.x * SLOTS_T;
  for (int64_t i = s0 + ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * SLOTS_T; i < n; i += stride) {
    uint4 R;
    const uint32_t tie = ph_ties16(rule, use_ge2 ? c2 : c, i, n, n_parts, pc, 2u, R);
    if (!tie) continue;
    uint4 A[4];
    ld_groups(reinterpret_cast<const uint32_t*>(a), i, n, tie, A);
    uint32_t cp = 0xFFu, cc = 0, at = 0;
#pragma unroll
    for (int s = 0; s < SLOTS_T; ++s) {
      if (!((tie >> s) & 1u)) continue;
      const uint32_t p = rule_at(R, s), ai = u4_at(A[s >> 2], s & 3);
      if (ai == pc.astar[p]) {
        at |= 1u << s;
      } else if (ai < pc.astar[p]) {
        if (p != cp) {
          if (cc) atomicAdd(&lts[cp], cc);
          cp = p; cc = 0;
        }
        ++cc;
      }
    }
    if (cc) atomicAdd(&lts[cp], cc);
    if (!at) continue;
#pragma unroll
    for (int s = 0; s < SLOTS_T; ++s)  // the few rows of the cut aid
      if ((at >> s) & 1u) atomicAdd(&h[(uint64_t)rule_at(R, s) * n_items + (uint32_t)b[i + s]], 1u);
  }
  __syncthreads();
  if (threadIdx.x < PH_MAXP && lts[threadIdx.x]) atomicAdd(&lt[threadIdx.x], (unsigned long long)lts[threadIdx.x]);
}
// smallest index j with incl[j] >= need (incl = inclusive prefix of one part's histogram)
__global__ void k_ph_find(const uint64_t* __restrict__ excl, const uint32_t* __restrict__ h, int64_t n, uint64_t need,
                          uint32_t* __restrict__ out) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const uint64_t lo = excl[j], hi = lo + h[j];
  if (h[j] && lo < need && need <= hi) { out[0] = (uint32_t)j; out[1] = (uint32_t)(need - lo); }
}
// kept slots (bit mask) of the 16 at i; V loaded for the live groups, A / B for the groups with a tie row
// (and with any kept row when want_ab)
__device__ __forceinline__ uint32_t ph_keep16(const uint8_t* __restrict__ rule, const int32_t* __restrict__ a,
                                              const int32_t* __restrict__ b, const uint32_t* __restrict__ c,
                                              const uint32_t* __restrict__ c2, int64_t i, int64_t n, int n_parts,
                                              int use_ge2, uint32_t thr, const PartCut& pc, bool want_ab, Slots16& S) {
  const uint4 R = ld_rule16(rule, i, n);
  uint32_t live = 0;
#pragma unroll
  for (int g = 0; g < 4; ++g) live |= (u4_at(R, g) != 0xFFFFFFFFu ? 15u : 0u) << (4 * g);
  if (!live) return 0u;
  ld_groups(use_ge2 ? c2 : c, i, n, live, S.V);
  uint32_t keep = 0, tie = 0;
#pragma unroll
  for (int s = 0; s < SLOTS_T; ++s) {
    const uint32_t p = rule_at(R, s), v = S.v(s);
    if (p >= (uint32_t)n_parts || v < thr) continue;
    const uint32_t cs = pc.cstar[p];
    if (v != cs) keep |= (v > cs ? 1u : 0u) << s;
    else if (pc.astar[p] == 0xFFFFFFFFu) keep |= 1u << s;
    else tie |= 1u << s;
  }
  const uint32_t need = tie | (want_ab ? keep : 0u);
  if (!need) return keep;
  ld_groups(reinterpret_cast<const uint32_t*>(a), i, n, need, S.A);
  // aid_next decides only the tie rows of the cut aid (few): without the outputs, B is read for their groups only
  uint32_t eq = 0;
#pragma unroll
  for (int s = 0; s < SLOTS_T; ++s) {
    if (!((tie >> s) & 1u)) continue;
    const uint32_t p = rule_at(R, s), ai = S.a(s);
    keep |= (ai < pc.astar[p] ? 1u : 0u) << s;
    eq |= (ai == pc.astar[p] ? 1u : 0u) << s;
  }
  const uint32_t needb = want_ab ? need : eq;
  if (!needb) return keep;
  ld_groups(reinterpret_cast<const uint32_t*>(b), i, n, needb, S.B);
#pragma unroll
  for (int s = 0; s < SLOTS_T; ++s) {
    if (!((eq >> s) & 1u)) continue;
    keep |= (S.b(s) <= pc.nstar[rule_at(R, s)] ? 1u : 0u) << s;
  }
  return keep;
}
__global__ __launch_bounds__(FIN_T) void k_ph_count(const uint8_t* __restrict__ rule, const int32_t* __restrict__ a,
                                                    const int32_t* __restrict__ b, const uint32_t* __restrict__ c,
                                                    const uint32_t* __restrict__ c2, int64_t n, int n_parts, int use_ge2,
                                                    uint32_t thr, PartCut pc_arg, uint32_t* __restrict__ bcnt,
                                                    int64_t blk0 = 0, const uint32_t* __restrict__ only = nullptr) {
  __shared__ uint32_t wt[FIN_T / 64];
  __shared__ PartCut pc;  // LDS copy (lane-indexed)
  const int64_t blk = blk0 + blockIdx.x;
  if (only && !only[blk]) return;  // block-uniform: counted by k_ph_combine
  if (threadIdx.x == 0) pc = pc_arg;
  __syncthreads();
  const int64_t i = blk * FIN_B + (int64_t)threadIdx.x * SLOTS_T;
  uint32_t k = 0;
  if (i < n) {
    Slots16 S;
    k = (uint32_t)__popc(ph_keep16(rule, a, b, c, c2, i, n, n_parts, use_ge2, thr, pc, false, S));
  }
  k = wave_sum(k);
  if ((threadIdx.x & 63) == 0) wt[threadIdx.x >> 6] = k;
  __syncthreads();
  if (threadIdx.x == 0) bcnt[blk] = wt[0] + wt[1] + wt[2] + wt[3];
}
// kept rows -> records {aid, aid_next, v, 0} (rule 0) at block offsets boff, in slot order
__global__ __launch_bounds__(FIN_T) void k_ph_compact(const uint8_t* __restrict__ rule, const int32_t* __restrict__ a,
                                                      const int32_t* __restrict__ b, const uint32_t* __restrict__ c,
                                                      const uint32_t* __restrict__ c2, int64_t n, int n_parts,
                                                      int use_ge2, uint32_t thr, PartCut pc_arg,
                                                      const uint64_t* __restrict__ boff, uint4* __restrict__ out) {
  __shared__ uint32_t wt[FIN_T / 64];
  __shared__ PartCut pc;  // LDS copy (lane-indexed)
  if (threadIdx.x == 0) pc = pc_arg;
  __syncthreads();
  const int w = threadIdx.x >> 6;
  const int64_t i = (int64_t)blockIdx.x * FIN_B + (int64_t)threadIdx.x * SLOTS_T;
  Slots16 S;
  const uint32_t keep = i < n ? ph_keep16(rule, a, b, c, c2, i, n, n_parts, use_ge2, thr, pc, true, S) : 0u;
  const uint32_t kc = (uint32_t)__popc(keep);
  const uint32_t incl = wave_incl_scan(kc);
  if ((threadIdx.x & 63) == 63) wt[w] = incl;
  __syncthreads();
  uint32_t pre = 0;
#pragma unroll
  for (int k = 0; k < FIN_T / 64; ++k) pre += k < w ? wt[k] : 0u;
  if (!keep) return;
  uint64_t p = boff[blockIdx.x] + pre + incl - kc;
#pragma unroll
  for (int s = 0; s < SLOTS_T; ++s)
    if ((keep >> s) & 1u) out[p++] = make_uint4(S.a(s), S.b(s), S.v(s), 0u);
}

// ------------------------------------------------------------------ finalize (merge A6)
__global__ void k_iota_key(const uint32_t* __restrict__ src, int64_t n, uint32_t* __restrict__ key,
                           uint32_t* __restrict__ val) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  key[i] = src[i]; val[i] = (uint32_t)i;
}
// key[i] = src[val[i]] (optionally inverted for a descending sort)
__global__ void k_gather_key(const uint32_t* __restrict__ src, const uint32_t* __restrict__ val, int64_t n,
                             int invert, uint32_t* __restrict__ key) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t v = src[val[i]];
  key[i] = invert ? ~v : v;
}
__global__ void k_fin_out(const uint32_t* __restrict__ val, int64_t n, const uint32_t* __restrict__ sa,
                          const uint32_t* __restrict__ sb, const uint32_t* __restrict__ sc,
                          int32_t* __restrict__ oa, int32_t* __restrict__ ob, int32_t* __restrict__ oc) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t j = val[i];
  if (oa) oa[i] = (int32_t)sa[j];
  if (ob) ob[i] = (int32_t)sb[j];
  if (oc) oc[i] = (int32_t)sc[j];
}

}  // namespace ottohip

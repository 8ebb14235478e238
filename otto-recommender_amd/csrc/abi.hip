// Host orchestration of the co-visitation engine and the C-ABI of include/ottohip.h.
#include <cstdarg>
#include <cstdlib>
#include <ctime>
#include <algorithm>
#include <mutex>
#include "prims.h"
#include "covis_kernels.h"
#include "table.h"

using namespace ottohip;

namespace ottohip {
static thread_local char g_err[1024] = "";
void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof g_err, fmt, ap);
  va_end(ap);
}
}  // namespace ottohip

namespace ottohip {
Ctx* ctx_base(ottohip_ctx* c) { return c; }

int ensure_part_stats(const ottohip_table* tc) {
  if (!tc || !tc->part_stats_pending) return 0;
  ottohip_table* T = const_cast<ottohip_table*>(tc);
  Ctx* ctx = T->ctx;
  // the null stream, ordered after the producer's stream by the event recorded there (a torch pool stream is
  // created non-blocking, so the null stream alone would not wait for the reduce that wrote the slots)
  const hipStream_t s = nullptr;
  OH_HIP(hipSetDevice(T->device));
  if (T->produced) OH_HIP(hipStreamWaitEvent(s, T->produced, 0));
  unsigned long long* ph;
  OH_TRY(ctx->ws.get("part_hist", 512, &ph));
  OH_HIP(hipMemsetAsync(ph, 0, 512 * 8, s));
  k_rule_hist<<<(unsigned)std::min<int64_t>(ceil_div((int64_t)T->n_slots, 256 * SLOTS_T), (int64_t)ctx->n_cu * 8), 256,
                0, s>>>(T->b.rule, T->b.count, T->n_slots, ph, ph + 256);
  OH_HIP(hipGetLastError());
  std::vector<unsigned long long> hh(512);
  OH_TRY(d2h(hh.data(), ph, hh.size(), s));
  for (int p = 0; p < T->part_stats_pending; ++p) {
    T->stats[p].n_rows = (int64_t)hh[p];
    T->stats[p].n_pairs = (int64_t)hh[256 + p];
  }
  T->part_stats_pending = 0;
  if (T->produced) {
    (void)hipEventDestroy(T->produced);
    T->produced = nullptr;
  }
  return 0;
}


static bool alloc_log_on() {
  static const bool on = getenv("OTTOHIP_ALLOC_LOG") != nullptr;
  return on;
}
double alloc_log_begin() {
  if (!alloc_log_on()) return 0.0;
  timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + 1e-9 * t.tv_nsec;
}
void alloc_log_end(double t0, const char* what, const char* name, size_t bytes) {
  if (!alloc_log_on()) return;
  timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  size_t fr = 0, tot = 0;
  (void)hipMemGetInfo(&fr, &tot);
  fprintf(stderr, "[ottohip alloc] %s %-14s %10.3f MB  %8.2f ms  free %.1f GB\n", what, name, bytes / 1e6,
          1e3 * (t.tv_sec + 1e-9 * t.tv_nsec - t0), fr / 1e9);
}

// ---- device block cache (common.h), one per device: a block is handed out again only on the device it was
// allocated on, and a trim (ottohip_ctx_trim) returns only the calling device's free blocks, so one context's
// trim never frees what another device's contexts cache
static std::mutex g_cache_mu;
struct DevCache {
  std::multimap<size_t, void*> free_;  // size -> block
};
static std::map<int, DevCache> g_cache;                       // device -> its free blocks
static std::map<void*, std::pair<int, size_t>> g_cache_live;  // block -> (device, size)

static int cur_device() {
  int d = 0;
  (void)hipGetDevice(&d);
  return d;
}

hipError_t dev_alloc(void** p, size_t bytes, const char* what) {
  std::lock_guard<std::mutex> lk(g_cache_mu);
  const int dev = cur_device();
  auto& fr = g_cache[dev].free_;
  auto it = fr.lower_bound(bytes);
  if (it != fr.end() && it->first <= 2 * bytes) {
    *p = it->second;
    g_cache_live[it->second] = {dev, it->first};
    fr.erase(it);
    return hipSuccess;
  }
  const double t0 = alloc_log_begin();
  hipError_t e = hipMalloc(p, bytes);
  if (e != hipSuccess && !fr.empty()) {  // give this device's cached blocks back and retry once
    (void)hipGetLastError();
    (void)hipDeviceSynchronize();
    for (auto& kv : fr) (void)hipFree(kv.second);
    fr.clear();
    e = hipMalloc(p, bytes);
  }
  alloc_log_end(t0, "hipMalloc", what, bytes);
  if (e != hipSuccess) { (void)hipGetLastError(); *p = nullptr; return e; }
  g_cache_live[*p] = {dev, bytes};
  return hipSuccess;
}

// cached bytes are capped per device (OTTOHIP_CACHE_GB, default 128) so memory the library no longer uses
// stays available to other allocators in the process (torch)
static size_t cache_cap() {
  static const size_t cap = (size_t)((getenv("OTTOHIP_CACHE_GB") ? atof(getenv("OTTOHIP_CACHE_GB")) : 128.0) * 1e9);
  return cap;
}

void dev_free(void* p) {
  if (!p) return;
  std::lock_guard<std::mutex> lk(g_cache_mu);
  auto it = g_cache_live.find(p);
  if (it == g_cache_live.end()) { (void)hipFree(p); return; }
  const int dev = it->second.first;
  auto& fr = g_cache[dev].free_;
  fr.emplace(it->second.second, p);
  g_cache_live.erase(it);
  size_t tot = 0;
  for (auto& kv : fr) tot += kv.first;
  if (tot <= cache_cap()) return;
  int prev = -1;
  (void)hipGetDevice(&prev);
  if (prev != dev) (void)hipSetDevice(dev);
  while (tot > cache_cap() && !fr.empty()) {  // largest blocks go back first
    auto last = std::prev(fr.end());
    tot -= last->first;
    (void)hipDeviceSynchronize();
    (void)hipFree(last->second);
    fr.erase(last);
  }
  if (prev != dev) (void)hipSetDevice(prev);
}

void dev_trim() {
  std::lock_guard<std::mutex> lk(g_cache_mu);
  auto it = g_cache.find(cur_device());
  if (it == g_cache.end() || it->second.free_.empty()) return;
  (void)hipDeviceSynchronize();
  for (auto& kv : it->second.free_) (void)hipFree(kv.second);
  it->second.free_.clear();
}
}


// ---------------------------------------------------------------- count stages
// S1-S3 state of one count call (device pointers live in the context workspace)
struct Front {
  RulesDev R;
  Layout Lt;
  int64_t E = 0, Sn = 0, NB = 0;
  int nl = 0;
  const int64_t* off = nullptr;
  int64_t *first = nullptr, *fb = nullptr, *d_loff = nullptr;
  int32_t* long_list = nullptr;
  uint32_t* fid = nullptr;
  uint64_t* evp = nullptr;
  uint64_t* lscr = nullptr;
  uint32_t* lpscr = nullptr;
  uint32_t* cnt = nullptr;
  uint32_t* link = nullptr;    // grouped row entries (one-GPU / owner-local fused layout), else null
  uint64_t* poff = nullptr;
  uint32_t* poff32 = nullptr;  // instead of poff when every word offset < 2^32 (one-GPU fused layout)
  uint64_t P = 0;
  int64_t Rn = 0;
  uint32_t* row_key = nullptr;
  uint64_t* row_begin = nullptr;
};

// a count's emitted words and rows, kept by the table (ottohip_file_opts.keep_words) for ottohip_table_count_parts
struct KeptEmission {
  uint32_t* words = nullptr;      // [P] row-major pair words, as emitted
  uint32_t* row_key = nullptr;    // [Rn] (type << A) | aid, ascending
  uint64_t* row_begin = nullptr;  // [Rn] first word of each row
  uint64_t P = 0;
  int64_t Rn = 0;
  RulesDev R;
  Layout Lt;
  int n_rules = 0, n_files = 0;
};
void kept_free(KeptEmission* k) {
  if (!k) return;
  dev_free(k->words);
  dev_free(k->row_key);
  dev_free(k->row_begin);
  delete k;
}

struct ottohip_emit {
  Front F;
  ottohip_events ev;
  int n_parts = 1;
  uint64_t gen = 0;
  ottohip_ctx* ctx = nullptr;
  std::vector<uint64_t> first_row, first_word;
};

static int check_events(const ottohip_events* ev) {
  const int64_t E = ev->n_events, Sn = ev->n_sessions;
  if (E < 0 || Sn < 0 || (E > 0 && (!ev->session_offsets || !ev->aid || !ev->ts || !ev->type))) {
    set_error("bad event table"); return OTTOHIP_EINVAL;
  }
  if (E >= ((int64_t)1 << 32)) { set_error("n_events=%lld >= 2^32 (split into shards)", (long long)E); return OTTOHIP_ELIMIT; }
  if (ev->n_files < 1 || !ev->file_session_bounds) { set_error("need >= 1 file"); return OTTOHIP_EINVAL; }
  if (ev->file_session_bounds[0] != 0 || ev->file_session_bounds[ev->n_files] != Sn) {
    set_error("file_session_bounds must start at 0 and end at n_sessions"); return OTTOHIP_EINVAL;
  }
  for (int f = 0; f < ev->n_files; ++f)
    if (ev->file_session_bounds[f + 1] < ev->file_session_bounds[f]) { set_error("file bounds not monotone"); return OTTOHIP_EINVAL; }
  if (ev->n_files > 65535) { set_error("n_files > 65535"); return OTTOHIP_ELIMIT; }
  return 0;
}

// allow_sym: emit a symmetric rule's pairs once (aid_j >= aid_i) and mirror its rows (RulesDev::sym_mask);
// OTTOHIP_SYMMETRIC=0 turns it off (A/B switch)
static int setup_rules(const ottohip_rule* rules, int n_rules, const ottohip_covis_params* params, int n_files_total,
                       RulesDev& R, Layout& Lt, bool allow_sym = false) {
  if (n_rules < 1 || n_rules > MAX_RULES) { set_error("n_rules=%d outside [1, %d]", n_rules, MAX_RULES); return OTTOHIP_EINVAL; }
  if (params->n_items < 1 || params->n_items > (1 << 30)) { set_error("n_items=%d outside [1, 2^30]", params->n_items); return OTTOHIP_ERANGE; }
  if (n_files_total > 65535) { set_error("n_files > 65535"); return OTTOHIP_ELIMIT; }
  memset(&R, 0, sizeof R);
  int max_per_type = 1;
  for (int r = 0; r < n_rules; ++r) {
    const ottohip_rule& q = rules[r];
    if (q.this_type < 0 || q.this_type > 2 || (q.next_type_mask & ~7u) || q.max_abs_dt < 0) {
      set_error("rule %d invalid", r); return OTTOHIP_EINVAL;
    }
    R.lo[r] = std::max(params->min_dt, -q.max_abs_dt);
    R.hi[r] = std::min(params->max_dt, q.max_abs_dt);
    R.mask[r] = q.next_type_mask;
    int t = q.this_type;
    R.rule_of_type[t][R.n_of_type[t]++] = r;
    max_per_type = std::max(max_per_type, R.n_of_type[t]);
  }
  for (int r = 0; r < n_rules; ++r)
    if (R.lo[r] > R.hi[r]) R.mask[r] = 0;  // empty window: never matches (count stays 0)
  static const bool sym_env = !(getenv("OTTOHIP_SYMMETRIC") && !strcmp(getenv("OTTOHIP_SYMMETRIC"), "0"));
  // next types == {this type}, dt window symmetric: (i, j) qualifies iff (j, i) does. At most one such
  // rule per event type is stored once: k_emit places an event's symmetric record after all of its
  // other records (its written length is known only to S2's count), so a second one would overwrite it
  if (allow_sym && sym_env)
    for (int r = 0; r < n_rules; ++r) {
      const int t = rules[r].this_type;
      bool taken = false;
      for (int q = 0; q < r; ++q) taken |= ((R.sym_mask >> q) & 1u) && rules[q].this_type == t;
      if (!taken && R.mask[r] == (1u << t) && R.lo[r] == -R.hi[r]) R.sym_mask |= 1u << r;
    }
  Lt.A = std::max(1, bits_for((uint64_t)params->n_items));
  Lt.F = bits_for((uint64_t)n_files_total);
  Lt.BR = bits_for((uint64_t)max_per_type);
  Lt.WB = Lt.BR + Lt.A + Lt.F;
  Lt.amask = (1u << Lt.A) - 1u;
  if (Lt.WB > 31) {  // W_EMPTY (all ones) must stay above every word
    set_error("word layout %d rule + %d aid + %d file bits > 31: reduce files per call", Lt.BR, Lt.A, Lt.F);
    return OTTOHIP_ELIMIT;
  }
  return 0;
}

static ottohip_table* new_table(ottohip_ctx* ctx, int n_rules, int32_t n_items) {
  ottohip_table* T = new ottohip_table();
  T->device = ctx->device;
  T->n_rules = n_rules;
  T->n_items = n_items;
  T->ctx = ctx;
  memset(T->stats, 0, sizeof T->stats);
  return T;
}

// The multi-GPU row keys' owner map for (n_items, G), in the context workspace: a2l[aid] = the aid's index among
// the aids of its owner (aid order), l2a[obase[o] + i] = the inverse; *LB = bits of the largest owner's count.
static int owner_map(ottohip_ctx* ctx, int32_t n_items, int G, hipStream_t s, const uint32_t** a2l,
                     const uint32_t** l2a, const uint32_t** obase, int* LB) {
  uint32_t *da2l, *dl2a, *dob;
  OH_TRY(ctx->ws.get("om_a2l", (size_t)std::max(n_items, 1), &da2l));
  OH_TRY(ctx->ws.get("om_l2a", (size_t)std::max(n_items, 1), &dl2a));
  OH_TRY(ctx->ws.get("om_obase", (size_t)G + 1, &dob));
  if (ctx->om_items != n_items || ctx->om_parts != G) {
    std::vector<uint32_t> cnt(G + 1, 0), a2l_h(std::max(n_items, 1)), l2a_h(std::max(n_items, 1));
    for (int32_t a = 0; a < n_items; ++a) a2l_h[a] = cnt[owner_dev((uint32_t)a, (uint32_t)G)]++;
    uint32_t mx = 0;
    std::vector<uint32_t> ob(G + 1, 0);
    for (int o = 0; o < G; ++o) { mx = std::max(mx, cnt[o]); ob[o + 1] = ob[o] + cnt[o]; }
    for (int32_t a = 0; a < n_items; ++a) l2a_h[ob[owner_dev((uint32_t)a, (uint32_t)G)] + a2l_h[a]] = (uint32_t)a;
    OH_HIP(hipMemcpyAsync(da2l, a2l_h.data(), (size_t)n_items * 4, hipMemcpyHostToDevice, s));
    OH_HIP(hipMemcpyAsync(dl2a, l2a_h.data(), (size_t)n_items * 4, hipMemcpyHostToDevice, s));
    OH_HIP(hipMemcpyAsync(dob, ob.data(), (size_t)(G + 1) * 4, hipMemcpyHostToDevice, s));
    OH_HIP(hipStreamSynchronize(s));  // the host vectors go out of scope
    ctx->om_items = n_items;
    ctx->om_parts = G;
    ctx->om_lb = std::max(1, bits_for((uint64_t)mx));
  }
  *a2l = da2l; *l2a = dl2a; *obase = dob; *LB = ctx->om_lb;
  return 0;
}

// S1 prep, S2 count, S3 rows. n_parts > 1: owner-major rows, and (emit handle) owner bounds.
static int covis_front(ottohip_ctx* ctx, const ottohip_events* ev, const ottohip_covis_params* params,
                       const int32_t* file_ids, int n_parts, Front& F, hipStream_t s, ottohip_emit* EM = nullptr) {
  ++ctx->gen;
  const int64_t E = ev->n_events, Sn = ev->n_sessions;
  F.E = E; F.Sn = Sn;
  F.P = 0; F.Rn = 0;
  if (E == 0 || Sn == 0) return 0;
  Workspace& ws = ctx->ws;
  const Layout& Lt = F.Lt;
  const RulesDev& R = F.R;
  const int64_t NB = ceil_div(E, EV_BLOCK);
  F.NB = NB;
  int32_t* n_long;
  int* err;
  const int64_t long_cap = E / (LCAP + 1) + 1;
  OH_TRY(ws.get("first", (size_t)NB + 1, &F.first));
  OH_TRY(ws.get("fb", (size_t)ev->n_files + 1, &F.fb));
  OH_TRY(ws.get("fid", (size_t)ev->n_files, &F.fid));
  OH_TRY(ws.get("long_list", (size_t)long_cap, &F.long_list));
  OH_TRY(ws.get("n_long", 4, &n_long));
  OH_TRY(ws.get("err", 4, &err));
  std::vector<uint32_t> fid(ev->n_files);
  for (int f = 0; f < ev->n_files; ++f) fid[f] = file_ids ? (uint32_t)file_ids[f] : (uint32_t)f;
  OH_HIP(hipMemcpyAsync(F.fb, ev->file_session_bounds, (ev->n_files + 1) * sizeof(int64_t), hipMemcpyHostToDevice, s));
  OH_HIP(hipMemcpyAsync(F.fid, fid.data(), ev->n_files * sizeof(uint32_t), hipMemcpyHostToDevice, s));
  OH_HIP(hipMemsetAsync(n_long, 0, 4 * sizeof(int32_t), s));
  OH_HIP(hipMemsetAsync(err, 0, sizeof(int), s));
  OH_HIP(hipStreamSynchronize(s));  // fid is a stack vector
  const int64_t* off = ev->session_offsets;
  F.off = off;

  // ---- S1 prep + S2 count (fused; sessions longer than LCAP: separate per-session kernels)
  uint32_t *rk, *pos, *rk2, *pos2;
  OH_TRY(ws.get("ev", (size_t)E, &F.evp));
  OH_TRY(ws.get("cnt", (size_t)E, &F.cnt));
  OH_TRY(ws.get("rk", (size_t)E, &rk));
  OH_TRY(ws.get("pos", (size_t)E, &pos));
  OH_TRY(ws.get("rk2", (size_t)E, &rk2));
  OH_TRY(ws.get("pos2", (size_t)E, &pos2));
  // S3's fused row layout (one GPU, rows < 2^24): S2 writes the row keys with their pair counts in
  // the byte above the sorted key bits, and the sort generates the event positions itself
  static const bool rows_legacy = getenv("OTTOHIP_ROWS") && !strcmp(getenv("OTTOHIP_ROWS"), "legacy");
  const int cshift = (Lt.A + 2 + 7) / 8 * 8;  // first byte above the sorted key bits
  // n_parts > 1: the fused layout with owner-local aid indices when (owner, type, local index) and the invalid
  // key G << (LB + 2) fit below the count byte (OTTOHIP_OWNER_LOCAL=0: the 4-pass owner-key sort)
  const bool ol_env = !(getenv("OTTOHIP_OWNER_LOCAL") && !strcmp(getenv("OTTOHIP_OWNER_LOCAL"), "0"));  // per call
  const uint32_t *om_a2l = nullptr, *om_l2a = nullptr, *om_obase = nullptr;
  int om_lb = 0;
  bool owner_local = false;
  if (!rows_legacy && n_parts > 1 && ol_env && cshift + 8 <= 32 && 3ull * (uint64_t)params->n_items < (1ull << 24)) {
    OH_TRY(owner_map(ctx, params->n_items, n_parts, s, &om_a2l, &om_l2a, &om_obase, &om_lb));
    owner_local = ((uint64_t)n_parts << (om_lb + 2)) < (1ull << cshift);
  }
  const bool fused = !rows_legacy && (n_parts == 1 || owner_local) && cshift + 8 <= 32 &&
                     3ull * (uint64_t)params->n_items < (1ull << 24);
  uint32_t* pos_w = fused ? nullptr : pos;
  static const bool rows_atomic = getenv("OTTOHIP_ROWS") && !strcmp(getenv("OTTOHIP_ROWS"), "atomic");
  // grouped row entries (fused layout): one S3 sort entry per (session, type, aid) with pairs; OTTOHIP_GROUP=0: one per
  // event (read per call, A/B switch)
  const bool group = fused && !rows_atomic && !(getenv("OTTOHIP_GROUP") && !strcmp(getenv("OTTOHIP_GROUP"), "0"));
  F.link = nullptr;
  if (group) OH_TRY(ws.get("link", (size_t)E, &F.link));
  int ph = ctx->begin("prep_count", s, 9.0 * E + 8.0 * (Sn + 1) + 8.0 * E + 12.0 * E);
  k_block_first<<<grid_for(Sn + 1), 256, 0, s>>>(off, Sn, NB, F.first, F.long_list, n_long);
  k_prep_count<<<(unsigned)NB, 64, 0, s>>>(off, F.first, NB, ev->aid, ev->ts, ev->type, F.evp, params->n_items,
                                           params->dedup, err, R, Lt.A, F.cnt, rk, pos_w, fused ? cshift : 0, F.link);
  if (hipGetLastError() != hipSuccess) { set_error("k_prep_count launch failed"); return OTTOHIP_EHIP; }
  int32_t nl = 0;
  OH_TRY(d2h(&nl, n_long, 1, s));
  F.nl = nl;
  if (nl > 0) {
    std::vector<int32_t> ll(nl);
    OH_TRY(d2h(ll.data(), F.long_list, (size_t)nl, s));
    std::sort(ll.begin(), ll.end());
    OH_HIP(hipMemcpy(F.long_list, ll.data(), nl * sizeof(int32_t), hipMemcpyHostToDevice));
    std::vector<int64_t> loff(nl + 1);
    loff[0] = 0;
    for (int i = 0; i < nl; ++i) {
      int64_t ab[2];
      OH_HIP(hipMemcpy(ab, off + ll[i], 2 * sizeof(int64_t), hipMemcpyDeviceToHost));
      loff[i + 1] = loff[i] + (ab[1] - ab[0]);
    }
    OH_TRY(ws.get("long_scr", (size_t)(2 * loff[nl]), &F.lscr));
    OH_TRY(ws.get("long_pscr", (size_t)(3 * (loff[nl] + nl)), &F.lpscr));
    OH_TRY(ws.get("long_off", (size_t)(nl + 1), &F.d_loff));
    OH_HIP(hipMemcpy(F.d_loff, loff.data(), (nl + 1) * sizeof(int64_t), hipMemcpyHostToDevice));
    k_prep_long<<<nl, 64, 0, s>>>(off, F.long_list, F.d_loff, F.lscr, ev->aid, ev->ts, ev->type, F.evp,
                                  params->n_items, params->dedup, err);
    k_count_long<<<nl, 64, 0, s>>>(off, F.long_list, F.d_loff, F.lscr, F.lpscr, F.evp, R, Lt.A, F.cnt, rk, pos_w,
                                   fused ? cshift : 0, F.link);
    if (hipGetLastError() != hipSuccess) { set_error("long-session launch failed"); return OTTOHIP_EHIP; }
  }
  ctx->end(ph, s);

  // ---- S3 rows (aid-major transpose; owner-major first when n_parts > 1)
  ph = ctx->begin("rows", s, 0);
  if (rows_atomic && fused) {  // no sort: dense rows, per-event ranks by returning atomics (k_rows_atomic)
    const uint32_t INVa = 3u << Lt.A;
    const uint32_t kmask_a = Lt.A + 2 >= 32 ? ~0u : (1u << (Lt.A + 2)) - 1u;
    const int64_t nk = (int64_t)3 << Lt.A;  // dense (type, aid) keys
    uint32_t* dcnt;
    uint64_t *doff, *tot;
    OH_TRY(ws.get("ra_cnt", (size_t)(nk * RA_SUB), &dcnt));
    OH_TRY(ws.get("ra_off", (size_t)(nk * RA_SUB), &doff));
    OH_TRY(ws.get("tot", 4, &tot));
    OH_HIP(hipMemsetAsync(dcnt, 0, (size_t)(nk * RA_SUB) * 4, s));
    k_rows_atomic<<<grid_for(E, 256 * RA_PER), 256, 0, s>>>(rk, F.cnt, E, kmask_a, INVa, dcnt, pos);
    OH_TRY(exclusive_scan_u32(ctx, dcnt, doff, nk * RA_SUB, tot, s));
    uint64_t PP = 0;
    OH_TRY(d2h(&PP, tot, 1, s));
    int herr = 0;
    OH_TRY(d2h(&herr, err, 1, s));
    if (herr) { set_error("input out of range: aid outside [0, n_items) or type outside {0,1,2}"); return OTTOHIP_ERANGE; }
    F.P = PP;
    F.Rn = nk;
    OH_TRY(ws.get("row_key", (size_t)nk, &F.row_key));
    OH_TRY(ws.get("row_begin", (size_t)nk, &F.row_begin));
    k_rows_dense<<<grid_for(nk), 256, 0, s>>>(doff, nk, F.row_key, F.row_begin);
    F.poff = nullptr; F.poff32 = nullptr;
    if (F.P < (1ull << 32)) OH_TRY(ws.get("poff32", (size_t)E, &F.poff32));
    else OH_TRY(ws.get("poff", (size_t)E, &F.poff));
    k_rows_atomic_off<<<grid_for(E, 256 * RA_PER), 256, 0, s>>>(rk, E, kmask_a, INVa, doff, pos, F.poff32, F.poff);
    OH_HIP(hipGetLastError());
    ctx->end(ph, s);
    return 0;
  }
  uint32_t INV = 3u << Lt.A;
  int kbits = Lt.A + 2;
  uint32_t kmask = Lt.A + 2 >= 32 ? ~0u : (1u << (Lt.A + 2)) - 1u;
  if (owner_local) {
    const uint32_t INV2 = (uint32_t)n_parts << (om_lb + 2);
    k_owner_key_local<<<grid_for(E), 256, 0, s>>>(rk, E, INV, Lt.A, (uint32_t)n_parts, om_lb, INV2,
                                                 (1u << cshift) - 1u, om_a2l);
    INV = INV2;
    kbits = bits_for((uint64_t)INV2 + 1);
    kmask = (1u << cshift) - 1u;
  } else if (n_parts > 1) {
    const uint32_t INV2 = (uint32_t)n_parts << (Lt.A + 2);
    k_owner_key<<<grid_for(E), 256, 0, s>>>(rk, E, INV, Lt.A, (uint32_t)n_parts, INV2);
    INV = INV2;
    kbits = Lt.A + 2 + bits_for((uint64_t)n_parts + 1);
    if (kbits > 32) { set_error("row key with owner bits > 32 bits"); return OTTOHIP_ELIMIT; }
  }
  // fused layout: counts ride in the keys' spare bits (written by S2), one u64 scan carries word
  // offset and row index; the sort's first pass takes the event positions from its own indices
  uint32_t *rks = rk, *poss = pos;
  // fused layout: the sort's first pass drops the keys without a row entry (events without pairs; grouped: members),
  // the later passes and the row passes below run over the En kept entries
  int64_t En = E;
  const SortSkip skip{fused ? (1u << cshift) - 1u : 0u, INV, &En};
  OH_TRY(radix_sort_pairs(ctx, rks, poss, rk2, pos2, E, kbits, s, fused, fused ? &skip : nullptr));
  uint64_t* tot;
  OH_TRY(ws.get("tot", 4, &tot));
  if (fused) {
    // saturated count bytes are read back from the link array (grouped: the group's total) or the counts
    const uint32_t* csrc = F.link ? F.link : F.cnt;
    const int64_t nb = ceil_div(En, RT_TILE);
    uint64_t *bsum, *boff;
    OH_TRY(ws.get("rt_sums", (size_t)std::max<int64_t>(nb, 1), &bsum));
    OH_TRY(ws.get("rt_offs", (size_t)std::max<int64_t>(nb, 1), &boff));
    if (nb > 0) k_rows_sums<<<(unsigned)nb, RT_T, 0, s>>>(rks, poss, csrc, En, kmask, INV, cshift, bsum);
    OH_TRY(exclusive_scan_u64(ctx, bsum, boff, nb, tot, s));
    uint64_t X = 0;
    OH_TRY(d2h(&X, tot, 1, s));
    int herr = 0;
    OH_TRY(d2h(&herr, err, 1, s));
    if (herr) { set_error("input out of range: aid outside [0, n_items) or type outside {0,1,2}"); return OTTOHIP_ERANGE; }
    F.P = X >> 24;
    F.Rn = (int64_t)(X & 0xFFFFFFull);
    OH_TRY(ws.get("row_key", (size_t)std::max<int64_t>(F.Rn, 1), &F.row_key));
    OH_TRY(ws.get("row_begin", (size_t)std::max<int64_t>(F.Rn, 1), &F.row_begin));
    // word offsets below 2^32: u32 per event (the random scatter of one offset per event and the
    // emit's reads move half the bytes; measured rows 12.3 -> 11.1 ms at 220 M events)
    static const char* p32env = getenv("OTTOHIP_POFF32");  // A/B switch: 0 = u64 offsets
    F.poff = nullptr; F.poff32 = nullptr;
    if (F.P < (1ull << 32) && !(p32env && !strcmp(p32env, "0"))) {
      OH_TRY(ws.get("poff32", (size_t)E, &F.poff32));
      // the offsets leave the tile pass in sorted order (coalesced), one radix pass partitions the
      // (position, offset) pairs by the positions' top 8 bits, and the final scatter writes one
      // 1/256 slice of poff32 at a time (OTTOHIP_POFF_PART=0: the tile pass scatters directly)
      static const char* ppenv = getenv("OTTOHIP_POFF_PART");  // A/B switch
      if (!(ppenv && !strcmp(ppenv, "0")) && En > 4096) {
        uint32_t* rkA = rks == rk ? rk2 : rk;  // the sort's idle pair
        uint32_t* posA = poss == pos ? pos2 : pos;
        k_rows_tile<<<(unsigned)nb, RT_T, 0, s>>>(rks, poss, csrc, En, kmask, INV, cshift, boff, nullptr, F.poff32, 0u,
                                                  0xFFFFFFFFu, 1, F.row_key, F.row_begin, rkA);
        const uint64_t* dstart = nullptr;
        int ntl = 0;
        OH_TRY(radix_pass(ctx, poss, rkA, posA, rks, En, std::max(0, bits_for((uint64_t)E) - 8), s, &dstart, &ntl));
        // OTTOHIP_POFF_XCD=1: the XCD-aware scatter (A/B switch, off: 6.47 vs 6.85 GB written per build, slower)
        static const bool pxcd = getenv("OTTOHIP_POFF_XCD") && !strcmp(getenv("OTTOHIP_POFF_XCD"), "1");
        if (pxcd)
          k_poff_scatter_xcd<<<(unsigned)(8 * std::max(1, ctx->n_cu)), 256, 0, s>>>(posA, rks, En, dstart, ntl, F.poff32);
        else
          k_poff_scatter<<<grid_for(En), 256, 0, s>>>(posA, rks, En, F.poff32);
      } else if (nb > 0) {
        k_rows_tile<<<(unsigned)nb, RT_T, 0, s>>>(rks, poss, csrc, En, kmask, INV, cshift, boff, nullptr, F.poff32, 0u,
                                                  0xFFFFFFFFu, 1, F.row_key, F.row_begin);
      }
    } else {
      OH_TRY(ws.get("poff", (size_t)E, &F.poff));
      if (nb > 0)
        k_rows_tile<<<(unsigned)nb, RT_T, 0, s>>>(rks, poss, csrc, En, kmask, INV, cshift, boff, F.poff, nullptr, 0u, 0u,
                                                  1, F.row_key, F.row_begin);
    }
    // grouped row entries: every member's word offset from its rep's (the emit reads one offset per event)
    if (F.link) k_link_fix<<<grid_for(E, 256 * LF_PER), 256, 0, s>>>(F.link, E, F.poff32, F.poff);
    // owner-local keys back to (type, aid): the rows downstream (owner bounds, pieces, reduce) read those
    if (owner_local && F.Rn > 0)
      k_rows_decode<<<grid_for(F.Rn), 256, 0, s>>>(F.row_key, F.Rn, Lt.A, om_lb, om_obase, om_l2a);
    OH_HIP(hipGetLastError());
    ctx->end(ph, s);
    return 0;
  }
  uint32_t *c_sorted = (rks == rk) ? rk2 : rk, *row_flag = (poss == pos) ? pos2 : pos;  // reuse the idle pair
  k_gather_counts<<<grid_for(E), 256, 0, s>>>(rks, poss, F.cnt, E, INV, c_sorted, row_flag);
  uint64_t *woff, *row_idx;
  OH_TRY(ws.get("woff", (size_t)E, &woff));
  OH_TRY(ws.get("row_idx", (size_t)E, &row_idx));
  OH_TRY(exclusive_scan_u32(ctx, c_sorted, woff, E, tot, s));
  OH_TRY(exclusive_scan_u32(ctx, row_flag, row_idx, E, tot + 1, s));
  uint64_t PR[2];
  OH_TRY(d2h(PR, tot, 2, s));
  int herr = 0;
  OH_TRY(d2h(&herr, err, 1, s));
  if (herr) { set_error("input out of range: aid outside [0, n_items) or type outside {0,1,2}"); return OTTOHIP_ERANGE; }
  F.P = PR[0];
  F.Rn = (int64_t)PR[1];
  OH_TRY(ws.get("poff", (size_t)E, &F.poff));
  F.poff32 = nullptr;
  OH_TRY(ws.get("row_key", (size_t)std::max<int64_t>(F.Rn, 1), &F.row_key));
  OH_TRY(ws.get("row_begin", (size_t)std::max<int64_t>(F.Rn, 1), &F.row_begin));
  k_rows<<<grid_for(E), 256, 0, s>>>(rks, poss, E, INV, kmask, woff, row_flag, row_idx, F.poff, F.row_key,
                                     F.row_begin);
  ctx->end(ph, s);
  return 0;
}

// S4: words of every qualifying pair at its row's offsets
static int covis_emit_words(ottohip_ctx* ctx, const Front& F, const ottohip_events* ev, uint32_t* w0, hipStream_t s) {
  int ph = ctx->begin("emit", s, 8.0 * F.E + 12.0 * F.E + 4.0 * (double)F.P);
  static const int dbg0 = getenv("OTTOHIP_EMIT_DBG") ? atoi(getenv("OTTOHIP_EMIT_DBG")) : 0;  // profiling ablations
  const int dbg = dbg0;
  const bool guard = getenv("OTTOHIP_DEBUG") != nullptr;  // bounds checks of the emit record arrays
  int* eerr;
  OH_TRY(ctx->ws.get("emit_err", 4, &eerr));
  OH_HIP(hipMemsetAsync(eerr, 0, sizeof(int), s));
  // per-type task lists in pass 3 (OTTOHIP_EMIT_TASKS=0: every (rule, next type) of the wave in turn; read per call)
  const bool tasks = !(getenv("OTTOHIP_EMIT_TASKS") && !strcmp(getenv("OTTOHIP_EMIT_TASKS"), "0"));
  // two pairs per lane per flush round (OTTOHIP_EMIT_FLUSH2=0: one; read per call)
  const bool fl2 = !(getenv("OTTOHIP_EMIT_FLUSH2") && !strcmp(getenv("OTTOHIP_EMIT_FLUSH2"), "0"));
  auto ek = guard ? (tasks ? k_emit<true, true, true> : k_emit<true, false, true>)
                  : (tasks ? (fl2 ? k_emit<false, true, true> : k_emit<false, true, false>) : k_emit<false, false, true>);
  if (F.NB > 0)
    ek<<<(unsigned)F.NB, 64, 0, s>>>(F.off, F.first, F.NB, F.evp, F.R, F.Lt, F.fb, ev->n_files, F.fid, F.cnt,
                                         EvOff{F.poff, F.poff32, nullptr}, w0, eerr, dbg);
  if (F.nl > 0)
    k_emit_long<<<F.nl, 64, 0, s>>>(F.off, F.long_list, F.d_loff, F.lscr, F.lpscr, F.evp, F.R, F.Lt, F.fb,
                                     ev->n_files, F.fid, F.cnt, EvOff{F.poff, F.poff32, nullptr}, w0);
  if (hipGetLastError() != hipSuccess) { set_error("k_emit launch failed"); return OTTOHIP_EHIP; }
  ctx->end(ph, s);
  int herr = 0;
  OH_TRY(d2h(&herr, eerr, 1, s));
  if (herr & 8) { set_error("emit: record index outside the flush's records (err=%d)", herr); return OTTOHIP_EHIP; }
  if (herr) { set_error("emit: pairs written per event disagree with the count stage (err=%d)", herr); return OTTOHIP_EHIP; }
  return 0;
}

// S5: words grouped by row -> table rows (count, count_ge2) and per-rule statistics
// ottohip_file_opts -> the kernels' FileOpts (device histogram / drop counter from the workspace)
static int file_opts_setup(ottohip_ctx* ctx, const ottohip_file_opts* o, int n_rules, const RulesDev& R,
                           FileOpts& fo, hipStream_t s) {
  if (o->rule < 0 || o->rule >= n_rules) { set_error("file_opts: rule %d outside the call's rules", o->rule); return OTTOHIP_EINVAL; }
  const bool want_hist = o->file_rows || o->file_rows_ge2;
  if (want_hist && (o->n_files < 1 || o->n_files > FO_MAXF)) {
    set_error("file_opts: n_files=%d outside [1, %d]", o->n_files, FO_MAXF); return OTTOHIP_ELIMIT;
  }
  memset(&fo, 0, sizeof fo);
  for (int t = 0; t < 3; ++t)
    for (int q = 0; q < R.n_of_type[t]; ++q)
      if (R.rule_of_type[t][q] == o->rule) { fo.type = t; fo.q = (uint32_t)q; }
  fo.sym = (uint32_t)((R.sym_mask >> o->rule) & 1u);
  if (fo.sym && (o->lo_file >= 0 || o->hi_file >= 0)) { set_error("file_opts: key cuts on a symmetric table"); return OTTOHIP_EINVAL; }
  fo.lo_file = o->lo_file < 0 ? 0xFFFFFFFFu : (uint32_t)o->lo_file;
  fo.hi_file = o->hi_file < 0 ? 0xFFFFFFFFu : (uint32_t)o->hi_file;
  fo.cuts = (o->lo_file >= 0 || o->hi_file >= 0) ? 1u : 0u;
  fo.lo_key = o->lo_key;
  fo.hi_key = o->hi_key;
  OH_TRY(ctx->ws.get("fo_dropped", 1, &fo.dropped));
  OH_HIP(hipMemsetAsync(fo.dropped, 0, 8, s));
  if (getenv("OTTOHIP_DEBUG")) {
    OH_TRY(ctx->ws.get("fo_dbg", 8, &fo.dbg));
    OH_HIP(hipMemsetAsync(fo.dbg, 0, 64, s));
  }
  if (want_hist) {
    fo.nf = (uint32_t)o->n_files;
    OH_TRY(ctx->ws.get("fo_hist", (size_t)fo.nf, &fo.hist));
    OH_HIP(hipMemsetAsync(fo.hist, 0, (size_t)fo.nf * 8, s));
  }
  return 0;
}

static int file_opts_finish(const ottohip_file_opts* o, const FileOpts& fo, hipStream_t s) {
  if (!fo.hist) return 0;
  std::vector<unsigned long long> h(fo.nf);
  OH_TRY(d2h(h.data(), fo.hist, h.size(), s));
  for (uint32_t f = 0; f < fo.nf; ++f) {
    if (o->file_rows) o->file_rows[f] = (int64_t)(h[f] & 0xFFFFFFFFull);
    if (o->file_rows_ge2) o->file_rows_ge2[f] = (int64_t)(h[f] >> 32);
  }
  return 0;
}

static int covis_reduce(ottohip_ctx* ctx, uint32_t* w0, uint32_t* w1, uint64_t P, const uint64_t* row_begin,
                        const uint32_t* row_key, int64_t Rn, const RulesDev& R, const Layout& Lt, int n_rules,
                        ottohip_table* T, hipStream_t s, const ottohip_file_opts* fopts = nullptr,
                        const FileOpts* fo_parts = nullptr, uint32_t* w2 = nullptr, uint64_t row_base = 0) {
  // w2: a third word buffer for the split levels >= 1 (level 0 splits w0 -> w1, then w1 <-> w2), so w0 keeps the
  // emitted words (ottohip_file_opts.keep_words); row_base: row_begin values are offsets + row_base (a row range)
  Workspace& ws = ctx->ws;
  int rc;
  int* err;
  OH_TRY(ws.get("err", 4, &err));
  FileOpts fo;
  memset(&fo, 0, sizeof fo);
  if (fopts) OH_TRY(file_opts_setup(ctx, fopts, n_rules, R, fo, s));
  if (fo_parts) {  // part mode: tables already on the device; a drop counter for the conservation check
    fo = *fo_parts;
    OH_TRY(ctx->ws.get("fo_dropped", 1, &fo.dropped));
    OH_HIP(hipMemsetAsync(fo.dropped, 0, 8, s));
  }
  const bool FOon = fopts != nullptr || fo_parts != nullptr;
  // per-file rows only (no key cuts, no parts): the register sorts keep their occupancy (k_agg_sort<M, 2>)
  const bool FOhist = FOon && !fo.cuts && !fo.parts && fo.hist != nullptr;
  const bool FOmir = FOon && fo.parts && fo.mirror_off != 0;  // part mode with explicit mirror rows
  // symmetric rules store one row per unordered pair; the readers produce the mirrors (T->sym_mask)
  // part mode with explicit mirror rows: slots [P, 2P) hold the mirror of the row at slot - P
  const uint64_t n_slots = (fo_parts && fo_parts->mirror_off) ? 2 * P : P;
  if (ctx->spare.cap >= n_slots) {
    T->b = ctx->spare;
    ctx->spare = TableBufs();
  } else {
    const double t0 = alloc_log_begin();
    (void)hipDeviceSynchronize();
    ctx->spare.release();
    OH_TRY(T->b.alloc(n_slots));
    alloc_log_end(t0, "table", "slots", (size_t)n_slots * 17);
  }
  unsigned long long *stats, *lcount;
  OH_TRY(ws.get("stats", (size_t)STAT_STRIPES * STAT_STRIDE, &stats));
  OH_TRY(ws.get("lcount", 8, &lcount));
  hipMemsetAsync(stats, 0, (size_t)STAT_STRIPES * STAT_STRIDE * 8, s);
  hipMemsetAsync(err, 0, sizeof(int), s);
  // rows are written at their task's word offsets; each leaf task marks the rest of its range
  // (rule 0xFF), so the slots need no fill (a debug ablation drops the sort kernels' stores)
  if (getenv("OTTOHIP_REDUCE_DBG")) hipMemsetAsync(T->b.rule, 0xFF, n_slots, s);
  OutRows O;
  O.rule = T->b.rule; O.aid = T->b.aid; O.aid_next = T->b.aid_next; O.count = T->b.count; O.count_ge2 = T->b.count_ge2;
  O.cap = n_slots; O.stats = stats;
  T->sym_mask = R.sym_mask;
  // profiling ablation: OTTOHIP_REDUCE_DBG=1 drops the register-sort kernels' row stores
  static const int rdbg = getenv("OTTOHIP_REDUCE_DBG") ? atoi(getenv("OTTOHIP_REDUCE_DBG")) : 0;
  OutRows Osort = O;
  if (rdbg & 1) Osort.cap = 0;
  int herr = 0;

  static const int split_mean = getenv("OTTOHIP_SPLIT_MEAN") ? atoi(getenv("OTTOHIP_SPLIT_MEAN")) : SPLIT_MEAN;
  if (split_mean != SPLIT_MEAN) {
    const uint32_t v = (uint32_t)std::max(64, split_mean);
    OH_HIP(hipMemcpyToSymbolAsync(HIP_SYMBOL(c_split_mean), &v, sizeof v, 0, hipMemcpyHostToDevice, s));
    OH_HIP(hipStreamSynchronize(s));
  }
  static const char* runs_env = getenv("OTTOHIP_SPLIT_RUNS");  // A/B switch
  if (runs_env && !strcmp(runs_env, "1")) {
    const uint32_t v = 1;
    OH_HIP(hipMemcpyToSymbolAsync(HIP_SYMBOL(c_split_runs), &v, sizeof v, 0, hipMemcpyHostToDevice, s));
    OH_HIP(hipStreamSynchronize(s));
  }
  static const char* fuse_env = getenv("OTTOHIP_SPLIT_FUSE");  // A/B switch
  if (fuse_env && !strcmp(fuse_env, "0")) {
    const uint32_t v = 0;
    OH_HIP(hipMemcpyToSymbolAsync(HIP_SYMBOL(c_split_fuse), &v, sizeof v, 0, hipMemcpyHostToDevice, s));
    OH_HIP(hipStreamSynchronize(s));
  }
  // LDS leaf (k_agg_lds) for rows and split buckets of (SORT_MAX, LDS_CAP] words, fed by splits of
  // LDS_SPLIT_MEAN-word buckets (OTTOHIP_LDS_LEAF=1, read per call; default: register sorts of
  // SPLIT_MEAN-word buckets only)
  const bool lds_leaf = getenv("OTTOHIP_LDS_LEAF") && !strcmp(getenv("OTTOHIP_LDS_LEAF"), "1");
  {
    static int8_t lds_state[64] = {};  // per device (the constants live in each device's code object): 0 unset, 1 off, 2 on
    int8_t& st = lds_state[ctx->device & 63];
    if (st != (lds_leaf ? 2 : 1)) {
      const uint32_t on = lds_leaf ? 1u : 0u;
      OH_HIP(hipMemcpyToSymbolAsync(HIP_SYMBOL(c_lds_leaf), &on, sizeof on, 0, hipMemcpyHostToDevice, s));
      if (split_mean == SPLIT_MEAN) {
        const uint32_t v = lds_leaf ? (uint32_t)LDS_SPLIT_MEAN : (uint32_t)SPLIT_MEAN;
        OH_HIP(hipMemcpyToSymbolAsync(HIP_SYMBOL(c_split_mean), &v, sizeof v, 0, hipMemcpyHostToDevice, s));
      }
      OH_HIP(hipStreamSynchronize(s));
      st = lds_leaf ? 2 : 1;
    }
  }
  static const int hash_prio = getenv("OTTOHIP_HASH_PRIO") ? atoi(getenv("OTTOHIP_HASH_PRIO")) : 0;  // A/B switch
  if (hash_prio) {
    const uint32_t v = (uint32_t)hash_prio;
    OH_HIP(hipMemcpyToSymbolAsync(HIP_SYMBOL(c_hash_prio), &v, sizeof v, 0, hipMemcpyHostToDevice, s));
    OH_HIP(hipStreamSynchronize(s));
  }
  int ph = ctx->begin("reduce", s, 4.0 * (double)P);
  // level 0 task lists come from the rows
  uint64_t cap0 = (uint64_t)std::max<int64_t>(Rn, 1);
  TaskLists TL;
  TL.n = lcount;
  // task lists double-buffered by level parity: level l's sorts (aux stream) may still read theirs
  // while level l + 1's classify fills the other set
  const uint64_t split_extra = P / 512 + 64;
  auto get_lists = [&](uint64_t capl, const char* split_name, int parity) -> int {
    static const char* names[2][N_SORT] = {{"t_sort0", "t_sort1", "t_sort2", "t_sort3", "t_sort4"},
                                           {"t_sort0b", "t_sort1b", "t_sort2b", "t_sort3b", "t_sort4b"}};
    for (int c = 0; c < N_SORT; ++c)
      if (int r = ws.get(names[parity][c], capl * sizeof(Task), reinterpret_cast<void**>(&TL.sort[c]))) return r;
    if (int r = ws.get(parity ? "t_hashb" : "t_hash", capl * sizeof(Task), reinterpret_cast<void**>(&TL.hash))) return r;
    if (int r = ws.get(parity ? "t_ldsb" : "t_lds", capl * sizeof(Task), reinterpret_cast<void**>(&TL.lds))) return r;
    // the split list also takes the LDS leaf's hot segments (> 512 words each)
    if (int r = ws.get(split_name, (capl + split_extra) * sizeof(Task), reinterpret_cast<void**>(&TL.split))) return r;
    TL.cap = capl;
    return 0;
  };
  if ((rc = get_lists(cap0, "t_splitA", 0))) return rc;
  hipMemsetAsync(lcount, 0, 8 * 8, s);
  k_classify_rows<<<grid_for(Rn), 256, 0, s>>>(row_begin, Rn, P, Lt.WB, TL, err, row_base);
  const int agg_grid = ctx->n_cu * 8;
  static const bool overlap = !(getenv("OTTOHIP_REDUCE_OVERLAP") && !strcmp(getenv("OTTOHIP_REDUCE_OVERLAP"), "0"));
  hipStream_t s2 = nullptr;
  if (overlap) {
    OH_TRY(ctx->aux_stream());
    s2 = ctx->aux;
  }
  bool srcA = true;
  bool drained = false;
  const bool dbg = getenv("OTTOHIP_DEBUG") != nullptr;
  if (dbg) fprintf(stderr, "[ottohip] P=%llu rows=%lld\n", (unsigned long long)P, (long long)Rn);
  uint32_t* wcur0 = w0;  // the word buffer of tasks with buf 0 at this level (w2 from level 1 on, if given)
  // Split pipelining (OTTOHIP_SPLIT_PIPE=1, read per call; off by default: step 57.0-57.3 vs 57.0-57.1 ms same box,
  // the early leaves and the second half's scatter contend for the same CUs): a large split scatters and classifies its tasks in
  // two halves; the next level's leaves of the first half's sub-buckets (hash, then register sorts, on the aux
  // stream) start while the second half is scattered on the main stream. done[c]: tasks of list c of the level
  // whose leaves were launched that way; hash_early: its hash leaves run on the aux stream (ev_hash).
  const char* pipe_env = getenv("OTTOHIP_SPLIT_PIPE");
  const bool pipe = s2 != nullptr && !lds_leaf && !dbg && getenv("OTTOHIP_HASH_PROF") == nullptr &&
                    (pipe_env && atoi(pipe_env) == 1);
  // splits of >= 2048 chunks (32 M words) are pipelined (OTTOHIP_SPLIT_PIPE_MIN: another bound, for tests)
  const uint64_t PIPE_MIN_CHUNKS = getenv("OTTOHIP_SPLIT_PIPE_MIN") ? (uint64_t)atoll(getenv("OTTOHIP_SPLIT_PIPE_MIN")) : 2048;
  unsigned long long done[N_LISTS] = {};
  bool hash_early = false;
  // leaves of tasks [lo[c], hi[c]) of the sort classes / [lo[N_SORT], hi[N_SORT]) of the hash list, buffer wb0 for
  // buf 0
  auto launch_hash_range = [&](uint64_t lo, uint64_t hi, uint32_t* wb0, hipStream_t st) {
    if (hi <= lo) return;
    const int64_t nh = (int64_t)(hi - lo);
    const Task* th = TL.hash + lo;
    const unsigned hg = (unsigned)std::min<int64_t>(nh, (int64_t)agg_grid);
    if (FOhist)
      k_agg_hash<2><<<hg, AGG_T, 0, st>>>(th, nh, wb0, w1, row_key, R, Lt, n_rules, O, TL.split, lcount + N_SORT + 1, fo);
    else if (FOmir)
      k_agg_hash<3><<<hg, AGG_T, 0, st>>>(th, nh, wb0, w1, row_key, R, Lt, n_rules, O, TL.split, lcount + N_SORT + 1, fo);
    else if (FOon)
      k_agg_hash<1><<<hg, AGG_T, 0, st>>>(th, nh, wb0, w1, row_key, R, Lt, n_rules, O, TL.split, lcount + N_SORT + 1, fo);
    else
      k_agg_hash<<<hg, AGG_T, 0, st>>>(th, nh, wb0, w1, row_key, R, Lt, n_rules, O, TL.split, lcount + N_SORT + 1, fo);
  };
  auto launch_sorts = [&](const unsigned long long* lo, const unsigned long long* hi, uint32_t* wb0, hipStream_t st) {
    const unsigned sgrid = (unsigned)ctx->n_cu * 32;
#define OH_SORT(c, M)                                                                                          \
    if (hi[c] > lo[c]) {                                                                                       \
      const int64_t n_ = (int64_t)(hi[c] - lo[c]);                                                             \
      const Task* t_ = TL.sort[c] + lo[c];                                                                     \
      const unsigned g_ = (unsigned)std::min<uint64_t>(ceil_div(n_, 4), sgrid);                                \
      if (FOhist)                                                                                              \
        k_agg_sort<M, 2><<<g_, 256, (size_t)fo.nf * 8, st>>>(t_, n_, wb0, w1, row_key, R, Lt, n_rules, Osort, fo); \
      else if (FOmir)                                                                                          \
        k_agg_sort<M, 3><<<g_, 256, 0, st>>>(t_, n_, wb0, w1, row_key, R, Lt, n_rules, Osort, fo);             \
      else if (FOon)                                                                                           \
        k_agg_sort<M, 1><<<g_, 256, 0, st>>>(t_, n_, wb0, w1, row_key, R, Lt, n_rules, Osort, fo);             \
      else                                                                                                     \
        k_agg_sort<M><<<g_, 256, 0, st>>>(t_, n_, wb0, w1, row_key, R, Lt, n_rules, Osort, fo);                \
    }
    OH_SORT(0, 1) OH_SORT(1, 2) OH_SORT(2, 4) OH_SORT(3, 8) OH_SORT(4, 16)
#undef OH_SORT
  };
  for (int level = 0; level < 40; ++level) {
    wcur0 = (level == 0 || !w2) ? w0 : w2;
    unsigned long long nlist[N_LISTS];
    if ((rc = d2h(nlist, lcount, N_LISTS, s))) return rc;
    if ((rc = d2h(&herr, err, 1, s))) return rc;
    if (herr) { set_error("task list overflow / row too large (err=%d)", herr); return OTTOHIP_ELIMIT; }
    if (dbg) {
      fprintf(stderr, "[ottohip] level %d: sort %llu/%llu/%llu/%llu/%llu hash %llu split %llu lds %llu\n", level, nlist[0],
              nlist[1], nlist[2], nlist[3], nlist[4], nlist[N_SORT], nlist[N_SORT + 1], nlist[N_SORT + 2]);
      Task* lists[N_LISTS] = {TL.sort[0], TL.sort[1], TL.sort[2], TL.sort[3], TL.sort[4], TL.hash, TL.split, TL.lds};
      fprintf(stderr, "[ottohip] level %d words:", level);
      for (int c = 0; c < N_LISTS; ++c) {
        std::vector<Task> tv(nlist[c]);
        if (nlist[c]) (void)d2h(tv.data(), lists[c], nlist[c], s);
        unsigned long long sw = 0, mx = 0;
        for (auto& t : tv) { sw += t.len; mx = std::max<unsigned long long>(mx, t.len); }
        fprintf(stderr, " %llu(max %llu)", sw, mx);
        if (c == N_SORT + 1 && !tv.empty()) {  // split tasks: words by log2(len) class
          unsigned long long hw[40] = {}, hn[40] = {};
          for (auto& t : tv) { const int b = 63 - __builtin_clzll((unsigned long long)t.len | 1ull); hw[b] += t.len; ++hn[b]; }
          fprintf(stderr, " [split by log2 len:");
          for (int b = 0; b < 40; ++b)
            if (hn[b]) fprintf(stderr, " 2^%d:%llu tasks/%llu words", b, hn[b], hw[b]);
          fprintf(stderr, "]");
        }
      }
      fprintf(stderr, "\n");
    }
    // the register-sort tasks of this level run on the aux stream, beside this level's hash and
    // split on s (VALU-bound sorts next to the LDS/HBM-bound split); their task lists are only
    // rewritten by the next level's classify, which waits for them (ev_join)
    hipStream_t ss = s2 ? s2 : s;
    if (s2) { OH_HIP(hipEventRecord(ctx->ev_fork, s)); OH_HIP(hipStreamWaitEvent(s2, ctx->ev_fork, 0)); }
    // the level's LDS-hash leaves are queued before its register sorts, so their few long-running
    // blocks take CU slots before the sorts' many short ones (step -0.5 ms same box; OTTOHIP_HASH_FIRST=0:
    // sorts first)
    static const bool hash_first = !(getenv("OTTOHIP_HASH_FIRST") && !strcmp(getenv("OTTOHIP_HASH_FIRST"), "0"));
    const bool hf = hash_first && nlist[N_SORT] > done[N_SORT];
    auto launch_hash = [&]() { launch_hash_range(done[N_SORT], nlist[N_SORT], wcur0, s); };
    if (hf) launch_hash();
    launch_sorts(done, nlist, wcur0, ss);
    if (s2) OH_HIP(hipEventRecord(ctx->ev_join[level & 1], s2));
    if (nlist[N_SORT + 2]) {  // LDS leaves (hot segments are appended to the split list)
      const unsigned lg = (unsigned)std::min<uint64_t>(nlist[N_SORT + 2], (uint64_t)ctx->n_cu * 4);
      if (FOon)
        k_agg_lds<true><<<lg, LDS_T, 0, s>>>(TL.lds, (int64_t)nlist[N_SORT + 2], wcur0, w1, row_key, R, Lt, O, TL.split,
                                             lcount + N_SORT + 1, TL.cap + split_extra, err, fo);
      else
        k_agg_lds<<<lg, LDS_T, 0, s>>>(TL.lds, (int64_t)nlist[N_SORT + 2], wcur0, w1, row_key, R, Lt, O, TL.split,
                                       lcount + N_SORT + 1, TL.cap + split_extra, err, fo);
    }
    if (nlist[N_SORT] > done[N_SORT]) {  // tasks that overflow the LDS table are appended to the split list
      static const bool hprof = getenv("OTTOHIP_HASH_PROF") != nullptr && !hash_first;  // per-task profile (debugging aid)
      if (hprof) {
        if ((rc = ws.get("hash_prof", (size_t)(2 * nlist[N_SORT]), &fo.prof))) return rc;
        OH_HIP(hipMemsetAsync(fo.prof, 0, 16 * nlist[N_SORT], s));
      }
      if (!hf) launch_hash();
      if (hprof) {
        std::vector<unsigned long long> pv(2 * nlist[N_SORT]);
        if ((rc = d2h(pv.data(), fo.prof, pv.size(), s))) return rc;
        std::vector<size_t> ord(nlist[N_SORT]);
        for (size_t i = 0; i < ord.size(); ++i) ord[i] = i;
        auto tk = [&](size_t i) { return pv[2 * i + 1] & ~(1ull << 63); };
        std::sort(ord.begin(), ord.end(), [&](size_t a, size_t b) { return tk(a) > tk(b); });
        unsigned long long tsum = 0, wsum = 0;
        for (size_t i = 0; i < ord.size(); ++i) { tsum += tk(i); wsum += (uint32_t)pv[2 * i]; }
        fprintf(stderr, "[ottohip] hash level %d: %zu tasks, %llu words, %.3f ms summed task time; slowest:", level,
                ord.size(), wsum, tsum / 1e5);
        for (size_t i = 0; i < ord.size() && i < 10; ++i)
          fprintf(stderr, " [len %u rows %u %.3f ms%s]", (uint32_t)pv[2 * ord[i]], (uint32_t)(pv[2 * ord[i]] >> 32),
                  tk(ord[i]) / 1e5, (pv[2 * ord[i] + 1] >> 63) ? " full" : "");
        fprintf(stderr, "\n");
        fo.prof = nullptr;
      }
    }
    if (hash_early) OH_HIP(hipStreamWaitEvent(s, ctx->ev_hash, 0));  // the early hash leaves' overflow tasks
    if (nlist[N_SORT] || nlist[N_SORT + 2])
      if ((rc = d2h(nlist, lcount, N_LISTS, s))) return rc;
    hash_early = false;
    for (int c = 0; c < N_LISTS; ++c) done[c] = 0;
    const int64_t ns = (int64_t)nlist[N_SORT + 1];
    if (dbg) fprintf(stderr, "[ottohip] level %d: split after hash overflow %lld\n", level, (long long)ns);
    if (ns == 0) {
      if (s2) OH_HIP(hipStreamWaitEvent(s, ctx->ev_join[level & 1], 0));
      drained = true;
      break;
    }
    if ((uint64_t)ns > TL.cap) { set_error("split list overflow"); return OTTOHIP_ELIMIT; }
    Task* cur_split = TL.split;
    // chunk / digit / count-matrix bases
    uint32_t *nch, *ndg, *nen;
    uint64_t *chb, *dgb, *mtb, *tot2;
    if ((rc = ws.get("sp_nch", (size_t)ns, &nch)) || (rc = ws.get("sp_ndg", (size_t)ns, &ndg)) ||
        (rc = ws.get("sp_nen", (size_t)ns, &nen)) || (rc = ws.get("sp_chb", (size_t)ns + 1, &chb)) ||
        (rc = ws.get("sp_dgb", (size_t)ns + 1, &dgb)) || (rc = ws.get("sp_mtb", (size_t)ns + 1, &mtb)) ||
        (rc = ws.get("sp_tot", 6, &tot2)))
      return rc;
    k_split_prepare<<<grid_for(ns), 256, 0, s>>>(cur_split, ns, nch, ndg, nen);
    if ((rc = exclusive_scan_u32(ctx, nch, chb, ns, tot2, s)) || (rc = exclusive_scan_u32(ctx, ndg, dgb, ns, tot2 + 1, s)) ||
        (rc = exclusive_scan_u32(ctx, nen, mtb, ns, tot2 + 2, s)))
      return rc;
    if (pipe) k_split_half<<<1, 64, 0, s>>>(chb, dgb, ns, tot2, tot2 + 3);  // (task, chunk, digit) of the halves' border
    uint64_t tt[6] = {0, 0, 0, 0, 0, 0};
    if ((rc = d2h(tt, tot2, pipe ? 6 : 3, s))) return rc;
    const int64_t nchunks = (int64_t)tt[0], ndig = (int64_t)tt[1], nent = (int64_t)tt[2];
    // pipelined when the split is large and the border falls strictly inside it
    const bool piped = pipe && (uint64_t)nchunks >= PIPE_MIN_CHUNKS && tt[3] > 0 && (int64_t)tt[3] < ns &&
                       tt[4] > 0 && (int64_t)tt[4] < nchunks && tt[5] > 0 && (int64_t)tt[5] < ndig;
    const uint32_t cA = piped ? (uint32_t)tt[4] : (uint32_t)nchunks;
    const int64_t dA = piped ? (int64_t)tt[5] : ndig;
    uint32_t *hmat, *ctask;
    uint64_t* hoff;
    if ((rc = ws.get("sp_hmat", (size_t)nent, &hmat)) || (rc = ws.get("sp_hoff", (size_t)nent + 1, &hoff)) ||
        (rc = ws.get("sp_ctask", (size_t)nchunks, &ctask)))
      return rc;
    k_split_chunk_task<<<grid_for(ns), 256, 0, s>>>(chb, nch, ns, ctask);
    k_split_hist<<<(unsigned)nchunks, SPLIT_T, 0, s>>>(cur_split, ns, chb, ctask, mtb, wcur0, w1, Lt.F, hmat);
    if ((rc = exclusive_scan_u32(ctx, hmat, hoff, nent, hoff + nent, s))) return rc;
    static const int sub = getenv("OTTOHIP_SPLIT_SUB") ? atoi(getenv("OTTOHIP_SPLIT_SUB")) : 4096;  // A/B switch
    auto scatter = [&](uint32_t c0, uint32_t c1) {
      if (c1 <= c0) return;
      if (sub == 8192)
        k_split_scatter<8192><<<c1 - c0, SPLIT_T, 0, s>>>(cur_split, ns, chb, ctask, mtb, hoff, wcur0, w1, Lt.F, hmat, c0);
      else
        k_split_scatter<4096><<<c1 - c0, SPLIT_T, 0, s>>>(cur_split, ns, chb, ctask, mtb, hoff, wcur0, w1, Lt.F, hmat, c0);
    };
    scatter(0, cA);
    // next lists (a sub-bucket is one task in exactly one list: ndig bounds every list): the other
    // parity's set, last read by the sorts of level - 1
    if (s2 && level >= 1) OH_HIP(hipStreamWaitEvent(s, ctx->ev_join[(level + 1) & 1], 0));
    const uint64_t capn = (uint64_t)ndig;
    if ((rc = get_lists(std::max(cap0, capn), srcA ? "t_splitB" : "t_splitA", (level + 1) & 1))) return rc;
    hipMemsetAsync(lcount, 0, 8 * 8, s);
    k_split_classify<<<grid_for(dA), 256, 0, s>>>(cur_split, ns, dgb, mtb, hoff, dA, TL, err, hmat, 0);
    if (piped) {
      if (getenv("OTTOHIP_SPLIT_PIPE_LOG")) fprintf(stderr, "[ottohip] level %d split pipelined at chunk %u of %lld\n", level, cA, (long long)nchunks);
      // the first half's sub-buckets are classified: its next-level leaves start on the aux stream (hash first,
      // then the register sorts) while the second half is scattered and classified here
      OH_HIP(hipEventRecord(ctx->ev_half, s));
      scatter(cA, (uint32_t)nchunks);
      if (ndig > dA)
        k_split_classify<<<grid_for(ndig - dA), 256, 0, s>>>(cur_split, ns, dgb, mtb, hoff, ndig, TL, err, hmat, dA);
      OH_HIP(hipStreamWaitEvent(ctx->aux2, ctx->ev_half, 0));
      unsigned long long nA[N_LISTS];
      if ((rc = d2h(nA, lcount, N_LISTS, ctx->aux2))) return rc;
      OH_HIP(hipStreamWaitEvent(s2, ctx->ev_half, 0));
      uint32_t* wb0 = w2 ? w2 : w0;  // the next level's buffer of buf-0 tasks
      if (nA[N_SORT]) {
        launch_hash_range(0, nA[N_SORT], wb0, s2);
        OH_HIP(hipEventRecord(ctx->ev_hash, s2));
        hash_early = true;
      }
      const unsigned long long zero[N_LISTS] = {};
      launch_sorts(zero, nA, wb0, s2);
      for (int c = 0; c <= N_SORT; ++c) done[c] = nA[c];
    }
    srcA = !srcA;
    if (hipGetLastError() != hipSuccess) { set_error("split launch failed"); return OTTOHIP_EHIP; }
  }
  ctx->end(ph, s);
  if (!drained) { set_error("reduce: split levels did not converge"); return OTTOHIP_ELIMIT; }
  std::vector<unsigned long long> stv((size_t)STAT_STRIPES * STAT_STRIDE);
  if ((rc = d2h(stv.data(), stats, stv.size(), s))) return rc;
  unsigned long long st[STAT_STRIDE] = {};
  for (int k = 0; k < STAT_STRIPES; ++k)
    for (int j = 0; j < STAT_STRIDE; ++j) st[j] += stv[(size_t)k * STAT_STRIDE + j];
  if (hipGetLastError() != hipSuccess) { set_error("reduce failed"); return OTTOHIP_EHIP; }
  unsigned long long U = 0, dropped = 0;
  for (int r = 0; r < n_rules; ++r) U += st[r * 4 + 0];
  const unsigned long long sum_pairs = st[STAT_RAW + 1], raw_rows = st[STAT_RAW];  // stored rows / pairs
  if (FOon) {
    if ((rc = d2h(&dropped, fo.dropped, 1, s))) return rc;
    if (fo.dbg) {
      unsigned long long dv[8];
      if ((rc = d2h(dv, fo.dbg, 8, s))) return rc;
      fprintf(stderr, "[ottohip] file opts: hash dropped %llu kept %llu (loaded %llu inserted %llu), sort dropped %llu kept %llu\n",
              dv[0], dv[1], dv[4], dv[5], dv[2], dv[3]);
    }
    if ((rc = file_opts_finish(fopts, fo, s))) return rc;
  }
  T->n_rows = (int64_t)U;
  T->n_slots = (int64_t)n_slots;
  if (sum_pairs + dropped != P || raw_rows > P) {  // conservation: every emitted pair is counted (or cut) exactly once
    set_error("reduce: %llu pairs counted + %llu cut of %llu emitted (rows %llu)", sum_pairs, dropped,
              (unsigned long long)P, raw_rows);
    static const bool warn_only = getenv("OTTOHIP_CONSERVATION_WARN") != nullptr;  // debugging aid
    if (!warn_only) return OTTOHIP_EHIP;
    fprintf(stderr, "[ottohip] WARNING %s\n", ottohip_last_error());
  }
  for (int r = 0; r < n_rules; ++r) {
    T->stats[r].n_rows = (int64_t)st[r * 4 + 0];
    T->stats[r].n_pairs = (int64_t)st[r * 4 + 1];
    T->stats[r].file_rows = (int64_t)st[r * 4 + 2];
    T->stats[r].file_rows_ge2 = (int64_t)st[r * 4 + 3];
  }
  return 0;
}

extern "C" {

const char* ottohip_last_error(void) { return ottohip::g_err; }

int ottohip_ctx_create(int device, ottohip_ctx** out) {
  if (!out) { set_error("ottohip_ctx_create: out is NULL"); return OTTOHIP_EINVAL; }
  OH_HIP(hipSetDevice(device));
  ottohip_ctx* c = new ottohip_ctx();
  c->device = device;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess) c->n_cu = prop.multiProcessorCount;
  if (hipHostMalloc(reinterpret_cast<void**>(&c->pinned), 64 * sizeof(uint64_t)) != hipSuccess) c->pinned = nullptr;
  *out = c;
  return 0;
}

void ottohip_ctx_destroy(ottohip_ctx* ctx) {
  if (!ctx) return;
  hipSetDevice(ctx->device);
  hipDeviceSynchronize();
  ctx->ws.release();
  ctx->spare.release();
  dev_trim();
  if (ctx->aux) {
    hipStreamDestroy(ctx->aux);
    if (ctx->aux2) hipStreamDestroy(ctx->aux2);
    if (ctx->ev_half) hipEventDestroy(ctx->ev_half);
    if (ctx->ev_hash) hipEventDestroy(ctx->ev_hash);
    hipEventDestroy(ctx->ev_fork);
    hipEventDestroy(ctx->ev_join[0]);
    hipEventDestroy(ctx->ev_join[1]);
  }
  for (auto e : ctx->event_pool) hipEventDestroy(e);
  if (ctx->pinned) hipHostFree(ctx->pinned);
  delete ctx;
}

int ottohip_ctx_trim(ottohip_ctx* ctx) {
  if (!ctx) return OTTOHIP_EINVAL;
  OH_HIP(hipSetDevice(ctx->device));
  OH_HIP(hipDeviceSynchronize());
  ctx->ws.release();
  ctx->spare.release();
  dev_trim();
  ctx->km_bvalid = false;  // the KMeans distance bounds lived in the released workspace
  ctx->km_hX = nullptr;     // and the attached half-precision rows
  ctx->om_items = -1;       // and the owner map
  return 0;
}

int ottohip_ctx_set_timing(ottohip_ctx* ctx, int enable) {
  if (!ctx) return OTTOHIP_EINVAL;
  ctx->timing = enable != 0;
  return 0;
}

int ottohip_ctx_timing(ottohip_ctx* ctx, int idx, const char** name, float* ms, double* bytes) {
  if (!ctx) return OTTOHIP_EINVAL;
  if (idx < 0) return (int)ctx->phases.size();
  if (idx >= (int)ctx->phases.size()) return OTTOHIP_EINVAL;
  Phase& p = ctx->phases[idx];
  OH_HIP(hipEventSynchronize(p.b));
  float t = 0;
  OH_HIP(hipEventElapsedTime(&t, p.a, p.b));
  if (name) *name = p.name.c_str();
  if (ms) *ms = t;
  if (bytes) *bytes = p.bytes;
  return 0;
}

int ottohip_test_exclusive_scan_u32(ottohip_ctx* ctx, const uint32_t* in, uint64_t* out, int64_t n,
                                    uint64_t* total_host, void* stream) {
  if (!ctx) return OTTOHIP_EINVAL;
  uint64_t* tot;
  OH_TRY(ctx->ws.get("test_total", 1, &tot));
  OH_TRY(exclusive_scan_u32(ctx, in, out, n, tot, S(stream)));
  if (total_host) OH_TRY(d2h(total_host, tot, 1, S(stream)));
  return 0;
}

__global__ void k_test_lanes(const uint32_t* __restrict__ in, uint32_t* __restrict__ out) {
  const uint32_t l = lane_id();
  const uint32_t v = in[l];
  out[0 * 64 + l] = xor_lane<1>(v);
  out[1 * 64 + l] = xor_lane<2>(v);
  out[2 * 64 + l] = xor_lane<4>(v);
  out[3 * 64 + l] = xor_lane<8>(v);
  out[4 * 64 + l] = xor_lane<16>(v);
  out[5 * 64 + l] = xor_lane<32>(v);
  out[6 * 64 + l] = dpp_incl_scan<false>(v);
  out[7 * 64 + l] = dpp_incl_scan<true>(v);
  out[8 * 64 + l] = lane_prev(v);
  out[9 * 64 + l] = lane_next(v);
}

int ottohip_test_lanes(const uint32_t* in, uint32_t* out, void* stream) {
  if (!in || !out) return OTTOHIP_EINVAL;
  k_test_lanes<<<1, 64, 0, S(stream)>>>(in, out);
  OH_HIP(hipGetLastError());
  return 0;
}

int ottohip_test_radix_sort_pairs(ottohip_ctx* ctx, uint32_t* keys, uint32_t* vals, int64_t n, int bits,
                                  void* stream) {
  if (!ctx || bits < 0 || bits > 32) return OTTOHIP_EINVAL;
  uint32_t *ka, *va;
  OH_TRY(ctx->ws.get("test_ka", (size_t)std::max<int64_t>(n, 1), &ka));
  OH_TRY(ctx->ws.get("test_va", (size_t)std::max<int64_t>(n, 1), &va));
  uint32_t *k = keys, *v = vals;
  OH_TRY(radix_sort_pairs(ctx, k, v, ka, va, n, bits, S(stream)));
  if (k != keys) {
    OH_HIP(hipMemcpyAsync(keys, k, n * sizeof(uint32_t), hipMemcpyDeviceToDevice, S(stream)));
    OH_HIP(hipMemcpyAsync(vals, v, n * sizeof(uint32_t), hipMemcpyDeviceToDevice, S(stream)));
  }
  return 0;
}

static void file_opts_zero(const ottohip_file_opts* o) {
  if (!o) return;
  for (int f = 0; f < o->n_files; ++f) {
    if (o->file_rows) o->file_rows[f] = 0;
    if (o->file_rows_ge2) o->file_rows_ge2[f] = 0;
  }
}

// the first word of each row type's rows in a row-key-ordered row list (keys (type << A) | aid) for types 0..2, and
// P: out[t] .. out[t + 1] is type t's word (= table slot) range
__global__ void k_type_slots(const uint32_t* __restrict__ rk, const uint64_t* __restrict__ rb, int64_t Rn, uint64_t P,
                             int A, uint64_t* __restrict__ out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  for (uint32_t t = 0; t < 3; ++t) {
    int64_t lo = 0, hi = Rn;
    while (lo < hi) {
      const int64_t m = (lo + hi) >> 1;
      if ((rk[m] >> A) < t) lo = m + 1; else hi = m;
    }
    out[t] = lo < Rn ? rb[lo] : P;
  }
  out[3] = P;
}
// a rule's slot range in table t: [*s0, *s1) (every slot when the table has no type ranges)
static int rule_slot_range(ottohip_table* t, int rule, hipStream_t s, int64_t* s0, int64_t* s1) {
  *s0 = 0; *s1 = t->n_slots;
  if (!t->type_slots_dev || rule < 0 || rule >= TABLE_MAX_IDS) return 0;
  const int ty = t->rule_type[rule];
  if (ty < 0 || ty > 2) return 0;
  if (!t->type_slots_known) {
    uint64_t h[4];
    OH_TRY(d2h(h, t->type_slots_dev, 4, s));
    for (int k = 0; k < 4; ++k) t->type_slots[k] = (int64_t)h[k];
    t->type_slots_known = true;
  }
  *s0 = std::min<int64_t>(t->type_slots[ty], t->n_slots);
  *s1 = std::min<int64_t>(t->type_slots[ty + 1], t->n_slots);
  if (*s1 < *s0) { *s0 = 0; *s1 = t->n_slots; }
  return 0;
}
// the finalize-scan blocks over a rule's slot range: first slot i0 (block-aligned: slots before the range hold other
// types' rows), end n, nb blocks of FIN_B slots (OTTOHIP_FIN_ALL=1: every slot; A/B switch, read per call)
static int rule_scan_blocks(const ottohip_table* t, int rule, hipStream_t s, int64_t* i0, int64_t* n, int64_t* nb) {
  int64_t s0 = 0, s1 = t->n_slots;
  if (!(getenv("OTTOHIP_FIN_ALL") && !strcmp(getenv("OTTOHIP_FIN_ALL"), "1")))
    OH_TRY(rule_slot_range(const_cast<ottohip_table*>(t), rule, s, &s0, &s1));
  *i0 = s0 / FIN_B * FIN_B;
  *n = s1;
  *nb = std::max<int64_t>(1, ceil_div(s1 - *i0, FIN_B));
  return 0;
}


int ottohip_covis_count_opts(ottohip_ctx* ctx, const ottohip_events* ev, const ottohip_rule* rules, int n_rules,
                             const ottohip_covis_params* params, const ottohip_file_opts* opts, ottohip_table** out,
                             void* stream) {
  if (!ctx || !ev || !rules || !params || !out) { set_error("ottohip_covis_count: NULL argument"); return OTTOHIP_EINVAL; }
  *out = nullptr;
  hipStream_t s = S(stream);
  OH_HIP(hipSetDevice(ctx->device));
  ctx->reset_timing();
  Front F;
  OH_TRY(check_events(ev));
  // symmetric storage stays on with per-file statistics only; key cuts need both orders of a pair stored
  const bool sym_ok = opts == nullptr || (opts->lo_file < 0 && opts->hi_file < 0);
  OH_TRY(setup_rules(rules, n_rules, params, ev->n_files, F.R, F.Lt, /*allow_sym=*/sym_ok));
  if (opts && (opts->file_rows || opts->file_rows_ge2) && opts->n_files < ev->n_files) {
    set_error("file_opts: n_files=%d < the call's %d files", opts->n_files, ev->n_files); return OTTOHIP_EINVAL;
  }
  file_opts_zero(opts);
  // options that change the reduce (key cuts, per-file rows); keep_words alone only keeps the words
  const ottohip_file_opts* fo_eff =
      (opts && (opts->lo_file >= 0 || opts->hi_file >= 0 || opts->file_rows || opts->file_rows_ge2)) ? opts : nullptr;
  const bool keep = opts && opts->keep_words;
  ottohip_table* T = new_table(ctx, n_rules, params->n_items);
  auto fail = [&](int rc) { ottohip_table_free(T); return rc; };
  int rc;
  if ((rc = covis_front(ctx, ev, params, nullptr, 1, F, s))) return fail(rc);
  if (F.P == 0) { *out = T; return 0; }
  uint32_t *w0, *w1, *w2 = nullptr;
  if ((rc = ctx->ws.get("words0", (size_t)F.P, &w0)) || (rc = ctx->ws.get("words1", (size_t)F.P, &w1))) return fail(rc);
  if (keep && (rc = ctx->ws.get("words2", (size_t)F.P, &w2))) return fail(rc);
  if ((rc = covis_emit_words(ctx, F, ev, w0, s))) return fail(rc);
  // the slot range of every row type (rows are type-major), for the per-rule readers; read back on first use
  // (queued before the reduce, whose closing statistics read synchronises the stream)
  if (dev_alloc(reinterpret_cast<void**>(&T->type_slots_dev), 4 * sizeof(uint64_t), "type_slots") == hipSuccess) {
    k_type_slots<<<1, 64, 0, s>>>(F.row_key, F.row_begin, F.Rn, F.P, F.Lt.A, T->type_slots_dev);
    for (int r = 0; r < n_rules; ++r) T->rule_type[r] = (int8_t)rules[r].this_type;
  }
  if ((rc = covis_reduce(ctx, w0, w1, F.P, F.row_begin, F.row_key, F.Rn, F.R, F.Lt, n_rules, T, s, fo_eff, nullptr, w2)))
    return fail(rc);
  if (keep) {  // the table takes the emitted words (w0, untouched by the three-buffer reduce) and the rows
    KeptEmission* K = new KeptEmission();
    K->words = static_cast<uint32_t*>(ctx->ws.take("words0"));
    K->row_key = static_cast<uint32_t*>(ctx->ws.take("row_key"));
    K->row_begin = static_cast<uint64_t*>(ctx->ws.take("row_begin"));
    K->P = F.P; K->Rn = F.Rn; K->R = F.R; K->Lt = F.Lt; K->n_rules = n_rules; K->n_files = ev->n_files;
    T->kept = K;
  }
  *out = T;
  return 0;
}

// rows [r0, r1) of one row type in a row-key-ordered row list (keys (type << A) | aid), and their words
__global__ void k_type_span(const uint32_t* __restrict__ rk, const uint64_t* __restrict__ rb, int64_t Rn, uint64_t P,
                            int A, uint32_t type, uint64_t* __restrict__ out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  int64_t r[2];
  for (int k = 0; k < 2; ++k) {
    int64_t lo = 0, hi = Rn;
    while (lo < hi) {
      const int64_t m = (lo + hi) >> 1;
      if ((rk[m] >> A) < type + (uint32_t)k) lo = m + 1; else hi = m;
    }
    r[k] = lo;
  }
  out[0] = (uint64_t)r[0]; out[1] = (uint64_t)r[1];
  out[2] = r[0] < Rn ? rb[r[0]] : P; out[3] = r[1] < Rn ? rb[r[1]] : P;
}

int ottohip_table_count_parts(ottohip_ctx* ctx, const ottohip_table* t, int rule, const ottohip_part_opts* po,
                                         ottohip_table** out, void* stream) {
  if (!ctx || !t || !po || !out || !po->first_part || (po->n_cuts > 0 && (!po->cut_file || !po->cut_key))) {
    set_error("table_count_parts: NULL argument"); return OTTOHIP_EINVAL;
  }
  *out = nullptr;
  if (!t->kept) { set_error("table_count_parts: the table kept no words (ottohip_file_opts.keep_words)"); return OTTOHIP_EINVAL; }
  const KeptEmission& K = *t->kept;
  if (rule < 0 || rule >= K.n_rules) { set_error("table_count_parts: rule %d outside the count's rules", rule); return OTTOHIP_EINVAL; }
  const int nf = K.n_files;
  if (po->n_files != nf) { set_error("table_count_parts: n_files=%d, the count had %d files", po->n_files, nf); return OTTOHIP_EINVAL; }
  if (nf > FO_MAXF) { set_error("table_count_parts: %d files > %d", nf, FO_MAXF); return OTTOHIP_ELIMIT; }
  if (po->n_parts < 1 || po->n_parts > 254) { set_error("table_count_parts: n_parts=%d outside [1, 254]", po->n_parts); return OTTOHIP_ELIMIT; }
  if (po->n_cuts < 0 || po->n_cuts > FO_MAXCUT) { set_error("table_count_parts: n_cuts=%d outside [0, %d]", po->n_cuts, FO_MAXCUT); return OTTOHIP_ELIMIT; }
  if (K.Lt.A > 24) { set_error("table_count_parts: n_items > 2^24"); return OTTOHIP_ELIMIT; }
  std::vector<uint8_t> part_of(nf), cut_of(nf, FO_NOCUT);
  for (int f = 0; f < nf; ++f) {
    if (po->first_part[f] < 0 || po->first_part[f] >= po->n_parts) { set_error("table_count_parts: first_part[%d] out of range", f); return OTTOHIP_EINVAL; }
    part_of[f] = (uint8_t)po->first_part[f];
  }
  for (int c = 0; c < po->n_cuts; ++c) {
    const int f = po->cut_file[c];
    if (f < 0 || f >= nf || cut_of[f] != FO_NOCUT || part_of[f] + 1 >= po->n_parts) {
      set_error("table_count_parts: cut %d (file %d) invalid: one cut per file, inside the parts", c, f); return OTTOHIP_EINVAL;
    }
    cut_of[f] = (uint8_t)c;
  }
  int type = -1, q = -1;
  for (int tt = 0; tt < 3; ++tt)
    for (int qq = 0; qq < K.R.n_of_type[tt]; ++qq)
      if (K.R.rule_of_type[tt][qq] == rule) { type = tt; q = qq; }
  if (type < 0) { set_error("table_count_parts: rule %d has no row type", rule); return OTTOHIP_EINVAL; }
  hipStream_t s = S(stream);
  OH_HIP(hipSetDevice(ctx->device));
  ctx->reset_timing();
  Workspace& ws = ctx->ws;
  uint64_t* span;
  OH_TRY(ws.get("tcp_span", 4, &span));
  k_type_span<<<1, 64, 0, s>>>(K.row_key, K.row_begin, K.Rn, K.P, K.Lt.A, (uint32_t)type, span);
  uint64_t sp[4];
  OH_TRY(d2h(sp, span, 4, s));
  const int64_t r0 = (int64_t)sp[0], r1 = (int64_t)sp[1];
  const uint64_t wlo = sp[2], Psub = sp[3] - sp[2];
  ottohip_table* T = new_table(ctx, 1, t->n_items);
  auto fail = [&](int rc) { ottohip_table_free(T); return rc; };
  T->n_rules = po->n_parts;
  if (Psub == 0 || r1 <= r0) { *out = T; return 0; }
  int rc;
  uint32_t *w1, *w2;
  if ((rc = ws.get("words1", (size_t)Psub, &w1)) || (rc = ws.get("words2", (size_t)Psub, &w2))) return fail(rc);
  FileOpts fo;
  memset(&fo, 0, sizeof fo);
  fo.type = type;
  fo.q = (uint32_t)q;
  fo.lo_file = fo.hi_file = 0xFFFFFFFFu;
  fo.nf = (uint32_t)nf;
  fo.parts = 1;
  fo.qonly = 1;  // the type's other rules' words are skipped (counted as dropped)
  fo.mirror_off = ((K.R.sym_mask >> rule) & 1u) ? Psub : 0ull;
  fo.ncut = (uint32_t)po->n_cuts;
  for (int c = 0; c < po->n_cuts; ++c) fo.cut_key[c] = po->cut_key[c];
  uint8_t *d_part, *d_cut;
  if ((rc = ws.get("fo_part_of", (size_t)nf, &d_part)) || (rc = ws.get("fo_cut_of", (size_t)nf, &d_cut))) return fail(rc);
  OH_HIP(hipMemcpyAsync(d_part, part_of.data(), nf, hipMemcpyHostToDevice, s));
  OH_HIP(hipMemcpyAsync(d_cut, cut_of.data(), nf, hipMemcpyHostToDevice, s));
  OH_HIP(hipStreamSynchronize(s));  // host vectors
  fo.part_of = d_part;
  fo.cut_of = d_cut;
  // the kept words are only read: the level-0 split writes w1, the later levels w1 <-> w2
  if ((rc = covis_reduce(ctx, K.words + wlo, w1, Psub, K.row_begin + r0, K.row_key + r0, r1 - r0, K.R, K.Lt, K.n_rules, T,
                         s, nullptr, &fo, w2, wlo)))
    return fail(rc);
  T->sym_mask = 0;  // explicit rows (the mirrors written by the leaves)
  T->aid_ordered = fo.mirror_off == 0;
  T->n_rules = po->n_parts;
  // per part: rows and pairs, counted when first read (ottohip_table_stats / _copy / _finalize): the part heads
  // (ottohip_table_part_heads) do not need them, and the table scan took 4.3 ms per A6 of click_to_click
  for (int p = 0; p < po->n_parts; ++p) T->stats[p] = ottohip_rule_stats{};
  T->part_stats_pending = po->n_parts;
  OH_HIP(hipEventCreateWithFlags(&T->produced, hipEventDisableTiming));
  OH_HIP(hipEventRecord(T->produced, s));
  *out = T;
  return 0;
}

int ottohip_covis_count_parts(ottohip_ctx* ctx, const ottohip_events* ev, const ottohip_rule* rules, int n_rules,
                              const ottohip_covis_params* params, const ottohip_part_opts* po, ottohip_table** out,
                              void* stream) {
  if (!ctx || !ev || !rules || !params || !po || !out || !po->first_part || (po->n_cuts > 0 && (!po->cut_file || !po->cut_key))) {
    set_error("ottohip_covis_count_parts: NULL argument"); return OTTOHIP_EINVAL;
  }
  *out = nullptr;
  if (n_rules != 1) { set_error("count_parts: one rule per call (got %d)", n_rules); return OTTOHIP_EINVAL; }
  OH_TRY(check_events(ev));
  const int nf = ev->n_files;
  if (po->n_files != nf) { set_error("count_parts: n_files=%d, the call has %d files", po->n_files, nf); return OTTOHIP_EINVAL; }
  if (nf > FO_MAXF) { set_error("count_parts: %d files > %d per call", nf, FO_MAXF); return OTTOHIP_ELIMIT; }
  if (po->n_parts < 1 || po->n_parts > 254 || po->n_parts > TABLE_MAX_IDS) {
    set_error("count_parts: n_parts=%d outside [1, 254]", po->n_parts); return OTTOHIP_ELIMIT;
  }
  if (po->n_cuts < 0 || po->n_cuts > FO_MAXCUT) { set_error("count_parts: n_cuts=%d outside [0, %d]", po->n_cuts, FO_MAXCUT); return OTTOHIP_ELIMIT; }
  if (params->n_items > (1 << 24)) { set_error("count_parts: n_items > 2^24"); return OTTOHIP_ELIMIT; }
  std::vector<uint8_t> part_of(nf), cut_of(nf, FO_NOCUT);
  for (int f = 0; f < nf; ++f) {
    if (po->first_part[f] < 0 || po->first_part[f] >= po->n_parts) { set_error("count_parts: first_part[%d] out of range", f); return OTTOHIP_EINVAL; }
    part_of[f] = (uint8_t)po->first_part[f];
  }
  for (int c = 0; c < po->n_cuts; ++c) {
    const int f = po->cut_file[c];
    if (f < 0 || f >= nf || cut_of[f] != FO_NOCUT || part_of[f] + 1 >= po->n_parts) {
      set_error("count_parts: cut %d (file %d) invalid: one cut per file, inside the parts", c, f); return OTTOHIP_EINVAL;
    }
    cut_of[f] = (uint8_t)c;
  }
  hipStream_t s = S(stream);
  OH_HIP(hipSetDevice(ctx->device));
  ctx->reset_timing();
  Front F;
  // OTTOHIP_A6_SYMPART=1 (read per call; experiment): a symmetric rule stores each unordered pair once and the
  // leaves write the mirrors as explicit rows with their own parts at slot + P (the table is then not in aid order)
  const bool sympart = getenv("OTTOHIP_A6_SYMPART") && !strcmp(getenv("OTTOHIP_A6_SYMPART"), "1");
  OH_TRY(setup_rules(rules, n_rules, params, nf, F.R, F.Lt, /*allow_sym=*/sympart));
  ottohip_table* T = new_table(ctx, n_rules, params->n_items);
  auto fail = [&](int rc) { ottohip_table_free(T); return rc; };
  int rc;
  if ((rc = covis_front(ctx, ev, params, nullptr, 1, F, s))) return fail(rc);
  T->n_rules = po->n_parts;
  if (F.P == 0) { *out = T; return 0; }
  uint32_t *w0, *w1;
  if ((rc = ctx->ws.get("words0", (size_t)F.P, &w0)) || (rc = ctx->ws.get("words1", (size_t)F.P, &w1))) return fail(rc);
  if ((rc = covis_emit_words(ctx, F, ev, w0, s))) return fail(rc);
  FileOpts fo;
  memset(&fo, 0, sizeof fo);
  fo.type = rules[0].this_type;
  fo.q = 0;
  fo.lo_file = fo.hi_file = 0xFFFFFFFFu;
  fo.nf = (uint32_t)nf;
  fo.parts = 1;
  fo.ncut = (uint32_t)po->n_cuts;
  for (int c = 0; c < po->n_cuts; ++c) fo.cut_key[c] = po->cut_key[c];
  uint8_t *d_part, *d_cut;
  if ((rc = ctx->ws.get("fo_part_of", (size_t)nf, &d_part)) || (rc = ctx->ws.get("fo_cut_of", (size_t)nf, &d_cut))) return fail(rc);
  OH_HIP(hipMemcpyAsync(d_part, part_of.data(), nf, hipMemcpyHostToDevice, s));
  OH_HIP(hipMemcpyAsync(d_cut, cut_of.data(), nf, hipMemcpyHostToDevice, s));
  OH_HIP(hipStreamSynchronize(s));  // host vectors
  fo.part_of = d_part;
  fo.cut_of = d_cut;
  fo.mirror_off = (F.R.sym_mask & 1u) ? F.P : 0ull;
  if ((rc = covis_reduce(ctx, w0, w1, F.P, F.row_begin, F.row_key, F.Rn, F.R, F.Lt, n_rules, T, s, nullptr, &fo)))
    return fail(rc);
  if (fo.mirror_off) {
    T->sym_mask = 0;  // explicit rows (the mirrors written by the leaves)
    T->aid_ordered = false;
  }
  // per part: rows and pairs (file statistics stay 0: the part-wise finalize is told which column to use)
  T->n_rules = po->n_parts;
  // per part: rows and pairs, counted when first read (ottohip_table_stats / _copy / _finalize): the part heads
  // (ottohip_table_part_heads) do not need them, and the table scan took 4.3 ms per A6 of click_to_click
  for (int p = 0; p < po->n_parts; ++p) T->stats[p] = ottohip_rule_stats{};
  T->part_stats_pending = po->n_parts;
  OH_HIP(hipEventCreateWithFlags(&T->produced, hipEventDisableTiming));
  OH_HIP(hipEventRecord(T->produced, s));
  *out = T;
  return 0;
}

int ottohip_covis_count(ottohip_ctx* ctx, const ottohip_events* ev, const ottohip_rule* rules, int n_rules,
                        const ottohip_covis_params* params, ottohip_table** out, void* stream) {
  return ottohip_covis_count_opts(ctx, ev, rules, n_rules, params, nullptr, out, stream);
}

int ottohip_covis_emit(ottohip_ctx* ctx, const ottohip_events* ev, const ottohip_rule* rules, int n_rules,
                       const ottohip_covis_params* params, const int32_t* file_ids, int32_t n_files_total,
                       int n_parts, ottohip_emit** out, int64_t* words_per_part, int64_t* rows_per_part,
                       void* stream) {
  if (!ctx || !ev || !rules || !params || !out || !words_per_part || !rows_per_part || n_parts < 1 ||
      n_parts > 256) {
    set_error("ottohip_covis_emit: bad arguments (n_parts in [1, 256])"); return OTTOHIP_EINVAL;
  }
  *out = nullptr;
  hipStream_t s = S(stream);
  OH_HIP(hipSetDevice(ctx->device));
  ctx->reset_timing();
  OH_TRY(check_events(ev));
  if (n_files_total < ev->n_files) { set_error("n_files_total < n_files"); return OTTOHIP_EINVAL; }
  for (int f = 0; f < ev->n_files && file_ids; ++f)
    if (file_ids[f] < 0 || file_ids[f] >= n_files_total) { set_error("file_ids[%d] outside [0, n_files_total)", f); return OTTOHIP_EINVAL; }
  ottohip_emit* E = new ottohip_emit();
  E->n_parts = n_parts;
  E->ev = *ev;
  int rc;
  if ((rc = setup_rules(rules, n_rules, params, n_files_total, E->F.R, E->F.Lt, /*allow_sym=*/params->sym != 0))) {
    delete E;
    return rc;
  }
  if ((rc = covis_front(ctx, ev, params, file_ids, n_parts, E->F, s))) { delete E; return rc; }
  E->gen = ctx->gen;
  E->ctx = ctx;
  E->first_row.assign(n_parts + 1, 0);
  E->first_word.assign(n_parts + 1, 0);
  if (E->F.Rn > 0) {
    uint64_t *d_fr, *d_fw;
    if ((rc = ctx->ws.get("part_first_row", (size_t)n_parts + 1, &d_fr)) ||
        (rc = ctx->ws.get("part_first_word", (size_t)n_parts + 1, &d_fw))) { delete E; return rc; }
    k_part_bounds<<<grid_for(E->F.Rn + 1), 256, 0, s>>>(E->F.row_key, E->F.Rn, E->F.Lt.A, (uint32_t)n_parts, d_fr);
    k_part_words<<<grid_for(n_parts + 1), 256, 0, s>>>(d_fr, E->F.row_begin, E->F.Rn, E->F.P, (uint32_t)n_parts, d_fw);
    if ((rc = d2h(E->first_row.data(), d_fr, (size_t)n_parts + 1, s)) ||
        (rc = d2h(E->first_word.data(), d_fw, (size_t)n_parts + 1, s))) { delete E; return rc; }
  }
  for (int p = 0; p < n_parts; ++p) {
    rows_per_part[p] = (int64_t)(E->first_row[p + 1] - E->first_row[p]);
    words_per_part[p] = (int64_t)(E->first_word[p + 1] - E->first_word[p]);
  }
  *out = E;
  return 0;
}

int ottohip_emit_write(ottohip_emit* E, uint32_t* words, uint64_t* pieces, void* stream) {
  if (!E || (E->F.P > 0 && !words) || (E->F.Rn > 0 && !pieces)) { set_error("emit_write: bad arguments"); return OTTOHIP_EINVAL; }
  if (E->gen != E->ctx->gen) {
    set_error("emit_write: the context ran another count after ottohip_covis_emit"); return OTTOHIP_EINVAL;
  }
  hipStream_t s = S(stream);
  OH_HIP(hipSetDevice(E->ctx->device));
  if (E->F.P > 0) OH_TRY(covis_emit_words(E->ctx, E->F, &E->ev, words, s));
  if (E->F.Rn > 0) {
    k_piece_pack<<<grid_for(E->F.Rn), 256, 0, s>>>(E->F.row_key, E->F.row_begin, E->F.Rn, E->F.P, pieces);
    OH_HIP(hipGetLastError());
  }
  return 0;
}

void ottohip_emit_free(ottohip_emit* E) { delete E; }

int ottohip_covis_reduce_received(ottohip_ctx* ctx, const ottohip_rule* rules, int n_rules,
                                  const ottohip_covis_params* params, int32_t n_files_total, const uint32_t* words,
                                  int64_t n_words, const uint64_t* pieces, int64_t n_pieces, ottohip_table** out,
                                  void* stream) {
  return ottohip_covis_reduce_received_opts(ctx, rules, n_rules, params, n_files_total, words, n_words, pieces,
                                            n_pieces, nullptr, out, stream);
}

int ottohip_covis_reduce_received_opts(ottohip_ctx* ctx, const ottohip_rule* rules, int n_rules,
                                       const ottohip_covis_params* params, int32_t n_files_total, const uint32_t* words,
                                       int64_t n_words, const uint64_t* pieces, int64_t n_pieces,
                                       const ottohip_file_opts* opts, ottohip_table** out, void* stream) {
  if (!ctx || !rules || !params || !out || n_words < 0 || n_pieces < 0 || (n_words > 0 && !words) ||
      (n_pieces > 0 && !pieces)) {
    set_error("ottohip_covis_reduce_received: bad arguments"); return OTTOHIP_EINVAL;
  }
  if (opts && (opts->file_rows || opts->file_rows_ge2) && opts->n_files < n_files_total) {
    set_error("file_opts: n_files=%d < n_files_total=%d", opts->n_files, n_files_total); return OTTOHIP_EINVAL;
  }
  file_opts_zero(opts);
  *out = nullptr;
  hipStream_t s = S(stream);
  OH_HIP(hipSetDevice(ctx->device));
  ctx->reset_timing();
  RulesDev R;
  Layout Lt;
  if (params->sym && opts && (opts->lo_file >= 0 || opts->hi_file >= 0)) {
    set_error("reduce_received: key cuts on symmetric storage (params->sym must be 0)"); return OTTOHIP_EINVAL;
  }
  // the senders' storage (ottohip_covis_emit with the same params->sym): symmetric rules once per unordered pair
  OH_TRY(setup_rules(rules, n_rules, params, std::max(n_files_total, 1), R, Lt, /*allow_sym=*/params->sym != 0));
  if (n_words >= ((int64_t)1 << 40) || n_pieces >= ((int64_t)1 << 32)) { set_error("received input too large"); return OTTOHIP_ELIMIT; }
  ottohip_table* T = new_table(ctx, n_rules, params->n_items);
  auto fail = [&](int rc) { ottohip_table_free(T); return rc; };
  if (n_words == 0) { *out = T; return 0; }
  Workspace& ws = ctx->ws;
  const int64_t n = n_pieces;
  uint32_t *key, *val, *k1, *v1, *len, *lsort, *head;
  uint64_t *src_off, *dst, *row_idx, *tot, *row_begin;
  uint32_t* row_key;
  int* err;
  int rc;
  if ((rc = ws.get("pc_key", (size_t)n, &key)) || (rc = ws.get("pc_val", (size_t)n, &val)) ||
      (rc = ws.get("pc_k1", (size_t)n, &k1)) || (rc = ws.get("pc_v1", (size_t)n, &v1)) ||
      (rc = ws.get("pc_len", (size_t)n, &len)) || (rc = ws.get("pc_lsort", (size_t)n, &lsort)) ||
      (rc = ws.get("pc_head", (size_t)n, &head)) || (rc = ws.get("pc_src", (size_t)n, &src_off)) ||
      (rc = ws.get("pc_dst", (size_t)n, &dst)) || (rc = ws.get("pc_ridx", (size_t)n, &row_idx)) ||
      (rc = ws.get("pc_tot", 4, &tot)) || (rc = ws.get("err", 4, &err)) ||
      (rc = ws.get("row_key", (size_t)n, &row_key)) || (rc = ws.get("row_begin", (size_t)n, &row_begin)))
    return fail(rc);
  const int kbits = Lt.A + 2;
  int ph = ctx->begin("assemble", s, 8.0 * (double)n_words + 24.0 * (double)n);
  hipMemsetAsync(err, 0, sizeof(int), s);
  k_piece_keys<<<grid_for(n), 256, 0, s>>>(pieces, n, key, val, len, 3u << Lt.A, err);
  // source offsets of the pieces (received order), then pieces by row key (stable: by source)
  if ((rc = exclusive_scan_u32(ctx, len, src_off, n, tot, s))) return fail(rc);
  uint32_t *ks = key, *vs = val;
  if ((rc = radix_sort_pairs(ctx, ks, vs, k1, v1, n, kbits, s))) return fail(rc);
  k_piece_order<<<grid_for(n), 256, 0, s>>>(ks, vs, len, n, lsort, head);
  if ((rc = exclusive_scan_u32(ctx, lsort, dst, n, tot + 1, s)) || (rc = exclusive_scan_u32(ctx, head, row_idx, n, tot + 2, s)))
    return fail(rc);
  uint64_t tt[3];
  int herr = 0;
  if ((rc = d2h(tt, tot, 3, s)) || (rc = d2h(&herr, err, 1, s))) return fail(rc);
  if (herr) { set_error("reduce_received: piece row key out of range"); return fail(OTTOHIP_ERANGE); }
  if ((int64_t)tt[0] != n_words) {
    set_error("reduce_received: pieces hold %llu words, %lld received", (unsigned long long)tt[0], (long long)n_words);
    return fail(OTTOHIP_EINVAL);
  }
  const uint64_t P = tt[0];
  const int64_t Rn = (int64_t)tt[2];
  uint32_t *w0, *w1;
  if ((rc = ws.get("words0", (size_t)P, &w0)) || (rc = ws.get("words1", (size_t)P, &w1))) return fail(rc);
  k_piece_rows<<<grid_for(n), 256, 0, s>>>(ks, head, row_idx, dst, n, row_key, row_begin);
  {
    uint32_t *nch, *cmap;
    uint64_t* cb;
    if ((rc = ws.get("pc_nch", (size_t)n, &nch)) || (rc = ws.get("pc_cb", (size_t)n, &cb))) return fail(rc);
    k_piece_nchunks<<<grid_for(n), 256, 0, s>>>(lsort, n, nch);
    if ((rc = exclusive_scan_u32(ctx, nch, cb, n, tot + 3, s))) return fail(rc);
    uint64_t nc = 0;
    if ((rc = d2h(&nc, tot + 3, 1, s))) return fail(rc);
    if ((rc = ws.get("pc_cmap", (size_t)std::max<uint64_t>(nc, 1), &cmap))) return fail(rc);
    k_chunk_map<<<grid_for(n), 256, 0, s>>>(nch, cb, n, cmap);
    k_piece_copy<<<grid_for((int64_t)nc, 4), 256, 0, s>>>(cmap, cb, (int64_t)nc, vs, len, src_off, dst, words, w0);
  }
  if (hipGetLastError() != hipSuccess) { set_error("assemble launch failed"); return fail(OTTOHIP_EHIP); }
  ctx->end(ph, s);
  if ((rc = covis_reduce(ctx, w0, w1, P, row_begin, row_key, Rn, R, Lt, n_rules, T, s, opts))) return fail(rc);
  *out = T;
  return 0;
}

int ottohip_table_set_file_stats(ottohip_table* t, int rule, int64_t file_rows, int64_t file_rows_ge2) {
  if (!t || rule < 0 || rule >= t->n_rules || file_rows < 0 || file_rows_ge2 < 0) {
    set_error("table_set_file_stats: bad args"); return OTTOHIP_EINVAL;
  }
  t->stats[rule].file_rows = file_rows;
  t->stats[rule].file_rows_ge2 = file_rows_ge2;
  return 0;
}

int ottohip_table_stats(const ottohip_table* t, int rule, ottohip_rule_stats* st) {
  if (!t || !st || rule < 0 || rule >= t->n_rules) { set_error("table_stats: bad args"); return OTTOHIP_EINVAL; }
  OH_TRY(ensure_part_stats(t));
  *st = t->stats[rule];
  return 0;
}

int ottohip_table_copy(const ottohip_table* t, int rule, int32_t* aid, int32_t* aid_next, uint32_t* count,
                       uint32_t* count_ge2, void* stream) {
  if (!t || rule < 0 || rule >= t->n_rules) { set_error("table_copy: bad args"); return OTTOHIP_EINVAL; }
  OH_TRY(ensure_part_stats(t));
  if (t->n_rows == 0 || t->stats[rule].n_rows == 0) return 0;
  hipStream_t s = S(stream);
  Ctx* ctx = t->ctx;
  int64_t i0, n, nb;
  OH_TRY(rule_scan_blocks(t, rule, s, &i0, &n, &nb));
  uint32_t* bcnt;
  uint64_t* boff;
  OH_TRY(ctx->ws.get("blk_cnt", (size_t)nb, &bcnt));
  OH_TRY(ctx->ws.get("blk_off", (size_t)nb, &boff));
  k_blk_count<<<(unsigned)nb, FIN_T, 0, s>>>(t->b.rule, t->b.aid, t->b.aid_next, t->b.count, t->b.count_ge2, n, rule, 0, 0u,
                                             t->sym(rule), bcnt, i0);
  OH_TRY(exclusive_scan_u32(ctx, bcnt, boff, nb, nullptr, s));
  k_blk_compact<<<(unsigned)nb, FIN_T, 0, s>>>(t->b.rule, t->b.aid, t->b.aid_next, t->b.count, t->b.count_ge2, n,
                                               rule, 0, 0u, t->sym(rule), boff, reinterpret_cast<uint32_t*>(aid),
                                               reinterpret_cast<uint32_t*>(aid_next), count, count_ge2, i0);
  OH_HIP(hipGetLastError());
  return 0;
}

__global__ void k_keys_at(const uint32_t* __restrict__ perm, const uint32_t* __restrict__ sa,
                          const uint32_t* __restrict__ sb, const int64_t* __restrict__ idx, int n,
                          uint64_t* __restrict__ keys) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t j = perm[idx[i]];
  keys[i] = ((uint64_t)sa[j] << 32) | sb[j];
}

// *uns = 1 where a compacted aid column descends (a rule's rows in slot order are in aid order when the
// table came from one count and the rule keeps both directions, e.g. every part of a part-mode table)
__global__ void k_sorted_check(const uint32_t* __restrict__ a, int64_t m, int* __restrict__ uns) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x + 1;
  if (i < m && a[i] < a[i - 1]) *uns = 1;
}
// one block per index of aid-ordered rows (sa ascending): the idx-th row in (aid, aid_next) order has aid
// sa[idx], and its aid_next is the (idx - g0)-th smallest aid_next of that aid's rows [g0, g1): a radix select
// (8 bits per pass over the group) instead of sorting every row of the rule
__global__ __launch_bounds__(256) void k_keys_at_sel(const uint32_t* __restrict__ sa, const uint32_t* __restrict__ sb,
                                                     int64_t m, const int64_t* __restrict__ idx,
                                                     uint64_t* __restrict__ keys) {
  __shared__ uint32_t hist[256];
  __shared__ uint32_t s_prefix, s_k;
  __shared__ int64_t s_g0, s_g1;
  const int64_t r = idx[blockIdx.x];
  const uint32_t a = sa[r];
  if (threadIdx.x == 0) {
    int64_t lo = 0, hi = r;  // first row of aid a
    while (lo < hi) { const int64_t md = (lo + hi) >> 1; if (sa[md] < a) lo = md + 1; else hi = md; }
    s_g0 = lo;
    lo = r + 1; hi = m;  // first row past aid a
    while (lo < hi) { const int64_t md = (lo + hi) >> 1; if (sa[md] <= a) lo = md + 1; else hi = md; }
    s_g1 = lo;
    s_k = (uint32_t)(r - s_g0);
    s_prefix = 0;
  }
  __syncthreads();
  const int64_t g0 = s_g0, g1 = s_g1;
  uint32_t mask = 0;
  for (int shift = 24; shift >= 0; shift -= 8) {
    hist[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t prefix = s_prefix;
    for (int64_t j = g0 + threadIdx.x; j < g1; j += blockDim.x) {
      const uint32_t v = sb[j];
      if ((v & mask) == prefix) atomicAdd(&hist[(v >> shift) & 255u], 1u);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t k = s_k, d = 0;
      while (hist[d] <= k) { k -= hist[d]; ++d; }
      s_k = k;
      s_prefix = prefix | (d << shift);
    }
    mask |= 255u << shift;
    __syncthreads();
  }
  if (threadIdx.x == 0) keys[blockIdx.x] = ((uint64_t)a << 32) | s_prefix;
}

int ottohip_table_keys_at(ottohip_ctx* ctx, const ottohip_table* t, int rule, int use_ge2, const int64_t* idx,
                          int n_idx, uint64_t* keys, void* stream) {
  if (!ctx || !t || rule < 0 || rule >= t->n_rules || n_idx < 0 || (n_idx > 0 && (!idx || !keys))) {
    set_error("table_keys_at: bad args"); return OTTOHIP_EINVAL;
  }
  if (n_idx == 0) return 0;
  hipStream_t s = S(stream);
  Workspace& ws = ctx->ws;
  int64_t i0, n, nb;
  OH_TRY(rule_scan_blocks(t, rule, s, &i0, &n, &nb));
  uint32_t* bcnt;
  uint64_t *boff, *tot;
  OH_TRY(ws.get("blk_cnt", (size_t)nb, &bcnt));
  OH_TRY(ws.get("blk_off", (size_t)nb, &boff));
  OH_TRY(ws.get("fin_tot", 1, &tot));
  uint64_t m = 0;
  if (t->n_rows > 0 && n > 0) {
    // rows of the rule (use_ge2: per-file count >= 2, i.e. count_ge2 >= 1)
    k_blk_count<<<(unsigned)nb, FIN_T, 0, s>>>(t->b.rule, t->b.aid, t->b.aid_next, t->b.count, t->b.count_ge2, n, rule,
                                               use_ge2 ? 1 : 0, use_ge2 ? 1u : 0u, t->sym(rule), bcnt, i0);
    OH_TRY(exclusive_scan_u32(ctx, bcnt, boff, nb, tot, s));
    OH_TRY(d2h(&m, tot, 1, s));
  }
  for (int i = 0; i < n_idx; ++i)
    if (idx[i] < 0 || (uint64_t)idx[i] >= m) {
      set_error("table_keys_at: index %lld outside the rule's %llu rows", (long long)idx[i], (unsigned long long)m);
      return OTTOHIP_ERANGE;
    }
  uint32_t *sa, *sb, *k0, *v0, *k1, *v1;
  int64_t* didx;
  uint64_t* dkeys;
  OH_TRY(ws.get("fin_sa", (size_t)m, &sa));
  OH_TRY(ws.get("fin_sb", (size_t)m, &sb));
  OH_TRY(ws.get("fin_k0", (size_t)m, &k0));
  OH_TRY(ws.get("fin_v0", (size_t)m, &v0));
  OH_TRY(ws.get("fin_k1", (size_t)m, &k1));
  OH_TRY(ws.get("fin_v1", (size_t)m, &v1));
  OH_TRY(ws.get("ka_idx", (size_t)n_idx, &didx));
  OH_TRY(ws.get("ka_keys", (size_t)n_idx, &dkeys));
  k_blk_compact<<<(unsigned)nb, FIN_T, 0, s>>>(t->b.rule, t->b.aid, t->b.aid_next, t->b.count, t->b.count_ge2, n,
                                               rule, use_ge2 ? 1 : 0, use_ge2 ? 1u : 0u, t->sym(rule), boff, sa, sb,
                                               nullptr, nullptr, i0);
  OH_HIP(hipMemcpyAsync(didx, idx, (size_t)n_idx * sizeof(int64_t), hipMemcpyHostToDevice, s));
  if (!t->sym(rule)) {  // rows already in aid order (one count): a select per index, no sort
    int* uns;
    OH_TRY(ws.get("ka_uns", 1, &uns));
    OH_HIP(hipMemsetAsync(uns, 0, sizeof(int), s));
    k_sorted_check<<<grid_for((int64_t)m), 256, 0, s>>>(sa, (int64_t)m, uns);
    int hu = 1;
    OH_TRY(d2h(&hu, uns, 1, s));
    if (!hu) {
      k_keys_at_sel<<<(unsigned)n_idx, 256, 0, s>>>(sa, sb, (int64_t)m, didx, dkeys);
      OH_HIP(hipGetLastError());
      OH_TRY(d2h(keys, dkeys, (size_t)n_idx, s));
      return 0;
    }
  }
  // LSD: aid_next, then aid (stable) -> (aid, aid_next) ascending
  const int abits = std::max(1, bits_for((uint64_t)t->n_items));
  uint32_t *k = k0, *v = v0;
  k_iota_key<<<grid_for((int64_t)m), 256, 0, s>>>(sb, (int64_t)m, k, v);
  OH_TRY(radix_sort_pairs(ctx, k, v, k == k0 ? k1 : k0, v == v0 ? v1 : v0, (int64_t)m, abits, s));
  uint32_t* kn = (k == k0) ? k1 : k0;
  k_gather_key<<<grid_for((int64_t)m), 256, 0, s>>>(sa, v, (int64_t)m, 0, kn);
  k = kn;
  OH_TRY(radix_sort_pairs(ctx, k, v, k == k0 ? k1 : k0, v == v0 ? v1 : v0, (int64_t)m, abits, s));
  k_keys_at<<<grid_for(n_idx), 256, 0, s>>>(v, sa, sb, didx, n_idx, dkeys);
  OH_HIP(hipGetLastError());
  OH_TRY(d2h(keys, dkeys, (size_t)n_idx, s));
  return 0;
}

int ottohip_table_keys_at_parts(ottohip_ctx* ctx, const ottohip_table* t, int n_parts, int use_ge2,
                                const int64_t* idx, const int32_t* n_idx, uint64_t* keys, void* stream) {
  if (!ctx || !t || !n_idx || n_parts < 1 || n_parts > t->n_rules) {
    set_error("table_keys_at_parts: bad args"); return OTTOHIP_EINVAL;
  }
  int64_t total = 0;
  for (int p = 0; p < n_parts; ++p) {
    if (n_idx[p] < 0) { set_error("table_keys_at_parts: n_idx[%d] < 0", p); return OTTOHIP_EINVAL; }
    total += n_idx[p];
  }
  if (total == 0) return 0;
  if (!idx || !keys) { set_error("table_keys_at_parts: NULL idx / keys"); return OTTOHIP_EINVAL; }
  bool one_pass = n_parts <= KP_MAXP && t->aid_ordered;
  for (int p = 0; p < n_parts; ++p) one_pass = one_pass && !t->sym(p);
  auto per_part = [&]() -> int {  // each part on its own (ottohip_table_keys_at)
    int64_t o = 0;
    for (int p = 0; p < n_parts; ++p) {
      if (n_idx[p]) OH_TRY(ottohip_table_keys_at(ctx, t, p, use_ge2, idx + o, n_idx[p], keys + o, stream));
      o += n_idx[p];
    }
    return 0;
  };
  if (!one_pass) return per_part();
  hipStream_t s = S(stream);
  Workspace& ws = ctx->ws;
  const int64_t n = t->n_slots;
  const int64_t nb = ceil_div(std::max<int64_t>(n, 1), FIN_B);
  uint32_t* bcnt;
  uint64_t *boff, *seg;
  OH_TRY(ws.get("kp_cnt", (size_t)(n_parts * nb), &bcnt));
  OH_TRY(ws.get("kp_off", (size_t)(n_parts * nb + 1), &boff));
  OH_TRY(ws.get("kp_seg", (size_t)n_parts + 1, &seg));
  std::vector<uint64_t> sg(n_parts + 1, 0);
  if (t->n_rows > 0 && n > 0) {
    const uint32_t thr = use_ge2 ? 1u : 0u;
    k_blk_parts<false><<<(unsigned)nb, FIN_T, 0, s>>>(t->b.rule, t->b.aid, t->b.aid_next, t->b.count, t->b.count_ge2, n,
                                                      n_parts, use_ge2 ? 1 : 0, thr, nb, bcnt, nullptr, nullptr, nullptr);
    OH_TRY(exclusive_scan_u32(ctx, bcnt, boff, n_parts * nb, boff + n_parts * nb, s));
    k_part_seg<<<1, 64, 0, s>>>(boff, nb, n_parts, seg);
    OH_TRY(d2h(sg.data(), seg, (size_t)n_parts + 1, s));
  }
  {
    int64_t o = 0;
    for (int p = 0; p < n_parts; ++p) {
      const uint64_t m = sg[p + 1] - sg[p];
      for (int64_t j = o; j < o + n_idx[p]; ++j)
        if (idx[j] < 0 || (uint64_t)idx[j] >= m) {
          set_error("table_keys_at_parts: index %lld outside part %d's %llu rows", (long long)idx[j], p,
                    (unsigned long long)m);
          return OTTOHIP_ERANGE;
        }
      o += n_idx[p];
    }
  }
  const uint64_t mt = sg[n_parts];
  uint32_t *sa, *sb;
  int64_t* didx;
  uint64_t* dkeys;
  int* uns;
  OH_TRY(ws.get("fin_sa", (size_t)mt, &sa));
  OH_TRY(ws.get("fin_sb", (size_t)mt, &sb));
  OH_TRY(ws.get("ka_idx", (size_t)total, &didx));
  OH_TRY(ws.get("ka_keys", (size_t)total, &dkeys));
  OH_TRY(ws.get("ka_uns", 1, &uns));
  const uint32_t thr = use_ge2 ? 1u : 0u;
  k_blk_parts<true><<<(unsigned)nb, FIN_T, 0, s>>>(t->b.rule, t->b.aid, t->b.aid_next, t->b.count, t->b.count_ge2, n,
                                                   n_parts, use_ge2 ? 1 : 0, thr, nb, nullptr, boff, sa, sb);
  OH_HIP(hipMemcpyAsync(didx, idx, (size_t)total * sizeof(int64_t), hipMemcpyHostToDevice, s));
  OH_HIP(hipMemsetAsync(uns, 0, sizeof(int), s));
  for (int p = 0; p < n_parts; ++p) {
    const int64_t m = (int64_t)(sg[p + 1] - sg[p]);
    if (m > 1) k_sorted_check<<<grid_for(m), 256, 0, s>>>(sa + sg[p], m, uns);
  }
  int hu = 1;
  OH_TRY(d2h(&hu, uns, 1, s));
  if (hu) return per_part();  // a part's rows not in aid order: the sort path per part
  int64_t o = 0;
  for (int p = 0; p < n_parts; ++p) {
    if (n_idx[p])
      k_keys_at_sel<<<(unsigned)n_idx[p], 256, 0, s>>>(sa + sg[p], sb + sg[p], (int64_t)(sg[p + 1] - sg[p]), didx + o,
                                                      dkeys + o);
    o += n_idx[p];
  }
  OH_HIP(hipGetLastError());
  OH_TRY(d2h(keys, dkeys, (size_t)total, s));
  return 0;
}

void ottohip_table_free(ottohip_table* t) {
  if (!t) return;
  (void)hipSetDevice(t->device);
  (void)hipDeviceSynchronize();
  if (t->ctx && t->b.cap > t->ctx->spare.cap) {  // keep the larger buffer set for the next call
    t->ctx->spare.release();
    t->ctx->spare = t->b;
  } else {
    t->b.release();
  }
  kept_free(t->kept);
  dev_free(t->type_slots_dev);
  if (t->produced) (void)hipEventDestroy(t->produced);
  delete t;
}

}  // extern "C"

extern "C" int ottohip_table_part_heads(ottohip_ctx* ctx, const ottohip_table* t, int n_parts, int use_ge2,
                                        int32_t min_count, int64_t max_rows_part, void* out_records, int64_t cap,
                                        int64_t* n_out, void* stream) {
  if (!ctx || !t || !n_out || n_parts < 1 || n_parts > PH_MAXP || n_parts > t->n_rules || max_rows_part < 0 ||
      (cap > 0 && !out_records) || t->sym_mask) {
    set_error("table_part_heads: bad arguments (n_parts in [1, %d], a part-mode table)", PH_MAXP); return OTTOHIP_EINVAL;
  }
  *n_out = 0;
  if (t->n_rows == 0 || t->n_slots == 0 || max_rows_part == 0) return 0;
  hipStream_t s = S(stream);
  OH_HIP(hipSetDevice(ctx->device));
  Workspace& ws = ctx->ws;
  const int64_t n = t->n_slots;
  const uint32_t thr = (uint32_t)std::max<int32_t>(min_count, 1);
  const unsigned sgrid = (unsigned)std::min<int64_t>(ceil_div(n, 256 * SLOTS_T), (int64_t)ctx->n_cu * 16);
  // (1) v histogram per part
  unsigned long long* hist;
  OH_TRY(ws.get("ph_hist", (size_t)n_parts * PH_VBINS, &hist));
  OH_HIP(hipMemsetAsync(hist, 0, (size_t)n_parts * PH_VBINS * 8, s));
  k_ph_hist<<<sgrid, 256, 0, s>>>(t->b.rule, t->b.count, t->b.count_ge2, n, n_parts, use_ge2, thr, hist);
  std::vector<unsigned long long> hh((size_t)n_parts * PH_VBINS);
  OH_TRY(d2h(hh.data(), hist, hh.size(), s));
  PartCut pc;
  memset(&pc, 0, sizeof pc);
  std::vector<uint64_t> need(n_parts, 0);
  int n_tie = 0;
  for (int p = 0; p < n_parts; ++p) {
    const unsigned long long* h = hh.data() + (size_t)p * PH_VBINS;
    unsigned long long above = 0;
    pc.cstar[p] = 0; pc.astar[p] = 0xFFFFFFFFu; pc.stage[p] = 0;
    int64_t v = PH_VBINS - 1;
    for (; v >= (int64_t)thr; --v) {
      if (above + h[v] >= (unsigned long long)max_rows_part) break;
      above += h[v];
    }
    if (v < (int64_t)thr) continue;  // the part has at most max_rows_part rows: all kept
    if (v == PH_VBINS - 1) { set_error("table_part_heads: a part's cut count >= %u", PH_VBINS - 1); return OTTOHIP_ELIMIT; }
    pc.cstar[p] = (uint32_t)v;
    need[p] = (uint64_t)max_rows_part - above;  // 1 <= need <= h[v]
    if (need[p] < h[v]) { pc.stage[p] = 1; ++n_tie; }  // ties at c*: cut by (aid, aid_next)
  }
  const int64_t ni = t->n_items;
  if (n_tie && !t->aid_ordered) {
    // stage 1 (a*) on slots not in aid order: a histogram over the aids of each part's tie rows, then the aid
    // where the tie rows' running count reaches the rank left
    int nq = 0;
    std::vector<int> qpart;
    for (int p = 0; p < n_parts; ++p)
      if (pc.stage[p] == 1u) { qpart.push_back(p); ++nq; }
    uint32_t *ah, *found;
    uint64_t* ex;
    OH_TRY(ws.get("ph_aid_hist", (size_t)nq * ni, &ah));
    OH_TRY(ws.get("ph_tie_ex", (size_t)ni, &ex));
    OH_TRY(ws.get("ph_found", 2 * PH_MAXP, &found));
    OH_HIP(hipMemsetAsync(ah, 0, (size_t)nq * ni * 4, s));
    k_ph_tie_aid_hist<<<sgrid, 256, 0, s>>>(t->b.rule, t->b.aid, t->b.count, t->b.count_ge2, n, n_parts, use_ge2, pc, ni,
                                            ah);
    for (int q = 0; q < nq; ++q) {
      const int p = qpart[q];
      OH_TRY(exclusive_scan_u32(ctx, ah + (size_t)q * ni, ex, ni, nullptr, s));
      OH_HIP(hipMemsetAsync(found, 0xFF, 8, s));
      k_ph_find<<<grid_for(ni), 256, 0, s>>>(ex, ah + (size_t)q * ni, ni, need[p], found);
      uint32_t fr[2];
      OH_TRY(d2h(fr, found, 2, s));
      if (fr[0] == 0xFFFFFFFFu) { set_error("table_part_heads: tie cut not found (part %d)", p); return OTTOHIP_EHIP; }
      pc.astar[p] = fr[0];
      pc.stage[p] = 2;
    }
  }
  // the rank pass' per-block counts (aid-ordered tables with tie cuts): k_ph_count then reads only the blocks of the
  // cut aids' ranges
  uint32_t *rk_cnt = nullptr, *rk_sure = nullptr, *rk_rng = nullptr;
  int rk_nq = 0;
  int64_t rk_lo = -1, rk_hi = -1;
  if (n_tie) {
    // stage 1 (a*): rank search over the parts' tie rows in slot order (= aid order)
    const int64_t nb1 = ceil_div(n, FIN_B);
    PhRank rk;
    memset(&rk, 0, sizeof rk);
    int nq = 0;
    for (int p = 0; p < n_parts; ++p)
      if (pc.stage[p] == 1u) { rk.need[nq] = need[p]; rk.part[nq] = (uint32_t)p; ++nq; }
    uint32_t* found;
    OH_TRY(ws.get("ph_found", 2 * PH_MAXP, &found));
    // stage 2 on an aid-ordered table scans only the blocks that can hold the cut aid (per-block first / last aids from
    // the rank pass); OTTOHIP_PH_FULL=1: the full-table stage-2 pass (A/B switch, read per call)
    const bool ranged = t->aid_ordered && !(getenv("OTTOHIP_PH_FULL") && !strcmp(getenv("OTTOHIP_PH_FULL"), "1"));
    std::vector<int64_t> rlo(PH_MAXP, -1), rhi(PH_MAXP, -1);
    std::vector<uint64_t> lbase(PH_MAXP, 0);
    if (nq > 0) {  // (none left when the unordered table's stage 1 above took every tie part)
    uint32_t *rcnt, *astar, *baid = nullptr, *sure = nullptr;
    uint64_t* rex;
    OH_TRY(ws.get("ph_rank_cnt", (size_t)nq * nb1, &rcnt));
    OH_TRY(ws.get("ph_rank_ex", (size_t)nq * nb1, &rex));
    OH_TRY(ws.get("ph_astar", PH_MAXP, &astar));
    if (ranged) {
      OH_TRY(ws.get("ph_baid", (size_t)2 * nb1, &baid));
      OH_TRY(ws.get("ph_sure", (size_t)nb1, &sure));
    }
    k_ph_rank_count<<<(unsigned)nb1, FIN_T, 0, s>>>(t->b.rule, t->b.count, t->b.count_ge2, n, n_parts, use_ge2, pc, nb1,
                                                     rcnt, t->b.aid, baid, thr, sure);
    if (ranged) { rk_cnt = rcnt; rk_sure = sure; rk_nq = nq; }
    OH_TRY(exclusive_scan_u32(ctx, rcnt, rex, nq * nb1, nullptr, s));
    OH_HIP(hipMemsetAsync(found, 0xFF, 2 * PH_MAXP * 4, s));
    OH_HIP(hipMemsetAsync(astar, 0xFF, PH_MAXP * 4, s));
    k_ph_find_multi<<<grid_for(nq * nb1), 256, 0, s>>>(rex, rcnt, nb1, nq, rk, found);
    k_ph_tie_pick<<<(unsigned)nq, FIN_T, 0, s>>>(t->b.rule, t->b.aid, t->b.count, t->b.count_ge2, n, n_parts, use_ge2, pc,
                                                  rk, found, astar);
    uint32_t as[PH_MAXP];
    OH_TRY(d2h(as, astar, (size_t)nq, s));
    for (int q = 0; q < nq; ++q) {
      const int p = (int)rk.part[q];
      if (as[q] == 0xFFFFFFFFu) { set_error("table_part_heads: tie cut not found (part %d)", p); return OTTOHIP_EHIP; }
      pc.astar[p] = as[q];
      pc.stage[p] = 2;
    }
    if (ranged) {
      // the block range of each cut aid; the tie rows before it (all with aid < a*) from the rank scan
      uint32_t* rng;
      OH_TRY(ws.get("ph_range", (size_t)2 * PH_MAXP, &rng));
      std::vector<uint32_t> rinit(2 * PH_MAXP);
      for (int q = 0; q < PH_MAXP; ++q) { rinit[2 * q] = 0xFFFFFFFFu; rinit[2 * q + 1] = 0u; }
      OH_HIP(hipMemcpyAsync(rng, rinit.data(), rinit.size() * 4, hipMemcpyHostToDevice, s));
      k_ph_aid_range<<<grid_for(nb1 * nq), 256, 0, s>>>(baid, nb1, nq, astar, rng);
      rk_rng = rng;
      std::vector<uint32_t> rh(2 * nq);
      OH_TRY(d2h(rh.data(), rng, rh.size(), s));  // (synchronizes: rinit stays valid until here)
      for (int q = 0; q < nq; ++q) {
        const int p = (int)rk.part[q];
        if (rh[2 * q] == 0xFFFFFFFFu || rh[2 * q + 1] < rh[2 * q]) {
          set_error("table_part_heads: cut aid range not found (part %d)", p); return OTTOHIP_EHIP;
        }
        rlo[p] = rh[2 * q]; rhi[p] = rh[2 * q + 1];
        rk_lo = rk_lo < 0 ? rlo[p] : std::min<int64_t>(rk_lo, rlo[p]);
        rk_hi = std::max<int64_t>(rk_hi, rhi[p]);
        uint64_t e2[2];
        OH_TRY(d2h(&e2[0], rex + (size_t)q * nb1 + rlo[p], 1, s));
        OH_TRY(d2h(&e2[1], rex + (size_t)q * nb1, 1, s));
        lbase[p] = e2[0] - e2[1];
      }
    }
    }
    // stage 2 (n*): aid_next histogram of the (c*, a*) tie rows; the rank left = need - ties with aid < a*
    uint32_t* th;
    uint64_t *ex, *lt;
    OH_TRY(ws.get("ph_tie", (size_t)n_parts * ni, &th));
    OH_TRY(ws.get("ph_tie_ex", (size_t)ni, &ex));
    OH_TRY(ws.get("ph_lt", PH_MAXP, &lt));
    OH_HIP(hipMemsetAsync(th, 0, (size_t)n_parts * ni * 4, s));
    OH_HIP(hipMemsetAsync(lt, 0, PH_MAXP * 8, s));
    bool all_ranged = ranged;
    for (int p = 0; p < n_parts; ++p)
      if (pc.stage[p] == 2u && rlo[p] < 0) all_ranged = false;
    if (all_ranged) {
      for (int p = 0; p < n_parts; ++p) {
        if (pc.stage[p] != 2u) continue;
        const int64_t a0 = rlo[p] * FIN_B, a1 = std::min<int64_t>(n, (rhi[p] + 1) * FIN_B);
        const unsigned g = (unsigned)std::max<int64_t>(1, std::min<int64_t>(ceil_div(a1 - a0, 256 * SLOTS_T), sgrid));
        k_ph_tie_hist2<<<g, 256, 0, s>>>(t->b.rule, t->b.aid, t->b.aid_next, t->b.count, t->b.count_ge2, a1, n_parts,
                                         use_ge2, pc, ni, th, reinterpret_cast<unsigned long long*>(lt), a0, p);
      }
    } else {
      k_ph_tie_hist2<<<sgrid, 256, 0, s>>>(t->b.rule, t->b.aid, t->b.aid_next, t->b.count, t->b.count_ge2, n, n_parts,
                                           use_ge2, pc, ni, th, reinterpret_cast<unsigned long long*>(lt));
    }
    uint64_t lth[PH_MAXP];
    OH_TRY(d2h(lth, lt, PH_MAXP, s));
    if (all_ranged)
      for (int p = 0; p < n_parts; ++p)
        if (pc.stage[p] == 2u) lth[p] += lbase[p];
    for (int p = 0; p < n_parts; ++p) {
      if (pc.stage[p] != 2u) continue;
      if (lth[p] >= need[p]) { set_error("table_part_heads: tie rank below the cut aid (part %d)", p); return OTTOHIP_EHIP; }
      OH_TRY(exclusive_scan_u32(ctx, th + (size_t)p * ni, ex, ni, nullptr, s));
      OH_HIP(hipMemsetAsync(found, 0xFF, 8, s));
      k_ph_find<<<grid_for(ni), 256, 0, s>>>(ex, th + (size_t)p * ni, ni, need[p] - lth[p], found);
      uint32_t fr[2];
      OH_TRY(d2h(fr, found, 2, s));
      if (fr[0] == 0xFFFFFFFFu) { set_error("table_part_heads: tie cut not found (part %d)", p); return OTTOHIP_EHIP; }
      pc.nstar[p] = fr[0];
      pc.stage[p] = 3;
    }
  }
  // (2) kept rows of every part -> records (a single pass with a decoupled look-back over the tiles measured 98 ms
  // against 3.9 + 8 ms for count, scan, compact: agent-scope status reads cross the XCDs at ~0.2 us a tile)
  const int64_t nb = ceil_div(n, FIN_B);
  uint32_t* bcnt;
  uint64_t *boff, *tot;
  OH_TRY(ws.get("blk_cnt", (size_t)nb, &bcnt));
  OH_TRY(ws.get("blk_off", (size_t)nb, &boff));
  OH_TRY(ws.get("fin_tot", 1, &tot));
  if (rk_sure && rk_rng && rk_lo >= 0 && rk_nq > 0) {
    // the rank pass' counts outside the cut aids' ranges, the exact count inside them
    uint32_t* inr;
    OH_TRY(ws.get("ph_inrange", (size_t)nb, &inr));
    k_ph_combine<<<grid_for(nb), 256, 0, s>>>(rk_sure, rk_cnt, nb, rk_nq, rk_rng, bcnt, inr);
    k_ph_count<<<(unsigned)(rk_hi - rk_lo + 1), FIN_T, 0, s>>>(t->b.rule, t->b.aid, t->b.aid_next, t->b.count,
                                                               t->b.count_ge2, n, n_parts, use_ge2, thr, pc, bcnt, rk_lo, inr);
  } else {
    k_ph_count<<<(unsigned)nb, FIN_T, 0, s>>>(t->b.rule, t->b.aid, t->b.aid_next, t->b.count, t->b.count_ge2, n, n_parts,
                                              use_ge2, thr, pc, bcnt);
  }
  OH_TRY(exclusive_scan_u32(ctx, bcnt, boff, nb, tot, s));
  uint64_t m = 0;
  OH_TRY(d2h(&m, tot, 1, s));
  if ((int64_t)m > cap) { set_error("table_part_heads: %llu rows > capacity %lld", (unsigned long long)m, (long long)cap); return OTTOHIP_ELIMIT; }
  if (m) k_ph_compact<<<(unsigned)nb, FIN_T, 0, s>>>(t->b.rule, t->b.aid, t->b.aid_next, t->b.count, t->b.count_ge2, n,
                                                      n_parts, use_ge2, thr, pc, boff, reinterpret_cast<uint4*>(out_records));
  OH_HIP(hipGetLastError());
  *n_out = (int64_t)m;
  return 0;
}

extern "C" int ottohip_table_finalize(ottohip_ctx* ctx, const ottohip_table* t, int rule,
                                      const ottohip_merge_params* mp, int32_t* aid, int32_t* aid_next,
                                      int32_t* count, int64_t* n_out, void* stream) {
  if (!ctx || !t || !mp || !n_out || rule < 0 || rule >= t->n_rules) { set_error("finalize: bad args"); return OTTOHIP_EINVAL; }
  *n_out = 0;
  hipStream_t s = S(stream);
  OH_TRY(ensure_part_stats(t));
  const ottohip_rule_stats& st = t->stats[rule];
  const bool use_ge2 = mp->click_rule && st.file_rows > mp->filter_rows;
  const int64_t n_after = use_ge2 ? st.file_rows_ge2 : st.file_rows;
  if (use_ge2 && mp->min_count_in_part != 2) {  // count_ge2 is accumulated with the per-file threshold 2
    set_error("finalize: min_count_in_part=%d, but the table's per-file filter column is count >= 2",
              (int)mp->min_count_in_part);
    return OTTOHIP_EINVAL;
  }
  if (n_after > mp->max_rows_groupby) {
    set_error("rule %d: %lld per-file rows > %lld: the reference's part-wise branch (count_co_events.py:135-166) "
              "is not implemented on the device", rule, (long long)n_after, (long long)mp->max_rows_groupby);
    return OTTOHIP_ELIMIT;
  }
  if (t->n_rows == 0) return 0;
  const uint32_t thr = (uint32_t)std::max<int32_t>(mp->min_count, 1);
  Workspace& ws = ctx->ws;
  int64_t i0, n, nb;  // only the rule's row type's slots
  OH_TRY(rule_scan_blocks(t, rule, s, &i0, &n, &nb));
  uint32_t* bcnt;
  uint64_t *boff, *tot;
  OH_TRY(ws.get("blk_cnt", (size_t)nb, &bcnt));
  OH_TRY(ws.get("blk_off", (size_t)nb, &boff));
  OH_TRY(ws.get("fin_tot", 1, &tot));
  k_blk_count<<<(unsigned)nb, FIN_T, 0, s>>>(t->b.rule, t->b.aid, t->b.aid_next, t->b.count, t->b.count_ge2, n, rule,
                                             use_ge2 ? 1 : 0, thr, t->sym(rule), bcnt, i0);
  OH_TRY(exclusive_scan_u32(ctx, bcnt, boff, nb, tot, s));
  uint64_t m = 0;
  OH_TRY(d2h(&m, tot, 1, s));
  if (m == 0) return 0;
  uint32_t *sa, *sb, *sc, *k0, *v0, *k1, *v1;
  OH_TRY(ws.get("fin_sa", (size_t)m, &sa));
  OH_TRY(ws.get("fin_sb", (size_t)m, &sb));
  OH_TRY(ws.get("fin_sc", (size_t)m, &sc));
  OH_TRY(ws.get("fin_k0", (size_t)m, &k0));
  OH_TRY(ws.get("fin_v0", (size_t)m, &v0));
  OH_TRY(ws.get("fin_k1", (size_t)m, &k1));
  OH_TRY(ws.get("fin_v1", (size_t)m, &v1));
  k_blk_compact<<<(unsigned)nb, FIN_T, 0, s>>>(t->b.rule, t->b.aid, t->b.aid_next, t->b.count, t->b.count_ge2, n,
                                               rule, use_ge2 ? 1 : 0, thr, t->sym(rule), boff, sa, sb, sc, nullptr, i0);
  // LSD: aid_next asc, then aid asc, then count desc (stable) -> (count desc, aid, aid_next);
  // aids are < n_items, so their passes cover bits_for(n_items) bits (3 x 8 at 1.86 M items)
  const int abits = std::max(1, bits_for((uint64_t)t->n_items));
  uint32_t *k = k0, *v = v0;
  k_iota_key<<<grid_for((int64_t)m), 256, 0, s>>>(sb, (int64_t)m, k, v);
  OH_TRY(radix_sort_pairs(ctx, k, v, k == k0 ? k1 : k0, v == v0 ? v1 : v0, (int64_t)m, abits, s));
  uint32_t* kn = (k == k0) ? k1 : k0;
  k_gather_key<<<grid_for((int64_t)m), 256, 0, s>>>(sa, v, (int64_t)m, 0, kn);
  k = kn;
  OH_TRY(radix_sort_pairs(ctx, k, v, k == k0 ? k1 : k0, v == v0 ? v1 : v0, (int64_t)m, abits, s));
  kn = (k == k0) ? k1 : k0;
  k_gather_key<<<grid_for((int64_t)m), 256, 0, s>>>(sc, v, (int64_t)m, 1, kn);
  k = kn;
  OH_TRY(radix_sort_pairs(ctx, k, v, k == k0 ? k1 : k0, v == v0 ? v1 : v0, (int64_t)m, 32, s));
  const int64_t keep = std::min<int64_t>((int64_t)m, mp->max_rows);
  k_fin_out<<<grid_for(keep), 256, 0, s>>>(v, keep, sa, sb, sc, aid, aid_next, count);
  OH_HIP(hipGetLastError());
  *n_out = keep;
  return 0;
}

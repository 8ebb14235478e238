// R1: per-aid top-N of a final co-visitation table with the reference's features
// (get_df_count_for_co_event_type, model/retrieve.py:18-63):
//   count_pop = Int16(min((c - min c) / (q - min c), 1) * 1e4), q = quantile(count, 0.9999)
//               with polars' default 'nearest' interpolation: sorted_asc[round((n - 1) * q)]  (:34-36)
//   perc_pop  = Int16(row_nr / n * 1e4), row_nr = 1-based position in FILE order              (:37-38)
//   rank      = ordinal rank of count (desc) within aid; ties by file order                    (:44)
//   count_rel = Int8(c / max_c(aid) * 100)                                                      (:45-49)
// rows with rank <= first_n, in (aid asc, rank asc) order. All f64 arithmetic as polars does it
// (integer operands promoted to f64, casts truncate toward zero).
#include <algorithm>
#include <cmath>
#include "prims.h"
#include "table.h"

namespace ottohip {

// count desc, stable on file order: key = ~count (counts are >= 0)
__global__ void k_r1_count_key(const int32_t* __restrict__ count, int64_t n, uint32_t* __restrict__ key,
                               uint32_t* __restrict__ val, int* __restrict__ err) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int32_t c = count[i];
  if (c < 0) atomicOr(err, 1);
  key[i] = ~(uint32_t)c;
  val[i] = (uint32_t)i;
}

__global__ void k_r1_aid_key(const int32_t* __restrict__ aid, const uint32_t* __restrict__ val, int64_t n,
                             uint32_t n_items, uint32_t* __restrict__ key, int* __restrict__ err) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int32_t a = aid[val[i]];
  if (a < 0 || (uint32_t)a >= n_items) atomicOr(err, 2);
  key[i] = (uint32_t)a;
}

// heads of aid groups in (aid, count desc, file order) order
__global__ void k_r1_heads(const uint32_t* __restrict__ key, int64_t n, uint32_t* __restrict__ head) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  head[i] = (i == 0 || key[i] != key[i - 1]) ? 1u : 0u;
}

// group start position of every sorted row (heads write theirs, others look it up by group id)
__global__ void k_r1_group_start(const uint32_t* __restrict__ head, const uint64_t* __restrict__ gid, int64_t n,
                                 uint32_t* __restrict__ gstart) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || !head[i]) return;
  gstart[gid[i]] = (uint32_t)i;
}

__global__ void k_r1_keep(const uint32_t* __restrict__ head, const uint64_t* __restrict__ gid,
                          const uint32_t* __restrict__ gstart, int64_t n, int first_n, uint32_t* __restrict__ keep) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t g = gid[i] + head[i] - 1;  // gid is the exclusive scan of head
  keep[i] = (i - (int64_t)gstart[g] + 1) <= first_n ? 1u : 0u;
}

__global__ void k_r1_out(const uint32_t* __restrict__ val, const uint32_t* __restrict__ head,
                         const uint64_t* __restrict__ gid, const uint32_t* __restrict__ gstart,
                         const uint32_t* __restrict__ keep, const uint64_t* __restrict__ oidx, int64_t n,
                         const int32_t* __restrict__ aid, const int32_t* __restrict__ aid_next,
                         const int32_t* __restrict__ count, int32_t cmin, int32_t q, double n_rows,
                         int32_t* __restrict__ o_aid, int32_t* __restrict__ o_next, int32_t* __restrict__ o_cnt,
                         int16_t* __restrict__ o_pop, int16_t* __restrict__ o_perc, int16_t* __restrict__ o_rank,
                         int8_t* __restrict__ o_rel) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || !keep[i]) return;
  const uint32_t src = val[i];
  const uint64_t g = gid[i] + head[i] - 1;
  const uint32_t g0 = gstart[g];
  const int32_t c = count[src];
  const int32_t cmax = count[val[g0]];
  const uint64_t o = oidx[i];
  o_aid[o] = aid[src];
  o_next[o] = aid_next[src];
  o_cnt[o] = c;
  // :34-36  ((c - min) / (q - min)).clip_max(1) * 10000 -> Int16
  double pop = (double)(c - cmin) / (double)(q - cmin);
  if (pop > 1.0) pop = 1.0;
  if (pop != pop) pop = 0.0;  // 0/0 when q == min (documented edge case)
  o_pop[o] = (int16_t)(pop * 10000.0);
  // :37-38  row_nr / count * 10000 -> Int16, row_nr 1-based in file order
  o_perc[o] = (int16_t)((double)(src + 1) / n_rows * 10000.0);
  o_rank[o] = (int16_t)(i - (int64_t)g0 + 1);
  o_rel[o] = (int8_t)((double)c / (double)cmax * 100.0);
}

}  // namespace ottohip

using namespace ottohip;

extern "C" int ottohip_topk_per_aid(ottohip_ctx* ctx, const int32_t* aid, const int32_t* aid_next,
                                    const int32_t* count, int64_t n, int32_t n_items, int first_n,
                                    int32_t* o_aid, int32_t* o_next, int32_t* o_cnt, int16_t* o_pop,
                                    int16_t* o_perc, int16_t* o_rank, int8_t* o_rel, int64_t* n_out,
                                    void* stream) {
  if (!ctx || !n_out || n < 0 || first_n < 0 || n_items < 1 ||
      (n > 0 && (!aid || !aid_next || !count || !o_aid || !o_next || !o_cnt || !o_pop || !o_perc || !o_rank || !o_rel))) {
    set_error("topk_per_aid: bad arguments");
    return OTTOHIP_EINVAL;
  }
  if (n >= ((int64_t)1 << 32)) { set_error("topk_per_aid: n >= 2^32"); return OTTOHIP_ELIMIT; }
  *n_out = 0;
  if (n == 0 || first_n == 0) return 0;
  hipStream_t s = S(stream);
  OH_HIP(hipSetDevice(ctx->device));
  Workspace& ws = ctx->ws;
  uint32_t *k0, *v0, *k1, *v1, *head, *gstart, *keep;
  uint64_t *gid, *oidx, *tot;
  int* err;
  OH_TRY(ws.get("r1_k0", (size_t)n, &k0));
  OH_TRY(ws.get("r1_v0", (size_t)n, &v0));
  OH_TRY(ws.get("r1_k1", (size_t)n, &k1));
  OH_TRY(ws.get("r1_v1", (size_t)n, &v1));
  OH_TRY(ws.get("r1_head", (size_t)n, &head));
  OH_TRY(ws.get("r1_gstart", (size_t)n, &gstart));
  OH_TRY(ws.get("r1_keep", (size_t)n, &keep));
  OH_TRY(ws.get("r1_gid", (size_t)n, &gid));
  OH_TRY(ws.get("r1_oidx", (size_t)n, &oidx));
  OH_TRY(ws.get("r1_tot", 2, &tot));
  OH_TRY(ws.get("r1_err", 1, &err));
  int ph = ctx->begin("topk_per_aid", s, 12.0 * n);
  OH_HIP(hipMemsetAsync(err, 0, sizeof(int), s));
  k_r1_count_key<<<grid_for(n), 256, 0, s>>>(count, n, k0, v0, err);
  uint32_t *k = k0, *v = v0;
  OH_TRY(radix_sort_pairs(ctx, k, v, k1, v1, n, 32, s));
  // min and the 0.9999 quantile (nearest) from the count-desc order: asc[j] = desc[n - 1 - j]
  // polars 'nearest': idx = ((n - 1) * q).round() (f64::round: half away from zero) into the sorted values
  const int64_t qi = (int64_t)std::llround((double)(n - 1) * 0.9999);
  uint32_t kmin = 0, kq = 0;
  OH_TRY(d2h(&kmin, k + (n - 1), 1, s));
  OH_TRY(d2h(&kq, k + (n - 1 - qi), 1, s));
  const int32_t cmin = (int32_t)~kmin, q = (int32_t)~kq;
  uint32_t* kn = (k == k0) ? k1 : k0;
  k_r1_aid_key<<<grid_for(n), 256, 0, s>>>(aid, v, n, (uint32_t)n_items, kn, err);
  k = kn;
  OH_TRY(radix_sort_pairs(ctx, k, v, k == k0 ? k1 : k0, v == v0 ? v1 : v0, n, std::max(1, bits_for((uint64_t)n_items)), s));
  k_r1_heads<<<grid_for(n), 256, 0, s>>>(k, n, head);
  OH_TRY(exclusive_scan_u32(ctx, head, gid, n, tot, s));
  k_r1_group_start<<<grid_for(n), 256, 0, s>>>(head, gid, n, gstart);
  k_r1_keep<<<grid_for(n), 256, 0, s>>>(head, gid, gstart, n, first_n, keep);
  OH_TRY(exclusive_scan_u32(ctx, keep, oidx, n, tot + 1, s));
  k_r1_out<<<grid_for(n), 256, 0, s>>>(v, head, gid, gstart, keep, oidx, n, aid, aid_next, count, cmin, q, (double)n,
                                       o_aid, o_next, o_cnt, o_pop, o_perc, o_rank, o_rel);
  OH_HIP(hipGetLastError());
  ctx->end(ph, s);
  uint64_t tt[2];
  int herr = 0;
  OH_TRY(d2h(tt, tot, 2, s));
  OH_TRY(d2h(&herr, err, 1, s));
  if (herr) { set_error("topk_per_aid: negative count or aid outside [0, n_items)"); return OTTOHIP_ERANGE; }
  *n_out = (int64_t)tt[1];
  return 0;
}

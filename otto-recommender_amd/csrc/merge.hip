// concat_files_w_stats over a list of finished tables (model/count_co_events.py:103-181) and
// the run histogram behind the sharded head cut.
//
//   ottohip_concat_tables : A6 on tables given as (aid, aid_next, count) columns concatenated in
//                           order -- the per-file tables of one folder, or the two thresholded
//                           folder tables of the train+test merge (A7, :218-226). Branch (2)
//                           slices rows of the concatenation exactly as the reference does.
//   ottohip_run_hist      : histogram of (x >> shift) & mask over a range of an array whose equal
//                           values are contiguous (a finalize output), two atomics per run.
#include <algorithm>
#include "prims.h"
#include "table.h"

namespace ottohip {

// flag[i] = row i of the table survives the per-row filter of :131-132 (count >= thr)
__global__ void k_ct_flag(const uint32_t* __restrict__ c, int64_t n, uint32_t thr, uint32_t* __restrict__ flag) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) flag[i] = c[i] >= thr ? 1u : 0u;
}

// surviving rows -> merge records {aid, aid_next, count, count} at their compacted positions
// (the record format of ottohip_table_from_records, rule 0)
__global__ void k_ct_pack(const int32_t* __restrict__ a, const int32_t* __restrict__ b, const uint32_t* __restrict__ c,
                          int64_t n, const uint32_t* __restrict__ flag, const uint64_t* __restrict__ idx,
                          uint4* __restrict__ rec) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || (flag && !flag[i])) return;
  const uint64_t p = flag ? idx[i] : (uint64_t)i;
  const uint32_t v = c[i];
  rec[p] = make_uint4((uint32_t)a[i], (uint32_t)b[i], v, v);
}

__global__ void k_out_records(const int32_t* __restrict__ a, const int32_t* __restrict__ b,
                              const int32_t* __restrict__ c, int64_t n, uint4* __restrict__ rec) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t v = (uint32_t)c[i];
  rec[i] = make_uint4((uint32_t)a[i], (uint32_t)b[i], v, v);
}

// equal keys form one run: the run [s, e] adds e + 1 at its end and subtracts s at its start
__global__ void k_run_hist(const int32_t* __restrict__ x, int64_t lo, int64_t hi, int shift, uint32_t mask,
                           int64_t n_bins, unsigned long long* __restrict__ hist, int* __restrict__ err) {
  const int64_t i = lo + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= hi) return;
  const uint32_t k = ((uint32_t)x[i] >> shift) & mask;
  if ((int64_t)k >= n_bins) { atomicOr(err, 1); return; }
  if (i == lo || ((((uint32_t)x[i - 1]) >> shift) & mask) != k) atomicAdd(&hist[k], (unsigned long long)(0 - (uint64_t)i));
  if (i + 1 == hi || ((((uint32_t)x[i + 1]) >> shift) & mask) != k) atomicAdd(&hist[k], (unsigned long long)(i + 1));
}

// order-independent digest of one rule's rows (the oracle's per-file sums are linear, so they
// equal these without a merge; oracle/covis_oracle.c row_mix is the same function)
__device__ __forceinline__ uint64_t row_mix(uint64_t rule, uint32_t a, uint32_t b, uint64_t seed) {
  uint64_t x = ((rule << 48) | ((uint64_t)a << 24) | (uint64_t)b) ^ seed;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

__global__ __launch_bounds__(256) void k_table_digest(const uint8_t* __restrict__ rule, const int32_t* __restrict__ aid,
                                                      const int32_t* __restrict__ aid_next,
                                                      const uint32_t* __restrict__ count,
                                                      const uint32_t* __restrict__ count_ge2, int64_t n, int r,
                                                      int sym, unsigned long long* __restrict__ out) {
  uint64_t d[5] = {0, 0, 0, 0, 0};
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    if (rule[i] != (uint8_t)r) continue;
    const uint64_t c = count[i], g = count_ge2[i];
    const uint32_t a = (uint32_t)aid[i], b = (uint32_t)aid_next[i];
    d[0] += row_mix((uint64_t)r, a, b, 1) * c;
    d[1] += row_mix((uint64_t)r, a, b, 2) * g;
    d[2] += c; d[3] += g; d[4] += 1;
    if (sym && a != b) {  // the mirror (b, a) of a row stored once
      d[0] += row_mix((uint64_t)r, b, a, 1) * c;
      d[1] += row_mix((uint64_t)r, b, a, 2) * g;
      d[2] += c; d[3] += g; d[4] += 1;
    }
  }
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    const uint64_t v = wave_sum64(d[k]);
    if (lane_id() == 0 && v) atomicAdd(&out[k], (unsigned long long)v);
  }
}

}  // namespace ottohip

using namespace ottohip;

extern "C" int ottohip_concat_tables(ottohip_ctx* ctx, int n_tables, const int32_t* const* aid,
                                     const int32_t* const* aid_next, const uint32_t* const* count,
                                     const int64_t* n_rows, int32_t n_items, const ottohip_merge_params* mp,
                                     int64_t optim_rows, int loaded_from_cache, int32_t* out_aid,
                                     int32_t* out_aid_next, int32_t* out_count, int64_t* n_out, void* stream) {
  if (!ctx || n_tables < 0 || (n_tables > 0 && (!aid || !aid_next || !count || !n_rows)) || !mp || !n_out ||
      n_items < 1 || optim_rows < 1 || mp->max_rows < 0) {
    set_error("concat_tables: bad arguments");
    return OTTOHIP_EINVAL;
  }
  *n_out = 0;
  hipStream_t s = S(stream);
  OH_HIP(hipSetDevice(ctx->device));
  int64_t N = 0;
  for (int t = 0; t < n_tables; ++t) {
    if (n_rows[t] < 0 || (n_rows[t] > 0 && (!aid[t] || !aid_next[t] || !count[t]))) {
      set_error("concat_tables: table %d has bad columns", t);
      return OTTOHIP_EINVAL;
    }
    N += n_rows[t];
  }
  if (N >= ((int64_t)1 << 32)) { set_error("concat_tables: %lld rows >= 2^32", (long long)N); return OTTOHIP_ELIMIT; }
  if (N == 0) return 0;
  Workspace& ws = ctx->ws;
  // (1) :131-132 -- click_to tables with more than filter_rows rows lose rows with count < thr
  const bool filt = mp->click_rule && N > mp->filter_rows && !loaded_from_cache;
  uint4* rec;
  OH_TRY(ws.get("ct_rec", (size_t)N, &rec));
  int64_t n1 = 0;
  int ph = ctx->begin("concat_pack", s, 28.0 * N);
  if (filt) {
    uint32_t* flag;
    uint64_t *idx, *tot;
    OH_TRY(ws.get("ct_flag", (size_t)N, &flag));
    OH_TRY(ws.get("ct_idx", (size_t)N, &idx));
    OH_TRY(ws.get("ct_tot", 1, &tot));
    const uint32_t thr = (uint32_t)std::max<int32_t>(mp->min_count_in_part, 1);
    int64_t o = 0;
    for (int t = 0; t < n_tables; ++t) {
      if (!n_rows[t]) continue;
      k_ct_flag<<<grid_for(n_rows[t]), 256, 0, s>>>(count[t], n_rows[t], thr, flag + o);
      o += n_rows[t];
    }
    OH_TRY(exclusive_scan_u32(ctx, flag, idx, N, tot, s));
    o = 0;
    for (int t = 0; t < n_tables; ++t) {
      if (!n_rows[t]) continue;
      k_ct_pack<<<grid_for(n_rows[t]), 256, 0, s>>>(aid[t], aid_next[t], count[t], n_rows[t], flag + o, idx + o, rec);
      o += n_rows[t];
    }
    uint64_t m = 0;
    OH_TRY(d2h(&m, tot, 1, s));
    n1 = (int64_t)m;
  } else {
    int64_t o = 0;
    for (int t = 0; t < n_tables; ++t) {
      if (!n_rows[t]) continue;
      k_ct_pack<<<grid_for(n_rows[t]), 256, 0, s>>>(aid[t], aid_next[t], count[t], n_rows[t], nullptr, nullptr, rec + o);
      o += n_rows[t];
    }
    n1 = N;
  }
  OH_HIP(hipGetLastError());
  ctx->end(ph, s);
  const int64_t HUGE_ROWS = (int64_t)1 << 62;
  ottohip_merge_params fin = *mp;
  fin.click_rule = 0;             // the row filter above already ran
  fin.filter_rows = HUGE_ROWS;
  fin.max_rows_groupby = HUGE_ROWS;
  const uint4* final_rec = rec;
  int64_t n_final = n1;
  int rc;
  // (2) :135-166 -- more than max_rows_groupby rows: ceil(n/optim_rows) row slices of the
  // concatenation, each groupby-sum -> count >= MIN_COUNT_IN_PART -> count desc -> head
  if (n1 > mp->max_rows_groupby && !loaded_from_cache) {
    const int64_t n_parts = ceil_div(n1, optim_rows);
    const int64_t max_rows_part = (int64_t)((double)mp->max_rows_groupby / (double)n1 * (double)optim_rows);
    const int64_t rows_part = ceil_div(n1, n_parts);
    uint4* prec;
    int32_t *pa, *pb, *pc;
    const int64_t cap = std::max<int64_t>(1, std::min<int64_t>(rows_part, max_rows_part));
    OH_TRY(ws.get("ct_prec", (size_t)std::max<int64_t>(1, std::min<int64_t>(n1, n_parts * cap)), &prec));
    OH_TRY(ws.get("ct_pa", (size_t)cap, &pa));
    OH_TRY(ws.get("ct_pb", (size_t)cap, &pb));
    OH_TRY(ws.get("ct_pc", (size_t)cap, &pc));
    ottohip_merge_params part = fin;
    part.min_count = std::max<int32_t>(mp->min_count_in_part, 1);
    part.max_rows = max_rows_part;
    int64_t np = 0;
    for (int64_t p = 0; p < n_parts; ++p) {
      const int64_t r0 = p * rows_part, r1 = std::min<int64_t>(n1, r0 + rows_part);
      if (r1 <= r0) break;
      ottohip_table* T = nullptr;
      if ((rc = ottohip_table_from_records(ctx, rec + r0, r1 - r0, 1, n_items, nullptr, &T, stream))) return rc;
      int64_t k = 0;
      rc = ottohip_table_finalize(ctx, T, 0, &part, pa, pb, pc, &k, stream);
      ottohip_table_free(T);
      if (rc) return rc;
      if (k) k_out_records<<<grid_for(k), 256, 0, s>>>(pa, pb, pc, k, prec + np);
      np += k;
    }
    OH_HIP(hipGetLastError());
    final_rec = prec;
    n_final = np;
  }
  // (3) :168-175 -- groupby-sum, count >= MIN_COUNT_TO_SAVE, count desc, head(max_rows)
  ottohip_table* T = nullptr;
  ottohip_rule_stats st = {};
  st.file_rows = n_final;
  if ((rc = ottohip_table_from_records(ctx, n_final ? final_rec : nullptr, n_final, 1, n_items, &st, &T, stream))) return rc;
  rc = ottohip_table_finalize(ctx, T, 0, &fin, out_aid, out_aid_next, out_count, n_out, stream);
  ottohip_table_free(T);
  return rc;
}

extern "C" int ottohip_run_hist(ottohip_ctx* ctx, const int32_t* x, int64_t lo, int64_t hi, int shift, uint32_t mask,
                                int64_t n_bins, uint64_t* hist, void* stream) {
  if (!ctx || !hist || lo < 0 || hi < lo || (hi > lo && !x) || shift < 0 || shift > 31 || n_bins < 1 ||
      (int64_t)mask + 1 < 1) {
    set_error("run_hist: bad arguments");
    return OTTOHIP_EINVAL;
  }
  hipStream_t s = S(stream);
  OH_HIP(hipSetDevice(ctx->device));
  int* err;
  OH_TRY(ctx->ws.get("rh_err", 1, &err));
  OH_HIP(hipMemsetAsync(hist, 0, (size_t)n_bins * 8, s));
  OH_HIP(hipMemsetAsync(err, 0, sizeof(int), s));
  if (hi > lo)
    k_run_hist<<<grid_for(hi - lo), 256, 0, s>>>(x, lo, hi, shift, mask, n_bins,
                                                reinterpret_cast<unsigned long long*>(hist), err);
  OH_HIP(hipGetLastError());
  int herr = 0;
  OH_TRY(d2h(&herr, err, 1, s));
  if (herr) { set_error("run_hist: key >= n_bins"); return OTTOHIP_ERANGE; }
  return 0;
}

extern "C" int ottohip_table_digest(ottohip_ctx* ctx, const ottohip_table* t, int rule, uint64_t* out, void* stream) {
  if (!ctx || !t || !out || rule < 0 || rule >= t->n_rules) { set_error("table_digest: bad arguments"); return OTTOHIP_EINVAL; }
  hipStream_t s = S(stream);
  OH_HIP(hipSetDevice(ctx->device));
  unsigned long long* d;
  OH_TRY(ctx->ws.get("digest", 5, &d));
  OH_HIP(hipMemsetAsync(d, 0, 5 * 8, s));
  if (t->n_slots > 0)
    k_table_digest<<<(unsigned)std::min<int64_t>(ceil_div(t->n_slots, 256), (int64_t)ctx->n_cu * 8), 256, 0, s>>>(
        t->b.rule, t->b.aid, t->b.aid_next, t->b.count, t->b.count_ge2, t->n_slots, rule, t->sym(rule), d);
  OH_HIP(hipGetLastError());
  OH_TRY(d2h(reinterpret_cast<unsigned long long*>(out), d, 5, s));
  return 0;
}

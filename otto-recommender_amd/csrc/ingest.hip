// Event ingest: reference-schema parquet rows -> session-sorted CSR in HBM.
//
// The reference's files hold rows (session:i32, aid:i32, ts:i32, type:i8), 100k sessions per file,
// the rows of a session contiguous (etl/jsonl_to_parquet.py:23-29, 59-84), and are read back at
// model/count_co_events.py:81,91. The host decodes parquet columns; everything after the raw column
// upload runs here:
//   k_csr_flags   : flag[i] = row i starts a run of equal session ids
//   (scan)        : run index of every row, R = number of runs
//   k_csr_heads   : offsets[run] = base + first row, ids[run] = session, head key (orderable u32)
//   k_csr_order   : are the run heads strictly ascending? (the reference's files: yes -> done)
//   otherwise the heads are radix-sorted and checked for a repeated id (a session split over runs);
//   only then are the rows stably radix-sorted by session and gathered, and the runs rebuilt.
// Algorithmic bytes on the common (already grouped) path: 4 B read by the flags, 4 + 8 + 4 B per
// run head, one 9 B/row column copy when the outputs are separate buffers.
#include <algorithm>
#include "prims.h"
#include "table.h"

namespace ottohip {

__global__ void k_csr_flags(const int32_t* __restrict__ sess, int64_t n, uint32_t* __restrict__ flag) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) flag[i] = (i == 0 || sess[i] != sess[i - 1]) ? 1u : 0u;
}

// run heads; the last row also writes the closing offset (base + n) at index R
__global__ void k_csr_heads(const int32_t* __restrict__ sess, int64_t n, const uint32_t* __restrict__ flag,
                            const uint64_t* __restrict__ idx, int64_t base, int64_t* __restrict__ off,
                            int32_t* __restrict__ ids, uint32_t* __restrict__ key) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (flag[i]) {
    const uint64_t r = idx[i];
    off[r] = base + i;
    if (ids) ids[r] = sess[i];
    key[r] = (uint32_t)sess[i] ^ 0x80000000u;  // orders like the signed id
  }
  if (i == n - 1) off[idx[i] + flag[i]] = base + n;
}

// err |= 1 if some key is not strictly above its predecessor (strict = no equal neighbours)
__global__ void k_csr_order(const uint32_t* __restrict__ key, int64_t m, int* __restrict__ err) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j > 0 && j < m && key[j] <= key[j - 1]) atomicOr(err, 1);
}

__global__ void k_csr_keys(const int32_t* __restrict__ sess, int64_t n, uint32_t* __restrict__ key) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) key[i] = (uint32_t)sess[i] ^ 0x80000000u;
}

// rows in (session, original position) order: gather the columns, and the sorted ids back
__global__ void k_csr_gather(const uint32_t* __restrict__ skey, const uint32_t* __restrict__ perm, int64_t n,
                             const int32_t* __restrict__ aid, const int32_t* __restrict__ ts,
                             const int8_t* __restrict__ type, int32_t* __restrict__ sess_out,
                             int32_t* __restrict__ aid_out, int32_t* __restrict__ ts_out,
                             int8_t* __restrict__ type_out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t p = perm[i];
  sess_out[i] = (int32_t)(skey[i] ^ 0x80000000u);
  aid_out[i] = aid[p];
  ts_out[i] = ts[p];
  type_out[i] = type[p];
}

// every file's first row starts a run (a session id repeated in the next file is another session)
__global__ void k_csr_mark(const int64_t* __restrict__ fstart, int nf, int64_t n, uint32_t* __restrict__ flag) {
  const int f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f < nf && fstart[f] < n) flag[fstart[f]] = 1u;
}

// run index of each file's first row -> file_session_bounds (the last entry is R)
__global__ void k_csr_bounds(const int64_t* __restrict__ fstart, int nf, int64_t n, const uint64_t* __restrict__ idx,
                             const uint64_t* __restrict__ tot, int64_t* __restrict__ bounds) {
  const int f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f <= nf) bounds[f] = (int64_t)(fstart[f] < n ? idx[fstart[f]] : *tot);
}

// runs of sess[0..n) -> offsets / ids / head keys; returns R. fstart (device, nf entries): rows
// that start a run whatever their id
static int csr_runs(Ctx* ctx, const int32_t* sess, int64_t n, int64_t base, int64_t* off, int32_t* ids,
                    uint32_t* key, int64_t* R, hipStream_t s, const int64_t* fstart = nullptr, int nf = 0) {
  Workspace& ws = ctx->ws;
  uint32_t* flag;
  uint64_t *idx, *tot;
  OH_TRY(ws.get("csr_flag", (size_t)n, &flag));
  OH_TRY(ws.get("csr_idx", (size_t)n, &idx));
  OH_TRY(ws.get("csr_tot", 1, &tot));
  k_csr_flags<<<grid_for(n), 256, 0, s>>>(sess, n, flag);
  if (nf > 0) k_csr_mark<<<grid_for(nf), 256, 0, s>>>(fstart, nf, n, flag);
  OH_TRY(exclusive_scan_u32(ctx, flag, idx, n, tot, s));
  k_csr_heads<<<grid_for(n), 256, 0, s>>>(sess, n, flag, idx, base, off, ids, key);
  OH_HIP(hipGetLastError());
  uint64_t r = 0;
  OH_TRY(d2h(&r, tot, 1, s));
  *R = (int64_t)r;
  return 0;
}

static int strictly_ascending(Ctx* ctx, const uint32_t* key, int64_t m, bool* out, hipStream_t s) {
  int* err;
  OH_TRY(ctx->ws.get("csr_err", 1, &err));
  OH_HIP(hipMemsetAsync(err, 0, sizeof(int), s));
  if (m > 1) k_csr_order<<<grid_for(m), 256, 0, s>>>(key, m, err);
  OH_HIP(hipGetLastError());
  int h = 0;
  OH_TRY(d2h(&h, err, 1, s));
  *out = h == 0;
  return 0;
}

}  // namespace ottohip

using namespace ottohip;

extern "C" int ottohip_events_csr(ottohip_ctx* c, const int32_t* session, const int32_t* aid, const int32_t* ts,
                                  const int8_t* type, int64_t n_rows, int64_t offset_base, int64_t* session_offsets,
                                  int32_t* session_ids, int32_t* aid_out, int32_t* ts_out, int8_t* type_out,
                                  int64_t* n_sessions, int* reordered, void* stream) {
  if (!c || n_rows < 0 || !session_offsets || !n_sessions || offset_base < 0 ||
      (n_rows > 0 && (!session || !aid || !ts || !type || !aid_out || !ts_out || !type_out))) {
    set_error("events_csr: bad arguments");
    return OTTOHIP_EINVAL;
  }
  if (n_rows >= ((int64_t)1 << 32)) { set_error("events_csr: %lld rows >= 2^32", (long long)n_rows); return OTTOHIP_ELIMIT; }
  ottohip_ctx* ctx = c;
  hipStream_t s = S(stream);
  OH_HIP(hipSetDevice(ctx->device));
  *n_sessions = 0;
  if (reordered) *reordered = 0;
  if (n_rows == 0) {
    OH_HIP(hipMemcpyAsync(session_offsets, &offset_base, sizeof(int64_t), hipMemcpyHostToDevice, s));
    OH_HIP(hipStreamSynchronize(s));
    return 0;
  }
  Workspace& ws = ctx->ws;
  const int64_t n = n_rows;
  uint32_t* key;
  OH_TRY(ws.get("csr_key", (size_t)n, &key));
  int64_t R = 0;
  OH_TRY(csr_runs(ctx, session, n, offset_base, session_offsets, session_ids, key, &R, s));
  bool grouped = false;
  OH_TRY(strictly_ascending(ctx, key, R, &grouped, s));
  if (!grouped) {
    // heads not ascending: a repeated head id means a session split over several runs
    uint32_t *k0 = key, *v0, *k1, *v1;
    OH_TRY(ws.get("csr_v0", (size_t)R, &v0));
    OH_TRY(ws.get("csr_k1", (size_t)R, &k1));
    OH_TRY(ws.get("csr_v1", (size_t)R, &v1));
    uint32_t *k = k0, *v = v0;
    OH_TRY(radix_sort_pairs(ctx, k, v, k1, v1, R, 32, s, true));
    bool unique = false;
    OH_TRY(strictly_ascending(ctx, k, R, &unique, s));
    grouped = unique;
  }
  if (grouped) {  // keep the file's row order
    if (aid_out != aid) OH_HIP(hipMemcpyAsync(aid_out, aid, (size_t)n * 4, hipMemcpyDeviceToDevice, s));
    if (ts_out != ts) OH_HIP(hipMemcpyAsync(ts_out, ts, (size_t)n * 4, hipMemcpyDeviceToDevice, s));
    if (type_out != type) OH_HIP(hipMemcpyAsync(type_out, type, (size_t)n, hipMemcpyDeviceToDevice, s));
  } else {  // stable sort of the rows by session, then the runs again
    uint32_t *k0, *v0, *k1, *v1;
    int32_t *ss, *ga, *gt;
    int8_t* gy;
    OH_TRY(ws.get("csr_rk0", (size_t)n, &k0));
    OH_TRY(ws.get("csr_rv0", (size_t)n, &v0));
    OH_TRY(ws.get("csr_rk1", (size_t)n, &k1));
    OH_TRY(ws.get("csr_rv1", (size_t)n, &v1));
    OH_TRY(ws.get("csr_ss", (size_t)n, &ss));
    OH_TRY(ws.get("csr_ga", (size_t)n, &ga));
    OH_TRY(ws.get("csr_gt", (size_t)n, &gt));
    OH_TRY(ws.get("csr_gy", (size_t)n, &gy));
    k_csr_keys<<<grid_for(n), 256, 0, s>>>(session, n, k0);
    OH_HIP(hipGetLastError());
    uint32_t *k = k0, *v = v0;
    OH_TRY(radix_sort_pairs(ctx, k, v, k1, v1, n, 32, s, true));
    // gather into scratch first: the outputs may alias the inputs
    k_csr_gather<<<grid_for(n), 256, 0, s>>>(k, v, n, aid, ts, type, ss, ga, gt, gy);
    OH_HIP(hipGetLastError());
    OH_HIP(hipMemcpyAsync(aid_out, ga, (size_t)n * 4, hipMemcpyDeviceToDevice, s));
    OH_HIP(hipMemcpyAsync(ts_out, gt, (size_t)n * 4, hipMemcpyDeviceToDevice, s));
    OH_HIP(hipMemcpyAsync(type_out, gy, (size_t)n, hipMemcpyDeviceToDevice, s));
    OH_TRY(csr_runs(ctx, ss, n, offset_base, session_offsets, session_ids, key, &R, s));
    if (reordered) *reordered = 1;
  }
  OH_HIP(hipStreamSynchronize(s));
  *n_sessions = R;
  return 0;
}

extern "C" int ottohip_events_csr_files(ottohip_ctx* c, const int32_t* session, const int32_t* aid, const int32_t* ts,
                                        const int8_t* type, int n_files, const int64_t* file_row_starts,
                                        int64_t* session_offsets, int32_t* session_ids, int32_t* aid_out,
                                        int32_t* ts_out, int8_t* type_out, int64_t* file_session_bounds,
                                        int* reordered, void* stream) {
  if (!c || n_files < 1 || !file_row_starts || !file_session_bounds || !session_offsets || file_row_starts[0] != 0) {
    set_error("events_csr_files: bad arguments");
    return OTTOHIP_EINVAL;
  }
  for (int f = 0; f < n_files; ++f)
    if (file_row_starts[f + 1] < file_row_starts[f]) { set_error("events_csr_files: file %d ends before it starts", f); return OTTOHIP_EINVAL; }
  const int64_t n = file_row_starts[n_files];
  if (n > 0 && (!session || !aid || !ts || !type || !aid_out || !ts_out || !type_out)) {
    set_error("events_csr_files: bad arguments");
    return OTTOHIP_EINVAL;
  }
  if (n >= ((int64_t)1 << 32)) { set_error("events_csr_files: %lld rows >= 2^32", (long long)n); return OTTOHIP_ELIMIT; }
  ottohip_ctx* ctx = c;
  hipStream_t s = S(stream);
  OH_HIP(hipSetDevice(ctx->device));
  if (reordered) *reordered = 0;
  int64_t R = 0;
  bool grouped = n == 0;
  if (n > 0) {
    // one pass over every file (runs forced at file starts); kept when the run heads ascend strictly
    // over all files, which the reference's files do (session ids increase from file to file)
    Workspace& ws = ctx->ws;
    uint32_t* key;
    int64_t *fs, *fb;
    OH_TRY(ws.get("csr_key", (size_t)n, &key));
    OH_TRY(ws.get("csr_fs", (size_t)n_files + 1, &fs));
    OH_TRY(ws.get("csr_fb", (size_t)n_files + 1, &fb));
    OH_HIP(hipMemcpyAsync(fs, file_row_starts, (size_t)(n_files + 1) * 8, hipMemcpyHostToDevice, s));
    OH_TRY(csr_runs(ctx, session, n, 0, session_offsets, session_ids, key, &R, s, fs, n_files));
    OH_TRY(strictly_ascending(ctx, key, R, &grouped, s));
    if (grouped) {
      uint64_t *idx, *tot;
      OH_TRY(ws.get("csr_idx", (size_t)n, &idx));
      OH_TRY(ws.get("csr_tot", 1, &tot));
      k_csr_bounds<<<grid_for(n_files + 1), 256, 0, s>>>(fs, n_files, n, idx, tot, fb);
      OH_HIP(hipGetLastError());
      OH_TRY(d2h(file_session_bounds, fb, (size_t)n_files + 1, s));
      if (aid_out != aid) OH_HIP(hipMemcpyAsync(aid_out, aid, (size_t)n * 4, hipMemcpyDeviceToDevice, s));
      if (ts_out != ts) OH_HIP(hipMemcpyAsync(ts_out, ts, (size_t)n * 4, hipMemcpyDeviceToDevice, s));
      if (type_out != type) OH_HIP(hipMemcpyAsync(type_out, type, (size_t)n, hipMemcpyDeviceToDevice, s));
      OH_HIP(hipStreamSynchronize(s));
      return 0;
    }
  }
  // otherwise file by file (each file grouped on its own, appended at its row offset)
  file_session_bounds[0] = 0;
  for (int f = 0; f < n_files; ++f) {
    const int64_t r0 = file_row_starts[f], rows = file_row_starts[f + 1] - r0, s0 = file_session_bounds[f];
    int64_t ns = 0;
    int re = 0;
    OH_TRY(ottohip_events_csr(c, session + r0, aid + r0, ts + r0, type + r0, rows, r0, session_offsets + s0,
                              session_ids ? session_ids + s0 : nullptr, aid_out + r0, ts_out + r0, type_out + r0,
                              &ns, &re, stream));
    file_session_bounds[f + 1] = s0 + ns;
    if (reordered && re) *reordered = 1;
  }
  return 0;
}

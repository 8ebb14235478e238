// Device primitives used by the co-visitation engine: exclusive scans and a stable LSD
// radix sort of (u32 key, u32 value) pairs. Written for wave64 / gfx950:
//   * scans: 256-thread blocks, 8 consecutive items per thread (32-B vector loads), wave
//     shuffle scan + one LDS hop across the 4 waves, recursive over block sums;
//   * radix sort: 8-bit digits, 4096-key tiles, stable wave-level multisplit by 8 ballots,
//     per-wave digit counters in LDS, keys staged in LDS in digit order so the global
//     scatter writes one contiguous run per (tile, digit).
#include "prims.h"

namespace ottohip {

constexpr int SCAN_T = 256, SCAN_I = 8, SCAN_TILE = SCAN_T * SCAN_I;

template <class T>
__global__ __launch_bounds__(SCAN_T) void k_block_sums(const T* __restrict__ in, int64_t n,
                                                       uint64_t* __restrict__ sums) {
  const int64_t base = (int64_t)blockIdx.x * SCAN_TILE + (int64_t)threadIdx.x * SCAN_I;
  uint64_t s = 0;
#pragma unroll
  for (int i = 0; i < SCAN_I; ++i)
    if (base + i < n) s += (uint64_t)in[base + i];
  __shared__ uint64_t ws[SCAN_T / 64];
  s = wave_incl_scan64(s);
  if ((threadIdx.x & 63) == 63) ws[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t t = 0;
    for (int w = 0; w < SCAN_T / 64; ++w) t += ws[w];
    sums[blockIdx.x] = t;
  }
}

// exclusive scan of one tile, plus the tile's offset from `offs` (or 0); total to *total
template <class T>
__global__ __launch_bounds__(SCAN_T) void k_scan_tile(const T* __restrict__ in, int64_t n,
                                                      uint64_t* __restrict__ out,
                                                      const uint64_t* __restrict__ offs,
                                                      uint64_t* __restrict__ total) {
  const int64_t base = (int64_t)blockIdx.x * SCAN_TILE + (int64_t)threadIdx.x * SCAN_I;
  uint64_t v[SCAN_I];
  uint64_t s = 0;
#pragma unroll
  for (int i = 0; i < SCAN_I; ++i) {
    v[i] = (base + i < n) ? (uint64_t)in[base + i] : 0;
    s += v[i];
  }
  __shared__ uint64_t ws[SCAN_T / 64];
  const uint64_t incl = wave_incl_scan64(s);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 63) ws[w] = incl;
  __syncthreads();
  uint64_t pre = offs ? offs[blockIdx.x] : 0;
  for (int k = 0; k < w; ++k) pre += ws[k];
  uint64_t run = pre + incl - s;
#pragma unroll
  for (int i = 0; i < SCAN_I; ++i) {
    if (base + i < n) out[base + i] = run;
    run += v[i];
  }
  if (total && threadIdx.x == SCAN_T - 1 && blockIdx.x == gridDim.x - 1) *total = run;
}

template <class T>
static int scan_rec(Ctx* ctx, const T* in, uint64_t* out, int64_t n, uint64_t* total, hipStream_t s,
                    int depth) {
  if (n <= 0) {
    if (total) OH_HIP(hipMemsetAsync(total, 0, sizeof(uint64_t), s));
    return 0;
  }
  const int64_t nb = ceil_div(n, SCAN_TILE);
  if (nb == 1) {
    k_scan_tile<T><<<1, SCAN_T, 0, s>>>(in, n, out, nullptr, total);
    OH_HIP(hipGetLastError());
    return 0;
  }
  char name[32];
  snprintf(name, sizeof name, "scan_sums%d", depth);
  uint64_t* sums;
  OH_TRY(ctx->ws.get(name, (size_t)nb, &sums));
  k_block_sums<T><<<(unsigned)nb, SCAN_T, 0, s>>>(in, n, sums);
  OH_HIP(hipGetLastError());
  OH_TRY(scan_rec<uint64_t>(ctx, sums, sums, nb, nullptr, s, depth + 1));  // in place is safe per tile
  k_scan_tile<T><<<(unsigned)nb, SCAN_T, 0, s>>>(in, n, out, sums, total);
  OH_HIP(hipGetLastError());
  return 0;
}

int exclusive_scan_u32(Ctx* ctx, const uint32_t* in, uint64_t* out, int64_t n, uint64_t* total,
                       hipStream_t s) {
  return scan_rec<uint32_t>(ctx, in, out, n, total, s, 0);
}
int exclusive_scan_u64(Ctx* ctx, const uint64_t* in, uint64_t* out, int64_t n, uint64_t* total,
                       hipStream_t s) {
  return scan_rec<uint64_t>(ctx, in, out, n, total, s, 0);
}

// ------------------------------------------------------------------ radix sort
#ifndef OH_RS_R
#define OH_RS_R 16
#endif
constexpr int RS_T = 256, RS_WAVES = RS_T / 64, RS_R = OH_RS_R, RS_TILE = RS_T * RS_R;  // 4096 (keys per thread: A/B build flag)
// a block sorts RS_SUB consecutive tiles in order, so the digit-count matrix (and its scan) has one
// column per 4 tiles: the scan of every pass was larger than the scatter's own work
constexpr int RS_SUB = 4, RS_BLOCK = RS_TILE * RS_SUB;

// Workgroups are dealt to the 8 XCDs round robin (block b -> XCD b % 8), each XCD with its own L2. With
// xcd != 0 block b takes tile xcd_tile(b): XCD x sorts the x-th eighth of the tiles, so consecutive tiles,
// whose digit runs meet inside one destination line, write that line through the same L2 (a line written
// in parts from two XCDs goes to HBM twice)
__device__ __forceinline__ int xcd_tile(int b, int nb, int xcd) {
  if (!xcd) return b;
  const int q = nb >> 3, r = nb & 7, x = b & 7;
  return x * q + min(x, r) + (b >> 3);
}

// SKIP (the compacting first pass of radix_sort_pairs): keys with (key & smask) == sinv are not counted
template <bool SKIP = false>
__global__ __launch_bounds__(RS_T) void k_rs_hist(const uint32_t* __restrict__ keys, int64_t n, int shift,
                                                  uint32_t* __restrict__ hist, int nb, int xcd, uint32_t smask = 0u,
                                                  uint32_t sinv = 0u) {
  const int tile = xcd_tile(blockIdx.x, nb, xcd);
  __shared__ uint32_t h[RS_WAVES][256];
  for (int i = threadIdx.x; i < RS_WAVES * 256; i += RS_T) (&h[0][0])[i] = 0;
  __syncthreads();
  const int w = threadIdx.x >> 6;
  const int64_t t0 = (int64_t)tile * RS_BLOCK;
#pragma unroll 4
  for (int r = 0; r < RS_R * RS_SUB; ++r) {
    const int64_t idx = t0 + r * RS_T + threadIdx.x;
    if constexpr (SKIP) {  // first pass over event-order keys: few runs of one digit, and skipped keys break runs
      const uint32_t k = idx < n ? keys[idx] : sinv;
      if ((k & smask) != sinv) atomicAdd(&h[w][(k >> shift) & 255u], 1u);
    } else {
      lds_add_runs(h[w], idx < n ? (keys[idx] >> shift) & 255u : 0u, idx < n);  // runs of one digit: one atomic
    }
  }
  __syncthreads();
  for (int d = threadIdx.x; d < 256; d += RS_T) {
    uint32_t c = 0;
    for (int k = 0; k < RS_WAVES; ++k) c += h[k][d];
    hist[(int64_t)d * nb + tile] = c;
  }
}

// SKIP: keys with (key & smask) == sinv are dropped (the output holds the others, densely)
template <bool SKIP = false>
__global__ __launch_bounds__(RS_T) void k_rs_scatter(const uint32_t* __restrict__ kin,
                                                     const uint32_t* __restrict__ vin,
                                                     uint32_t* __restrict__ kout,
                                                     uint32_t* __restrict__ vout, int64_t n, int shift,
                                                     const uint64_t* __restrict__ gofs, int nb, int iota, int xcd,
                                                     uint32_t smask = 0u, uint32_t sinv = 0u) {
  const int tile = xcd_tile(blockIdx.x, nb, xcd);
  __shared__ uint32_t wcnt[RS_WAVES][256];
  __shared__ uint32_t bstart[256];
  __shared__ uint32_t tcnt[256];  // the sub-tile's count per digit
  __shared__ uint32_t run[256];   // keys of each digit written by the block's earlier sub-tiles
  __shared__ uint32_t wsum[RS_WAVES];
  __shared__ uint32_t tvalid;     // SKIP: the sub-tile's kept keys
  __shared__ uint32_t stage_k[RS_TILE];
  __shared__ uint32_t stage_v[RS_TILE];
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  run[tid] = 0;  // RS_T == 256 digits
  for (int sub = 0; sub < RS_SUB; ++sub) {
    const int64_t t0 = (int64_t)tile * RS_BLOCK + (int64_t)sub * RS_TILE;
    if (t0 >= n) break;
    for (int i = tid; i < RS_WAVES * 256; i += RS_T) (&wcnt[0][0])[i] = 0;
    __syncthreads();
    uint32_t key[RS_R], val[RS_R], rnk[RS_R];
    uint32_t vmask = 0;  // SKIP: kept keys of this thread (bit r)
    // wave w owns the contiguous quarter [t0 + w*1024, t0 + (w+1)*1024): stable order
#pragma unroll
    for (int r = 0; r < RS_R; ++r) {
      const int64_t idx = t0 + w * (RS_R * 64) + r * 64 + l;
      bool valid = idx < n;
      key[r] = valid ? kin[idx] : 0u;
      if constexpr (SKIP) valid = valid && (key[r] & smask) != sinv;
      vmask |= valid ? (1u << r) : 0u;
      val[r] = valid ? (iota ? (uint32_t)idx : vin[idx]) : 0u;
      const uint32_t d = (key[r] >> shift) & 255u;
      uint64_t m = __ballot(valid);
#pragma unroll
      for (int b = 0; b < 8; ++b) {
        const bool bit = (d >> b) & 1u;
        const uint64_t bb = __ballot(bit);
        m &= bit ? bb : ~bb;
      }
      const uint32_t below = mbcnt(m);
      const uint32_t old = wcnt[w][d];
      __builtin_amdgcn_wave_barrier();
      if (valid && below == 0) wcnt[w][d] = old + (uint32_t)__popcll(m);
      __builtin_amdgcn_wave_barrier();
      rnk[r] = old + below;
    }
    __syncthreads();
    // per digit: wave offsets (exclusive over waves) and the tile-local digit start
    {
      const int d = tid;  // RS_T == 256 digits
      uint32_t tot = 0;
#pragma unroll
      for (int k = 0; k < RS_WAVES; ++k) { uint32_t c = wcnt[k][d]; wcnt[k][d] = tot; tot += c; }
      tcnt[d] = tot;
      const uint32_t incl = wave_incl_scan(tot);
      if (l == 63) wsum[w] = incl;
      __syncthreads();
      uint32_t pre = 0;
      for (int k = 0; k < w; ++k) pre += wsum[k];
      bstart[d] = pre + incl - tot;
      if (d == 255) tvalid = pre + incl;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < RS_R; ++r) {
      if ((vmask >> r) & 1u) {
        const uint32_t d = (key[r] >> shift) & 255u;
        const uint32_t p = bstart[d] + wcnt[w][d] + rnk[r];
        stage_k[p] = key[r];
        stage_v[p] = val[r];
      }
    }
    __syncthreads();
    const int64_t tn = SKIP ? (int64_t)tvalid : (n - t0 < RS_TILE ? n - t0 : RS_TILE);
    for (int p = tid; p < tn; p += RS_T) {
      const uint32_t k = stage_k[p];
      const uint32_t d = (k >> shift) & 255u;
      const uint64_t dst = gofs[(int64_t)d * nb + tile] + run[d] + (uint64_t)(p - bstart[d]);
      kout[dst] = k;
      vout[dst] = stage_v[p];
    }
    __syncthreads();  // run / stage / wcnt are rewritten by the next sub-tile
    run[tid] += tcnt[tid];
  }
}

// XCD-aware tile order in the radix passes (OTTOHIP_RS_XCD=1; A/B switch, off: rows 11.9 -> 13.1-14.1 ms with it
// on and the scatter's written bytes unchanged, 9.2 GB per build)
static int rs_xcd() {
  static const int v = getenv("OTTOHIP_RS_XCD") && !strcmp(getenv("OTTOHIP_RS_XCD"), "1");
  return v;
}

// one stable 8-bit pass on digit (key >> shift) & 255: (kin, vin) -> (kout, vout)
// digit_start / n_tiles (optional): the pass's per-(digit, tile) output offsets; digit d starts at
// (*digit_start)[d * *n_tiles]
int radix_pass(Ctx* ctx, const uint32_t* kin, const uint32_t* vin, uint32_t* kout, uint32_t* vout, int64_t n,
               int shift, hipStream_t s, const uint64_t** digit_start, int* n_tiles) {
  if (n <= 0) return 0;
  if (n >= ((int64_t)1 << 32)) { set_error("radix_pass: n=%lld too large", (long long)n); return OTTOHIP_ELIMIT; }
  const int nb = (int)ceil_div(n, RS_BLOCK);
  uint32_t* hist; uint64_t* gofs;
  OH_TRY(ctx->ws.get("rs_hist", (size_t)nb * 256, &hist));
  OH_TRY(ctx->ws.get("rs_gofs", (size_t)nb * 256, &gofs));
  k_rs_hist<<<nb, RS_T, 0, s>>>(kin, n, shift, hist, nb, rs_xcd());
  OH_HIP(hipGetLastError());
  OH_TRY(exclusive_scan_u32(ctx, hist, gofs, (int64_t)nb * 256, nullptr, s));
  k_rs_scatter<<<nb, RS_T, 0, s>>>(kin, vin, kout, vout, n, shift, gofs, nb, 0, rs_xcd());
  OH_HIP(hipGetLastError());
  if (digit_start) *digit_start = gofs;
  if (n_tiles) *n_tiles = nb;
  return 0;
}

int radix_sort_pairs(Ctx* ctx, uint32_t*& keys, uint32_t*& vals, uint32_t* keys_alt, uint32_t* vals_alt,
                     int64_t n, int bits, hipStream_t s, bool iota_vals, const SortSkip* skip) {
  if (skip) {  // the compacting first pass generates the values and drops the skipped keys
    if (!iota_vals || bits <= 0) { set_error("radix_sort_pairs: skipping needs iota values and bits > 0"); return OTTOHIP_EINVAL; }
    *skip->n_out = 0;
    if (n <= 0) return 0;
  } else if (n <= 1 || bits <= 0) {  // nothing to sort; generated values still have to be written
    if (iota_vals && n > 1) { set_error("radix_sort_pairs: iota values need bits > 0"); return OTTOHIP_EINVAL; }
    if (iota_vals && n == 1) OH_HIP(hipMemsetAsync(vals, 0, sizeof(uint32_t), s));
    return 0;
  }
  if (n >= ((int64_t)1 << 32)) { set_error("radix_sort_pairs: n=%lld too large", (long long)n); return OTTOHIP_ELIMIT; }
  int nb = (int)ceil_div(n, RS_BLOCK);
  uint32_t* hist; uint64_t* gofs;
  OH_TRY(ctx->ws.get("rs_hist", (size_t)nb * 256, &hist));
  OH_TRY(ctx->ws.get("rs_gofs", (size_t)nb * 256, &gofs));
  uint32_t *ka = keys, *va = vals, *kb = keys_alt, *vb = vals_alt;
  for (int shift = 0; shift < bits; shift += 8) {
    if (skip && shift == 0) {
      uint64_t* tot;
      OH_TRY(ctx->ws.get("rs_total", 1, &tot));
      k_rs_hist<true><<<nb, RS_T, 0, s>>>(ka, n, 0, hist, nb, rs_xcd(), skip->mask, skip->inv);
      OH_HIP(hipGetLastError());
      OH_TRY(exclusive_scan_u32(ctx, hist, gofs, (int64_t)nb * 256, tot, s));
      k_rs_scatter<true><<<nb, RS_T, 0, s>>>(ka, va, kb, vb, n, 0, gofs, nb, 1, rs_xcd(), skip->mask, skip->inv);
      OH_HIP(hipGetLastError());
      uint64_t kept = 0;
      OH_HIP(hipMemcpyAsync(&kept, tot, sizeof kept, hipMemcpyDeviceToHost, s));
      OH_HIP(hipStreamSynchronize(s));
      n = (int64_t)kept;
      *skip->n_out = n;
      nb = (int)ceil_div(n, RS_BLOCK);
      std::swap(ka, kb); std::swap(va, vb);
      if (n <= 1) break;  // nothing left to order: (ka, va) hold the kept key, if any
      continue;
    }
    k_rs_hist<<<nb, RS_T, 0, s>>>(ka, n, shift, hist, nb, rs_xcd());
    OH_HIP(hipGetLastError());
    OH_TRY(exclusive_scan_u32(ctx, hist, gofs, (int64_t)nb * 256, nullptr, s));
    k_rs_scatter<<<nb, RS_T, 0, s>>>(ka, va, kb, vb, n, shift, gofs, nb, iota_vals && shift == 0 ? 1 : 0, rs_xcd());
    OH_HIP(hipGetLastError());
    std::swap(ka, kb); std::swap(va, vb);
  }
  keys = ka; vals = va;  // result buffers (may be the alternates)
  return 0;
}

}  // namespace ottohip

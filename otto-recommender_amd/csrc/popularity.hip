// Pop-cluster source of config 5 and the session-item similarity R7.
//
//   C1 k_sess_emb     compute_sessions_embeddings (model/kmeans_sessions.py:40-86): one wave per
//                     session, w = f32(max(0.1, 1 - (max_ts - ts) / 259200) * {0.1, 0.3, 0.6}[type]),
//                     e_s = round6(sum w e_aid / sum w); aids without an embedding add 0 but keep w
//   C2 k_km_assign    Lloyd step of KMeans (model/kmeans_sessions.py:140-171): nearest centroid
//                     per session (centroids in LDS) and per-cluster sums accumulated in 2^-24 fixed
//                     point with int64 atomics, so the update is independent of the atomic order
//   C3 k_pop_*        count_popularity.py:53-85: per (cluster, aid) counts by type and over the
//                     last 7 days, ordinal rank desc within the cluster (ties: aid asc), clip 999,
//                     keep min rank <= keep_top_k
//   R7 k_sim          model/retrieve.py:604-625: dot, norms, cos and Euclidean distance between the
//                     session embedding and each candidate's item embedding (fp32)
#include <algorithm>
#include <cmath>
#include "prims.h"
#include "table.h"

namespace ottohip {

constexpr int EMB_MAXD = 128;

// ---------------------------------------------------------------- C1
__global__ __launch_bounds__(64) void k_sess_emb(const int64_t* __restrict__ off, int64_t S,
                                                 const int32_t* __restrict__ aid, const int32_t* __restrict__ ts,
                                                 const int8_t* __restrict__ type, const int32_t* __restrict__ row_of_aid,
                                                 int32_t n_aid_map, const float* __restrict__ emb, int dim,
                                                 float* __restrict__ out) {
  const int l = threadIdx.x;
  const int64_t s = blockIdx.x;
  if (s >= S) return;
  const int64_t e0 = off[s], e1 = off[s + 1];
  int32_t mx = INT32_MIN;
  for (int64_t e = e0 + l; e < e1; e += 64) mx = max(mx, ts[e]);
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) mx = max(mx, __shfl_xor(mx, o));
  float acc0 = 0.f, acc1 = 0.f, wsum = 0.f;
  const float wt[3] = {0.1f, 0.3f, 0.6f};
  // lanes fetch 64 events' weights and embedding rows at once (independent loads); the sums then
  // run over the events in order, exactly as one event at a time
  for (int64_t b = e0; b < e1; b += 64) {
    const int64_t e = b + l;
    float w = 0.f;
    int32_t r = -1;
    if (e < e1) {
      double wtime = 1.0 - (double)(mx - ts[e]) / 259200.0;
      if (wtime < 0.10) wtime = 0.10;
      const int y = type[e];
      w = (float)(wtime * (double)wt[y < 0 ? 0 : (y > 2 ? 2 : y)]);
      const int32_t a = aid[e];
      r = (a >= 0 && a < n_aid_map) ? row_of_aid[a] : -1;
    }
    const int cnt = (int)(e1 - b < 64 ? e1 - b : 64);
#pragma unroll 4
    for (int j = 0; j < cnt; ++j) {
      const float wj = __shfl(w, j);
      const int32_t rj = __shfl(r, j);
      wsum += wj;
      if (rj >= 0) {
        const float* v = emb + (int64_t)rj * dim;
        if (l < dim) acc0 += v[l] * wj;
        if (l + 64 < dim) acc1 += v[l + 64] * wj;
      }
    }
  }
  float* o = out + s * dim;
  if (l < dim) o[l] = (float)(nearbyint((double)(acc0 / wsum) * 1e6) / 1e6);
  if (l + 64 < dim) o[l + 64] = (float)(nearbyint((double)(acc1 / wsum) * 1e6) / 1e6);
}

// ---------------------------------------------------------------- C2
constexpr int KM_MAXK = 64;
constexpr double KM_FX = 16777216.0;  // 2^24 fixed point for the cluster sums

// Centroids transposed to [dim][KP] with squared norms (padding: 0 and +inf, never chosen), so the
// assignment kernel reads them with wave-uniform scalar loads (SGPR operands of the FMAs).
__global__ void k_km_prep(const float* __restrict__ C, int k, int dim, int KP, float* __restrict__ Ct,
                          float* __restrict__ cn) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (Ct && i < KP * dim) {  // (the MFMA kernels read C itself: Ct may be null)
    const int d = i / KP, c = i % KP;
    Ct[i] = c < k ? C[c * dim + d] : 0.f;
  }
  if (i < KM_MAXK) {  // 64 entries: the MFMA kernel reads two full blocks of 32
    float s = 0.f;
    for (int d = 0; d < dim && i < k; ++d) s += C[i * dim + d] * C[i * dim + d];
    cn[i] = i < k ? s : INFINITY;
  }
}

// One lane per row for the distances: |x - c|^2 = |x|^2 - 2 x.c + |c|^2, the row streamed once
// (16-B loads), all KP dots accumulated against scalar-loaded centroid columns. Then the wave
// walks its 64 rows with lanes over dimensions and adds each row into its cluster's per-block
// sums in LDS (2^-24 fixed point, int64: the update is independent of the atomic order),
// flushed with one device atomic per (cluster, dim).
template <int KP>
__global__ __launch_bounds__(256) void k_km_assign(const float* __restrict__ X, int64_t n, int dim,
                                                   const float* __restrict__ Ct, const float* __restrict__ cn, int k,
                                                   int32_t* __restrict__ label, unsigned long long* __restrict__ sums,
                                                   unsigned long long* __restrict__ cnt, double* __restrict__ inertia,
                                                   unsigned long long* __restrict__ changed, float* __restrict__ dist) {
  extern __shared__ unsigned long long smem64[];
  unsigned long long* ls = smem64;            // k * dim sums (fixed point, two's complement)
  unsigned long long* lc = smem64 + k * dim;  // k counts
  if (sums) {
    for (int i = threadIdx.x; i < k * dim; i += blockDim.x) ls[i] = 0ull;
    for (int i = threadIdx.x; i < k; i += blockDim.x) lc[i] = 0ull;
  }
  __syncthreads();
  const int l = threadIdx.x & 63;
  double part = 0.0;
  uint32_t nchg = 0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i0 = (int64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63); i0 < n; i0 += stride) {
    const int64_t i = i0 + l;
    const bool valid = i < n;
    const float* x = X + (valid ? i : i0) * dim;
    float xn = 0.f;
    float dot[KP];
#pragma unroll
    for (int c = 0; c < KP; ++c) dot[c] = 0.f;
    if ((dim & 3) == 0) {
      const float4* x4 = reinterpret_cast<const float4*>(x);
      for (int d4 = 0; d4 < (dim >> 2); ++d4) {
        const float4 v = x4[d4];
#pragma unroll 1
        for (int u = 0; u < 4; ++u) {  // one centroid column (KP SGPRs) at a time
          const float xv = u == 0 ? v.x : (u == 1 ? v.y : (u == 2 ? v.z : v.w));
          const float* col = Ct + (4 * d4 + u) * KP;
          xn += xv * xv;
#pragma unroll
          for (int c = 0; c < KP; ++c) dot[c] += xv * col[c];
        }
      }
    } else {
      for (int d = 0; d < dim; ++d) {
        const float xv = x[d];
        const float* col = Ct + d * KP;
        xn += xv * xv;
#pragma unroll
        for (int c = 0; c < KP; ++c) dot[c] += xv * col[c];
      }
    }
    float best = INFINITY;
    int bc = 0;
#pragma unroll
    for (int c = 0; c < KP; ++c) {
      const float dd = xn - 2.f * dot[c] + cn[c];
      if (dd < best) { best = dd; bc = c; }  // ties: lowest cluster index
    }
    if (valid) {
      if (changed) nchg += label[i] != bc;  // sklearn's strict-convergence test (labels == labels_old)
      label[i] = bc;
      part += (double)fmaxf(best, 0.f);
      if (dist) dist[i] = fmaxf(best, 0.f);
    }
    if (sums) {  // rows of this wave, lanes over dimensions
      const int nr = (int)min<int64_t>(64, n - i0);
      for (int r0 = 0; r0 < nr; r0 += 8) {  // 8 rows' loads in flight
        float xa[8], xb[8];
        int cc[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const int r = r0 + q < nr ? r0 + q : nr - 1;
          cc[q] = __shfl(bc, r);
          const float* xr = X + (i0 + r) * dim;
          xa[q] = l < dim ? xr[l] : 0.f;
          xb[q] = l + 64 < dim ? xr[l + 64] : 0.f;
        }
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          if (r0 + q >= nr) break;
          unsigned long long* row = ls + cc[q] * dim;  // exact 2^24 scaling
          if (l < dim) atomicAdd(&row[l], (unsigned long long)__float2ll_rn(xa[q] * 16777216.0f));
          if (l + 64 < dim) atomicAdd(&row[l + 64], (unsigned long long)__float2ll_rn(xb[q] * 16777216.0f));
          if (l == 0) atomicAdd(&lc[cc[q]], 1ull);
        }
      }
    }
  }
  __syncthreads();
  if (sums) {
    for (int i = threadIdx.x; i < k * dim; i += blockDim.x)
      if (ls[i]) atomicAdd(&sums[i], ls[i]);
    for (int i = threadIdx.x; i < k; i += blockDim.x)
      if (lc[i]) atomicAdd(&cnt[i], lc[i]);
  }
  // inertia: block partial in fixed order over waves then one atomic (f64; reporting only)
  for (int o = 32; o >= 1; o >>= 1) {
    const uint64_t b = __double_as_longlong(part);
    const uint32_t lo = __shfl_xor((uint32_t)b, o), hi = __shfl_xor((uint32_t)(b >> 32), o);
    part += __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
  }
  if ((threadIdx.x & 63) == 0) atomicAdd(inertia, part);
  if (changed) {
    const uint32_t w = wave_sum(nchg);
    if ((threadIdx.x & 63) == 0 && w) atomicAdd(changed, (unsigned long long)w);
  }
}

// C2 on the matrix cores (k <= 64, dim <= 128, dim % 4 == 0): a wave scores a tile of 32 rows
// against 32 centroids per v_mfma_f32_32x32x2f32 (NB = 1 or 2 centroid blocks). Lane (i, h)
// loads 16-B pieces of row i (dims 8q + 4h .. 8q + 4h + 3); the same dims of centroid i come
// from LDS, so MFMA (q, u) pairs dim 8q + u (h = 0) with dim 8q + 4 + u (h = 1). The MFMA is an
// exact f32 fma chain: only the summation order differs from k_km_assign. Centroids are the A
// operand and rows the B operand, so lane (i, h) holds row i's scores of 16 (32) clusters: the
// argmin over |c|^2 - 2 x.c (|x|^2 is common to the row, as in sklearn's Lloyd step; ties to the
// lowest cluster) is an in-lane min and lowest-index scan plus one exchange with lane i ^ 32
// (the former row-operand layout needed a 5-step cross-lane butterfly of 64-bit keys:
// Lloyd step 1.87 -> 1.68 ms). Per-cluster sums as in k_km_assign (2^-24 fixed point).
typedef float km_f32x16 __attribute__((ext_vector_type(16)));
constexpr int KM_MT = 512;  // threads per block (8 waves)
constexpr int KM_NQ = 16;   // 16-B pieces per row half (dim <= 128)

__device__ __forceinline__ uint32_t km_ord(float x) {  // order-preserving f32 -> u32
  const uint32_t b = __float_as_uint(x);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ float km_unord(uint32_t o) {
  return __uint_as_float((o & 0x80000000u) ? (o & 0x7FFFFFFFu) : ~o);
}
// x * 2^24 rounded to the nearest integer as int64: one f32 -> i32 conversion when |x| < 128
// (the product is exact and below 2^31), the general f32 -> i64 sequence otherwise
__device__ __forceinline__ long long km_fx(float x) {
  const float y = x * 16777216.0f;
  return fabsf(x) < 128.f ? (long long)__float2int_rn(y) : __float2ll_rn(y);
}

// The rows of a wave whose vector enters a cluster's block sums (one per flagged lane: row, new
// cluster, previous cluster or -1 to leave none), listed in the wave's LDS slot (3 x 32 ints), then
// lanes over dims: 2^-24 fixed-point adds into the block's LDS sums (exact, order-independent).
// RB: rows whose loads are in flight together (8; 16 in k_km_ties' fold of the split pass's move lists)
template <int RB = 8>
__device__ __forceinline__ void km_move_rows(const float* __restrict__ X, int dim, unsigned long long* ls,
                                             unsigned long long* lc, int32_t* labl, bool flag, int64_t row,
                                             uint32_t to, int32_t from) {
  const int l = (int)lane_id();
  const uint64_t bm = __ballot(flag);
  if (flag) {
    const int p = (int)mbcnt(bm);
    labl[p] = (int32_t)row;
    labl[32 + p] = (int32_t)to;
    labl[64 + p] = from;
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  const int nr = (int)__popcll(bm);
  for (int rr = 0; rr < nr; rr += RB) {  // RB rows' loads in flight
    float xa[RB], xb[RB];
    int cc[RB], co[RB];
#pragma unroll
    for (int q = 0; q < RB; ++q) {
      const int pq = rr + q < nr ? rr + q : nr - 1;
      const int64_t r = labl[pq];
      cc[q] = labl[32 + pq];
      co[q] = labl[64 + pq];
      const float* xq = X + r * dim;
      xa[q] = l < dim ? xq[l] : 0.f;
      xb[q] = l + 64 < dim ? xq[l + 64] : 0.f;
    }
    // exact 2^24 scaling: one f32 -> i32 conversion per value while every |x| < 128 (the
    // product is exact and below 2^31); the general f32 -> i64 sequence only for a wave
    // that holds a larger value
    bool big = false;
#pragma unroll
    for (int q = 0; q < RB; ++q) big |= fabsf(xa[q]) >= 128.f || fabsf(xb[q]) >= 128.f;
    long long fa[RB], fb[RB];
    if (__builtin_expect(__ballot(big) != 0, 0)) {
#pragma unroll
      for (int q = 0; q < RB; ++q) { fa[q] = __float2ll_rn(xa[q] * 16777216.0f); fb[q] = __float2ll_rn(xb[q] * 16777216.0f); }
    } else {
#pragma unroll
      for (int q = 0; q < RB; ++q) {
        fa[q] = (long long)__float2int_rn(xa[q] * 16777216.0f);
        fb[q] = (long long)__float2int_rn(xb[q] * 16777216.0f);
      }
    }
#pragma unroll
    for (int q = 0; q < RB; ++q) {
      if (rr + q >= nr) break;
      unsigned long long* rw = ls + cc[q] * dim;
      if (l < dim) atomicAdd(&rw[l], (unsigned long long)fa[q]);
      if (l + 64 < dim) atomicAdd(&rw[l + 64], (unsigned long long)fb[q]);
      if (l == 0) atomicAdd(&lc[cc[q]], 1ull);
      if (co[q] >= 0) {  // two's-complement deltas: the block's sums may go below zero
        unsigned long long* orow = ls + co[q] * dim;
        if (l < dim) atomicAdd(&orow[l], (unsigned long long)(-fa[q]));
        if (l + 64 < dim) atomicAdd(&orow[l + 64], (unsigned long long)(-fb[q]));
        if (l == 0) atomicAdd(&lc[co[q]], ~0ull);
      }
    }
  }
  __builtin_amdgcn_wave_barrier();  // labl is rewritten by the next tile
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
}

// NQ: 16-B pieces per row half as a constant (13 for dim 100: the row registers of the unused
// pieces are not allocated, which keeps the kernel at <= 128 VGPRs = 2 blocks per CU)
// LIST: score only the rows lrows[0, *lnrows) (the split-precision pass's near ties)
template <int NB, int NQ, bool LIST = false>
__global__ __launch_bounds__(KM_MT, (NQ <= 13 ? 4 : 2)) void k_km_assign_mfma(const float* __restrict__ X, int64_t n, int dim, int nq,
                                                        const float* __restrict__ C, const float* __restrict__ cn,
                                                        int k, int32_t* __restrict__ label,
                                                        unsigned long long* __restrict__ sums,
                                                        unsigned long long* __restrict__ cnt,
                                                        double* __restrict__ inertia,
                                                        unsigned long long* __restrict__ changed,
                                                        float* __restrict__ dist, int inc,
                                                        const int* __restrict__ gate,
                                                        const uint32_t* __restrict__ lrows = nullptr,
                                                        const unsigned long long* __restrict__ lnrows = nullptr) {
  if (gate && __builtin_amdgcn_readfirstlane(*gate)) return;  // batched Lloyd steps: converged earlier
  extern __shared__ unsigned long long smem64[];
  float4* Bl = reinterpret_cast<float4*>(smem64);                              // [NB][nq][64]
  int32_t* labl = reinterpret_cast<int32_t*>(Bl + NB * nq * 64);                // [waves][3][32]: row, new, old
  float* cnl = reinterpret_cast<float*>(labl + (KM_MT / 64) * 96);             // [64]
  unsigned long long* ls = reinterpret_cast<unsigned long long*>(cnl + 64);    // k * dim sums, k counts
  unsigned long long* lc = ls + k * dim;
  const int tid = threadIdx.x, l = tid & 63, wv = tid >> 6, h = l >> 5, i32 = l & 31;
  for (int e = tid; e < NB * nq * 64; e += KM_MT) {
    const int ll = e & 63, q = (e >> 6) % nq, b = (e >> 6) / nq;
    const int c = b * 32 + (ll & 31), d0 = 8 * q + 4 * (ll >> 5);
    float4 f = make_float4(0.f, 0.f, 0.f, 0.f);
    if (c < k && d0 < dim) f = *reinterpret_cast<const float4*>(C + (int64_t)c * dim + d0);
    Bl[e] = f;
  }
  if (tid < 64) cnl[tid] = cn[tid];
  if (sums)
    for (int i = tid; i < k * dim + k; i += KM_MT) ls[i] = 0ull;
  __syncthreads();
  double part = 0.0;
  uint32_t nchg = 0;
  const int64_t nl = LIST ? (int64_t)__builtin_amdgcn_readfirstlane((int)*lnrows) : n;  // rows to score
  const int64_t ntile = (nl + 31) >> 5;
  const int64_t nwv = (int64_t)gridDim.x * (KM_MT / 64);
  for (int64_t t = (int64_t)blockIdx.x * (KM_MT / 64) + wv; t < ntile; t += nwv) {
    const int64_t r0 = t << 5;
    const bool in_l = r0 + i32 < nl;
    const int64_t row = LIST ? (int64_t)lrows[in_l ? r0 + i32 : nl - 1] : (in_l ? r0 + i32 : n - 1);
    const float* x = X + row * dim;
    float4 a[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int d0 = 8 * q + 4 * h;
      a[q] = (q < nq && d0 < dim) ? *reinterpret_cast<const float4*>(x + d0) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    float xs = 0.f;
#pragma unroll
    for (int q = 0; q < NQ; ++q) xs += a[q].x * a[q].x + a[q].y * a[q].y + a[q].z * a[q].z + a[q].w * a[q].w;
    xs += __shfl_xor(xs, 32);
    // centroids as the A operand, rows as B: lane (i32, h) ends with row r0 + i32's scores of the
    // clusters (r & 3) + 8 (r >> 2) + 4 h in register r (+ 32 in acc1), so the argmin is an
    // in-lane scan plus one exchange with lane i32 + 32 (no cross-lane butterfly over clusters)
    km_f32x16 acc0 = {}, acc1 = {};
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      if (q < nq) {
        const float4 b0 = Bl[q * 64 + l];
        acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(b0.x, a[q].x, acc0, 0, 0, 0);
        acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(b0.y, a[q].y, acc0, 0, 0, 0);
        acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(b0.z, a[q].z, acc0, 0, 0, 0);
        acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(b0.w, a[q].w, acc0, 0, 0, 0);
        if (NB == 2) {
          const float4 b1 = Bl[(nq + q) * 64 + l];
          acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(b1.x, a[q].x, acc1, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(b1.y, a[q].y, acc1, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(b1.z, a[q].z, acc1, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(b1.w, a[q].w, acc1, 0, 0, 0);
        }
      }
    }
    // score |c|^2 - 2 x.c (exact: 2 x.c is exact, one rounding as before); the minimum, then the
    // lowest cluster holding it (clusters ascend with r within a block)
    float m = INFINITY;

#pragma unroll
    for (int j = 0; j < 4; ++j) {  // scores in place of the dot products
      const float4 n0 = *reinterpret_cast<const float4*>(cnl + 8 * j + 4 * h);
      acc0[4 * j + 0] = n0.x - 2.f * acc0[4 * j + 0];
      acc0[4 * j + 1] = n0.y - 2.f * acc0[4 * j + 1];
      acc0[4 * j + 2] = n0.z - 2.f * acc0[4 * j + 2];
      acc0[4 * j + 3] = n0.w - 2.f * acc0[4 * j + 3];
      if (NB == 2) {
        const float4 n1 = *reinterpret_cast<const float4*>(cnl + 32 + 8 * j + 4 * h);
        acc1[4 * j + 0] = n1.x - 2.f * acc1[4 * j + 0];
        acc1[4 * j + 1] = n1.y - 2.f * acc1[4 * j + 1];
        acc1[4 * j + 2] = n1.z - 2.f * acc1[4 * j + 2];
        acc1[4 * j + 3] = n1.w - 2.f * acc1[4 * j + 3];
      }
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      m = fminf(m, acc0[r]);
      if (NB == 2) m = fminf(m, acc1[r]);
    }
    int mc = 64;
#pragma unroll
    for (int r = 15; r >= 0; --r) {
      if (NB == 2) mc = acc1[r] == m ? 32 + (r & 3) + 8 * (r >> 2) + 4 * h : mc;
    }
#pragma unroll
    for (int r = 15; r >= 0; --r) mc = acc0[r] == m ? (r & 3) + 8 * (r >> 2) + 4 * h : mc;
    {  // the other half of the row's clusters (lane i32 ^ 32): smaller score, then lower cluster
      const float pm = __shfl_xor(m, 32);
      const int pc = __shfl_xor(mc, 32);
      if (pm < m || (pm == m && pc < mc)) { m = pm; mc = pc; }
    }
    const float xr = xs;
    const uint32_t mi = (uint32_t)mc;
    int32_t old = -1;
    const bool mine = h == 0 && in_l;
    if (mine) {
      if (changed || inc) old = label[row];
      if (changed) nchg += old != (int32_t)mi;
      label[row] = (int32_t)mi;
      const float dd = fmaxf(xr + m, 0.f);
      part += (double)dd;
      if (dist) dist[row] = dd;
    }
    if (sums) km_move_rows(X, dim, ls, lc, labl + wv * 96, mine && (!inc || old != (int32_t)mi), row, mi, inc ? old : -1);
  }
  __syncthreads();
  if (sums) {
    for (int i = tid; i < k * dim; i += KM_MT)
      if (ls[i]) atomicAdd(&sums[i], ls[i]);
    for (int i = tid; i < k; i += KM_MT)
      if (lc[i]) atomicAdd(&cnt[i], lc[i]);
  }
  for (int o = 32; o >= 1; o >>= 1) {
    const uint64_t b = __double_as_longlong(part);
    const uint32_t lo = __shfl_xor((uint32_t)b, o), hi = __shfl_xor((uint32_t)(b >> 32), o);
    part += __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
  }
  if (l == 0) atomicAdd(inertia, part);
  if (changed) {
    const uint32_t w = wave_sum(nchg);
    if (l == 0 && w) atomicAdd(changed, (unsigned long long)w);
  }
}

// Split-precision E-step (one Lloyd step of every row): x = xh + xl and c = ch + cl in bf16 (hi and the
// rounded rest), x.c ~ xh.ch + xh.cl + xl.ch on v_mfma_f32_32x32x16_bf16 (products exact in f32, f32
// accumulation): |x.c - approx| <= (3 u^2 + gamma_336) sum |x_i c_i| with u = 2^-8, under 6.6e-5 |x| |c|,
// so a score |c|^2 - 2 x.c is off by <= 1.32e-4 |x| |c|, and the f32 kernel's (k_km_assign_mfma) by
// <= 2 gamma_128 |x||c| = 1.5e-5 |x||c| (same |c|^2 in both). A row is decided when its two smallest
// approximate scores differ by more than twice the sum, 2.94e-4 |x| max|c|: the exact f32 step would
// then pick the same cluster, strictly. KMS_SEP = 6e-4 keeps a 2x margin over that. Decided rows get
// their label and sums here; the others (near ties, ~1-2 % of rows on session embeddings) are
// listed for the exact kernel (per block in LDS, one global atomic per block). Same output layout as
// k_km_assign_mfma: lane (i, h) ends with row i's scores of clusters (r & 3) + 8 (r >> 2) + 4 h.
typedef __bf16 km_bf16x8 __attribute__((ext_vector_type(8)));
constexpr float KMS_SEP = 6e-4f;
constexpr int KMS_AMB = 1024;  // near-tie rows staged per block before they spill to the global list
__device__ __forceinline__ uint16_t km_bf16(float f) {  // round to nearest even (finite values)
  uint32_t u = __float_as_uint(f);
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}
typedef __bf16 km_bf16x2 __attribute__((ext_vector_type(2)));
typedef float km_f32x2 __attribute__((ext_vector_type(2)));
// v = hi + lo + r: hi = RN_bf16(v), lo = RN_bf16(v - hi) (v_cvt_pk_bf16_f32, round to nearest even;
// v - hi is exact in f32), |r| <= u^2 |v|
__device__ __forceinline__ void km_split8(const float (&v)[8], uint4& hi, uint4& lo) {
  uint32_t hw[4], lw[4];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const km_f32x2 a = {v[2 * p], v[2 * p + 1]};
    const uint32_t hu = __builtin_bit_cast(uint32_t, __builtin_convertvector(a, km_bf16x2));
    const km_f32x2 r = {v[2 * p] - __uint_as_float(hu << 16), v[2 * p + 1] - __uint_as_float(hu & 0xFFFF0000u)};
    hw[p] = hu;
    lw[p] = __builtin_bit_cast(uint32_t, __builtin_convertvector(r, km_bf16x2));
  }
  hi = make_uint4(hw[0], hw[1], hw[2], hw[3]);
  lo = make_uint4(lw[0], lw[1], lw[2], lw[3]);
}

// Distance bounds across Lloyd steps (Hamerly's single lower bound), so a step scores only the rows
// whose label could change. Per row: ub >= |x - c_a| (a = its label) and lb <= min_{j != a} |x - c_j|,
// both for the centres Cp the bounds were last made valid for. A step first takes
// delta_j >= |C_j - Cp_j| (k_km_delta, then Cp = C), so by the triangle inequality u = ub + delta_a and
// l = lb - max_{j != a} delta_j bound the distances to the new centres C. The exact f32 kernel
// (k_km_assign_mfma) scores s_j = |c_j|^2 - 2 x.c_j within 2e-5 cmax (|x| + cmax) (its MFMA dot,
// the stored |c|^2 and two roundings; cmax = max |c_j|), so it keeps label a whenever
// l^2 - u^2 > 4e-5 cmax (|x| + cmax); with |x| <= u + cmax the filter asks for
// (l - u)(l + u) > KMB_SKIP cmax (u + 2 cmax), KMB_SKIP = 2e-4 (5x margin). Such rows keep their
// label and sums (nothing to move); the others are listed for the split-precision pass, which
// rebuilds their bounds from its approximate scores (error within 2e-4 cmax (|x| + cmax) there, so
// u^2 <= m + |x|^2 + e and l^2 >= m2 + |x|^2 - e with m, m2 the two smallest scores), and near ties
// get lb = 0 (scored again next step). Every bound is rounded outwards (relative 2^-20 / 1e-6).
constexpr float KMB_SKIP = 2e-4f;
constexpr float KMB_ERR = 2e-4f;
// Half-precision E-step (H16: the rows as f16, xh = RN_f16(x) with the row's rounding residual e = x - xh, |e| <=
// 2^-11 |x| + 2^-25 sqrt(dim); c = ch + cl in f16 within 2^-22 |c| + 2^-25 per element): x.c ~ xh.ch + xh.cl on
// v_mfma_f32_32x32x16_f16 (products exact, f32 sums of 224 terms) is off by <= |e.c| + |xh.(c - ch - cl)| + the
// sums' rounding <= |e| |c| + 1.45e-5 |x| |c| + 3e-7 (|x| + |c|) (Cauchy-Schwarz on the residual), a score by
// twice that. Decided when the two smallest scores differ by more than twice the sum with the exact kernel's
// 1.5e-5 |x||c| (4 |e| cmax + 8.8e-5 |x| cmax), kept with a 2x margin: KMH_SEP_E = 8 (|e| cmax) + KMH_SEP_X = 1.76e-4
// (|x| cmax) + KMH_ABS = 2.5e-6 (|x| + cmax). |e| is the row's own residual norm (ottohip_kmeans_attach_half, rounded
// up), ~0.3 of the worst case 2^-11 |x| the first version assumed for every row (KMH_SEP = 4.1e-3 |x| cmax, 8.6 %
// of the scored rows near ties on session embeddings). Every row reads 208 B instead of 400.
constexpr float KMH_SEP_E = 8.f;
constexpr float KMH_SEP_X = 1.76e-4f;
constexpr float KMH_ABS = 2.5e-6f;
// score error for the rebuilt distance bounds: 2 |e| cmax + 2.9e-5 |x| cmax with a 1.2x margin, plus |c|^2's f32
// rounding (cmax^2 units)
constexpr float KMH_ERR_E = 2.4f;
constexpr float KMH_ERR_X = 3.5e-5f;
constexpr float KMH_ERR_C = 1.2e-5f;
constexpr int KMH_AMB = 8192;       // near-tie rows staged per block (~5 % of a block's ~50 k rows)
constexpr int KMH_MT = 768;         // H16 block: 12 waves (136-170 VGPRs: 3 waves per SIMD)
// KMH_MAXABS: the f16 copy is refused above this |x| (f16 overflows at 65504; centroids are row means, so their
// f16 hi / lo split stays finite below it). The bits of max |x| (NaN included: its bits exceed inf's) reach
// *amax by one atomicMax per wave.
constexpr float KMH_MAXABS = 3.0e4f;
__global__ void k_km_half_rows(const float* __restrict__ X, int64_t n, int dim, int kc, uint4* __restrict__ X16,
                               float* __restrict__ xn2, unsigned* __restrict__ amax) {
  // one wave per row: lanes over the row's 16-B f16 chunks (kc per row, zero padded past dim), squared norm by
  // a wave sum of the f32 elements
  const int64_t row = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int l = threadIdx.x & 63;
  if (row >= n) return;
  const float* xp = X + row * dim;
  float ss = 0.f, es = 0.f;
  unsigned mx = 0u;  // bits of max |x| over the lane's elements (non-negative floats order as unsigned ints)
  if (l < kc) {
    _Float16 h[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int d = 8 * l + j;
      const float v = d < dim ? xp[d] : 0.f;
      ss += v * v;
      h[j] = (_Float16)v;
      const float r = v - (float)h[j];  // exact in f32
      es += r * r;
      mx = max(mx, __float_as_uint(v) & 0x7FFFFFFFu);
    }
    X16[row * kc + l] = __builtin_bit_cast(uint4, h);
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    ss += __shfl_xor(ss, o);
    es += __shfl_xor(es, o);
    mx = max(mx, (unsigned)__shfl_xor((int)mx, o));
  }
  if (l == 0) {
    // |x - xh| rounded up (f32 sum of <= 128 squares: relative error < 1e-5, sqrt half an ulp)
    reinterpret_cast<float2*>(xn2)[row] = make_float2(ss, sqrtf(es * 1.00002f) * 1.000001f);
    if (mx > __float_as_uint(KMH_MAXABS)) atomicMax(amax, mx);
  }
}
// dl: [0, 64) delta_j, [64] largest delta, [65] second largest, [66] its cluster (as float), [67] cmax
constexpr int KMD_T = 1024;  // k_km_delta: 16 waves, one centroid per wave at a time, lanes over the dims
__global__ __launch_bounds__(KMD_T) void k_km_delta(const float* __restrict__ C, float* __restrict__ Cp,
                                                     const float* __restrict__ cn, int k, int dim, int force,
                                                     float* __restrict__ dl, const int* __restrict__ gate,
                                                     unsigned long long* __restrict__ n_eval) {
  if (gate && __builtin_amdgcn_readfirstlane(*gate)) return;  // stopped: Cp stays the bounds' centres
  __shared__ float sdl[64];
  const int wv = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (threadIdx.x < 64) sdl[threadIdx.x] = 0.f;
  __syncthreads();
  for (int j = wv; j < k; j += KMD_T / 64) {  // |C_j - Cp_j| in f64, rounded up
    double s = 0.0;
    for (int i = l; i < dim; i += 64) {
      const double t = (double)C[(int64_t)j * dim + i] - (double)Cp[(int64_t)j * dim + i];
      s += t * t;
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o);
    if (l == 0) sdl[j] = force ? INFINITY : (float)(sqrt(s) * (1.0 + 1e-6));
  }
  __syncthreads();  // every read of Cp before it is overwritten
  for (int i = threadIdx.x; i < k * dim; i += KMD_T) Cp[i] = C[i];
  if (wv != 0) return;
  const int j = l;
  const float d = j < k ? sdl[j] : 0.f;
  // largest and second largest delta (ties: any cluster holding the largest, the second equals it)
  float m1 = d;
  int a1 = j;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const float pm = __shfl_xor(m1, o);
    const int pa = __shfl_xor(a1, o);
    if (pm > m1 || (pm == m1 && pa < a1)) { m1 = pm; a1 = pa; }
  }
  float m2 = j == a1 ? 0.f : d;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) m2 = fmaxf(m2, __shfl_xor(m2, o));
  float c2 = j < k ? cn[j] : 0.f;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) c2 = fmaxf(c2, __shfl_xor(c2, o));
  dl[j] = d;
  if (j == 0) {
    dl[64] = m1;
    dl[65] = m2;
    dl[66] = (float)a1;
    dl[67] = sqrtf(c2) * 1.000001f;
    *n_eval = 0;
  }
}

// rows whose bounds leave their label certain keep it (bounds moved to the new centres); the
// others are listed in row order: a block takes KMF_PER * 256 consecutive rows, one device atomic
// per block reserves its list range
constexpr int KMF_PER = 16;
__global__ __launch_bounds__(256) void k_km_filter(int64_t n, int k, const int32_t* __restrict__ label,
                                                   float* __restrict__ ub, float* __restrict__ lb,
                                                   const float* __restrict__ dl, uint32_t* __restrict__ erows,
                                                   unsigned long long* __restrict__ n_eval,
                                                   const int* __restrict__ gate) {
  if (gate && __builtin_amdgcn_readfirstlane(*gate)) return;
  __shared__ float sd[68];
  __shared__ uint32_t wc[KMF_PER * 4];
  __shared__ unsigned long long base;
  if (threadIdx.x < 68) sd[threadIdx.x] = dl[threadIdx.x];
  __syncthreads();
  const float d1 = sd[64], d2 = sd[65], cmax = sd[67];
  const int a1 = (int)sd[66];
  const int wv = threadIdx.x >> 6;
  const int64_t r0 = (int64_t)blockIdx.x * (KMF_PER * 256);
  uint32_t evm = 0;  // bit j: row r0 + j * 256 + tid is scored
#pragma unroll  // every row's loads in flight together, unconditionally (4 rows at a time behind the label
                // branch: 85 us per step at 12.9 M rows)
  for (int j = 0; j < KMF_PER; ++j) {
    const int64_t i = r0 + j * 256 + threadIdx.x;
    const int64_t ic = i < n ? i : n - 1;
    const int32_t a = label[ic];
    const float ubv = ub[ic], lbv = lb[ic];
    const bool lab_ok = a >= 0 && a < k;
    const float u = (ubv + sd[lab_ok ? a : 0]) * (1.f + 0x1p-20f);
    const float lo = (lbv - (a == a1 ? d2 : d1)) * (1.f - 0x1p-20f);
    const bool keep = i < n && lab_ok && lo > u && (lo - u) * (lo + u) > KMB_SKIP * cmax * (u + 2.f * cmax);
    if (keep) {
      ub[i] = u;
      lb[i] = lo;
    }
    const bool ev = i < n && !keep;
    evm |= ev ? (1u << j) : 0u;
    const uint64_t m = __ballot(ev);
    if (lane_id() == 0) wc[j * 4 + wv] = (uint32_t)__popcll(m);
  }
  __syncthreads();
  if (threadIdx.x < 64) {  // exclusive scan of the (row step, wave) counts, one reservation
    const uint32_t c = wc[threadIdx.x];
    const uint32_t incl = wave_incl_scan(c);
    wc[threadIdx.x] = incl - c;
    if (threadIdx.x == 63) base = incl ? atomicAdd(n_eval, (unsigned long long)incl) : 0ull;
  }
  __syncthreads();
  const unsigned long long b0 = base;
#pragma unroll 4
  for (int j = 0; j < KMF_PER; ++j) {
    const bool ev = (evm >> j) & 1u;
    const uint64_t m = __ballot(ev);
    if (ev) erows[b0 + wc[j * 4 + wv] + mbcnt(m)] = (uint32_t)(r0 + j * 256 + threadIdx.x);
  }
}

// BL: score the rows erows[0, *n_eval) (k_km_filter's list) and rebuild their bounds
typedef _Float16 km_f16x8 __attribute__((ext_vector_type(8)));
// v = hi + lo + r in f16 (round to nearest), |r| <= 2^-22 |v| + 2^-25
__device__ __forceinline__ void km_split8_h(const float (&v)[8], uint4& hi, uint4& lo) {
  _Float16 h[8], r[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    h[j] = (_Float16)v[j];
    r[j] = (_Float16)(v[j] - (float)h[j]);
  }
  hi = __builtin_bit_cast(uint4, h);
  lo = __builtin_bit_cast(uint4, r);
}
// H16: the rows from X16 (f16, 2 KS chunks per row) and their squared norms xn2 (ottohip_kmeans_attach_half)
// MV: a decided row whose label changes is listed {row, old | new << 16} in the block's own region of mv_list
// (mv_cap entries per block, count in mv_cnt[block]); k_km_ties folds the regions into the sums (no LDS sums,
// no per-row gather of the f32 row while the wave waits)
template <int NB, int KS, bool BL = false, bool H16 = false, bool MV = false>
__global__ __launch_bounds__(H16 ? KMH_MT : KM_MT, H16 ? 1 : 2) void k_km_assign_split(const float* __restrict__ X, int64_t n, int dim,
                                                             const float* __restrict__ C, const float* __restrict__ cn,
                                                             int k, int32_t* __restrict__ label,
                                                             unsigned long long* __restrict__ sums,
                                                             unsigned long long* __restrict__ cnt,
                                                             unsigned long long* __restrict__ changed,
                                                             const int* __restrict__ gate,
                                                             uint32_t* __restrict__ amb_rows,
                                                             unsigned long long* __restrict__ n_amb,
                                                             const uint32_t* __restrict__ erows = nullptr,
                                                             const unsigned long long* __restrict__ n_eval = nullptr,
                                                             float* __restrict__ ub = nullptr,
                                                             float* __restrict__ lb = nullptr,
                                                             const uint4* __restrict__ X16 = nullptr,
                                                             const float* __restrict__ xn2 = nullptr,  // {|x|^2, |x - xh|}
                                                             uint2* __restrict__ mv_list = nullptr,
                                                             uint32_t* __restrict__ mv_cnt = nullptr,
                                                             uint32_t mv_cap = 0) {
  if (gate && __builtin_amdgcn_readfirstlane(*gate)) return;
  constexpr int AMB = H16 ? KMH_AMB : KMS_AMB;
  constexpr int MT = H16 ? KMH_MT : KM_MT;  // threads per block (H16: 12 waves, its registers allow 3 per SIMD)
  extern __shared__ unsigned long long smem64[];
  uint4* Cf = reinterpret_cast<uint4*>(smem64);                               // [NB][KS][hi, lo][64]
  unsigned long long* ls = reinterpret_cast<unsigned long long*>(Cf + NB * KS * 2 * 64);  // k * dim sums
  unsigned long long* lc = ls + (MV ? 0 : k * dim);                            // k counts
  int32_t* labl = reinterpret_cast<int32_t*>(lc + (MV ? 0 : k));              // [waves][3][32]
  float* cnl = reinterpret_cast<float*>(labl + (MT / 64) * 96);             // [64]
  uint32_t* amb = reinterpret_cast<uint32_t*>(cnl + 64);                       // [AMB]
  __shared__ uint32_t namb, nmv;
  __shared__ unsigned long long abase;
  const int tid = threadIdx.x, l = tid & 63, wv = tid >> 6, h = l >> 5, i32 = l & 31;
  // centroid fragments: lane (r, h) of block b, k-step s holds centroid 32 b + r, dims 16 s + 8 h .. + 7
  for (int e = tid; e < NB * KS * 64; e += MT) {
    const int ll = e & 63, sb = e >> 6, s_ = sb % KS, b = sb / KS;
    const int c = b * 32 + (ll & 31), d0 = 16 * s_ + 8 * (ll >> 5);
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (c < k && d0 + j < dim) ? C[(int64_t)c * dim + d0 + j] : 0.f;
    uint4 hi, lo;
    if constexpr (H16) km_split8_h(v, hi, lo);
    else km_split8(v, hi, lo);
    Cf[(sb * 2 + 0) * 64 + ll] = hi;
    Cf[(sb * 2 + 1) * 64 + ll] = lo;
  }
  if (tid < 64) cnl[tid] = cn[tid];
  if constexpr (!MV)
    for (int i = tid; i < k * dim + k; i += MT) ls[i] = 0ull;
  if (tid == 0) { namb = 0; nmv = 0; }
  __syncthreads();
  float c2 = l < k ? cnl[l] : 0.f;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) c2 = fmaxf(c2, __shfl_xor(c2, o));
  const float cmax = sqrtf(c2);
  uint32_t nchg = 0;
  const int64_t nl = BL ? (int64_t)__builtin_amdgcn_readfirstlane((int)*n_eval) : n;  // rows to score
  const int64_t ntile = (nl + 31) >> 5;
  const int64_t nwv = (int64_t)gridDim.x * (MT / 64);
  // the next tile's rows (and its rows' current labels) are loaded while this tile is scored
  float4 raw[H16 ? 1 : 2 * KS];
  uint4 raw16[H16 ? KS : 1];
  float xn_n = 0.f, en_n = 0.f;
  int32_t lab_n = -1;
  int64_t row_n = 0;
  auto load = [&](int64_t tt) __attribute__((always_inline)) {
    const int64_t ri = (tt << 5) + i32 < nl ? (tt << 5) + i32 : nl - 1;
    const int64_t rr = BL ? (int64_t)erows[ri] : ri;
    row_n = rr;
    if constexpr (H16) {
#pragma unroll
      for (int s_ = 0; s_ < KS; ++s_) {
        const int d0 = 16 * s_ + 8 * h;  // the chunk's zero padding past dim is stored: only wholly-past chunks skip
        raw16[s_] = d0 < dim ? X16[rr * ((dim + 7) >> 3) + 2 * s_ + h] : make_uint4(0u, 0u, 0u, 0u);
      }
      const float2 ne = reinterpret_cast<const float2*>(xn2)[rr];
      xn_n = ne.x;
      en_n = ne.y;
    } else {
      const float* xp = X + rr * dim;
#pragma unroll
      for (int s_ = 0; s_ < KS; ++s_) {
        const int d0 = 16 * s_ + 8 * h;  // dim % 4 == 0: a 16-B piece is all in or all out
        raw[2 * s_] = d0 < dim ? *reinterpret_cast<const float4*>(xp + d0) : make_float4(0.f, 0.f, 0.f, 0.f);
        raw[2 * s_ + 1] = d0 + 4 < dim ? *reinterpret_cast<const float4*>(xp + d0 + 4) : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
    lab_n = label[rr];
  };
  const int64_t t_first = (int64_t)blockIdx.x * (MT / 64) + wv;
  if (t_first < ntile) load(t_first);
  for (int64_t t = t_first; t < ntile; t += nwv) {
    const int64_t r0 = t << 5;
    const bool in_r = r0 + i32 < nl;
    const int64_t row = row_n;
    km_bf16x8 xh[H16 ? 1 : KS], xl[H16 ? 1 : KS];
    km_f16x8 xq[H16 ? KS : 1];
    float xs = 0.f, ee = 0.f;
    if constexpr (H16) {
#pragma unroll
      for (int s_ = 0; s_ < KS; ++s_) xq[s_] = __builtin_bit_cast(km_f16x8, raw16[s_]);
      xs = xn_n;
      ee = en_n;
    } else {
#pragma unroll
      for (int s_ = 0; s_ < KS; ++s_) {
        const float4 p0 = raw[2 * s_], p1 = raw[2 * s_ + 1];
        const float v[8] = {p0.x, p0.y, p0.z, p0.w, p1.x, p1.y, p1.z, p1.w};
#pragma unroll
        for (int j = 0; j < 8; ++j) xs += v[j] * v[j];
        uint4 hi, lo;
        km_split8(v, hi, lo);
        xh[s_] = __builtin_bit_cast(km_bf16x8, hi);
        xl[s_] = __builtin_bit_cast(km_bf16x8, lo);
      }
    }
    const int32_t lab_cur = lab_n;
    if (t + nwv < ntile) load(t + nwv);
    if constexpr (!H16) xs += __shfl_xor(xs, 32);
    km_f32x16 acc0 = {}, acc1 = {};
#pragma unroll
    for (int s_ = 0; s_ < KS; ++s_) {
      if constexpr (H16) {  // xh.ch + xh.cl
        const km_f16x8 ch0 = __builtin_bit_cast(km_f16x8, Cf[((0 * KS + s_) * 2 + 0) * 64 + l]);
        const km_f16x8 cl0 = __builtin_bit_cast(km_f16x8, Cf[((0 * KS + s_) * 2 + 1) * 64 + l]);
        acc0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ch0, xq[s_], acc0, 0, 0, 0);
        acc0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(cl0, xq[s_], acc0, 0, 0, 0);
        if (NB == 2) {
          const km_f16x8 ch1 = __builtin_bit_cast(km_f16x8, Cf[((1 * KS + s_) * 2 + 0) * 64 + l]);
          const km_f16x8 cl1 = __builtin_bit_cast(km_f16x8, Cf[((1 * KS + s_) * 2 + 1) * 64 + l]);
          acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ch1, xq[s_], acc1, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(cl1, xq[s_], acc1, 0, 0, 0);
        }
      } else {
        const km_bf16x8 ch0 = __builtin_bit_cast(km_bf16x8, Cf[((0 * KS + s_) * 2 + 0) * 64 + l]);
        const km_bf16x8 cl0 = __builtin_bit_cast(km_bf16x8, Cf[((0 * KS + s_) * 2 + 1) * 64 + l]);
        acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ch0, xh[s_], acc0, 0, 0, 0);
        acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ch0, xl[s_], acc0, 0, 0, 0);
        acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cl0, xh[s_], acc0, 0, 0, 0);
        if (NB == 2) {
          const km_bf16x8 ch1 = __builtin_bit_cast(km_bf16x8, Cf[((1 * KS + s_) * 2 + 0) * 64 + l]);
          const km_bf16x8 cl1 = __builtin_bit_cast(km_bf16x8, Cf[((1 * KS + s_) * 2 + 1) * 64 + l]);
          acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ch1, xh[s_], acc1, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ch1, xl[s_], acc1, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cl1, xh[s_], acc1, 0, 0, 0);
        }
      }
    }
    // approximate scores |c|^2 - 2 x.c; the smallest, the lowest cluster holding it, the second smallest
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float4 n0 = *reinterpret_cast<const float4*>(cnl + 8 * j + 4 * h);
      acc0[4 * j + 0] = n0.x - 2.f * acc0[4 * j + 0];
      acc0[4 * j + 1] = n0.y - 2.f * acc0[4 * j + 1];
      acc0[4 * j + 2] = n0.z - 2.f * acc0[4 * j + 2];
      acc0[4 * j + 3] = n0.w - 2.f * acc0[4 * j + 3];
      if (NB == 2) {
        const float4 n1 = *reinterpret_cast<const float4*>(cnl + 32 + 8 * j + 4 * h);
        acc1[4 * j + 0] = n1.x - 2.f * acc1[4 * j + 0];
        acc1[4 * j + 1] = n1.y - 2.f * acc1[4 * j + 1];
        acc1[4 * j + 2] = n1.z - 2.f * acc1[4 * j + 2];
        acc1[4 * j + 3] = n1.w - 2.f * acc1[4 * j + 3];
      }
    }
    float m = INFINITY;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      m = fminf(m, acc0[r]);
      if (NB == 2) m = fminf(m, acc1[r]);
    }
    int mc = 64;
#pragma unroll
    for (int r = 15; r >= 0; --r) {
      if (NB == 2) mc = acc1[r] == m ? 32 + (r & 3) + 8 * (r >> 2) + 4 * h : mc;
    }
#pragma unroll
    for (int r = 15; r >= 0; --r) mc = acc0[r] == m ? (r & 3) + 8 * (r >> 2) + 4 * h : mc;
    {
      const float pm = __shfl_xor(m, 32);
      const int pc = __shfl_xor(mc, 32);
      if (pm < m || (pm == m && pc < mc)) { m = pm; mc = pc; }
    }
    float m2 = INFINITY;  // smallest score of any other cluster
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int c0 = (r & 3) + 8 * (r >> 2) + 4 * h;
      m2 = fminf(m2, c0 == mc ? INFINITY : acc0[r]);
      if (NB == 2) m2 = fminf(m2, c0 + 32 == mc ? INFINITY : acc1[r]);
    }
    m2 = fminf(m2, __shfl_xor(m2, 32));
    const bool decided = H16 ? m2 - m > (KMH_SEP_E * ee + KMH_SEP_X * sqrtf(xs)) * cmax + KMH_ABS * (sqrtf(xs) + cmax)
                             : m2 - m > KMS_SEP * sqrtf(xs) * cmax;
    if (BL && h == 0 && in_r) {  // the row's bounds for these centres (near ties: none, lb = 0)
      const float cm = cmax * 1.000001f;
      const float e = H16 ? (KMH_ERR_E * ee + KMH_ERR_X * sqrtf(xs) * 1.0001f + KMH_ERR_C * cm) * cm + KMH_ABS * (sqrtf(xs) + cm)
                          : KMB_ERR * cm * (sqrtf(xs) * 1.0001f + cm);
      ub[row] = decided ? sqrtf(fmaxf(m + xs * 1.00001f + e, 0.f)) * 1.000001f : 0.f;
      lb[row] = decided ? sqrtf(fmaxf(m2 + xs * 0.99999f - e, 0.f)) * 0.999999f : 0.f;
    }
    const uint32_t mi = (uint32_t)mc;
    const bool mine = h == 0 && in_r && decided;
    int32_t old = -1;
    if (mine) {
      old = lab_cur;
      nchg += old != (int32_t)mi;
      if (old != (int32_t)mi) label[row] = (int32_t)mi;
    }
    // near ties: staged in LDS for the exact kernel (overflow: straight to the global list)
    const bool tie = h == 0 && in_r && !decided;
    const uint64_t tm = __ballot(tie);
    if (tm) {
      uint32_t b = 0;
      if (l == 0) b = atomicAdd(&namb, (uint32_t)__popcll(tm));
      b = __shfl(b, 0);
      if (tie) {
        const uint32_t p = b + mbcnt(tm);
        if (p < (uint32_t)AMB) amb[p] = (uint32_t)row;
        else amb_rows[atomicAdd(n_amb, 1ull)] = (uint32_t)row;
      }
    }
    if constexpr (MV) {
      const bool mvf = mine && old != (int32_t)mi;
      const uint64_t mm = __ballot(mvf);
      if (mm) {
        uint32_t b = 0;
        if (l == 0) b = atomicAdd(&nmv, (uint32_t)__popcll(mm));
        b = __shfl(b, 0);
        if (mvf)
          mv_list[(size_t)blockIdx.x * mv_cap + b + mbcnt(mm)] =
              make_uint2((uint32_t)row, (old < 0 ? 0xFFFFu : (uint32_t)old) | (mi << 16));
      }
    } else {
      km_move_rows(X, dim, ls, lc, labl + wv * 96, mine && old != (int32_t)mi, row, mi, old);
    }
  }
  __syncthreads();
  if constexpr (MV) {
    if (tid == 0) mv_cnt[blockIdx.x] = nmv;
  } else {
    for (int i = tid; i < k * dim; i += MT)
      if (ls[i]) atomicAdd(&sums[i], ls[i]);
    for (int i = tid; i < k; i += MT)
      if (lc[i]) atomicAdd(&cnt[i], lc[i]);
  }
  const uint32_t na = namb < (uint32_t)AMB ? namb : (uint32_t)AMB;
  if (tid == 0) abase = na ? atomicAdd(n_amb, (unsigned long long)na) : 0ull;
  __syncthreads();
  for (uint32_t i = tid; i < na; i += MT) amb_rows[abase + i] = amb[i];
  const uint32_t w = wave_sum(nchg);
  if (l == 0 && w) atomicAdd(changed, (unsigned long long)w);
}

// The H16 pass of the bounded batched steps with move lists (the production E-step of C2), rebuilt for issue
// cost (k_km_assign_split<NB, KS, true, true, true> spent ~445 VALU instructions per 32-row tile):
// - two register sets in ping-pong (no copy of the prefetched row into the working registers) and the row
//   indices of erows two tiles ahead, so a row gather never waits on its index load;
// - rows of ceil(dim / 8) chunks read unconditionally (the chunk past a row is the next row's first, masked);
// - accumulators start at -|c|^2 / 2, so acc = x.c - |c|^2 / 2 = -score / 2 comes out of the MFMA chain (no
//   per-score fma; the chain's f32 rounding now also covers |c|^2 / 2: + 1.45e-5 cmax^2 per score, in the
//   decision threshold (KMH_SEP_C) and the rebuilt bounds (KMH_ERR_C16));
// - largest and second largest acc by a max / med3 chain (2 ops per score), then the lowest cluster holding
//   the largest (the approximate argmin only labels rows whose gap is above the threshold, where it is unique).
// the cluster bits in the 6 low mantissa bits (k_km_split16) move a value by < 64 ulp = 7.63e-6 |acc|, |acc| <=
// |x| cmax + cmax^2 / 2: a score gap by <= 3.05e-5 |x| cmax + 1.53e-5 cmax^2 (2x margin below), a score by half
constexpr float KMH_SEP_X16 = 1.76e-4f + 6.1e-5f;  // |x| cmax units (2x margin)
constexpr float KMH_SEP_C = 5.8e-5f + 3.1e-5f;     // cmax^2 units (2x margin)
constexpr float KMH_ERR_X16 = 3.5e-5f + 1.9e-5f;   // |x| cmax units (1.2x margin)
constexpr float KMH_ERR_C16 = 2.5e-5f + 9.2e-6f;   // cmax^2 units: chain rounding of |c|^2 / 2, |c|^2's own, cluster bits
template <int NB, int KS>
__global__ __launch_bounds__(KMH_MT, 1) void k_km_split16(int64_t n, int dim, const float* __restrict__ C,
                                                          const float* __restrict__ cn, int k,
                                                          int32_t* __restrict__ label,
                                                          unsigned long long* __restrict__ changed,
                                                          const int* __restrict__ gate,
                                                          uint32_t* __restrict__ amb_rows,
                                                          unsigned long long* __restrict__ n_amb,
                                                          const uint32_t* __restrict__ erows,
                                                          const unsigned long long* __restrict__ n_eval,
                                                          float* __restrict__ ub, float* __restrict__ lb,
                                                          const uint4* __restrict__ X16, const float2* __restrict__ xne,
                                                          uint2* __restrict__ mv_list, uint32_t* __restrict__ mv_cnt,
                                                          uint32_t mv_cap) {
  if (gate && __builtin_amdgcn_readfirstlane(*gate)) return;
  constexpr int MT = KMH_MT, W = MT / 64;
  extern __shared__ unsigned long long smem64[];
  uint4* Cf = reinterpret_cast<uint4*>(smem64);                  // [NB][KS][hi, lo][64]
  float* cnl = reinterpret_cast<float*>(Cf + NB * KS * 2 * 64);  // [64]: -|c|^2 / 2
  uint32_t* amb = reinterpret_cast<uint32_t*>(cnl + 64);          // [KMH_AMB]
  __shared__ uint32_t namb, nmv;
  __shared__ unsigned long long abase;
  const int tid = threadIdx.x, l = tid & 63, wv = tid >> 6, h = l >> 5, i32 = l & 31;
  for (int e = tid; e < NB * KS * 64; e += MT) {
    const int ll = e & 63, sb = e >> 6, s_ = sb % KS, b = sb / KS;
    const int c = b * 32 + (ll & 31), d0 = 16 * s_ + 8 * (ll >> 5);
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (c < k && d0 + j < dim) ? C[(int64_t)c * dim + d0 + j] : 0.f;
    uint4 hi, lo;
    km_split8_h(v, hi, lo);
    Cf[(sb * 2 + 0) * 64 + ll] = hi;
    Cf[(sb * 2 + 1) * 64 + ll] = lo;
  }
  // padding clusters: -FLT_MAX (finite, so the cluster bits below keep it a number, and never the largest)
  if (tid < 64) cnl[tid] = tid < k ? -0.5f * cn[tid] : -3.402823466e38f;
  if (tid == 0) { namb = 0; nmv = 0; }
  __syncthreads();
  float c2 = l < k ? cn[l] : 0.f;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) c2 = fmaxf(c2, __shfl_xor(c2, o));
  const float cmax = sqrtf(c2);
  const int kch = (dim + 7) >> 3;
  const uint32_t lastmask = 2 * (KS - 1) + h < kch ? ~0u : 0u;  // the lane's last chunk lies inside the row
  uint32_t nchg = 0;
  const int64_t nl = (int64_t)__builtin_amdgcn_readfirstlane((int)*n_eval);
  const int64_t ntile = (nl + 31) >> 5;
  const int64_t nwv = (int64_t)gridDim.x * W;
  auto ridx = [&](int64_t tt) __attribute__((always_inline)) -> uint32_t {
    const int64_t ri = (tt << 5) + i32 < nl ? (tt << 5) + i32 : nl - 1;
    return erows[ri];
  };
  auto load = [&](uint4 (&x)[KS], float2& ne, int32_t& lab, uint32_t rr) __attribute__((always_inline)) {
    const uint4* p = X16 + (size_t)rr * kch + h;
#pragma unroll
    for (int s_ = 0; s_ < KS; ++s_) x[s_] = p[2 * s_];
    ne = xne[rr];
    lab = label[rr];
  };
  auto score = [&](const uint4 (&x)[KS], float2 ne, int32_t lab_cur, uint32_t row, int64_t t)
                   __attribute__((always_inline)) {
    const bool in_r = (t << 5) + i32 < nl;
    km_f32x16 acc0, acc1;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float4 n0 = *reinterpret_cast<const float4*>(cnl + 8 * j + 4 * h);
      acc0[4 * j + 0] = n0.x; acc0[4 * j + 1] = n0.y; acc0[4 * j + 2] = n0.z; acc0[4 * j + 3] = n0.w;
      if (NB == 2) {
        const float4 n1 = *reinterpret_cast<const float4*>(cnl + 32 + 8 * j + 4 * h);
        acc1[4 * j + 0] = n1.x; acc1[4 * j + 1] = n1.y; acc1[4 * j + 2] = n1.z; acc1[4 * j + 3] = n1.w;
      }
    }
#pragma unroll
    for (int s_ = 0; s_ < KS; ++s_) {
      uint4 xv = x[s_];
      if (s_ == KS - 1) {  // masked here, not at the load (a mask there waits for the load)
        xv.x &= lastmask;
        xv.y &= lastmask;
        xv.z &= lastmask;
        xv.w &= lastmask;
      }
      const km_f16x8 xq = __builtin_bit_cast(km_f16x8, xv);
      const km_f16x8 ch0 = __builtin_bit_cast(km_f16x8, Cf[((0 * KS + s_) * 2 + 0) * 64 + l]);
      const km_f16x8 cl0 = __builtin_bit_cast(km_f16x8, Cf[((0 * KS + s_) * 2 + 1) * 64 + l]);
      acc0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ch0, xq, acc0, 0, 0, 0);
      acc0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(cl0, xq, acc0, 0, 0, 0);
      if (NB == 2) {
        const km_f16x8 ch1 = __builtin_bit_cast(km_f16x8, Cf[((1 * KS + s_) * 2 + 0) * 64 + l]);
        const km_f16x8 cl1 = __builtin_bit_cast(km_f16x8, Cf[((1 * KS + s_) * 2 + 1) * 64 + l]);
        acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ch1, xq, acc1, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(cl1, xq, acc1, 0, 0, 0);
      }
    }
    // +inf the compiler cannot see as a constant: med3(a, b, +inf) would fold to a max that canonicalizes its
    // operands (one more instruction per score)
    // each value carries its cluster in the 6 low mantissa bits (within 63 ulp: 7.6e-6 |acc|, in the
    // thresholds), so the largest value names its cluster: no compare / select scan for the argmax
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const uint32_t c0 = (uint32_t)((r & 3) + 8 * (r >> 2) + 4 * h);
      acc0[r] = __uint_as_float((__float_as_uint(acc0[r]) & ~63u) | c0);
      if (NB == 2) acc1[r] = __uint_as_float((__float_as_uint(acc1[r]) & ~63u) | (c0 + 32u));
    }
    // +inf the compiler cannot see as a constant: med3(a, b, +inf) would fold to a max that canonicalizes its
    // operands (one more instruction per score)
    const float pinf = __uint_as_float(0x7F800000u | ((uint32_t)k >> 31));
    float a1 = -INFINITY, a2 = -INFINITY;  // largest, second largest (a tie at the top: a2 == a1)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      a2 = __builtin_amdgcn_fmed3f(a1, a2, acc0[r]);
      a1 = __builtin_amdgcn_fmed3f(a1, acc0[r], pinf);
      if (NB == 2) {
        a2 = __builtin_amdgcn_fmed3f(a1, a2, acc1[r]);
        a1 = __builtin_amdgcn_fmed3f(a1, acc1[r], pinf);
      }
    }
    {
      const float p1 = __shfl_xor(a1, 32), p2 = __shfl_xor(a2, 32);
      a2 = fmaxf(fminf(a1, p1), fmaxf(a2, p2));
      a1 = fmaxf(a1, p1);
    }
    const int mc = (int)(__float_as_uint(a1) & 63u);
    const float xs = ne.x, ee = ne.y, xn = sqrtf(xs);
    const float m = -2.f * a1, m2 = -2.f * a2;  // the two smallest approximate scores |c|^2 - 2 x.c
    const bool decided = m2 - m > (KMH_SEP_E * ee + KMH_SEP_X16 * xn + KMH_SEP_C * cmax) * cmax + KMH_ABS * (xn + cmax);
    if (h == 0 && in_r) {  // the row's bounds for these centres (near ties: none, lb = 0)
      const float cm = cmax * 1.000001f;
      const float e = (KMH_ERR_E * ee + KMH_ERR_X16 * xn * 1.0001f + KMH_ERR_C16 * cm) * cm + KMH_ABS * (xn + cm);
      ub[row] = decided ? sqrtf(fmaxf(m + xs * 1.00001f + e, 0.f)) * 1.000001f : 0.f;
      lb[row] = decided ? sqrtf(fmaxf(m2 + xs * 0.99999f - e, 0.f)) * 0.999999f : 0.f;
    }
    const int32_t mi = mc;
    const bool mvf = h == 0 && in_r && decided && lab_cur != mi;
    if (mvf) label[row] = mi;
    nchg += mvf;
    const uint64_t mm = __ballot(mvf);
    if (mm) {
      uint32_t b = 0;
      if (l == 0) b = atomicAdd(&nmv, (uint32_t)__popcll(mm));
      b = __shfl(b, 0);
      if (mvf)
        mv_list[(size_t)blockIdx.x * mv_cap + b + mbcnt(mm)] =
            make_uint2(row, (lab_cur < 0 ? 0xFFFFu : (uint32_t)lab_cur) | ((uint32_t)mi << 16));
    }
    const bool tie = h == 0 && in_r && !decided;
    const uint64_t tm = __ballot(tie);
    if (tm) {
      uint32_t b = 0;
      if (l == 0) b = atomicAdd(&namb, (uint32_t)__popcll(tm));
      b = __shfl(b, 0);
      if (tie) {
        const uint32_t p = b + mbcnt(tm);
        if (p < (uint32_t)KMH_AMB) amb[p] = row;
        else amb_rows[atomicAdd(n_amb, 1ull)] = row;
      }
    }
  };
  // tiles t0, t0 + nwv, ... of this wave: set A scores tile t while set B's rows are in flight, and back. The
  // loads are unconditional (no register merges that wait on them): past the last tile ridx gives row
  // erows[nl - 1] to every lane, one line.
  const int64_t t0 = (int64_t)blockIdx.x * W + wv;
  if (t0 < ntile) {
    uint4 xa[KS], xb[KS];
    float2 nea, neb;
    int32_t laba, labb;
    uint32_t rA = ridx(t0), rB = ridx(t0 + nwv);
    load(xa, nea, laba, rA);
    for (int64_t t = t0; t < ntile; t += 2 * nwv) {
      // each index load is issued before the row loads it must not wait behind (vmcnt counts in issue order)
      const int64_t t1 = t + nwv;
      const uint32_t rC = ridx(t + 2 * nwv);
      load(xb, neb, labb, rB);
      score(xa, nea, laba, rA, t);
      const uint32_t rD = ridx(t + 3 * nwv);
      load(xa, nea, laba, rC);
      if (t1 < ntile) score(xb, neb, labb, rB, t1);
      rA = rC;
      rB = rD;
    }
  }
  __syncthreads();
  if (tid == 0) mv_cnt[blockIdx.x] = nmv;
  const uint32_t na = namb < (uint32_t)KMH_AMB ? namb : (uint32_t)KMH_AMB;
  if (tid == 0) abase = na ? atomicAdd(n_amb, (unsigned long long)na) : 0ull;
  __syncthreads();
  for (uint32_t i = tid; i < na; i += MT) amb_rows[abase + i] = amb[i];
  const uint32_t w = wave_sum(nchg);
  if (l == 0 && w) atomicAdd(changed, (unsigned long long)w);
}

// n_init runs in lockstep over ONE read of X (C2, the reference's 10 independent runs): the split-precision
// E-step of k_km_assign_split for G runs, each with its own centroid fragments (LDS), labels, near-tie list
// and stop gate. One pass reads X for G runs (5.2 GB per pass at 12.9 M x 100) and gives the MFMA units G
// runs' products per row tile. The per-cluster sums are not kept in LDS here (G x 40 KB would not fit beside
// the fragments): every decided row whose label changes is appended to its run's move list (row, old, new),
// which k_km_apply_moves folds into the run's fixed-point sums afterwards (the same exact integer adds as
// km_move_rows). Every run sees exactly the arithmetic of k_km_assign_split (same scores, same near-tie
// test, same sums), so its labels, centres and stopping step are those of the run alone (no distance bounds).
constexpr int KMM_MAXG = 4;  // runs per pass over X
struct KmMulti {
  const float* C[KMM_MAXG];
  const float* cn[KMM_MAXG];
  int32_t* label[KMM_MAXG];
  unsigned long long* changed[KMM_MAXG];
  const int* gate[KMM_MAXG];
  uint32_t* amb_rows[KMM_MAXG];
  unsigned long long* n_amb[KMM_MAXG];
  uint2* moves[KMM_MAXG];                // {row, old | new << 16} (old 0xFFFF: none)
  unsigned long long* n_moves[KMM_MAXG];
};
template <int G, int NB, int KS>
__global__ __launch_bounds__(KM_MT, 1) void k_km_assign_split_multi(const float* __restrict__ X, int64_t n, int dim,
                                                                    int k, KmMulti P) {
  // per-run state lives in LDS (the run loop is not unrolled: one copy of the MFMA chain, no spills)
  __shared__ float s_cmax[KMM_MAXG];
  __shared__ int s_act[KMM_MAXG];
  __shared__ uint32_t s_nchg[KMM_MAXG];
  // the tile's current labels of every run (loaded with the tile's rows one tile ahead: a label load inside
  // the run loop waited for the next tile's row loads as well, vmcnt counting in order)
  __shared__ int32_t s_lab[KM_MT / 64][KMM_MAXG][64];
  bool any = false;
  for (int g = 0; g < G; ++g) any |= !(P.gate[g] && __builtin_amdgcn_readfirstlane(*P.gate[g]));
  if (!any) return;
  extern __shared__ unsigned long long smem64[];
  uint4* Cf = reinterpret_cast<uint4*>(smem64);                       // [G][NB][KS][hi, lo][64]
  float* cnl = reinterpret_cast<float*>(Cf + G * NB * KS * 2 * 64);   // [G][64]
  const int tid = threadIdx.x, l = tid & 63, h = l >> 5, i32 = l & 31;
  for (int e = tid; e < G * NB * KS * 64; e += KM_MT) {
    const int ll = e & 63, gsb = e >> 6, g = gsb / (NB * KS), sb = gsb % (NB * KS), s_ = sb % KS, b = sb / KS;
    const int c = b * 32 + (ll & 31), d0 = 16 * s_ + 8 * (ll >> 5);
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (c < k && d0 + j < dim) ? P.C[g][(int64_t)c * dim + d0 + j] : 0.f;
    uint4 hi, lo;
    km_split8(v, hi, lo);
    Cf[((g * NB * KS + sb) * 2 + 0) * 64 + ll] = hi;
    Cf[((g * NB * KS + sb) * 2 + 1) * 64 + ll] = lo;
  }
  for (int i = tid; i < G * 64; i += KM_MT) cnl[i] = P.cn[i >> 6][i & 63];
  if (tid < G) {
    s_act[tid] = !(P.gate[tid] && *P.gate[tid]);
    s_nchg[tid] = 0;
  }
  __syncthreads();
  if (tid < 64 * G) {  // wave g: the run's largest centroid norm
    const int g = tid >> 6;
    float c2 = l < k ? cnl[g * 64 + l] : 0.f;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) c2 = fmaxf(c2, __shfl_xor(c2, o));
    if (l == 0) s_cmax[g] = sqrtf(c2);
  }
  __syncthreads();
  const int64_t ntile = (n + 31) >> 5;
  const int64_t nwv = (int64_t)gridDim.x * (KM_MT / 64);
  float4 raw[2 * KS];
  int32_t lab_n[G];
  int64_t row_n = 0;
  const int wv = tid >> 6;
  auto load = [&](int64_t tt) __attribute__((always_inline)) {
    const int64_t rr = (tt << 5) + i32 < n ? (tt << 5) + i32 : n - 1;
    row_n = rr;
    const float* xp = X + rr * dim;
#pragma unroll
    for (int s_ = 0; s_ < KS; ++s_) {
      const int d0 = 16 * s_ + 8 * h;
      raw[2 * s_] = d0 < dim ? *reinterpret_cast<const float4*>(xp + d0) : make_float4(0.f, 0.f, 0.f, 0.f);
      raw[2 * s_ + 1] = d0 + 4 < dim ? *reinterpret_cast<const float4*>(xp + d0 + 4) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int g = 0; g < G; ++g) lab_n[g] = s_act[g] ? P.label[g][rr] : -1;
  };
  const int64_t t_first = (int64_t)blockIdx.x * (KM_MT / 64) + (tid >> 6);
  if (t_first < ntile) load(t_first);
  for (int64_t t = t_first; t < ntile; t += nwv) {
    const int64_t r0 = t << 5;
    const bool in_r = r0 + i32 < n;
    const int64_t row = row_n;
    km_bf16x8 xh[KS], xl[KS];
    float xs = 0.f;
#pragma unroll
    for (int s_ = 0; s_ < KS; ++s_) {
      const float4 p0 = raw[2 * s_], p1 = raw[2 * s_ + 1];
      const float v[8] = {p0.x, p0.y, p0.z, p0.w, p1.x, p1.y, p1.z, p1.w};
#pragma unroll
      for (int j = 0; j < 8; ++j) xs += v[j] * v[j];
      uint4 hi, lo;
      km_split8(v, hi, lo);
      xh[s_] = __builtin_bit_cast(km_bf16x8, hi);
      xl[s_] = __builtin_bit_cast(km_bf16x8, lo);
    }
#pragma unroll
    for (int g = 0; g < G; ++g) s_lab[wv][g][l] = lab_n[g];
    if (t + nwv < ntile) load(t + nwv);
    xs += __shfl_xor(xs, 32);
    const float xn = sqrtf(xs);
#pragma unroll 1
    for (int g = 0; g < G; ++g) {
      if (!s_act[g]) continue;  // block-uniform
      const int32_t lab_cur = s_lab[wv][g][l];
      const uint4* Cg = Cf + g * NB * KS * 2 * 64;
      const float* cng = cnl + g * 64;
      km_f32x16 acc0 = {}, acc1 = {};
#pragma unroll
      for (int s_ = 0; s_ < KS; ++s_) {
        const km_bf16x8 ch0 = __builtin_bit_cast(km_bf16x8, Cg[((0 * KS + s_) * 2 + 0) * 64 + l]);
        const km_bf16x8 cl0 = __builtin_bit_cast(km_bf16x8, Cg[((0 * KS + s_) * 2 + 1) * 64 + l]);
        acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ch0, xh[s_], acc0, 0, 0, 0);
        acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ch0, xl[s_], acc0, 0, 0, 0);
        acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cl0, xh[s_], acc0, 0, 0, 0);
        if (NB == 2) {
          const km_bf16x8 ch1 = __builtin_bit_cast(km_bf16x8, Cg[((1 * KS + s_) * 2 + 0) * 64 + l]);
          const km_bf16x8 cl1 = __builtin_bit_cast(km_bf16x8, Cg[((1 * KS + s_) * 2 + 1) * 64 + l]);
          acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ch1, xh[s_], acc1, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ch1, xl[s_], acc1, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cl1, xh[s_], acc1, 0, 0, 0);
        }
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float4 n0 = *reinterpret_cast<const float4*>(cng + 8 * j + 4 * h);
        acc0[4 * j + 0] = n0.x - 2.f * acc0[4 * j + 0];
        acc0[4 * j + 1] = n0.y - 2.f * acc0[4 * j + 1];
        acc0[4 * j + 2] = n0.z - 2.f * acc0[4 * j + 2];
        acc0[4 * j + 3] = n0.w - 2.f * acc0[4 * j + 3];
        if (NB == 2) {
          const float4 n1 = *reinterpret_cast<const float4*>(cng + 32 + 8 * j + 4 * h);
          acc1[4 * j + 0] = n1.x - 2.f * acc1[4 * j + 0];
          acc1[4 * j + 1] = n1.y - 2.f * acc1[4 * j + 1];
          acc1[4 * j + 2] = n1.z - 2.f * acc1[4 * j + 2];
          acc1[4 * j + 3] = n1.w - 2.f * acc1[4 * j + 3];
        }
      }
      float m = INFINITY;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        m = fminf(m, acc0[r]);
        if (NB == 2) m = fminf(m, acc1[r]);
      }
      int mc = 64;
#pragma unroll
      for (int r = 15; r >= 0; --r) {
        if (NB == 2) mc = acc1[r] == m ? 32 + (r & 3) + 8 * (r >> 2) + 4 * h : mc;
      }
#pragma unroll
      for (int r = 15; r >= 0; --r) mc = acc0[r] == m ? (r & 3) + 8 * (r >> 2) + 4 * h : mc;
      {
        const float pm = __shfl_xor(m, 32);
        const int pc = __shfl_xor(mc, 32);
        if (pm < m || (pm == m && pc < mc)) { m = pm; mc = pc; }
      }
      float m2 = INFINITY;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int c0 = (r & 3) + 8 * (r >> 2) + 4 * h;
        m2 = fminf(m2, c0 == mc ? INFINITY : acc0[r]);
        if (NB == 2) m2 = fminf(m2, c0 + 32 == mc ? INFINITY : acc1[r]);
      }
      m2 = fminf(m2, __shfl_xor(m2, 32));
      const bool decided = m2 - m > KMS_SEP * xn * s_cmax[g];
      const uint32_t mi = (uint32_t)mc;
      const bool mine = h == 0 && in_r && decided;
      const bool mv = mine && lab_cur != (int32_t)mi;
      if (mv) P.label[g][row] = (int32_t)mi;
      // moves and near ties: one list reservation per wave each
      const uint64_t mm = __ballot(mv);
      if (mm) {
        unsigned long long b = 0;
        if (l == 0) {
          b = atomicAdd(P.n_moves[g], (unsigned long long)__popcll(mm));
          atomicAdd(&s_nchg[g], (uint32_t)__popcll(mm));
        }
        b = __shfl(b, 0);
        if (mv)
          P.moves[g][b + mbcnt(mm)] = make_uint2((uint32_t)row, (lab_cur < 0 ? 0xFFFFu : (uint32_t)lab_cur) | (mi << 16));
      }
      const bool tie = h == 0 && in_r && !decided;
      const uint64_t tm = __ballot(tie);
      if (tm) {
        unsigned long long b = 0;
        if (l == 0) b = atomicAdd(P.n_amb[g], (unsigned long long)__popcll(tm));
        b = __shfl(b, 0);
        if (tie) P.amb_rows[g][b + mbcnt(tm)] = (uint32_t)row;
      }
    }
  }
  __syncthreads();
  if (tid < G && s_nchg[tid]) atomicAdd(P.changed[tid], (unsigned long long)s_nchg[tid]);
}

// the move list of one run (k_km_assign_split_multi) into its fixed-point sums / counts: 32 moves per wave
// round through km_move_rows (the rows' vectors added to the new cluster and subtracted from the old one in
// the block's LDS sums, then one atomic per nonzero sum)
__global__ __launch_bounds__(KM_MT) void k_km_apply_moves(const float* __restrict__ X, int dim, int k,
                                                          const uint2* __restrict__ moves,
                                                          const unsigned long long* __restrict__ n_moves,
                                                          unsigned long long* __restrict__ sums,
                                                          unsigned long long* __restrict__ cnt, const int* __restrict__ gate) {
  if (gate && __builtin_amdgcn_readfirstlane(*gate)) return;
  const int64_t nm = (int64_t)*n_moves;
  if ((int64_t)blockIdx.x * 32 * (KM_MT / 64) >= nm) return;
  extern __shared__ unsigned long long smem64[];
  unsigned long long* ls = smem64;   // k * dim
  unsigned long long* lc = ls + k * dim;
  int32_t* labl = reinterpret_cast<int32_t*>(lc + k);  // [waves][3][32]
  const int tid = threadIdx.x, l = tid & 63, wv = tid >> 6;
  for (int i = tid; i < k * dim + k; i += KM_MT) ls[i] = 0ull;
  __syncthreads();
  const int64_t nwv = (int64_t)gridDim.x * (KM_MT / 64);
  for (int64_t b = ((int64_t)blockIdx.x * (KM_MT / 64) + wv) * 32; b < nm; b += nwv * 32) {
    const int64_t i = b + l;
    const bool f = l < 32 && i < nm;
    uint2 m = make_uint2(0u, 0u);
    if (f) m = moves[i];
    const uint32_t from = m.y & 0xFFFFu;
    km_move_rows(X, dim, ls, lc, labl + wv * 96, f, (int64_t)m.x, m.y >> 16, from == 0xFFFFu ? -1 : (int32_t)from);
  }
  __syncthreads();
  for (int i = tid; i < k * dim; i += KM_MT)
    if (ls[i]) atomicAdd(&sums[i], ls[i]);
  for (int i = tid; i < k; i += KM_MT)
    if (lc[i]) atomicAdd(&cnt[i], lc[i]);
}

// The near ties of a split pass with its move list (MV): one block per CU. Phase A folds the split pass's
// move regions (the f32 rows of the decided label changes, gathered 8 rows per lane group at a time)
// into the block's LDS sums; phase B scores the listed near-tie rows exactly as k_km_assign_mfma<LIST>
// (same f32 MFMA chain, same argmin and ties) with the next tile's row index, row pieces and label
// loaded while the current one is scored, and a changed row's vector added from the registers that
// hold it (lanes i and i + 32: dims 8q + 4h .. + 3) instead of a second read of the row. One flush of
// the block's sums; changed-row count and the near ties' inertia part once per block.
template <int NB, int NQ>
__global__ __launch_bounds__(KM_MT, 2) void k_km_ties(const float* __restrict__ X, int dim, int nq,
                                                      const float* __restrict__ C, const float* __restrict__ cn,
                                                      int k, int32_t* __restrict__ label,
                                                      unsigned long long* __restrict__ sums,
                                                      unsigned long long* __restrict__ cnt,
                                                      double* __restrict__ inertia,
                                                      unsigned long long* __restrict__ changed,
                                                      const int* __restrict__ gate,
                                                      const uint32_t* __restrict__ lrows,
                                                      const unsigned long long* __restrict__ lnrows,
                                                      const uint2* __restrict__ mv_list,
                                                      const uint32_t* __restrict__ mv_cnt, uint32_t mv_cap,
                                                      int n_regions) {
  if (gate && __builtin_amdgcn_readfirstlane(*gate)) return;
  extern __shared__ unsigned long long smem64[];
  float4* Bl = reinterpret_cast<float4*>(smem64);                              // [NB][nq][64]
  int32_t* labl = reinterpret_cast<int32_t*>(Bl + NB * nq * 64);                // [waves][3][32]
  float* cnl = reinterpret_cast<float*>(labl + (KM_MT / 64) * 96);             // [64]
  unsigned long long* ls = reinterpret_cast<unsigned long long*>(cnl + 64);    // k * dim sums, k counts
  unsigned long long* lc = ls + k * dim;
  __shared__ uint32_t s_chg;
  __shared__ double s_part;
  const int tid = threadIdx.x, l = tid & 63, wv = tid >> 6, h = l >> 5, i32 = l & 31;
  for (int e = tid; e < NB * nq * 64; e += KM_MT) {
    const int ll = e & 63, q = (e >> 6) % nq, b = (e >> 6) / nq;
    const int c = b * 32 + (ll & 31), d0 = 8 * q + 4 * (ll >> 5);
    float4 f = make_float4(0.f, 0.f, 0.f, 0.f);
    if (c < k && d0 < dim) f = *reinterpret_cast<const float4*>(C + (int64_t)c * dim + d0);
    Bl[e] = f;
  }
  if (tid < 64) cnl[tid] = cn[tid];
  for (int i = tid; i < k * dim + k; i += KM_MT) ls[i] = 0ull;
  if (tid == 0) { s_chg = 0; s_part = 0.0; }
  __syncthreads();
  // phase A: the split pass's label changes (their rows leave the old cluster, enter the new one)
  for (int r = blockIdx.x; r < n_regions; r += gridDim.x) {
    const int64_t nm = mv_cnt[r];
    const uint2* ml = mv_list + (size_t)r * mv_cap;
    for (int64_t b = (int64_t)wv * 32; b < nm; b += (KM_MT / 64) * 32) {
      const bool f = l < 32 && b + l < nm;
      uint2 m = make_uint2(0u, 0u);
      if (f) m = ml[b + l];
      const uint32_t from = m.y & 0xFFFFu;
      km_move_rows<16>(X, dim, ls, lc, labl + wv * 96, f, (int64_t)m.x, m.y >> 16, from == 0xFFFFu ? -1 : (int32_t)from);
    }
  }
  // phase B: the near ties
  double part = 0.0;
  uint32_t nchg = 0;
  const int64_t nl = (int64_t)__builtin_amdgcn_readfirstlane((int)*lnrows);
  const int64_t ntile = (nl + 31) >> 5;
  const int64_t nwv = (int64_t)gridDim.x * (KM_MT / 64);
  float4 an[NQ];
  int64_t row_n = 0;
  int32_t lab_n = -1;
  auto load = [&](int64_t tt) __attribute__((always_inline)) {
    const int64_t ri = (tt << 5) + i32 < nl ? (tt << 5) + i32 : nl - 1;
    const int64_t rr = (int64_t)lrows[ri];
    const float* x = X + rr * dim;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int d0 = 8 * q + 4 * h;
      an[q] = (q < nq && d0 < dim) ? *reinterpret_cast<const float4*>(x + d0) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    row_n = rr;
    lab_n = label[rr];
  };
  const int64_t t_first = (int64_t)blockIdx.x * (KM_MT / 64) + wv;
  if (t_first < ntile) load(t_first);
  for (int64_t t = t_first; t < ntile; t += nwv) {
    const bool in_l = (t << 5) + i32 < nl;
    const int64_t row = row_n;
    const int32_t lab_cur = lab_n;
    float4 a[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) a[q] = an[q];
    if (t + nwv < ntile) load(t + nwv);
    float xs = 0.f;
#pragma unroll
    for (int q = 0; q < NQ; ++q) xs += a[q].x * a[q].x + a[q].y * a[q].y + a[q].z * a[q].z + a[q].w * a[q].w;
    xs += __shfl_xor(xs, 32);
    km_f32x16 acc0 = {}, acc1 = {};
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      if (q < nq) {
        const float4 b0 = Bl[q * 64 + l];
        acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(b0.x, a[q].x, acc0, 0, 0, 0);
        acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(b0.y, a[q].y, acc0, 0, 0, 0);
        acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(b0.z, a[q].z, acc0, 0, 0, 0);
        acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(b0.w, a[q].w, acc0, 0, 0, 0);
        if (NB == 2) {
          const float4 b1 = Bl[(nq + q) * 64 + l];
          acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(b1.x, a[q].x, acc1, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(b1.y, a[q].y, acc1, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(b1.z, a[q].z, acc1, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(b1.w, a[q].w, acc1, 0, 0, 0);
        }
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float4 n0 = *reinterpret_cast<const float4*>(cnl + 8 * j + 4 * h);
      acc0[4 * j + 0] = n0.x - 2.f * acc0[4 * j + 0];
      acc0[4 * j + 1] = n0.y - 2.f * acc0[4 * j + 1];
      acc0[4 * j + 2] = n0.z - 2.f * acc0[4 * j + 2];
      acc0[4 * j + 3] = n0.w - 2.f * acc0[4 * j + 3];
      if (NB == 2) {
        const float4 n1 = *reinterpret_cast<const float4*>(cnl + 32 + 8 * j + 4 * h);
        acc1[4 * j + 0] = n1.x - 2.f * acc1[4 * j + 0];
        acc1[4 * j + 1] = n1.y - 2.f * acc1[4 * j + 1];
        acc1[4 * j + 2] = n1.z - 2.f * acc1[4 * j + 2];
        acc1[4 * j + 3] = n1.w - 2.f * acc1[4 * j + 3];
      }
    }
    float m = INFINITY;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      m = fminf(m, acc0[r]);
      if (NB == 2) m = fminf(m, acc1[r]);
    }
    int mc = 64;
#pragma unroll
    for (int r = 15; r >= 0; --r) {
      if (NB == 2) mc = acc1[r] == m ? 32 + (r & 3) + 8 * (r >> 2) + 4 * h : mc;
    }
#pragma unroll
    for (int r = 15; r >= 0; --r) mc = acc0[r] == m ? (r & 3) + 8 * (r >> 2) + 4 * h : mc;
    {
      const float pm = __shfl_xor(m, 32);
      const int pc = __shfl_xor(mc, 32);
      if (pm < m || (pm == m && pc < mc)) { m = pm; mc = pc; }
    }
    const int32_t mi = mc;
    const bool chg = in_l && lab_cur != mi;  // both lanes of the row agree (same row, label and argmin)
    if (h == 0 && in_l) {
      nchg += chg;
      if (chg) label[row] = mi;
      part += (double)fmaxf(xs + m, 0.f);
    }
    if (__ballot(chg)) {
      if (chg) {  // the row's dims held by this lane into the new cluster's sums, out of the old one's
        unsigned long long* rw = ls + mi * dim;
        unsigned long long* ow = ls + (lab_cur >= 0 ? lab_cur : 0) * dim;
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
          const float v4[4] = {a[q].x, a[q].y, a[q].z, a[q].w};
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int d = 8 * q + 4 * h + u;
            if (q < nq && d < dim) {
              const long long v = km_fx(v4[u]);
              atomicAdd(&rw[d], (unsigned long long)v);
              if (lab_cur >= 0) atomicAdd(&ow[d], (unsigned long long)(-v));
            }
          }
        }
        if (h == 0) {
          atomicAdd(&lc[mi], 1ull);
          if (lab_cur >= 0) atomicAdd(&lc[lab_cur], ~0ull);
        }
      }
    }
  }
  for (int o = 32; o >= 1; o >>= 1) {
    const uint64_t b = __double_as_longlong(part);
    const uint32_t lo = __shfl_xor((uint32_t)b, o), hi = __shfl_xor((uint32_t)(b >> 32), o);
    part += __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
  }
  const uint32_t w = wave_sum(nchg);
  if (l == 0) {
    if (w) atomicAdd(&s_chg, w);
    atomicAdd(&s_part, part);
  }
  __syncthreads();
  for (int i = tid; i < k * dim; i += KM_MT)
    if (ls[i]) atomicAdd(&sums[i], ls[i]);
  for (int i = tid; i < k; i += KM_MT)
    if (lc[i]) atomicAdd(&cnt[i], lc[i]);
  if (tid == 0) {
    if (s_chg) atomicAdd(changed, (unsigned long long)s_chg);
    atomicAdd(inertia, s_part);
  }
}

// inc: sums / cnt hold the exact sums / counts of the rows under `labels` (the previous labels) and
// are updated by the rows whose label changes (MFMA kernel); otherwise they are accumulated from
// scratch by every row (the caller zeroes them)
// the MFMA E-step's operand conditions (the VALU kernel takes every other shape)
static bool km_mfma_ok(int k, int dim, const float* X, const float* C) {
  static const bool km_valu = getenv("OTTOHIP_KM_VALU") != nullptr;  // A/B switch
  return !km_valu && k <= 64 && dim <= 8 * KM_NQ && (dim & 3) == 0 && ((uintptr_t)X & 15) == 0 &&
         ((uintptr_t)C & 15) == 0;
}

// distance bounds in the batched Lloyd steps (OTTOHIP_KM_BOUNDS=0 / OTTOHIP_KM_SPLIT=0: A/B switches, read per call)
static bool km_bounds_on(int64_t n) {
  const char* be = getenv("OTTOHIP_KM_BOUNDS");
  const char* se = getenv("OTTOHIP_KM_SPLIT");
  return n <= 0xFFFFFFFFll && !(be && !strcmp(be, "0")) && !(se && !strcmp(se, "0"));
}

// gate (MFMA kernel only): device flag, nonzero = skip (batched Lloyd steps after convergence)
static int launch_km_assign(Ctx* ctx, int k, hipStream_t s, const float* X, int64_t n, int dim, const float* C,
                            int32_t* labels, unsigned long long* sums, unsigned long long* cnt, double* inr,
                            unsigned long long* changed = nullptr, float* dist = nullptr, int inc = 0,
                            const int* gate = nullptr, bool split = false, int bounds = -1) {
  const int KP = (k + 7) / 8 * 8;
  float *Ct, *cn;
  OH_TRY(ctx->ws.get("km_ct", (size_t)KP * dim, &Ct));
  OH_TRY(ctx->ws.get("km_cn", (size_t)KM_MAXK, &cn));
  k_km_prep<<<grid_for(std::max<int64_t>((int64_t)KP * dim, KM_MAXK)), 256, 0, s>>>(C, k, dim, KP, Ct, cn);
  // the MFMA kernel measured 6.4 ms per Lloyd step at 12.9 M x 100, k = 50, against 5.1 ms for
  // the VALU kernel below (argmin butterflies and half the rows per wave): opt-in A/B switch only
  if (km_mfma_ok(k, dim, X, C)) {
    const int nq = (dim + 7) / 8, NB = k <= 32 ? 1 : 2;
    const size_t lds = (size_t)NB * nq * 64 * 16 + (KM_MT / 64) * 96 * 4 + 64 * 4 +
                       (sums ? ((size_t)k * dim + k) * 8 : 8);
    const int64_t ntile = ceil_div(n, 32);
    const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>(ceil_div(ntile, KM_MT / 64),
                                                                           (int64_t)ctx->n_cu * 2));
    // split: the split-precision pass decides (almost) every row, the exact kernel scores the near ties
    // (incremental sums, a changed-label count and no distances: the batched Lloyd steps)
    const char* se = getenv("OTTOHIP_KM_SPLIT");  // A/B switch, read per call
    split = split && inc && sums && changed && !dist && !(se && !strcmp(se, "0"));
    uint32_t* amb = nullptr;
    unsigned long long* n_amb = nullptr;
    bool h16 = false, mv = false;
    uint2* mv_list = nullptr;
    uint32_t* mv_cnt = nullptr;
    uint32_t mv_cap = 0;
    if (split) {
      OH_TRY(ctx->ws.get("km_amb", (size_t)std::max<int64_t>(n, 1), &amb));
      OH_TRY(ctx->ws.get("km_namb", 1, &n_amb));
      OH_HIP(hipMemsetAsync(n_amb, 0, 8, s));
      const int KS = dim <= 112 ? 7 : 8;
      // the half-precision rows of an attached X (OTTOHIP_KM_H16=0: the bf16 split of the f32 rows; read per call)
      const char* he = getenv("OTTOHIP_KM_H16");
      h16 = ctx->km_hX == X && ctx->km_hn == n && ctx->km_hdim == dim && !(he && !strcmp(he, "0"));
      const int smt = h16 ? KMH_MT : KM_MT;  // the split kernel's block size
      const size_t lds2 = (size_t)NB * KS * 2 * 64 * 16 + ((size_t)k * dim + k) * 8 + (smt / 64) * 96 * 4 + 64 * 4 +
                          (size_t)(h16 ? KMH_AMB : KMS_AMB) * 4;
      // bounds >= 0 (batched steps): skip the rows whose distance bounds keep their label; 1 = the
      // bounds are not valid for these rows (every row scored, bounds rebuilt)
      const bool bl = bounds >= 0 && km_bounds_on(n);
      // MV (H16 with bounds): label changes to per-block move lists, folded by k_km_ties (OTTOHIP_KM_MV=0: the
      // split pass's own LDS sums; A/B switch, read per call)
      const char* mve = getenv("OTTOHIP_KM_MV");
      mv = h16 && bl && !(mve && !strcmp(mve, "0"));
      const size_t lds2m = lds2 - (mv ? ((size_t)k * dim + k) * 8 : 0);
      auto sk = KS == 7 ? (NB == 1 ? k_km_assign_split<1, 7> : k_km_assign_split<2, 7>)
                        : (NB == 1 ? k_km_assign_split<1, 8> : k_km_assign_split<2, 8>);
      if (bl)
        sk = KS == 7 ? (NB == 1 ? k_km_assign_split<1, 7, true> : k_km_assign_split<2, 7, true>)
                     : (NB == 1 ? k_km_assign_split<1, 8, true> : k_km_assign_split<2, 8, true>);
      if (h16 && mv)
        sk = KS == 7 ? (NB == 1 ? k_km_assign_split<1, 7, true, true, true> : k_km_assign_split<2, 7, true, true, true>)
                     : (NB == 1 ? k_km_assign_split<1, 8, true, true, true> : k_km_assign_split<2, 8, true, true, true>);
      else if (h16)
        sk = bl ? (KS == 7 ? (NB == 1 ? k_km_assign_split<1, 7, true, true> : k_km_assign_split<2, 7, true, true>)
                           : (NB == 1 ? k_km_assign_split<1, 8, true, true> : k_km_assign_split<2, 8, true, true>))
                : (KS == 7 ? (NB == 1 ? k_km_assign_split<1, 7, false, true> : k_km_assign_split<2, 7, false, true>)
                           : (NB == 1 ? k_km_assign_split<1, 8, false, true> : k_km_assign_split<2, 8, false, true>));
      const uint4* x16 = h16 ? reinterpret_cast<const uint4*>(ctx->km_x16) : nullptr;
      const float* xn2 = h16 ? ctx->km_xn2 : nullptr;
      OH_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(sk), hipFuncAttributeMaxDynamicSharedMemorySize,
                                 (int)lds2m));
      // one resident block per CU (the kernel's registers allow one 8-wave block): one round of blocks,
      // so each block's LDS set-up and sum flush happen once
      const unsigned sgrid = (unsigned)std::max<int64_t>(1, std::min<int64_t>(ceil_div(ntile, smt / 64), ctx->n_cu));
      if (bl) {
        float *ub, *lb, *cp, *dl;
        uint32_t* erows;
        unsigned long long* n_eval;
        OH_TRY(ctx->ws.get("km_ub", (size_t)n, &ub));
        OH_TRY(ctx->ws.get("km_lb", (size_t)n, &lb));
        OH_TRY(ctx->ws.get("km_cp", (size_t)k * dim, &cp));
        OH_TRY(ctx->ws.get("km_dl", 68, &dl));
        OH_TRY(ctx->ws.get("km_erows", (size_t)n, &erows));
        OH_TRY(ctx->ws.get("km_neval", 1, &n_eval));
        k_km_delta<<<1, KMD_T, 0, s>>>(C, cp, cn, k, dim, bounds, dl, gate, n_eval);
        const unsigned fgrid = (unsigned)std::max<int64_t>(1, ceil_div(n, KMF_PER * 256));
        k_km_filter<<<fgrid, 256, 0, s>>>(n, k, labels, ub, lb, dl, erows, n_eval, gate);
        static const bool bdbg = getenv("OTTOHIP_KM_BDBG") != nullptr;  // rows scored per step (debugging aid)
        if (bdbg) {
          unsigned long long ne = 0;
          float dh[68];
          OH_TRY(d2h(&ne, n_eval, 1, s));
          OH_TRY(d2h(dh, dl, 68, s));
          std::vector<float> ds(dh, dh + k);
          std::sort(ds.begin(), ds.end());
          fprintf(stderr, "[ottohip] kmeans bounds: %llu of %lld rows scored (force %d, delta max %.4g / %.4g, "
                  "median %.4g, p10 %.4g, cmax %.4g)\n", ne, (long long)n, bounds, dh[64], dh[65], ds[k / 2],
                  ds[k / 10], dh[67]);
        }
        if (mv) {  // a block's region holds every row it can score: its tiles' share of ceil(n / 32)
          const int64_t wpb = smt / 64, nwv = (int64_t)ctx->n_cu * wpb;
          mv_cap = (uint32_t)(ceil_div(ceil_div(n, 32), nwv) * wpb * 32);
          OH_TRY(ctx->ws.get("km_mv", (size_t)ctx->n_cu * mv_cap, &mv_list));
          OH_TRY(ctx->ws.get("km_mvc", (size_t)ctx->n_cu, &mv_cnt));
        }
        const char* s16e = getenv("OTTOHIP_KM_S16");  // A/B switch, read per call
        if (mv && !(s16e && !strcmp(s16e, "0"))) {
          auto s16 = KS == 7 ? (NB == 1 ? k_km_split16<1, 7> : k_km_split16<2, 7>)
                             : (NB == 1 ? k_km_split16<1, 8> : k_km_split16<2, 8>);
          const size_t lds16 = (size_t)NB * KS * 2 * 64 * 16 + 64 * 4 + (size_t)KMH_AMB * 4;
          OH_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(s16), hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)lds16));
          s16<<<(unsigned)ctx->n_cu, KMH_MT, lds16, s>>>(n, dim, C, cn, k, labels, changed, gate, amb, n_amb, erows,
                                                         n_eval, ub, lb, x16, reinterpret_cast<const float2*>(xn2),
                                                         mv_list, mv_cnt, mv_cap);
        } else {
          sk<<<(unsigned)ctx->n_cu, smt, lds2m, s>>>(X, n, dim, C, cn, k, labels, sums, cnt, changed, gate, amb, n_amb,
                                                     erows, n_eval, ub, lb, x16, xn2, mv_list, mv_cnt, mv_cap);
        }
      } else {
        sk<<<sgrid, smt, lds2, s>>>(X, n, dim, C, cn, k, labels, sums, cnt, changed, gate, amb, n_amb, nullptr, nullptr,
                                     nullptr, nullptr, x16, xn2, nullptr, nullptr, 0);
      }
      OH_HIP(hipGetLastError());
    }
    auto kern = nq == 13 ? (NB == 1 ? k_km_assign_mfma<1, 13> : k_km_assign_mfma<2, 13>)
                         : (NB == 1 ? k_km_assign_mfma<1, KM_NQ> : k_km_assign_mfma<2, KM_NQ>);
    if (split)
      kern = nq == 13 ? (NB == 1 ? k_km_assign_mfma<1, 13, true> : k_km_assign_mfma<2, 13, true>)
                      : (NB == 1 ? k_km_assign_mfma<1, KM_NQ, true> : k_km_assign_mfma<2, KM_NQ, true>);
    OH_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)lds));
    // near ties only: about 1-2 % of the rows (bf16 split: half a block per CU) or ~5 % (H16: one block per CU,
    // C2 1.143 s against 1.168 s at two and 1.245 s at half a block per CU); OTTOHIP_KM_EGRID = blocks (A/B)
    const char* ege = getenv("OTTOHIP_KM_EGRID");
    const int eg_env = ege ? atoi(ege) : 0;
    const unsigned egrid = split ? (unsigned)std::max(1, eg_env > 0 ? eg_env : (h16 ? ctx->n_cu : ctx->n_cu / 2)) : grid;
    if (mv) {
      auto tk = nq == 13 ? (NB == 1 ? k_km_ties<1, 13> : k_km_ties<2, 13>)
                         : (NB == 1 ? k_km_ties<1, KM_NQ> : k_km_ties<2, KM_NQ>);
      OH_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(tk), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
      tk<<<egrid, KM_MT, lds, s>>>(X, dim, nq, C, cn, k, labels, sums, cnt, inr, changed, gate, amb, n_amb, mv_list,
                                   mv_cnt, mv_cap, ctx->n_cu);
      OH_HIP(hipGetLastError());
      static const bool bdbg = getenv("OTTOHIP_KM_BDBG") != nullptr;  // near ties and split-pass moves per step
      if (bdbg) {
        unsigned long long na = 0;
        std::vector<uint32_t> mc(ctx->n_cu);
        OH_TRY(d2h(&na, n_amb, 1, s));
        OH_TRY(d2h(mc.data(), mv_cnt, (size_t)ctx->n_cu, s));
        uint64_t nm = 0, mx = 0;
        for (uint32_t v : mc) { nm += v; mx = std::max<uint64_t>(mx, v); }
        fprintf(stderr, "[ottohip] kmeans step: %llu near ties, %llu split-pass moves (max %llu per block)\n", na,
                (unsigned long long)nm, (unsigned long long)mx);
      }
      return 0;
    }
    kern<<<egrid, KM_MT, lds, s>>>(X, n, dim, nq, C, cn, k, labels, sums, cnt, inr, changed, dist, inc, gate,
                                   amb, n_amb);
    OH_HIP(hipGetLastError());
    return 0;
  }
  if (gate) { set_error("kmeans: batched steps need the MFMA E-step"); return OTTOHIP_EINVAL; }
  if (inc && sums) {  // the VALU kernel accumulates from scratch
    OH_HIP(hipMemsetAsync(sums, 0, (size_t)k * dim * 8, s));
    OH_HIP(hipMemsetAsync(cnt, 0, (size_t)k * 8, s));
  }
  const size_t lds = sums ? ((size_t)k * dim + k) * 8 : 8;
  const unsigned grid = (unsigned)std::min<int64_t>(ceil_div(n, 256), (int64_t)ctx->n_cu * 4);
  switch (KP / 8) {
#define KM_CASE(q) case q: k_km_assign<8 * q><<<grid, 256, lds, s>>>(X, n, dim, Ct, cn, k, labels, sums, cnt, inr, changed, dist); break;
    KM_CASE(1) KM_CASE(2) KM_CASE(3) KM_CASE(4) KM_CASE(5) KM_CASE(6) KM_CASE(7) KM_CASE(8)
#undef KM_CASE
    default: break;
  }
  OH_HIP(hipGetLastError());
  return 0;
}

// squared distance of every row to the centroid of its label (inertia of a given labelling,
// and the per-row distances sklearn's empty-cluster relocation ranks)
// inertia: one f64 atomic per wave (order-dependent last bits); wparts: the per-wave partials instead (k_sum_fixed)
__global__ __launch_bounds__(256) void k_km_labelled(const float* __restrict__ X, int64_t n, int dim,
                                                     const float* __restrict__ C, const int32_t* __restrict__ label,
                                                     float* __restrict__ dist, double* __restrict__ inertia,
                                                     double* __restrict__ wparts = nullptr) {
  // half a wave per row: lanes over the row's dims (coalesced), sum by a 32-lane butterfly
  double part = 0.0;
  const int hl = threadIdx.x & 31;
  const int64_t nhalf = ((int64_t)gridDim.x * blockDim.x) >> 5;
  for (int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 5; i < n; i += nhalf) {
    const float* x = X + i * dim;
    const float* c = C + (int64_t)label[i] * dim;
    float acc = 0.f;
    for (int d = hl; d < dim; d += 32) {
      const float t = x[d] - c[d];
      acc = fmaf(t, t, acc);
    }
#pragma unroll
    for (int o = 16; o >= 1; o >>= 1) acc += __shfl_xor(acc, o);
    if (hl == 0) {
      if (dist) dist[i] = acc;
      part += (double)acc;
    }
  }
  for (int o = 32; o >= 1; o >>= 1) {
    const uint64_t b = __double_as_longlong(part);
    const uint32_t lo = __shfl_xor((uint32_t)b, o), hi = __shfl_xor((uint32_t)(b >> 32), o);
    part += __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
  }
  if ((threadIdx.x & 63) == 0 && inertia) atomicAdd(inertia, part);
  if ((threadIdx.x & 63) == 0 && wparts) wparts[((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6] = part;
}
// sum of the per-wave partials in a fixed order (one block): the same rows and centres give the same bits, so
// two n_init runs that reach one partition (their labels a permutation) tie exactly, and the first is kept
__global__ __launch_bounds__(1024) void k_sum_fixed(const double* __restrict__ parts, int64_t n, double* __restrict__ out) {
  __shared__ double sh[1024];
  double a = 0.0;
  for (int64_t i = threadIdx.x; i < n; i += 1024) a += parts[i];
  sh[threadIdx.x] = a;
  __syncthreads();
  for (int w = 512; w >= 1; w >>= 1) {
    if ((int)threadIdx.x < w) sh[threadIdx.x] += sh[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) *out = sh[0];
}

// argmax of dist over rows not yet taken: key = ordered(dist) << 32 | ~row (ties: lowest row)
__global__ __launch_bounds__(256) void k_km_argmax(const float* __restrict__ dist, int64_t n,
                                                   const int64_t* __restrict__ taken, int n_taken,
                                                   unsigned long long* __restrict__ best) {
  unsigned long long b = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    bool t = false;
    for (int j = 0; j < n_taken; ++j) t |= taken[j] == i;
    if (t) continue;
    const unsigned long long key = ((unsigned long long)km_ord(dist[i]) << 32) | (uint32_t)(~(uint32_t)i);
    b = key > b ? key : b;
  }
  for (int o = 32; o >= 1; o >>= 1) {
    const unsigned long long v = shfl64(b, (int)(lane_id() ^ o));
    b = v > b ? v : b;
  }
  if (lane_id() == 0 && b) atomicMax(best, b);
}

// sklearn _relocate_empty_clusters_dense on the fixed-point sums: the vector moves from its old
// cluster's sums to the empty cluster's
__global__ void k_km_relocate(unsigned long long* __restrict__ sums, unsigned long long* __restrict__ cnt, int dim,
                              const float* __restrict__ vecs, const int32_t* __restrict__ moves, int m) {
  const int d = blockIdx.x * blockDim.x + threadIdx.x;
  for (int j = 0; j < m; ++j) {  // sequential over moves (an old cluster may lose several)
    const int oc = moves[2 * j], nc = moves[2 * j + 1];
    if (d < dim) {
      const unsigned long long v = (unsigned long long)__float2ll_rn(vecs[(int64_t)j * dim + d] * 16777216.0f);
      sums[(int64_t)oc * dim + d] -= v;
      sums[(int64_t)nc * dim + d] = v;
    }
    if (d == 0) { cnt[oc] -= 1ull; cnt[nc] = 1ull; }
  }
}

// M-step on the device (one block): centroids = sums / counts for non-empty clusters, squared
// centre shift reduced in a fixed order (deterministic), number of empty clusters. With
// commit_if_full, a step that finds an empty cluster leaves the centroids untouched: the host
// relocates (sklearn's order: relocation before the update) and calls the update again.
// st: [0] shift^2 (double), [1] empty clusters (u64)
constexpr int KM_UT = 256;
// ctl (batched Lloyd steps, else nullptr): [0] stop reason (0 running, 1 no label changed, 2 shift^2 <=
// tol, 3 empty cluster: centroids untouched, the host relocates), [1] steps run; a step after a
// stop does nothing (its E-step was skipped too)
__global__ __launch_bounds__(KM_UT) void k_km_update(float* __restrict__ C, const long long* __restrict__ sums,
                                                     const long long* __restrict__ cnt, int k, int dim,
                                                     int commit_if_full, double* __restrict__ st,
                                                     int* __restrict__ ctl = nullptr,
                                                     const unsigned long long* __restrict__ changed = nullptr,
                                                     double tol = 0.0) {
  __shared__ double red[KM_UT];
  __shared__ int n_empty;
  const int tid = threadIdx.x;
  if (ctl && __builtin_amdgcn_readfirstlane(ctl[0])) return;
  if (tid == 0) n_empty = 0;
  __syncthreads();
  for (int c = tid; c < k; c += KM_UT)
    if (cnt[c] <= 0) atomicAdd(&n_empty, 1);
  __syncthreads();
  const int ne = n_empty;
  const bool commit = !(commit_if_full && ne > 0);
  double sh = 0.0;
  if (commit)
    for (int i = tid; i < k * dim; i += KM_UT) {
      const int c = i / dim;
      if (cnt[c] <= 0) continue;
      const float nv = (float)((double)sums[i] / KM_FX / (double)cnt[c]);
      const double df = (double)nv - (double)C[i];
      sh += df * df;
      C[i] = nv;
    }
  red[tid] = sh;
  __syncthreads();
  for (int o = KM_UT / 2; o >= 1; o >>= 1) {
    if (tid < o) red[tid] += red[tid + o];
    __syncthreads();
  }
  if (tid == 0) {
    st[0] = commit ? red[0] : -1.0;
    reinterpret_cast<unsigned long long*>(st)[1] = (unsigned long long)ne;
    if (ctl) {  // sklearn 1.2 _kmeans_single_lloyd's checks after each step
      ctl[1] += 1;
      ctl[0] = !commit ? 3 : (*changed == 0 ? 1 : (red[0] <= tol ? 2 : 0));
    }
  }
}

__global__ void k_km_gate_reset(const int* __restrict__ ctl, double* __restrict__ st) {
  if (threadIdx.x < 4 && !ctl[0]) st[threadIdx.x] = 0.0;
}

// per column: sum of x and of (x - center)^2 in 2^-24 fixed point (exact, order-independent);
// threads over columns, blocks over row chunks
__global__ __launch_bounds__(128) void k_col_sums(const float* __restrict__ X, int64_t n, int dim,
                                                  const float* __restrict__ center, unsigned long long* __restrict__ s1,
                                                  unsigned long long* __restrict__ s2) {
  const int d = threadIdx.x;
  if (d >= dim) return;
  const float c = center ? center[d] : 0.f;
  long long a = 0, b = 0;
  for (int64_t i = blockIdx.x; i < n; i += gridDim.x) {
    const float x = X[i * dim + d];
    const float t = x - c;
    a += __float2ll_rn(x * 16777216.0f);
    b += __float2ll_rn(t * t * 16777216.0f);
  }
  atomicAdd(&s1[d], (unsigned long long)a);
  atomicAdd(&s2[d], (unsigned long long)b);
}

__global__ void k_center_rows(const float* __restrict__ X, int64_t n, int dim, const float* __restrict__ mean,
                              float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n * dim) out[i] = X[i] - mean[i % dim];
}

// ---------------------------------------------------------------- C3
// counters: [6][n_clusters * n_items] u32: n_clicks, n_carts, n_orders, *_7d
__global__ void k_pop_count(const int64_t* __restrict__ off, int64_t S, const int32_t* __restrict__ aid,
                            const int32_t* __restrict__ ts, const int8_t* __restrict__ type,
                            const int32_t* __restrict__ session_cl, int32_t n_items, int32_t n_clusters,
                            int32_t ts_7d, uint32_t* __restrict__ cnt, uint32_t* __restrict__ present,
                            int* __restrict__ err) {
  const int64_t s = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (s >= S) return;
  const int c = session_cl[s];
  if (c < 0 || c >= n_clusters) { if ((threadIdx.x & 63) == 0) atomicOr(err, 1); return; }
  const int64_t NS = (int64_t)n_clusters * n_items;
  for (int64_t e = off[s] + (threadIdx.x & 63); e < off[s + 1]; e += 64) {
    const int32_t a = aid[e];
    const int y = type[e];
    if (a < 0 || a >= n_items || y < 0 || y > 2) { atomicOr(err, 2); continue; }
    const int64_t slot = (int64_t)c * n_items + a;
    atomicAdd(&cnt[y * NS + slot], 1u);
    if (ts[e] > ts_7d) atomicAdd(&cnt[(3 + y) * NS + slot], 1u);
    present[slot] = 1u;
  }
}

__global__ void k_pop_present(const uint32_t* __restrict__ cnt, int64_t NS, uint32_t* __restrict__ present) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < NS) present[i] = (cnt[i] | cnt[NS + i] | cnt[2 * NS + i]) != 0u;
}

__global__ void k_pop_pairs(const uint32_t* __restrict__ present, const uint64_t* __restrict__ idx, int64_t NS,
                            uint32_t* __restrict__ pair_slot) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < NS && present[i]) pair_slot[idx[i]] = (uint32_t)i;
}

// LSD keys for one counter: aid asc, then count desc, then cluster asc (stable)
__global__ void k_pop_key(const uint32_t* __restrict__ pair_slot, const uint32_t* __restrict__ val, int64_t n,
                          const uint32_t* __restrict__ cnt, int32_t n_items, int which, uint32_t* __restrict__ key) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t slot = pair_slot[val ? val[i] : i];
  if (which == 0) key[i] = slot % (uint32_t)n_items;       // aid
  else if (which == 1) key[i] = ~cnt[slot];                // count desc
  else key[i] = slot / (uint32_t)n_items;                  // cluster
}

__global__ void k_pop_iota(uint32_t* __restrict__ v, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) v[i] = (uint32_t)i;
}

__global__ void k_pop_rank(const uint32_t* __restrict__ pair_slot, const uint32_t* __restrict__ val, int64_t n,
                           int32_t n_items, const uint64_t* __restrict__ cl_first, uint16_t* __restrict__ rank) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t p = val[i];
  const uint32_t c = pair_slot[p] / (uint32_t)n_items;
  const int64_t r = i - (int64_t)cl_first[c] + 1;
  rank[p] = (uint16_t)(r > 999 ? 999 : r);
}

// pairs are in slot = (cluster, aid) order: the first pair of each cluster from the boundaries
// (a histogram here would be a few same-address atomics per pair)
__global__ void k_pop_cluster_first(const uint32_t* __restrict__ pair_slot, int64_t n, int32_t n_items,
                                    int32_t n_clusters, uint64_t* __restrict__ cl_first) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i > n) return;
  const int64_t prev = i == 0 ? -1 : (int64_t)(pair_slot[i - 1] / (uint32_t)n_items);
  const int64_t cur = i == n ? (int64_t)n_clusters : (int64_t)(pair_slot[i] / (uint32_t)n_items);
  for (int64_t c = prev + 1; c <= cur; ++c) cl_first[c] = (uint64_t)i;
}

__global__ void k_pop_keep(const uint16_t* __restrict__ rank, int64_t n, int keep_top_k, uint32_t* __restrict__ keep) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  int m = 999;
#pragma unroll
  for (int t = 0; t < 6; ++t) m = min(m, (int)rank[t * n + i]);
  keep[i] = m <= keep_top_k ? 1u : 0u;
}

__global__ void k_pop_out(const uint32_t* __restrict__ pair_slot, const uint16_t* __restrict__ rank,
                          const uint32_t* __restrict__ keep, const uint64_t* __restrict__ oidx, int64_t n,
                          int32_t n_items, int32_t* __restrict__ o_aid, int32_t* __restrict__ o_cl,
                          int16_t* __restrict__ o_rank) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || !keep[i]) return;
  const uint64_t o = oidx[i];
  o_aid[o] = (int32_t)(pair_slot[i] % (uint32_t)n_items);
  o_cl[o] = (int32_t)(pair_slot[i] / (uint32_t)n_items);
#pragma unroll
  for (int t = 0; t < 6; ++t) o_rank[o * 6 + t] = (int16_t)rank[t * n + i];
}

// ---------------------------------------------------------------- R7
__global__ __launch_bounds__(256) void k_sim(const int64_t* __restrict__ cand_off, int64_t S,
                                             const int32_t* __restrict__ cnext, const float* __restrict__ sess_emb,
                                             const uint8_t* __restrict__ sess_has, const int32_t* __restrict__ row_of_aid,
                                             int32_t n_aid_map, const float* __restrict__ emb, int dim,
                                             float* __restrict__ cos_out, float* __restrict__ eucl_out) {
  const int64_t s = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (s >= S) return;
  const int l = threadIdx.x & 63;
  const float* q = sess_emb + s * dim;
  const bool hs = sess_has == nullptr || sess_has[s];
  for (int64_t i = cand_off[s] + l; i < cand_off[s + 1]; i += 64) {
    const int32_t a = cnext[i];
    const int32_t r = (a >= 0 && a < n_aid_map) ? row_of_aid[a] : -1;
    if (!hs || r < 0) { cos_out[i] = 0.f; eucl_out[i] = -1.f; continue; }  // inner joins miss: fill 0 / -1
    const float* v = emb + (int64_t)r * dim;
    float dot = 0.f, nq = 0.f, nv = 0.f, d2 = 0.f;
    for (int d = 0; d < dim; ++d) {
      const float x = q[d], y = v[d];
      dot += x * y; nq += x * x; nv += y * y;
      const float z = x - y;
      d2 += z * z;
    }
    cos_out[i] = dot / (sqrtf(nq) * sqrtf(nv));
    eucl_out[i] = sqrtf(d2);
  }
}

// R7, coalesced: 16 lanes per candidate, each lane holding 4 + 4 of the session's (<= 128, dim % 4 == 0)
// dimensions and reading the item row as two float4 (one 400-B row = 25 float4 in one load instruction per
// group), 4 candidates per wave per round, two rounds in flight; dot / |v|^2 / |q - v|^2 by 4 xor-shuffle
// steps. k_sim above (one lane per candidate, dimension by dimension) read each row 4 B at a time, 64 rows
// per load instruction.
constexpr int SIM_U = 2;  // rounds of 4 candidates in flight per wave
__global__ __launch_bounds__(256) void k_sim16(const int64_t* __restrict__ cand_off, int64_t S,
                                               const int32_t* __restrict__ cnext, const float* __restrict__ sess_emb,
                                               const uint8_t* __restrict__ sess_has, const int32_t* __restrict__ row_of_aid,
                                               int32_t n_aid_map, const float* __restrict__ emb, int dim,
                                               float* __restrict__ cos_out, float* __restrict__ eucl_out) {
  const int l = threadIdx.x & 63, g = l >> 4, j = l & 15;
  const int64_t nw = (int64_t)gridDim.x * (blockDim.x >> 6);
  const int d0 = 4 * j, d1 = 64 + 4 * j;
  const bool h0 = d0 < dim, h1 = d1 < dim;
  for (int64_t s = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); s < S; s += nw) {
    const float* q = sess_emb + s * dim;
    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
    const float4 q0 = h0 ? *reinterpret_cast<const float4*>(q + d0) : z4;
    const float4 q1 = h1 ? *reinterpret_cast<const float4*>(q + d1) : z4;
    float nq = q0.x * q0.x + q0.y * q0.y + q0.z * q0.z + q0.w * q0.w + q1.x * q1.x + q1.y * q1.y + q1.z * q1.z +
               q1.w * q1.w;
#pragma unroll
    for (int m = 1; m < 16; m <<= 1) nq += __shfl_xor(nq, m);
    const float sq = sqrtf(nq);
    const bool hs = sess_has == nullptr || sess_has[s];
    const int64_t b = cand_off[s], e = cand_off[s + 1];
    for (int64_t i0 = b; i0 < e; i0 += 4 * SIM_U) {
      int32_t r[SIM_U];
      float4 v0[SIM_U], v1[SIM_U];
#pragma unroll
      for (int u = 0; u < SIM_U; ++u) {
        const int64_t i = i0 + 4 * u + g;
        const int32_t a = i < e ? cnext[i] : -1;
        r[u] = (hs && a >= 0 && a < n_aid_map) ? row_of_aid[a] : -1;
        const float* v = emb + (int64_t)(r[u] < 0 ? 0 : r[u]) * dim;
        v0[u] = (r[u] >= 0 && h0) ? *reinterpret_cast<const float4*>(v + d0) : z4;
        v1[u] = (r[u] >= 0 && h1) ? *reinterpret_cast<const float4*>(v + d1) : z4;
      }
#pragma unroll
      for (int u = 0; u < SIM_U; ++u) {
        const float4 a0 = v0[u], a1 = v1[u];
        float dot = q0.x * a0.x + q0.y * a0.y + q0.z * a0.z + q0.w * a0.w + q1.x * a1.x + q1.y * a1.y + q1.z * a1.z +
                    q1.w * a1.w;
        float nv = a0.x * a0.x + a0.y * a0.y + a0.z * a0.z + a0.w * a0.w + a1.x * a1.x + a1.y * a1.y + a1.z * a1.z +
                   a1.w * a1.w;
        float x, d2 = 0.f;
        x = q0.x - a0.x; d2 += x * x; x = q0.y - a0.y; d2 += x * x; x = q0.z - a0.z; d2 += x * x; x = q0.w - a0.w; d2 += x * x;
        x = q1.x - a1.x; d2 += x * x; x = q1.y - a1.y; d2 += x * x; x = q1.z - a1.z; d2 += x * x; x = q1.w - a1.w; d2 += x * x;
#pragma unroll
        for (int m = 1; m < 16; m <<= 1) {
          dot += __shfl_xor(dot, m);
          nv += __shfl_xor(nv, m);
          d2 += __shfl_xor(d2, m);
        }
        const int64_t i = i0 + 4 * u + g;
        if (j == 0 && i < e) {
          const bool hit = r[u] >= 0;  // inner joins miss: 0 / -1
          cos_out[i] = hit ? dot / (sq * sqrtf(nv)) : 0.f;
          eucl_out[i] = hit ? sqrtf(d2) : -1.f;
        }
      }
    }
  }
}


// ---------------------------------------------------------------- KMeans init seeds (host)
// sklearn 1.2 KMeans(init='random') draws the initial centres of run r as
// RandomState(random_state).permutation(n)[:k], the runs drawing successively from one stream
// (model/kmeans_sessions.py:152-159 -> sklearn _init_centroids). numpy's legacy permutation is
// arange(n) shuffled by Fisher-Yates from the top, j = random_interval(i) (mask-and-reject over
// 32-bit MT19937 outputs). Only the first k positions are needed: the draws are stored, then the
// swaps are replayed backwards from position p < k, so each of the k values is traced to its
// origin with a bitmap of the traced positions instead of a random-access pass over n values.
struct RsState {
  uint32_t key[624];
  int pos = 624;
  std::vector<uint32_t> J;
  std::vector<uint64_t> bits;
};
static void rs_seed(RsState& r, uint32_t seed) {
  for (int p = 0; p < 624; ++p) {
    r.key[p] = seed;
    seed = 1812433253u * (seed ^ (seed >> 30)) + (uint32_t)p + 1u;
  }
  r.pos = 624;
}
static void rs_gen(RsState& r) {
  constexpr int N = 624, M = 397;
  constexpr uint32_t A = 0x9908b0dfu, U = 0x80000000u, L = 0x7fffffffu;
  uint32_t* k = r.key;
  int i = 0;
  for (; i < N - M; ++i) {
    const uint32_t y = (k[i] & U) | (k[i + 1] & L);
    k[i] = k[i + M] ^ (y >> 1) ^ ((0u - (y & 1u)) & A);
  }
  for (; i < N - 1; ++i) {
    const uint32_t y = (k[i] & U) | (k[i + 1] & L);
    k[i] = k[i + (M - N)] ^ (y >> 1) ^ ((0u - (y & 1u)) & A);
  }
  const uint32_t y = (k[N - 1] & U) | (k[0] & L);
  k[N - 1] = k[M - 1] ^ (y >> 1) ^ ((0u - (y & 1u)) & A);
  r.pos = 0;
}
static inline uint32_t rs_next32(RsState& r) {
  if (r.pos == 624) rs_gen(r);
  uint32_t y = r.key[r.pos++];
  y ^= y >> 11;
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= y >> 18;
  return y;
}
static inline uint32_t rs_interval(RsState& r, uint32_t mx) {  // numpy random_interval, max < 2^32
  if (mx == 0) return 0;
  uint32_t mask = mx;
  mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4; mask |= mask >> 8; mask |= mask >> 16;
  uint32_t v;
  while ((v = (rs_next32(r) & mask)) > mx) {}
  return v;
}
}  // namespace ottohip

struct ottohip_rs : public ottohip::RsState {};

namespace ottohip {
}  // namespace ottohip

using namespace ottohip;

extern "C" {

int ottohip_session_embeddings(ottohip_ctx* ctx, const int64_t* session_offsets, int64_t n_sessions,
                               const int32_t* aid, const int32_t* ts, const int8_t* type, const int32_t* row_of_aid,
                               int32_t n_aid_map, const float* emb, int dim, float* out, void* stream) {
  if (!ctx || n_sessions < 0 || dim < 1 || dim > EMB_MAXD || (n_sessions > 0 && (!session_offsets || !aid || !ts ||
      !type || !row_of_aid || !emb || !out))) {
    set_error("session_embeddings: bad arguments (dim <= %d)", EMB_MAXD); return OTTOHIP_EINVAL;
  }
  if (n_sessions == 0) return 0;
  hipStream_t s = S(stream);
  OH_HIP(hipSetDevice(ctx->device));
  int ph = ctx->begin("sess_emb", s, 0);
  k_sess_emb<<<(unsigned)n_sessions, 64, 0, s>>>(session_offsets, n_sessions, aid, ts, type, row_of_aid, n_aid_map,
                                                emb, dim, out);
  OH_HIP(hipGetLastError());
  ctx->end(ph, s);
  return 0;
}

// One Lloyd iteration: labels, new centroids (empty clusters keep theirs), center shift^2, inertia.
int ottohip_kmeans_step(ottohip_ctx* ctx, const float* X, int64_t n, int dim, float* centroids, int k,
                        int32_t* labels, double* shift2, double* inertia, void* stream) {
  if (!ctx || !X || !centroids || !labels || n < 1 || dim < 1 || dim > EMB_MAXD || k < 1 || k > KM_MAXK) {
    set_error("kmeans_step: bad arguments (k <= %d, dim <= %d)", KM_MAXK, EMB_MAXD); return OTTOHIP_EINVAL;
  }
  if (((size_t)k * dim + k) * 8 > 65536) {
    set_error("kmeans_step: k * dim too large for LDS"); return OTTOHIP_ELIMIT;
  }
  hipStream_t s = S(stream);
  ctx->km_bvalid = false;  // labels written outside the batched steps: their distance bounds are stale
  OH_HIP(hipSetDevice(ctx->device));
  unsigned long long* sums;
  unsigned long long* cnt;
  double* inr;
  OH_TRY(ctx->ws.get("km_sums", (size_t)k * dim, &sums));
  OH_TRY(ctx->ws.get("km_cnt", (size_t)k, &cnt));
  OH_TRY(ctx->ws.get("km_inertia", 1, &inr));
  OH_HIP(hipMemsetAsync(sums, 0, (size_t)k * dim * 8, s));
  OH_HIP(hipMemsetAsync(cnt, 0, (size_t)k * 8, s));
  OH_HIP(hipMemsetAsync(inr, 0, 8, s));
  OH_TRY(launch_km_assign(ctx, k, s, X, n, dim, centroids, labels, sums, cnt, inr));
  std::vector<unsigned long long> hs((size_t)k * dim);
  std::vector<unsigned long long> hc(k);
  std::vector<float> hcen((size_t)k * dim);
  OH_TRY(d2h(hs.data(), sums, hs.size(), s));
  OH_TRY(d2h(hc.data(), cnt, hc.size(), s));
  OH_TRY(d2h(hcen.data(), centroids, hcen.size(), s));
  double inertia_h = 0.0;
  OH_TRY(d2h(&inertia_h, inr, 1, s));
  double sh = 0.0;
  for (int c = 0; c < k; ++c) {
    if (hc[c] == 0) continue;
    for (int d = 0; d < dim; ++d) {
      const float nv = (float)((double)(long long)hs[(size_t)c * dim + d] / KM_FX / (double)hc[c]);
      const double df = (double)nv - (double)hcen[(size_t)c * dim + d];
      sh += df * df;
      hcen[(size_t)c * dim + d] = nv;
    }
  }
  OH_HIP(hipMemcpyAsync(centroids, hcen.data(), hcen.size() * sizeof(float), hipMemcpyHostToDevice, s));
  OH_HIP(hipStreamSynchronize(s));
  if (shift2) *shift2 = sh;
  if (inertia) *inertia = inertia_h;
  return 0;
}

// E-step + partial M-step of one Lloyd iteration on this rank's rows (the
// sums are all-reduced by the host layer between this and ottohip_kmeans_update)
int ottohip_kmeans_partial(ottohip_ctx* ctx, const float* X, int64_t n, int dim, const float* centroids, int k,
                           int32_t* labels, int64_t* sums, int64_t* counts, double* inertia, int64_t* n_changed,
                           void* stream) {
  if (!ctx || (n > 0 && !X) || !centroids || (n > 0 && !labels) || !sums || !counts || n < 0 || dim < 1 ||
      dim > EMB_MAXD || k < 1 || k > KM_MAXK) {
    set_error("kmeans_partial: bad arguments (k <= %d, dim <= %d)", KM_MAXK, EMB_MAXD); return OTTOHIP_EINVAL;
  }
  if (((size_t)k * dim + k) * 8 > 65536) { set_error("kmeans_partial: k * dim too large for LDS"); return OTTOHIP_ELIMIT; }
  hipStream_t s = S(stream);
  ctx->km_bvalid = false;  // labels written outside the batched steps: their distance bounds are stale
  OH_HIP(hipSetDevice(ctx->device));
  double* st;  // [inertia, changed]
  OH_TRY(ctx->ws.get("km_stats", 4, &st));
  unsigned long long* chg = reinterpret_cast<unsigned long long*>(st + 1);
  OH_HIP(hipMemsetAsync(sums, 0, (size_t)k * dim * 8, s));
  OH_HIP(hipMemsetAsync(counts, 0, (size_t)k * 8, s));
  OH_HIP(hipMemsetAsync(st, 0, 2 * 8, s));
  if (n > 0)
    OH_TRY(launch_km_assign(ctx, k, s, X, n, dim, centroids, labels, reinterpret_cast<unsigned long long*>(sums),
                            reinterpret_cast<unsigned long long*>(counts), st, chg, nullptr));
  double h[2] = {0.0, 0.0};
  OH_TRY(d2h(h, st, 2, s));
  if (inertia) *inertia = h[0];
  if (n_changed) { unsigned long long c; memcpy(&c, &h[1], 8); *n_changed = (int64_t)c; }
  return 0;
}

// M-step: centroids = sums / counts for non-empty clusters (empty ones keep theirs), shift^2
int ottohip_kmeans_update(ottohip_ctx* ctx, float* centroids, const int64_t* sums, const int64_t* counts, int k,
                          int dim, double* shift2, void* stream) {
  if (!ctx || !centroids || !sums || !counts || k < 1 || dim < 1) { set_error("kmeans_update: bad arguments"); return OTTOHIP_EINVAL; }
  hipStream_t s = S(stream);
  double* st;
  OH_TRY(ctx->ws.get("km_ustats", 2, &st));
  k_km_update<<<1, KM_UT, 0, s>>>(centroids, reinterpret_cast<const long long*>(sums),
                                  reinterpret_cast<const long long*>(counts), k, dim, 0, st);
  OH_HIP(hipGetLastError());
  double h[2];
  OH_TRY(d2h(h, st, 2, s));
  if (shift2) *shift2 = h[0];
  return 0;
}

// One whole Lloyd iteration on one GPU with a single device->host copy: E-step (labels, fixed-point
// sums, counts, changed labels, inertia) and, unless a cluster came out empty, the M-step. sums /
// counts are incremental: on entry they hold the exact sums / counts of the rows under `labels`
// (zero with labels = -1 at the start of a run); only rows whose label changes move their vector.
// out[0] inertia, [1] changed labels, [2] shift^2 (-1: not updated), [3] empty clusters. With
// out[3] > 0 the centroids are unchanged; sums / counts are ready for ottohip_kmeans_relocate and
// ottohip_kmeans_update (sklearn 1.2 _kmeans_single_lloyd order).
int ottohip_kmeans_lloyd_iter(ottohip_ctx* ctx, const float* X, int64_t n, int dim, float* centroids, int k,
                              int32_t* labels, int64_t* sums, int64_t* counts, double* out, void* stream) {
  if (!ctx || !X || !centroids || !labels || !sums || !counts || !out || n < 1 || dim < 1 || dim > EMB_MAXD ||
      k < 1 || k > KM_MAXK) {
    set_error("kmeans_lloyd_iter: bad arguments (k <= %d, dim <= %d)", KM_MAXK, EMB_MAXD); return OTTOHIP_EINVAL;
  }
  if (((size_t)k * dim + k) * 8 > 65536) { set_error("kmeans_lloyd_iter: k * dim too large for LDS"); return OTTOHIP_ELIMIT; }
  hipStream_t s = S(stream);
  ctx->km_bvalid = false;  // labels written outside the batched steps: their distance bounds are stale
  OH_HIP(hipSetDevice(ctx->device));
  double* st;  // [inertia, changed, shift, empty]
  OH_TRY(ctx->ws.get("km_stats", 4, &st));
  OH_HIP(hipMemsetAsync(st, 0, 4 * 8, s));
  OH_TRY(launch_km_assign(ctx, k, s, X, n, dim, centroids, labels, reinterpret_cast<unsigned long long*>(sums),
                          reinterpret_cast<unsigned long long*>(counts), st,
                          reinterpret_cast<unsigned long long*>(st + 1), nullptr, 1));
  k_km_update<<<1, KM_UT, 0, s>>>(centroids, reinterpret_cast<const long long*>(sums),
                                  reinterpret_cast<const long long*>(counts), k, dim, 1, st + 2);
  OH_HIP(hipGetLastError());
  double h[4];
  OH_TRY(d2h(h, st, 4, s));
  unsigned long long c, e;
  memcpy(&c, &h[1], 8);
  memcpy(&e, &h[3], 8);
  out[0] = h[0];
  out[1] = (double)c;
  out[2] = h[2];
  out[3] = (double)e;
  return 0;
}

// Up to max_steps Lloyd iterations with one device->host copy: each step's update kernel checks
// sklearn's stop conditions on the device and gates the later steps. out[0..3] as lloyd_iter for the
// last step run, out[4] steps run, out[5] stop reason (0 none, 1 no label changed, 2 shift^2 <= tol,
// 3 empty cluster: centroids untouched, relocate then ottohip_kmeans_update). Each E-step is the
// split-precision pass plus the exact f32 kernel on its near ties (OTTOHIP_KM_SPLIT=0: the exact kernel on
// every row; labels, sums and stop checks are identical): out[0] then holds the near ties' inertia only
// (the run's inertia is ottohip_kmeans_inertia's).
int ottohip_kmeans_attach_half(ottohip_ctx* ctx, const float* X, int64_t n, int dim, void* stream) {
  if (!ctx || !X || n < 1 || dim < 1 || dim > EMB_MAXD || (dim & 3)) {
    set_error("kmeans_attach_half: bad arguments (dim <= %d, dim %% 4 == 0)", EMB_MAXD); return OTTOHIP_EINVAL;
  }
  hipStream_t s = S(stream);
  OH_HIP(hipSetDevice(ctx->device));
  // 16-B chunks per row (8 dims each; the last one zero padded past dim), one pad chunk after the last row:
  // k_km_split16 reads a row's KS chunk pairs unconditionally and masks the one past the row
  const int kc = (dim + 7) / 8;
  uint4* x16;
  float* xn2;
  OH_TRY(ctx->ws.get("km_x16", (size_t)n * kc + 1, &x16));
  OH_HIP(hipMemsetAsync(x16 + (size_t)n * kc, 0, sizeof(uint4), s));
  OH_TRY(ctx->ws.get("km_xn2", (size_t)n * 2, &xn2));  // {|x|^2, |x - xh|} per row
  unsigned* amax;
  OH_TRY(ctx->ws.get("km_amax", 1, &amax));
  ctx->km_hX = nullptr;  // no half copy is attached unless this one is accepted
  OH_HIP(hipMemsetAsync(amax, 0, sizeof(unsigned), s));
  k_km_half_rows<<<(unsigned)ceil_div(n * 64, 256), 256, 0, s>>>(X, n, dim, kc, x16, xn2, amax);
  OH_HIP(hipGetLastError());
  unsigned hmax = 0;
  OH_TRY(d2h(&hmax, amax, 1, s));
  if (hmax > __builtin_bit_cast(unsigned, KMH_MAXABS)) {
    set_error("kmeans_attach_half: max |x| = %g exceeds the f16 range bound %g (or is not finite)",
              (double)__builtin_bit_cast(float, hmax), (double)KMH_MAXABS);
    return OTTOHIP_ELIMIT;
  }
  ctx->km_hX = X; ctx->km_hn = n; ctx->km_hdim = dim; ctx->km_x16 = x16; ctx->km_xn2 = xn2;
  return 0;
}

int ottohip_kmeans_detach_half(ottohip_ctx* ctx) {
  if (!ctx) return OTTOHIP_EINVAL;
  ctx->km_hX = nullptr;
  return 0;
}

int ottohip_kmeans_lloyd_steps(ottohip_ctx* ctx, const float* X, int64_t n, int dim, float* centroids, int k,
                               int32_t* labels, int64_t* sums, int64_t* counts, int max_steps, double tol,
                               double* out, void* stream) {
  if (!ctx || !X || !centroids || !labels || !sums || !counts || !out || n < 1 || dim < 1 || dim > EMB_MAXD ||
      k < 1 || k > KM_MAXK || max_steps < 1) {
    set_error("kmeans_lloyd_steps: bad arguments (k <= %d, dim <= %d)", KM_MAXK, EMB_MAXD); return OTTOHIP_EINVAL;
  }
  if (((size_t)k * dim + k) * 8 > 65536) { set_error("kmeans_lloyd_steps: k * dim too large for LDS"); return OTTOHIP_ELIMIT; }
  if (!km_mfma_ok(k, dim, X, centroids)) {  // VALU E-step: one step, stop reason from the host
    OH_TRY(ottohip_kmeans_lloyd_iter(ctx, X, n, dim, centroids, k, labels, sums, counts, out, stream));
    out[4] = 1;
    out[5] = out[3] > 0 ? 3 : (out[1] == 0 ? 1 : (out[2] <= tol ? 2 : 0));
    return 0;
  }
  hipStream_t s = S(stream);
  OH_HIP(hipSetDevice(ctx->device));
  double* st;  // [inertia, changed, shift, empty]
  int* ctl;
  OH_TRY(ctx->ws.get("km_stats", 4, &st));
  OH_TRY(ctx->ws.get("km_ctl", 2, &ctl));
  OH_HIP(hipMemsetAsync(ctl, 0, 2 * sizeof(int), s));
  // the distance bounds carry over from the previous call on the same rows and labels (a new run
  // resets its labels to -1, which scores those rows); otherwise the first step rebuilds them
  const bool bvalid = ctx->km_bvalid && ctx->km_bX == X && ctx->km_bL == labels && ctx->km_bn == n &&
                      ctx->km_bdim == dim && ctx->km_bk == k;
  ctx->km_bvalid = false;
  for (int i = 0; i < max_steps; ++i) {
    k_km_gate_reset<<<1, 64, 0, s>>>(ctl, st);
    OH_TRY(launch_km_assign(ctx, k, s, X, n, dim, centroids, labels, reinterpret_cast<unsigned long long*>(sums),
                            reinterpret_cast<unsigned long long*>(counts), st,
                            reinterpret_cast<unsigned long long*>(st + 1), nullptr, 1, ctl, true,
                            (i == 0 && !bvalid) ? 1 : 0));
    k_km_update<<<1, KM_UT, 0, s>>>(centroids, reinterpret_cast<const long long*>(sums),
                                    reinterpret_cast<const long long*>(counts), k, dim, 1, st + 2, ctl,
                                    reinterpret_cast<const unsigned long long*>(st + 1), tol);
  }
  OH_HIP(hipGetLastError());
  double h[4];
  int c2[2];
  OH_TRY(d2h(h, st, 4, s));
  OH_TRY(d2h(c2, ctl, 2, s));
  ctx->km_bX = X; ctx->km_bL = labels; ctx->km_bn = n; ctx->km_bdim = dim; ctx->km_bk = k;
  ctx->km_bvalid = km_bounds_on(n);
  unsigned long long c, e;
  memcpy(&c, &h[1], 8);
  memcpy(&e, &h[3], 8);
  out[0] = h[0];
  out[1] = (double)c;
  out[2] = h[2];
  out[3] = (double)e;
  out[4] = c2[1];
  out[5] = c2[0];
  return 0;
}

// ottohip_kmeans_lloyd_steps for up to KMM_MAXG runs in lockstep (k_km_assign_split_multi: one read of X per
// step for all of them). Per run the same steps, stop checks and outputs as ottohip_kmeans_lloyd_steps; a run
// that stops (its gate) costs nothing in the other runs' later steps.
__global__ void k_km_gate_set(int* __restrict__ ctl, int reason) {
  if (threadIdx.x == 0 && ctl[0] == 0) ctl[0] = reason;
}

int ottohip_kmeans_lloyd_steps_multi(ottohip_ctx* ctx, const float* X, int64_t n, int dim, float* const* centroids,
                                     int k, int32_t* const* labels, int64_t* const* sums, int64_t* const* counts,
                                     const int* max_steps, int n_runs, double tol, double* out, void* stream) {
  if (!ctx || !X || !centroids || !labels || !sums || !counts || !out || !max_steps || n < 1 || dim < 1 ||
      dim > EMB_MAXD || k < 1 || k > KM_MAXK || n_runs < 1 || n_runs > KMM_MAXG) {
    set_error("kmeans_lloyd_steps_multi: bad arguments (k <= %d, dim <= %d, 1 <= n_runs <= %d)", KM_MAXK, EMB_MAXD,
              KMM_MAXG);
    return OTTOHIP_EINVAL;
  }
  for (int g = 0; g < n_runs; ++g)
    if (max_steps[g] < 0 || !centroids[g] || !labels[g] || !sums[g] || !counts[g] || !km_mfma_ok(k, dim, X, centroids[g]) ||
        k <= 32 || dim > 112 || n > 0xFFFFFFFFll) {
      set_error("kmeans_lloyd_steps_multi: needs the MFMA E-step (32 < k <= 64, dim <= 112, aligned operands)");
      return OTTOHIP_ELIMIT;
    }
  hipStream_t s = S(stream);
  OH_HIP(hipSetDevice(ctx->device));
  ctx->km_bvalid = false;  // no distance bounds in lockstep steps
  constexpr int NB = 2, KS = 7;
  const int G = n_runs;
  const int KP = (k + 7) / 8 * 8, nq = (dim + 7) / 8;
  double* st;  // [G][inertia, changed, shift, empty]
  int* ctl;    // [G][reason, steps]
  OH_TRY(ctx->ws.get("kmm_stats", (size_t)4 * KMM_MAXG, &st));
  OH_TRY(ctx->ws.get("kmm_ctl", (size_t)2 * KMM_MAXG, &ctl));
  OH_HIP(hipMemsetAsync(ctl, 0, (size_t)2 * KMM_MAXG * sizeof(int), s));
  KmMulti P;
  memset(&P, 0, sizeof P);
  float* cn[KMM_MAXG] = {};
  for (int g = 0; g < G; ++g) {
    char nm[32];
    snprintf(nm, sizeof nm, "kmm_cn%d", g);
    OH_TRY(ctx->ws.get(nm, (size_t)KM_MAXK, &cn[g]));
    snprintf(nm, sizeof nm, "kmm_amb%d", g);
    OH_TRY(ctx->ws.get(nm, (size_t)n, &P.amb_rows[g]));
    snprintf(nm, sizeof nm, "kmm_namb%d", g);
    OH_TRY(ctx->ws.get(nm, 2, &P.n_amb[g]));  // [near ties, moves]
    P.n_moves[g] = P.n_amb[g] + 1;
    snprintf(nm, sizeof nm, "kmm_mv%d", g);
    OH_TRY(ctx->ws.get(nm, (size_t)n, &P.moves[g]));
    P.C[g] = centroids[g];
    P.cn[g] = cn[g];
    P.label[g] = labels[g];
    P.changed[g] = reinterpret_cast<unsigned long long*>(st + 4 * g + 1);
    P.gate[g] = ctl + 2 * g;
  }
  const size_t ldsm = (size_t)G * NB * KS * 2 * 64 * 16 + (size_t)G * 64 * 4;
  const void* mk = nullptr;
  switch (G) {
    case 1: mk = reinterpret_cast<const void*>(k_km_assign_split_multi<1, NB, KS>); break;
    case 2: mk = reinterpret_cast<const void*>(k_km_assign_split_multi<2, NB, KS>); break;
    case 3: mk = reinterpret_cast<const void*>(k_km_assign_split_multi<3, NB, KS>); break;
    default: mk = reinterpret_cast<const void*>(k_km_assign_split_multi<4, NB, KS>); break;
  }
  OH_HIP(hipFuncSetAttribute(mk, hipFuncAttributeMaxDynamicSharedMemorySize, (int)ldsm));
  const size_t ldsa = ((size_t)k * dim + k) * 8 + (KM_MT / 64) * 96 * 4;
  OH_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(k_km_apply_moves), hipFuncAttributeMaxDynamicSharedMemorySize,
                             (int)ldsa));
  auto ek = nq == 13 ? k_km_assign_mfma<NB, 13, true> : k_km_assign_mfma<NB, KM_NQ, true>;
  const size_t lds = (size_t)NB * nq * 64 * 16 + (KM_MT / 64) * 96 * 4 + 64 * 4 + ((size_t)k * dim + k) * 8;
  OH_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(ek), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  const int64_t ntile = ceil_div(n, 32);
  const unsigned pgrid = (unsigned)std::max<int64_t>(1, std::min<int64_t>(ceil_div(ntile, KM_MT / 64), ctx->n_cu));
  const unsigned egrid = (unsigned)std::max(1, ctx->n_cu / 2);
  const unsigned agrid = (unsigned)std::max(1, ctx->n_cu);
  int steps = 0;
  for (int g = 0; g < G; ++g) steps = std::max(steps, max_steps[g]);
  for (int i = 0; i < steps; ++i) {
    for (int g = 0; g < G; ++g) {
      if (i == max_steps[g]) k_km_gate_set<<<1, 64, 0, s>>>(ctl + 2 * g, 4);  // this run's step budget is spent
      k_km_gate_reset<<<1, 64, 0, s>>>(ctl + 2 * g, st + 4 * g);
      k_km_prep<<<grid_for(std::max<int64_t>((int64_t)KP * dim, KM_MAXK)), 256, 0, s>>>(centroids[g], k, dim, KP,
                                                                                       nullptr, cn[g]);
      OH_HIP(hipMemsetAsync(P.n_amb[g], 0, 16, s));
    }
    switch (G) {
      case 1: k_km_assign_split_multi<1, NB, KS><<<pgrid, KM_MT, ldsm, s>>>(X, n, dim, k, P); break;
      case 2: k_km_assign_split_multi<2, NB, KS><<<pgrid, KM_MT, ldsm, s>>>(X, n, dim, k, P); break;
      case 3: k_km_assign_split_multi<3, NB, KS><<<pgrid, KM_MT, ldsm, s>>>(X, n, dim, k, P); break;
      default: k_km_assign_split_multi<4, NB, KS><<<pgrid, KM_MT, ldsm, s>>>(X, n, dim, k, P); break;
    }
    for (int g = 0; g < G; ++g) {
      unsigned long long* sg = reinterpret_cast<unsigned long long*>(sums[g]);
      unsigned long long* cg = reinterpret_cast<unsigned long long*>(counts[g]);
      k_km_apply_moves<<<agrid, KM_MT, ldsa, s>>>(X, dim, k, P.moves[g], P.n_moves[g], sg, cg, P.gate[g]);
      // the near ties of the run, exact f32 scores
      ek<<<egrid, KM_MT, lds, s>>>(X, n, dim, nq, centroids[g], cn[g], k, labels[g], sg, cg, st + 4 * g, P.changed[g],
                                   nullptr, 1, P.gate[g], P.amb_rows[g], P.n_amb[g]);
      k_km_update<<<1, KM_UT, 0, s>>>(centroids[g], reinterpret_cast<const long long*>(sums[g]),
                                      reinterpret_cast<const long long*>(counts[g]), k, dim, 1, st + 4 * g + 2,
                                      ctl + 2 * g, reinterpret_cast<const unsigned long long*>(st + 4 * g + 1), tol);
    }
  }
  OH_HIP(hipGetLastError());
  double h[4 * KMM_MAXG];
  int c2[2 * KMM_MAXG];
  OH_TRY(d2h(h, st, (size_t)4 * KMM_MAXG, s));
  OH_TRY(d2h(c2, ctl, (size_t)2 * KMM_MAXG, s));
  for (int g = 0; g < G; ++g) {
    unsigned long long c, e;
    memcpy(&c, &h[4 * g + 1], 8);
    memcpy(&e, &h[4 * g + 3], 8);
    out[6 * g + 0] = h[4 * g];
    out[6 * g + 1] = (double)c;
    out[6 * g + 2] = h[4 * g + 2];
    out[6 * g + 3] = (double)e;
    out[6 * g + 4] = c2[2 * g + 1];
    out[6 * g + 5] = c2[2 * g] == 4 ? 0 : c2[2 * g];  // 4: stopped by its step budget, not a stop check
  }
  return 0;
}

int ottohip_kmeans_lloyd_steps_pair(ottohip_ctx* ctx, const float* X, int64_t n, int dim, float* const* centroids,
                                    int k, int32_t* const* labels, int64_t* const* sums, int64_t* const* counts,
                                    const int* max_steps, double tol, double* out, void* stream) {
  return ottohip_kmeans_lloyd_steps_multi(ctx, X, n, dim, centroids, k, labels, sums, counts, max_steps, 2, tol, out,
                                          stream);
}

// the m rows farthest from their labelled centroid, (distance desc, row asc)
int ottohip_kmeans_farthest(ottohip_ctx* ctx, const float* X, int64_t n, int dim, const float* centroids,
                            const int32_t* labels, int m, int64_t* rows, float* d2, void* stream) {
  if (!ctx || (n > 0 && (!X || !labels)) || !centroids || m < 0 || m > KM_MAXK || (m > 0 && (!rows || !d2)) ||
      n < 0 || dim < 1) {
    set_error("kmeans_farthest: bad arguments"); return OTTOHIP_EINVAL;
  }
  hipStream_t s = S(stream);
  OH_HIP(hipSetDevice(ctx->device));
  const int mm = (int)std::min<int64_t>(m, n);
  for (int j = mm; j < m; ++j) { rows[j] = -1; d2[j] = -1.f; }
  if (mm == 0) return 0;
  float* dist;
  int64_t* taken;
  unsigned long long* best;
  OH_TRY(ctx->ws.get("km_dist", (size_t)n, &dist));
  OH_TRY(ctx->ws.get("km_taken", (size_t)KM_MAXK, &taken));
  OH_TRY(ctx->ws.get("km_best", 1, &best));
  const unsigned grid = (unsigned)std::min<int64_t>(ceil_div(n, 256), (int64_t)ctx->n_cu * 8);
  k_km_labelled<<<grid, 256, 0, s>>>(X, n, dim, centroids, labels, dist, nullptr);
  for (int j = 0; j < mm; ++j) {
    OH_HIP(hipMemsetAsync(best, 0, 8, s));
    k_km_argmax<<<grid, 256, 0, s>>>(dist, n, taken, j, best);
    unsigned long long b = 0;
    OH_TRY(d2h(&b, best, 1, s));
    rows[j] = (int64_t)(uint32_t)~(uint32_t)b;
    const uint32_t o = (uint32_t)(b >> 32), bits = (o & 0x80000000u) ? (o & 0x7FFFFFFFu) : ~o;
    memcpy(&d2[j], &bits, 4);
    OH_HIP(hipMemcpyAsync(taken + j, rows + j, 8, hipMemcpyHostToDevice, s));
  }
  OH_HIP(hipStreamSynchronize(s));
  return 0;
}

// sklearn's empty-cluster relocation on the (all-reduced) sums: vecs (device m x dim) move from
// cluster old_new[2j] to the empty cluster old_new[2j + 1] (old_new HOST)
int ottohip_kmeans_relocate(ottohip_ctx* ctx, int64_t* sums, int64_t* counts, int k, int dim, const float* vecs,
                            const int32_t* old_new, int m, void* stream) {
  if (!ctx || !sums || !counts || m < 0 || (m > 0 && (!vecs || !old_new)) || k < 1 || dim < 1 || dim > 1024) {
    set_error("kmeans_relocate: bad arguments"); return OTTOHIP_EINVAL;
  }
  for (int j = 0; j < 2 * m; ++j)
    if (old_new[j] < 0 || old_new[j] >= k) { set_error("kmeans_relocate: cluster out of range"); return OTTOHIP_ERANGE; }
  if (m == 0) return 0;
  hipStream_t s = S(stream);
  int32_t* mv;
  OH_TRY(ctx->ws.get("km_moves", (size_t)2 * m, &mv));
  OH_HIP(hipMemcpyAsync(mv, old_new, (size_t)2 * m * 4, hipMemcpyHostToDevice, s));
  k_km_relocate<<<grid_for(dim), 256, 0, s>>>(reinterpret_cast<unsigned long long*>(sums),
                                              reinterpret_cast<unsigned long long*>(counts), dim, vecs, mv, m);
  OH_HIP(hipGetLastError());
  OH_HIP(hipStreamSynchronize(s));
  return 0;
}

// sum over rows of |x - centroid[label]|^2 (sklearn's _inertia for a given labelling)
int ottohip_kmeans_inertia(ottohip_ctx* ctx, const float* X, int64_t n, int dim, const float* centroids,
                           const int32_t* labels, double* inertia, void* stream) {
  if (!ctx || (n > 0 && (!X || !labels)) || !centroids || !inertia || n < 0 || dim < 1) {
    set_error("kmeans_inertia: bad arguments"); return OTTOHIP_EINVAL;
  }
  hipStream_t s = S(stream);
  double *inr, *wp;
  OH_TRY(ctx->ws.get("km_inertia", 1, &inr));
  OH_HIP(hipMemsetAsync(inr, 0, 8, s));
  if (n > 0) {  // deterministic: per-wave partials summed in a fixed order (sklearn keeps the first of equal runs)
    const unsigned g = (unsigned)std::min<int64_t>(ceil_div(n, 256), (int64_t)ctx->n_cu * 8);
    OH_TRY(ctx->ws.get("km_inertia_parts", (size_t)g * 4, &wp));
    k_km_labelled<<<g, 256, 0, s>>>(X, n, dim, centroids, labels, nullptr, nullptr, wp);
    k_sum_fixed<<<1, 1024, 0, s>>>(wp, (int64_t)g * 4, inr);
  }
  OH_HIP(hipGetLastError());
  OH_TRY(d2h(inertia, inr, 1, s));
  return 0;
}

int ottohip_col_sums(ottohip_ctx* ctx, const float* X, int64_t n, int dim, const float* center, int64_t* sum_x,
                     int64_t* sum_sq, void* stream) {
  if (!ctx || (n > 0 && !X) || !sum_x || !sum_sq || n < 0 || dim < 1 || dim > 128) {
    set_error("col_sums: bad arguments (dim <= 128)"); return OTTOHIP_EINVAL;
  }
  hipStream_t s = S(stream);
  OH_HIP(hipSetDevice(ctx->device));
  OH_HIP(hipMemsetAsync(sum_x, 0, (size_t)dim * 8, s));
  OH_HIP(hipMemsetAsync(sum_sq, 0, (size_t)dim * 8, s));
  if (n > 0)
    k_col_sums<<<(unsigned)std::min<int64_t>(n, (int64_t)ctx->n_cu * 16), 128, 0, s>>>(
        X, n, dim, center, reinterpret_cast<unsigned long long*>(sum_x), reinterpret_cast<unsigned long long*>(sum_sq));
  OH_HIP(hipGetLastError());
  return 0;
}

int ottohip_center_rows(ottohip_ctx* ctx, const float* X, int64_t n, int dim, const float* mean, float* out,
                        void* stream) {
  if (!ctx || (n > 0 && (!X || !out)) || !mean || n < 0 || dim < 1) { set_error("center_rows: bad arguments"); return OTTOHIP_EINVAL; }
  if (n == 0) return 0;
  hipStream_t s = S(stream);
  OH_HIP(hipSetDevice(ctx->device));
  k_center_rows<<<grid_for(n * dim), 256, 0, s>>>(X, n, dim, mean, out);
  OH_HIP(hipGetLastError());
  return 0;
}

// labels only (final assignment after the last update, as sklearn's labels_)
int ottohip_kmeans_assign(ottohip_ctx* ctx, const float* X, int64_t n, int dim, const float* centroids, int k,
                          int32_t* labels, double* inertia, void* stream) {
  if (!ctx || !X || !centroids || !labels || n < 1 || dim < 1 || dim > EMB_MAXD || k < 1 || k > KM_MAXK) {
    set_error("kmeans_assign: bad arguments"); return OTTOHIP_EINVAL;
  }

  hipStream_t s = S(stream);
  ctx->km_bvalid = false;  // labels written outside the batched steps: their distance bounds are stale
  double* inr;
  OH_TRY(ctx->ws.get("km_inertia", 1, &inr));
  OH_HIP(hipMemsetAsync(inr, 0, 8, s));
  OH_TRY(launch_km_assign(ctx, k, s, X, n, dim, centroids, labels, nullptr, nullptr, inr));
  double h = 0.0;
  OH_TRY(d2h(&h, inr, 1, s));
  if (inertia) *inertia = h;
  return 0;
}

struct ottohip_pop {
  int64_t n = 0;
  int32_t* aid = nullptr;
  int32_t* cl = nullptr;
  int16_t* rank = nullptr;  // [n][6]
};

int ottohip_pop_counts(ottohip_ctx* ctx, const int64_t* session_offsets, int64_t n_sessions, const int32_t* aid,
                       const int32_t* ts, const int8_t* type, const int32_t* session_cl, int32_t n_items,
                       int32_t n_clusters, int32_t ts_7d, uint32_t* counts, void* stream) {
  if (!ctx || !counts || n_sessions < 0 || n_items < 1 || n_clusters < 1 ||
      (n_sessions > 0 && (!session_offsets || !aid || !ts || !type || !session_cl))) {
    set_error("pop_counts: bad arguments"); return OTTOHIP_EINVAL;
  }
  const int64_t NS = (int64_t)n_clusters * n_items;
  if (NS >= ((int64_t)1 << 32)) { set_error("pop_counts: n_clusters * n_items >= 2^32"); return OTTOHIP_ELIMIT; }
  hipStream_t s = S(stream);
  OH_HIP(hipSetDevice(ctx->device));
  uint32_t* present;
  int* err;
  OH_TRY(ctx->ws.get("pop_present", (size_t)NS, &present));  // scratch for k_pop_count's presence marks
  OH_TRY(ctx->ws.get("pop_err", 1, &err));
  OH_HIP(hipMemsetAsync(err, 0, sizeof(int), s));
  if (n_sessions > 0)
    k_pop_count<<<(unsigned)ceil_div(n_sessions, 4), 256, 0, s>>>(session_offsets, n_sessions, aid, ts, type, session_cl,
                                                                   n_items, n_clusters, ts_7d, counts, present, err);
  OH_HIP(hipGetLastError());
  int herr = 0;
  OH_TRY(d2h(&herr, err, 1, s));
  if (herr) { set_error("pop_counts: cluster, aid or type out of range"); return OTTOHIP_ERANGE; }
  return 0;
}

int ottohip_popularity_from_counts(ottohip_ctx* ctx, const uint32_t* cnt, int32_t n_items, int32_t n_clusters,
                                   int keep_top_k, ottohip_pop** out, int64_t* n_out, void* stream) {
  if (!ctx || !cnt || !out || !n_out || n_items < 1 || n_clusters < 1) {
    set_error("popularity_from_counts: bad arguments"); return OTTOHIP_EINVAL;
  }
  const int64_t NS = (int64_t)n_clusters * n_items;
  if (NS >= ((int64_t)1 << 32)) { set_error("popularity_from_counts: n_clusters * n_items >= 2^32"); return OTTOHIP_ELIMIT; }
  *out = nullptr;
  *n_out = 0;
  hipStream_t s = S(stream);
  OH_HIP(hipSetDevice(ctx->device));
  Workspace& ws = ctx->ws;
  uint32_t* present;
  uint64_t *pidx, *tot;
  OH_TRY(ws.get("pop_present", (size_t)NS, &present));
  OH_TRY(ws.get("pop_pidx", (size_t)NS, &pidx));
  OH_TRY(ws.get("pop_tot", 2, &tot));
  int ph = ctx->begin("pop_ranks", s, 0);
  k_pop_present<<<grid_for(NS), 256, 0, s>>>(cnt, NS, present);
  OH_TRY(exclusive_scan_u32(ctx, present, pidx, NS, tot, s));
  uint64_t np_ = 0;
  OH_TRY(d2h(&np_, tot, 1, s));
  ottohip_pop* P = new ottohip_pop();
  const int64_t n = (int64_t)np_;
  if (n == 0) { *out = P; return 0; }
  uint32_t *slot, *k0, *v0, *k1, *v1, *keep;
  uint16_t* rank;
  uint64_t *cl_first, *oidx;
  auto fail = [&](int rc) { dev_free(P->aid); dev_free(P->cl); dev_free(P->rank); delete P; return rc; };
  int rc;
  if ((rc = ws.get("pop_slot", (size_t)n, &slot)) || (rc = ws.get("pop_k0", (size_t)n, &k0)) ||
      (rc = ws.get("pop_v0", (size_t)n, &v0)) || (rc = ws.get("pop_k1", (size_t)n, &k1)) ||
      (rc = ws.get("pop_v1", (size_t)n, &v1)) || (rc = ws.get("pop_rank", (size_t)n * 6, &rank)) ||
      (rc = ws.get("pop_clf", (size_t)n_clusters + 1, &cl_first)) ||
      (rc = ws.get("pop_keep", (size_t)n, &keep)) || (rc = ws.get("pop_oidx", (size_t)n, &oidx)))
    return fail(rc);
  k_pop_pairs<<<grid_for(NS), 256, 0, s>>>(present, pidx, NS, slot);
  k_pop_cluster_first<<<grid_for(n + 1), 256, 0, s>>>(slot, n, n_items, n_clusters, cl_first);
  const int cbits = std::max(1, bits_for((uint64_t)n_clusters));
  for (int t = 0; t < 6; ++t) {
    const uint32_t* c = cnt + (size_t)t * NS;
    uint32_t *k = k0, *v = v0;
    // pairs are in (cluster, aid) order, so aid asc is the stable base: sort by count desc, then cluster
    k_pop_key<<<grid_for(n), 256, 0, s>>>(slot, nullptr, n, c, n_items, 1, k);
    k_pop_iota<<<grid_for(n), 256, 0, s>>>(v, n);
    if ((rc = radix_sort_pairs(ctx, k, v, k1, v1, n, 32, s))) return fail(rc);
    uint32_t* kn = (k == k0) ? k1 : k0;
    k_pop_key<<<grid_for(n), 256, 0, s>>>(slot, v, n, c, n_items, 2, kn);
    k = kn;
    if ((rc = radix_sort_pairs(ctx, k, v, k == k0 ? k1 : k0, v == v0 ? v1 : v0, n, cbits, s))) return fail(rc);
    k_pop_rank<<<grid_for(n), 256, 0, s>>>(slot, v, n, n_items, cl_first, rank + (size_t)t * n);
  }
  k_pop_keep<<<grid_for(n), 256, 0, s>>>(rank, n, keep_top_k, keep);
  if ((rc = exclusive_scan_u32(ctx, keep, oidx, n, tot + 1, s))) return fail(rc);
  uint64_t nk = 0;
  if ((rc = d2h(&nk, tot + 1, 1, s))) return fail(rc);
  P->n = (int64_t)nk;
  if (dev_alloc(reinterpret_cast<void**>(&P->aid), std::max<uint64_t>(nk, 1) * 4, "pop_aid") ||
      dev_alloc(reinterpret_cast<void**>(&P->cl), std::max<uint64_t>(nk, 1) * 4, "pop_cl") ||
      dev_alloc(reinterpret_cast<void**>(&P->rank), std::max<uint64_t>(nk, 1) * 12, "pop_rank"))
    return fail(OTTOHIP_ENOMEM);
  k_pop_out<<<grid_for(n), 256, 0, s>>>(slot, rank, keep, oidx, n, n_items, P->aid, P->cl, P->rank);
  OH_HIP(hipGetLastError());
  ctx->end(ph, s);
  *out = P;
  *n_out = P->n;
  return 0;
}

int ottohip_popularity_ranks(ottohip_ctx* ctx, const int64_t* session_offsets, int64_t n_sessions,
                             const int32_t* aid, const int32_t* ts, const int8_t* type, const int32_t* session_cl,
                             int32_t n_items, int32_t n_clusters, int32_t ts_7d, int keep_top_k,
                             ottohip_pop** out, int64_t* n_out, void* stream) {
  if (!ctx || !out || !n_out || n_items < 1 || n_clusters < 1) { set_error("popularity_ranks: bad arguments"); return OTTOHIP_EINVAL; }
  const int64_t NS = (int64_t)n_clusters * n_items;
  if (NS >= ((int64_t)1 << 32)) { set_error("popularity_ranks: n_clusters * n_items >= 2^32"); return OTTOHIP_ELIMIT; }
  hipStream_t s = S(stream);
  OH_HIP(hipSetDevice(ctx->device));
  uint32_t* cnt;
  OH_TRY(ctx->ws.get("pop_cnt", (size_t)NS * 6, &cnt));
  OH_HIP(hipMemsetAsync(cnt, 0, (size_t)NS * 6 * 4, s));
  OH_TRY(ottohip_pop_counts(ctx, session_offsets, n_sessions, aid, ts, type, session_cl, n_items, n_clusters, ts_7d,
                            cnt, stream));
  return ottohip_popularity_from_counts(ctx, cnt, n_items, n_clusters, keep_top_k, out, n_out, stream);
}

int ottohip_pop_copy(const ottohip_pop* p, int32_t* aid, int32_t* cl, int16_t* ranks6, void* stream) {
  if (!p) { set_error("pop_copy: NULL"); return OTTOHIP_EINVAL; }
  if (p->n == 0) return 0;
  hipStream_t s = S(stream);
  if (aid) OH_HIP(hipMemcpyAsync(aid, p->aid, p->n * 4, hipMemcpyDeviceToDevice, s));
  if (cl) OH_HIP(hipMemcpyAsync(cl, p->cl, p->n * 4, hipMemcpyDeviceToDevice, s));
  if (ranks6) OH_HIP(hipMemcpyAsync(ranks6, p->rank, p->n * 12, hipMemcpyDeviceToDevice, s));
  return 0;
}

void ottohip_pop_free(ottohip_pop* p) {
  if (!p) return;
  (void)hipDeviceSynchronize();
  dev_free(p->aid);
  dev_free(p->cl);
  dev_free(p->rank);
  delete p;
}

int ottohip_session_item_similarity(ottohip_ctx* ctx, const int64_t* cand_off, int64_t n_sessions,
                                    const int32_t* aid_next, const float* sess_emb, const uint8_t* sess_has,
                                    const int32_t* row_of_aid, int32_t n_aid_map, const float* emb, int dim,
                                    float* cos_out, float* eucl_out, void* stream) {
  if (!ctx || n_sessions < 0 || dim < 1 || (n_sessions > 0 && (!cand_off || !sess_emb || !row_of_aid || !emb ||
      !cos_out || !eucl_out))) {
    set_error("session_item_similarity: bad arguments"); return OTTOHIP_EINVAL;
  }
  if (n_sessions == 0) return 0;
  hipStream_t s = S(stream);
  OH_HIP(hipSetDevice(ctx->device));
  int ph = ctx->begin("r7_sim", s, 0);
  const bool vec = dim <= 128 && dim % 4 == 0 && (reinterpret_cast<uintptr_t>(emb) & 15) == 0 &&
                   (reinterpret_cast<uintptr_t>(sess_emb) & 15) == 0;
  if (vec)
    k_sim16<<<(unsigned)std::min<int64_t>(ceil_div(n_sessions, 4), (int64_t)ctx->n_cu * 16), 256, 0, s>>>(
        cand_off, n_sessions, aid_next, sess_emb, sess_has, row_of_aid, n_aid_map, emb, dim, cos_out, eucl_out);
  else
    k_sim<<<(unsigned)ceil_div(n_sessions, 4), 256, 0, s>>>(cand_off, n_sessions, aid_next, sess_emb, sess_has,
                                                            row_of_aid, n_aid_map, emb, dim, cos_out, eucl_out);
  OH_HIP(hipGetLastError());
  ctx->end(ph, s);
  return 0;
}


int ottohip_rs_create(uint32_t seed, ottohip_rs** out) {
  if (!out) { set_error("rs_create: out is NULL"); return OTTOHIP_EINVAL; }
  ottohip_rs* r = new ottohip_rs();
  rs_seed(*r, seed);
  *out = r;
  return 0;
}

void ottohip_rs_destroy(ottohip_rs* r) { delete r; }

int ottohip_rs_permutation_head(ottohip_rs* r, int64_t n, int k, int64_t* out) {
  if (!r || n < 0 || k < 0 || k > n || (k > 0 && !out)) { set_error("rs_permutation_head: bad arguments"); return OTTOHIP_EINVAL; }
  if (n > (int64_t)0xFFFFFFFFll) { set_error("rs_permutation_head: n >= 2^32"); return OTTOHIP_ELIMIT; }
  if (n <= 1) { for (int p = 0; p < k; ++p) out[p] = p; return 0; }
  std::vector<uint32_t>& J = r->J;
  J.resize((size_t)n);
  for (int64_t i = n - 1; i >= 1; --i) J[(size_t)i] = rs_interval(*r, (uint32_t)i);  // the shuffle's draw order
  std::vector<uint64_t>& B = r->bits;
  B.assign((size_t)((n + 63) >> 6), 0ull);
  std::vector<int64_t> ptr((size_t)k);
  for (int p = 0; p < k; ++p) { ptr[(size_t)p] = p; B[(size_t)p >> 6] |= 1ull << (p & 63); }
  auto test = [&](int64_t x) { return (B[(size_t)x >> 6] >> (x & 63)) & 1ull; };
  auto flip = [&](int64_t x) { B[(size_t)x >> 6] ^= 1ull << (x & 63); };
  for (int64_t i = 1; i < n; ++i) {  // swaps replayed last-to-first: value at i <-> value at J[i]
    const int64_t j = J[(size_t)i];
    if (j == i) continue;
    const uint64_t bi = test(i), bj = test(j);
    if (!(bi | bj)) continue;
    for (int p = 0; p < k; ++p) {
      if (ptr[(size_t)p] == i) ptr[(size_t)p] = j;
      else if (ptr[(size_t)p] == j) ptr[(size_t)p] = i;
    }
    if (bi != bj) { flip(i); flip(j); }
  }
  for (int p = 0; p < k; ++p) out[p] = ptr[(size_t)p];
  return 0;
}
}  // extern "C"

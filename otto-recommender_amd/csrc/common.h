// Shared host/device helpers for libottohip.so (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>
#include <map>
#include <type_traits>

#include "ottohip.h"

namespace ottohip {

constexpr int MAX_RULES = 8;  // rules per count call (5 in the reference)

void set_error(const char* fmt, ...);
struct Ctx;
Ctx* ctx_base(ottohip_ctx* c);  // abi.hip

#define OH_HIP(expr)                                                              \
  do {                                                                            \
    hipError_t e_ = (expr);                                                       \
    if (e_ != hipSuccess) {                                                       \
      ::ottohip::set_error("%s:%d %s -> %s", __FILE__, __LINE__, #expr,           \
                           hipGetErrorString(e_));                                \
      return e_ == hipErrorOutOfMemory ? OTTOHIP_ENOMEM : OTTOHIP_EHIP;           \
    }                                                                             \
  } while (0)

#define OH_TRY(expr)                 \
  do {                               \
    int rc_ = (expr);                \
    if (rc_ != 0) return rc_;        \
  } while (0)

// OTTOHIP_ALLOC_LOG=1: every device (re)allocation with its host-side duration on stderr
double alloc_log_begin();
void alloc_log_end(double t0, const char* what, const char* name, size_t bytes);

// Device block cache of the library (abi.hip): freed blocks are kept and handed out again
// (best fit within 2x of the request), so repeated calls do not go back to hipMalloc / hipFree,
// whose cost at 100+ GB resident is erratic (0.5-2 s stalls measured on the box). Blocks are
// reused in stream order: the library issues a call's work on one stream. dev_trim() returns
// every cached block to the driver (ottohip_ctx_trim / ottohip_ctx_destroy).
hipError_t dev_alloc(void** p, size_t bytes, const char* what);
void dev_free(void* p);
void dev_trim();

// Named, grow-only device buffers owned by a context (no allocation inside launches).
struct Workspace {
  struct Buf { void* p = nullptr; size_t bytes = 0; };
  std::map<std::string, Buf> bufs;
  int get(const char* name, size_t bytes, void** out) {
    Buf& b = bufs[name];
    if (b.bytes < bytes) {
      if (b.p) { (void)hipDeviceSynchronize(); dev_free(b.p); b.p = nullptr; b.bytes = 0; }
      size_t want = bytes < 256 ? 256 : bytes;
      hipError_t e = dev_alloc(&b.p, want, name);
      if (e != hipSuccess) {
        set_error("workspace '%s': hipMalloc(%zu) failed: %s", name, want, hipGetErrorString(e));
        return OTTOHIP_ENOMEM;
      }
      b.bytes = want;
    }
    *out = b.p;
    return 0;
  }
  template <class T> int get(const char* name, size_t n, T** out) {
    return get(name, n * sizeof(T), reinterpret_cast<void**>(out));
  }
  void release() {
    for (auto& kv : bufs) if (kv.second.p) dev_free(kv.second.p);
    bufs.clear();
  }
  // hand a buffer over to the caller (who frees it with dev_free); the next get() allocates a new one
  void* take(const char* name) {
    auto it = bufs.find(name);
    if (it == bufs.end()) return nullptr;
    void* p = it->second.p;
    bufs.erase(it);
    return p;
  }
};

struct Phase { std::string name; hipEvent_t a, b; double bytes; };

struct Ctx {
  int device = 0;
  int n_cu = 256;
  Workspace ws;
  uint64_t* pinned = nullptr;   // small host staging for D2H scalars
  bool timing = false;
  std::vector<Phase> phases;
  std::vector<hipEvent_t> event_pool;
  size_t event_used = 0;
  // second stream of the reduce (register-sort tasks overlap the split of the same level)
  hipStream_t aux = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join[2] = {nullptr, nullptr};  // join: by reduce level parity
  // split pipelining: a third stream for the host's read of the first half's task counts; ev_half: the first
  // half classified, ev_hash: the next level's first-half hash leaves done
  hipStream_t aux2 = nullptr;
  hipEvent_t ev_half = nullptr, ev_hash = nullptr;
  int aux_stream() {
    if (aux) return 0;
    if (hipStreamCreateWithFlags(&aux, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&aux2, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&ev_half, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&ev_hash, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&ev_fork, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&ev_join[0], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&ev_join[1], hipEventDisableTiming) != hipSuccess) {
      set_error("aux stream creation failed");
      return OTTOHIP_EHIP;
    }
    return 0;
  }
  hipEvent_t take_event() {
    if (event_used == event_pool.size()) {
      hipEvent_t e; hipEventCreate(&e); event_pool.push_back(e);
    }
    return event_pool[event_used++];
  }
  void reset_timing() { phases.clear(); event_used = 0; }
  // open a named phase on the stream (no-op unless timing is enabled)
  int begin(const char* name, hipStream_t s, double bytes = 0) {
    if (!timing) return -1;
    Phase p; p.name = name; p.a = take_event(); p.b = take_event(); p.bytes = bytes;
    hipEventRecord(p.a, s);
    phases.push_back(p);
    return (int)phases.size() - 1;
  }
  void end(int id, hipStream_t s) { if (id >= 0) hipEventRecord(phases[id].b, s); }
  // KMeans distance bounds (batched Lloyd steps): valid for the rows of (X, labels, n, dim, k) of the
  // last ottohip_kmeans_lloyd_steps call; every other entry point that writes labels clears km_bvalid
  const void* km_bX = nullptr;
  const void* km_bL = nullptr;
  int64_t km_bn = -1;
  int km_bdim = 0, km_bk = 0;
  bool km_bvalid = false;
  // half-precision rows of an attached KMeans matrix (ottohip_kmeans_attach_half): the E-step of
  // ottohip_kmeans_lloyd_steps on that X reads them (and the rows' exact squared norms) instead of the f32 rows
  const void* km_hX = nullptr;
  int64_t km_hn = -1;
  int km_hdim = 0;
  const void* km_x16 = nullptr;
  const float* km_xn2 = nullptr;
  // multi-GPU row keys (abi.hip owner_map): per aid its index among its owner's aids (aid order) and the inverse,
  // for (n_items, G) = (om_items, om_parts); om_lb = bits of the largest owner's aid count
  int64_t om_items = -1;
  int om_parts = 0, om_lb = 0;
};

inline int bits_for(uint64_t n_values) {  // bits needed to store values in [0, n_values)
  int b = 0;
  while (b < 64 && (uint64_t(1) << b) < n_values) ++b;
  return b;
}
__host__ __device__ inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// ---------------------------------------------------------------- device helpers
__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }
__device__ __forceinline__ uint32_t mbcnt(uint64_t m) {  // popcount of m below this lane
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
__device__ __forceinline__ uint64_t shfl64(uint64_t v, int src) {
  uint32_t lo = __shfl((uint32_t)v, src), hi = __shfl((uint32_t)(v >> 32), src);
  return ((uint64_t)hi << 32) | lo;
}
// ---- cross-lane moves without the LDS crossbar: DPP (GFX9 control codes: quad_perm 0x00-0xFF,
// row_shl:n 0x100+n (lane i <- i+n), row_shr:n 0x110+n (lane i <- i-n), row_ror:n 0x120+n) and
// the gfx950 half-row / half-wave swaps
template <int J>
__device__ __forceinline__ uint32_t xor_lane(uint32_t v) {  // value of lane (this ^ J)
  if constexpr (J == 1) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, true);  // quad_perm [1,0,3,2]
  } else if constexpr (J == 2) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, true);  // quad_perm [2,3,0,1]
  } else if constexpr (J == 4) {  // ds_swizzle bitmask mode (xor 4, within 32 lanes): one LDS-crossbar
                                   // instruction instead of two DPP moves and a select
    return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, (4 << 10) | 0x1F);
  } else if constexpr (J == 8) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x128, 0xF, 0xF, true);  // row_ror:8
  } else if constexpr (J == 16) {
    const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    return (lane_id() & 16u) ? r[0] : r[1];
  } else {
    static_assert(J == 32, "xor_lane: J in {1,2,4,8,16,32}");
    const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    return (lane_id() & 32u) ? r[0] : r[1];
  }
}
// J folds to a constant once the caller's loops are unrolled
__device__ __forceinline__ uint32_t xor_lane_n(uint32_t v, int J) {
  switch (J) {
    case 1: return xor_lane<1>(v);
    case 2: return xor_lane<2>(v);
    case 4: return xor_lane<4>(v);
    case 8: return xor_lane<8>(v);
    case 16: return xor_lane<16>(v);
    case 32: return xor_lane<32>(v);
    default: return __shfl_xor(v, J);
  }
}
// inclusive scan over the wave (sum / max) by DPP row shifts and row broadcasts
template <bool MAX>
__device__ __forceinline__ uint32_t dpp_step(uint32_t v, uint32_t t) { return MAX ? (v > t ? v : t) : v + t; }
template <bool MAX>
__device__ __forceinline__ uint32_t dpp_incl_scan(uint32_t v) {
  v = dpp_step<MAX>(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false));
  v = dpp_step<MAX>(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false));
  v = dpp_step<MAX>(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false));
  v = dpp_step<MAX>(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false));
  v = dpp_step<MAX>(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false));  // row_bcast:15
  v = dpp_step<MAX>(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false));  // row_bcast:31
  return v;
}
// value of lane l-1 (0 in lane 0) / lane l+1 (0 in lane 63)
__device__ __forceinline__ uint32_t lane_prev(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x138, 0xF, 0xF, false);  // wave_shr:1
}
__device__ __forceinline__ uint32_t lane_next(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x130, 0xF, 0xF, false);  // wave_shl:1
}
// LDS histogram add of digit d by a wave whose valid lanes form a prefix: runs of equal digits over consecutive
// lanes (consecutive words; a hot key's words arrive in runs, so one digit can fill a wave) take one atomic of
// the run length at the run's first lane; returns the lane's rank among the digit's words (same-address LDS
// atomics of one wave instruction serialise). Wave-uniform call.
__device__ __forceinline__ uint32_t lds_add_runs(uint32_t* h, uint32_t d, bool valid) {
  const uint32_t l = lane_id();
  const uint32_t pd = lane_prev(d);
  const bool head = valid && (l == 0u || pd != d);
  const uint64_t hm = __ballot(head);
  const uint32_t nv = (uint32_t)__popcll(__ballot(valid));
  const uint64_t le = l == 63u ? ~0ull : ((2ull << l) - 1ull);
  const uint64_t after = hm & ~le;
  const uint32_t nh = after ? (uint32_t)__ffsll((long long)after) - 1u : 64u;
  const uint32_t end = nh < nv ? nh : nv;
  uint32_t base = head ? atomicAdd(&h[d], end - l) : 0u;
  const uint64_t upto = hm & le;
  const int hl = upto ? 63 - __clzll((long long)upto) : 0;
  base = (uint32_t)__shfl((int)base, hl);
  return valid ? base + (l - (uint32_t)hl) : 0u;
}

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) { return dpp_incl_scan<false>(v); }
__device__ __forceinline__ uint64_t wave_incl_scan64(uint64_t v) {
  const uint32_t l = lane_id();
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    uint32_t lo = __shfl_up((uint32_t)v, d), hi = __shfl_up((uint32_t)(v >> 32), d);
    uint64_t t = ((uint64_t)hi << 32) | lo;
    if (l >= (uint32_t)d) v += t;
  }
  return v;
}
__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_readlane((int)dpp_incl_scan<false>(v), 63);
}
__device__ __forceinline__ uint64_t wave_sum64(uint64_t v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    const uint32_t lo = __shfl_xor((uint32_t)v, d), hi = __shfl_xor((uint32_t)(v >> 32), d);
    v += ((uint64_t)hi << 32) | lo;
  }
  return v;
}

// owner rank of an aid for the multi-GPU layout: multiplicative hash, range-reduced (no modulo)
__host__ __device__ __forceinline__ uint32_t owner_dev(uint32_t aid, uint32_t n_parts) {
  return (uint32_t)(((uint64_t)(aid * 0x9E3779B1u) * n_parts) >> 32);
}

// Packed event: high 32 = ts ^ 0x80000000 (orders like signed ts), low 32 = aid << 2 | type.
// Sorting packed events ascending orders a session by (ts, aid, type); equal words are the
// exact duplicates removed by df.unique() (model/count_co_events.py:92).
constexpr uint64_t EV_INVALID = ~uint64_t(0);
__device__ __forceinline__ uint64_t ev_pack(int32_t aid, int32_t ts, int32_t type) {
  return ((uint64_t)((uint32_t)ts ^ 0x80000000u) << 32) | ((uint32_t)aid << 2) | (uint32_t)type;
}
__device__ __forceinline__ int32_t ev_ts(uint64_t e) { return (int32_t)((uint32_t)(e >> 32) ^ 0x80000000u); }
__device__ __forceinline__ int32_t ev_aid(uint64_t e) { return (int32_t)(((uint32_t)e) >> 2); }
__device__ __forceinline__ int32_t ev_type(uint64_t e) { return (int32_t)(e & 3u); }

}  // namespace ottohip

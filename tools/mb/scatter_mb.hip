// Microbenchmark (development only): random 8-B / 4-B scatter throughput vs target array size
// (does the 256 MB MALL absorb random writes?). hipcc --offload-arch=gfx950 -O3 scatter_mb.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
__global__ void k_perm(uint32_t* idx, uint64_t n, uint64_t m, uint32_t seed) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint64_t x = (i + 1) * 0x9E3779B97F4A7C15ull ^ seed;
  x ^= x >> 31; x *= 0xBF58476D1CE4E5B9ull; x ^= x >> 27;
  idx[i] = (uint32_t)(x % m);
}
template <class T>
__global__ void k_scatter(const uint32_t* __restrict__ idx, uint64_t n, T* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[idx[i]] = (T)i;
}
template <class T>
__global__ void k_gather(const uint32_t* __restrict__ idx, uint64_t n, const T* __restrict__ in, T* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = in[idx[i]];
}
int main() {
  const uint64_t n = 220000000ull;
  uint32_t* idx; hipMalloc(&idx, n * 4);
  uint64_t* big; hipMalloc(&big, n * 8);
  uint64_t* outv; hipMalloc(&outv, n * 8);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  const uint64_t sizes[] = {8ull << 20, 32ull << 20, 128ull << 20, 256ull << 20, 512ull << 20, 1024ull << 20};
  for (uint64_t bytes : sizes) {
    if (bytes > n * 8) { printf("skip %llu MB: beyond the buffer\n", (unsigned long long)(bytes >> 20)); continue; }
    for (int w = 0; w < 2; ++w) {
      const uint64_t esz = w ? 4 : 8, m = bytes / esz;
      k_perm<<<(n + 255) / 256, 256>>>(idx, n, m, 12345);
      float best[3] = {1e9f, 1e9f, 1e9f};
      for (int rep = 0; rep < 3; ++rep) {
        hipEventRecord(a);
        if (w) k_scatter<uint32_t><<<(n + 255) / 256, 256>>>(idx, n, (uint32_t*)big);
        else k_scatter<uint64_t><<<(n + 255) / 256, 256>>>(idx, n, big);
        hipEventRecord(b); hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b); if (ms < best[0]) best[0] = ms;
        hipEventRecord(a);
        if (w) k_gather<uint32_t><<<(n + 255) / 256, 256>>>(idx, n, (uint32_t*)big, (uint32_t*)outv);
        else k_gather<uint64_t><<<(n + 255) / 256, 256>>>(idx, n, big, outv);
        hipEventRecord(b); hipEventSynchronize(b);
        hipEventElapsedTime(&ms, a, b); if (ms < best[1]) best[1] = ms;
      }
      printf("target %5llu MB  elem %llu B: scatter %.3f ms (%.1f G/s)  gather %.3f ms (%.1f G/s)\n",
             (unsigned long long)(bytes >> 20), (unsigned long long)esz, best[0], n / best[0] / 1e6, best[1], n / best[1] / 1e6);
    }
  }
  return 0;
}

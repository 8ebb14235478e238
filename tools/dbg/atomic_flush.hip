// Microbenchmark: cost of the KMeans per-block flush (G blocks each adding k*dim+k u64 partials into one
// global array) as device-scope atomics vs. plain partial rows + one column-sum kernel.
// hipcc --offload-arch=gfx950 -O3 tools/dbg/atomic_flush.hip -o tools/dbg/atomic_flush
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ __launch_bounds__(768) void k_flush_atomic(unsigned long long* sums, int n, int dens) {
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const unsigned long long v = ((i * 7 + blockIdx.x) % 100) < dens ? (unsigned long long)(i + blockIdx.x) : 0ull;
    if (v) atomicAdd(&sums[i], v);
  }
}
__global__ __launch_bounds__(768) void k_flush_rows(unsigned long long* part, int n, int dens) {
  unsigned long long* row = part + (size_t)blockIdx.x * n;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const unsigned long long v = ((i * 7 + blockIdx.x) % 100) < dens ? (unsigned long long)(i + blockIdx.x) : 0ull;
    row[i] = v;
  }
}
__global__ __launch_bounds__(256) void k_col_sum(const unsigned long long* part, int nb, int n, unsigned long long* sums) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  unsigned long long s = 0;
  for (int b = 0; b < nb; ++b) s += part[(size_t)b * n + i];
  sums[i] += s;
}

int main() {
  const int n = 5050, G = 256, R = 200;
  unsigned long long *sums, *part;
  hipMalloc(&sums, n * 8);
  hipMalloc(&part, (size_t)G * n * 8);
  hipMemset(sums, 0, n * 8);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int dens : {100, 50, 10}) {
    for (int mode = 0; mode < 2; ++mode) {
      for (int w = 0; w < 2; ++w) {
        hipEventRecord(a);
        for (int r = 0; r < R; ++r) {
          if (mode == 0) k_flush_atomic<<<G, 768>>>(sums, n, dens);
          else {
            k_flush_rows<<<G, 768>>>(part, n, dens);
            k_col_sum<<<(n + 255) / 256, 256>>>(part, G, n, sums);
          }
        }
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        if (w) printf("density %3d%% %-8s %.4f ms per flush\n", dens, mode ? "rows+sum" : "atomic", ms / R);
      }
    }
  }
  return 0;
}

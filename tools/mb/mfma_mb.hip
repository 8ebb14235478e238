// Back-to-back issue cost of the bf16 MFMA shapes on one SIMD (one wave per SIMD, 4 independent
// accumulators): cycles per instruction from s_memtime around 4096 instructions.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __attribute__((__vector_size__(8 * sizeof(__bf16)))) __bf16 bf16x8;
typedef __attribute__((__vector_size__(4 * sizeof(short)))) short s16x4;
typedef __attribute__((__vector_size__(16 * sizeof(float)))) float f32x16;

template <int KIND>
__global__ __launch_bounds__(256) void k_mb(float* out, long long* cyc, int n) {
  f32x16 acc[4] = {};
  bf16x8 a, b;
  s16x4 a4, b4;
  for (int i = 0; i < 8; ++i) { a[i] = (__bf16)(threadIdx.x * 0.001f + i); b[i] = (__bf16)(i * 0.5f); }
  for (int i = 0; i < 4; ++i) { a4[i] = (short)(threadIdx.x + i); b4[i] = (short)(i * 3); }
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < n; ++it) {
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      if constexpr (KIND == 0) acc[j & 3] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[j & 3], 0, 0, 0);
      else acc[j & 3] = __builtin_amdgcn_mfma_f32_32x32x8bf16_1k(a4, b4, acc[j & 3], 0, 0, 0);
    }
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0;
  for (int c = 0; c < 4; ++c)
    for (int i = 0; i < 16; ++i) s += acc[c][i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0 && blockIdx.x == 0) cyc[KIND] = t1 - t0;
}

int main() {
  float* out;
  long long* cyc;
  hipMalloc(&out, 256 * 256 * 4);
  hipMalloc(&cyc, 16);
  const int n = 256;
  for (int rep = 0; rep < 2; ++rep) {
    k_mb<0><<<256, 256>>>(out, cyc, n);
    k_mb<1><<<256, 256>>>(out, cyc, n);
    hipDeviceSynchronize();
  }
  long long h[2];
  hipMemcpy(h, cyc, 16, hipMemcpyDeviceToHost);
  // s_memtime counts at the shader clock on gfx950? report raw ticks per instruction and the ratio
  printf("32x32x16_bf16: %.2f ticks/instr\n", (double)h[0] / (n * 16));
  printf("32x32x8bf16_1k: %.2f ticks/instr\n", (double)h[1] / (n * 16));
  printf("ratio x8/x16: %.3f\n", (double)h[1] / h[0]);
  return 0;
}

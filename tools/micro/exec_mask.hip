// Does a wave64 VALU instruction cost less when only lanes 0..31 (or 0..15)
// are active?  Same dependent-free FMA stream under three exec masks.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int ACTIVE>
__global__ __launch_bounds__(64) void fma_stream(float* out, int iters) {
  const int lane = threadIdx.x;
  float a0 = lane * 1e-3f, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  if (lane < ACTIVE) {
    for (int i = 0; i < iters; i++) {
#pragma unroll
      for (int k = 0; k < 16; k++) {
        a0 = fmaf(a0, 0.999f, 0.001f); a1 = fmaf(a1, 0.999f, 0.001f); a2 = fmaf(a2, 0.999f, 0.001f);
        a3 = fmaf(a3, 0.999f, 0.001f); a4 = fmaf(a4, 0.999f, 0.001f); a5 = fmaf(a5, 0.999f, 0.001f);
        a6 = fmaf(a6, 0.999f, 0.001f); a7 = fmaf(a7, 0.999f, 0.001f);
      }
    }
  }
  out[blockIdx.x * 64 + lane] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}

template <int A>
float run(float* d, int blocks, int iters) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL(fma_stream<A>, dim3(blocks), dim3(64), 0, 0, d, iters);
  hipEventRecord(e0);
  for (int r = 0; r < 5; r++) hipLaunchKernelGGL(fma_stream<A>, dim3(blocks), dim3(64), 0, 0, d, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  return ms / 5;
}

int main() {
  float* d;
  const int blocks = 4096, iters = 2000;
  hipMalloc(&d, sizeof(float) * blocks * 64);
  for (int rep = 0; rep < 2; rep++) {
    float t64 = run<64>(d, blocks, iters), t32 = run<32>(d, blocks, iters), t16 = run<16>(d, blocks, iters),
          t1 = run<1>(d, blocks, iters);
    const double inst = (double)blocks * iters * 16 * 8;  // wave-instructions
    printf("active 64: %.3f ms  32: %.3f ms  16: %.3f ms  1: %.3f ms   (%.2f / %.2f / %.2f / %.2f cycles per wave-FMA per SIMD at 2.4 GHz)\n",
           t64, t32, t16, t1, t64 * 1e-3 * 2.4e9 * 1024 / inst, t32 * 1e-3 * 2.4e9 * 1024 / inst,
           t16 * 1e-3 * 2.4e9 * 1024 / inst, t1 * 1e-3 * 2.4e9 * 1024 / inst);
  }
  return 0;
}

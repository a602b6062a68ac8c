// How many cycles does a SIMD spend per wave64 VALU instruction when 1, 2, 4
// or 8 waves share it?  Independent FMA streams (8 accumulators per wave),
// plain v_fma_f32 vs packed v_pk_fma_f32, timed with s_memtime inside the
// kernel (per wave) and hipEvents around it.  Diagnostic.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));

template <bool PK>
__global__ __launch_bounds__(64) void fma_stream(float* out, long long* cyc, int iters) {
  const int lane = threadIdx.x;
  float a[8];
  f2 p[8];
  for (int k = 0; k < 8; k++) { a[k] = lane * 1e-3f + k; p[k] = f2{a[k], a[k] + 0.5f}; }
  const long long t0 = __builtin_readcyclecounter();
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int r = 0; r < 16; r++)
#pragma unroll
      for (int k = 0; k < 8; k++) {
        if constexpr (PK) p[k] = __builtin_elementwise_fma(p[k], f2{0.999f, 0.999f}, f2{0.001f, 0.001f});
        else a[k] = fmaf(a[k], 0.999f, 0.001f);
      }
  }
  const long long t1 = __builtin_readcyclecounter();
  float s = 0.f;
  for (int k = 0; k < 8; k++) s += PK ? p[k].x + p[k].y : a[k];
  out[blockIdx.x * 64 + lane] = s;
  if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

template <bool PK>
void run(float* d, long long* c, int waves_per_simd, int iters) {
  const int blocks = 256 * 4 * waves_per_simd;  // 256 CUs x 4 SIMDs
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL(fma_stream<PK>, dim3(blocks), dim3(64), 0, 0, d, c, iters);
  hipEventRecord(e0);
  hipLaunchKernelGGL(fma_stream<PK>, dim3(blocks), dim3(64), 0, 0, d, c, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  static long long h[256 * 4 * 16];
  hipMemcpy(h, c, sizeof(long long) * blocks, hipMemcpyDeviceToHost);
  double mean = 0;
  for (int b = 0; b < blocks; b++) mean += h[b];
  mean /= blocks;
  const double insts = (double)iters * 16 * 8;  // per wave
  // elapsed cycles at the measured clock: derive from mean per-wave cycles
  printf("%s waves/SIMD %d: %.3f ms, per-wave counter cycles per instruction %.2f, "
         "SIMD cycles per instruction (counter / waves) %.2f, flops %.1f TF\n",
         PK ? "v_pk_fma_f32" : "v_fma_f32  ", waves_per_simd, ms, mean / insts, mean / insts / waves_per_simd,
         (double)blocks * 64 * insts * 2 * (PK ? 2 : 1) / (ms * 1e-3) / 1e12);
}

int main() {
  float* d;
  long long* c;
  hipMalloc(&d, sizeof(float) * 256 * 4 * 16 * 64);
  hipMalloc(&c, sizeof(long long) * 256 * 4 * 16);
  for (int w : {1, 2, 4, 8}) run<false>(d, c, w, 2000);
  for (int w : {1, 2, 4, 8}) run<true>(d, c, w, 2000);
  return 0;
}

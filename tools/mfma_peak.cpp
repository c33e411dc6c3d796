// Diagnostic: sustained v_mfma_f32_32x32x2_f32 rate with no memory traffic (the clock the matrix
// cores actually hold under a full-chip f32 MFMA load), so GEMM efficiencies can be read against
// what the part delivers as well as against the 157.3 TF/s data-sheet peak.  Not part of the product.
//   hipcc --offload-arch=gfx950 -O3 tools/mfma_peak.cpp -o tools/mfma_peak && tools/mfma_peak
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int CHAINS>
__global__ __launch_bounds__(512) void mfma_loop(float* out, int iters, float a, float b) {
  f32x16 acc[CHAINS];
#pragma unroll
  for (int c = 0; c < CHAINS; ++c)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[c][i] = 0.f;
  const float x = a + threadIdx.x * 1e-7f, y = b - threadIdx.x * 1e-7f;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) acc[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(x, y, acc[c], 0, 0, 0);
  }
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < CHAINS; ++c)
#pragma unroll
    for (int i = 0; i < 16; ++i) s += acc[c][i];
  if (s == 12345.f) out[0] = s;   // keep the chains alive
}

int main() {
  float* out;
  hipMalloc(&out, 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const int iters = 4000;
  for (int waves : {4, 8}) {
    const int blocks = cus * 2;
    for (int rep = 0; rep < 2; ++rep) {
      hipEventRecord(e0);
      hipLaunchKernelGGL(mfma_loop<4>, dim3(blocks), dim3(64 * waves), 0, 0, out, iters, 1.f, 2.f);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0.f;
      hipEventElapsedTime(&ms, e0, e1);
      const double flops = (double)blocks * waves * iters * 4 * (2.0 * 32 * 32 * 2);
      if (rep == 1)
        printf("f32 32x32x2 MFMA, %d CUs, %d blocks x %d waves, 4 chains/wave: %.2f ms  %.1f TF/s  (%.3f of 157.3)\n",
               cus, blocks, waves, ms, flops / (ms * 1e-3) / 1e12, flops / (ms * 1e-3) / 1e12 / 157.3);
    }
  }
  return 0;
}

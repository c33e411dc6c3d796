// Diagnostic: device time of fx_gemm against K at fixed M x N (HIP events over back-to-back launches),
// to split a kernel's time into a fixed per-launch part and a per-64-deep-stage part.  Not part of the
// product.
//   hipcc --offload-arch=gfx950 -O2 -I include tools/gemm_sweep.cpp -Lfact-clip_amd/factmx/_lib -lfactmx \
//     -o tools/gemm_sweep && LD_LIBRARY_PATH=fact-clip_amd/factmx/_lib tools/gemm_sweep
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "factmx.h"

static float* dalloc(size_t n) {
  std::vector<float> h(n);
  for (size_t i = 0; i < n; ++i) h[i] = (float)rand() / RAND_MAX - 0.5f;
  float* d = nullptr;
  if (hipMalloc(&d, n * sizeof(float)) != hipSuccess) return nullptr;
  if (hipMemcpy(d, h.data(), n * sizeof(float), hipMemcpyHostToDevice) != hipSuccess) return nullptr;
  return d;
}

static double run(int M, int N, int K, const float* a, const float* b, float* c, int conv) {
  fx_gemm_desc d{};
  d.M = M; d.N = N; d.K = K; d.batch = 1; d.alpha = 1.f; d.split_k = 1;
  d.a.ptr = a; d.a.ld = conv ? K / 3 : K; d.a.conv_dir = 1;
  if (conv) { d.a.conv_taps = 3; d.a.conv_cin = K / 3; d.a.conv_dil = 4; d.a.seq_len = 4096; }
  d.b.ptr = b; d.b.ld = K; d.b.conv_dir = 1;
  d.c = c; d.ldc = N;
  if (fx_gemm(&d, nullptr)) { printf("error %s\n", fx_last_error()); return -1; }
  for (int i = 0; i < 5; ++i) (void)fx_gemm(&d, nullptr);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipDeviceSynchronize();
  const int it = 100;
  (void)hipEventRecord(e0, 0);
  for (int i = 0; i < it; ++i) (void)fx_gemm(&d, nullptr);
  (void)hipEventRecord(e1, 0);
  (void)hipEventSynchronize(e1);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, e0, e1);
  return ms * 1e3 / it;
}

int main() {
  const int M = 8192, N = 256, KMAX = 3072;
  float* a = dalloc((size_t)M * KMAX);
  float* b = dalloc((size_t)N * KMAX);
  float* c = dalloc((size_t)M * N);
  if (!a || !b || !c) return 1;
  for (int prec = 0; prec < 2; ++prec) {
  fx_set_stream_precision(nullptr, prec);
  printf("-- precision %s\n", prec ? "bf16" : "fp32");
  for (int conv = 0; conv < 2; ++conv) {
    for (int K : {192, 384, 768, 1536, 3072}) {
      if (!conv && K % 64) continue;
      const double us = run(M, N, K, a, b, c, conv);
      printf("%s M=%d N=%d K=%5d  %8.2f us  %7.1f TF/s\n", conv ? "conv(3 taps)" : "rows x rows ", M, N, K, us,
             2.0 * M * N * K / us / 1e6);
    }
  }
  }
  fx_set_stream_precision(nullptr, 0);
  for (int K : {256, 768}) {
    const double us = run(4096, N, K, a, b, c, 0);
    printf("rows x rows  M=4096 N=%d K=%5d  %8.2f us  %7.1f TF/s\n", N, K, us, 2.0 * 4096 * N * K / us / 1e6);
  }
  return 0;
}

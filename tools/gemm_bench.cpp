// gemm_bench — times phx::launch_gemm / launch_gemm_dgrad on the EfficientDet-D0 1x1-conv shapes
// and checks each result against a naive fp32 GEMM.  Build: make -C tools ; run on the GPU box.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../mladversarialobjectdetection_amd/csrc/kernels.hpp"

using namespace phx;

__global__ void k_ref(const float* A, const float* Bt, const float* bias, float* C, int M, int N, int K) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)M * N) return;
  int m = i / N, n = i % N;
  double s = bias ? bias[n] : 0.0;
  for (int k = 0; k < K; ++k) s += (double)A[(long)m * K + k] * Bt[(long)n * K + k];
  C[i] = (float)s;
}

static void fill(float* d, size_t n, unsigned seed) {
  std::vector<float> h(n);
  srand(seed);
  for (auto& v : h) v = (float)rand() / RAND_MAX * 2.f - 1.f;
  hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice);
}

int main(int argc, char** argv) {
  struct S { int M, N, K; bool bias; bool stats; };
  std::vector<S> shapes = {
      {1048576, 96, 16, false, true},  {1048576, 16, 96, false, false}, {1048576, 16, 32, false, true},
      {262144, 144, 24, false, true},  {262144, 24, 144, false, true},  {65536, 810, 64, true, false},
      {65536, 64, 64, true, true},     {16384, 672, 112, false, true},  {16384, 112, 672, false, true},
      {4096, 1152, 192, false, true},  {4096, 192, 1152, false, true},  {16384, 64, 64, true, true},
      {4096, 64, 64, true, true},      {4096, 320, 1152, false, true}};
  size_t maxA = 0, maxB = 0, maxC = 0, maxP = 0;
  for (auto& s : shapes) {
    maxA = std::max(maxA, (size_t)s.M * s.K);
    maxB = std::max(maxB, (size_t)s.N * s.K);
    maxC = std::max(maxC, (size_t)s.M * s.N);
    maxP = std::max(maxP, gemm_partial_floats(s.M, s.N, s.K));
  }
  float *A, *Bt, *bias, *C, *R, *part;
  float2* sp;
  float* sc;
  hipMalloc(&A, maxA * 4); hipMalloc(&Bt, maxB * 4); hipMalloc(&bias, 4096 * 4);
  hipMalloc(&C, maxC * 4); hipMalloc(&R, maxC * 4); hipMalloc(&part, std::max<size_t>(1, maxP) * 4);
  hipMalloc(&sp, (size_t)1 << 26); hipMalloc(&sc, (size_t)1 << 22);
  fill(A, maxA, 1); fill(Bt, maxB, 2); fill(bias, 4096, 3);
  hipStream_t st;
  hipStreamCreate(&st);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  double tot_us = 0, tot_roof = 0, tot1 = 0;
  const int wgs = argc > 1 ? atoi(argv[1]) : 1024;
  for (auto& s : shapes) {
    InX ax{A, nullptr, nullptr, nullptr, 0};
    StatSink sink = s.stats ? StatSink{sp, sc, s.N, 0} : StatSink{};
    int impl = 1;
    auto run = [&]() {
      if (impl == 1)
        gemm1_run(0, ax, GradX{}, Bt, s.bias ? bias : nullptr, C, s.M, s.N, s.K, false, nullptr, 1, st, part, sink);
      else
        gemm2_run(0, ax, GradX{}, Bt, s.bias ? bias : nullptr, C, s.M, s.N, s.K, false, nullptr, 1, st, part, sink,
                  wgs);
    };
    for (impl = 1; impl <= 2; ++impl) {
    run();
    hipLaunchKernelGGL(k_ref, dim3(((long)s.M * s.N + 255) / 256), dim3(256), 0, st, A, Bt, s.bias ? bias : nullptr,
                       R, s.M, s.N, s.K);
    hipStreamSynchronize(st);
    std::vector<float> hc((size_t)s.M * s.N), hr(hc.size());
    hipMemcpy(hc.data(), C, hc.size() * 4, hipMemcpyDeviceToHost);
    hipMemcpy(hr.data(), R, hr.size() * 4, hipMemcpyDeviceToHost);
    double maxerr = 0;
    for (size_t i = 0; i < hc.size(); ++i) maxerr = std::max(maxerr, (double)std::fabs(hc[i] - hr[i]));
    const int it = 20;
    for (int i = 0; i < 3; ++i) run();
    hipEventRecord(e0, st);
    for (int i = 0; i < it; ++i) run();
    hipEventRecord(e1, st);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double us = ms * 1e3 / it;
    const double by = 4.0 * ((double)s.M * s.K + (double)s.M * s.N + (double)s.N * s.K);
    const double fl = 2.0 * s.M * s.N * s.K;
    const double roof = std::max(by / 8e12, fl / 157.3e12) * 1e6;
    if (impl == 2) {
      tot_us += us;
      tot_roof += roof;
    }
    GemmPlan p = plan_gemm(s.M, s.N, s.K);
    Gemm2Plan q = plan_gemm2(s.M, s.N, s.K, wgs);
    if (impl == 1) { tot1 += us; }
    printf("impl%d M=%8d N=%5d K=%5d stats=%d  %8.1f us  %6.0f GB/s  %6.1f TF/s  roof %6.1f us (%4.0f%%)  grid=%dx%dx%d  err=%.2e\n",
           impl, s.M, s.N, s.K, (int)s.stats, us, by / us * 1e-3, fl / us * 1e-6, roof, 100 * roof / us,
           impl == 1 ? p.gx : q.gx, impl == 1 ? p.gy : q.gy, impl == 1 ? p.splits : q.splits, maxerr);
    }
  }
  printf("impl1 total %.1f us; impl2 total %.1f us, roofline %.1f us (%.0f%%)\n", tot1, tot_us, tot_roof,
         100 * tot_roof / tot_us);
  return 0;
}

// sep_probe — times phx::launch_sep_fwd (the fused separable conv) against the two-launch path it
// replaces (launch_dw_fwd / launch_dw_fwd_fused + launch_gemm) on the EfficientDet-D0 BiFPN / head
// level shapes, each alone on the device (events around 50 back-to-back launches), and checks the
// fused output against the unfused one.  Build: make -C tools sep_probe ; run on the GPU box.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../mladversarialobjectdetection_amd/csrc/kernels.hpp"

using namespace phx;

static void fill(float* d, size_t n, unsigned seed, float lo, float hi) {
  std::vector<float> h(n);
  srand(seed);
  for (auto& v : h) v = lo + (hi - lo) * ((float)rand() / RAND_MAX);
  (void)hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice);
}

__global__ void k_empty(float* p) {
  if (p && threadIdx.x == 1000) p[0] = 0.f;
}

template <class F>
static float time_us(F f, int reps = 50) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (int i = 0; i < 5; ++i) f();
  (void)hipEventRecord(a, 0);
  for (int i = 0; i < reps; ++i) f();
  (void)hipEventRecord(b, 0);
  (void)hipEventSynchronize(b);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, a, b);
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  return 1e3f * ms / reps;
}

int main() {
  const int B = 16, C = 64, N = 64;
  const int sizes[] = {64, 32, 16, 8, 4};
  const long maxe = (long)B * 64 * 64 * C;
  float *x0, *x1, *y1, *y2, *tmp, *wd, *bt, *bias, *mu, *sc, *be, *ws0, *ws1, *part, *cnt, *gpart;
  (void)hipMalloc(&x0, maxe * 4);
  (void)hipMalloc(&x1, maxe * 4);
  (void)hipMalloc(&y1, maxe * 4);
  (void)hipMalloc(&y2, maxe * 4);
  (void)hipMalloc(&tmp, maxe * 4);
  (void)hipMalloc(&wd, 9 * C * 4);
  (void)hipMalloc(&bt, N * C * 4);
  (void)hipMalloc(&bias, N * 4);
  (void)hipMalloc(&mu, C * 4);
  (void)hipMalloc(&sc, C * 4);
  (void)hipMalloc(&be, C * 4);
  (void)hipMalloc(&ws0, 4);
  (void)hipMalloc(&ws1, 4);
  (void)hipMalloc(&part, (size_t)1 << 24);
  (void)hipMalloc(&cnt, (size_t)1 << 20);
  (void)hipMalloc(&gpart, (size_t)1 << 26);
  fill(x0, maxe, 1, -1.f, 1.f);
  fill(x1, maxe, 2, -1.f, 1.f);
  fill(wd, 9 * C, 3, -0.5f, 0.5f);
  fill(bt, N * C, 4, -0.2f, 0.2f);
  fill(bias, N, 5, -0.1f, 0.1f);
  fill(mu, C, 6, -0.1f, 0.1f);
  fill(sc, C, 7, 0.5f, 1.5f);
  fill(be, C, 8, -0.1f, 0.1f);
  fill(ws0, 1, 9, 0.5f, 1.f);
  fill(ws1, 1, 10, 0.5f, 1.f);
  // the pointwise kernel in HWIO [C][N] for launch_gemm's Bt = [N][C] (bt is already [N][C])
  printf("empty kernel: %.2f us\n", time_us([&] { hipLaunchKernelGGL(k_empty, dim3(16), dim3(256), 0, 0, nullptr); }));
  for (int fuse = 0; fuse < 2; ++fuse)
    for (int S : sizes) {
      const InX xv{x0, mu, sc, be, 1, 0};
      FuseView fv{};
      fv.nin = 2;
      fv.x[0] = InX{x0, mu, sc, be, 0, 0};
      fv.x[1] = InX{x1, nullptr, nullptr, nullptr, 0, 0};
      fv.w[0] = ws0;
      fv.w[1] = ws1;
      fv.method = 0;
      fv.act = 1;
      const int M = B * S * S;
      SepMember m{};
      m.x = xv;
      m.f = fv;
      m.fuse = fuse != 0;
      m.y = y1;
      m.H = S;
      m.W = S;
      const int P = sep_stat_partials(B, S, S);
      m.sink = StatSink{reinterpret_cast<float2*>(part), cnt, N, P};
      int nps[kMaxSeg];
      const float t_sep = time_us([&] { launch_sep_fwd(&m, 1, B, C, N, wd, bt, bias, 0, nps); });
      m.sink = StatSink{};
      const float t_sep0 = time_us([&] { launch_sep_fwd(&m, 1, B, C, N, wd, bt, bias, 0, nps); });
      // the two-launch path
      const int pg = gemm_stat_partials(M, N, C);
      StatSink gs{reinterpret_cast<float2*>(part), cnt, N, pg};
      auto two = [&] {
        if (fuse) launch_dw_fwd_fused(fv, wd, tmp, B, S, S, C, S, S, 3, 1, 1, 1, 0);
        else launch_dw_fwd(xv, wd, tmp, B, S, S, C, S, S, 3, 1, 1, 1, 0);
        launch_gemm(InX{tmp, nullptr, nullptr, nullptr, 0, 0}, bt, bias, y2, M, N, C, false, nullptr, 1, 0, gpart, gs);
      };
      const float t_two = time_us(two);
      const float t_dw = time_us([&] {
        if (fuse) launch_dw_fwd_fused(fv, wd, tmp, B, S, S, C, S, S, 3, 1, 1, 1, 0);
        else launch_dw_fwd(xv, wd, tmp, B, S, S, C, S, S, 3, 1, 1, 1, 0);
      });
      // check
      m.y = y1;
      launch_sep_fwd(&m, 1, B, C, N, wd, bt, bias, 0, nps);
      two();
      (void)hipDeviceSynchronize();
      std::vector<float> a((size_t)M * N), b((size_t)M * N);
      (void)hipMemcpy(a.data(), y1, a.size() * 4, hipMemcpyDeviceToHost);
      (void)hipMemcpy(b.data(), y2, b.size() * 4, hipMemcpyDeviceToHost);
      size_t ndiff = 0;
      double md = 0;
      for (size_t i = 0; i < a.size(); ++i) {
        if (a[i] != b[i]) ++ndiff;
        md = std::max(md, (double)std::fabs(a[i] - b[i]));
      }
      const double mb = 4.0 * ((double)M * C * (fuse ? 2 : 1) + (double)M * N) / 1e6;
      printf("%s %2dx%2d: sep %7.2f us (no stats %7.2f)  two-launch %7.2f us (dw %6.2f)  %6.1f MB -> sep %6.0f GB/s"
             "  diff %zu (max %.2e)\n",
             fuse ? "fuse" : "bn  ", S, S, t_sep, t_sep0, t_two, t_dw, mb, mb * 1e3 / t_sep, ndiff, md);
    }
  return 0;
}

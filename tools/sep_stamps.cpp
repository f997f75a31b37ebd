// sep_stamps — the fused separable conv built with PHX_SEP_STAMPS: per phase, the shader-clock cycles
// wave 0 of the first workgroup spends (tools/Makefile: sep_stamps; run on the GPU box).
#define PHX_SEP_STAMPS 1
#include "../mladversarialobjectdetection_amd/csrc/kernels_sep.hip"

#include <cstdio>
#include <vector>

using namespace phx;

int main() {
  const int B = 16, C = 64, N = 64;
  const long maxe = (long)B * 64 * 64 * C;
  float *x0, *x1, *y, *wd, *bt, *bias, *mu, *sc, *be, *ws, *part, *cnt;
  (void)hipMalloc(&x0, maxe * 4);
  (void)hipMalloc(&x1, maxe * 4);
  (void)hipMalloc(&y, maxe * 4);
  (void)hipMalloc(&wd, 9 * C * 4);
  (void)hipMalloc(&bt, N * C * 4);
  (void)hipMalloc(&bias, N * 4);
  (void)hipMalloc(&mu, C * 4);
  (void)hipMalloc(&sc, C * 4);
  (void)hipMalloc(&be, C * 4);
  (void)hipMalloc(&ws, 8);
  (void)hipMalloc(&part, (size_t)1 << 24);
  (void)hipMalloc(&cnt, (size_t)1 << 20);
  (void)hipMemset(x0, 0, maxe * 4);
  (void)hipMemset(x1, 0, maxe * 4);
  (void)hipMemset(wd, 0, 9 * C * 4);
  (void)hipMemset(bt, 0, N * C * 4);
  (void)hipMemset(bias, 0, N * 4);
  (void)hipMemset(mu, 0, C * 4);
  (void)hipMemset(sc, 0, C * 4);
  (void)hipMemset(be, 0, C * 4);
  (void)hipMemset(ws, 0, 8);
  const char* names[] = {"entry", "staged", "sync1", "dw", "B+sync", "mfma", "epilogue", "stats-sync", "end"};
  for (int fuse = 0; fuse < 2; ++fuse)
    for (int S : {64, 16, 4}) {
      SepMember m{};
      m.x = InX{x0, mu, sc, be, 1, 0};
      m.f.nin = 2;
      m.f.x[0] = InX{x0, mu, sc, be, 0, 0};
      m.f.x[1] = InX{x1, nullptr, nullptr, nullptr, 0, 0};
      m.f.w[0] = ws;
      m.f.w[1] = ws + 1;
      m.f.method = 0;
      m.f.act = 1;
      m.fuse = fuse != 0;
      m.y = y;
      m.H = m.W = S;
      m.sink = StatSink{reinterpret_cast<float2*>(part), cnt, N, sep_stat_partials(B, S, S)};
      int nps[kMaxSeg];
      for (int r = 0; r < 5; ++r) launch_sep_fwd(&m, 1, B, C, N, wd, bt, bias, 0, nps);
      (void)hipDeviceSynchronize();
      unsigned long long st[16];
      (void)hipMemcpyFromSymbol(st, HIP_SYMBOL(sep_stamps), sizeof st);
      printf("%s %2dx%2d:", fuse ? "fuse" : "bn  ", S, S);
      for (int k = 1; k <= 8; ++k) printf("  %s %llu", names[k], st[k] - st[k - 1]);
      printf("  total %llu cycles\n", st[8] - st[0]);
    }
  return 0;
}

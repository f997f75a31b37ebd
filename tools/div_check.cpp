// div_check — GPU check that phx::div_surv (common.hpp: the drop-connect division without
// v_div_fmas) equals IEEE float division n / d bit for bit: 2^26 random numerators per denominator
// (magnitudes 2^-110 .. 2^110, both signs, zeros) for the survival probabilities of D1-D7 and random
// d in (0.5, 1].  Build: make -C tools div_check; run on a GPU: ./tools/div_check
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../mladversarialobjectdetection_amd/csrc/common.hpp"

__global__ void k_check(const float* ds, int nd, unsigned long long n, unsigned long long seed,
                        unsigned long long* bad, float* example) {
  const unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  unsigned long long x = (i + 1) * 0x9e3779b97f4a7c15ull ^ seed;
  x ^= x >> 31; x *= 0xbf58476d1ce4e5b9ull; x ^= x >> 29;
  const unsigned e = 127 - 110 + (unsigned)((x >> 8) % 221);  // exponent 2^-110 .. 2^110
  unsigned bits = ((unsigned)x & 0x807fffffu) | (e << 23);
  if ((x >> 40) % 997 == 0) bits &= 0x80000000u;                  // signed zeros
  const float num = __uint_as_float(bits);
  const float d = ds[(x >> 20) % nd];
  const float a = phx::div_surv(num, d), b = num / d;
  if (__float_as_uint(a) != __float_as_uint(b)) {
    const unsigned long long k = atomicAdd(bad, 1ull);
    if (k == 0) { example[0] = num; example[1] = d; example[2] = a; example[3] = b; }
  }
}

int main() {
  std::vector<float> ds;
  for (int n : {16, 23, 32, 39, 45, 55, 64}) for (int b = 0; b < n; ++b) ds.push_back(1.f - 0.2f * (float)b / (float)n);
  srand(7);
  for (int k = 0; k < 256; ++k) ds.push_back(0.5f + 0.5f * (float)rand() / (float)RAND_MAX);
  float *dd, *ex;
  unsigned long long* bad;
  hipMalloc(&dd, ds.size() * 4);
  hipMalloc(&ex, 16);
  hipMalloc(&bad, 8);
  hipMemcpy(dd, ds.data(), ds.size() * 4, hipMemcpyHostToDevice);
  hipMemset(bad, 0, 8);
  const unsigned long long n = 1ull << 30;
  for (int r = 0; r < 4; ++r)
    hipLaunchKernelGGL(k_check, dim3((unsigned)(n / 256)), dim3(256), 0, 0, dd, (int)ds.size(), n, 1234ull + r, bad, ex);
  unsigned long long hb = 0;
  float he[4] = {0, 0, 0, 0};
  hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost);
  hipMemcpy(he, ex, 16, hipMemcpyDeviceToHost);
  printf("div_surv vs n / d: %llu mismatches in %llu pairs (%zu denominators)\n", hb, 4 * n, ds.size());
  if (hb) printf("  e.g. %a / %a: %a vs %a\n", he[0], he[1], he[2], he[3]);
  return hb ? 1 : 0;
}

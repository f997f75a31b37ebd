// mfma_probe — does VALU work issue beside v_mfma_f32_32x32x2_f32 on one SIMD, or does it add to the
// MFMA time?  One workgroup of 4 waves per CU (one wave per SIMD) or 8 (two per SIMD) runs a loop of
// 16 MFMAs (four independent accumulators) plus V dependent-free VALU ops (exp / fma mix, the cost of
// a BN + swish view element) per iteration; cycles per iteration vs V tells whether they overlap.
// Also the bf16 32x32x16 form for comparison.  Build: hipcc --offload-arch=gfx950 -O3 -o mfma_probe mfma_probe.cpp
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));

template <int V, bool BF>
__global__ __launch_bounds__(512) void k_probe(float* out, int iters, long long* cyc) {
  floatx16 acc[4];
  for (int i = 0; i < 4; ++i)
    for (int e = 0; e < 16; ++e) acc[i][e] = 0.f;
  float a = threadIdx.x * 1e-3f, b = 1.0f + threadIdx.x * 1e-4f;
  bf16x8_t fa, fb;
  for (int e = 0; e < 8; ++e) {
    fa[e] = (__bf16)(a + e);
    fb[e] = (__bf16)(b - e);
  }
  float v[8];
  for (int j = 0; j < 8; ++j) v[j] = a + j * 0.01f;
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if constexpr (BF)
          acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa, fb, acc[i], 0, 0, 0);
        else
          acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[i], 0, 0, 0);
      }
#pragma unroll
      for (int k = 0; k < V / 4; ++k) {
        const int j = k & 7;
        // the per-element work of a BN + swish view: (x - mu) * sc + be, then x * sigmoid(x)
        float z = fmaf(v[j] - 0.1f, 1.01f, 0.02f);
        v[j] = z * __builtin_amdgcn_rcpf(1.0f + __expf(-z));
      }
    }
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
  for (int i = 0; i < 4; ++i)
    for (int e = 0; e < 16; ++e) s += acc[i][e];
  for (int j = 0; j < 8; ++j) s += v[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int V, bool BF>
static void run(int threads, float* out, long long* cyc) {
  const int iters = 2000;
  hipLaunchKernelGGL((k_probe<V, BF>), dim3(256), dim3(threads), 0, 0, out, iters, cyc);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL((k_probe<V, BF>), dim3(256), dim3(threads), 0, 0, out, iters, cyc);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  long long h[256];
  hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
  long long mx = 0;
  for (int i = 0; i < 256; ++i) mx = h[i] > mx ? h[i] : mx;
  const double mfma_per_iter = 16.0;
  // s_memtime ticks at the shader clock; report ticks per MFMA of one wave
  printf("%s waves/SIMD=%d VALU-elements/iter=%3d: %.3f ms, %.1f memtime ticks per MFMA (per wave)\n",
         BF ? "bf16 32x32x16" : "f32 32x32x2 ", threads / 256, V, ms, (double)mx / iters / mfma_per_iter);
}

int main() {
  float* out;
  long long* cyc;
  hipMalloc(&out, 256 * 512 * 4);
  hipMalloc(&cyc, 256 * 8);
  for (int threads : {256, 512}) {
    run<0, false>(threads, out, cyc);
    run<8, false>(threads, out, cyc);
    run<16, false>(threads, out, cyc);
    run<32, false>(threads, out, cyc);
    run<64, false>(threads, out, cyc);
    run<0, true>(threads, out, cyc);
    run<8, true>(threads, out, cyc);
    run<16, true>(threads, out, cyc);
    run<32, true>(threads, out, cyc);
  }
  return 0;
}

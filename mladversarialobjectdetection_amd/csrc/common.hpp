// common.hpp — shared device helpers for the phx HIP kernels (gfx950 / CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <stdexcept>
#include <string>

namespace phx {

struct HipError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

#define PHX_HIP(expr)                                                                  \
  do {                                                                                 \
    hipError_t e_ = (expr);                                                            \
    if (e_ != hipSuccess)                                                              \
      throw ::phx::HipError(std::string(#expr) + ": " + hipGetErrorString(e_) + " @" + \
                            __FILE__ + ":" + std::to_string(__LINE__));                \
  } while (0)

#define PHX_LAUNCH_CHECK() PHX_HIP(hipGetLastError())

constexpr int kWave = 64;

inline int cdiv(long a, long b) { return (int)((a + b - 1) / b); }

// ------------------------------------------------------------------------------------------
// activations (utils.py:36-53).  swish = x*sigmoid(x) (tf.nn.swish); relu6 grad passes on
// the open interval (0,6) (TF Relu6Grad).
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + __expf(-x)); }

__device__ __forceinline__ float act_fwd(float z, int act) {
  if (act == 1) return z * sigmoidf_(z);
  if (act == 2) return fminf(fmaxf(z, 0.0f), 6.0f);
  return z;
}
// d act / d z
__device__ __forceinline__ float act_grad(float z, int act) {
  if (act == 1) {
    float s = sigmoidf_(z);
    return s * (1.0f + z * (1.0f - s));
  }
  if (act == 2) return (z > 0.0f && z < 6.0f) ? 1.0f : 0.0f;
  return 1.0f;
}

// ------------------------------------------------------------------------------------------
// Philox4x32-10 (Salmon et al., SC'11), counter-based: identical draws for a given
// (key, counter) on any device / GPU count.  Matches oracle/philox.py bit for bit.
// ------------------------------------------------------------------------------------------
struct u32x4 {
  uint32_t x, y, z, w;
};

__host__ __device__ inline u32x4 philox4x32_10(u32x4 c, uint32_t k0, uint32_t k1) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint64_t p0 = (uint64_t)M0 * c.x;
    uint64_t p1 = (uint64_t)M1 * c.z;
    uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    c = u32x4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
    k0 += W0;
    k1 += W1;
  }
  return c;
}

// [0,1) with 24 random bits (exact in fp32)
__host__ __device__ inline float u01(uint32_t v) { return (float)(v >> 8) * (1.0f / 16777216.0f); }
// (0,1]
__host__ __device__ inline float u01_open0(uint32_t v) {
  return (float)((v >> 8) + 1u) * (1.0f / 16777216.0f);
}

// RNG streams (counter word w = step << 8 | stream)
enum RngStream : uint32_t {
  RNG_PRINT = 1,      // per image: print-variation w[3], b[3] (attacker.py:365-372)
  RNG_PLACE = 2,      // per box: centre jitter (attacker.py:474-475)
  RNG_BOX = 3,        // per box: brightness delta, angle (attacker.py:427, 436)
  RNG_NOISE = 4,      // per box element: U(-.01,.01) noise (attacker.py:426)
};

}  // namespace phx

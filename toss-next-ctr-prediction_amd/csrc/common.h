// Shared device/host helpers for the gfx950 CTR hot-path kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cmath>
#include <cstdio>
#include <string>

namespace ctr {

// ----------------------------------------------------------------------------------------------
// error plumbing: every extern "C" entry returns 0 / negative and records a thread-local message
// ----------------------------------------------------------------------------------------------
void set_error(const std::string& msg);
int check_launch(const char* what);

#define CTR_REQUIRE(cond, msg)                        \
  do {                                                \
    if (!(cond)) {                                    \
      ::ctr::set_error(std::string(__func__) + ": " + (msg)); \
      return -1;                                      \
    }                                                 \
  } while (0)

constexpr int WAVE = 64;

// ----------------------------------------------------------------------------------------------
// dropout RNG: counter-based, identical to oracle/rng.py (lowbias32 finaliser)
//   key  = per (step seed, site), computed on the host (tossctr/rng.py)
//   bits = mix32(idx ^ key);  keep = (bits >> 8) >= thresh24   (one lowbias32 round per element: the
//   key is already a mixed per-(step, site) value; 2 quarter-rate integer multiplies per element)
// ----------------------------------------------------------------------------------------------
struct Drop {
  uint32_t key;
  uint32_t thresh;   // round(p * 2^24); 0 => no dropout
  float scale;       // 1 / (1 - p) in fp32 (reference: bernoulli_(1-p).div_(1-p))
};

__host__ __device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

__device__ __forceinline__ bool drop_keep(const Drop& d, uint32_t idx) {
  uint32_t b = mix32(idx ^ d.key);
  return (b >> 8) >= d.thresh;
}

// x * (mask / (1-p)): the value the reference's dropout produces
__device__ __forceinline__ float drop_apply(const Drop& d, uint32_t idx, float x) {
  if (d.thresh == 0) return x;
  return drop_keep(d, idx) ? x * d.scale : 0.0f;
}

// ----------------------------------------------------------------------------------------------
// reductions
// ----------------------------------------------------------------------------------------------
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// sum over groups of G consecutive lanes (G power of two <= 64)
template <int G>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int o = G / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// deterministic block reduction (fixed tree); `red` must hold blockDim.x/64 floats
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) red[w] = v;
  __syncthreads();
  float s = 0.f;
  const int nw = (blockDim.x + 63) >> 6;
  for (int i = 0; i < nw; ++i) s += red[i];
  return s;
}

// ----------------------------------------------------------------------------------------------
// activations (reference: nn.GELU() exact erf form; torch GeluBackward formula)
// ----------------------------------------------------------------------------------------------
__device__ __forceinline__ float gelu_f(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f)); }

__device__ __forceinline__ float gelu_grad(float x) {
  const float cdf = 0.5f * (1.0f + erff(x * 0.70710678118654752f));
  const float pdf = expf(-0.5f * x * x) * 0.39894228040143268f;
  return cdf + x * pdf;
}

__device__ __forceinline__ float softplus_f(float x) {  // torch F.softplus(beta=1, threshold=20)
  return x > 20.f ? x : log1pf(expf(x));
}

__device__ __forceinline__ float sigmoid_f(float x) { return 1.0f / (1.0f + expf(-x)); }

__host__ __device__ inline int cdiv(long a, long b) { return (int)((a + b - 1) / b); }

}  // namespace ctr

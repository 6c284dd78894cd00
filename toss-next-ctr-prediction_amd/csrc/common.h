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
//   bits = mix32((idx >> 1) ^ key);  u = idx odd ? bits >> 16 : bits & 0xFFFF;  keep = u >= thresh16
// One lowbias32 round (2 quarter-rate integer multiplies) serves the element pair (2k, 2k+1): the
// kernels that hold both elements of a pair (attention rows, the FFN forward via a lane swap) hash
// once per pair.  p resolves to 2^-16 (thresh16 = round(p * 65536), at least 1 for p > 0).
// ----------------------------------------------------------------------------------------------
struct Drop {
  uint32_t key;
  uint32_t thresh;   // round(p * 2^16); 0 => no dropout
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
  const uint32_t b = mix32((idx >> 1) ^ d.key);
  return ((idx & 1u) ? b >> 16 : b & 0xFFFFu) >= d.thresh;
}

// the pair hash of elements 2k, 2k+1 (bits: drop_pair_keep)
__device__ __forceinline__ uint32_t drop_pair_bits(const Drop& d, uint32_t pair) { return mix32(pair ^ d.key); }
__device__ __forceinline__ bool drop_pair_keep(const Drop& d, uint32_t bits, uint32_t odd) {
  return (odd ? bits >> 16 : bits & 0xFFFFu) >= d.thresh;
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

// Raw buffer access (buffer_load / buffer_store with a 128-bit resource in SGPRs): the per-lane part of
// the address is a 32-bit VGPR byte offset, a wave-uniform part can ride in `soff` (an SGPR), and
// accesses whose VGPR offset (+ immediate) is >= `bytes` read 0 / are dropped -- bounds checks without
// branches, which keeps the compiler's vmcnt bookkeeping exact across a software-pipelined loop.
// `soff` is not range-checked: only wave-uniform, in-range offsets go there.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ float buf_ld(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff = 0) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0));
}
__device__ __forceinline__ uint32_t buf_ld_u16(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff = 0) {
  return (uint32_t)__builtin_amdgcn_raw_buffer_load_b16(r, voff, soff, 0);
}
__device__ __forceinline__ void buf_st(float v, __amdgpu_buffer_rsrc_t r, uint32_t voff) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), r, voff, 0, 0);
}
__device__ __forceinline__ void buf_st_u16(uint32_t v, __amdgpu_buffer_rsrc_t r, uint32_t voff) {
  __builtin_amdgcn_raw_buffer_store_b16((unsigned short)v, r, voff, 0, 0);
}
__device__ __forceinline__ void buf_st_u8(uint32_t v, __amdgpu_buffer_rsrc_t r, uint32_t voff) {
  __builtin_amdgcn_raw_buffer_store_b8((unsigned char)v, r, voff, 0, 0);
}
constexpr uint32_t BUF_OOB = 0x80000000u;   // a VGPR offset past any resource: load 0 / drop the store

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
// Phi(z) = 0.5 (1 + erf(z / sqrt2)) without a branch: erfc(x) = t exp(-x^2 + P(t)), t = 1 / (1 + x/2),
// x = |z| / sqrt2, P the 9th-degree Chebyshev fit (relative error < 1.2e-7 on erfc for all x >= 0);
// Phi = erfc/2 below 0 and 1 - erfc/2 above.  ocml's erff takes two divergent polynomial paths per
// wave (|x| < 1 and >= 1) -- both run -- and cancels in the lower tail; this is one path, ~16 VALU ops.
// Max relative error of Phi in fp32 over [-12, 12]: 2.3e-5 at the far tail, 3.4e-6 on z > -5 (erff's
// 1 + erf form: 4.8e-2 there), tests/test_gpu_kernels.py checks it against torch's fp64 GELU.
__device__ __forceinline__ float norm_cdf(float z) {
  const float x = fabsf(z) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.5f, x, 1.0f));
  float p = 0.17087277f;
  p = fmaf(p, t, -0.82215223f);
  p = fmaf(p, t, 1.48851587f);
  p = fmaf(p, t, -1.13520398f);
  p = fmaf(p, t, 0.27886807f);
  p = fmaf(p, t, -0.18628806f);
  p = fmaf(p, t, 0.09678418f);
  p = fmaf(p, t, 0.37409196f);
  p = fmaf(p, t, 1.00002368f);
  p = fmaf(p, t, -1.26551223f);
  const float h = 0.5f * t * __builtin_amdgcn_exp2f(fmaf(-x, x, p) * 1.44269504088896341f);
  return z < 0.f ? h : 1.0f - h;
}

__device__ __forceinline__ float gelu_f(float x) { return x * norm_cdf(x); }

__device__ __forceinline__ float gelu_grad(float x) {
  const float pdf = __builtin_amdgcn_exp2f(-0.72134752044448170f * x * x) * 0.39894228040143268f;
  return fmaf(x, pdf, norm_cdf(x));
}

__device__ __forceinline__ float softplus_f(float x) {  // torch F.softplus(beta=1, threshold=20)
  return x > 20.f ? x : log1pf(expf(x));
}

__device__ __forceinline__ float sigmoid_f(float x) { return 1.0f / (1.0f + expf(-x)); }

__host__ __device__ inline int cdiv(long a, long b) { return (int)((a + b - 1) / b); }

}  // namespace ctr

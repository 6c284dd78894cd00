// Device-wide prefix sum of uint32 words in two launches, no host work: (1) each block of SCAN_CH words writes its
// sum; (2) each block adds the sums of the blocks before it (at most SCAN_FLAT_MAX words, in order), scans its own
// words in LDS and writes them.  Beyond SCAN_FLAT_MAX blocks (n > 2M words) the block sums are first scanned in place
// by one workgroup (scan_prefix_kernel) and each block reads its own prefix: the in-block loop would read nb^2 / 2
// words.  Replaces rocPRIM's lookback scans on the training step's path: their host side queried
// hipGetDeviceProperties at every call (rocprim is_sleep_scan_state_used), which stalled the host's issue of the
// step's other streams.  The sums are exact (integers), so the result equals any other scan's.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace ctr {
namespace {     // per translation unit: the header's kernels are not shared across objects

constexpr int SCAN_T = 256, SCAN_IPT = 8, SCAN_CH = SCAN_T * SCAN_IPT;
constexpr int SCAN_FLAT_MAX = 1024;     // block sums a write block adds itself (<= 4 loads per thread)

__device__ __forceinline__ uint32_t scan_block_sum(uint32_t v, uint32_t* red) {
  for (int o = 32; o >= 1; o >>= 1) v += (uint32_t)__shfl_xor((int)v, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  uint32_t t = 0;
#pragma unroll
  for (int w = 0; w < SCAN_T / 64; ++w) t += red[w];
  __syncthreads();
  return t;
}

__global__ __launch_bounds__(SCAN_T) void scan_bsum_kernel(const uint32_t* __restrict__ in, long n,
                                                           uint32_t* __restrict__ bsum) {
  __shared__ uint32_t red[SCAN_T / 64];
  const long i0 = (long)blockIdx.x * SCAN_CH + (long)threadIdx.x * SCAN_IPT;
  uint32_t v[SCAN_IPT], c = 0;
#pragma unroll
  for (int u = 0; u < SCAN_IPT; ++u) v[u] = i0 + u < n ? in[i0 + u] : 0u;
#pragma unroll
  for (int u = 0; u < SCAN_IPT; ++u) c += v[u];
  const uint32_t t = scan_block_sum(c, red);
  if (threadIdx.x == 0) bsum[blockIdx.x] = t;
}

// in place: w[i] = w[0] + ... + w[i - 1], one workgroup walking the nb words in SCAN_CH chunks with a running carry
__global__ __launch_bounds__(SCAN_T) void scan_prefix_kernel(uint32_t* __restrict__ w, int nb) {
  __shared__ uint32_t sc[SCAN_T];
  uint32_t carry = 0;
  for (int c0 = 0; c0 < nb; c0 += SCAN_CH) {
    const int i0 = c0 + threadIdx.x * SCAN_IPT;
    uint32_t v[SCAN_IPT], c = 0;
#pragma unroll
    for (int u = 0; u < SCAN_IPT; ++u) v[u] = i0 + u < nb ? w[i0 + u] : 0u;
#pragma unroll
    for (int u = 0; u < SCAN_IPT; ++u) c += v[u];
    sc[threadIdx.x] = c;
    __syncthreads();
    for (int o = 1; o < SCAN_T; o <<= 1) {
      const uint32_t x = threadIdx.x >= o ? sc[threadIdx.x - o] : 0u;
      __syncthreads();
      sc[threadIdx.x] += x;
      __syncthreads();
    }
    uint32_t run = carry + sc[threadIdx.x] - c;
#pragma unroll
    for (int u = 0; u < SCAN_IPT; ++u)
      if (i0 + u < nb) {
        w[i0 + u] = run;
        run += v[u];
      }
    carry += sc[SCAN_T - 1];
    __syncthreads();
  }
}

// the prefix of block blockIdx.x: its own entry of the pre-scanned sums, or the sum of the blocks before it
__device__ __forceinline__ uint32_t scan_block_prefix(const uint32_t* __restrict__ bsum, bool prescanned,
                                                      uint32_t* red) {
  if (prescanned) return bsum[blockIdx.x];
  uint32_t pre = 0;
  for (int q = threadIdx.x; q < (int)blockIdx.x; q += SCAN_T) pre += bsum[q];
  return scan_block_sum(pre, red);
}

template <bool INCLUSIVE>
__global__ __launch_bounds__(SCAN_T) void scan_write_kernel(const uint32_t* __restrict__ in, long n,
                                                            const uint32_t* __restrict__ bsum, int prescanned,
                                                            uint32_t* __restrict__ out) {
  __shared__ uint32_t red[SCAN_T / 64];
  __shared__ uint32_t sc[SCAN_T];
  const uint32_t pre = scan_block_prefix(bsum, prescanned != 0, red);
  const long i0 = (long)blockIdx.x * SCAN_CH + (long)threadIdx.x * SCAN_IPT;
  uint32_t v[SCAN_IPT], c = 0;
#pragma unroll
  for (int u = 0; u < SCAN_IPT; ++u) v[u] = i0 + u < n ? in[i0 + u] : 0u;
#pragma unroll
  for (int u = 0; u < SCAN_IPT; ++u) c += v[u];
  sc[threadIdx.x] = c;
  __syncthreads();
  for (int o = 1; o < SCAN_T; o <<= 1) {
    const uint32_t x = threadIdx.x >= o ? sc[threadIdx.x - o] : 0u;
    __syncthreads();
    sc[threadIdx.x] += x;
    __syncthreads();
  }
  uint32_t run = pre + sc[threadIdx.x] - c;
#pragma unroll
  for (int u = 0; u < SCAN_IPT; ++u) {
    if (i0 + u >= n) break;
    if (INCLUSIVE) {
      run += v[u];
      out[i0 + u] = run;
    } else {
      out[i0 + u] = run;
      run += v[u];
    }
  }
}

// scratch words for scan_u32's block sums
inline long scan_ws_words(long n) { return (n + SCAN_CH - 1) / SCAN_CH; }

// out[i] = in[0] + ... + in[i] (inclusive) or in[0] + ... + in[i - 1] (exclusive); in and out may not alias
inline void scan_u32(const uint32_t* in, uint32_t* out, long n, bool inclusive, uint32_t* bsum, hipStream_t s) {
  if (n <= 0) return;
  const int nb = (int)scan_ws_words(n);
  scan_bsum_kernel<<<nb, SCAN_T, 0, s>>>(in, n, bsum);
  const int pre = nb > SCAN_FLAT_MAX;
  if (pre) scan_prefix_kernel<<<1, SCAN_T, 0, s>>>(bsum, nb);
  if (inclusive) scan_write_kernel<true><<<nb, SCAN_T, 0, s>>>(in, n, bsum, pre, out);
  else scan_write_kernel<false><<<nb, SCAN_T, 0, s>>>(in, n, bsum, pre, out);
}

}  // namespace
}  // namespace ctr

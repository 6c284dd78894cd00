// Deterministic row-wise gradient dedup for the embedding tables.
//
// Replaces embedding_dense_backward (index_add of row grads into a zero-filled dense grad, one per
// nn.Embedding: src/models/dare.py:89-90, src/models/wrapper.py:34).  Instead of materialising a
// 10M x D dense grad, contributions (key = row id, value = one grad row) are
//   1. stably radix-sorted by key (rocPRIM, library primitive; stable => members of a key keep
//      their contribution order),
//   2. run-length grouped into (unique key, first index) by two small kernels (rle_count / rle_write),
//   3. summed per unique key by one wave each, in contribution order (bitwise reproducible).
// The optimizer stream (optim.hip) then reads the compact (keys, rows) directly.
// Keys equal to INVALID (0xFFFFFFFF: pad tokens, whose grads padding_idx drops) sort last.
#include <cstring>
#include <rocprim/device/device_radix_sort.hpp>

#include "common.h"
#include "ctr_hip.h"
#include "scan.h"

namespace ctr {

__global__ void iota_kernel(uint32_t* v, int n) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) v[i] = (uint32_t)i;
}

// Run-length groups of the sorted keys without rocPRIM's run_length_encode / exclusive_scan: their lookback scans
// query hipGetDeviceProperties on the host at every call (is_sleep_scan_state_used), which stalled the host's
// issue of the step's other stream for ~0.1 ms per dedupe.  Two passes over RLE_CH-key blocks: (1) each block
// counts its run heads (i == 0 or key[i] != key[i-1]); (2) each block sums the counts of the blocks before it
// (in order; beyond SCAN_FLAT_MAX blocks they are scanned once first, scan.h), scans its threads' head counts in LDS and writes, per run, the unique key and
// its first index; the last block writes n_uniq and offsets[n_uniq] = n, so a run's length is
// offsets[u + 1] - offsets[u].  Deterministic and in key order, as the rocPRIM pair was.
constexpr int RLE_T = SCAN_T, RLE_IPT = SCAN_IPT, RLE_CH = SCAN_CH;     // scan.h's block shape (shared helpers)

__device__ __forceinline__ uint32_t rle_heads(const uint32_t* __restrict__ skeys, int n, int i0, bool (&h)[RLE_IPT]) {
  uint32_t k[RLE_IPT + 1];
  k[0] = i0 > 0 && i0 - 1 < n ? skeys[i0 - 1] : 0u;
#pragma unroll
  for (int u = 0; u < RLE_IPT; ++u) k[u + 1] = skeys[min(i0 + u, n - 1)];
  uint32_t c = 0;
#pragma unroll
  for (int u = 0; u < RLE_IPT; ++u) {
    const int i = i0 + u;
    h[u] = i < n && (i == 0 || k[u + 1] != k[u]);
    c += h[u] ? 1u : 0u;
  }
  return c;
}

__global__ __launch_bounds__(RLE_T) void rle_count_kernel(const uint32_t* __restrict__ skeys, int n,
                                                          uint32_t* __restrict__ bcount) {
  __shared__ uint32_t red[RLE_T / 64];
  bool h[RLE_IPT];
  const uint32_t c = rle_heads(skeys, n, blockIdx.x * RLE_CH + threadIdx.x * RLE_IPT, h);
  const uint32_t t = scan_block_sum(c, red);
  if (threadIdx.x == 0) bcount[blockIdx.x] = t;
}

__global__ __launch_bounds__(RLE_T) void rle_write_kernel(const uint32_t* __restrict__ skeys, int n,
                                                          const uint32_t* __restrict__ bcount, int prescanned,
                                                          uint32_t* __restrict__ uniq_keys,
                                                          uint32_t* __restrict__ offsets,
                                                          uint32_t* __restrict__ n_uniq) {
  __shared__ uint32_t red[RLE_T / 64];
  __shared__ uint32_t sc[RLE_T];
  const uint32_t pre = scan_block_prefix(bcount, prescanned != 0, red);   // the heads of the blocks before this one
  bool h[RLE_IPT];
  const int i0 = blockIdx.x * RLE_CH + threadIdx.x * RLE_IPT;
  const uint32_t c = rle_heads(skeys, n, i0, h);
  sc[threadIdx.x] = c;
  __syncthreads();
  for (int o = 1; o < RLE_T; o <<= 1) {          // inclusive scan of the threads' head counts
    const uint32_t v = threadIdx.x >= o ? sc[threadIdx.x - o] : 0u;
    __syncthreads();
    sc[threadIdx.x] += v;
    __syncthreads();
  }
  uint32_t seg = pre + sc[threadIdx.x] - c;
#pragma unroll
  for (int u = 0; u < RLE_IPT; ++u)
    if (h[u]) {
      uniq_keys[seg] = skeys[i0 + u];
      offsets[seg] = (uint32_t)(i0 + u);
      ++seg;
    }
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == RLE_T - 1) {
    const uint32_t total = pre + sc[RLE_T - 1];
    n_uniq[0] = total;
    offsets[total] = (uint32_t)n;
  }
}

// one wave per SS_KPW consecutive unique keys, lane = column; each key's members summed in (stable) contribution
// order.  The keys' slot loads, their first members' indices and the first members' rows are each issued for all
// SS_KPW keys together (most keys have one member: three dependent round trips per key became three per SS_KPW
// keys); a key with more than SS_CH members continues in chunks of SS_CH.  The sums add in member order exactly
// as one key per wave did.  The INVALID group (pad tokens: dropped by padding_idx) is skipped -- it is by far the
// largest group (every short history contributes pads to its top-K) and its sum is never read.
constexpr int SS_KPW = 4, SS_CH = 4;

template <int NA>
__device__ __forceinline__ void segsum_keys(const float* const (&src)[NA], float* const (&dst)[NA], int ld, int width,
                                            int col, const uint32_t* __restrict__ uniq_keys,
                                            const uint32_t* __restrict__ sorted_idx,
                                            const uint32_t* __restrict__ offsets, const uint32_t* __restrict__ n_uniq,
                                            uint32_t n, uint32_t u0, int a) {
  uint32_t key[SS_KPW], off[SS_KPW], cnt[SS_KPW];
#pragma unroll
  for (int j = 0; j < SS_KPW; ++j) {      // slots past n_uniq read in-bounds workspace words; they are not used
    const uint32_t u = min(u0 + j, n - 1);
    key[j] = uniq_keys[u];
    off[j] = offsets[u];
    cnt[j] = offsets[u + 1];
  }
  const uint32_t nu = *n_uniq;
#pragma unroll
  for (int j = 0; j < SS_KPW; ++j) cnt[j] -= off[j];
  if (col >= width) return;
  bool live[SS_KPW];
  uint32_t ix[SS_KPW][SS_CH];
#pragma unroll
  for (int j = 0; j < SS_KPW; ++j) {
    live[j] = u0 + j < nu && key[j] != 0xFFFFFFFFu;
    const uint32_t c1 = live[j] && cnt[j] > 0 ? cnt[j] - 1 : 0;
#pragma unroll
    for (int q = 0; q < SS_CH; ++q) ix[j][q] = sorted_idx[min(off[j] + min((uint32_t)q, c1), n - 1)];
  }
  float v[SS_KPW][SS_CH];
#pragma unroll
  for (int j = 0; j < SS_KPW; ++j)
#pragma unroll
    for (int q = 0; q < SS_CH; ++q) v[j][q] = src[a][(long)ix[j][q] * ld + col];
#pragma unroll
  for (int j = 0; j < SS_KPW; ++j) {
    const uint32_t u = u0 + j;
    if (u >= nu) break;
    if (!live[j]) {                        // the INVALID group: zero row (never read)
      dst[a][(long)u * width + col] = 0.f;
      continue;
    }
    float acc = 0.f;
#pragma unroll
    for (int q = 0; q < SS_CH; ++q)
      if ((uint32_t)q < cnt[j]) acc += v[j][q];
    for (uint32_t i = SS_CH; i < cnt[j]; i += SS_CH) {      // long groups: further chunks, loads issued together
      float w[SS_CH];
#pragma unroll
      for (int q = 0; q < SS_CH; ++q)
        w[q] = src[a][(long)sorted_idx[off[j] + min(i + q, cnt[j] - 1)] * ld + col];
#pragma unroll
      for (int q = 0; q < SS_CH; ++q)
        if (i + q < cnt[j]) acc += w[q];
    }
    dst[a][(long)u * width + col] = acc;
  }
}

__global__ __launch_bounds__(256) void segsum_kernel(const float* __restrict__ contrib, int ld, int width,
                                                     const uint32_t* __restrict__ uniq_keys,
                                                     const uint32_t* __restrict__ sorted_idx,
                                                     const uint32_t* __restrict__ offsets,
                                                     const uint32_t* __restrict__ n_uniq, uint32_t n,
                                                     float* __restrict__ out) {
  const uint32_t u0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * SS_KPW;
  if (u0 >= n) return;
  const float* const src[1] = {contrib};
  float* const dst[1] = {out};
  segsum_keys<1>(src, dst, ld, width, threadIdx.x & 63, uniq_keys, sorted_idx, offsets, n_uniq, n, u0, 0);
}

// Two contribution arrays sharing the keys (the DARE att / rep rows, width <= 32): lanes [0, 32) sum array a and
// lanes [32, 64) array b -- one set of index loads for both and no idle half-wave.
__global__ __launch_bounds__(256) void segsum2_kernel(const float* __restrict__ ca, const float* __restrict__ cb,
                                                      int ld, int width, const uint32_t* __restrict__ uniq_keys,
                                                      const uint32_t* __restrict__ sorted_idx,
                                                      const uint32_t* __restrict__ offsets,
                                                      const uint32_t* __restrict__ n_uniq, uint32_t n,
                                                      float* __restrict__ oa, float* __restrict__ ob) {
  const uint32_t u0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * SS_KPW;
  if (u0 >= n) return;
  const int lane = threadIdx.x & 63;
  const float* const src[2] = {ca, cb};
  float* const dst[2] = {oa, ob};
  segsum_keys<2>(src, dst, ld, width, lane & 31, uniq_keys, sorted_idx, offsets, n_uniq, n, u0, lane >> 5);
}

struct RowgradWs {
  size_t temp_bytes;
  size_t total;
  size_t off_iota, off_skeys, off_sidx, off_bcount, off_offsets;
};

static size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

// the sort's temporary size depends on n (and the device's arch): the last few (device, n) cached per host thread
// (the step alternates two or three n; ctypes releases the GIL, so two threads may be in here at once)
static RowgradWs rowgrad_layout(int n) {
  thread_local int cached_n[4] = {-1, -1, -1, -1}, cached_dev[4] = {-1, -1, -1, -1};
  thread_local RowgradWs cached[4];
  thread_local int next = 0;
  int dev = 0;
  (void)hipGetDevice(&dev);
  for (int q = 0; q < 4; ++q)
    if (cached_n[q] == n && cached_dev[q] == dev) return cached[q];
  RowgradWs w{};
  size_t t1 = 0;
  (void)rocprim::radix_sort_pairs(nullptr, t1, (const uint32_t*)nullptr, (uint32_t*)nullptr, (const uint32_t*)nullptr,
                                  (uint32_t*)nullptr, (size_t)n, 0, 32);
  w.temp_bytes = align256(t1);
  const size_t a = align256((size_t)n * sizeof(uint32_t));
  w.off_iota = w.temp_bytes;
  w.off_skeys = w.off_iota + a;
  w.off_sidx = w.off_skeys + a;
  w.off_bcount = w.off_sidx + a;
  w.off_offsets = w.off_bcount + align256((size_t)cdiv(n, RLE_CH) * sizeof(uint32_t));
  w.total = w.off_offsets + align256(((size_t)n + 1) * sizeof(uint32_t));
  cached_n[next] = n;
  cached_dev[next] = dev;
  cached[next] = w;
  next = (next + 1) & 3;
  return w;
}

}  // namespace ctr

using namespace ctr;

extern "C" size_t ctr_rowgrad_ws_size(int n) { return n > 0 ? rowgrad_layout(n).total : 0; }

// sort + run-length encode + offsets shared by every contribution array keyed by `keys`
static int rowgrad_core(const uint32_t* keys, const float* const* contrib, float* const* uniq_grad, int ncontrib,
                        int n, int width, int ld, int key_bits, uint32_t* uniq_keys, uint32_t* n_uniq, void* ws,
                        size_t ws_bytes, hipStream_t s) {
  if (n == 0) {
    (void)hipMemsetAsync(n_uniq, 0, sizeof(uint32_t), s);
    return check_launch("rowgrad");
  }
  CTR_REQUIRE(width >= 1 && width <= 64, "row width must be in [1, 64]");
  CTR_REQUIRE(key_bits >= 1 && key_bits <= 32, "key_bits must be in [1, 32]");
  RowgradWs w = rowgrad_layout(n);
  CTR_REQUIRE(ws_bytes >= w.total, "rowgrad workspace too small");
  char* base = (char*)ws;
  uint32_t* iota = (uint32_t*)(base + w.off_iota);
  uint32_t* skeys = (uint32_t*)(base + w.off_skeys);
  uint32_t* sidx = (uint32_t*)(base + w.off_sidx);
  uint32_t* bcount = (uint32_t*)(base + w.off_bcount);
  uint32_t* offsets = (uint32_t*)(base + w.off_offsets);
  iota_kernel<<<std::min(cdiv(n, 256), 4096), 256, 0, s>>>(iota, n);
  size_t tb = w.temp_bytes;
  hipError_t e = rocprim::radix_sort_pairs(base, tb, keys, skeys, (const uint32_t*)iota, sidx, (size_t)n, 0,
                                           (unsigned)key_bits, s);
  CTR_REQUIRE(e == hipSuccess, "radix_sort_pairs failed");
  const int nb = cdiv(n, RLE_CH);
  rle_count_kernel<<<nb, RLE_T, 0, s>>>(skeys, n, bcount);
  const int pre = nb > SCAN_FLAT_MAX;         // > 2M keys: the block counts scanned once (scan.h)
  if (pre) scan_prefix_kernel<<<1, SCAN_T, 0, s>>>(bcount, nb);
  rle_write_kernel<<<nb, RLE_T, 0, s>>>(skeys, n, bcount, pre, uniq_keys, offsets, n_uniq);
  if (ncontrib == 2 && width <= 32)
    segsum2_kernel<<<cdiv(n, 4 * SS_KPW), 256, 0, s>>>(contrib[0], contrib[1], ld, width, uniq_keys, sidx, offsets,
                                                         n_uniq, (uint32_t)n, uniq_grad[0], uniq_grad[1]);
  else
    for (int q = 0; q < ncontrib; ++q)
      segsum_kernel<<<cdiv(n, 4 * SS_KPW), 256, 0, s>>>(contrib[q], ld, width, uniq_keys, sidx, offsets, n_uniq,
                                                          (uint32_t)n, uniq_grad[q]);
  return check_launch("rowgrad");
}

extern "C" int ctr_rowgrad(const uint32_t* keys, const float* contrib, int n, int width, int ld, int key_bits,
                           uint32_t* uniq_keys, float* uniq_grad, uint32_t* n_uniq, void* ws, size_t ws_bytes,
                           void* stream) {
  return rowgrad_core(keys, &contrib, &uniq_grad, 1, n, width, ld, key_bits, uniq_keys, n_uniq, ws, ws_bytes,
                      (hipStream_t)stream);
}

extern "C" int ctr_rowgrad2(const uint32_t* keys, const float* contrib_a, const float* contrib_b, int n, int width,
                            int ld, int key_bits, uint32_t* uniq_keys, float* uniq_a, float* uniq_b, uint32_t* n_uniq,
                            void* ws, size_t ws_bytes, void* stream) {
  const float* c[2] = {contrib_a, contrib_b};
  float* u[2] = {uniq_a, uniq_b};
  return rowgrad_core(keys, c, u, 2, n, width, ld, key_bits, uniq_keys, n_uniq, ws, ws_bytes, (hipStream_t)stream);
}

namespace ctr {
__global__ void scatter_rows_kernel(const uint32_t* __restrict__ keys, const float* __restrict__ G,
                                    const uint32_t* __restrict__ n_uniq, int width, int ld, uint32_t key_base,
                                    long n_rows, float* __restrict__ out) {
  const uint32_t nu = *n_uniq;
  const long total = (long)nu * width;
  for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q < total; q += (long)gridDim.x * blockDim.x) {
    const long u = q / width;
    const int k = (int)(q % width);
    const uint32_t key = keys[u];
    if (key < key_base || (long)(key - key_base) >= n_rows) continue;
    out[(long)(key - key_base) * width + k] = G[u * ld + k];
  }
}
}  // namespace ctr

// compact -> dense table gradient (only for the torch-autograd compatibility path: loss.backward())
extern "C" int ctr_scatter_rows(const uint32_t* keys, const float* G, const uint32_t* n_uniq, int max_uniq, int width,
                                int ld, uint32_t key_base, long n_rows, float* out, void* stream) {
  if (max_uniq == 0) return 0;
  int blocks = std::min(cdiv((long)max_uniq * width, 256), 8192);
  scatter_rows_kernel<<<blocks, 256, 0, (hipStream_t)stream>>>(keys, G, n_uniq, width, ld, key_base, n_rows, out);
  return check_launch("scatter_rows");
}

namespace ctr {
__global__ void mask_tail_keys_kernel(uint32_t* __restrict__ keys, int n, int world, const uint32_t* __restrict__ counts) {
  const long total = (long)n * world;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int r = (int)(i / n);
    if ((uint32_t)(i - (long)r * n) >= counts[r]) keys[i] = 0xFFFFFFFFu;
  }
}
}  // namespace ctr

// data parallel: after all-gathering every rank's compact (keys, rows) buffers (n slots each, the first
// counts[r] valid), invalidate the unused slots so a second ctr_rowgrad merges them across ranks
extern "C" int ctr_mask_tail_keys(uint32_t* keys, int n, int world, const uint32_t* counts, void* stream) {
  if ((long)n * world == 0) return 0;
  int blocks = std::min(cdiv((long)n * world, 256), 8192);
  mask_tail_keys_kernel<<<blocks, 256, 0, (hipStream_t)stream>>>(keys, n, world, counts);
  return check_launch("mask_tail_keys");
}

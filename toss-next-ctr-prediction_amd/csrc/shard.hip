// Row-sharded embedding tables (BASELINE config 5: hash_buckets=1e8, emb_dim=64 --
// 60 B table parameters, more than one GPU's HBM).
//
// Row r of a table lives on rank r % W at local row r / W (hashed ids are uniform, so modulo spreads
// both rows and traffic evenly).  Per step and table group (sequence tokens -> both DARE tables;
// hashed categoricals -> the 35 tables) a rank:
//   1. ctr_shard_plan   -- maps every id of its batch to an owner-major key
//                          okey = owner << lbits | local_key, sorts and deduplicates them, and remaps
//                          the batch to fetched-row ids (1 + position in the sorted unique list; 0 is
//                          the pad token, whose rows padding_idx keeps at zero).  Owner-major order
//                          makes each owner's request one contiguous run: send_counts[w].
//   2. all-to-all of the requested keys (tossctr/shard.py, RCCL), then on the owner:
//      ctr_shard_strip (okey -> local key), ctr_lazy_touch (rows brought current), ctr_shard_gather
//      (rows into the reply buffer), and an all-to-all of the rows back: the requester receives them
//      in exactly its unique-key order, i.e. fetched row u+1 is unique key u.
//   3. backward: the row-grad dedup (rowgrad.hip) runs on fetched-row ids; its rows are scattered to the
//      fetched-row order (ctr_scatter_rows; rows without a gradient stay 0, which AdamW treats exactly as
//      an untouched row), so the grads travel back along the forward's request splits -- no second count
//      exchange -- and the owner's second dedup over the keys it was asked for merges the ranks'
//      contributions in rank order (deterministic) before the optimizer.
// Categorical rows and grads travel at their table's width d_c (ctr_shard_offsets / _pack / _unpack:
// per-key widths, exclusive-scan offsets, per-owner float counts for the exchange's splits), not in the
// 64-float fetched-row layout the forward kernels read.
#include <rocprim/device/device_radix_sort.hpp>

#include "common.h"
#include "scan.h"
#include "ctr_hip.h"

namespace ctr {

constexpr uint32_t SH_INVALID = 0xFFFFFFFFu;

// mode 0 (sequence): okey of token v, INVALID for the pad token
// mode 1 (categorical): X (n / ncols, ncols), column c -> table c with local key base lbase[c]
__global__ void shard_keys_kernel(const int32_t* __restrict__ X, long n, int ncols, int mode, int pad_id,
                                  const uint32_t* __restrict__ lbase, uint32_t world, int lbits,
                                  uint32_t* __restrict__ okeys, uint32_t* __restrict__ iota) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int32_t v = X[i];
    uint32_t k;
    if (mode == 0) {
      k = v == pad_id ? SH_INVALID : (((uint32_t)v % world) << lbits) | ((uint32_t)v / world);
    } else {
      const int c = (int)(i % ncols);
      k = (((uint32_t)v % world) << lbits) | (lbase[c] + (uint32_t)v / world);
    }
    okeys[i] = k;
    iota[i] = (uint32_t)i;
  }
}

__global__ void shard_flags_kernel(const uint32_t* __restrict__ skeys, long n, uint32_t* __restrict__ flags) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    flags[i] = (i == 0 || skeys[i] != skeys[i - 1]) ? 1u : 0u;
}

// seg = inclusive scan of the run-head flags: seg[i] - 1 is the unique index of sorted element i
__global__ void shard_finalize_kernel(const uint32_t* __restrict__ skeys, const uint32_t* __restrict__ sidx,
                                      const uint32_t* __restrict__ flags, const uint32_t* __restrict__ seg, long n,
                                      uint32_t* __restrict__ uniq, uint32_t* __restrict__ n_uniq,
                                      int32_t* __restrict__ remap) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const uint32_t k = skeys[i], s = seg[i];
    if (flags[i]) uniq[s - 1] = k;
    remap[sidx[i]] = k == SH_INVALID ? 0 : (int32_t)s;
    if (i == n - 1) *n_uniq = s;
  }
}

__device__ __forceinline__ uint32_t lower_bound_u32(const uint32_t* a, uint32_t n, uint64_t v) {
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if ((uint64_t)a[mid] < v) lo = mid + 1; else hi = mid;
  }
  return lo;
}

// per-owner run lengths of the sorted unique okeys (INVALID, if present, is last and counted nowhere)
__global__ void shard_counts_kernel(const uint32_t* __restrict__ uniq, const uint32_t* __restrict__ n_uniq, int world,
                                    int lbits, long long* __restrict__ counts) {
  const int w = threadIdx.x;
  if (w >= world) return;
  const uint32_t n = *n_uniq;
  const uint32_t a = lower_bound_u32(uniq, n, (uint64_t)w << lbits);
  const uint32_t b = lower_bound_u32(uniq, n, (uint64_t)(w + 1) << lbits);
  counts[w] = (long long)(b - a);
}

__global__ void shard_strip_kernel(const uint32_t* __restrict__ okeys, long n, uint32_t mask,
                                   int32_t* __restrict__ local) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    local[i] = (int32_t)(okeys[i] & mask);
}

// mode 0: rows of tabs[0] (att) -> out0, tabs[1] (rep) -> out1, row width tabs[0].width (== out_ld)
// mode 1: key -> table (last key_base <= key), row zero-padded to out_ld floats -> out0
__global__ void shard_gather_kernel(const int32_t* __restrict__ local, long n, int mode,
                                    const ctr_lazy_tab_t* __restrict__ tabs, int ntabs, const float* __restrict__ P,
                                    float* __restrict__ out0, float* __restrict__ out1, int out_ld) {
  const long total = n * out_ld;
  for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q < total; q += (long)gridDim.x * blockDim.x) {
    const long i = q / out_ld;
    const int k = (int)(q - i * out_ld);
    const uint32_t key = (uint32_t)local[i];
    if (mode == 0) {
      const long o = (long)key * tabs[0].width + k;
      out0[q] = P[tabs[0].p_off + o];
      out1[q] = P[tabs[1].p_off + o];
    } else {
      int a = 0, b = ntabs;
      while (b - a > 1) {
        const int mid = (a + b) >> 1;
        if (tabs[mid].key_base <= key) a = mid; else b = mid;
      }
      const ctr_lazy_tab_t tb = tabs[a];
      const long row = (long)(key - tb.key_base);
      out0[q] = (k < tb.width && row < tb.rows) ? P[tb.p_off + row * tb.width + k] : 0.f;
    }
  }
}

// ragged categorical rows on the wire (d_c floats each instead of the 64-float fetched-row layout):
// width of unique key i = dims[table of its local key] (table = last lbase <= local key); keys past
// *n (or INVALID) have width 0
__global__ void shard_widths_kernel(const uint32_t* __restrict__ keys, const uint32_t* __restrict__ n_ptr, long n_fix,
                                    long cap, uint32_t mask, const uint32_t* __restrict__ lbase,
                                    const int32_t* __restrict__ dims, int ntabs, uint32_t* __restrict__ width) {
  const long n = n_ptr ? (long)*n_ptr : n_fix;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < cap; i += (long)gridDim.x * blockDim.x) {
    uint32_t wd = 0;
    if (i < n && keys[i] != SH_INVALID) {
      const uint32_t lk = keys[i] & mask;
      int a = 0, b = ntabs;
      while (b - a > 1) {
        const int mid = (a + b) >> 1;
        if (lbase[mid] <= lk) a = mid; else b = mid;
      }
      wd = (uint32_t)dims[a];
    }
    width[i] = wd;
  }
}

// per-owner float counts of the owner-major unique keys: the width sums over each owner's run
__global__ void shard_float_counts_kernel(const uint32_t* __restrict__ uniq, const uint32_t* __restrict__ n_uniq,
                                          const uint32_t* __restrict__ offsets, int world, int lbits,
                                          long long* __restrict__ counts) {
  const int w = threadIdx.x;
  if (w >= world) return;
  const uint32_t n = *n_uniq;
  const uint32_t a = lower_bound_u32(uniq, n, (uint64_t)w << lbits);
  const uint32_t b = lower_bound_u32(uniq, n, (uint64_t)(w + 1) << lbits);
  counts[w] = (long long)offsets[b] - (long long)offsets[a];
}

// rows (n, ld) -> packed[off_i .. off_{i+1}) (row i's first off_{i+1} - off_i floats)
__global__ void shard_pack_kernel(const float* __restrict__ rows, int ld, long n, const uint32_t* __restrict__ off,
                                  float* __restrict__ packed) {
  for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q < n * ld; q += (long)gridDim.x * blockDim.x) {
    const long i = q / ld;
    const uint32_t k = (uint32_t)(q - i * ld), o = off[i], w = off[i + 1] - o;
    if (k < w) packed[o + k] = rows[q];
  }
}

// packed -> rows (row0 + i, out_ld), zero-padded past each row's width
__global__ void shard_unpack_kernel(const float* __restrict__ packed, const uint32_t* __restrict__ off, long n,
                                    float* __restrict__ out, int out_ld) {
  for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q < n * out_ld; q += (long)gridDim.x * blockDim.x) {
    const long i = q / out_ld;
    const uint32_t k = (uint32_t)(q - i * out_ld), o = off[i], w = off[i + 1] - o;
    out[q] = k < w ? packed[o + k] : 0.f;
  }
}

// ctr_copy_segments: one workgroup row per segment (blockIdx.y), the segment table passed by value in the
// kernel arguments (no upload).  16-byte moves when both ends are 16-byte aligned (att / rep rows of D floats
// always are), 4-byte moves otherwise (the packed categorical runs start at arbitrary floats).
constexpr int SEG_MAX = 96;
struct SegArgs {
  ctr_seg_t s[SEG_MAX];
};

__global__ __launch_bounds__(256) void copy_segments_kernel(const SegArgs a) {
  const ctr_seg_t sg = a.s[blockIdx.y];
  const long n = (long)sg.n;
  const long t0 = blockIdx.x * 256L + threadIdx.x, step = gridDim.x * 256L;
  if ((((uintptr_t)sg.src | (uintptr_t)sg.dst) & 15) == 0) {
    const long n4 = n >> 2;
    const uint4* s4 = (const uint4*)sg.src;
    uint4* d4 = (uint4*)sg.dst;
    for (long i = t0; i < n4; i += step) d4[i] = s4[i];
    for (long i = (n4 << 2) + t0; i < n; i += step) ((uint32_t*)sg.dst)[i] = ((const uint32_t*)sg.src)[i];
  } else {
    const uint32_t* s = (const uint32_t*)sg.src;
    uint32_t* d = (uint32_t*)sg.dst;
    for (long i = t0; i < n; i += step) d[i] = s[i];
  }
}

struct PlanWs {
  size_t temp_bytes, total;
  size_t off_okeys, off_iota, off_skeys, off_sidx, off_flags, off_seg;
};

static size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

static PlanWs plan_layout(long n) {
  PlanWs w{};
  size_t t1 = 0;
  (void)rocprim::radix_sort_pairs(nullptr, t1, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                  (const uint32_t*)nullptr, (uint32_t*)nullptr, (size_t)n, 0, 32);
  // the sort's temporary space doubles as the scan's block sums (the sort is done when the scan runs)
  w.temp_bytes = al256(std::max(t1, (size_t)scan_ws_words(n) * sizeof(uint32_t)));
  const size_t a = al256((size_t)n * sizeof(uint32_t));
  w.off_okeys = w.temp_bytes;
  w.off_iota = w.off_okeys + a;
  w.off_skeys = w.off_iota + a;
  w.off_sidx = w.off_skeys + a;
  w.off_flags = w.off_sidx + a;
  w.off_seg = w.off_flags + a;
  w.total = w.off_seg + a;
  return w;
}

static int grid_for(long n) { return (int)std::min<long>((n + 255) / 256, 8192); }

}  // namespace ctr

using namespace ctr;

extern "C" size_t ctr_shard_plan_ws_size(long n) { return n > 0 ? plan_layout(n).total : 0; }

extern "C" int ctr_shard_plan(const int32_t* X, long n, int ncols, int mode, int pad_id, const uint32_t* lbase,
                              int world, int lbits, int key_bits, uint32_t* uniq, uint32_t* n_uniq, int32_t* remap,
                              long long* send_counts, void* ws, size_t ws_bytes, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  CTR_REQUIRE(mode == 0 || mode == 1, "mode must be 0 (sequence) or 1 (categorical)");
  CTR_REQUIRE(world >= 1 && world <= 64, "world must be in [1, 64]");
  CTR_REQUIRE(lbits >= 1 && key_bits >= lbits && key_bits <= 32, "bad key widths");
  CTR_REQUIRE(mode == 0 || (ncols >= 1 && lbase != nullptr), "categorical plan needs ncols and lbase");
  if (n <= 0) {
    (void)hipMemsetAsync(n_uniq, 0, sizeof(uint32_t), s);
    (void)hipMemsetAsync(send_counts, 0, sizeof(long long) * world, s);
    return check_launch("shard_plan");
  }
  CTR_REQUIRE(n < (1L << 31), "too many ids");
  const PlanWs w = plan_layout(n);
  CTR_REQUIRE(ws_bytes >= w.total, "shard_plan workspace too small");
  char* base = (char*)ws;
  uint32_t* okeys = (uint32_t*)(base + w.off_okeys);
  uint32_t* iota = (uint32_t*)(base + w.off_iota);
  uint32_t* skeys = (uint32_t*)(base + w.off_skeys);
  uint32_t* sidx = (uint32_t*)(base + w.off_sidx);
  uint32_t* flags = (uint32_t*)(base + w.off_flags);
  uint32_t* seg = (uint32_t*)(base + w.off_seg);
  const int g = grid_for(n);
  shard_keys_kernel<<<g, 256, 0, s>>>(X, n, ncols, mode, pad_id, lbase, (uint32_t)world, lbits, okeys, iota);
  size_t tb = w.temp_bytes;
  // valid okeys < 2^key_bits - 1 (host picks lbits so), so INVALID (all ones in the low bits) sorts last
  hipError_t e = rocprim::radix_sort_pairs(base, tb, (const uint32_t*)okeys, skeys, (const uint32_t*)iota, sidx,
                                           (size_t)n, 0, (unsigned)key_bits, s);
  CTR_REQUIRE(e == hipSuccess, "radix_sort_pairs failed");
  shard_flags_kernel<<<g, 256, 0, s>>>(skeys, n, flags);
  scan_u32(flags, seg, n, true, (uint32_t*)base, s);
  shard_finalize_kernel<<<g, 256, 0, s>>>(skeys, sidx, flags, seg, n, uniq, n_uniq, remap);
  shard_counts_kernel<<<1, 64, 0, s>>>(uniq, n_uniq, world, lbits, send_counts);
  return check_launch("shard_plan");
}

extern "C" int ctr_shard_strip(const uint32_t* okeys, long n, uint32_t mask, int32_t* local, void* stream) {
  if (n <= 0) return 0;
  shard_strip_kernel<<<grid_for(n), 256, 0, (hipStream_t)stream>>>(okeys, n, mask, local);
  return check_launch("shard_strip");
}

extern "C" int ctr_shard_gather(const int32_t* local, long n, int mode, const ctr_lazy_tab_t* tabs, int ntabs,
                                const float* P, float* out0, float* out1, int out_ld, void* stream) {
  CTR_REQUIRE(mode == 0 || mode == 1, "mode must be 0 (sequence) or 1 (categorical)");
  CTR_REQUIRE(mode == 1 || (ntabs == 2 && out1 != nullptr), "sequence gather needs the att and rep tables");
  CTR_REQUIRE(out_ld >= 1 && out_ld <= 64, "out_ld must be in [1, 64]");
  if (n <= 0) return 0;
  shard_gather_kernel<<<grid_for(n * out_ld), 256, 0, (hipStream_t)stream>>>(local, n, mode, tabs, ntabs, P, out0,
                                                                             out1, out_ld);
  return check_launch("shard_gather");
}

extern "C" size_t ctr_shard_offsets_ws_size(long cap) {
  return al256((size_t)scan_ws_words(cap + 1) * sizeof(uint32_t)) + al256(((size_t)cap + 1) * sizeof(uint32_t));
}

extern "C" int ctr_shard_offsets(const uint32_t* keys, const uint32_t* n_ptr, long n, long cap, uint32_t mask,
                                 const uint32_t* lbase, const int32_t* dims, int ntabs, uint32_t* offsets, int world,
                                 int lbits, long long* float_counts, void* ws, size_t ws_bytes, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  CTR_REQUIRE(cap >= 0 && ntabs >= 1, "ctr_shard_offsets: bad sizes");
  CTR_REQUIRE(ws_bytes >= ctr_shard_offsets_ws_size(cap), "ctr_shard_offsets: workspace too small");
  CTR_REQUIRE(!float_counts || (n_ptr && world >= 1 && world <= 64), "ctr_shard_offsets: per-owner counts need n_uniq");
  const size_t tb = al256((size_t)scan_ws_words(cap + 1) * sizeof(uint32_t));
  char* base = (char*)ws;
  uint32_t* width = (uint32_t*)(base + tb);
  // cap + 1 widths (the last one 0) -> cap + 1 exclusive offsets: offsets[i + 1] - offsets[i] = width i
  shard_widths_kernel<<<grid_for(cap + 1), 256, 0, s>>>(keys, n_ptr, n, cap + 1, mask, lbase, dims, ntabs, width);
  scan_u32(width, offsets, cap + 1, false, (uint32_t*)base, s);
  if (float_counts) shard_float_counts_kernel<<<1, 64, 0, s>>>(keys, n_ptr, offsets, world, lbits, float_counts);
  return check_launch("shard_offsets");
}

extern "C" int ctr_shard_pack(const float* rows, int ld, long n, const uint32_t* offsets, float* packed, void* stream) {
  CTR_REQUIRE(ld >= 1 && ld <= 64, "ctr_shard_pack: ld must be in [1, 64]");
  if (n <= 0) return 0;
  shard_pack_kernel<<<grid_for(n * ld), 256, 0, (hipStream_t)stream>>>(rows, ld, n, offsets, packed);
  return check_launch("shard_pack");
}

extern "C" int ctr_shard_unpack(const float* packed, const uint32_t* offsets, long n, float* out, int out_ld,
                                void* stream) {
  CTR_REQUIRE(out_ld >= 1 && out_ld <= 64, "ctr_shard_unpack: out_ld must be in [1, 64]");
  if (n <= 0) return 0;
  shard_unpack_kernel<<<grid_for(n * out_ld), 256, 0, (hipStream_t)stream>>>(packed, offsets, n, out, out_ld);
  return check_launch("shard_unpack");
}

extern "C" int ctr_copy_segments(const ctr_seg_t* segs, int nseg, void* stream) {
  CTR_REQUIRE(nseg >= 0 && (nseg == 0 || segs != nullptr), "ctr_copy_segments: bad segment table");
  for (int s0 = 0; s0 < nseg; s0 += SEG_MAX) {
    SegArgs a{};
    int k = 0;
    long maxn = 0;
    for (int s = s0; s < nseg && s < s0 + SEG_MAX; ++s) {
      if (segs[s].n <= 0) continue;
      CTR_REQUIRE(segs[s].src != nullptr && segs[s].dst != nullptr, "ctr_copy_segments: null segment pointer");
      a.s[k++] = segs[s];
      maxn = std::max<long>(maxn, (long)segs[s].n);
    }
    if (k == 0) continue;
    // ~4 KB per workgroup pass at 16-byte moves; at most 64 workgroups per segment
    const int gx = (int)std::min<long>(std::max<long>((maxn + 4095) / 4096, 1), 64);
    copy_segments_kernel<<<dim3(gx, k), 256, 0, (hipStream_t)stream>>>(a);
  }
  return check_launch("copy_segments");
}

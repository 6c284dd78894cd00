// Co-visitation features on device (src/features/covis.py, driven by src/tools/build_covis_features.py):
// the (token, target, time_bin) pair statistics of the exploded seq column and the per-row aggregates of
// a left join against them -- the reference does both with polars group_by / join over ~10^9 exploded
// rows on the host.
//
// Input (tossctr/covis.py): the seq column exploded once on the host (csrc/hostio.cpp ctr_covis_explode):
// tok / pos / ok per exploded element, row_ptr (int64, n_rows + 1) per source row, and per source row its
// target code (-1 null), time-bin code (-1 null) and clicked flag.  A pair key packs
//   ((tok ^ 0x80000000) << 32) | (target << tb_bits) | tbin          (u64; ascending = (token, target, tbin))
// Keys with a null part can never match the left join (polars join_nulls=False) and are not tabled.
//
//   ctr_covis_pair_stats   _pair_stats_from_scan (covis.py:155-213) over the rows with keep[row] != 0:
//                          keys -> stable radix sort (element index as value) -> run-length groups ->
//                          one thread per group sums its run in element order (impr, clicks, w_rec_sum,
//                          max_pos: deterministic, the oracle's order) -> beta-smoothed, clipped ctr.
//                          p0 = mean(clicked) over every exploded element of the kept rows (nulls included,
//                          covis.py:199-201).
//   ctr_covis_row_features _row_features_from_pair_tbl (covis.py:233-292) for a list of source rows: one
//                          thread per row walks its exploded tokens in order, binary-searches the sorted
//                          pair keys, and produces the 8 aggregates of AGG_ORDER (oracle/covis.py).
// HBM-bound integer work (sort + gathers); the f64 sums run in the oracle's order.
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_run_length_encode.hpp>
#include <rocprim/device/device_scan.hpp>

#include "common.h"
#include "ctr_hip.h"

namespace ctr {

constexpr uint64_t COVIS_NONE = ~0ull;
constexpr int COVIS_TOPN_MAX = 16;

__device__ __forceinline__ uint64_t covis_key(int32_t tok, int32_t tgt, int32_t tb, int tb_bits) {
  return ((uint64_t)((uint32_t)tok ^ 0x80000000u) << 32) | ((uint64_t)(uint32_t)tgt << tb_bits) | (uint32_t)tb;
}

// keys of the exploded elements (COVIS_NONE for rows not kept / null key parts) + integer p0 sums
__global__ void covis_keys_kernel(const int32_t* __restrict__ tok, const uint8_t* __restrict__ ok,
                                  const int32_t* __restrict__ erow, long n, const int32_t* __restrict__ tgt,
                                  const int32_t* __restrict__ tb, const uint8_t* __restrict__ click,
                                  const uint8_t* __restrict__ keep, int tb_bits, uint64_t* __restrict__ keys,
                                  uint32_t* __restrict__ idx, unsigned long long* __restrict__ sums) {
  unsigned long long cnt = 0, clk = 0;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < n; e += (long)gridDim.x * blockDim.x) {
    const int r = erow[e];
    uint64_t k = COVIS_NONE;
    if (keep == nullptr || keep[r]) {
      cnt += 1;
      clk += click[r];
      if (ok[e] && tgt[r] >= 0 && tb[r] >= 0) k = covis_key(tok[e], tgt[r], tb[r], tb_bits);
    }
    keys[e] = k;
    idx[e] = (uint32_t)e;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    cnt += __shfl_xor(cnt, o, 64);
    clk += __shfl_xor(clk, o, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    atomicAdd(sums + 0, cnt);         // integer sums: order-independent
    atomicAdd(sums + 1, clk);
  }
}

struct CovisPairOut {
  uint64_t* keys;      // sorted unique keys (ascending), n_pairs of them
  int32_t* impr;
  int64_t* clicks;
  double* w_rec_sum;
  int32_t* max_pos;
  double* ctr;
  uint8_t* lowcount;
  int64_t* n_pairs;    // device scalar
  double* p0;          // device scalar
};

// one thread per run of equal keys; runs are in ascending key order, the sentinel run (if any) is last
__global__ void covis_groups_kernel(const uint64_t* __restrict__ ukeys, const uint32_t* __restrict__ counts,
                                    const uint32_t* __restrict__ starts, const uint32_t* __restrict__ nruns,
                                    const uint32_t* __restrict__ sidx, const int32_t* __restrict__ pos,
                                    const int32_t* __restrict__ erow, const uint8_t* __restrict__ click,
                                    const unsigned long long* __restrict__ sums, double tau, double S, double lo,
                                    double hi, int min_impr, CovisPairOut o) {
  const uint32_t nr = *nruns;
  const bool has_none = nr > 0 && ukeys[nr - 1] == COVIS_NONE;
  const uint32_t np = nr - (has_none ? 1u : 0u);
  const unsigned long long cnt = sums[0], clk = sums[1];
  const double p0 = cnt ? (double)clk / (double)cnt : 0.019;   // covis.py:200-201 (0.019 when empty)
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    *o.n_pairs = np;
    *o.p0 = p0;
  }
  const double alpha = p0 * S, beta = (1.0 - p0) * S;
  for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < np; j += gridDim.x * blockDim.x) {
    const uint32_t s = starts[j], c = counts[j];
    long clicks = 0;
    double w = 0.0;
    int mp = INT32_MIN;
    for (uint32_t t = s; t < s + c; ++t) {
      const uint32_t e = sidx[t];
      clicks += click[erow[e]];
      w += exp(-(double)pos[e] / tau);
      mp = max(mp, pos[e]);
    }
    double v = ((double)clicks + alpha) / ((double)c + alpha + beta);   // _beta_smooth_ctr (covis.py:106-109)
    v = fmin(fmax(v, 1e-9), 1.0 - 1e-9);
    v = fmin(fmax(v, lo), hi);                                          // ctr_clip (covis.py:208-210)
    o.keys[j] = ukeys[j];
    o.impr[j] = (int32_t)c;
    o.clicks[j] = clicks;
    o.w_rec_sum[j] = w;
    o.max_pos[j] = mp;
    o.ctr[j] = v;
    o.lowcount[j] = (int)c < min_impr;
  }
}

__device__ __forceinline__ long covis_find(const uint64_t* __restrict__ keys, long n, uint64_t k) {
  long a = 0, b = n;
  while (a < b) {
    const long m = (a + b) >> 1;
    if (keys[m] < k) a = m + 1; else b = m;
  }
  return (a < n && keys[a] == k) ? a : -1;
}

// out[i*8 + c]: sum_ctr, mean_ctr, max_ctr, top-n mean, wmean_ctr, sum_impr, max_impr, pnorm_ctr
__global__ void covis_rows_kernel(const int64_t* __restrict__ rows, long nq, const int64_t* __restrict__ row_ptr,
                                  const int32_t* __restrict__ tok, const int32_t* __restrict__ pos,
                                  const uint8_t* __restrict__ ok, const int32_t* __restrict__ tgt,
                                  const int32_t* __restrict__ tb, int tb_bits, double tau,
                                  const uint64_t* __restrict__ keys, const double* __restrict__ ctr,
                                  const int32_t* __restrict__ impr, const int64_t* __restrict__ n_pairs, int topn,
                                  double* __restrict__ out) {
  const long np = *n_pairs;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < nq; i += (long)gridDim.x * blockDim.x) {
    const long r = rows[i];
    const int32_t g = tgt[r], b = tb[r];
    double s = 0.0, ss = 0.0, mx = 0.0, wnum = 0.0, wden = 0.0;
    long n = 0, nulls = 0, simpr = 0, mimpr = 0;
    double top[COVIS_TOPN_MAX];                 // the n largest ctr so far, descending
#pragma unroll
    for (int q = 0; q < COVIS_TOPN_MAX; ++q) top[q] = -1.0;
    for (long e = row_ptr[r]; e < row_ptr[r + 1]; ++e) {
      const double w = exp(-(double)pos[e] / tau);
      wden += w;
      const long j = (ok[e] && g >= 0 && b >= 0) ? covis_find(keys, np, covis_key(tok[e], g, b, tb_bits)) : -1;
      if (j < 0) {
        ++nulls;
        continue;
      }
      const double c = ctr[j];
      const long im = impr[j];
      s += c;
      ss += c * c;
      wnum += c * w;
      mx = n ? fmax(mx, c) : c;
      ++n;
      simpr += im;
      mimpr = im > mimpr ? im : mimpr;
      double x = c;                             // insert into the descending top list
#pragma unroll
      for (int q = 0; q < COVIS_TOPN_MAX; ++q) {
        if (q < topn && x > top[q]) {
          const double t = top[q];
          top[q] = x;
          x = t;
        }
      }
    }
    // ctr.sort(descending=True).head(n): polars puts nulls first, so unmatched tokens take head slots
    const long kv = nulls >= topn ? 0 : (n < topn - nulls ? n : topn - nulls);
    double hs = 0.0;
#pragma unroll
    for (int q = 0; q < COVIS_TOPN_MAX; ++q)
      if (q < kv) hs += top[q];
    double* o = out + i * 8;
    o[0] = s;
    o[1] = n ? s / (double)n : 0.0;
    o[2] = n ? mx : 0.0;
    o[3] = kv ? hs / (double)kv : 0.0;
    o[4] = wnum / wden;
    o[5] = (double)simpr;
    o[6] = (double)mimpr;
    o[7] = n ? sqrt(ss / (double)n) : 0.0;
  }
}

struct CovisWs {
  size_t keys, skeys, idx, sidx, counts, starts, nruns, sums, temp, temp_bytes, total;
};

static CovisWs covis_layout(long n) {
  CovisWs w{};
  size_t t1 = 0, t2 = 0, t3 = 0;
  (void)rocprim::radix_sort_pairs(nullptr, t1, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                                  (const uint32_t*)nullptr, (uint32_t*)nullptr, (size_t)n);
  (void)rocprim::run_length_encode(nullptr, t2, (const uint64_t*)nullptr, (size_t)n, (uint64_t*)nullptr,
                                   (uint32_t*)nullptr, (uint32_t*)nullptr);
  (void)rocprim::exclusive_scan(nullptr, t3, (const uint32_t*)nullptr, (uint32_t*)nullptr, 0u, (size_t)n,
                                rocprim::plus<uint32_t>());
  size_t tb = t1 > t2 ? t1 : t2;
  if (t3 > tb) tb = t3;
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  size_t off = 0;
  w.keys = off; off += al(8 * (size_t)n);
  w.skeys = off; off += al(8 * (size_t)n);
  w.idx = off; off += al(4 * (size_t)n);
  w.sidx = off; off += al(4 * (size_t)n);
  w.counts = off; off += al(4 * (size_t)n);
  w.starts = off; off += al(4 * (size_t)n);
  w.nruns = off; off += al(4);
  w.sums = off; off += al(16);
  w.temp = off; off += al(tb);
  w.temp_bytes = tb;
  w.total = off;
  return w;
}

}  // namespace ctr

using namespace ctr;

extern "C" size_t ctr_covis_ws_size(long n) { return covis_layout(n > 0 ? n : 1).total; }

extern "C" int ctr_covis_pair_stats(const int32_t* tok, const int32_t* pos, const uint8_t* ok, const int32_t* erow,
                                    long n, const int32_t* tgt, const int32_t* tb, const uint8_t* click,
                                    const uint8_t* keep, int tb_bits, double tau, double prior_strength,
                                    double clip_lo, double clip_hi, int min_impr, uint64_t* out_keys,
                                    int32_t* out_impr, int64_t* out_clicks, double* out_wsum, int32_t* out_maxpos,
                                    double* out_ctr, uint8_t* out_low, int64_t* n_pairs, double* p0, void* ws,
                                    size_t ws_bytes, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  CTR_REQUIRE(n >= 0 && n < ((long)1 << 32), "ctr_covis_pair_stats: exploded length must fit 32 bits");
  CTR_REQUIRE(tb_bits >= 0 && tb_bits <= 31, "ctr_covis_pair_stats: tb_bits out of range");
  CTR_REQUIRE(tau > 0.0, "ctr_covis_pair_stats: recency_tau must be positive");
  const CovisWs w = covis_layout(n > 0 ? n : 1);
  CTR_REQUIRE(ws && ws_bytes >= w.total, "ctr_covis_pair_stats: workspace too small (ctr_covis_ws_size)");
  char* base = (char*)ws;
  uint64_t* keys = (uint64_t*)(base + w.keys);
  uint64_t* skeys = (uint64_t*)(base + w.skeys);
  uint32_t* idx = (uint32_t*)(base + w.idx);
  uint32_t* sidx = (uint32_t*)(base + w.sidx);
  uint32_t* counts = (uint32_t*)(base + w.counts);
  uint32_t* starts = (uint32_t*)(base + w.starts);
  uint32_t* nruns = (uint32_t*)(base + w.nruns);
  unsigned long long* sums = (unsigned long long*)(base + w.sums);
  void* temp = base + w.temp;
  (void)hipMemsetAsync(sums, 0, 16, s);
  (void)hipMemsetAsync(nruns, 0, 4, s);
  if (n > 0) {
    const int g = (int)std::min<long>(cdiv(n, 256), 4096);
    covis_keys_kernel<<<g, 256, 0, s>>>(tok, ok, erow, n, tgt, tb, click, keep, tb_bits, keys, idx, sums);
    size_t tbytes = w.temp_bytes;
    hipError_t e = rocprim::radix_sort_pairs(temp, tbytes, keys, skeys, idx, sidx, (size_t)n, 0, 64, s);
    CTR_REQUIRE(e == hipSuccess, "ctr_covis_pair_stats: radix sort failed");
    tbytes = w.temp_bytes;
    e = rocprim::run_length_encode(temp, tbytes, skeys, (size_t)n, keys /* unique keys: scratch */, counts, nruns, s);
    CTR_REQUIRE(e == hipSuccess, "ctr_covis_pair_stats: run-length encode failed");
    tbytes = w.temp_bytes;
    e = rocprim::exclusive_scan(temp, tbytes, counts, starts, 0u, (size_t)n, rocprim::plus<uint32_t>(), s);
    CTR_REQUIRE(e == hipSuccess, "ctr_covis_pair_stats: offsets scan failed");
  }
  CovisPairOut o{out_keys, out_impr, out_clicks, out_wsum, out_maxpos, out_ctr, out_low, n_pairs, p0};
  const int g2 = (int)std::max<long>(1, std::min<long>(cdiv(n, 256), 4096));
  covis_groups_kernel<<<g2, 256, 0, s>>>(keys, counts, starts, nruns, sidx, pos, erow, click, sums, tau,
                                         prior_strength, clip_lo, clip_hi, min_impr, o);
  return check_launch("covis_pair_stats");
}

extern "C" int ctr_covis_row_features(const int64_t* rows, long nq, const int64_t* row_ptr, const int32_t* tok,
                                      const int32_t* pos, const uint8_t* ok, const int32_t* tgt, const int32_t* tb,
                                      int tb_bits, double tau, const uint64_t* keys, const double* ctr,
                                      const int32_t* impr, const int64_t* n_pairs, int topn, double* out,
                                      void* stream) {
  CTR_REQUIRE(topn >= 0 && topn <= COVIS_TOPN_MAX, "ctr_covis_row_features: agg topn must be in [0, 16]");
  CTR_REQUIRE(tau > 0.0 && tb_bits >= 0 && tb_bits <= 31, "ctr_covis_row_features: bad tau / tb_bits");
  if (nq <= 0) return 0;
  const int g = (int)std::min<long>(cdiv(nq, 256), 8192);
  covis_rows_kernel<<<g, 256, 0, (hipStream_t)stream>>>(rows, nq, row_ptr, tok, pos, ok, tgt, tb, tb_bits, tau, keys,
                                                        ctr, impr, n_pairs, topn, out);
  return check_launch("covis_row_features");
}

// Fused gradient clip + AdamW + EMA over the whole parameter arena -- the HBM-bound stream that
// dominates a training step.
//
// Replaces, per step: nn.utils.clip_grad_norm_ (src/train.py:194), torch.optim.AdamW.step
// (src/train.py:138,195; torch/optim/adam.py _single_tensor_adam, decoupled weight decay) and
// ModelEMA.update (src/utils/ema.py:92-131).  Semantics are the dense reference ones: EVERY
// element of every table is decayed / moment-updated each step, rows that no sample touched see
// grad = 0.  What differs is that no dense table gradient ever exists: table grads arrive as the
// compact (sorted unique keys, summed rows) produced by rowgrad.hip, and each workgroup maps the
// touched rows of its chunk into an LDS slot table (binary search + forward scan of the sorted keys).
// Per element: read p, m, v, ema (+ g) and write p, m, v, ema once -- 32 B/param of HBM traffic.
#include "adam.h"
#include "common.h"
#include "ctr_hip.h"

namespace ctr {

constexpr int OPT_CHUNK = 8192;                 // elements per workgroup
constexpr int OPT_MAXROWS = OPT_CHUNK / 4 + 2;  // sparse segments need width >= 4

// For every sparse-segment chunk: [lo, hi) = index range of the sorted unique keys that fall in the
// chunk's rows.  One thread per chunk (binary searches run in parallel, not as a serial prologue of
// every streaming workgroup).
// (hist != null: thread 0 also records the tick's scalars in the lazy tables' history -- the separate one-thread
// launch before it cost a dispatch and its boundary every step)
__global__ __launch_bounds__(256) void chunk_key_range_kernel(const ctr_opt_chunk_t* __restrict__ chunks, int nchunks,
                                                              const ctr_opt_seg_t* __restrict__ segs,
                                                              uint32_t* __restrict__ range,
                                                              OptScalars* __restrict__ hist = nullptr, int tick = 0,
                                                              OptScalars hs = OptScalars{}) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (hist && c == 0) hist[tick] = hs;
  if (c >= nchunks) return;
  const ctr_opt_chunk_t ch = chunks[c];
  const ctr_opt_seg_t sg = segs[ch.seg];
  uint32_t lo = 0, hi = 0;
  if (sg.kind == 1) {
    const uint32_t nu = *sg.n_uniq;
    const uint32_t k0 = sg.key_base + (uint32_t)(ch.e0 / sg.width);
    const uint32_t k1 = sg.key_base + (uint32_t)((min(ch.e1, sg.n) - 1) / sg.width);   // real rows only
    uint32_t a = 0, b = nu;
    while (a < b) { const uint32_t mid = (a + b) >> 1; if (sg.keys[mid] < k0) a = mid + 1; else b = mid; }
    lo = a;
    b = nu;
    while (a < b) { const uint32_t mid = (a + b) >> 1; if (sg.keys[mid] <= k1) a = mid + 1; else b = mid; }
    hi = a;
  }
  range[2 * c] = lo;
  range[2 * c + 1] = hi;
}

__device__ __forceinline__ float row_grad(const ctr_opt_seg_t& sg, const int* map, int nrows, int rel, int width,
                                          float coef) {
  const int row = rel / width;
  const int slot = row < nrows ? map[row] : -1;
  return slot >= 0 ? sg.G[(long)slot * sg.g_ld + (rel - row * width)] * coef : 0.0f;
}

// Streams one OPT_CHUNK-element chunk of one segment per workgroup, one float4 of each of p, m, v,
// ema per thread per iteration (registers only -- no address-taken arrays, so nothing spills to
// scratch).  Segments are streamed in whole float4s: the tail float4 lies inside the param's
// 64-element arena padding.  Sparse segments: the touched rows of the chunk are mapped into an LDS
// slot table from the precomputed key range; untouched rows get grad 0 (dense AdamW semantics).
// INLINE (ctr_adamw_ema_hist): no chunk_key_range launch before it -- block 0 records the tick's scalars in the
// history, and a sparse chunk's key range is searched by the workgroup itself (the same binary searches: the same
// range).  The lazy step's chunk lists hold no sparse segment, so there the launch and its boundary simply go.
template <bool INLINE = false>
__global__ __launch_bounds__(256) void adamw_ema_kernel(const ctr_opt_chunk_t* __restrict__ chunks,
                                                        const ctr_opt_seg_t* __restrict__ segs,
                                                        const uint32_t* __restrict__ krange,
                                                        float* __restrict__ P, float* __restrict__ M,
                                                        float* __restrict__ V, float* __restrict__ E,
                                                        const float* __restrict__ dgrad,
                                                        const float* __restrict__ coef_ptr, OptScalars s,
                                                        OptScalars* __restrict__ hist = nullptr, int tick = 0) {
  __shared__ int map[OPT_MAXROWS];
  __shared__ uint32_t srange[2];
  if (INLINE && blockIdx.x == 0 && threadIdx.x == 0) hist[tick] = s;
  const ctr_opt_chunk_t ch = chunks[blockIdx.x];
  const ctr_opt_seg_t sg = segs[ch.seg];
  const float coef = coef_ptr ? *coef_ptr : 1.0f;
  const bool adam = s.do_adam && sg.kind != 2;
  const bool sparse = adam && sg.kind == 1;
  const int tid = threadIdx.x;
  const int width = sg.width;
  const long r0 = ch.e0 / width;
  const int off0 = (int)(ch.e0 - r0 * width);     // chunk start inside its first row
  int nrows = 0;
  if (sparse) {
    nrows = (int)((ch.e1 - 1) / width - r0 + 1);
    for (int i = tid; i < nrows; i += 256) map[i] = -1;
    __syncthreads();
    uint32_t lo, hi;
    if (INLINE) {
      if (tid == 0) {      // chunk_key_range_kernel's searches for this chunk
        const uint32_t nu = *sg.n_uniq;
        const uint32_t k0 = sg.key_base + (uint32_t)(ch.e0 / sg.width);
        const uint32_t k1 = sg.key_base + (uint32_t)((min(ch.e1, sg.n) - 1) / sg.width);
        uint32_t a = 0, b = nu;
        while (a < b) { const uint32_t mid = (a + b) >> 1; if (sg.keys[mid] < k0) a = mid + 1; else b = mid; }
        srange[0] = a;
        b = nu;
        while (a < b) { const uint32_t mid = (a + b) >> 1; if (sg.keys[mid] <= k1) a = mid + 1; else b = mid; }
        srange[1] = a;
      }
      __syncthreads();
      lo = srange[0];
      hi = srange[1];
    } else {
      lo = krange[2 * blockIdx.x];
      hi = krange[2 * blockIdx.x + 1];
    }
    const uint32_t k0 = sg.key_base + (uint32_t)r0;
    for (uint32_t i = lo + tid; i < hi; i += 256) map[sg.keys[i] - k0] = (int)i;
    __syncthreads();
  }
  float* p = P + sg.p_off + ch.e0;
  float* m = M + sg.p_off + ch.e0;
  float* v = V + sg.p_off + ch.e0;
  float* e = E + sg.p_off + ch.e0;
  const float* gd = dgrad + sg.g_off + ch.e0;
  const int n = (int)(ch.e1 - ch.e0);             // multiple of 4
#pragma unroll 2
  for (int lq = tid * 4; lq < n; lq += 1024) {
    float4 pv = *(const float4*)(p + lq);
    float4 mv = {0.f, 0.f, 0.f, 0.f}, vv = {0.f, 0.f, 0.f, 0.f}, ev = {0.f, 0.f, 0.f, 0.f};
    float4 g = {0.f, 0.f, 0.f, 0.f};
    if (adam) {
      mv = *(const float4*)(m + lq);
      vv = *(const float4*)(v + lq);
      if (sg.kind == 0) {
        g = *(const float4*)(gd + lq);
        g.x *= coef; g.y *= coef; g.z *= coef; g.w *= coef;
      } else {
        const int rel = off0 + lq;
        g.x = row_grad(sg, map, nrows, rel, width, coef);
        g.y = row_grad(sg, map, nrows, rel + 1, width, coef);
        g.z = row_grad(sg, map, nrows, rel + 2, width, coef);
        g.w = row_grad(sg, map, nrows, rel + 3, width, coef);
      }
    }
    if (s.do_ema) ev = *(const float4*)(e + lq);
    adam_ema_elem(s, pv.x, mv.x, vv.x, ev.x, g.x, adam);
    adam_ema_elem(s, pv.y, mv.y, vv.y, ev.y, g.y, adam);
    adam_ema_elem(s, pv.z, mv.z, vv.z, ev.z, g.z, adam);
    adam_ema_elem(s, pv.w, mv.w, vv.w, ev.w, g.w, adam);
    if (adam) {
      *(float4*)(p + lq) = pv;
      *(float4*)(m + lq) = mv;
      *(float4*)(v + lq) = vv;
    }
    if (s.do_ema) *(float4*)(e + lq) = ev;
  }
}

// ---------------- global grad norm (clip_grad_norm_) ----------------
constexpr int NORM_BLOCKS = 256;

// block bx of gx: its partial of sum x^2 (the thread's own sum; the caller reduces the block)
__device__ __forceinline__ float sqnorm_dense_part(const float* __restrict__ x, long n, int bx, int gx) {
  float s = 0.f;
  if ((((uintptr_t)x) & 15) == 0) {   // 16-byte loads, four independent chains; scalar tail
    const long n4 = n >> 2;
    const float4* x4 = (const float4*)x;
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
#pragma unroll 4
    for (long i = bx * 256L + threadIdx.x; i < n4; i += (long)gx * 256) {
      const float4 v = x4[i];
      s0 = fmaf(v.x, v.x, s0);
      s1 = fmaf(v.y, v.y, s1);
      s2 = fmaf(v.z, v.z, s2);
      s3 = fmaf(v.w, v.w, s3);
    }
    s = (s0 + s1) + (s2 + s3);
    for (long i = 4 * n4 + bx * 256L + threadIdx.x; i < n; i += (long)gx * 256) s = fmaf(x[i], x[i], s);
  } else {
    for (long i = bx * 256L + threadIdx.x; i < n; i += (long)gx * 256) s = fmaf(x[i], x[i], s);
  }
  return s;
}

__global__ __launch_bounds__(256) void sqnorm_dense_kernel(const float* __restrict__ x, long n,
                                                           float* __restrict__ part) {
  __shared__ float red[4];
  const float s = block_sum(sqnorm_dense_part(x, n, blockIdx.x, gridDim.x), red);
  if (threadIdx.x == 0) part[blockIdx.x] = s;
}

// Compact row grads: rows are sorted by key and the INVALID group (if any) is the last row, so the
// valid rows are one contiguous prefix -- summed as a flat float4 stream (padding columns are zero).
__device__ __forceinline__ float sqnorm_rows_part(const uint32_t* __restrict__ keys, const float* __restrict__ G,
                                                 const uint32_t* __restrict__ n_uniq, int width, int ld,
                                                 uint32_t invalid_key, int bx, int gx) {
  const uint32_t nu = *n_uniq;
  const uint32_t nv = (nu > 0 && keys[nu - 1] == invalid_key) ? nu - 1 : nu;
  float s = 0.f;
  if ((ld & 3) == 0) {
    const long total4 = (long)nv * ld / 4;
    const float4* G4 = (const float4*)G;
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;   // four chains, four loads in flight
#pragma unroll 4
    for (long i = bx * 256L + threadIdx.x; i < total4; i += (long)gx * 256) {
      const float4 g = G4[i];
      s0 = fmaf(g.x, g.x, s0);
      s1 = fmaf(g.y, g.y, s1);
      s2 = fmaf(g.z, g.z, s2);
      s3 = fmaf(g.w, g.w, s3);
    }
    s = (s0 + s1) + (s2 + s3);
  } else {
    const long total = (long)nv * width;
    for (long i = bx * 256L + threadIdx.x; i < total; i += (long)gx * 256) {
      const long u = i / width;
      const float g = G[u * ld + (i - u * width)];
      s = fmaf(g, g, s);
    }
  }
  return s;
}

__global__ __launch_bounds__(256) void sqnorm_rows_kernel(const uint32_t* __restrict__ keys,
                                                          const float* __restrict__ G,
                                                          const uint32_t* __restrict__ n_uniq, int width, int ld,
                                                          uint32_t invalid_key, float* __restrict__ part) {
  __shared__ float red[4];
  const float s = block_sum(sqnorm_rows_part(keys, G, n_uniq, width, ld, invalid_key, blockIdx.x, gridDim.x), red);
  if (threadIdx.x == 0) part[blockIdx.x] = s;
}

// the dense grads and up to CTR_SQNORM_MAX_ROWS compact row-grad tables in ONE launch: grid row y = 0 the dense
// stream, y = 1 + j table j, each row of NORM_BLOCKS blocks writing the partials ctr_sqnorm_dense /
// ctr_sqnorm_rows write (the same per-block sums: the same bits) at part[y * NORM_BLOCKS ..]
struct SqnormRowsSet {
  ctr_sqnorm_rows_t r[CTR_SQNORM_MAX_ROWS];
};
__global__ __launch_bounds__(256) void sqnorm_all_kernel(const float* __restrict__ x, long n, SqnormRowsSet rs,
                                                         uint32_t invalid_key, float* __restrict__ part) {
  __shared__ float red[4];
  const int y = blockIdx.y;
  float s;
  if (y == 0) {
    s = sqnorm_dense_part(x, n, blockIdx.x, gridDim.x);
  } else {
    const ctr_sqnorm_rows_t& r = rs.r[y - 1];
    s = sqnorm_rows_part(r.keys, r.G, r.n_uniq, r.width, r.ld, invalid_key, blockIdx.x, gridDim.x);
  }
  s = block_sum(s, red);
  if (threadIdx.x == 0) part[(long)y * gridDim.x + blockIdx.x] = s;
}

// grad_scale = 1/world under data parallelism: grads were summed across ranks, the reference
// (DDP semantics) clips and steps on their mean.
__global__ __launch_bounds__(256) void clip_finalize_kernel(const float* __restrict__ part, int nparts, float max_norm,
                                                            float grad_scale, float* __restrict__ out) {
  __shared__ float red[4];
  float s = 0.f;
  for (int i = threadIdx.x; i < nparts; i += 256) s += part[i];
  s = block_sum(s, red);
  if (threadIdx.x == 0) {
    const float norm = sqrtf(s) * grad_scale;
    out[0] = norm;
    out[1] = (max_norm > 0.f ? fminf(max_norm / (norm + 1e-6f), 1.0f) : 1.0f) * grad_scale;
  }
}

}  // namespace ctr

using namespace ctr;

extern "C" int ctr_opt_chunk_elems(void) { return OPT_CHUNK; }

extern "C" int ctr_adamw_ema(const ctr_opt_chunk_t* chunks, int nchunks, const ctr_opt_seg_t* segs, uint32_t* krange,
                             float* P, float* M, float* V, float* E, const float* dgrad, const float* coef, float lr,
                             float wd, float beta1, float beta2, float eps, int step, float ema_decay, int do_adam,
                             int do_ema, void* stream) {
  if (nchunks == 0) return 0;
  const OptScalars s = make_opt_scalars(lr, wd, beta1, beta2, eps, step, ema_decay, do_adam, do_ema);
  hipStream_t st = (hipStream_t)stream;
  if (do_adam) chunk_key_range_kernel<<<cdiv(nchunks, 256), 256, 0, st>>>(chunks, nchunks, segs, krange);
  adamw_ema_kernel<false><<<nchunks, 256, 0, st>>>(chunks, segs, krange, P, M, V, E, dgrad, coef, s);
  return check_launch("adamw_ema");
}

extern "C" int ctr_adamw_ema_hist(const ctr_opt_chunk_t* chunks, int nchunks, const ctr_opt_seg_t* segs,
                                  uint32_t* krange, float* P, float* M, float* V, float* E, const float* dgrad,
                                  const float* coef, float lr, float wd, float beta1, float beta2, float eps, int step,
                                  float ema_decay, int do_ema, void* hist, int tick, void* stream) {
  CTR_REQUIRE(hist != nullptr && tick > 0, "ctr_adamw_ema_hist: bad history / tick");
  const OptScalars s = make_opt_scalars(lr, wd, beta1, beta2, eps, step, ema_decay, 1, do_ema);
  hipStream_t st = (hipStream_t)stream;
  if (nchunks > 0)     // one launch: the history record and any sparse chunk's key range inside (adamw_ema_kernel<true>)
    adamw_ema_kernel<true><<<nchunks, 256, 0, st>>>(chunks, segs, krange, P, M, V, E, dgrad, coef, s, (OptScalars*)hist,
                                                    tick);
  else
    chunk_key_range_kernel<<<1, 256, 0, st>>>(chunks, 0, segs, krange, (OptScalars*)hist, tick, s);
  return check_launch("adamw_ema_hist");
}

extern "C" int ctr_norm_nparts_per_call(void) { return NORM_BLOCKS; }

extern "C" int ctr_sqnorm_dense(const float* x, long n, float* part, void* stream) {
  sqnorm_dense_kernel<<<NORM_BLOCKS, 256, 0, (hipStream_t)stream>>>(x, n, part);
  return check_launch("sqnorm_dense");
}

extern "C" int ctr_sqnorm_rows(const uint32_t* keys, const float* G, const uint32_t* n_uniq, int width, int ld,
                               uint32_t invalid_key, float* part, void* stream) {
  sqnorm_rows_kernel<<<NORM_BLOCKS, 256, 0, (hipStream_t)stream>>>(keys, G, n_uniq, width, ld, invalid_key, part);
  return check_launch("sqnorm_rows");
}

extern "C" int ctr_sqnorm_all(const float* x, long n, const ctr_sqnorm_rows_t* rows, int nrows, uint32_t invalid_key,
                              float* part, void* stream) {
  CTR_REQUIRE(nrows >= 0 && nrows <= CTR_SQNORM_MAX_ROWS && (nrows == 0 || rows), "ctr_sqnorm_all: bad row tables");
  SqnormRowsSet rs{};
  for (int j = 0; j < nrows; ++j) rs.r[j] = rows[j];
  sqnorm_all_kernel<<<dim3(NORM_BLOCKS, 1 + nrows), 256, 0, (hipStream_t)stream>>>(x, n, rs, invalid_key, part);
  return check_launch("sqnorm_all");
}

extern "C" int ctr_clip_finalize(const float* part, int nparts, float max_norm, float grad_scale, float* out,
                                 void* stream) {
  clip_finalize_kernel<<<1, 256, 0, (hipStream_t)stream>>>(part, nparts, max_norm, grad_scale, out);
  return check_launch("clip_finalize");
}

// Row/column reductions on the hot path:
//   rmsnorm fwd/bwd : src/models/dare.py:6-13 (encoder norms, rows of D), src/models/qnn_alpha.py:6-12,
//                     109-113 (QNN pre-norm over F*D = 6400)
//   colsum          : bias / gain gradients (sum over the batch rows), deterministic two-level tree
//   loss            : bce_wll_style, src/train.py:71-90 (+ aux term src/train.py:165-168) fused with
//                     its backward seed (class-balanced: counts are a batch-wide reduction)
#include "common.h"
#include "ctr_hip.h"

namespace ctr {

// ---------------- big-row RMSNorm forward: one workgroup per row ----------------
__global__ __launch_bounds__(256) void rmsnorm_fwd_big(const float* __restrict__ x, long ldx, int N,
                                                       const float* __restrict__ w, float eps,
                                                       float* __restrict__ y, long ldy, float* __restrict__ r) {
  __shared__ float red[4];
  const long row = blockIdx.x;
  const float* xr = x + row * ldx;
  float ss = 0.f;
  for (int j = threadIdx.x; j < N; j += 256) ss = fmaf(xr[j], xr[j], ss);
  ss = block_sum(ss, red);
  const float rr = 1.0f / sqrtf(ss / (float)N + eps);
  if (threadIdx.x == 0) r[row] = rr;
  float* yr = y + row * ldy;
  for (int j = threadIdx.x; j < N; j += 256) yr[j] = w[j] * xr[j] * rr;
}

// big rows held in registers: 16-byte loads, NQ float4 per thread (N <= 1024 * NQ, N % 4 == 0, 16-byte
// aligned rows) -- one read of the row instead of two, and a quarter of the load instructions
template <int NQ>
__global__ __launch_bounds__(256) void rmsnorm_fwd_big_vec(const float* __restrict__ x, long ldx, int N,
                                                           const float* __restrict__ w, float eps,
                                                           float* __restrict__ y, long ldy, float* __restrict__ r,
                                                           __bf16* __restrict__ ybf = nullptr, long ldybf = 0) {
  typedef float f4 __attribute__((ext_vector_type(4)));
  typedef __bf16 b4 __attribute__((ext_vector_type(4)));
  __shared__ float red[4];
  const long row = blockIdx.x;
  const f4* xr = (const f4*)(x + row * ldx);
  const int n4 = N >> 2;
  f4 v[NQ], wv[NQ];
  float ss = 0.f;
  const f4* w4 = (const f4*)w;
#pragma unroll
  for (int k = 0; k < NQ; ++k) {
    const int j = threadIdx.x + 256 * k;
    v[k] = j < n4 ? xr[j] : f4{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int k = 0; k < NQ; ++k) {       // the weights too, before the row reduction's barrier (not one round trip after)
    const int j = threadIdx.x + 256 * k;
    wv[k] = w4[j < n4 ? j : 0];
  }
#pragma unroll
  for (int k = 0; k < NQ; ++k) {
    ss = fmaf(v[k].x, v[k].x, ss);
    ss = fmaf(v[k].y, v[k].y, ss);
    ss = fmaf(v[k].z, v[k].z, ss);
    ss = fmaf(v[k].w, v[k].w, ss);
  }
  ss = block_sum(ss, red);
  const float rr = 1.0f / sqrtf(ss / (float)N + eps);
  if (threadIdx.x == 0) r[row] = rr;
  f4* yr = (f4*)(y + row * ldy);
#pragma unroll
  for (int k = 0; k < NQ; ++k) {
    const int j = threadIdx.x + 256 * k;
    if (j < n4) {
      const f4 o = wv[k] * v[k] * rr;
      if (y) yr[j] = o;
      if (ybf) *(b4*)(ybf + row * ldybf + 4 * j) = __builtin_convertvector(o, b4);   // amp: the GEMM's bf16 image
    }
  }
}

// ---------------- RMSNorm backward ----------------
// dh = w*dy*r - h * r^3/N * sum_k(w_k dy_k h_k) (+ add);  dw partial = sum_rows dy*h*r
// small rows (N <= 64): TPR threads per row, each covers N/TPR columns (ceil); rows_per_block rows.
template <int TPR>
__global__ __launch_bounds__(256) void rmsnorm_bwd_small(const float* __restrict__ dy, long ldy,
                                                         const float* __restrict__ h, long ldh,
                                                         const float* __restrict__ r, const float* __restrict__ w,
                                                         int M, int N, float* __restrict__ dh, long lddh,
                                                         const float* __restrict__ add, long ld_add,
                                                         int rows_per_block, float* __restrict__ dw_part) {
  constexpr int CPT = 64 / TPR;   // columns per thread (N <= 64)
  const int sub = threadIdx.x % TPR, rr = threadIdx.x / TPR;
  constexpr int RPP = 256 / TPR;
  const int m0 = blockIdx.x * rows_per_block, m1 = min(M, m0 + rows_per_block);
  float dwacc[CPT];
#pragma unroll
  for (int c = 0; c < CPT; ++c) dwacc[c] = 0.f;
  for (int mb = m0; mb < m1; mb += RPP) {
    const int m = mb + rr;
    const bool ok = m < m1;
    float gy[CPT], hv[CPT];
    float dot = 0.f;
    const float rm = ok ? r[m] : 0.f;
#pragma unroll
    for (int c = 0; c < CPT; ++c) {
      const int n = sub + c * TPR;
      gy[c] = 0.f;
      hv[c] = 0.f;
      if (ok && n < N) {
        gy[c] = dy[(long)m * ldy + n];
        hv[c] = h[(long)m * ldh + n];
        dot = fmaf(w[n] * gy[c], hv[c], dot);
      }
    }
    dot = group_sum<TPR>(dot);
    const float coef = rm * rm * rm / (float)N * dot;
#pragma unroll
    for (int c = 0; c < CPT; ++c) {
      const int n = sub + c * TPR;
      if (ok && n < N) {
        float g = w[n] * gy[c] * rm - hv[c] * coef;
        if (add) g += add[(long)m * ld_add + n];
        dh[(long)m * lddh + n] = g;
        dwacc[c] = fmaf(gy[c] * hv[c], rm, dwacc[c]);
      }
    }
  }
  // reduce dw across the RPP row groups of the block (fixed order through LDS)
  __shared__ float sdw[256 * CPT];
#pragma unroll
  for (int c = 0; c < CPT; ++c) sdw[threadIdx.x * CPT + c] = dwacc[c];
  __syncthreads();
  for (int n = threadIdx.x; n < N; n += 256) {
    const int s = n % TPR, c = n / TPR;
    float acc = 0.f;
    for (int g = 0; g < RPP; ++g) acc += sdw[(g * TPR + s) * CPT + c];
    dw_part[(long)blockIdx.x * N + n] = acc;
  }
}

// big rows (QNN pre-norm, N = F*D = 6400): a workgroup takes rows_per_block rows; each thread keeps its
// NPT columns of w*dy and h in registers, so dy and h are read once, and accumulates its columns'
// dw partials across the rows in registers (dw_part: one row per workgroup).
template <int NPT>
__global__ __launch_bounds__(256) void rmsnorm_bwd_big(const float* __restrict__ dy, long ldy,
                                                       const float* __restrict__ h, long ldh,
                                                       const float* __restrict__ r, const float* __restrict__ w,
                                                       int M, int N, float* __restrict__ dh, long lddh,
                                                       int rows_per_block, float* __restrict__ dw_part) {
  __shared__ float red[4];
  const int m0 = blockIdx.x * rows_per_block, m1 = min(M, m0 + rows_per_block);
  float wv[NPT], acc[NPT];
#pragma unroll
  for (int k = 0; k < NPT; ++k) {
    const int n = threadIdx.x + 256 * k;
    wv[k] = n < N ? w[n] : 0.f;
    acc[k] = 0.f;
  }
  for (int m = m0; m < m1; ++m) {
    const float* gy = dy + (long)m * ldy;
    const float* hv = h + (long)m * ldh;
    const float rm = r[m];
    float g[NPT], hh[NPT];
    float dot = 0.f;
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
      const int n = threadIdx.x + 256 * k;
      g[k] = n < N ? gy[n] : 0.f;
      hh[k] = n < N ? hv[n] : 0.f;
      dot = fmaf(wv[k] * g[k], hh[k], dot);
      acc[k] = fmaf(g[k] * hh[k], rm, acc[k]);
    }
    dot = block_sum(dot, red);
    const float coef = rm * rm * rm / (float)N * dot;
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
      const int n = threadIdx.x + 256 * k;
      if (n < N) dh[(long)m * lddh + n] = wv[k] * g[k] * rm - hh[k] * coef;
    }
  }
#pragma unroll
  for (int k = 0; k < NPT; ++k) {
    const int n = threadIdx.x + 256 * k;
    if (n < N) dw_part[(long)blockIdx.x * N + n] = acc[k];
  }
}

// big rows with 16-byte loads (N % 4 == 0, aligned rows; NQ float4 per thread, NT threads): the next row's dy
// and h are loaded before this row's block reduction, so the load latency hides behind the reduction barrier.
// NT = 1024 covers rows up to 16384 wide in one pass over dy and h (the QNN input norm at D = 64).
template <int NQ, int NT = 256>
__global__ __launch_bounds__(NT) void rmsnorm_bwd_big_vec(const float* __restrict__ dy, long ldy,
                                                           const float* __restrict__ h, long ldh,
                                                           const float* __restrict__ r, const float* __restrict__ w,
                                                           int M, int N, float* __restrict__ dh, long lddh,
                                                           int rows_per_block, float* __restrict__ dw_part) {
  typedef float f4 __attribute__((ext_vector_type(4)));
  __shared__ float red[NT / 64];
  const int m0 = blockIdx.x * rows_per_block, m1 = min(M, m0 + rows_per_block);
  const int n4 = N >> 2;
  f4 wv[NQ], acc[NQ], g[NQ], hh[NQ];
#pragma unroll
  for (int k = 0; k < NQ; ++k) {
    const int j = threadIdx.x + NT * k;
    wv[k] = j < n4 ? ((const f4*)w)[j] : f4{0.f, 0.f, 0.f, 0.f};
    acc[k] = f4{0.f, 0.f, 0.f, 0.f};
  }
  auto load = [&](int m, f4* gg, f4* hv) {
    const f4* gy = (const f4*)(dy + (long)m * ldy);
    const f4* hr = (const f4*)(h + (long)m * ldh);
#pragma unroll
    for (int k = 0; k < NQ; ++k) {
      const int j = threadIdx.x + NT * k;
      gg[k] = j < n4 ? gy[j] : f4{0.f, 0.f, 0.f, 0.f};
      hv[k] = j < n4 ? hr[j] : f4{0.f, 0.f, 0.f, 0.f};
    }
  };
  if (m0 < m1) load(m0, g, hh);
  for (int m = m0; m < m1; ++m) {
    const float rm = r[m];
    float dot = 0.f;
#pragma unroll
    for (int k = 0; k < NQ; ++k) {
      dot = fmaf(wv[k].x * g[k].x, hh[k].x, dot);
      dot = fmaf(wv[k].y * g[k].y, hh[k].y, dot);
      dot = fmaf(wv[k].z * g[k].z, hh[k].z, dot);
      dot = fmaf(wv[k].w * g[k].w, hh[k].w, dot);
      acc[k].x = fmaf(g[k].x * hh[k].x, rm, acc[k].x);
      acc[k].y = fmaf(g[k].y * hh[k].y, rm, acc[k].y);
      acc[k].z = fmaf(g[k].z * hh[k].z, rm, acc[k].z);
      acc[k].w = fmaf(g[k].w * hh[k].w, rm, acc[k].w);
    }
    f4 gn[NQ], hn[NQ];
    if (m + 1 < m1) load(m + 1, gn, hn);
    dot = block_sum(dot, red);
    const float coef = rm * rm * rm / (float)N * dot;
    f4* o = (f4*)(dh + (long)m * lddh);
#pragma unroll
    for (int k = 0; k < NQ; ++k) {
      const int j = threadIdx.x + NT * k;
      if (j < n4) o[j] = wv[k] * g[k] * rm - hh[k] * coef;
    }
    if (m + 1 < m1) {
#pragma unroll
      for (int k = 0; k < NQ; ++k) {
        g[k] = gn[k];
        hh[k] = hn[k];
      }
    }
  }
  f4* dp = (f4*)(dw_part + (long)blockIdx.x * N);
#pragma unroll
  for (int k = 0; k < NQ; ++k) {
    const int j = threadIdx.x + NT * k;
    if (j < n4) dp[j] = acc[k];
  }
}

// fallback for rows wider than 32 * 256: two passes over the row
__global__ __launch_bounds__(256) void rmsnorm_bwd_huge(const float* __restrict__ dy, long ldy,
                                                        const float* __restrict__ h, long ldh,
                                                        const float* __restrict__ r, const float* __restrict__ w,
                                                        int M, int N, float* __restrict__ dh, long lddh,
                                                        int rows_per_block, float* __restrict__ dw_part) {
  __shared__ float red[4];
  const int m0 = blockIdx.x * rows_per_block, m1 = min(M, m0 + rows_per_block);
  for (int m = m0; m < m1; ++m) {
    const float* gy = dy + (long)m * ldy;
    const float* hv = h + (long)m * ldh;
    const float rm = r[m];
    float dot = 0.f;
    for (int n = threadIdx.x; n < N; n += 256) dot = fmaf(w[n] * gy[n], hv[n], dot);
    dot = block_sum(dot, red);
    const float coef = rm * rm * rm / (float)N * dot;
    for (int n = threadIdx.x; n < N; n += 256) dh[(long)m * lddh + n] = w[n] * gy[n] * rm - hv[n] * coef;
  }
  for (int n = threadIdx.x; n < N; n += 256) {
    float acc = 0.f;
    for (int m = m0; m < m1; ++m) acc = fmaf(dy[(long)m * ldy + n] * h[(long)m * ldh + n], r[m], acc);
    dw_part[(long)blockIdx.x * N + n] = acc;
  }
}

// ---------------- column sums: out[n] = sum_m X[m, n] (two-level, fixed order) ----------------
// block = (64-column tile) x (row chunk); 4 row groups of 64 lanes stride the chunk, combined in order
__global__ __launch_bounds__(256) void colsum_partial(const float* __restrict__ X, long ld, int M, int N,
                                                      int rows_per_block, float* __restrict__ part) {
  __shared__ float red[4][64];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int n = blockIdx.x * 64 + tx;
  const int m0 = blockIdx.y * rows_per_block, m1 = min(M, m0 + rows_per_block);
  float s = 0.f;
  if (n < N) {
    int m = m0 + ty;
    for (; m + 12 < m1; m += 16) {
      const float a0 = X[(long)m * ld + n], a1 = X[(long)(m + 4) * ld + n];
      const float a2 = X[(long)(m + 8) * ld + n], a3 = X[(long)(m + 12) * ld + n];
      s += a0;
      s += a1;
      s += a2;
      s += a3;
    }
    for (; m < m1; m += 4) s += X[(long)m * ld + n];
  }
  red[ty][tx] = s;
  __syncthreads();
  if (ty == 0 && n < N) part[(long)blockIdx.y * N + n] = ((red[0][tx] + red[1][tx]) + red[2][tx]) + red[3][tx];
}

// same reduction over 256-column tiles, a lane owning four adjacent columns (one 16-byte load per row;
// X 16-byte aligned, ld and N multiples of 4): each column keeps the scalar kernel's summation order
__global__ __launch_bounds__(256) void colsum_partial_v4(const float* __restrict__ X, long ld, int M, int N,
                                                         int rows_per_block, float* __restrict__ part) {
  __shared__ float4 red[4][64];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int n = (blockIdx.x * 64 + tx) * 4;
  const int m0 = blockIdx.y * rows_per_block, m1 = min(M, m0 + rows_per_block);
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (n < N) {
    int m = m0 + ty;
    for (; m + 12 < m1; m += 16) {
      const float4 a0 = *reinterpret_cast<const float4*>(X + (long)m * ld + n);
      const float4 a1 = *reinterpret_cast<const float4*>(X + (long)(m + 4) * ld + n);
      const float4 a2 = *reinterpret_cast<const float4*>(X + (long)(m + 8) * ld + n);
      const float4 a3 = *reinterpret_cast<const float4*>(X + (long)(m + 12) * ld + n);
      s.x += a0.x; s.y += a0.y; s.z += a0.z; s.w += a0.w;
      s.x += a1.x; s.y += a1.y; s.z += a1.z; s.w += a1.w;
      s.x += a2.x; s.y += a2.y; s.z += a2.z; s.w += a2.w;
      s.x += a3.x; s.y += a3.y; s.z += a3.z; s.w += a3.w;
    }
    for (; m < m1; m += 4) {
      const float4 a = *reinterpret_cast<const float4*>(X + (long)m * ld + n);
      s.x += a.x; s.y += a.y; s.z += a.z; s.w += a.w;
    }
  }
  red[ty][tx] = s;
  __syncthreads();
  if (ty == 0 && n < N) {
    const float4 r0 = red[0][tx], r1 = red[1][tx], r2 = red[2][tx], r3 = red[3][tx];
    float4 o;
    o.x = ((r0.x + r1.x) + r2.x) + r3.x;
    o.y = ((r0.y + r1.y) + r2.y) + r3.y;
    o.z = ((r0.z + r1.z) + r2.z) + r3.z;
    o.w = ((r0.w + r1.w) + r2.w) + r3.w;
    *reinterpret_cast<float4*>(part + (long)blockIdx.y * N + n) = o;
  }
}

// few partials (a slab of a few hundred rows): one thread per column, partials summed in order, the
// loads of a partial row coalesced across the threads
__global__ __launch_bounds__(256) void colsum_final_cols(const float* __restrict__ part, int nparts, int N, float div,
                                                         float* __restrict__ out) {
  const int n = blockIdx.x * 256 + threadIdx.x;
  if (n >= N) return;
  float s = 0.f;
  for (int p = 0; p < nparts; ++p) s += part[(long)p * N + n];
  out[n] = div == 1.0f ? s : s / div;
}

// one wave per column: lanes stride the partials, fixed xor-tree combine
__global__ __launch_bounds__(64) void colsum_final(const float* __restrict__ part, int nparts, int N, float div,
                                                   float* __restrict__ out) {
  const int n = blockIdx.x;
  float s = 0.f;
  for (int p = threadIdx.x; p < nparts; p += 64) s += part[(long)p * N + n];
  s = wave_sum(s);
  if (threadIdx.x == 0) out[n] = div == 1.0f ? s : s / div;
}

// ---------------- several column sums in one launch pair (ctr_colsum_multi) ----------------
// The backward's per-layer weight-grad slabs (fused FFN, encoder projections) are summed together once the
// encoder layers are done: two launches instead of two per slab.  Per segment the partial pass is
// colsum_partial_v4's (256-column tiles, row chunks of rpb rows, four row groups combined in order) and the
// final pass sums the chunk partials in chunk order -- deterministic, one fixed order per segment.
struct ColsumSegs {
  int nseg;
  int blk0[CTR_COLSUM_MAXSEG + 1];   // partial-pass block prefix over the segments
  int q0[CTR_COLSUM_MAXSEG + 1];     // final-pass column-quad prefix
  const float* X[CTR_COLSUM_MAXSEG];
  float* out[CTR_COLSUM_MAXSEG];
  long ld[CTR_COLSUM_MAXSEG];
  long ws0[CTR_COLSUM_MAXSEG];       // float offset of the segment's partials in the workspace
  int M[CTR_COLSUM_MAXSEG], N[CTR_COLSUM_MAXSEG], rpb[CTR_COLSUM_MAXSEG], np[CTR_COLSUM_MAXSEG];
  int ctiles[CTR_COLSUM_MAXSEG];
  float div[CTR_COLSUM_MAXSEG];
};

__device__ __forceinline__ int seg_of(const int* pre, int n, int x) {
  int s = 0;
  while (s + 1 < n && pre[s + 1] <= x) ++s;
  return s;
}

__global__ __launch_bounds__(256) void colsum_multi_partial(ColsumSegs S, float* __restrict__ ws) {
  __shared__ float4 red[4][64];
  const int s = seg_of(S.blk0, S.nseg, blockIdx.x);
  const int local = blockIdx.x - S.blk0[s];
  const int tile = local % S.ctiles[s], part = local / S.ctiles[s];
  const float* X = S.X[s];
  const long ld = S.ld[s];
  const int M = S.M[s], N = S.N[s];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int n = (tile * 64 + tx) * 4;
  const int m0 = part * S.rpb[s], m1 = min(M, m0 + S.rpb[s]);
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  if (n < N) {
    int m = m0 + ty;
    for (; m + 12 < m1; m += 16) {
      const float4 a0 = *reinterpret_cast<const float4*>(X + (long)m * ld + n);
      const float4 a1 = *reinterpret_cast<const float4*>(X + (long)(m + 4) * ld + n);
      const float4 a2 = *reinterpret_cast<const float4*>(X + (long)(m + 8) * ld + n);
      const float4 a3 = *reinterpret_cast<const float4*>(X + (long)(m + 12) * ld + n);
      a.x += a0.x; a.y += a0.y; a.z += a0.z; a.w += a0.w;
      a.x += a1.x; a.y += a1.y; a.z += a1.z; a.w += a1.w;
      a.x += a2.x; a.y += a2.y; a.z += a2.z; a.w += a2.w;
      a.x += a3.x; a.y += a3.y; a.z += a3.z; a.w += a3.w;
    }
    for (; m < m1; m += 4) {
      const float4 v = *reinterpret_cast<const float4*>(X + (long)m * ld + n);
      a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
    }
  }
  red[ty][tx] = a;
  __syncthreads();
  if (ty == 0 && n < N) {
    const float4 r0 = red[0][tx], r1 = red[1][tx], r2 = red[2][tx], r3 = red[3][tx];
    float4 o;
    o.x = ((r0.x + r1.x) + r2.x) + r3.x;
    o.y = ((r0.y + r1.y) + r2.y) + r3.y;
    o.z = ((r0.z + r1.z) + r2.z) + r3.z;
    o.w = ((r0.w + r1.w) + r2.w) + r3.w;
    *reinterpret_cast<float4*>(ws + S.ws0[s] + (long)part * N + n) = o;
  }
}

__global__ __launch_bounds__(256) void colsum_multi_final(ColsumSegs S, const float* __restrict__ ws) {
  const int q = blockIdx.x * 256 + threadIdx.x;
  if (q >= S.q0[S.nseg]) return;
  const int s = seg_of(S.q0, S.nseg, q);
  const int n = 4 * (q - S.q0[s]), N = S.N[s];
  const float* p = ws + S.ws0[s] + n;
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int k = 0; k < S.np[s]; ++k) {
    const float4 v = *reinterpret_cast<const float4*>(p + (long)k * N);
    a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
  }
  const float d = S.div[s];
  if (d != 1.0f) {
    a.x /= d; a.y /= d; a.z /= d; a.w /= d;
  }
  float* o = S.out[s] + n;
  o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w;    // out need not be 16-byte aligned
}

// row chunk of a segment's partial pass: about 1024 blocks over the segment, at least 64 rows
static int multi_rpb(int M, int N) {
  const int ctiles = cdiv(N, 256);
  return std::min(4096, std::max(64, cdiv((long)M * ctiles, 1024)));
}

static bool multi_seg_ok(const ctr_colsum_seg_t& g) {
  return g.X && g.out && g.M > 0 && g.N > 0 && (g.N & 3) == 0 && (g.ld & 3) == 0 && (((uintptr_t)g.X) & 15) == 0 &&
         g.ld >= g.N;
}

// ---------------- loss: bce_wll_style(logits) + aux_w * bce_wll_style(aux) and d/dz ----------------
__global__ __launch_bounds__(1024) void loss_kernel(const float* __restrict__ z, const float* __restrict__ za,
                                                    const float* __restrict__ y, int B, float aux_w,
                                                    float* __restrict__ loss, float* __restrict__ dz,
                                                    float* __restrict__ dza) {
  __shared__ float red[16][5];
  float npos = 0.f, sp = 0.f, sn = 0.f, spa = 0.f, sna = 0.f;
  // a thread's elements i = t, t + 1024, ... in chunks of four whose loads are issued together (one round trip
  // per chunk instead of per element: the step's batch of 4096 is one chunk); the same per-thread order
  for (int i0 = threadIdx.x; i0 < B; i0 += 4 * 1024) {
    float yv[4], zv[4], zav[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = min(i0 + 1024 * u, B - 1);
      yv[u] = y[i];
      zv[u] = z[i];
      zav[u] = za ? za[i] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (i0 + 1024 * u >= B) break;
      const bool pos = yv[u] > 0.5f;
      npos += pos ? 1.f : 0.f;
      if (pos) sp += softplus_f(-zv[u]);
      else sn += softplus_f(zv[u]);
      if (za) {
        if (pos) spa += softplus_f(-zav[u]);
        else sna += softplus_f(zav[u]);
      }
    }
  }
  {  // the five block sums in one LDS round (each: wave sums, then the 16 waves in order)
    float v[5] = {wave_sum(npos), wave_sum(sp), wave_sum(sn), wave_sum(spa), wave_sum(sna)};
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0)
#pragma unroll
      for (int j = 0; j < 5; ++j) red[w][j] = v[j];
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 5; ++j) {
      float t = 0.f;
      for (int i = 0; i < 16; ++i) t += red[i][j];
      v[j] = t;
    }
    npos = v[0];
    sp = v[1];
    sn = v[2];
    spa = v[3];
    sna = v[4];
  }
  const float nneg = (float)B - npos;
  const float lp = npos > 0.f ? sp / npos : 0.f, ln = nneg > 0.f ? sn / nneg : 0.f;
  float L = 0.5f * (lp + ln);
  if (za) {
    const float lpa = npos > 0.f ? spa / npos : 0.f, lna = nneg > 0.f ? sna / nneg : 0.f;
    L = L + aux_w * (0.5f * (lpa + lna));
  }
  if (threadIdx.x == 0) loss[0] = L;
  // d softplus(x)/dx = sigmoid(x) (torch: 1 above the threshold 20)
  for (int i0 = threadIdx.x; i0 < B; i0 += 4 * 1024) {
    float yv[4], zv[4], zav[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = min(i0 + 1024 * u, B - 1);
      yv[u] = y[i];
      zv[u] = z[i];
      zav[u] = za ? za[i] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = i0 + 1024 * u;
      if (i >= B) break;
      const bool pos = yv[u] > 0.5f;
      float g;
      if (pos) {
        const float x = -zv[u];
        g = -(x > 20.f ? 1.f : sigmoid_f(x)) * (0.5f / npos);
      } else {
        const float x = zv[u];
        g = (x > 20.f ? 1.f : sigmoid_f(x)) * (0.5f / nneg);
      }
      dz[i] = g;
      if (za) {
        float ga;
        if (pos) {
          const float x = -zav[u];
          ga = -(x > 20.f ? 1.f : sigmoid_f(x)) * (0.5f / npos);
        } else {
          const float x = zav[u];
          ga = (x > 20.f ? 1.f : sigmoid_f(x)) * (0.5f / nneg);
        }
        dza[i] = aux_w * ga;
      }
    }
  }
}

}  // namespace ctr

using namespace ctr;

extern "C" int ctr_rmsnorm_fwd(const float* x, long ldx, int M, int N, const float* w, float eps, float* y, long ldy,
                               float* r, void* stream) {
  if (M == 0) return 0;
  const bool vec = (N % 4) == 0 && (ldx % 4) == 0 && (ldy % 4) == 0 && ((((uintptr_t)x) | ((uintptr_t)y) |
                                                                        ((uintptr_t)w)) & 15) == 0;
  if (vec && N <= 1024 * 8)
    rmsnorm_fwd_big_vec<8><<<M, 256, 0, (hipStream_t)stream>>>(x, ldx, N, w, eps, y, ldy, r);
  else if (vec && N <= 1024 * 16)
    rmsnorm_fwd_big_vec<16><<<M, 256, 0, (hipStream_t)stream>>>(x, ldx, N, w, eps, y, ldy, r);
  else
    rmsnorm_fwd_big<<<M, 256, 0, (hipStream_t)stream>>>(x, ldx, N, w, eps, y, ldy, r);
  return check_launch("rmsnorm_fwd");
}

extern "C" int ctr_rmsnorm_fwd_bf(const float* x, long ldx, int M, int N, const float* w, float eps, float* y, long ldy,
                                  float* r, void* ybf, long ldybf, void* stream) {
  if (M == 0) return 0;
  const bool vec = (N % 4) == 0 && (ldx % 4) == 0 && (ldy % 4) == 0 && (ldybf % 4) == 0 &&
                   ((((uintptr_t)x) | ((uintptr_t)y) | ((uintptr_t)w)) & 15) == 0 && (((uintptr_t)ybf) & 7) == 0;
  CTR_REQUIRE(vec && N <= 1024 * 16, "ctr_rmsnorm_fwd_bf: needs N % 4 == 0, N <= 16384 and aligned rows");
  CTR_REQUIRE(ybf != nullptr, "ctr_rmsnorm_fwd_bf: the bf16 image is required (y may be null)");
  if (N <= 1024 * 8)
    rmsnorm_fwd_big_vec<8><<<M, 256, 0, (hipStream_t)stream>>>(x, ldx, N, w, eps, y, ldy, r, (__bf16*)ybf, ldybf);
  else
    rmsnorm_fwd_big_vec<16><<<M, 256, 0, (hipStream_t)stream>>>(x, ldx, N, w, eps, y, ldy, r, (__bf16*)ybf, ldybf);
  return check_launch("rmsnorm_fwd_bf");
}

// big rows: ~512 workgroups (2 per CU), at least 2 rows each
static int big_rows_per_block(int M) { return std::max(2, cdiv(M, 512)); }

extern "C" int ctr_rmsnorm_bwd_nparts(int M, int N) {
  if (N <= 64) return cdiv(M, 256);
  return cdiv(M, big_rows_per_block(M));
}

extern "C" int ctr_rmsnorm_bwd(const float* dy, long ldy, const float* h, long ldh, const float* r, const float* w,
                               int M, int N, float* dh, long lddh, const float* add, long ld_add, float* dw_part,
                               void* stream) {
  if (M == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  if (N <= 64) {
    const int rpb = 256;
    const int nb = cdiv(M, rpb);
    if (N <= 16) rmsnorm_bwd_small<4><<<nb, 256, 0, s>>>(dy, ldy, h, ldh, r, w, M, N, dh, lddh, add, ld_add, rpb, dw_part);
    else if (N <= 32) rmsnorm_bwd_small<8><<<nb, 256, 0, s>>>(dy, ldy, h, ldh, r, w, M, N, dh, lddh, add, ld_add, rpb, dw_part);
    else rmsnorm_bwd_small<16><<<nb, 256, 0, s>>>(dy, ldy, h, ldh, r, w, M, N, dh, lddh, add, ld_add, rpb, dw_part);
  } else {
    CTR_REQUIRE(add == nullptr, "big-row rmsnorm bwd: add unsupported");
    const int rpb = big_rows_per_block(M);
    const int nb = cdiv(M, rpb);
    const bool vec = (N % 4) == 0 && (ldy % 4) == 0 && (ldh % 4) == 0 && (lddh % 4) == 0 &&
                     ((((uintptr_t)dy) | ((uintptr_t)h) | ((uintptr_t)w) | ((uintptr_t)dh) | ((uintptr_t)dw_part)) &
                      15) == 0;
    if (vec && N > 256 * 8 && N <= 1024 * 8)
      rmsnorm_bwd_big_vec<8><<<nb, 256, 0, s>>>(dy, ldy, h, ldh, r, w, M, N, dh, lddh, rpb, dw_part);
    else if (vec && N > 1024 * 8 && N <= 1024 * 16)
      rmsnorm_bwd_big_vec<4, 1024><<<nb, 1024, 0, s>>>(dy, ldy, h, ldh, r, w, M, N, dh, lddh, rpb, dw_part);
    else if (N <= 256 * 8) rmsnorm_bwd_big<8><<<nb, 256, 0, s>>>(dy, ldy, h, ldh, r, w, M, N, dh, lddh, rpb, dw_part);
    else if (N <= 256 * 16) rmsnorm_bwd_big<16><<<nb, 256, 0, s>>>(dy, ldy, h, ldh, r, w, M, N, dh, lddh, rpb, dw_part);
    else if (N <= 256 * 32) rmsnorm_bwd_big<32><<<nb, 256, 0, s>>>(dy, ldy, h, ldh, r, w, M, N, dh, lddh, rpb, dw_part);
    else rmsnorm_bwd_huge<<<nb, 256, 0, s>>>(dy, ldy, h, ldh, r, w, M, N, dh, lddh, rpb, dw_part);
  }
  return check_launch("rmsnorm_bwd");
}

// float4 form: target block count and minimum row chunk (multiple of 16)
#ifndef COLSUM_V4_BLOCKS
#define COLSUM_V4_BLOCKS 1024
#endif
#ifndef COLSUM_V4_MIN_ROWS
#define COLSUM_V4_MIN_ROWS 64
#endif

extern "C" size_t ctr_colsum_ws_size(int M, int N) {
  return (size_t)cdiv(M, std::min(64, COLSUM_V4_MIN_ROWS)) * N * sizeof(float);
}

// out[n] = (sum_m X[m, n]) / div   (div = 1 for plain sums, B for torch .mean(dim=0))
extern "C" int ctr_colsum(const float* X, long ld, int M, int N, float div, float* out, float* ws, void* stream) {
  if (N == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  const bool v4 = (N % 4) == 0 && (ld % 4) == 0 && (((uintptr_t)X) & 15) == 0;
  const int ctiles = cdiv(N, v4 ? 256 : 64);
  const int rpb = v4 ? std::min(4096, std::max(COLSUM_V4_MIN_ROWS, cdiv((long)M * ctiles, COLSUM_V4_BLOCKS)))
                     : std::min(4096, std::max(64, cdiv((long)M * ctiles, 1024)));   // ~1024 blocks
  const int np = M > 0 ? cdiv(M, rpb) : 0;
  if (np > 0 && v4) colsum_partial_v4<<<dim3(ctiles, np), 256, 0, s>>>(X, ld, M, N, rpb, ws);
  else if (np > 0) colsum_partial<<<dim3(ctiles, np), 256, 0, s>>>(X, ld, M, N, rpb, ws);
  if (np <= 16) colsum_final_cols<<<cdiv(N, 256), 256, 0, s>>>(ws, np, N, div, out);
  else colsum_final<<<N, 64, 0, s>>>(ws, np, N, div, out);
  return check_launch("colsum");
}

extern "C" int ctr_colsum_multi_ok(const ctr_colsum_seg_t* seg) { return seg && multi_seg_ok(*seg) ? 1 : 0; }

extern "C" size_t ctr_colsum_multi_ws_size(const ctr_colsum_seg_t* segs, int nseg) {
  size_t n = 0;
  for (int i = 0; i < nseg; ++i) n += (size_t)cdiv(segs[i].M, multi_rpb(segs[i].M, segs[i].N)) * segs[i].N;
  return n * sizeof(float);
}

extern "C" int ctr_colsum_multi(const ctr_colsum_seg_t* segs, int nseg, float* ws, size_t ws_bytes, void* stream) {
  CTR_REQUIRE(nseg >= 0 && nseg <= CTR_COLSUM_MAXSEG, "ctr_colsum_multi: 0 .. CTR_COLSUM_MAXSEG segments");
  if (nseg == 0) return 0;
  CTR_REQUIRE(ws_bytes >= ctr_colsum_multi_ws_size(segs, nseg), "ctr_colsum_multi: workspace too small");
  ColsumSegs S = {};
  S.nseg = nseg;
  long wsoff = 0;
  for (int i = 0; i < nseg; ++i) {
    const ctr_colsum_seg_t& g = segs[i];
    CTR_REQUIRE(multi_seg_ok(g), "ctr_colsum_multi: a segment needs M, N > 0, N and ld multiples of 4, 16-byte X");
    S.X[i] = g.X; S.out[i] = g.out; S.ld[i] = g.ld; S.M[i] = g.M; S.N[i] = g.N;
    S.div[i] = g.div == 0.0f ? 1.0f : g.div;
    S.rpb[i] = multi_rpb(g.M, g.N);
    S.np[i] = cdiv(g.M, S.rpb[i]);
    S.ctiles[i] = cdiv(g.N, 256);
    S.ws0[i] = wsoff;
    wsoff += (long)S.np[i] * g.N;
    S.blk0[i + 1] = S.blk0[i] + S.ctiles[i] * S.np[i];
    S.q0[i + 1] = S.q0[i] + g.N / 4;
  }
  hipStream_t s = (hipStream_t)stream;
  colsum_multi_partial<<<S.blk0[nseg], 256, 0, s>>>(S, ws);
  colsum_multi_final<<<cdiv(S.q0[nseg], 256), 256, 0, s>>>(S, ws);
  return check_launch("colsum_multi");
}

extern "C" int ctr_loss(const float* z, const float* za, const float* y, int B, float aux_w, float* loss, float* dz,
                        float* dza, void* stream) {
  loss_kernel<<<1, 1024, 0, (hipStream_t)stream>>>(z, aux_w > 0.f ? za : nullptr, y, B, aux_w, loss, dz, dza);
  return check_launch("loss");
}

// ---------------- small helpers ----------------
namespace ctr {
__global__ void sigmoid_kernel(const float* __restrict__ x, int n, float* __restrict__ y) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) y[i] = sigmoid_f(x[i]);
}
__global__ void copy2d_kernel(const float* __restrict__ src, long lds, float* __restrict__ dst, long ldd, int rows,
                              int cols) {
  const long n = (long)rows * cols;
  for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q < n; q += (long)gridDim.x * blockDim.x) {
    const long r = q / cols;
    const int c = (int)(q % cols);
    dst[r * ldd + c] = src[r * lds + c];
  }
}
}  // namespace ctr

// prob = sigmoid(logits)  (src/models/wrapper.py:175)
extern "C" int ctr_sigmoid(const float* x, int n, float* y, void* stream) {
  if (n == 0) return 0;
  sigmoid_kernel<<<std::min(cdiv(n, 256), 4096), 256, 0, (hipStream_t)stream>>>(x, n, y);
  return check_launch("sigmoid");
}

namespace ctr {
// one wave per output row; rows are whole 4-byte words (f32 / i32 shard columns staged in HBM)
__global__ __launch_bounds__(256) void gather_rows_kernel(const uint32_t* __restrict__ src, long row_words,
                                                          const long* __restrict__ idx, int n,
                                                          uint32_t* __restrict__ dst) {
  const int lane = threadIdx.x & 63;
  for (long r = blockIdx.x * 4L + (threadIdx.x >> 6); r < n; r += (long)gridDim.x * 4) {
    const uint32_t* s = src + idx[r] * row_words;
    uint32_t* d = dst + r * row_words;
    for (long w = lane; w < row_words; w += 64) d[w] = s[w];
  }
}
}  // namespace ctr

// batch assembly from HBM-resident shards: dst[r] = src[idx[r]] (replaces ShardedDataset.__getitem__
// + collate_sharded, src/data/dataset.py:77-80, 98-124, for device-staged data)
extern "C" int ctr_gather_rows(const void* src, long row_words, const long* idx, int n, void* dst, void* stream) {
  if (n == 0 || row_words == 0) return 0;
  int blocks = std::min(cdiv(n, 4), 8192);
  gather_rows_kernel<<<blocks, 256, 0, (hipStream_t)stream>>>((const uint32_t*)src, row_words, idx, n,
                                                              (uint32_t*)dst);
  return check_launch("gather_rows");
}

namespace ctr {
__global__ void step_marker_kernel(int tag) { (void)tag; }

// dst[0, n) = 0: 16-byte stores, grid-stride (the dense grad arena before each backward)
__global__ void zero_f32_kernel(float* __restrict__ dst, long n) {
  typedef float zf4 __attribute__((ext_vector_type(4)));
  const long n4 = n / 4;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n4; i += (long)gridDim.x * 256)
    ((zf4*)dst)[i] = zf4{0.f, 0.f, 0.f, 0.f};
  for (long i = 4 * n4 + blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) dst[i] = 0.f;
}
}  // namespace ctr

extern "C" int ctr_zero_f32(float* dst, long n, void* stream) {
  CTR_REQUIRE(n >= 0 && (((uintptr_t)dst) & 15) == 0, "ctr_zero_f32: needs a 16-byte aligned buffer");
  if (n == 0) return 0;
  const int blocks = (int)std::min<long>((n / 4 + 255) / 256 + 1, 2048);
  zero_f32_kernel<<<blocks, 256, 0, (hipStream_t)stream>>>(dst, n);
  return check_launch("zero_f32");
}

// an empty dispatch that marks a point of the stream in a rocprofv3 kernel trace (bench.py --markers)
extern "C" int ctr_step_marker(int tag, void* stream) {
  step_marker_kernel<<<1, 64, 0, (hipStream_t)stream>>>(tag);
  return check_launch("step_marker");
}

// strided 2-D copy (feature concatenation for the fc head, src/models/wrapper.py:168-172)
extern "C" int ctr_copy2d(const float* src, long lds, float* dst, long ldd, int rows, int cols, void* stream) {
  if ((long)rows * cols == 0) return 0;
  int blocks = (int)std::min<long>(((long)rows * cols + 255) / 256, 8192);
  copy2d_kernel<<<blocks, 256, 0, (hipStream_t)stream>>>(src, lds, dst, ldd, rows, cols);
  return check_launch("copy2d");
}

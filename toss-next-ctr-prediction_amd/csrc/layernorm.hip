// LayerNorm for the `norm` options other than "rms": src/models/dare.py:15-18 `make_norm` returns nn.LayerNorm(d)
// (eps 1e-5, elementwise affine) for any other name -- the encoder layers' norm1 / norm2 (dare.py:44,49) and the QNN
// pre-norm (src/models/qnn_alpha.py:64,112).  No reference config selects it; the path exists so such a config
// runs.  fp32 throughout, two passes over the row held in registers (the mean, then the centred squares: the
// biased variance torch uses, without an E[x^2] - mean^2 cancellation):
//   y = (x - mean) rstd w + b,   rstd = 1 / sqrt(var + eps)
// backward (torch's LayerNorm backward), xhat = (x - mean) rstd:
//   dx = rstd (g w - mean_n(g w) - xhat mean_n(g w xhat)),   dw = sum_m g xhat,   db = sum_m g
// Rows of N <= 64 (the encoder's D): a wave per row, lane = column, wave reductions only; wider rows (the QNN's
// F D): a 256-thread block per row, NPT columns per thread.  Weight / bias grads go to per-block (or per-wave)
// partial rows that ctr_colsum reduces in a fixed order -- deterministic, no atomics.
#include "common.h"
#include "ctr_hip.h"

namespace ctr {
namespace {

__global__ __launch_bounds__(256) void ln_fwd_wave(const float* __restrict__ x, long ldx, int M, int N,
                                                   const float* __restrict__ w, const float* __restrict__ b, float eps,
                                                   float* __restrict__ y, long ldy, float* __restrict__ mean,
                                                   float* __restrict__ rstd, __bf16* __restrict__ ybf, long ldybf) {
  const int lane = threadIdx.x & 63;
  const long m = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (m >= M) return;
  const bool on = lane < N;
  const float v = on ? x[m * ldx + lane] : 0.f;
  const float mu = wave_sum(v) / (float)N;
  const float d = on ? v - mu : 0.f;
  const float rs = 1.0f / sqrtf(wave_sum(d * d) / (float)N + eps);
  if (on) {
    const float o = d * rs * w[lane] + b[lane];
    y[m * ldy + lane] = o;
    if (ybf) ybf[m * ldybf + lane] = (__bf16)o;
  }
  if (lane == 0) {
    mean[m] = mu;
    rstd[m] = rs;
  }
}

template <int NPT>
__global__ __launch_bounds__(256) void ln_fwd_block(const float* __restrict__ x, long ldx, int N,
                                                    const float* __restrict__ w, const float* __restrict__ b, float eps,
                                                    float* __restrict__ y, long ldy, float* __restrict__ mean,
                                                    float* __restrict__ rstd, __bf16* __restrict__ ybf, long ldybf) {
  __shared__ float red[4];
  const long m = blockIdx.x;
  float v[NPT];
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < NPT; ++k) {
    const int n = threadIdx.x + 256 * k;
    v[k] = n < N ? x[m * ldx + n] : 0.f;
    s += v[k];
  }
  const float mu = block_sum(s, red) / (float)N;
  float q = 0.f;
#pragma unroll
  for (int k = 0; k < NPT; ++k) {
    const int n = threadIdx.x + 256 * k;
    const float d = n < N ? v[k] - mu : 0.f;
    q = fmaf(d, d, q);
  }
  const float rs = 1.0f / sqrtf(block_sum(q, red) / (float)N + eps);
#pragma unroll
  for (int k = 0; k < NPT; ++k) {
    const int n = threadIdx.x + 256 * k;
    if (n < N) {
      const float o = (v[k] - mu) * rs * w[n] + b[n];
      y[m * ldy + n] = o;
      if (ybf) ybf[m * ldybf + n] = (__bf16)o;
    }
  }
  if (threadIdx.x == 0) {
    mean[m] = mu;
    rstd[m] = rs;
  }
}

// N <= 64: block blk's wave v walks rows m0 + v, m0 + v + 4, ... of [m0, m1) and writes its weight / bias grad
// partial to row 4 blk + v
__global__ __launch_bounds__(256) void ln_bwd_wave(const float* __restrict__ dy, long ldy, const float* __restrict__ x,
                                                   long ldx, const float* __restrict__ mean,
                                                   const float* __restrict__ rstd, const float* __restrict__ w, int M,
                                                   int N, float* __restrict__ dx, long lddx,
                                                   const float* __restrict__ add, long ld_add, int rows_per_block,
                                                   float* __restrict__ dw_part, float* __restrict__ db_part) {
  const int lane = threadIdx.x & 63, v = threadIdx.x >> 6;
  const bool on = lane < N;
  const float wl = on ? w[lane] : 0.f;
  const long m0 = (long)blockIdx.x * rows_per_block, m1 = min((long)M, m0 + rows_per_block);
  float aw = 0.f, ab = 0.f;
  for (long m = m0 + v; m < m1; m += 4) {
    const float g = on ? dy[m * ldy + lane] : 0.f;
    const float rs = rstd[m];
    const float xh = on ? (x[m * ldx + lane] - mean[m]) * rs : 0.f;
    const float gw = g * wl;
    const float c1 = wave_sum(gw * xh) / (float)N, c2 = wave_sum(gw) / (float)N;
    if (on) {
      float o = rs * (gw - c2 - xh * c1);
      if (add) o += add[m * ld_add + lane];
      dx[m * lddx + lane] = o;
    }
    aw = fmaf(g, xh, aw);
    ab += g;
  }
  if (on) {
    const long p = (long)blockIdx.x * 4 + v;
    dw_part[p * N + lane] = aw;
    db_part[p * N + lane] = ab;
  }
}

// 64 < N <= 256 NPT: block blk takes rows [m0, m1), a row at a time, NPT columns per thread
template <int NPT>
__global__ __launch_bounds__(256) void ln_bwd_block(const float* __restrict__ dy, long ldy,
                                                    const float* __restrict__ x, long ldx,
                                                    const float* __restrict__ mean, const float* __restrict__ rstd,
                                                    const float* __restrict__ w, int M, int N, float* __restrict__ dx,
                                                    long lddx, const float* __restrict__ add, long ld_add,
                                                    int rows_per_block, float* __restrict__ dw_part,
                                                    float* __restrict__ db_part) {
  __shared__ float red[4];
  float wv[NPT], aw[NPT], ab[NPT];
#pragma unroll
  for (int k = 0; k < NPT; ++k) {
    const int n = threadIdx.x + 256 * k;
    wv[k] = n < N ? w[n] : 0.f;
    aw[k] = ab[k] = 0.f;
  }
  const long m0 = (long)blockIdx.x * rows_per_block, m1 = min((long)M, m0 + rows_per_block);
  for (long m = m0; m < m1; ++m) {
    const float rs = rstd[m], mu = mean[m];
    float g[NPT], xh[NPT];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
      const int n = threadIdx.x + 256 * k;
      g[k] = n < N ? dy[m * ldy + n] : 0.f;
      xh[k] = n < N ? (x[m * ldx + n] - mu) * rs : 0.f;
      const float gw = g[k] * wv[k];
      s1 = fmaf(gw, xh[k], s1);
      s2 += gw;
    }
    const float c1 = block_sum(s1, red) / (float)N, c2 = block_sum(s2, red) / (float)N;
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
      const int n = threadIdx.x + 256 * k;
      if (n < N) {
        float o = rs * (g[k] * wv[k] - c2 - xh[k] * c1);
        if (add) o += add[m * ld_add + n];
        dx[m * lddx + n] = o;
      }
      aw[k] = fmaf(g[k], xh[k], aw[k]);
      ab[k] += g[k];
    }
  }
#pragma unroll
  for (int k = 0; k < NPT; ++k) {
    const int n = threadIdx.x + 256 * k;
    if (n < N) {
      dw_part[(long)blockIdx.x * N + n] = aw[k];
      db_part[(long)blockIdx.x * N + n] = ab[k];
    }
  }
}

// wider rows: per row two strided passes (the sums, then dx), then the block's column sums over its rows
__global__ __launch_bounds__(256) void ln_bwd_wide(const float* __restrict__ dy, long ldy, const float* __restrict__ x,
                                                   long ldx, const float* __restrict__ mean,
                                                   const float* __restrict__ rstd, const float* __restrict__ w, int M,
                                                   int N, float* __restrict__ dx, long lddx,
                                                   const float* __restrict__ add, long ld_add, int rows_per_block,
                                                   float* __restrict__ dw_part, float* __restrict__ db_part) {
  __shared__ float red[4];
  const long m0 = (long)blockIdx.x * rows_per_block, m1 = min((long)M, m0 + rows_per_block);
  for (long m = m0; m < m1; ++m) {
    const float rs = rstd[m], mu = mean[m];
    float s1 = 0.f, s2 = 0.f;
    for (int n = threadIdx.x; n < N; n += 256) {
      const float gw = dy[m * ldy + n] * w[n];
      s1 = fmaf(gw, (x[m * ldx + n] - mu) * rs, s1);
      s2 += gw;
    }
    const float c1 = block_sum(s1, red) / (float)N, c2 = block_sum(s2, red) / (float)N;
    for (int n = threadIdx.x; n < N; n += 256) {
      float o = rs * (dy[m * ldy + n] * w[n] - c2 - (x[m * ldx + n] - mu) * rs * c1);
      if (add) o += add[m * ld_add + n];
      dx[m * lddx + n] = o;
    }
  }
  for (int n = threadIdx.x; n < N; n += 256) {
    float aw = 0.f, ab = 0.f;
    for (long m = m0; m < m1; ++m) {
      const float g = dy[m * ldy + n];
      aw = fmaf(g, (x[m * ldx + n] - mean[m]) * rstd[m], aw);
      ab += g;
    }
    dw_part[(long)blockIdx.x * N + n] = aw;
    db_part[(long)blockIdx.x * N + n] = ab;
  }
}

// rows per block of the backward: ~512 blocks (two per CU), at least 4 rows (wave form) / 2 rows
int ln_rows_per_block(int M, int N) { return std::max(N <= 64 ? 4 : 2, cdiv(M, 512)); }

}  // namespace
}  // namespace ctr

using namespace ctr;

extern "C" int ctr_layernorm_fwd(const float* x, long ldx, int M, int N, const float* w, const float* b, float eps,
                                 float* y, long ldy, float* mean, float* rstd, void* ybf, long ldybf, void* stream) {
  CTR_REQUIRE(N > 0 && N <= 64 * 256, "row width in [1, 16384]");
  if (M <= 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  __bf16* yb = (__bf16*)ybf;
  if (N <= 64) ln_fwd_wave<<<cdiv(M, 4), 256, 0, s>>>(x, ldx, M, N, w, b, eps, y, ldy, mean, rstd, yb, ldybf);
  else if (N <= 256) ln_fwd_block<1><<<M, 256, 0, s>>>(x, ldx, N, w, b, eps, y, ldy, mean, rstd, yb, ldybf);
  else if (N <= 1024) ln_fwd_block<4><<<M, 256, 0, s>>>(x, ldx, N, w, b, eps, y, ldy, mean, rstd, yb, ldybf);
  else if (N <= 4096) ln_fwd_block<16><<<M, 256, 0, s>>>(x, ldx, N, w, b, eps, y, ldy, mean, rstd, yb, ldybf);
  else ln_fwd_block<64><<<M, 256, 0, s>>>(x, ldx, N, w, b, eps, y, ldy, mean, rstd, yb, ldybf);
  return check_launch("layernorm_fwd");
}

extern "C" int ctr_layernorm_bwd_nparts(int M, int N) {
  const int nb = cdiv(std::max(M, 1), ln_rows_per_block(std::max(M, 1), N));
  return N <= 64 ? 4 * nb : nb;
}

extern "C" int ctr_layernorm_bwd(const float* dy, long ldy, const float* x, long ldx, const float* mean,
                                 const float* rstd, const float* w, int M, int N, float* dx, long lddx,
                                 const float* add, long ld_add, float* dw_part, float* db_part, void* stream) {
  CTR_REQUIRE(N > 0, "row width");
  if (M <= 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  const int rpb = ln_rows_per_block(M, N), nb = cdiv(M, rpb);
  if (N <= 64)
    ln_bwd_wave<<<nb, 256, 0, s>>>(dy, ldy, x, ldx, mean, rstd, w, M, N, dx, lddx, add, ld_add, rpb, dw_part, db_part);
  else if (N <= 256)
    ln_bwd_block<1><<<nb, 256, 0, s>>>(dy, ldy, x, ldx, mean, rstd, w, M, N, dx, lddx, add, ld_add, rpb, dw_part,
                                       db_part);
  else if (N <= 2048)
    ln_bwd_block<8><<<nb, 256, 0, s>>>(dy, ldy, x, ldx, mean, rstd, w, M, N, dx, lddx, add, ld_add, rpb, dw_part,
                                       db_part);
  else
    ln_bwd_wide<<<nb, 256, 0, s>>>(dy, ldy, x, ldx, mean, rstd, w, M, N, dx, lddx, add, ld_add, rpb, dw_part, db_part);
  return check_launch("layernorm_bwd");
}

// QNN-alpha feature interaction (src/models/qnn_alpha.py):
//   pair_interaction_all (l.86-97): per head h, A = z @ U_h (B,F,r); s = sum_F A; quad = s*s - sum_F A*A;
//                                   out_h = quad @ V_h.   A for all heads comes from ONE MFMA GEMM
//                                   (B*F, D) x (D, H*r) (gemm.hip) on the head-concatenated U; this file
//                                   holds the F-reduction + block-diagonal V product and their backward.
//   SEBlock (l.17-26): gate = sigmoid(W2 relu(W1 mean_B(x) + b1) + b2); x * gate  (batch-coupled).
#include "common.h"
#include "ctr_hip.h"

namespace ctr {

// U (H, D, R) <-> Ucat (D, H*R)
__global__ void ucat_kernel(const float* __restrict__ src, int H, int D, int R, float* __restrict__ dst, int inverse) {
  const int n = H * D * R;
  for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < n; q += gridDim.x * blockDim.x) {
    const int h = q / (D * R), rem = q % (D * R), d = rem / R, r = rem % R;
    const int c = d * (H * R) + h * R + r;
    if (!inverse) dst[c] = src[q];
    else dst[q] = src[c];
  }
}

// one workgroup per sample: S[c] = sum_f A[f,c], quad[c] = S^2 - sum_f A^2, inter[h*P+p] = sum_r quad[h*R+r] V[h,r,p]
__global__ __launch_bounds__(256) void qnn_reduce_fwd_kernel(const float* __restrict__ A, int F, int H, int R,
                                                             const float* __restrict__ V, int P,
                                                             float* __restrict__ S, float* __restrict__ quad,
                                                             float* __restrict__ inter) {
  extern __shared__ float sq[];
  const int b = blockIdx.x, C = H * R;
  const float* Ab = A + (long)b * F * C;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float s = 0.f, s2 = 0.f;
    for (int f = 0; f < F; ++f) {
      const float a = Ab[(long)f * C + c];
      s += a;
      s2 += a * a;
    }
    const float qd = s * s - s2;
    S[(long)b * C + c] = s;
    quad[(long)b * C + c] = qd;
    sq[c] = qd;
  }
  __syncthreads();
  for (int o = threadIdx.x; o < H * P; o += blockDim.x) {
    const int h = o / P, p = o % P;
    float acc = 0.f;
    for (int r = 0; r < R; ++r) acc = fmaf(sq[h * R + r], V[((long)h * R + r) * P + p], acc);
    inter[(long)b * H * P + o] = acc;
  }
}

// dquad[c] = sum_p dinter[h*P+p] V[h,r,p]; dA[f,c] = 2*dquad[c]*(S[c] - A[f,c])
__global__ __launch_bounds__(256) void qnn_reduce_bwd_kernel(const float* __restrict__ A, int F, int H, int R,
                                                             const float* __restrict__ V, int P,
                                                             const float* __restrict__ S,
                                                             const float* __restrict__ dinter,
                                                             float* __restrict__ dA) {
  extern __shared__ float sd[];
  const int b = blockIdx.x, C = H * R;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    const int h = c / R, r = c % R;
    float acc = 0.f;
    for (int p = 0; p < P; ++p) acc = fmaf(dinter[(long)b * H * P + h * P + p], V[((long)h * R + r) * P + p], acc);
    sd[c] = acc;
  }
  __syncthreads();
  const float* Ab = A + (long)b * F * C;
  float* dAb = dA + (long)b * F * C;
  for (int q = threadIdx.x; q < F * C; q += blockDim.x) {
    const int c = q % C;
    const float g = sd[c];
    // autograd of s*s - sum(A*A): ds = g*s + g*s ; dA = ds - (g*A + g*A)
    const float s = S[(long)b * C + c];
    dAb[q] = (g * s + g * s) - (g * Ab[q] + g * Ab[q]);
  }
}

// ---------------- SE block ----------------
// tiny vector MLP, one workgroup: g1 = relu(W1 m + b1) (Cr), gate = sigmoid(W2 g1 + b2) (C)
// y[r] = act(A[r, :] . x + bias[r]) for row-major A (R x N): one wave per row (coalesced row reads,
// fixed-order wave reduction); act 0 none, 1 relu, 2 sigmoid.  The SE gate's two tiny matvecs
// (src/models/qnn_alpha.py:44-52) run as two such grids instead of one serial workgroup.
__global__ __launch_bounds__(256) void matvec_rows_kernel(const float* __restrict__ A, int R, int N,
                                                          const float* __restrict__ x, const float* __restrict__ bias,
                                                          int act, float* __restrict__ y) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (r >= R) return;
  float s = 0.f;
  for (int c = lane; c < N; c += 64) s = fmaf(A[(long)r * N + c], x[c], s);
  s = wave_sum(s);
  if (lane == 0) {
    float v = s + (bias ? bias[r] : 0.f);
    if (act == 1) v = v > 0.f ? v : 0.f;
    else if (act == 2) v = sigmoid_f(v);
    y[r] = v;
  }
}

// y[n] = sum_r x[r] * A[r][n] for row-major A (R x N): one wave per output column, lanes stride the
// rows (strided reads of a small, L2-resident matrix), fixed-order wave reduction.
// mask (nullable): y[n] = 0 where mask[n] <= 0 (relu').  y2: copy.
__global__ __launch_bounds__(256) void matvec_cols_kernel(const float* __restrict__ A, int R, int N,
                                                          const float* __restrict__ x, const float* __restrict__ mask,
                                                          float* __restrict__ y, float* __restrict__ y2) {
  const int n = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (n >= N) return;
  float s = 0.f;
#pragma unroll 4
  for (int r = lane; r < R; r += 64) s = fmaf(x[r], A[(long)r * N + n], s);
  s = wave_sum(s);
  if (lane == 0) {
    float v = s;
    if (mask) v = mask[n] > 0.f ? v : 0.f;
    y[n] = v;
    if (y2) y2[n] = v;
  }
}

// out[b,c] = drop(x[b,c] * gate[c])   (gate nullable: no SE)
__global__ void scale_drop_kernel(const float* __restrict__ x, int B, int C, const float* __restrict__ gate,
                                  Drop drop, float* __restrict__ out, long out_ld) {
  const long n = (long)B * C;
  for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q < n; q += (long)gridDim.x * blockDim.x) {
    const int c = (int)(q % C);
    const long b = q / C;
    float v = x[q];
    if (gate) v = v * gate[c];
    out[b * out_ld + c] = drop_apply(drop, (uint32_t)q, v);
  }
}

// dpost = drop_bwd(dout); dx_direct = dpost*gate; part(dgate) = sum_b dpost*x over row chunks
__global__ __launch_bounds__(256) void se_bwd_partial(const float* __restrict__ dout, long dout_ld,
                                                      const float* __restrict__ x, int B, int C,
                                                      const float* __restrict__ gate, Drop drop,
                                                      int rows_per_block, float* __restrict__ dx,
                                                      float* __restrict__ part) {
  const int b0 = blockIdx.y * rows_per_block, b1 = min(B, b0 + rows_per_block);
  for (int c = blockIdx.x * 256 + threadIdx.x; c < C; c += gridDim.x * 256) {
    float acc = 0.f;
    for (int b = b0; b < b1; ++b) {
      const long q = (long)b * C + c;
      float g = dout[(long)b * dout_ld + c];
      if (drop.thresh) g = drop_keep(drop, (uint32_t)q) ? g * drop.scale : 0.f;
      if (gate) {
        dx[q] = g * gate[c];
        acc = fmaf(g, x[q], acc);
      } else {
        dx[q] = g;
      }
    }
    if (part) part[(long)blockIdx.y * C + c] = acc;
  }
}

// dgate[c] = sum of the row-block partials (fixed order); dz2 = dgate * sigmoid'(.)  -> db2, dz2
__global__ __launch_bounds__(256) void se_dgate_kernel(const float* __restrict__ part, int nparts, int C,
                                                       const float* __restrict__ gate, float* __restrict__ db2,
                                                       float* __restrict__ dz2) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  float dg = 0.f;
  for (int p = 0; p < nparts; ++p) dg += part[(long)p * C + c];
  const float s = gate[c];
  const float v = dg * (s * (1.f - s));
  db2[c] = v;
  dz2[c] = v;
}

// grid: dW2 = dz2 (x) g1, dW1 = dz1 (x) mean
__global__ __launch_bounds__(256) void se_mlp_bwd_outer(int C, int Cr, const float* __restrict__ mean,
                                                        const float* __restrict__ g1, const float* __restrict__ dz2,
                                                        const float* __restrict__ dz1, float* __restrict__ dW1,
                                                        float* __restrict__ dW2) {
  const long q = blockIdx.x * 256L + threadIdx.x;
  const long n2 = (long)C * Cr;
  if (q < n2) {
    dW2[q] = dz2[q / Cr] * g1[q % Cr];
  } else if (q < 2 * n2) {
    const long r = q - n2;
    dW1[r] = dz1[r / C] * mean[r % C];
  }
}

// dx[b,c] += dmean[c] / B   (MeanBackward: grad.expand() / numel)
__global__ void add_row_bcast(float* __restrict__ dx, int B, int C, const float* __restrict__ v, float div) {
  const long n = (long)B * C;
  for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q < n; q += (long)gridDim.x * blockDim.x)
    dx[q] += v[q % C] / div;
}

}  // namespace ctr

using namespace ctr;

extern "C" int ctr_qnn_ucat(const float* src, int H, int D, int R, float* dst, int inverse, void* stream) {
  ucat_kernel<<<cdiv((long)H * D * R, 256), 256, 0, (hipStream_t)stream>>>(src, H, D, R, dst, inverse);
  return check_launch("qnn_ucat");
}

extern "C" int ctr_qnn_reduce_fwd(const float* A, int B, int F, int H, int R, const float* V, int P, float* S,
                                  float* quad, float* inter, void* stream) {
  if (B == 0) return 0;
  qnn_reduce_fwd_kernel<<<B, 256, H * R * sizeof(float), (hipStream_t)stream>>>(A, F, H, R, V, P, S, quad, inter);
  return check_launch("qnn_reduce_fwd");
}

extern "C" int ctr_qnn_reduce_bwd(const float* A, int B, int F, int H, int R, const float* V, int P, const float* S,
                                  const float* dinter, float* dA, void* stream) {
  if (B == 0) return 0;
  qnn_reduce_bwd_kernel<<<B, 256, H * R * sizeof(float), (hipStream_t)stream>>>(A, F, H, R, V, P, S, dinter, dA);
  return check_launch("qnn_reduce_bwd");
}

extern "C" int ctr_se_fwd_gate(const float* mean, int C, int Cr, const float* W1, const float* b1, const float* W2,
                               const float* b2, float* g1, float* gate, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  matvec_rows_kernel<<<cdiv(Cr, 4), 256, 0, s>>>(W1, Cr, C, mean, b1, 1, g1);
  matvec_rows_kernel<<<cdiv(C, 4), 256, 0, s>>>(W2, C, Cr, g1, b2, 2, gate);
  return check_launch("se_fwd_gate");
}

extern "C" int ctr_scale_drop(const float* x, int B, int C, const float* gate, uint32_t drop_key, uint32_t drop_thresh,
                              float drop_scale, float* out, long out_ld, void* stream) {
  if (B == 0) return 0;
  long n = (long)B * C;
  int blocks = (int)std::min<long>((n + 255) / 256, 16384);
  scale_drop_kernel<<<blocks, 256, 0, (hipStream_t)stream>>>(x, B, C, gate, Drop{drop_key, drop_thresh, drop_scale},
                                                             out, out_ld);
  return check_launch("scale_drop");
}

extern "C" size_t ctr_se_bwd_ws(int B, int C) { return ((size_t)cdiv(B, 64) * C + 3 * (size_t)C) * sizeof(float); }

extern "C" int ctr_se_bwd(const float* dout, long dout_ld, const float* x, int B, int C, int Cr, const float* gate,
                          const float* g1, const float* mean, const float* W1, const float* W2, uint32_t drop_key,
                          uint32_t drop_thresh, float drop_scale, float* dx, float* dW1, float* db1, float* dW2,
                          float* db2, float* ws, void* stream) {
  if (B == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  const int rpb = 64;
  const int np = cdiv(B, rpb);
  float* part = ws;                      // [np][C]
  float* dmean = ws + (size_t)np * C;    // [C]
  Drop d{drop_key, drop_thresh, drop_scale};
  se_bwd_partial<<<dim3(cdiv(C, 256), np), 256, 0, s>>>(dout, dout_ld, x, B, C, gate, d, rpb, dx,
                                                       gate ? part : nullptr);
  if (gate) {
    float* dz2 = dmean + C;                // [C]
    float* dz1 = dz2 + C;                  // [Cr <= C]
    se_dgate_kernel<<<cdiv(C, 256), 256, 0, s>>>(part, np, C, gate, db2, dz2);
    matvec_cols_kernel<<<cdiv(Cr, 4), 256, 0, s>>>(W2, C, Cr, dz2, g1, db1, dz1);     // dz1 = relu'(W2^T dz2)
    matvec_cols_kernel<<<cdiv(C, 4), 256, 0, s>>>(W1, Cr, C, dz1, nullptr, dmean, nullptr);   // W1^T dz1
    se_mlp_bwd_outer<<<cdiv(2L * C * Cr, 256), 256, 0, s>>>(C, Cr, mean, g1, dz2, dz1, dW1, dW2);
    long n = (long)B * C;
    int blocks = (int)std::min<long>((n + 255) / 256, 16384);
    add_row_bcast<<<blocks, 256, 0, s>>>(dx, B, C, dmean, (float)B);
  }
  return check_launch("se_bwd");
}

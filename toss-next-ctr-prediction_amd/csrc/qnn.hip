// QNN-alpha feature interaction (src/models/qnn_alpha.py):
//   pair_interaction_all (l.86-97): per head h, A = z @ U_h (B,F,r); s = sum_F A; quad = s*s - sum_F A*A;
//                                   out_h = quad @ V_h.
//   SEBlock (l.17-26): gate = sigmoid(W2 relu(W1 mean_B(x) + b1) + b2); x * gate  (batch-coupled).
//
// The (B*F) x (H*r) tensor A is never formed.  With Ucat = [U_1 .. U_H] (D x QR) and per-sample
// Gram matrices G_b = z_b^T z_b (D x D) and zsum_b = sum_f z_bf:
//   s    = zsum_b @ Ucat,                 sum_f A^2 = diag(Ucat^T G_b Ucat)
//   dz_f = sum_c dA_fc U_c = 2 U (dquad o s) - 2 (U diag(dquad) U^T) z_f      (dA = 2 dquad (s - A))
//   dU   = 2 [ zsum^T (dquad o s) - sum_b G_b U diag(dquad_b) ]               (batched GEMMs)
// i.e. the same sums re-associated (fp32 rounding differs at the 1e-7 level): the interaction costs
// two passes over z (105 MB at cfg2) instead of a 315 MB A tensor written, read and its gradient
// written and read twice.  The head-block-diagonal V products are plain GEMMs on Vfull (QR x H*P).
#include "common.h"
#include "ctr_hip.h"

namespace ctr {

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 mfma4q(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

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

// V (H, R, P) <-> block-diagonal Vfull (H*R, H*P); forward expand writes the zeros too
__global__ void vfull_kernel(const float* __restrict__ src, int H, int R, int P, float* __restrict__ dst,
                             int inverse) {
  const long QR = (long)H * R, C = (long)H * P;
  if (!inverse) {
    for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q < QR * C; q += (long)gridDim.x * blockDim.x) {
      const long row = q / C, col = q % C;
      const long h = row / R, hc = col / P;
      dst[q] = (h == hc) ? src[(h * R + row % R) * P + col % P] : 0.f;
    }
  } else {
    for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q < QR * P; q += (long)gridDim.x * blockDim.x) {
      const long h = q / ((long)R * P), rp = q % ((long)R * P), r = rp / P, pp = rp % P;
      dst[q] = src[(h * R + r) * C + h * P + pp];
    }
  }
}

// Ucat staged in LDS, zero-padded to QRp = 16*ceil(QR/16) columns, row stride QRp + 1
template <int D>
__device__ __forceinline__ void stage_ucat(const float* __restrict__ ucat, int QR, int QRp, float* sU) {
  for (int q = threadIdx.x; q < D * QRp; q += blockDim.x) {
    const int d = q / QRp, c = q % QRp;
    sU[d * (QRp + 1) + c] = c < QR ? ucat[d * QR + c] : 0.f;
  }
}

// One wave per sample.  G = z^T z by MFMA with the F rows as the contraction (A and B operands are the
// same loaded values: lane (g, c) holds z[4s+g][16i+c]); then H = G Ucat using the symmetric G's
// C-layout registers directly as A operands (k-set {16i + 4g + r}), and sum_f A^2 = sum_d U o H.
// ld: a sample's z row stride (F D, or wider for one feature block of the rows); acc: G and quad are added to
// what the buffers hold (pair_grouping 'block': the blocks' Gram matrices and quads summed, zsum / S per block)
template <int D>
__global__ __launch_bounds__(256) void qnn_gram_fwd_kernel(const float* __restrict__ z, long ld, int B, int F,
                                                           const float* __restrict__ ucat, int QR,
                                                           float* __restrict__ zsum_out, float* __restrict__ G_out,
                                                           float* __restrict__ S_out, float* __restrict__ quad_out,
                                                           int acc_out) {
  constexpr int NT = D / 16;
  extern __shared__ float sU[];
  const int QRp = (QR + 15) / 16 * 16, US = QRp + 1;
  float* szs = sU + D * US;                      // [4 waves][D] zsum
  stage_ucat<D>(ucat, QR, QRp, sU);
  __syncthreads();
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
  const int b = blockIdx.x * 4 + w;
  if (b >= B) return;
  const float* zb = z + (long)b * ld;
  f32x4 acc[NT][NT];
#pragma unroll
  for (int i = 0; i < NT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float zs[NT];
#pragma unroll
  for (int i = 0; i < NT; ++i) zs[i] = 0.f;
  // FU row quads per step: their loads go out together (one quad's loads per round trip left the wave
  // latency-bound: 50 dependent round trips per sample at F = 200); sums and products in the same order
#ifndef QNN_FU
#define QNN_FU 8
#endif
  constexpr int FU = QNN_FU;
  for (int f00 = 0; f00 < F; f00 += 4 * FU) {
    float v[FU][NT];
#pragma unroll
    for (int u = 0; u < FU; ++u) {
      const int f = f00 + 4 * u + g;
#pragma unroll
      for (int i = 0; i < NT; ++i) v[u][i] = f < F ? zb[(long)f * D + 16 * i + c] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < FU; ++u) {
      if (f00 + 4 * u >= F) break;
#pragma unroll
      for (int i = 0; i < NT; ++i) zs[i] += v[u][i];
#pragma unroll
      for (int i = 0; i < NT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[i][j] = mfma4q(v[u][i], v[u][j], acc[i][j]);
    }
  }
#pragma unroll
  for (int i = 0; i < NT; ++i) {
    zs[i] += __shfl_xor(zs[i], 16);
    zs[i] += __shfl_xor(zs[i], 32);
  }
  float* zw = szs + w * D;
  if (g == 0) {
#pragma unroll
    for (int i = 0; i < NT; ++i) {
      zw[16 * i + c] = zs[i];
      zsum_out[(long)b * D + 16 * i + c] = zs[i];
    }
  }
  // G (row-major D x D per sample): reg r of tile (i, j) = G[16i + 4g + r][16j + c]
  float* Gb = G_out + (long)b * D * D;
#pragma unroll
  for (int i = 0; i < NT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float* gp = Gb + (16 * i + 4 * g + r) * D + 16 * j + c;
        *gp = acc_out ? *gp + acc[i][j][r] : acc[i][j][r];
      }
  __builtin_amdgcn_wave_barrier();
  for (int t = 0; t < QRp / 16; ++t) {
    const int cc = 16 * t + c;
    // S[cc] = zsum . U[:, cc]
    float sv = 0.f;
#pragma unroll 8
    for (int d = 0; d < D; ++d) sv = fmaf(zw[d], sU[d * US + cc], sv);
    // H[:, t-block] = G U[:, t-block]; sa2 = sum_d U[d][cc] H[d][cc]
    float sa2 = 0.f;
#pragma unroll
    for (int jd = 0; jd < NT; ++jd) {
      f32x4 h = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < NT; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) h = mfma4q(acc[i][jd][r], sU[(16 * i + 4 * g + r) * US + cc], h);
#pragma unroll
      for (int r = 0; r < 4; ++r) sa2 = fmaf(h[r], sU[(16 * jd + 4 * g + r) * US + cc], sa2);
    }
    sa2 += __shfl_xor(sa2, 16);
    sa2 += __shfl_xor(sa2, 32);
    if (g == 0 && cc < QR) {
      S_out[(long)b * QR + cc] = sv;
      float* qp = quad_out + (long)b * QR + cc;
      *qp = acc_out ? *qp + (sv * sv - sa2) : sv * sv - sa2;
    }
  }
}

// the residual addend of the Gram backward: fp32, or bf16 (amp) loaded as a zero-extended 16-bit word into a full
// register and widened at its use -- as a __bf16 value the loads went to register halves (d16), each waiting
// for the one before it
template <class TA>
struct GramAdd {
  using R = float;
  static __device__ __forceinline__ R load(const float* p) { return *p; }
  static __device__ __forceinline__ float widen(R r) { return r; }
};
template <>
struct GramAdd<__bf16> {
  using R = uint32_t;
  static __device__ __forceinline__ R load(const __bf16* p) { return *(const unsigned short*)p; }
  static __device__ __forceinline__ float widen(R r) { return __builtin_bit_cast(float, r << 16); }
};

// One sample per 4-wave workgroup: M = U diag(dquad) U^T (MFMA over the QR columns; the waves share its
// 16x16 tiles via LDS) and w = U (dquad o S) (QR quarters summed in fixed wave order); then the waves take
// every fourth 16-row F block: dz_f = 2 w - 2 M z_f (+ dz_add) with M's C-layout registers as the B
// operand (k-set {16i+4g+r}).  (One wave per sample left only 4 waves per SIMD at B = 4096, each a long
// serial load -> MFMA chain.)
template <int D, class TA, bool ADD>
__global__ __launch_bounds__(256) void qnn_gram_bwd_kernel(const float* __restrict__ z, long ld, int B, int F,
                                                           const float* __restrict__ ucat, int QR,
                                                           const float* __restrict__ S,
                                                           const float* __restrict__ dquad,
                                                           const TA* __restrict__ dz_add, float* __restrict__ dz,
                                                           float* __restrict__ DS) {
  constexpr int NT = D / 16;
  extern __shared__ float sU[];
  const int QRp = (QR + 15) / 16 * 16, US = QRp + 1;
  float* dq = sU + D * US;                       // [QRp] dquad
  float* dqs = dq + QRp;                         // [QRp] dquad * S
  float* sM = dqs + QRp;                         // [NT*NT tiles][4][64] M (C layout)
  float* sW = sM + NT * NT * 4 * 64;             // [4 waves][D] w partials
  const int b = blockIdx.x;
  // the first PF row blocks of this wave's z / dz_add rows are loaded before anything else: their round trips
  // overlap the U staging and the M / w products instead of following them (wait-mem 0.75 with the loads issued
  // per block after the barriers).  cfg2 (F = 200: 3-4 blocks per wave): 104 -> 80 us (4.0 TB/s) at PF = 1 or 2,
  // 96 / 100 us at PF = 3 / 4 (the registers held cost occupancy)
#ifndef QNN_PF
#define QNN_PF 2
#endif
  constexpr int PF = QNN_PF;
  const float* zb = z + (long)b * ld;                 // z, dz_add and dz share the row stride ld
  const TA* ab = ADD ? dz_add + (long)b * ld : nullptr;
  f32x4 zpre[PF][NT];
  using AR = typename GramAdd<TA>::R;
  AR apre[PF][4][NT];
  {
    const int w0 = threadIdx.x >> 6, l0 = threadIdx.x & 63, g0 = l0 >> 4, c0 = l0 & 15;
#pragma unroll
    for (int it = 0; it < PF; ++it) {
      const int f0 = 16 * w0 + 64 * it, fa = f0 + c0;
#pragma unroll
      for (int i = 0; i < NT; ++i)
        zpre[it][i] = *(const f32x4*)(zb + (long)(fa < F ? fa : F - 1) * D + 16 * i + 4 * g0);   // rows past F: never stored
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int f = f0 + 4 * g0 + r;
#pragma unroll
        for (int j = 0; j < NT; ++j)     // rows past F: row F - 1 re-read (in bounds, never stored)
          apre[it][r][j] = ADD ? GramAdd<TA>::load(ab + (long)(f < F ? f : F - 1) * D + 16 * j + c0) : AR(0);
      }
    }
  }
  stage_ucat<D>(ucat, QR, QRp, sU);
  for (int q = threadIdx.x; q < QRp; q += 256) {
    const float d = q < QR ? dquad[(long)b * QR + q] : 0.f;
    const float sv = q < QR ? S[(long)b * QR + q] : 0.f;
    dq[q] = d;
    dqs[q] = d * sv;
    if (q < QR) DS[(long)b * QR + q] = d * sv;
  }
  __syncthreads();
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
  // M tiles (i, j) = t, t + 4, ... of this wave over the whole QR range
  for (int t = w; t < NT * NT; t += 4) {
    const int i = t / NT, j = t - i * NT;
    f32x4 Mt = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int k0 = 0; k0 < QRp; k0 += 4) {
      const int k = k0 + g;
      const float bi = sU[(16 * i + c) * US + k];
      const float bj = sU[(16 * j + c) * US + k];
      Mt = mfma4q(bi * dq[k], bj, Mt);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) sM[(t * 4 + r) * 64 + lane] = Mt[r];
  }
  {
    // w partial: this wave's QR quarter; lane (g, c) sums q = k0w + g, k0w + g + 4, ... for e = 16j + c
    const int kq = QRp / 4;
    const int k0w = w * kq, k1w = k0w + kq;
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      float a = 0.f;
      for (int q = k0w + g; q < k1w; q += 4) a = fmaf(sU[(16 * j + c) * US + q], dqs[q], a);
      a += __shfl_xor(a, 16);
      a += __shfl_xor(a, 32);
      if (g == 0) sW[w * D + 16 * j + c] = a;
    }
  }
  __syncthreads();
  f32x4 M[NT][NT];
#pragma unroll
  for (int i = 0; i < NT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) M[i][j][r] = sM[((i * NT + j) * 4 + r) * 64 + lane];
  float wv[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int e = 16 * j + c;
    wv[j] = 2.f * (((sW[e] + sW[D + e]) + sW[2 * D + e]) + sW[3 * D + e]);
  }
  float* ob = dz + (long)b * ld;
  int it = 0;
  for (int f0 = 16 * w; f0 < F; f0 += 64, ++it) {
    const int fa = f0 + c;                       // A-operand row of this lane
    f32x4 acc[NT];
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // the lane's four A values of a 16-column block are contiguous: one 16-byte load per block
    f32x4 zq[NT];
    AR aq[4][NT];
    if (it < PF) {
#pragma unroll
      for (int q = 0; q < PF; ++q)
        if (q == it) {
#pragma unroll
          for (int i = 0; i < NT; ++i) zq[i] = zpre[q][i];
#pragma unroll
          for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int j = 0; j < NT; ++j) aq[r][j] = apre[q][r][j];
        }
    } else {
#pragma unroll
      for (int i = 0; i < NT; ++i)
        zq[i] = *(const f32x4*)(zb + (long)(fa < F ? fa : F - 1) * D + 16 * i + 4 * g);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int f = f0 + 4 * g + r;
#pragma unroll
        for (int j = 0; j < NT; ++j)
          aq[r][j] = ADD ? GramAdd<TA>::load(ab + (long)(f < F ? f : F - 1) * D + 16 * j + c) : AR(0);
      }
    }
#pragma unroll
    for (int i = 0; i < NT; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[j] = mfma4q(zq[i][r], M[i][j][r], acc[j]);
      }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int f = f0 + 4 * g + r;
      if (f < F) {
#pragma unroll
        for (int j = 0; j < NT; ++j) {
          const int e = 16 * j + c;
          float v = wv[j] - 2.f * acc[j][r];
          if (ADD) v += GramAdd<TA>::widen(aq[r][j]);
          ob[(long)f * D + e] = v;
        }
      }
    }
  }
}

// ---------------- amp: the pair interaction on bf16(z) ----------------
// Under autocast(bfloat16) the reference's A = z @ U_h (qnn_alpha.py:90) takes z rounded to bf16.  These forms read
// z from the bf16 image of [z | inter] the QNN pre-norm writes for the MLP (RNE of the fp32 z, row stride ldz) and
// compute the same Gram-form sums exactly as a function of bf16(z): G = bf16(z)^T bf16(z) on
// v_mfma_f32_16x16x32_bf16 (products exact, fp32 accumulation) and zsum = sum of the bf16 values in fp32 -- so
// s^2 - sum A^2 cancels consistently -- and, backward, dz_f = 2 w - 2 M bf16(z_f) with M = U diag(dquad) U^T in
// fp32 rounded to bf16 for the product (the reference rounds dA and U to bf16 for dA @ U^T).  D in {32, 64}.
typedef __bf16 gbf16x8 __attribute__((ext_vector_type(8)));
typedef uint32_t gu32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ f32x4 mfma_g(gbf16x8 a, gbf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ float bfw(uint32_t h) { return __builtin_bit_cast(float, h << 16); }

// One wave per sample (as qnn_gram_fwd_kernel).  K-step of 32 rows: lane (g, c) holds rows 8g .. 8g+7 of column
// 16i + c -- the A operand of tile (i, j) and the B operand of tile (j, i) at once (G is symmetric); the next
// step's rows are loaded while this step multiplies.
template <int D>
__global__ __launch_bounds__(256) void qnn_gram_fwd_bf_kernel(const unsigned short* __restrict__ zbf, long ldz, int B,
                                                              int F, const float* __restrict__ ucat, int QR,
                                                              float* __restrict__ zsum_out, float* __restrict__ G_out,
                                                              float* __restrict__ S_out, float* __restrict__ quad_out,
                                                              int acc_out) {
  constexpr int NT = D / 16;
  extern __shared__ float sU[];
  const int QRp = (QR + 15) / 16 * 16, US = QRp + 1;
  float* szs = sU + D * US;
  stage_ucat<D>(ucat, QR, QRp, sU);
  __syncthreads();
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
  const int b = blockIdx.x * 4 + w;
  if (b >= B) return;
  const unsigned short* zb = zbf + (long)b * ldz;
  f32x4 acc[NT][NT];
#pragma unroll
  for (int i = 0; i < NT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float zs[NT];
#pragma unroll
  for (int i = 0; i < NT; ++i) zs[i] = 0.f;
  uint32_t cur[NT][8], nxt[NT][8];
  auto load = [&](int f0, uint32_t (&v)[NT][8]) {
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const int f = f0 + 8 * g + t;
#pragma unroll
      for (int i = 0; i < NT; ++i) v[i][t] = f < F ? (uint32_t)zb[(long)f * D + 16 * i + c] : 0u;
    }
  };
  if (F > 0) load(0, cur);
  for (int f0 = 0; f0 < F; f0 += 32) {
    if (f0 + 32 < F) load(f0 + 32, nxt);
    gbf16x8 fr[NT];
#pragma unroll
    for (int i = 0; i < NT; ++i) {
#pragma unroll
      for (int t = 0; t < 8; ++t) zs[i] += bfw(cur[i][t]);
      const gu32x4 u = {cur[i][0] | (cur[i][1] << 16), cur[i][2] | (cur[i][3] << 16), cur[i][4] | (cur[i][5] << 16),
                        cur[i][6] | (cur[i][7] << 16)};
      fr[i] = __builtin_bit_cast(gbf16x8, u);
    }
#pragma unroll
    for (int i = 0; i < NT; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j) acc[i][j] = mfma_g(fr[i], fr[j], acc[i][j]);
#pragma unroll
    for (int i = 0; i < NT; ++i)
#pragma unroll
      for (int t = 0; t < 8; ++t) cur[i][t] = nxt[i][t];
  }
#pragma unroll
  for (int i = 0; i < NT; ++i) {
    zs[i] += __shfl_xor(zs[i], 16);
    zs[i] += __shfl_xor(zs[i], 32);
  }
  float* zw = szs + w * D;
  if (g == 0) {
#pragma unroll
    for (int i = 0; i < NT; ++i) {
      zw[16 * i + c] = zs[i];
      zsum_out[(long)b * D + 16 * i + c] = zs[i];
    }
  }
  float* Gb = G_out + (long)b * D * D;
#pragma unroll
  for (int i = 0; i < NT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float* gp = Gb + (16 * i + 4 * g + r) * D + 16 * j + c;
        *gp = acc_out ? *gp + acc[i][j][r] : acc[i][j][r];
      }
  __builtin_amdgcn_wave_barrier();
  for (int t = 0; t < QRp / 16; ++t) {        // S = zsum U, sum_f A^2 = diag(U^T G U): as qnn_gram_fwd_kernel
    const int cc = 16 * t + c;
    float sv = 0.f;
#pragma unroll 8
    for (int d = 0; d < D; ++d) sv = fmaf(zw[d], sU[d * US + cc], sv);
    float sa2 = 0.f;
#pragma unroll
    for (int jd = 0; jd < NT; ++jd) {
      f32x4 h = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < NT; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) h = mfma4q(acc[i][jd][r], sU[(16 * i + 4 * g + r) * US + cc], h);
#pragma unroll
      for (int r = 0; r < 4; ++r) sa2 = fmaf(h[r], sU[(16 * jd + 4 * g + r) * US + cc], sa2);
    }
    sa2 += __shfl_xor(sa2, 16);
    sa2 += __shfl_xor(sa2, 32);
    if (g == 0 && cc < QR) {
      S_out[(long)b * QR + cc] = sv;
      float* qp = quad_out + (long)b * QR + cc;
      *qp = acc_out ? *qp + (sv * sv - sa2) : sv * sv - sa2;
    }
  }
}

// One sample per 4-wave workgroup (as qnn_gram_bwd_kernel): M and w in fp32 as there; then each wave takes every
// fourth 16-row F block: dz_f = 2 w - 2 M bf16(z_f) (+ dz_add) on v_mfma_f32_16x16x32_bf16 -- A = the block's bf16 z
// rows (lane (g, c): row f0 + c, columns 32 kh + 8g .. +7, one 16-byte load), B = bf16(M) columns read from the fp32
// M tiles in LDS once per wave.  dz_add / dz rows have their own stride ld.
template <int D, class TA, bool ADD>
__global__ __launch_bounds__(256) void qnn_gram_bwd_bf_kernel(const unsigned short* __restrict__ zbf, long ldz, long ld,
                                                              int B, int F, const float* __restrict__ ucat, int QR,
                                                              const float* __restrict__ S,
                                                              const float* __restrict__ dquad,
                                                              const TA* __restrict__ dz_add, float* __restrict__ dz,
                                                              float* __restrict__ DS) {
  constexpr int NT = D / 16, KH = D / 32;
  extern __shared__ float sU[];
  const int QRp = (QR + 15) / 16 * 16, US = QRp + 1;
  float* dq = sU + D * US;
  float* dqs = dq + QRp;
  float* sM = dqs + QRp;                         // [NT*NT tiles][4][64] M (C layout)
  float* sW = sM + NT * NT * 4 * 64;
  const int b = blockIdx.x;
  const unsigned short* zb = zbf + (long)b * ldz;
  const TA* ab = ADD ? dz_add + (long)b * ld : nullptr;
  using AR = typename GramAdd<TA>::R;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
  // this wave's first block's z rows and addends, loaded before the staging (their round trips overlap it)
  auto load_blk = [&](int f0, gu32x4 (&zq)[KH], AR (&aq)[4][NT]) {
    const int fa = min(f0 + c, F - 1);           // rows past F: row F - 1 re-read (never stored)
#pragma unroll
    for (int kh = 0; kh < KH; ++kh) zq[kh] = *(const gu32x4*)(zb + (long)fa * D + 32 * kh + 8 * g);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int f = min(f0 + 4 * g + r, F - 1);
#pragma unroll
      for (int j = 0; j < NT; ++j) aq[r][j] = ADD ? GramAdd<TA>::load(ab + (long)f * D + 16 * j + c) : AR(0);
    }
  };
  gu32x4 zc[KH], zn[KH];
  AR ac[4][NT], an[4][NT];
  if (16 * w < F) load_blk(16 * w, zc, ac);
  stage_ucat<D>(ucat, QR, QRp, sU);
  for (int q = threadIdx.x; q < QRp; q += 256) {
    const float d = q < QR ? dquad[(long)b * QR + q] : 0.f;
    const float sv = q < QR ? S[(long)b * QR + q] : 0.f;
    dq[q] = d;
    dqs[q] = d * sv;
    if (q < QR) DS[(long)b * QR + q] = d * sv;
  }
  __syncthreads();
  for (int t = w; t < NT * NT; t += 4) {
    const int i = t / NT, j = t - i * NT;
    f32x4 Mt = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int k0 = 0; k0 < QRp; k0 += 4) {
      const int k = k0 + g;
      const float bi = sU[(16 * i + c) * US + k];
      const float bj = sU[(16 * j + c) * US + k];
      Mt = mfma4q(bi * dq[k], bj, Mt);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) sM[(t * 4 + r) * 64 + lane] = Mt[r];
  }
  {
    const int kq = QRp / 4;
    const int k0w = w * kq, k1w = k0w + kq;
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      float a = 0.f;
      for (int q = k0w + g; q < k1w; q += 4) a = fmaf(sU[(16 * j + c) * US + q], dqs[q], a);
      a += __shfl_xor(a, 16);
      a += __shfl_xor(a, 32);
      if (g == 0) sW[w * D + 16 * j + c] = a;
    }
  }
  __syncthreads();
  // B operand of output column block j, k-step kh: lane (g, c) <- bf16(M[32 kh + 8g + t][16 j + c]), t < 8; M's C
  // layout keeps M[16 i + 4 g' + r][16 j + c'] at sM[((i NT + j) 4 + r) 64 + 16 g' + c']
  gbf16x8 mb[NT][KH];
#pragma unroll
  for (int j = 0; j < NT; ++j)
#pragma unroll
    for (int kh = 0; kh < KH; ++kh) {
      float mv[8];
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        const int row = 32 * kh + 8 * g + t, i = row >> 4, gg = (row & 15) >> 2, r = row & 3;
        mv[t] = sM[((i * NT + j) * 4 + r) * 64 + 16 * gg + c];
      }
      mb[j][kh] = gbf16x8{(__bf16)mv[0], (__bf16)mv[1], (__bf16)mv[2], (__bf16)mv[3],
                          (__bf16)mv[4], (__bf16)mv[5], (__bf16)mv[6], (__bf16)mv[7]};
    }
  float wv[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int e = 16 * j + c;
    wv[j] = 2.f * (((sW[e] + sW[D + e]) + sW[2 * D + e]) + sW[3 * D + e]);
  }
  float* ob = dz + (long)b * ld;
  for (int f0 = 16 * w; f0 < F; f0 += 64) {
    const bool more = f0 + 64 < F;
    if (more) load_blk(f0 + 64, zn, an);
    f32x4 acc[NT];
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kh = 0; kh < KH; ++kh) acc[j] = mfma_g(__builtin_bit_cast(gbf16x8, zc[kh]), mb[j][kh], acc[j]);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int f = f0 + 4 * g + r;
      if (f < F) {
#pragma unroll
        for (int j = 0; j < NT; ++j) {
          float v = wv[j] - 2.f * acc[j][r];
          if (ADD) v += GramAdd<TA>::widen(ac[r][j]);
          ob[(long)f * D + 16 * j + c] = v;
        }
      }
    }
    if (more) {
#pragma unroll
      for (int kh = 0; kh < KH; ++kh) zc[kh] = zn[kh];
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int j = 0; j < NT; ++j) ac[r][j] = an[r][j];
    }
  }
}

// dUcat[d][c] = 2 (T1[d][c] - sum_e U[e][c] T[d*D + e][c])
__global__ void qnn_du_combine_kernel(const float* __restrict__ T1, const float* __restrict__ T,
                                      const float* __restrict__ ucat, int D, int QR, float* __restrict__ du) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= D * QR) return;
  const int d = q / QR, c = q % QR;
  float s = 0.f;
  for (int e = 0; e < D; ++e) s = fmaf(ucat[e * QR + c], T[((long)d * D + e) * QR + c], s);
  du[q] = 2.f * (T1[q] - s);
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
                                  Drop drop, float* __restrict__ out, long out_ld, __bf16* __restrict__ obf = nullptr,
                                  long obf_ld = 0) {
  const long n = (long)B * C;
  for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q < n; q += (long)gridDim.x * blockDim.x) {
    const int c = (int)(q % C);
    const long b = q / C;
    float v = x[q];
    if (gate) v = v * gate[c];
    const float o = drop_apply(drop, (uint32_t)q, v);
    out[b * out_ld + c] = o;
    if (obf) obf[b * obf_ld + c] = (__bf16)o;     // amp: the GEMM's bf16 image
  }
}

// dpost = drop_bwd(dout); dx_direct = dpost*gate; part(dgate) = sum_b dpost*x over row chunks.  A thread's rows go
// in chunks of 16 whose loads are issued together (the per-row flag branches had put a wait behind every load)
template <class TD, bool GATE, bool DROP>
__global__ __launch_bounds__(256) void se_bwd_partial(const TD* __restrict__ dout, long dout_ld,
                                                      const float* __restrict__ x, int B, int C,
                                                      const float* __restrict__ gate, Drop drop,
                                                      int rows_per_block, float* __restrict__ dx,
                                                      float* __restrict__ part) {
  constexpr int CH = 16;
  const int b0 = blockIdx.y * rows_per_block, b1 = min(B, b0 + rows_per_block);
  for (int c = blockIdx.x * 256 + threadIdx.x; c < C; c += gridDim.x * 256) {
    float acc = 0.f;
    const float gc = GATE ? gate[c] : 1.f;
    for (int r0 = b0; r0 < b1; r0 += CH) {
      float gv[CH], xv[CH];
#pragma unroll
      for (int u = 0; u < CH; ++u) {
        const int b = min(r0 + u, b1 - 1);
        gv[u] = (float)dout[(long)b * dout_ld + c];
        xv[u] = GATE ? x[(long)b * C + c] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < CH; ++u) {
        const int b = r0 + u;
        if (b >= b1) break;
        const long q = (long)b * C + c;
        float g = gv[u];
        if (DROP) g = drop_keep(drop, (uint32_t)q) ? g * drop.scale : 0.f;
        if (GATE) {
          dx[q] = g * gc;
          acc = fmaf(g, xv[u], acc);
        } else {
          dx[q] = g;
        }
      }
    }
    if (GATE && part) part[(long)blockIdx.y * C + c] = acc;
  }
}

template <class TD>
static void se_bwd_partial_launch(dim3 grid, hipStream_t s, const TD* dout, long dout_ld, const float* x, int B, int C,
                                  const float* gate, Drop d, int rpb, float* dx, float* part) {
  if (gate && d.thresh) se_bwd_partial<TD, true, true><<<grid, 256, 0, s>>>(dout, dout_ld, x, B, C, gate, d, rpb, dx, part);
  else if (gate) se_bwd_partial<TD, true, false><<<grid, 256, 0, s>>>(dout, dout_ld, x, B, C, gate, d, rpb, dx, part);
  else if (d.thresh) se_bwd_partial<TD, false, true><<<grid, 256, 0, s>>>(dout, dout_ld, x, B, C, gate, d, rpb, dx, part);
  else se_bwd_partial<TD, false, false><<<grid, 256, 0, s>>>(dout, dout_ld, x, B, C, gate, d, rpb, dx, part);
}

// dgate[c] = sum of the row-block partials (fixed order); dz2 = dgate * sigmoid'(.)  -> db2, dz2
// (64 columns per workgroup; its four waves sum interleaved quarters of the partials, combined in order)
__global__ __launch_bounds__(256) void se_dgate_kernel(const float* __restrict__ part, int nparts, int C,
                                                       const float* __restrict__ gate, float* __restrict__ db2,
                                                       float* __restrict__ dz2) {
  __shared__ float red[4][64];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + tx;
  float t = 0.f;
  if (c < C)
    for (int p = ty; p < nparts; p += 4) t += part[(long)p * C + c];
  red[ty][tx] = t;
  __syncthreads();
  if (ty != 0 || c >= C) return;
  const float dg = ((red[0][tx] + red[1][tx]) + red[2][tx]) + red[3][tx];
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

extern "C" int ctr_qnn_vfull(const float* V, int H, int R, int P, float* vfull, int inverse, void* stream) {
  const long n = inverse ? (long)H * R * P : (long)H * R * H * P;
  vfull_kernel<<<(unsigned)std::min<long>(cdiv(n, 256L), 4096L), 256, 0, (hipStream_t)stream>>>(V, H, R, P, vfull,
                                                                                              inverse);
  return check_launch("qnn_vfull");
}

static size_t gram_lds(int D, int QR) {
  const int QRp = (QR + 15) / 16 * 16;
  return ((size_t)D * (QRp + 1) + 8 * (size_t)std::max(D, QRp)) * sizeof(float);
}

extern "C" int ctr_qnn_gram_fwd_ex(const float* z, long ld, int B, int F, int D, const float* ucat, int QR,
                                   float* zsum, float* G, float* S, float* quad, int accumulate, void* stream) {
  CTR_REQUIRE(D == 16 || D == 32 || D == 64, "qnn gram: D must be 16, 32 or 64");
  CTR_REQUIRE(ld >= (long)F * D, "qnn gram: row stride shorter than F D");
  if (B == 0) return 0;
  const size_t sm = gram_lds(D, QR);
  CTR_REQUIRE(sm <= 64 * 1024, "qnn gram: U exceeds LDS");
  hipStream_t s = (hipStream_t)stream;
  const int blocks = cdiv(B, 4);
  if (D == 16) qnn_gram_fwd_kernel<16><<<blocks, 256, sm, s>>>(z, ld, B, F, ucat, QR, zsum, G, S, quad, accumulate);
  else if (D == 32) qnn_gram_fwd_kernel<32><<<blocks, 256, sm, s>>>(z, ld, B, F, ucat, QR, zsum, G, S, quad, accumulate);
  else qnn_gram_fwd_kernel<64><<<blocks, 256, sm, s>>>(z, ld, B, F, ucat, QR, zsum, G, S, quad, accumulate);
  return check_launch("qnn_gram_fwd");
}

extern "C" int ctr_qnn_gram_fwd(const float* z, int B, int F, int D, const float* ucat, int QR, float* zsum,
                                float* G, float* S, float* quad, void* stream) {
  return ctr_qnn_gram_fwd_ex(z, (long)F * D, B, F, D, ucat, QR, zsum, G, S, quad, 0, stream);
}

template <class TA, bool ADD>
static void gram_bwd_launch(int D, int blocks, size_t sm, hipStream_t s, const float* z, long ld, int B, int F,
                            const float* ucat, int QR, const float* S, const float* dquad, const TA* dz_add, float* dz,
                            float* DS) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)qnn_gram_bwd_kernel<16, TA, ADD>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute((const void*)qnn_gram_bwd_kernel<32, TA, ADD>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute((const void*)qnn_gram_bwd_kernel<64, TA, ADD>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  if (D == 16) qnn_gram_bwd_kernel<16, TA, ADD><<<blocks, 256, sm, s>>>(z, ld, B, F, ucat, QR, S, dquad, dz_add, dz, DS);
  else if (D == 32) qnn_gram_bwd_kernel<32, TA, ADD><<<blocks, 256, sm, s>>>(z, ld, B, F, ucat, QR, S, dquad, dz_add, dz, DS);
  else qnn_gram_bwd_kernel<64, TA, ADD><<<blocks, 256, sm, s>>>(z, ld, B, F, ucat, QR, S, dquad, dz_add, dz, DS);
}

extern "C" int ctr_qnn_gram_bwd_ex(const float* z, long ld, int B, int F, int D, const float* ucat, int QR,
                                   const float* S, const float* dquad, const void* dz_add, int add_bf16, float* dz,
                                   float* DS, void* stream) {
  CTR_REQUIRE(D == 16 || D == 32 || D == 64, "qnn gram: D must be 16, 32 or 64");
  CTR_REQUIRE(ld >= (long)F * D, "qnn gram: row stride shorter than F D");
  if (B == 0) return 0;
  const int QRp = (QR + 15) / 16 * 16, NT = D / 16;
  const size_t sm = ((size_t)D * (QRp + 1) + 2 * (size_t)QRp + (size_t)NT * NT * 4 * 64 + 4 * (size_t)D) *
                    sizeof(float);
  CTR_REQUIRE(sm <= 160 * 1024, "qnn gram bwd: U + M partials exceed LDS");
  hipStream_t s = (hipStream_t)stream;
  if (!dz_add) gram_bwd_launch<float, false>(D, B, sm, s, z, ld, B, F, ucat, QR, S, dquad, nullptr, dz, DS);
  else if (add_bf16)
    gram_bwd_launch<__bf16, true>(D, B, sm, s, z, ld, B, F, ucat, QR, S, dquad, (const __bf16*)dz_add, dz, DS);
  else gram_bwd_launch<float, true>(D, B, sm, s, z, ld, B, F, ucat, QR, S, dquad, (const float*)dz_add, dz, DS);
  return check_launch("qnn_gram_bwd");
}

extern "C" int ctr_qnn_gram_bwd(const float* z, int B, int F, int D, const float* ucat, int QR, const float* S,
                                const float* dquad, const void* dz_add, int add_bf16, float* dz, float* DS,
                                void* stream) {
  return ctr_qnn_gram_bwd_ex(z, (long)F * D, B, F, D, ucat, QR, S, dquad, dz_add, add_bf16, dz, DS, stream);
}

extern "C" int ctr_qnn_gram_fwd_zbf(const uint16_t* zbf, long ldz, int B, int F, int D, const float* ucat, int QR,
                                    float* zsum, float* G, float* S, float* quad, int accumulate, void* stream) {
  CTR_REQUIRE(D == 32 || D == 64, "qnn gram (bf16 z): D must be 32 or 64");
  CTR_REQUIRE(ldz >= (long)F * D && (ldz % 8) == 0, "qnn gram (bf16 z): row stride");
  if (B == 0) return 0;
  const size_t sm = gram_lds(D, QR);
  CTR_REQUIRE(sm <= 64 * 1024, "qnn gram: U exceeds LDS");
  hipStream_t s = (hipStream_t)stream;
  const int blocks = cdiv(B, 4);
  const unsigned short* z = (const unsigned short*)zbf;
  if (D == 32) qnn_gram_fwd_bf_kernel<32><<<blocks, 256, sm, s>>>(z, ldz, B, F, ucat, QR, zsum, G, S, quad, accumulate);
  else qnn_gram_fwd_bf_kernel<64><<<blocks, 256, sm, s>>>(z, ldz, B, F, ucat, QR, zsum, G, S, quad, accumulate);
  return check_launch("qnn_gram_fwd_zbf");
}

template <class TA, bool ADD>
static void gram_bwd_bf_launch(int D, size_t sm, hipStream_t s, const unsigned short* z, long ldz, long ld, int B,
                               int F, const float* ucat, int QR, const float* S, const float* dquad, const TA* dz_add,
                               float* dz, float* DS) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)qnn_gram_bwd_bf_kernel<32, TA, ADD>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute((const void*)qnn_gram_bwd_bf_kernel<64, TA, ADD>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  if (D == 32) qnn_gram_bwd_bf_kernel<32, TA, ADD><<<B, 256, sm, s>>>(z, ldz, ld, B, F, ucat, QR, S, dquad, dz_add, dz, DS);
  else qnn_gram_bwd_bf_kernel<64, TA, ADD><<<B, 256, sm, s>>>(z, ldz, ld, B, F, ucat, QR, S, dquad, dz_add, dz, DS);
}

extern "C" int ctr_qnn_gram_bwd_zbf(const uint16_t* zbf, long ldz, long ld, int B, int F, int D, const float* ucat,
                                    int QR, const float* S, const float* dquad, const void* dz_add, int add_bf16,
                                    float* dz, float* DS, void* stream) {
  CTR_REQUIRE(D == 32 || D == 64, "qnn gram (bf16 z): D must be 32 or 64");
  CTR_REQUIRE(ldz >= (long)F * D && (ldz % 8) == 0 && ld >= (long)F * D, "qnn gram (bf16 z): row strides");
  CTR_REQUIRE((((uintptr_t)zbf) & 15) == 0, "qnn gram (bf16 z): 16-byte aligned rows");
  if (B == 0) return 0;
  const int QRp = (QR + 15) / 16 * 16, NT = D / 16;
  const size_t sm = ((size_t)D * (QRp + 1) + 2 * (size_t)QRp + (size_t)NT * NT * 4 * 64 + 4 * (size_t)D) *
                    sizeof(float);
  CTR_REQUIRE(sm <= 160 * 1024, "qnn gram bwd: U + M partials exceed LDS");
  hipStream_t s = (hipStream_t)stream;
  const unsigned short* z = (const unsigned short*)zbf;
  if (!dz_add) gram_bwd_bf_launch<float, false>(D, sm, s, z, ldz, ld, B, F, ucat, QR, S, dquad, nullptr, dz, DS);
  else if (add_bf16)
    gram_bwd_bf_launch<__bf16, true>(D, sm, s, z, ldz, ld, B, F, ucat, QR, S, dquad, (const __bf16*)dz_add, dz, DS);
  else gram_bwd_bf_launch<float, true>(D, sm, s, z, ldz, ld, B, F, ucat, QR, S, dquad, (const float*)dz_add, dz, DS);
  return check_launch("qnn_gram_bwd_zbf");
}

// pair_grouping 'block': the rows' columns outside every interaction block (single-feature blocks, e.g. the DARE
// output u) take no interaction gradient -- dz = the MLP's input-grad addend (fp32 or bf16), or 0 without one
__global__ void qnn_passthrough_kernel(const void* __restrict__ add, int add_bf16, long ld_add, int B, int ncols,
                                       float* __restrict__ dst, long ld) {
  const long n = (long)B * ncols;
  for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q < n; q += (long)gridDim.x * blockDim.x) {
    const long b = q / ncols, j = q - b * ncols;
    float v = 0.f;
    if (add) {
      if (add_bf16) v = __builtin_bit_cast(float, (uint32_t)((const unsigned short*)add)[b * ld_add + j] << 16);
      else v = ((const float*)add)[b * ld_add + j];
    }
    dst[b * ld + j] = v;
  }
}

extern "C" int ctr_qnn_passthrough(const void* add, int add_bf16, long ld_add, int B, int ncols, float* dst, long ld,
                                   void* stream) {
  if (B == 0 || ncols == 0) return 0;
  const long n = (long)B * ncols;
  qnn_passthrough_kernel<<<(unsigned)std::min<long>(cdiv(n, 256L), 2048), 256, 0, (hipStream_t)stream>>>(
      add, add_bf16, ld_add, B, ncols, dst, ld);
  return check_launch("qnn_passthrough");
}

extern "C" int ctr_qnn_du_combine(const float* T1, const float* T, const float* ucat, int D, int QR, float* ducat,
                                  void* stream) {
  qnn_du_combine_kernel<<<cdiv((long)D * QR, 256L), 256, 0, (hipStream_t)stream>>>(T1, T, ucat, D, QR, ducat);
  return check_launch("qnn_du_combine");
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

extern "C" int ctr_scale_drop_bf(const float* x, int B, int C, const float* gate, uint32_t drop_key, uint32_t drop_thresh,
                                 float drop_scale, float* out, long out_ld, void* obf, long obf_ld, void* stream) {
  if (B == 0) return 0;
  long n = (long)B * C;
  int blocks = (int)std::min<long>((n + 255) / 256, 16384);
  scale_drop_kernel<<<blocks, 256, 0, (hipStream_t)stream>>>(x, B, C, gate, Drop{drop_key, drop_thresh, drop_scale},
                                                             out, out_ld, (__bf16*)obf, obf_ld);
  return check_launch("scale_drop_bf");
}

constexpr int SE_RPB = 32;     // rows per se_bwd_partial workgroup (B = 4096: 5 x 128 workgroups)

extern "C" size_t ctr_se_bwd_ws(int B, int C) {
  return ((size_t)cdiv(B, SE_RPB) * C + 3 * (size_t)C) * sizeof(float);
}

extern "C" int ctr_se_bwd(const void* dout, long dout_ld, int dout_bf16, const float* x, int B, int C, int Cr,
                          const float* gate,
                          const float* g1, const float* mean, const float* W1, const float* W2, uint32_t drop_key,
                          uint32_t drop_thresh, float drop_scale, float* dx, float* dW1, float* db1, float* dW2,
                          float* db2, float* ws, void* stream) {
  if (B == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  const int rpb = SE_RPB;
  const int np = cdiv(B, rpb);
  float* part = ws;                      // [np][C]
  float* dmean = ws + (size_t)np * C;    // [C]
  Drop d{drop_key, drop_thresh, drop_scale};
  const dim3 grid(cdiv(C, 256), np);
  if (dout_bf16)
    se_bwd_partial_launch(grid, s, (const __bf16*)dout, dout_ld, x, B, C, gate, d, rpb, dx, gate ? part : nullptr);
  else
    se_bwd_partial_launch(grid, s, (const float*)dout, dout_ld, x, B, C, gate, d, rpb, dx, gate ? part : nullptr);
  if (gate) {
    float* dz2 = dmean + C;                // [C]
    float* dz1 = dz2 + C;                  // [Cr <= C]
    se_dgate_kernel<<<cdiv(C, 64), 256, 0, s>>>(part, np, C, gate, db2, dz2);
    matvec_cols_kernel<<<cdiv(Cr, 4), 256, 0, s>>>(W2, C, Cr, dz2, g1, db1, dz1);     // dz1 = relu'(W2^T dz2)
    matvec_cols_kernel<<<cdiv(C, 4), 256, 0, s>>>(W1, Cr, C, dz1, nullptr, dmean, nullptr);   // W1^T dz1
    se_mlp_bwd_outer<<<cdiv(2L * C * Cr, 256), 256, 0, s>>>(C, Cr, mean, g1, dz2, dz1, dW1, dW2);
    long n = (long)B * C;
    int blocks = (int)std::min<long>((n + 255) / 256, 16384);
    add_row_bcast<<<blocks, 256, 0, s>>>(dx, B, C, dmean, (float)B);
  }
  return check_launch("se_bwd");
}

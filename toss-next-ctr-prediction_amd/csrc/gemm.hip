// fp32 GEMM on CDNA4 matrix cores (v_mfma_f32_16x16x4_f32) with fused epilogues.
//
// One 256-thread workgroup (4 waves, 2x2) computes a BM x BN tile; BK = 16 k-slices are staged
// global -> registers -> LDS (double buffered, one barrier per k-slice).  LDS rows are strided
// BM+16 / BN+16 floats (== 16 mod 32 banks) so the two 16-lane halves of a ds_read_b32 that read
// adjacent k-rows never hit the same bank.  The epilogue re-stages the accumulator tile through
// LDS so stores are row-contiguous and row-wise epilogues (residual + RMSNorm) see whole rows.
//
// f32-input MFMA is bit-for-bit a k-ordered fmaf chain per lane; results differ from the reference's
// MKL sgemm only by summation order (covered by the 1e-4 parity tolerance).
//
// BF = true (amp: bf16, the reference's torch.autocast(bfloat16) Linear / matmul): the same loaders read
// fp32 from HBM, the staging store rounds to bf16 (v_cvt_pk_bf16_f32, round-to-nearest-even) into
// [row][k] LDS tiles of BK = 32, and v_mfma_f32_16x16x32_bf16 accumulates in fp32 -- one MFMA per
// 16x16 block and k-slice where the fp32 form issues eight.  Outputs and epilogues stay fp32.
#include <cstdlib>

#include "common.h"
#include "ctr_hip.h"

namespace ctr {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

struct GemmArgs {
  int M, N, K;
  const float* A;
  int lda;
  const float* B;
  int ldb;
  float* C;
  int ldc;
  ctr_gemm_epi_t epi;
  int klen;        // K elements per split
  float* ws;       // split-K slabs [splits][M][N]
  int vecA, vecB;  // 16-byte loads legal
  // operand / result segments (ctr_gemm_seg): A columns k >= ka from A2, B columns n >= nb from B2 (both
  // non-transposed), C columns n >= nc to C2 -- one launch for a GEMM over concatenated buffers
  const float* A2;
  int lda2, ka;
  const float* B2;
  int ldb2, nb;
  float* C2;
  int ldc2, nc;
};

__device__ __forceinline__ float* cptr(const GemmArgs& g, int m, int n) {
  return (g.C2 && n >= g.nc) ? g.C2 + (long)m * g.ldc2 + (n - g.nc) : g.C + (long)m * g.ldc + n;
}

__device__ __forceinline__ float epi_elem(const ctr_gemm_epi_t& e, float v, int m, int n, int N, int ldc) {
  if (e.dact) {
    if (e.drop_thresh) {
      Drop d{e.drop_key, e.drop_thresh, e.drop_scale};
      v = drop_keep(d, (uint32_t)((long)m * N + n)) ? v * e.drop_scale : 0.0f;
    }
    const float a = e.aux[(long)m * ldc + n];
    v = (e.dact == 1) ? (a > 0.f ? v : 0.f) : v * gelu_grad(a);
  }
  if (e.bias) v += e.bias[n];
  if (e.add) v += e.add[(long)m * e.ld_add + n];
  if (e.pre) e.pre[(long)m * ldc + n] = v;
  if (e.act == 1) v = v > 0.f ? v : 0.f;
  else if (e.act == 2) v = gelu_f(v);
  if (!e.dact && e.drop_thresh) {
    Drop d{e.drop_key, e.drop_thresh, e.drop_scale};
    v = drop_apply(d, (uint32_t)((long)m * N + n), v);
  }
  return v;
}

template <int BM, int BN, bool TA, bool TB, int BFK = 0>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(BFK ? 2 : 4))) void gemm_kernel(GemmArgs g) {
  constexpr bool BF = BFK > 0;               // BFK: bf16 k-slice depth (32 or 64), 0 = fp32
  constexpr int BK = BF ? BFK : 16;
  constexpr int SA = BM + 16, SB = BN + 16;
  constexpr int SK = BK + 8;                 // bf16 tiles: [row][k] rows of 40 bf16 (80 B: conflict-free b128)
  constexpr int WM = BM / 2, WN = BN / 2;
  constexpr int TM = WM / 16, TN = WN / 16;
  constexpr int SC = BN + 4;
  constexpr int LDS_K = BF ? (2 * (BM + BN) * SK + 1) / 2 : 2 * BK * (SA + SB);
  // only the fused residual+RMSNorm epilogue (BN <= 64 tiles) stages the tile through LDS; every other
  // epilogue runs straight from the accumulator registers (keeps big tiles at 4 workgroups / CU)
  constexpr int LDS_E = BN <= 64 ? BM * SC : 0;
  constexpr int LDS = LDS_K > LDS_E ? LDS_K : LDS_E;
  __shared__ __attribute__((aligned(16))) float smem[LDS];
  float* As = smem;
  float* Bs = smem + 2 * BK * SA;
  __bf16* Ah = (__bf16*)smem;                // BF: [2][BM][SK]
  __bf16* Bh = Ah + 2 * BM * SK;             // BF: [2][BN][SK]

  constexpr int A_V = BM * BK / 4, B_V = BN * BK / 4;           // float4 slots per tile
  // BF with the operand stored k-major (A: TA, B: !TB): each thread loads a 4k x 4row block (four float4
  // rows, lanes of one row block cover its eight k blocks: 128-B lines) and stores it transposed as four
  // 8-byte bf16x4 row segments -- [row][k] tiles without 2-byte scattered stores (16-way bank conflicts)
  constexpr bool A_BLK = BF && TA, B_BLK = BF && !TB;
  constexpr int A_NB = BM * BK / 16, B_NB = BN * BK / 16;       // 4x4 blocks per tile
  constexpr int A_IT = A_BLK ? 4 * ((A_NB + 255) / 256) : (A_V + 255) / 256;
  constexpr int B_IT = B_BLK ? 4 * ((B_NB + 255) / 256) : (B_V + 255) / 256;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = (wid >> 1) * WM, wn = (wid & 1) * WN;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  const int kz0 = blockIdx.z * g.klen;
  const int kz1 = min(g.K, kz0 + g.klen);
  const int nkt = kz1 > kz0 ? (kz1 - kz0 + BK - 1) / BK : 0;

  f32x4 ra[A_IT], rb[B_IT];

  auto load_a = [&](int k0) {
    if constexpr (A_BLK) {      // A stored [k][m]: block (kb, ib) = k 4kb.., rows 4ib..
#pragma unroll
      for (int bi = 0; bi < A_IT / 4; ++bi) {
        const int e = tid + bi * 256, kb = e % (BK / 4), ib = e / (BK / 4);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          f32x4 v = {0.f, 0.f, 0.f, 0.f};
          const int kk = k0 + 4 * kb + t, m = m0 + 4 * ib;
          if (e < A_NB && kk < kz1) {
            const float* p = g.A + (long)kk * g.lda + m;
            if (g.vecA && m + 3 < g.M) v = *(const f32x4*)p;
            else {
#pragma unroll
              for (int j = 0; j < 4; ++j) v[j] = (m + j < g.M) ? p[j] : 0.f;
            }
          }
          ra[4 * bi + t] = v;
        }
      }
      return;
    }
#pragma unroll
    for (int it = 0; it < A_IT; ++it) {
      const int e = tid + it * 256;
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (e < A_V) {
        if (!TA) {  // A[m][k], k contiguous
          const int i = e / (BK / 4), kq = (e % (BK / 4)) * 4;
          const int m = m0 + i, k = k0 + kq;
          if (m < g.M) {
            if (g.A2 == nullptr || k + 3 < g.ka) {
              const float* p = g.A + (long)m * g.lda + k;
              if (g.vecA && k + 3 < kz1) v = *(const f32x4*)p;
              else {
#pragma unroll
                for (int j = 0; j < 4; ++j) v[j] = (k + j < kz1) ? p[j] : 0.f;
              }
            } else if (k >= g.ka) {
              const float* p = g.A2 + (long)m * g.lda2 + (k - g.ka);
              if (g.vecA && k + 3 < kz1) v = *(const f32x4*)p;
              else {
#pragma unroll
                for (int j = 0; j < 4; ++j) v[j] = (k + j < kz1) ? p[j] : 0.f;
              }
            } else {
#pragma unroll
              for (int j = 0; j < 4; ++j) {
                const int kk = k + j;
                v[j] = kk >= kz1 ? 0.f : kk < g.ka ? g.A[(long)m * g.lda + kk] : g.A2[(long)m * g.lda2 + (kk - g.ka)];
              }
            }
          }
        } else {    // A stored [k][m], m contiguous
          const int k = e / (BM / 4), iq = (e % (BM / 4)) * 4;
          const int kk = k0 + k, m = m0 + iq;
          if (kk < kz1) {
            const float* p = g.A + (long)kk * g.lda + m;
            if (g.vecA && m + 3 < g.M) v = *(const f32x4*)p;
            else {
#pragma unroll
              for (int j = 0; j < 4; ++j) v[j] = (m + j < g.M) ? p[j] : 0.f;
            }
          }
        }
      }
      ra[it] = v;
    }
  };
  auto load_b = [&](int k0) {
    if constexpr (B_BLK) {      // B stored [k][n] (n columns 0..nb from B, past nb from B2)
#pragma unroll
      for (int bi = 0; bi < B_IT / 4; ++bi) {
        const int e = tid + bi * 256, kb = e % (BK / 4), nbk = e / (BK / 4);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          f32x4 v = {0.f, 0.f, 0.f, 0.f};
          const int kk = k0 + 4 * kb + t, n = n0 + 4 * nbk;
          if (e < B_NB && kk < kz1) {
            if (g.B2 == nullptr || n + 3 < g.nb) {
              const float* p = g.B + (long)kk * g.ldb + n;
              if (g.vecB && n + 3 < g.N) v = *(const f32x4*)p;
              else {
#pragma unroll
                for (int j = 0; j < 4; ++j) v[j] = (n + j < g.N) ? p[j] : 0.f;
              }
            } else if (n >= g.nb) {
              const float* p = g.B2 + (long)kk * g.ldb2 + (n - g.nb);
              if (g.vecB && n + 3 < g.N) v = *(const f32x4*)p;
              else {
#pragma unroll
                for (int j = 0; j < 4; ++j) v[j] = (n + j < g.N) ? p[j] : 0.f;
              }
            } else {
#pragma unroll
              for (int j = 0; j < 4; ++j) {
                const int nn = n + j;
                v[j] = nn >= g.N ? 0.f : nn < g.nb ? g.B[(long)kk * g.ldb + nn] : g.B2[(long)kk * g.ldb2 + (nn - g.nb)];
              }
            }
          }
          rb[4 * bi + t] = v;
        }
      }
      return;
    }
#pragma unroll
    for (int it = 0; it < B_IT; ++it) {
      const int e = tid + it * 256;
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (e < B_V) {
        if (!TB) {  // B[k][n], n contiguous
          const int k = e / (BN / 4), nq = (e % (BN / 4)) * 4;
          const int kk = k0 + k, n = n0 + nq;
          if (kk < kz1) {
            if (g.B2 == nullptr || n + 3 < g.nb) {
              const float* p = g.B + (long)kk * g.ldb + n;
              if (g.vecB && n + 3 < g.N) v = *(const f32x4*)p;
              else {
#pragma unroll
                for (int j = 0; j < 4; ++j) v[j] = (n + j < g.N) ? p[j] : 0.f;
              }
            } else if (n >= g.nb) {
              const float* p = g.B2 + (long)kk * g.ldb2 + (n - g.nb);
              if (g.vecB && n + 3 < g.N) v = *(const f32x4*)p;
              else {
#pragma unroll
                for (int j = 0; j < 4; ++j) v[j] = (n + j < g.N) ? p[j] : 0.f;
              }
            } else {
#pragma unroll
              for (int j = 0; j < 4; ++j) {
                const int nn = n + j;
                v[j] = nn >= g.N ? 0.f : nn < g.nb ? g.B[(long)kk * g.ldb + nn] : g.B2[(long)kk * g.ldb2 + (nn - g.nb)];
              }
            }
          }
        } else {    // B stored [n][k], k contiguous
          const int n = e / (BK / 4), kq = (e % (BK / 4)) * 4;
          const int nn = n0 + n, k = k0 + kq;
          if (nn < g.N) {
            const float* p = g.B + (long)nn * g.ldb + k;
            if (g.vecB && k + 3 < kz1) v = *(const f32x4*)p;
            else {
#pragma unroll
              for (int j = 0; j < 4; ++j) v[j] = (k + j < kz1) ? p[j] : 0.f;
            }
          }
        }
      }
      rb[it] = v;
    }
  };
  auto store_ab_bf = [&](int buf) {
    __bf16* a = Ah + buf * BM * SK;
    __bf16* b = Bh + buf * BN * SK;
    // a 4k x 4row block -> four bf16x4 row segments (row 4ib + j: k 4kb .. 4kb + 3)
    auto put_block = [&](__bf16* dst, const f32x4* r, int e, int nblk) {
      if (e >= nblk) return;
      const int kb = e % (BK / 4), ib = e / (BK / 4);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        *(bf16x4*)&dst[(4 * ib + j) * SK + 4 * kb] = bf16x4{(__bf16)r[0][j], (__bf16)r[1][j], (__bf16)r[2][j], (__bf16)r[3][j]};
    };
    if constexpr (A_BLK) {
#pragma unroll
      for (int bi = 0; bi < A_IT / 4; ++bi) put_block(a, &ra[4 * bi], tid + bi * 256, A_NB);
    }
    if constexpr (B_BLK) {
#pragma unroll
      for (int bi = 0; bi < B_IT / 4; ++bi) put_block(b, &rb[4 * bi], tid + bi * 256, B_NB);
    }
#pragma unroll
    for (int it = 0; it < (A_BLK ? 0 : A_IT); ++it) {
      const int e = tid + it * 256;
      if (e < A_V) {
        if (!TA) {
          const int i = e / (BK / 4), kq = (e % (BK / 4)) * 4;
          *(bf16x4*)&a[i * SK + kq] = __builtin_convertvector(ra[it], bf16x4);
        } else {
          const int k = e / (BM / 4), iq = (e % (BM / 4)) * 4;
#pragma unroll
          for (int j = 0; j < 4; ++j) a[(iq + j) * SK + k] = (__bf16)ra[it][j];
        }
      }
    }
#pragma unroll
    for (int it = 0; it < (B_BLK ? 0 : B_IT); ++it) {
      const int e = tid + it * 256;
      if (e < B_V) {
        if (!TB) {
          const int k = e / (BN / 4), nq = (e % (BN / 4)) * 4;
#pragma unroll
          for (int j = 0; j < 4; ++j) b[(nq + j) * SK + k] = (__bf16)rb[it][j];
        } else {
          const int n = e / (BK / 4), kq = (e % (BK / 4)) * 4;
          *(bf16x4*)&b[n * SK + kq] = __builtin_convertvector(rb[it], bf16x4);
        }
      }
    }
  };
  auto store_ab = [&](int buf) {
    if constexpr (BF) {
      store_ab_bf(buf);
      return;
    }
    float* a = As + buf * BK * SA;
    float* b = Bs + buf * BK * SB;
#pragma unroll
    for (int it = 0; it < A_IT; ++it) {
      const int e = tid + it * 256;
      if (e < A_V) {
        if (!TA) {
          const int i = e / (BK / 4), kq = (e % (BK / 4)) * 4;
#pragma unroll
          for (int j = 0; j < 4; ++j) a[(kq + j) * SA + i] = ra[it][j];
        } else {
          const int k = e / (BM / 4), iq = (e % (BM / 4)) * 4;
          *(f32x4*)&a[k * SA + iq] = ra[it];
        }
      }
    }
#pragma unroll
    for (int it = 0; it < B_IT; ++it) {
      const int e = tid + it * 256;
      if (e < B_V) {
        if (!TB) {
          const int k = e / (BN / 4), nq = (e % (BN / 4)) * 4;
          *(f32x4*)&b[k * SB + nq] = rb[it];
        } else {
          const int n = e / (BK / 4), kq = (e % (BK / 4)) * 4;
#pragma unroll
          for (int j = 0; j < 4; ++j) b[(kq + j) * SB + n] = rb[it][j];
        }
      }
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (nkt > 0) {
    load_a(kz0);
    load_b(kz0);
    store_ab(0);
    __syncthreads();
  }
  for (int kt = 0; kt < nkt; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nkt) {
      load_a(kz0 + (kt + 1) * BK);
      load_b(kz0 + (kt + 1) * BK);
    }
    if constexpr (BF) {
      // lane (g, c) reads row 16i + c, k = 8g .. 8g + 7 of the A tile (row 16j + c of the B tile)
#pragma unroll
      for (int ks = 0; ks < BK; ks += 32) {
      const __bf16* a = Ah + cur * BM * SK + (lane & 15) * SK + 8 * (lane >> 4) + ks;
      const __bf16* b = Bh + cur * BN * SK + (lane & 15) * SK + 8 * (lane >> 4) + ks;
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = *(const bf16x8*)(a + (wm + i * 16) * SK);
#pragma unroll
      for (int j = 0; j < TN; ++j) bfr[j] = *(const bf16x8*)(b + (wn + j * 16) * SK);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    } else {
    const float* a = As + cur * BK * SA;
    const float* b = Bs + cur * BK * SB;
#pragma unroll
    for (int kk = 0; kk < BK; kk += 4) {
      const int kr = kk + (lane >> 4);
      float af[TM], bf[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = a[kr * SA + wm + i * 16 + (lane & 15)];
#pragma unroll
      for (int j = 0; j < TN; ++j) bf[j] = b[kr * SB + wn + j * 16 + (lane & 15)];
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], bf[j], acc[i][j], 0, 0, 0);
    }
    }
    if (kt + 1 < nkt) store_ab(cur ^ 1);
    __syncthreads();
  }

  const ctr_gemm_epi_t& e = g.epi;
  // accumulator (i, j, r) of this lane holds C[m0 + wm + 16i + 4(lane>>4) + r][n0 + wn + 16j + (lane&15)]
  const int lrow = wm + (lane >> 4) * 4, lcol = wn + (lane & 15);
  if (gridDim.z > 1) {  // split-K partial: raw slab, epilogue happens in the reduce kernel
    float* slab = g.ws + (long)blockIdx.z * g.M * g.N;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = n0 + lcol + j * 16;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + lrow + i * 16 + r;
          if (m < g.M && n < g.N) slab[(long)m * g.N + n] = acc[i][j][r];
        }
      }
    return;
  }
  if constexpr (LDS_E == 0) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = n0 + lcol + j * 16;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + lrow + i * 16 + r;
          if (m < g.M && n < g.N) *cptr(g, m, n) = epi_elem(e, acc[i][j][r], m, n, g.N, g.ldc);
        }
      }
    return;
  } else {
  // ---- fused-norm tiles: stage the accumulator tile through LDS (Cs[i][j], row stride SC) so each
  // row is visible to one thread group ----
  float* Cs = smem;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        Cs[(wm + i * 16 + (lane >> 4) * 4 + r) * SC + wn + j * 16 + (lane & 15)] = acc[i][j][r];
  __syncthreads();

  if (e.norm_w) {  // full row in this tile (host guarantees N <= BN, gridDim.y == 1)
    constexpr int TPR = BN / 4;          // threads per row
    constexpr int RPP = 256 / TPR;       // rows per pass
    const int sub = tid % TPR, rr = tid / TPR;
    for (int i0 = 0; i0 < BM; i0 += RPP) {
      const int i = i0 + rr, m = m0 + i;
      float h[4];
      float ss = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = sub * 4 + j;
        h[j] = 0.f;
        if (m < g.M && n < g.N) {
          float v = Cs[i * SC + n];
          if (e.bias) v += e.bias[n];
          h[j] = e.resid[(long)m * e.ld_resid + n] + v;
          ss += h[j] * h[j];
        }
      }
      ss = group_sum<TPR>(ss);
      const float r = 1.0f / sqrtf(ss / (float)g.N + e.norm_eps);
      if (m < g.M) {
        if (sub == 0 && e.norm_r) e.norm_r[m] = r;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int n = sub * 4 + j;
          if (n < g.N) {
            if (e.norm_h) e.norm_h[(long)m * g.ldc + n] = h[j];
            g.C[(long)m * g.ldc + n] = e.norm_w[n] * h[j] * r;
          }
        }
      }
    }
    return;
  }
  const bool vecC = ((g.ldc & 3) == 0) && ((((uintptr_t)g.C) & 15) == 0);
  for (int q = tid; q < BM * BN / 4; q += 256) {
    const int i = q / (BN / 4), jq = (q % (BN / 4)) * 4;
    const int m = m0 + i, n = n0 + jq;
    if (m >= g.M) continue;
    f32x4 v;
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = (n + j < g.N) ? epi_elem(e, Cs[i * SC + jq + j], m, n + j, g.N, g.ldc) : 0.f;
    float* p = g.C + (long)m * g.ldc + n;
    if (g.C2) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (n + j < g.N) *cptr(g, m, n + j) = v[j];
    } else if (vecC && n + 3 < g.N) *(f32x4*)p = v;
    else {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (n + j < g.N) p[j] = v[j];
    }
  }
  }
}

__global__ void splitk_reduce_kernel(GemmArgs g, int splits) {
  const long MN = (long)g.M * g.N;
  for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q < MN; q += (long)gridDim.x * blockDim.x) {
    float s = 0.f;
    int z = 0;
    for (; z + 8 <= splits; z += 8) {   // 8 independent loads in flight, summed in slab order
      float a[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) a[j] = g.ws[(z + j) * MN + q];
#pragma unroll
      for (int j = 0; j < 8; ++j) s += a[j];
    }
    for (; z < splits; ++z) s += g.ws[z * MN + q];
    const int m = (int)(q / g.N), n = (int)(q % g.N);
    *cptr(g, m, n) = epi_elem(g.epi, s, m, n, g.N, g.ldc);
  }
}

// K <= 4 (e.g. the outer product of the logit grad with the last MLP weight): one thread per C element
__global__ void gemm_smallk_kernel(GemmArgs g, int ta, int tb) {
  const long MN = (long)g.M * g.N;
  for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q < MN; q += (long)gridDim.x * blockDim.x) {
    const int m = (int)(q / g.N), n = (int)(q % g.N);
    float acc = 0.f;
    for (int k = 0; k < g.K; ++k) {
      const float a = ta ? g.A[(long)k * g.lda + m] : g.A[(long)m * g.lda + k];
      const float b = tb ? g.B[(long)n * g.ldb + k] : g.B[(long)k * g.ldb + n];
      acc = fmaf(a, b, acc);
    }
    g.C[(long)m * g.ldc + n] = epi_elem(g.epi, acc, m, n, g.N, g.ldc);
  }
}

template <int BM, int BN, int BF>
static void launch_tile_t(GemmArgs& g, int ta, int tb, int splits, hipStream_t s) {
  dim3 grid(cdiv(g.M, BM), cdiv(g.N, BN), splits);
  if (!ta && !tb) gemm_kernel<BM, BN, false, false, BF><<<grid, 256, 0, s>>>(g);
  else if (!ta && tb) gemm_kernel<BM, BN, false, true, BF><<<grid, 256, 0, s>>>(g);
  else if (ta && !tb) gemm_kernel<BM, BN, true, false, BF><<<grid, 256, 0, s>>>(g);
  else gemm_kernel<BM, BN, true, true, BF><<<grid, 256, 0, s>>>(g);
}

template <int BM, int BN>
static void launch_tile(GemmArgs& g, int ta, int tb, int splits, hipStream_t s, int bf) {
  if (bf == 64) launch_tile_t<BM, BN, 64>(g, ta, tb, splits, s);
  else if (bf) launch_tile_t<BM, BN, 32>(g, ta, tb, splits, s);
  else launch_tile_t<BM, BN, 0>(g, ta, tb, splits, s);
}

// ------------------------------------------------------------------------------------------------
// bf16-operand GEMM (amp: bf16; operands already bf16 in HBM, e.g. the QNN MLP's [z | inter] image).
// 128 x 128 tile, 256 threads (2 x 2 waves of 64 x 64), BK = 64, both operand tiles staged by
// global_load_lds (16 B per lane, no VGPR round trip) into two LDS buffers -- the next k-slice's DMA is in
// flight while the current one is multiplied; one barrier per k-slice.  Operand layouts in LDS:
//   k-contiguous operand (A[m][k] / B[n][k]): [128 rows][64 k] with 128-B rows, the 16-B chunk c of row r
//     stored at chunk c ^ ((r >> 1) & 7) (the swizzle is applied to the per-lane GLOBAL address: the
//     DMA writes lane-linear); fragments are ds_read_b128 -- the 16 rows a read touches land on 16
//     different 16-B bank groups;
//   k-major operand (A[k][m] / B[k][n]): [8 k-blocks][8 col-blocks][8 k][16 cols] 256-B blocks, rows 0-3 and
//     4-7 of odd k-blocks swapped; fragments are two ds_read_b64_tr_b16 (4 k x 16 cols, transposed).
// Rows / columns past M / N are clamped to the last valid one (their results are never stored); K must
// be a multiple of 64 per split.  blockIdx -> (split, m-tile, n-tile) runs n fastest after a bijective
// XCD remap, so the n-tiles sharing an A slab run on one XCD (one L2).
struct GemmBfArgs {
  GemmArgs g;            // shapes, C / C2, epilogue, split-K slabs (A/B fields unused)
  const __bf16* A;
  const __bf16* B;
  int mt, nt;            // tiles along M, N
  int gm;                // tile order: -1 XCD column partition, 0 n fastest (bf_tile)
  int vec;               // 4-element result stores legal (C / C2 / slab rows and nc multiples of 4, aligned)
  int obf;               // C / C2 are bf16 (RNE of the fp32 accumulation): the reference's autocast output dtype
};

__device__ __forceinline__ __bf16* cptr_bf(const GemmArgs& g, int m, int n) {
  return (g.C2 && n >= g.nc) ? (__bf16*)g.C2 + (long)m * g.ldc2 + (n - g.nc) : (__bf16*)g.C + (long)m * g.ldc + n;
}

__device__ __forceinline__ void glds16(const void* src, void* lds) {
  __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)src,
                                   (void __attribute__((address_space(3)))*)lds, 16, 0, 0);
}

typedef short s16x4_g __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4_g __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2_g __attribute__((ext_vector_type(2)));
__device__ __forceinline__ bf16x4 lds_tr4_g(const __bf16* p) {
  return __builtin_bit_cast(bf16x4, __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                                        (__attribute__((address_space(3))) s16x4_g*)p));
}

// stage rows [r0, r0 + 128) x k [k0, k0 + 64) of a k-contiguous operand; wave w issues 4 x 1 KB
__device__ __forceinline__ void stage_kc(const __bf16* __restrict__ src, long ld, int r0, int nvalid, int k0,
                                         __bf16* tile, int w, int lane) {
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int q = w * 4 + t, r = q * 8 + (lane >> 3);
    const int kc = (lane & 7) ^ ((r >> 1) & 7);
    const int gr = min(r0 + r, nvalid - 1);
    glds16(src + (long)gr * ld + k0 + 8 * kc, tile + q * 512);
  }
}

// stage k [k0, k0 + 64) x cols [c0, c0 + 128) of a k-major operand; wave w issues 4 x 1 KB (instruction q:
// k-block q / 2, col-blocks 4 (q % 2) .. +3; lane: block + lane / 16, row (lane % 16) / 2, half lane % 2)
__device__ __forceinline__ void stage_km(const __bf16* __restrict__ src, long ld, int c0, int nvalid, int k0,
                                         __bf16* tile, int w, int lane) {
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int q = w * 4 + t, kb = q >> 1, cb = 4 * (q & 1) + (lane >> 4);
    const int row = ((lane & 15) >> 1) ^ (4 * (kb & 1));
    const int col = min(c0 + 16 * cb + 8 * (lane & 1), nvalid - 8);
    glds16(src + (long)(k0 + 8 * kb + row) * ld + col, tile + q * 512);
  }
}

// fragment (16 rows/cols x 32 k) of k-slice ks (0/1) at tile row/col base rb: lane (g, c) gets row rb + c,
// k 32 ks + 8 g .. + 7
__device__ __forceinline__ bf16x8 frag_kc(const __bf16* tile, int rb, int ks, int lane) {
  const int r = rb + (lane & 15), kc = 4 * ks + (lane >> 4);
  return *(const bf16x8*)(tile + r * 64 + 8 * (kc ^ ((r >> 1) & 7)));
}
__device__ __forceinline__ bf16x8 frag_km(const __bf16* tile, int cb16, int ks, int lane) {
  const int kb = 4 * ks + (lane >> 4), l = lane & 15;
  const __bf16* blk = tile + (kb * 8 + cb16) * 128;
  const int sw = 4 * (kb & 1);
  const __bf16* p0 = blk + ((l >> 2) ^ sw) * 16 + 4 * (l & 3);          // k rows 0..3
  const __bf16* p1 = blk + (((l >> 2) + 4) ^ sw) * 16 + 4 * (l & 3);    // k rows 4..7
  const bf16x4 lo = lds_tr4_g(p0), hi = lds_tr4_g(p1);
  return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

// tile t of a workgroup's sequence -> (split z, m-tile, n-tile); false past the end.
//   gm < 0, XCD column partition (nt >= 8): workgroups are dealt round-robin to the 8 XCDs, so XCD x runs ids
//     x, x + 8, ...; it takes the n-tiles [nt x / 8, nt (x + 1) / 8) -- a B column group that stays in its L2 --
//     for every m-tile, m slow / n fast, so the workgroups running at once also share a few A slabs.  (n fastest
//     over all tiles made every XCD stream all of B once per m-tile from the MALL: 241 MB of L2 fills for the
//     QNN MLP input grad's 12 MB of operands.)
//   gm = 0: n fastest, then m, then z, after a bijective XCD remap, strided by the grid.
__device__ __forceinline__ bool bf_tile(const GemmBfArgs& p, int nsplit, int t, int& z, int& mt_i, int& nt_i) {
  if (p.gm < 0) {
    const int x = blockIdx.x & 7, gx = gridDim.x >> 3;
    const int nlo = p.nt * x / 8, nw = p.nt * (x + 1) / 8 - nlo;
    const int idx = (blockIdx.x >> 3) + t * gx, per = p.mt * nw;
    if (nw == 0 || idx >= per * nsplit) return false;
    z = idx / per;
    const int r = idx - z * per;
    mt_i = r / nw;
    nt_i = nlo + r % nw;
    return true;
  }
  // bijective XCD remap: consecutive ids on one XCD (dispatch is round-robin over the 8 XCDs), so the tiles of
  // one split's k range share that XCD's L2
  const int nwg = gridDim.x, orig = blockIdx.x, xcd = orig % 8, qq = nwg / 8, rr = nwg % 8;
  const int id = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + orig / 8;
  const int idx = id + t * nwg, per = p.mt * p.nt;
  if (idx >= per * nsplit) return false;
  z = idx / per;
  const int r = idx - z * per;
  mt_i = r / p.nt;
  nt_i = r % p.nt;
  return true;
}

// Persistent: a workgroup walks its tiles (bf_tile), and the first k-slice of its NEXT tile is staged while the
// current tile's epilogue stores go out, so a tile's store drain overlaps the next tile's first DMA (one
// workgroup per tile left the next workgroup on that CU waiting for both in turn: the 124 MB fp32 output of
// the QNN MLP's input grad took more time to store than to compute).
template <bool TA, bool TB>
__global__ __launch_bounds__(256) void gemm_bf_kernel(GemmBfArgs p) {
  __shared__ __attribute__((aligned(16))) __bf16 smem[2 * 2 * 128 * 64];     // [stage][A | B][128 x 64]
  const GemmArgs& g = p.g;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int nsplit = (g.K + g.klen - 1) / g.klen;
  const int wm = (w >> 1) * 64, wn = (w & 1) * 64;
  const long lda = g.lda, ldb = g.ldb;

  auto stage = [&](int buf, int m0, int n0, int k0) {
    __bf16* ta = smem + buf * 2 * 8192;
    __bf16* tb = ta + 8192;
    if (TA) stage_km(p.A, lda, m0, g.M, k0, ta, w, lane);
    else stage_kc(p.A, lda, m0, g.M, k0, ta, w, lane);
    if (TB) stage_kc(p.B, ldb, n0, g.N, k0, tb, w, lane);
    else stage_km(p.B, ldb, n0, g.N, k0, tb, w, lane);
  };

  int z, mt_i, nt_i;
  if (!bf_tile(p, nsplit, 0, z, mt_i, nt_i)) return;
  int bi = 0;                                // LDS buffer holding the current k-slice
  stage(0, mt_i * 128, nt_i * 128, z * g.klen);
  __builtin_amdgcn_s_waitcnt(0);             // vmcnt(0) lgkmcnt(0)...: the DMA has landed
  __syncthreads();
  for (int t = 0;; ++t) {
    const int m0 = mt_i * 128, n0 = nt_i * 128;
    const int kz0 = z * g.klen, kz1 = min(g.K, kz0 + g.klen);
    const int nkt = kz1 > kz0 ? (kz1 - kz0) / 64 : 0;
    int zn, mn, nn;
    const bool more = bf_tile(p, nsplit, t + 1, zn, mn, nn);
    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int kt = 0; kt < nkt; ++kt) {
      const int cur = bi;
      if (kt + 1 < nkt) stage(cur ^ 1, m0, n0, kz0 + (kt + 1) * 64);
      else if (more) stage(cur ^ 1, mn * 128, nn * 128, zn * g.klen);   // the next tile's first slice
      const __bf16* ta = smem + cur * 2 * 8192;
      const __bf16* tb = ta + 8192;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        bf16x8 af[4], bfr[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) af[i] = TA ? frag_km(ta, (wm >> 4) + i, ks, lane) : frag_kc(ta, wm + 16 * i, ks, lane);
#pragma unroll
        for (int j = 0; j < 4; ++j) bfr[j] = TB ? frag_kc(tb, wn + 16 * j, ks, lane) : frag_km(tb, (wn >> 4) + j, ks, lane);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
      }
      bi ^= 1;
      if (kt + 1 < nkt) {
        __builtin_amdgcn_s_waitcnt(0);       // the next slice's DMA (and this slice's reads) complete
        __syncthreads();
      }
    }

    // the products ran as C^T tiles (B fragment first): lane (g, c) holds row m = .. + c, columns n .. n + 3 of
    // each 16 x 16 block in its four registers -- one 16-byte store per block instead of four 4-byte ones
    const ctr_gemm_epi_t& e = g.epi;
    const int lrow = wm + (lane & 15), lcol = wn + (lane >> 4) * 4;
    if (g.ws) {   // split-K partial: raw slab, the reduce kernel applies the epilogue
      float* slab = g.ws + (long)z * g.M * g.N;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = m0 + lrow + i * 16;
        if (m >= g.M) continue;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int n = n0 + lcol + j * 16;
          float* d = slab + (long)m * g.N + n;
          if (p.vec && n + 3 < g.N) {
            *(f32x4*)d = acc[i][j];
          } else {
#pragma unroll
            for (int r = 0; r < 4; ++r)
              if (n + r < g.N) d[r] = acc[i][j][r];
          }
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = m0 + lrow + i * 16;
        if (m >= g.M) continue;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int n = n0 + lcol + j * 16;
          if (n >= g.N) continue;
          f32x4 v = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int r = 0; r < 4; ++r)     // columns past N: no epilogue (it stores pre-activations, reads aux / add)
            if (n + r < g.N) v[r] = epi_elem(e, acc[i][j][r], m, n + r, g.N, g.ldc);
          // a 4-column group never straddles nc (nc % 4 == 0 when vec)
          if (p.obf) {
            if (p.vec && n + 3 < g.N) {
              *(bf16x4*)cptr_bf(g, m, n) = __builtin_convertvector(v, bf16x4);
            } else {
#pragma unroll
              for (int r = 0; r < 4; ++r)
                if (n + r < g.N) *cptr_bf(g, m, n + r) = (__bf16)v[r];
            }
          } else if (p.vec && n + 3 < g.N) {
            *(f32x4*)cptr(g, m, n) = v;
          } else {
#pragma unroll
            for (int r = 0; r < 4; ++r)
              if (n + r < g.N) *cptr(g, m, n + r) = v[r];
          }
        }
      }
    }
    if (!more) break;
    __builtin_amdgcn_s_waitcnt(0);           // the next tile's first slice (and this tile's stores)
    __syncthreads();
    z = zn;
    mt_i = mn;
    nt_i = nn;
  }
}

// ------------------------------------------------------------------------------------------------
// bf16-operand GEMM, ring form (round 5): ONE 512-thread workgroup per CU walks its tiles' 64-deep k-steps as
// one flat sequence through a ring of NS LDS stages filled by global_load_lds, NS - 1 steps ahead --
// across tile boundaries, so a tile's first steps are in flight while the previous tile computes and stores.
// Each step: a COUNTED s_waitcnt vmcnt (this wave's pieces of the step have landed; the younger steps' DMA and
// the recent epilogue stores stay in flight), a raw s_barrier (every wave's pieces landed, and every wave is
// done reading the stage the next DMA overwrites), the DMA of step + NS - 1, then the MFMAs.  The
// two-stage kernel above waited for vmcnt(0) -- every DMA and store in flight -- at each of its barriers.
// Tile 256 x 128 (8 waves as 4 (M) x 2 (N) of 64 x 64, C^T accumulators as above): operand re-reads from L2 are
// 3/4 of the 128 x 128 tile's per output element.  The epilogue's stores are raw buffer stores, exactly 16 per
// lane per tile (32 with a C2 segment: one to each, the other dropped) -- out-of-range rows / columns dropped
// by the resource bound instead of skipped -- so the counted waits stay exact; epilogues with operands of their
// own (bias, activation, ...) take a vmcnt(0) at the next two steps.
constexpr int G8_BN = 128;
template <int BM, int NS>
struct G8 {
  static constexpr int A = BM * 64, B = G8_BN * 64, STAGE = A + B;   // bf16 elements
  static constexpr int LDS = NS * STAGE * 2;
  static constexpr int PL = (BM + G8_BN) * 128 / 1024 / 8;         // DMA pieces per lane per step
  static constexpr int WR = BM / 64, WC = 8 / WR;                   // wave grid (each 64 rows)
  static constexpr int WN = G8_BN / WC, NJ = WN / 16;               // wave columns, 16-col blocks
  static_assert(LDS <= 160 * 1024, "G8: LDS");
};
int g_gemm_bf_variant = 0;     // test / bench hook (ctr_gemm_bf16_set_variant): 0 auto, 1 two-stage, 2 ring 256, 3 ring 128

// rows [r0, r0 + NR) x k [k0, k0 + 64) of a k-contiguous operand into a swizzled [NR][64] image (as stage_kc)
template <int NR>
__device__ __forceinline__ void stage_kc8(const __bf16* __restrict__ src, long ld, int r0, int nvalid, int k0,
                                          __bf16* tile, int w, int lane) {
  constexpr int PW = NR / 64;
#pragma unroll
  for (int t = 0; t < PW; ++t) {
    const int q = w * PW + t, r = q * 8 + (lane >> 3);
    const int kc = (lane & 7) ^ ((r >> 1) & 7);
    const int gr = min(r0 + r, nvalid - 1);
    glds16(src + (long)gr * ld + k0 + 8 * kc, tile + q * 512);
  }
}
// k [k0, k0 + 64) x cols [c0, c0 + NC) of a k-major operand into [8 k-blocks][NC / 16 col-blocks][8][16] (as stage_km)
template <int NC>
__device__ __forceinline__ void stage_km8(const __bf16* __restrict__ src, long ld, int c0, int nvalid, int k0,
                                          __bf16* tile, int w, int lane) {
  constexpr int PW = NC / 64, QB = NC / 64;     // pieces per wave; pieces per k-block (4 col-blocks each)
#pragma unroll
  for (int t = 0; t < PW; ++t) {
    const int q = w * PW + t, kb = q / QB, cb = 4 * (q % QB) + (lane >> 4);
    const int row = ((lane & 15) >> 1) ^ (4 * (kb & 1));
    const int col = min(c0 + 16 * cb + 8 * (lane & 1), nvalid - 8);
    glds16(src + (long)(k0 + 8 * kb + row) * ld + col, tile + q * 512);
  }
}
template <int NCB>
__device__ __forceinline__ bf16x8 frag_km8(const __bf16* tile, int cb16, int ks, int lane) {
  const int kb = 4 * ks + (lane >> 4), l = lane & 15;
  const __bf16* blk = tile + (kb * NCB + cb16) * 128;
  const int sw = 4 * (kb & 1);
  const bf16x4 lo = lds_tr4_g(blk + ((l >> 2) ^ sw) * 16 + 4 * (l & 3));
  const bf16x4 hi = lds_tr4_g(blk + (((l >> 2) + 4) ^ sw) * 16 + 4 * (l & 3));
  return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

// s_waitcnt vmcnt(n) (n <= 63), lgkmcnt / expcnt not waited for
template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N <= 63, "vmcnt");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}
__device__ __forceinline__ void wait_vm_n(int n) {
  switch (n) {
    case 0: wait_vm<0>(); break;
    case 1: wait_vm<1>(); break;
    case 2: wait_vm<2>(); break;
    case 3: wait_vm<3>(); break;
    case 4: wait_vm<4>(); break;
    case 5: wait_vm<5>(); break;
    case 6: wait_vm<6>(); break;
    case 7: wait_vm<7>(); break;
    case 8: wait_vm<8>(); break;
    case 9: wait_vm<9>(); break;
    case 10: wait_vm<10>(); break;
    case 11: wait_vm<11>(); break;
    case 12: wait_vm<12>(); break;
    case 13: wait_vm<13>(); break;
    case 14: wait_vm<14>(); break;
    case 15: wait_vm<15>(); break;
    case 16: wait_vm<16>(); break;
    case 17: wait_vm<17>(); break;
    case 18: wait_vm<18>(); break;
    case 19: wait_vm<19>(); break;
    case 20: wait_vm<20>(); break;
    case 21: wait_vm<21>(); break;
    case 22: wait_vm<22>(); break;
    case 23: wait_vm<23>(); break;
    case 24: wait_vm<24>(); break;
    case 25: wait_vm<25>(); break;
    case 26: wait_vm<26>(); break;
    case 27: wait_vm<27>(); break;
    case 28: wait_vm<28>(); break;
    case 29: wait_vm<29>(); break;
    case 30: wait_vm<30>(); break;
    case 31: wait_vm<31>(); break;
    case 32: wait_vm<32>(); break;
    case 33: wait_vm<33>(); break;
    case 34: wait_vm<34>(); break;
    case 35: wait_vm<35>(); break;
    case 36: wait_vm<36>(); break;
    case 37: wait_vm<37>(); break;
    case 38: wait_vm<38>(); break;
    case 39: wait_vm<39>(); break;
    case 40: wait_vm<40>(); break;
    case 41: wait_vm<41>(); break;
    case 42: wait_vm<42>(); break;
    case 43: wait_vm<43>(); break;
    case 44: wait_vm<44>(); break;
    case 45: wait_vm<45>(); break;
    case 46: wait_vm<46>(); break;
    case 47: wait_vm<47>(); break;
    case 48: wait_vm<48>(); break;
    case 49: wait_vm<49>(); break;
    case 50: wait_vm<50>(); break;
    case 51: wait_vm<51>(); break;
    case 52: wait_vm<52>(); break;
    case 53: wait_vm<53>(); break;
    case 54: wait_vm<54>(); break;
    case 55: wait_vm<55>(); break;
    case 56: wait_vm<56>(); break;
    case 57: wait_vm<57>(); break;
    case 58: wait_vm<58>(); break;
    case 59: wait_vm<59>(); break;
    case 60: wait_vm<60>(); break;
    case 61: wait_vm<61>(); break;
    case 62: wait_vm<62>(); break;
    case 63: wait_vm<63>(); break;
    default: wait_vm<0>(); break;     // never under-waits
  }
}

template <bool TA, bool TB, int BM, int NS>
__global__ __launch_bounds__(512) void gemm_bf8_kernel(GemmBfArgs p) {
  using C8 = G8<BM, NS>;
  constexpr int NJ = C8::NJ;
  extern __shared__ __attribute__((aligned(16))) __bf16 sm8[];
  const GemmArgs& g = p.g;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int nsplit = (g.K + g.klen - 1) / g.klen;
  const int wm = (w / C8::WC) * 64, wn = (w % C8::WC) * C8::WN;
  auto nk_of = [&](int z) {
    const int k0 = z * g.klen, k1 = min(g.K, k0 + g.klen);
    return k1 > k0 ? (k1 - k0) / 64 : 0;
  };
  // producer cursor: the next k-step to stage
  int pt = 0, pk = 0, pz = 0, pm = 0, pn = 0;
  bool pv = bf_tile(p, nsplit, 0, pz, pm, pn);
  int pnk = pv ? nk_of(pz) : 0;
  int nprod = 0;       // k-steps staged so far
  auto produce = [&](int st) {
    if (!pv) return;
    ++nprod;
    __bf16* ta = sm8 + st * C8::STAGE;
    __bf16* tb = ta + C8::A;
    const int k0 = pz * g.klen + pk * 64;
    if (TA) stage_km8<BM>(p.A, g.lda, pm * BM, g.M, k0, ta, w, lane);
    else stage_kc8<BM>(p.A, g.lda, pm * BM, g.M, k0, ta, w, lane);
    if (TB) stage_kc8<G8_BN>(p.B, g.ldb, pn * G8_BN, g.N, k0, tb, w, lane);
    else stage_km8<G8_BN>(p.B, g.ldb, pn * G8_BN, g.N, k0, tb, w, lane);
    if (++pk == pnk) {
      pk = 0;
      ++pt;
      pv = bf_tile(p, nsplit, pt, pz, pm, pn);
      pnk = pv ? nk_of(pz) : 0;
    }
  };
  int ct = 0, cz, cm, cn;
  if (!bf_tile(p, nsplit, 0, cz, cm, cn)) return;
  int cnk = nk_of(cz), ck = 0;
#pragma unroll
  for (int st = 0; st < NS - 1; ++st) produce(st);

  // epilogue store plan: fast = raw buffer stores only (exactly SPT per lane per tile)
  const ctr_gemm_epi_t& e = g.epi;
  const bool plain = !e.dact && !e.bias && !e.add && !e.pre && !e.act && !e.drop_thresh;
  const bool fast = p.vec && (g.ws || plain);
  const bool two = !g.ws && g.C2 != nullptr;
  const int SPT = (two ? 2 : 1) * 4 * NJ;
  const int esz = g.ws ? 4 : (p.obf ? 2 : 4);
  const __amdgpu_buffer_rsrc_t rc = g.ws ? buf_rsrc(g.ws, 0x7FFFFFFF)
                                         : buf_rsrc(g.C, (uint32_t)(((long)(g.M - 1) * g.ldc + min(g.N, g.nc)) * esz));
  const __amdgpu_buffer_rsrc_t rc2 = two ? buf_rsrc(g.C2, (uint32_t)(((long)(g.M - 1) * g.ldc2 + (g.N - g.nc)) * esz))
                                         : rc;
  int epi_iter[2] = {-99, -99};     // iterations of the last two epilogues (their stores are younger than some DMA)
  bool epi_slow[2] = {false, false};

  f32x4 acc[4][NJ];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int sidx = 0;; ++sidx) {
    // this step's DMA was issued NS - 1 iterations ago (or in the prologue); younger than it: the DMA of the
    // steps issued after it, and the stores of every epilogue since (iterations sidx - NS + 1 .. sidx - 1)
    int younger = C8::PL * (nprod - sidx - 1);
    {
      bool slow = false;
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int age = sidx - epi_iter[q];
        if (age >= 1 && age <= NS - 1) {
          younger += SPT;
          slow |= epi_slow[q];
        }
      }
      if (slow) younger = 0;
    }
    wait_vm_n(min(younger, 63));
    // raw barrier, no fence (a workgroup fence would drain the DMA in flight: vmcnt(0)); the empty asm keeps the
    // compiler from moving LDS reads or the next DMA across it
    __asm__ volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __asm__ volatile("" ::: "memory");
    produce((sidx + NS - 1) % NS);
    const __bf16* ta = sm8 + (sidx % NS) * C8::STAGE;
    const __bf16* tb = ta + C8::A;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 af[4], bfr[NJ];
#pragma unroll
      for (int i = 0; i < 4; ++i)
        af[i] = TA ? frag_km8<BM / 16>(ta, (wm >> 4) + i, ks, lane) : frag_kc(ta, wm + 16 * i, ks, lane);
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        bfr[j] = TB ? frag_kc(tb, wn + 16 * j, ks, lane) : frag_km8<G8_BN / 16>(tb, (wn >> 4) + j, ks, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
    }
    if (++ck < cnk) continue;
    // ---- epilogue of tile (cz, cm, cn)
    const int m0 = cm * BM, n0 = cn * G8_BN;
    const int lrow = wm + (lane & 15), lcol = wn + (lane >> 4) * 4;
    if (fast) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = m0 + lrow + i * 16;
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const int n = n0 + lcol + j * 16;
          const bool ok = m < g.M && n < g.N;
          if (g.ws) {
            const long off = (((long)cz * g.M + m) * g.N + n) * 4;
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_g, acc[i][j]), rc,
                                                   ok ? (uint32_t)off : BUF_OOB, 0, 0);
          } else {
            const bool in2 = two && n >= g.nc;
            const long o1 = ((long)m * g.ldc + n) * esz, o2 = ((long)m * g.ldc2 + (n - g.nc)) * esz;
            if (p.obf) {
              const bf16x4 v = __builtin_convertvector(acc[i][j], bf16x4);
              __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2_g, v), rc,
                                                    ok && !in2 ? (uint32_t)o1 : BUF_OOB, 0, 0);
              if (two)
                __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2_g, v), rc2,
                                                      ok && in2 ? (uint32_t)o2 : BUF_OOB, 0, 0);
            } else {
              __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_g, acc[i][j]), rc,
                                                     ok && !in2 ? (uint32_t)o1 : BUF_OOB, 0, 0);
              if (two)
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_g, acc[i][j]), rc2,
                                                       ok && in2 ? (uint32_t)o2 : BUF_OOB, 0, 0);
            }
          }
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = m0 + lrow + i * 16;
        if (m >= g.M) continue;
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const int n = n0 + lcol + j * 16;
          if (n >= g.N) continue;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            if (n + r >= g.N) continue;
            if (g.ws) {
              g.ws[((long)cz * g.M + m) * g.N + n + r] = acc[i][j][r];
            } else {
              const float v = epi_elem(e, acc[i][j][r], m, n + r, g.N, g.ldc);
              if (p.obf) *cptr_bf(g, m, n + r) = (__bf16)v;
              else *cptr(g, m, n + r) = v;
            }
          }
        }
      }
    }
    epi_iter[1] = epi_iter[0];
    epi_slow[1] = epi_slow[0];
    epi_iter[0] = sidx;
    epi_slow[0] = !fast;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    ck = 0;
    ++ct;
    if (!bf_tile(p, nsplit, ct, cz, cm, cn)) break;
    cnk = nk_of(cz);
  }
  wait_vm<0>();
}

// fp32 (rows, cols) with row stride lds -> bf16 with row stride ldd (RNE); 4 elements per thread
__global__ void to_bf16_kernel(const float* __restrict__ src, long lds, int rows, int cols, __bf16* __restrict__ dst,
                               long ldd) {
  const int cq = (cols + 3) / 4;
  const long n = (long)rows * cq;
  for (long q = blockIdx.x * 256L + threadIdx.x; q < n; q += (long)gridDim.x * 256) {
    const int r = (int)(q / cq), c = (int)(q % cq) * 4;
    const float* s = src + r * lds + c;
    __bf16* d = dst + r * ldd + c;
    if (c + 3 < cols && ((((uintptr_t)s) & 15) == 0) && ((((uintptr_t)d) & 7) == 0)) {
      *(bf16x4*)d = __builtin_convertvector(*(const f32x4*)s, bf16x4);
    } else {
      for (int j = 0; j < 4 && c + j < cols; ++j) d[j] = (__bf16)s[j];
    }
  }
}

}  // namespace ctr

using namespace ctr;

extern "C" size_t ctr_gemm_ws_size(int M, int N, int splits) {
  return splits > 1 ? (size_t)splits * M * N * sizeof(float) : 0;
}

static int gemm_core(int M, int N, int K, const float* A, int lda, int ta, const float* B, int ldb, int tb,
                     float* C, int ldc, const ctr_gemm_epi_t* epi, int splits, float* ws, const ctr_gemm_seg_t* seg,
                     void* stream, int bf = 0) {
  CTR_REQUIRE(M >= 0 && N >= 0 && K >= 0, "negative dims");
  if (M == 0 || N == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  GemmArgs g;
  g.M = M; g.N = N; g.K = K; g.A = A; g.lda = lda; g.B = B; g.ldb = ldb; g.C = C; g.ldc = ldc;
  ctr_gemm_epi_t zero = {};
  g.epi = epi ? *epi : zero;
  CTR_REQUIRE(!(g.epi.dact && !g.epi.aux), "dact needs aux");
  CTR_REQUIRE(!(g.epi.norm_w && (N > 64 || !g.epi.resid)), "fused RMSNorm needs N <= 64 and resid");
  if (splits < 1) splits = 1;
  CTR_REQUIRE(!(splits > 1 && (g.epi.norm_w || !ws)), "split-K needs ws and no fused norm");
  g.vecA = ((lda & 3) == 0) && ((((uintptr_t)A) & 15) == 0);
  g.vecB = ((ldb & 3) == 0) && ((((uintptr_t)B) & 15) == 0);
  g.A2 = nullptr; g.lda2 = 0; g.ka = K;
  g.B2 = nullptr; g.ldb2 = 0; g.nb = N;
  g.C2 = nullptr; g.ldc2 = 0; g.nc = N;
  if (seg) {
    CTR_REQUIRE(!(seg->A2 && ta) && !(seg->B2 && tb), "gemm segments: A2 needs ta = 0, B2 needs tb = 0");
    CTR_REQUIRE(!seg->A2 || (seg->ka >= 0 && seg->ka <= K), "gemm segments: ka out of range");
    CTR_REQUIRE(!seg->B2 || (seg->nb >= 0 && seg->nb <= N), "gemm segments: nb out of range");
    CTR_REQUIRE(!seg->C2 || (seg->nc >= 0 && seg->nc <= N && N > 96 && !g.epi.norm_w && !g.epi.aux && !g.epi.pre &&
                             !g.epi.add),
                "gemm segments: C2 needs N > 96 and no row-indexed epilogue operand");
    if (seg->A2) {
      g.A2 = seg->A2; g.lda2 = seg->lda2; g.ka = seg->ka;
      g.vecA = g.vecA && ((seg->lda2 & 3) == 0) && ((((uintptr_t)seg->A2) & 15) == 0) && ((seg->ka & 3) == 0);
    }
    if (seg->B2) {
      g.B2 = seg->B2; g.ldb2 = seg->ldb2; g.nb = seg->nb;
      g.vecB = g.vecB && ((seg->ldb2 & 3) == 0) && ((((uintptr_t)seg->B2) & 15) == 0) && ((seg->nb & 3) == 0);
    }
    if (seg->C2) { g.C2 = seg->C2; g.ldc2 = seg->ldc2; g.nc = seg->nc; }
  }
  const int BK = bf ? bf : 16;
  int klen = K;
  if (splits > 1) {
    klen = ((K + splits - 1) / splits + BK - 1) / BK * BK;
    splits = (K + klen - 1) / klen;
  }
  g.klen = klen > 0 ? klen : 1;
  g.ws = ws;
  if (K <= 4 && !g.epi.norm_w && splits == 1 && !seg && !bf) {
    const long MN = (long)M * N;
    gemm_smallk_kernel<<<(int)std::min<long>((MN + 255) / 256, 8192), 256, 0, s>>>(g, ta, tb);
    return check_launch("ctr_gemm");
  }
  if (g.epi.norm_w) {
    if (N <= 32) launch_tile<128, 32>(g, ta, tb, 1, s, bf);
    else launch_tile<128, 64>(g, ta, tb, 1, s, bf);
  } else if (N <= 32) {
    launch_tile<128, 32>(g, ta, tb, splits, s, bf);
  } else if (N <= 64) {
    launch_tile<128, 64>(g, ta, tb, splits, s, bf);
  } else if (N <= 96) {
    launch_tile<128, 96>(g, ta, tb, splits, s, bf);
  } else if (M <= 64) {
    launch_tile<64, 128>(g, ta, tb, splits, s, bf);
  } else if ((long)((M + 127) / 128) * ((N + 127) / 128) * splits < 512) {
    launch_tile<64, 64>(g, ta, tb, splits, s, bf);     // too few 128x128 tiles to fill the chip
  } else {
    launch_tile<128, 128>(g, ta, tb, splits, s, bf);
  }
  if (splits > 1) {
    const long MN = (long)M * N;
    int blocks = (int)std::min<long>((MN + 255) / 256, 4096);
    splitk_reduce_kernel<<<blocks, 256, 0, s>>>(g, splits);
  }
  return check_launch("ctr_gemm");
}

extern "C" int ctr_gemm(int M, int N, int K, const float* A, int lda, int ta, const float* B, int ldb, int tb,
                        float* C, int ldc, const ctr_gemm_epi_t* epi, int splits, float* ws, void* stream) {
  return gemm_core(M, N, K, A, lda, ta, B, ldb, tb, C, ldc, epi, splits, ws, nullptr, stream);
}

extern "C" int ctr_gemm_seg(int M, int N, int K, const float* A, int lda, int ta, const float* B, int ldb, int tb,
                            float* C, int ldc, const ctr_gemm_epi_t* epi, int splits, float* ws,
                            const ctr_gemm_seg_t* seg, void* stream) {
  return gemm_core(M, N, K, A, lda, ta, B, ldb, tb, C, ldc, epi, splits, ws, seg, stream);
}

extern "C" int ctr_gemm_ex(int M, int N, int K, const float* A, int lda, int ta, const float* B, int ldb, int tb,
                           float* C, int ldc, const ctr_gemm_epi_t* epi, int splits, float* ws, const ctr_gemm_seg_t* seg,
                           int flags, void* stream) {
  CTR_REQUIRE((flags & ~(CTR_GEMM_BF16 | 2)) == 0, "ctr_gemm_ex: unknown flags");
  const int bf = (flags & CTR_GEMM_BF16) ? ((flags & 2) ? 64 : 32) : 0;
  return gemm_core(M, N, K, A, lda, ta, B, ldb, tb, C, ldc, epi, splits, ws, seg, stream, bf);
}

extern "C" int ctr_to_bf16(const float* src, long lds, int rows, int cols, void* dst, long ldd, void* stream) {
  CTR_REQUIRE(rows >= 0 && cols >= 0 && lds >= cols && ldd >= cols, "ctr_to_bf16: bad shape");
  if (rows == 0 || cols == 0) return 0;
  const long n = (long)rows * ((cols + 3) / 4);
  to_bf16_kernel<<<(int)std::min<long>((n + 255) / 256, 8192), 256, 0, (hipStream_t)stream>>>(src, lds, rows, cols,
                                                                                          (__bf16*)dst, ldd);
  return check_launch("ctr_to_bf16");
}

template <bool TA, bool TB, int BM, int NS>
static void launch_g8_t(const GemmBfArgs& p, int grid, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)gemm_bf8_kernel<TA, TB, BM, NS>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              G8<BM, NS>::LDS);
    attr = true;
  }
  gemm_bf8_kernel<TA, TB, BM, NS><<<grid, 512, G8<BM, NS>::LDS, s>>>(p);
}
template <int BM, int NS>
static void launch_g8_b(const GemmBfArgs& p, int ta, int tb, int grid, hipStream_t s) {
  if (!ta && tb) launch_g8_t<false, true, BM, NS>(p, grid, s);
  else if (!ta && !tb) launch_g8_t<false, false, BM, NS>(p, grid, s);
  else if (ta && !tb) launch_g8_t<true, false, BM, NS>(p, grid, s);
  else launch_g8_t<true, true, BM, NS>(p, grid, s);
}
static void launch_g8(const GemmBfArgs& p, int ta, int tb, int BM, int grid, hipStream_t s) {
  if (BM == 256) launch_g8_b<256, 3>(p, ta, tb, grid, s);
  else launch_g8_b<128, 4>(p, ta, tb, grid, s);
}

extern "C" void ctr_gemm_bf16_set_variant(int v) { g_gemm_bf_variant = v; }

extern "C" int ctr_gemm_bf16_ok(int M, int N, int K, int lda, int ta, int ldb, int tb, int splits) {
  if (M < 8 || N < 8 || K <= 0 || K % 64) return 0;
  if (splits < 1) splits = 1;
  const int klen = ((K + splits - 1) / splits + 63) / 64 * 64;
  (void)klen;
  // 16-byte aligned rows (glds); k-major operands need 8-column groups inside the row
  if ((lda % 8) || (ldb % 8)) return 0;
  if (ta && M % 8) return 0;
  if (!tb && N % 8) return 0;
  return 1;
}

extern "C" int ctr_gemm_bf16(int M, int N, int K, const void* A, int lda, int ta, const void* B, int ldb, int tb,
                             float* C, int ldc, const ctr_gemm_epi_t* epi, int splits, float* ws,
                             const ctr_gemm_seg_t* seg, void* stream) {
  return ctr_gemm_bf16_ex(M, N, K, A, lda, ta, B, ldb, tb, C, ldc, epi, splits, ws, seg, 0, stream);
}

extern "C" int ctr_gemm_bf16_ex(int M, int N, int K, const void* A, int lda, int ta, const void* B, int ldb, int tb,
                                void* C, int ldc, const ctr_gemm_epi_t* epi, int splits, float* ws,
                                const ctr_gemm_seg_t* seg, int flags, void* stream) {
  CTR_REQUIRE((flags & ~CTR_GEMM_OUT_BF16) == 0, "ctr_gemm_bf16_ex: unknown flags");
  const int obf = (flags & CTR_GEMM_OUT_BF16) ? 1 : 0;
  CTR_REQUIRE(ctr_gemm_bf16_ok(M, N, K, lda, ta, ldb, tb, splits), "ctr_gemm_bf16: unsupported shape / layout");
  CTR_REQUIRE(((uintptr_t)A & 15) == 0 && ((uintptr_t)B & 15) == 0, "ctr_gemm_bf16: operands need 16-byte alignment");
  CTR_REQUIRE(!seg || (!seg->A2 && !seg->B2), "ctr_gemm_bf16: only the C2 result segment is supported");
  GemmBfArgs p = {};
  GemmArgs& g = p.g;
  g.M = M; g.N = N; g.K = K; g.lda = lda; g.ldb = ldb; g.C = (float*)C; g.ldc = ldc;
  ctr_gemm_epi_t zero = {};
  g.epi = epi ? *epi : zero;
  CTR_REQUIRE(!(g.epi.dact && !g.epi.aux), "dact needs aux");
  CTR_REQUIRE(!g.epi.norm_w, "ctr_gemm_bf16: no fused RMSNorm epilogue");
  CTR_REQUIRE(!obf || !g.epi.pre, "ctr_gemm_bf16_ex: bf16 output has no pre-activation store");
  g.C2 = nullptr; g.ldc2 = 0; g.nc = N;
  if (seg && seg->C2) {
    CTR_REQUIRE(seg->nc >= 0 && seg->nc <= N && !g.epi.aux && !g.epi.pre && !g.epi.add,
                "ctr_gemm_bf16: C2 needs no row-indexed epilogue operand");
    g.C2 = seg->C2; g.ldc2 = seg->ldc2; g.nc = seg->nc;
  }
  if (splits < 1) splits = 1;
  int klen = ((K + splits - 1) / splits + 63) / 64 * 64;
  splits = (K + klen - 1) / klen;
  g.klen = klen;
  CTR_REQUIRE(splits == 1 || ws, "ctr_gemm_bf16: split-K needs ws");
  CTR_REQUIRE(splits == 1 || !obf, "ctr_gemm_bf16_ex: bf16 output needs splits = 1");
  g.ws = splits > 1 ? ws : nullptr;
  p.A = (const __bf16*)A;
  p.B = (const __bf16*)B;
  p.obf = obf;
  const uintptr_t al = obf ? 7 : 15;       // bf16x4 / f32x4 stores
  p.vec = (N % 4 == 0) && (ldc % 4 == 0) && (((uintptr_t)C & al) == 0) && (!ws || ((uintptr_t)ws & 15) == 0) &&
          (!g.C2 || ((g.ldc2 % 4 == 0) && (g.nc % 4 == 0) && (((uintptr_t)g.C2 & al) == 0)));
  hipStream_t s = (hipStream_t)stream;
  // the ring kernel where it measured faster: wide outputs (the QNN MLP's input grad, N = 7552); the forward
  // (N = 512) and the k-major weight grad keep the two-stage kernel (tools/kbench.py --which gemmbf)
  int var = g_gemm_bf_variant;
  if (var == 0) var = (M >= 256 && N >= 2048 && !ta) ? 2 : 1;
  if (var >= 2 && M >= 128) {
    const int BM = var == 2 ? 256 : 128;
    p.mt = cdiv(M, BM);
    p.nt = cdiv(N, G8_BN);
    p.gm = p.nt >= 8 ? -1 : 0;
    const int tiles = p.gm < 0 ? 8 * p.mt * cdiv(p.nt, 8) * splits : p.mt * p.nt * splits;
    const int grid = std::min(tiles, 256);
    launch_g8(p, ta, tb, BM, grid, s);  } else {
    p.mt = cdiv(M, 128);
    p.nt = cdiv(N, 128);
    // XCD column partition where there are n-tiles for every XCD; persistent grid: two workgroups per CU (64 KB
    // of LDS each) at most, a multiple of 8 for the partition
    p.gm = p.nt >= 8 ? -1 : 0;
    const int tiles = p.gm < 0 ? 8 * p.mt * cdiv(p.nt, 8) * splits : p.mt * p.nt * splits;
    const int grid = std::min(tiles, 512);
    if (!ta && tb) gemm_bf_kernel<false, true><<<grid, 256, 0, s>>>(p);
    else if (!ta && !tb) gemm_bf_kernel<false, false><<<grid, 256, 0, s>>>(p);
    else if (ta && !tb) gemm_bf_kernel<true, false><<<grid, 256, 0, s>>>(p);
    else gemm_bf_kernel<true, true><<<grid, 256, 0, s>>>(p);
  }
  if (splits > 1) {
    const long MN = (long)M * N;
    int blocks = (int)std::min<long>((MN + 255) / 256, 4096);
    g.ws = ws;
    splitk_reduce_kernel<<<blocks, 256, 0, s>>>(g, splits);
  }
  return check_launch("ctr_gemm_bf16");
}

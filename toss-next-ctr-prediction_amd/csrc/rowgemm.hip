// Row-streaming GEMMs of the DARE encoder layer (src/models/dare.py:53-62: MHA in_proj / out_proj and
// their backward, D = 16 or 32): M = B*K rows (245,760 at cfg2) against a weight of a few KB.  These
// products are HBM-bound (K, N <= 96: ~2-3 flop per byte), so the kernels are shaped for streaming,
// not for MFMA tiles:
//
//   ctr_rowgemm       C[m, :] = epi(A[m, :] W^T or A[m, :] W)   (epilogues: bias, add, residual+RMSNorm)
//     No LDS and no barrier: every wave keeps its B operand (the whole weight, K*N/64 floats per lane)
//     in registers and walks 32-row blocks.  The A operand uses the k-order freedom of a contraction:
//     lane group g (16 lanes) takes k in [g*K/4, (g+1)*K/4), so lane (g, c) reads row 16i + c's segment
//     with 16-byte loads straight into MFMA operand registers; the C layout (rows 4g + r, column c)
//     holds whole 16-column strips of a row per lane group -> the RMSNorm row sum is a 16-lane
//     reduction.
//   ctr_rowgemm_wgrad dW = dY^T X over all rows, plus db = colsum(dY), for one nn.Linear
//     Each workgroup owns a contiguous row range (its four waves interleaved row groups); a k-step of the
//     MFMA is 4 rows (lane group g = row); the bias grad is a VALU sum of the same dY loads.  Each workgroup writes its partial [dW | db] slab row laid out like the gradient arena
//     (weight, then the bias at o_db); ctr_colsum reduces the slab rows in a fixed order -- deterministic,
//     no atomics.
// f32-input MFMA = an exact fmaf chain per lane: results differ from torch's sgemm only in summation
// order.
#include "common.h"
#include "ctr_hip.h"

namespace ctr {

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 rg_mfma(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

struct RowGemmArgs {
  int M;
  const void* A;           // float, or bf16 (the A16 forms: amp's bf16 dqkv, exact in fp32)
  int lda;
  const float* W;          // tb: (N, K) (nn.Linear weight: C = A W^T); else (K, N) (C = A W)
  int tb;
  float* C;
  int ldc;
  const float* bias;       // (N) or null
  const float* add;        // C += add[m, :] (after the bias) or null
  int ld_add;
  const float* resid;      // fused RMSNorm: h = resid + (acc + bias), C = norm_w * h * rsqrt(mean(h^2) + eps)
  int ld_resid;
  const float* norm_w;
  float* norm_h;           // (M, N) saved h, row stride ldc (nullable)
  float* norm_r;           // (M) saved rsqrt (nullable)
  float eps;
};

// row blocks of 16 * NI rows per wave iteration
#ifndef RG_NI
#define RG_NI 2
#endif

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

template <int K, int N, bool SIDE, bool A16 = false>
__global__ __launch_bounds__(256) void rowgemm_kernel(RowGemmArgs a) {
  constexpr int KQ = K / 4, NJ = N / 16, NI = RG_NI;
  constexpr int NS = SIDE ? NJ : 1;      // per-row epilogue operand (add / residual) slots
  const int lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
  const int wave = blockIdx.x * 4 + (threadIdx.x >> 6), nwaves = gridDim.x * 4;
  float w[NJ][KQ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int n = 16 * j + c;
    if (a.tb) {         // W[n][g*KQ .. +KQ) is contiguous: 16-byte loads
#pragma unroll
      for (int q = 0; q < KQ / 4; ++q) {
        const f32x4 v = *(const f32x4*)(a.W + n * K + g * KQ + 4 * q);
#pragma unroll
        for (int t = 0; t < 4; ++t) w[j][4 * q + t] = v[t];
      }
    } else {
#pragma unroll
      for (int kk = 0; kk < KQ; ++kk) w[j][kk] = a.W[(g * KQ + kk) * N + n];
    }
  }
  float bj[NJ], nw[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    bj[j] = a.bias ? a.bias[16 * j + c] : 0.f;
    nw[j] = a.norm_w ? a.norm_w[16 * j + c] : 0.f;
  }
  const float* side = a.norm_w ? a.resid : a.add;     // per-row epilogue operand (nullable)
  const int ld_side = a.norm_w ? a.ld_resid : a.ld_add;
  // the next block's A rows and epilogue operand are loaded while this block computes and stores
  f32x4 av[NI][KQ / 4];
  float sv[NI][4][NS];
  auto load_blk = [&](int blk, f32x4 (&A)[NI][KQ / 4], float (&S)[NI][4][NS]) {
    const int b0 = blk * 16 * NI;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      // rows clamped into range, not skipped (a conditional load is a branch that waits for every load before
      // it); the results of rows past M are never stored
      const long row = min(b0 + 16 * i + c, a.M - 1);
      if constexpr (A16) {     // 16-byte loads of 8 bf16, widened exactly
        static_assert(KQ % 8 == 0, "bf16 A rows in 16-byte pieces");
        const __bf16* ap = (const __bf16*)a.A + row * a.lda + g * KQ;
#pragma unroll
        for (int q = 0; q < KQ / 8; ++q) {
          const bf16x8 v = *(const bf16x8*)(ap + 8 * q);
          A[i][2 * q] = f32x4{(float)v[0], (float)v[1], (float)v[2], (float)v[3]};
          A[i][2 * q + 1] = f32x4{(float)v[4], (float)v[5], (float)v[6], (float)v[7]};
        }
      } else {
#pragma unroll
        for (int q = 0; q < KQ / 4; ++q) A[i][q] = *(const f32x4*)((const float*)a.A + row * a.lda + g * KQ + 4 * q);
      }
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const long orow = min(b0 + 16 * i + 4 * g + rr, a.M - 1);
#pragma unroll
        for (int j = 0; j < NS; ++j) S[i][rr][j] = SIDE ? side[orow * ld_side + 16 * j + c] : 0.f;
      }
    }
  };
  const int nblk = (a.M + 16 * NI - 1) / (16 * NI);
  if (wave < nblk) load_blk(wave, av, sv);
  for (int blk = wave; blk < nblk; blk += nwaves) {
    const int r0 = blk * 16 * NI;
    f32x4 acc[NI][NJ];
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < KQ; ++kk)
#pragma unroll
      for (int i = 0; i < NI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = rg_mfma(av[i][kk >> 2][kk & 3], w[j][kk], acc[i][j]);
    float cur[NI][4][NS];
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr)
#pragma unroll
        for (int j = 0; j < NS; ++j) cur[i][rr][j] = sv[i][rr][j];
    if (blk + nwaves < nblk) load_blk(blk + nwaves, av, sv);
    // epilogue: lane holds C[r0 + 16i + 4g + rr][16j + c]
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int row = r0 + 16 * i + 4 * g + rr;
        const bool live = row < a.M;
        float v[NJ];
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          v[j] = acc[i][j][rr] + bj[j];
          if (SIDE && a.add) v[j] += cur[i][rr][SIDE ? j : 0];
        }
        if (a.norm_w) {
          float ss = 0.f;
#pragma unroll
          for (int j = 0; j < NJ; ++j) {
            v[j] = (SIDE ? cur[i][rr][SIDE ? j : 0] : 0.f) + v[j];
            ss += v[j] * v[j];
          }
          ss = group_sum<16>(ss);
          const float r = 1.0f / sqrtf(ss / (float)N + a.eps);
          if (live) {
            if (c == 0 && a.norm_r) a.norm_r[row] = r;
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
              if (a.norm_h) a.norm_h[(long)row * a.ldc + 16 * j + c] = v[j];
              a.C[(long)row * a.ldc + 16 * j + c] = nw[j] * v[j] * r;
            }
          }
        } else if (live) {
#pragma unroll
          for (int j = 0; j < NJ; ++j) a.C[(long)row * a.ldc + 16 * j + c] = v[j];
        }
      }
  }
}

// dW[NO x NIN] partial of one workgroup over rows [m_begin, m_end): C tile (I, J) = dY[:, 16I..]^T X[:, 16J..].
// Four waves take interleaved groups of 4U rows of the range; a wave's next group is loaded into a second register
// set while the MFMAs of the current one run (loads stay in flight through the whole loop; the loads are
// unconditional, at rows clamped into the range, and dY of a row past it is zeroed at use).  db = colsum(dY) is a
// per-lane VALU sum over the lane's rows, reduced over the four lane groups at the end.  The waves' partials are
// summed in LDS in a fixed wave order and the workgroup writes one slab row -- deterministic.
template <int NO, int NIN, typename TY = float>
__global__ __launch_bounds__(256) void rowgemm_wgrad_kernel(const TY* __restrict__ dY, int ldy,
                                                            const float* __restrict__ X, int ldx, int M,
                                                            int rows_per_wg, float* __restrict__ slab,
                                                            long ld_slab, int o_db) {
  constexpr int IO = NO / 16, JW = NIN / 16;
  constexpr int U = NO >= 96 ? 4 : 8;                       // k-steps (4 rows each) of one group
  constexpr int NA = IO * JW * 4 + IO;                       // accumulator floats per lane (+ the bias sums)
  constexpr int STEP = 4 * 4 * U;                            // rows of one pass of the four waves
  __shared__ float red[3][NA][64];
  const int lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);    // wave-uniform: the loop runs on scalars
  const int m_begin = blockIdx.x * rows_per_wg, m_end = min(M, m_begin + rows_per_wg);
  f32x4 acc[IO][JW];
  float db[IO];
#pragma unroll
  for (int i = 0; i < IO; ++i) {
    db[i] = 0.f;
#pragma unroll
    for (int j = 0; j < JW; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  auto load = [&](int m0, float (&ay)[U][IO], float (&bx)[U][JW]) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long m = min(m0 + 4 * u + g, m_end - 1);
#pragma unroll
      for (int i = 0; i < IO; ++i) ay[u][i] = (float)dY[m * ldy + 16 * i + c];
#pragma unroll
      for (int j = 0; j < JW; ++j) bx[u][j] = X[m * ldx + 16 * j + c];
    }
  };
  auto compute = [&](int m0, const float (&ay)[U][IO], const float (&bx)[U][JW]) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const bool ok = m0 + 4 * u + g < m_end;
#pragma unroll
      for (int i = 0; i < IO; ++i) {
        const float y = ok ? ay[u][i] : 0.f;
        db[i] += y;
#pragma unroll
        for (int j = 0; j < JW; ++j) acc[i][j] = rg_mfma(y, bx[u][j], acc[i][j]);
      }
    }
  };
  float ya[U][IO], xa[U][JW], yb[U][IO], xb[U][JW];
  const int mw = m_begin + 4 * U * w;
  if (mw < m_end) load(mw, ya, xa);
  // Two groups per trip and no branch inside: a skipped load (or a break between a load and its use, which lets
  // the compiler sink the loads past it) makes the wait counts assume the newest loads are the ones a compute
  // needs.  A group past the range (at most one per wave) runs on clamped rows with dY zeroed.
  for (int m0 = mw; m0 < m_end; m0 += 2 * STEP) {
    load(m0 + STEP, yb, xb);
    compute(m0, ya, xa);
    load(m0 + 2 * STEP, ya, xa);
    compute(m0 + STEP, yb, xb);
  }
#pragma unroll
  for (int i = 0; i < IO; ++i) {                             // lane (g, c) -> column 16i + c over all four g
    db[i] += __shfl_xor(db[i], 16, 64);
    db[i] += __shfl_xor(db[i], 32, 64);
  }
  if (w > 0) {
#pragma unroll
    for (int i = 0; i < IO; ++i) {
#pragma unroll
      for (int j = 0; j < JW; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) red[w - 1][(i * JW + j) * 4 + r][lane] = acc[i][j][r];
      red[w - 1][IO * JW * 4 + i][lane] = db[i];
    }
  }
  __syncthreads();
  if (w != 0) return;
#pragma unroll 1
  for (int src = 0; src < 3; ++src)
#pragma unroll
    for (int i = 0; i < IO; ++i) {
#pragma unroll
      for (int j = 0; j < JW; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[i][j][r] += red[src][(i * JW + j) * 4 + r][lane];
      db[i] += red[src][IO * JW * 4 + i][lane];
    }
  float* out = slab + (long)blockIdx.x * ld_slab;
#pragma unroll
  for (int i = 0; i < IO; ++i) {
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int o = 16 * i + 4 * g + rr;
#pragma unroll
      for (int j = 0; j < JW; ++j) out[(long)o * NIN + 16 * j + c] = acc[i][j][rr];
    }
    if (g == 0) out[o_db + 16 * i + c] = db[i];
  }
}

// persistent grid: as many workgroups as fit the chip at once (register-limited occupancy)
template <int K, int N, bool SIDE, bool A16 = false>
static int resident_grid(int M) {
  static int per_cu = 0;
  if (per_cu == 0) {
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, rowgemm_kernel<K, N, SIDE, A16>, 256, 0) != hipSuccess || nb < 1)
      nb = 1;
    per_cu = std::min(nb, 4);
  }
  const int nblk = (M + 16 * RG_NI - 1) / (16 * RG_NI);
  return std::max(1, std::min((nblk + 3) / 4, 256 * per_cu));
}

template <int K, int N>
static void launch_rowgemm(const RowGemmArgs& a, hipStream_t s) {
  if (a.add || a.norm_w) rowgemm_kernel<K, N, true><<<resident_grid<K, N, true>(a.M), 256, 0, s>>>(a);
  else rowgemm_kernel<K, N, false><<<resident_grid<K, N, false>(a.M), 256, 0, s>>>(a);
}

static bool rowgemm_shape(int K, int N) {
  return (K == 16 && (N == 16 || N == 48)) || (K == 48 && N == 16) || (K == 32 && (N == 32 || N == 96)) ||
         (K == 96 && N == 32);
}

static bool wgrad_shape(int NO, int NIN) {
  return (NIN == 16 && (NO == 16 || NO == 48)) || (NIN == 32 && (NO == 32 || NO == 96));
}

// workgroup b of the weight-grad kernel owns rows [b*rpw, (b+1)*rpw): ~512 workgroups of four waves (two per
// CU), rpw a multiple of 128 (one 32-row group per wave per pass) -- a <= 512-row slab for the column sum
// (1024 or 2048 workgroups measured 7-10% slower at cfg2)
static void wgrad_split(int M, int* rpw, int* waves) {
  const int target = std::max(1, std::min(512, (M + 255) / 256));
  *rpw = ((M + target - 1) / target + 127) / 128 * 128;
  *waves = (M + *rpw - 1) / *rpw;
}

}  // namespace ctr

using namespace ctr;

extern "C" int ctr_rowgemm_supported(int K, int N) { return rowgemm_shape(K, N) ? 1 : 0; }

extern "C" int ctr_rowgemm(int M, int K, int N, const float* A, int lda, const float* W, int tb, float* C, int ldc,
                           const float* bias, const float* add, int ld_add, const float* resid, int ld_resid,
                           const float* norm_w, float* norm_h, float* norm_r, float eps, void* stream) {
  CTR_REQUIRE(rowgemm_shape(K, N), "ctr_rowgemm: unsupported (K, N)");
  CTR_REQUIRE((lda & 3) == 0 && (((uintptr_t)A) & 15) == 0, "ctr_rowgemm: A rows must be 16-byte aligned");
  CTR_REQUIRE(!norm_w || resid, "ctr_rowgemm: the fused RMSNorm needs the residual");
  if (M <= 0) return 0;
  RowGemmArgs a{M, A, lda, W, tb, C, ldc, bias, add, ld_add, resid, ld_resid, norm_w, norm_h, norm_r, eps};
  hipStream_t s = (hipStream_t)stream;
  if (K == 16 && N == 16) launch_rowgemm<16, 16>(a, s);
  else if (K == 16) launch_rowgemm<16, 48>(a, s);
  else if (K == 48) launch_rowgemm<48, 16>(a, s);
  else if (K == 32 && N == 32) launch_rowgemm<32, 32>(a, s);
  else if (K == 32) launch_rowgemm<32, 96>(a, s);
  else launch_rowgemm<96, 32>(a, s);
  return check_launch("rowgemm");
}

extern "C" int ctr_rowgemm_wgrad_rows(int M) {
  int rpw, waves;
  wgrad_split(std::max(M, 1), &rpw, &waves);
  return waves;
}

extern "C" int ctr_rowgemm_wgrad(const float* dY, int ldy, const float* X, int ldx, int M, int NO, int NIN,
                                 float* slab, long ld_slab, int o_db, void* stream) {
  CTR_REQUIRE(wgrad_shape(NO, NIN), "ctr_rowgemm_wgrad: unsupported (NO, NIN)");
  CTR_REQUIRE(o_db >= NO * NIN && ld_slab >= (long)o_db + NO, "ctr_rowgemm_wgrad: slab layout");
  if (M <= 0) return 0;
  int rpw, grid;
  wgrad_split(M, &rpw, &grid);
  hipStream_t s = (hipStream_t)stream;
  if (NIN == 16 && NO == 16) rowgemm_wgrad_kernel<16, 16><<<grid, 256, 0, s>>>(dY, ldy, X, ldx, M, rpw, slab, ld_slab, o_db);
  else if (NIN == 16) rowgemm_wgrad_kernel<48, 16><<<grid, 256, 0, s>>>(dY, ldy, X, ldx, M, rpw, slab, ld_slab, o_db);
  else if (NO == 32) rowgemm_wgrad_kernel<32, 32><<<grid, 256, 0, s>>>(dY, ldy, X, ldx, M, rpw, slab, ld_slab, o_db);
  else rowgemm_wgrad_kernel<96, 32><<<grid, 256, 0, s>>>(dY, ldy, X, ldx, M, rpw, slab, ld_slab, o_db);
  return check_launch("rowgemm_wgrad");
}

extern "C" int ctr_rowgemm_a16(int M, int K, int N, const uint16_t* A, int lda, const float* W, int tb, float* C, int ldc,
                               const float* bias, const float* add, int ld_add, void* stream) {
  CTR_REQUIRE(K == 96 && N == 32, "ctr_rowgemm_a16: (K, N) = (96, 32)");
  CTR_REQUIRE((lda & 7) == 0 && (((uintptr_t)A) & 15) == 0, "ctr_rowgemm_a16: A rows must be 16-byte aligned");
  if (M <= 0) return 0;
  RowGemmArgs a{M, A, lda, W, tb, C, ldc, bias, add, ld_add, nullptr, 0, nullptr, nullptr, nullptr, 0.f};
  hipStream_t s = (hipStream_t)stream;
  if (add) rowgemm_kernel<96, 32, true, true><<<resident_grid<96, 32, true, true>(M), 256, 0, s>>>(a);
  else rowgemm_kernel<96, 32, false, true><<<resident_grid<96, 32, false, true>(M), 256, 0, s>>>(a);
  return check_launch("rowgemm_a16");
}

extern "C" int ctr_rowgemm_wgrad_y16(const uint16_t* dY, int ldy, const float* X, int ldx, int M, int NO, int NIN,
                                     float* slab, long ld_slab, int o_db, void* stream) {
  CTR_REQUIRE(NO == 96 && NIN == 32, "ctr_rowgemm_wgrad_y16: (NO, NIN) = (96, 32)");
  CTR_REQUIRE(o_db >= NO * NIN && ld_slab >= (long)o_db + NO, "ctr_rowgemm_wgrad_y16: slab layout");
  if (M <= 0) return 0;
  int rpw, grid;
  wgrad_split(M, &rpw, &grid);
  rowgemm_wgrad_kernel<96, 32, __bf16><<<grid, 256, 0, (hipStream_t)stream>>>((const __bf16*)dY, ldy, X, ldx, M, rpw,
                                                                             slab, ld_slab, o_db);
  return check_launch("rowgemm_wgrad_y16");
}

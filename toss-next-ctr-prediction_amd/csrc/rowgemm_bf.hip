// amp: bf16 row-streaming GEMMs of the DARE encoder layer at the widths the fp32 row kernels (rowgemm.hip) do
// not hold in registers: D = 64 (cfgs/v3_k148_s1.yaml, and dare_qnn_next.yaml as written).  Under
// autocast(bfloat16) the reference runs MHA's in_proj / out_proj (src/models/dare.py:53-62, F.linear inside
// nn.MultiheadAttention) and their backward as bf16 matmuls (src/train.py:158-168): operands rounded to bf16,
// fp32 accumulation.  These kernels do the same on v_mfma_f32_16x16x32_bf16 and keep fp32 outputs (the
// reference rounds the outputs to bf16 as well; the fp32 result is the more precise of the two).
//
//   ctr_rowgemm_bf       C[m, :] = epi(A[m, :] W^T or A[m, :] W)   (epilogues: bias, add, residual + RMSNorm)
//     The weight (a few tens of KB) is rounded into an LDS operand image once per workgroup: entry
//     (j, s, lane) holds the 8 bf16 k-values of column 16 j + c that lane (g, c) feeds step s -- one
//     conflict-free 16-byte LDS read per MFMA B operand.  The A operand uses the k-order freedom of the
//     contraction as rowgemm.hip does: lane group g takes k in [g K/4, (g+1) K/4), so lane (g, c) reads row
//     16 i + c's segment with 16-byte loads and rounds it to bf16 in registers; the C layout (rows 4 g + r,
//     column c) puts 16-column strips of a row in a lane group -> the RMSNorm row sum is a 16-lane reduction.
//     Persistent waves walk row blocks with the next block's rows in flight during the epilogue.
//   ctr_rowgemm_bf_wgrad dW = dY^T X over all rows (bf16 operands) plus db = colsum(dY) (fp32, from the fp32
//     dY), for one nn.Linear.  MFMA k = rows: lane (g, c) supplies rows 8 g .. 8 g + 7 of a 32-row step; the
//     four waves of a workgroup split the output rows (NO / 64 tiles of 16 each) and walk the workgroup's
//     whole row range, so no cross-wave reduction is needed; each workgroup writes one slab row laid out like
//     the grad arena (weight, then the bias at o_db) and ctr_colsum reduces the rows in a fixed order --
//     deterministic, no atomics.
#include "common.h"
#include "ctr_hip.h"

namespace ctr {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 mfma_bf(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ bf16x8 pack8(f32x4 lo, f32x4 hi) {     // round to nearest even
  const bf16x4 l = __builtin_convertvector(lo, bf16x4), h = __builtin_convertvector(hi, bf16x4);
  return bf16x8{l[0], l[1], l[2], l[3], h[0], h[1], h[2], h[3]};
}

struct RowGemmBfArgs {
  int M;
  const float* A;
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

// 16-row blocks per wave iteration: two where the registers allow (K, N <= 64)
template <int K, int N>
struct RgBf {
  static constexpr int KL = K / 4;            // k-range of one lane group
  static constexpr int KS = KL / 8;           // MFMA steps
  static constexpr int NJ = N / 16;
  static constexpr int NI = (K <= 64 && N <= 64) ? 2 : 1;
  static constexpr int IMG = NJ * KS * 64;    // bf16x8 entries of the weight image
};

// EPI: 0 = + bias, 1 = + bias + add, 2 = residual + RMSNorm (compile-time: no per-row branches)
template <int K, int N, int EPI>
__global__ __launch_bounds__(256) void rowgemm_bf_kernel(RowGemmBfArgs a) {
  using S = RgBf<K, N>;
  constexpr int KL = S::KL, KS = S::KS, NJ = S::NJ, NI = S::NI;
  constexpr bool SIDE = EPI != 0;
  constexpr int NS = SIDE ? NJ : 1;      // per-row epilogue operand (add / residual) slots
  __shared__ bf16x8 wimg[S::IMG];
#pragma unroll 1
  for (int e = threadIdx.x; e < S::IMG; e += 256) {
    const int l = e & 63, s = (e >> 6) % KS, j = (e >> 6) / KS;
    const int n = 16 * j + (l & 15), k0 = (l >> 4) * KL + 8 * s;
    f32x4 lo, hi;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      lo[t] = a.tb ? a.W[n * K + k0 + t] : a.W[(k0 + t) * N + n];
      hi[t] = a.tb ? a.W[n * K + k0 + 4 + t] : a.W[(k0 + 4 + t) * N + n];
    }
    wimg[e] = pack8(lo, hi);
  }
  const int lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
  const int wave = blockIdx.x * 4 + (threadIdx.x >> 6), nwaves = gridDim.x * 4;
  float bj[NJ], nw[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    bj[j] = a.bias ? a.bias[16 * j + c] : 0.f;
    nw[j] = EPI == 2 ? a.norm_w[16 * j + c] : 0.f;
  }
  const float* side = EPI == 2 ? a.resid : a.add;
  const int ld_side = EPI == 2 ? a.ld_resid : a.ld_add;
  f32x4 av[NI][KL / 4];
  auto load_blk = [&](int blk) {
    const int b0 = blk * 16 * NI;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      // rows clamped into range, not skipped; the results of rows past M are never stored
      const long row = min(b0 + 16 * i + c, a.M - 1);
#pragma unroll
      for (int q = 0; q < KL / 4; ++q) av[i][q] = *(const f32x4*)(a.A + row * a.lda + g * KL + 4 * q);
    }
  };
  const int nblk = (a.M + 16 * NI - 1) / (16 * NI);
  if (wave < nblk) load_blk(wave);
  __syncthreads();
  for (int blk = wave; blk < nblk; blk += nwaves) {
    // the weight image is re-read from LDS every block: hoisted out of the loop it would hold K N / 128
    // registers for the whole walk (occupancy 3 -> 2 waves per SIMD at 64 x 192)
    __asm__ volatile("" ::: "memory");
    const int r0 = blk * 16 * NI;
    bf16x8 ab[NI][KS];
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int s = 0; s < KS; ++s) ab[i][s] = pack8(av[i][2 * s], av[i][2 * s + 1]);
    // the block's epilogue operand, in flight during the MFMAs
    float cur[NI][4][NS];
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const long orow = min(r0 + 16 * i + 4 * g + rr, a.M - 1);
#pragma unroll
        for (int j = 0; j < NS; ++j) cur[i][rr][j] = SIDE ? side[orow * ld_side + 16 * j + c] : 0.f;
      }
    f32x4 acc[NI][NJ];
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const bf16x8 b = wimg[(j * KS + s) * 64 + lane];
#pragma unroll
        for (int i = 0; i < NI; ++i) acc[i][j] = mfma_bf(ab[i][s], b, acc[i][j]);
      }
    // the next block's rows: in flight during this block's epilogue (loaded after the MFMAs have consumed av)
    if (blk + nwaves < nblk) load_blk(blk + nwaves);
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
          if (EPI == 1) v[j] += cur[i][rr][SIDE ? j : 0];
        }
        if (EPI == 2) {
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

// dW[NO x NIN] partial of one workgroup over rows [m_begin, m_end).  Wave w owns output rows
// [16 IW w, 16 IW (w + 1)) (IW = NO / 64 tiles) and walks all rows of the range in 32-row steps, two per trip
// with the next step's loads in flight (unconditional loads at rows clamped into the range; dY of a row past
// it is zeroed at use, so the trip needs no branch).
template <int NO, int NIN>
__global__ __launch_bounds__(256) void rowgemm_bf_wgrad_kernel(const float* __restrict__ dY, int ldy,
                                                               const float* __restrict__ X, int ldx, int M,
                                                               int rows_per_wg, float* __restrict__ slab,
                                                               long ld_slab, int o_db) {
  constexpr int IW = NO / 64, JW = NIN / 16;
  const int lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int m_begin = blockIdx.x * rows_per_wg, m_end = min(M, m_begin + rows_per_wg);
  const int o_base = 16 * IW * w;
  f32x4 acc[IW][JW];
  float db[IW];
#pragma unroll
  for (int i = 0; i < IW; ++i) {
    db[i] = 0.f;
#pragma unroll
    for (int j = 0; j < JW; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  auto load = [&](int m0, float (&ay)[IW][8], float (&bx)[JW][8]) {
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const long m = min(m0 + 8 * g + t, m_end - 1);
#pragma unroll
      for (int i = 0; i < IW; ++i) ay[i][t] = dY[m * ldy + o_base + 16 * i + c];
#pragma unroll
      for (int j = 0; j < JW; ++j) bx[j][t] = X[m * ldx + 16 * j + c];
    }
  };
  auto compute = [&](int m0, const float (&ay)[IW][8], const float (&bx)[JW][8]) {
    bf16x8 xb[JW];
#pragma unroll
    for (int j = 0; j < JW; ++j)
      xb[j] = pack8(f32x4{bx[j][0], bx[j][1], bx[j][2], bx[j][3]}, f32x4{bx[j][4], bx[j][5], bx[j][6], bx[j][7]});
#pragma unroll
    for (int i = 0; i < IW; ++i) {
      float y[8];
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        y[t] = (m0 + 8 * g + t < m_end) ? ay[i][t] : 0.f;
        db[i] += y[t];
      }
      const bf16x8 yb = pack8(f32x4{y[0], y[1], y[2], y[3]}, f32x4{y[4], y[5], y[6], y[7]});
#pragma unroll
      for (int j = 0; j < JW; ++j) acc[i][j] = mfma_bf(yb, xb[j], acc[i][j]);
    }
  };
  float ya[IW][8], xa[JW][8], yb[IW][8], xb[JW][8];
  load(m_begin, ya, xa);
  for (int m0 = m_begin; m0 < m_end; m0 += 64) {
    load(m0 + 32, yb, xb);
    compute(m0, ya, xa);
    load(m0 + 64, ya, xa);
    compute(m0 + 32, yb, xb);
  }
#pragma unroll
  for (int i = 0; i < IW; ++i) {                 // lane (g, c) -> column o_base + 16i + c over all four g
    db[i] += __shfl_xor(db[i], 16, 64);
    db[i] += __shfl_xor(db[i], 32, 64);
  }
  float* out = slab + (long)blockIdx.x * ld_slab;
#pragma unroll
  for (int i = 0; i < IW; ++i) {
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int o = o_base + 16 * i + 4 * g + rr;
#pragma unroll
      for (int j = 0; j < JW; ++j) out[(long)o * NIN + 16 * j + c] = acc[i][j][rr];
    }
    if (g == 0) out[o_db + o_base + 16 * i + c] = db[i];
  }
}

template <int K, int N, int EPI>
int bf_grid(int M) {
  static int per_cu = 0;
  if (per_cu == 0) {
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, rowgemm_bf_kernel<K, N, EPI>, 256, 0) != hipSuccess ||
        nb < 1)
      nb = 1;
    per_cu = std::min(nb, 4);
  }
  const int nblk = (M + 16 * RgBf<K, N>::NI - 1) / (16 * RgBf<K, N>::NI);
  return std::max(1, std::min((nblk + 3) / 4, 256 * per_cu));
}

template <int K, int N>
void launch_bf(const RowGemmBfArgs& a, hipStream_t s) {   // the epilogues the encoder layer uses per shape
  if (a.norm_w) rowgemm_bf_kernel<K, N, 2><<<bf_grid<K, N, 2>(a.M), 256, 0, s>>>(a);
  else if (a.add) rowgemm_bf_kernel<K, N, 1><<<bf_grid<K, N, 1>(a.M), 256, 0, s>>>(a);
  else rowgemm_bf_kernel<K, N, 0><<<bf_grid<K, N, 0>(a.M), 256, 0, s>>>(a);
}

bool bf_shape(int K, int N) {
  return (K == 64 && (N == 64 || N == 192)) || (K == 192 && N == 64);
}
bool bf_wgrad_shape(int NO, int NIN) { return NIN == 64 && (NO == 64 || NO == 192); }

// rows of one workgroup: ~512 workgroups (two per CU), a multiple of 64 rows (one trip of a wave)
void bf_wgrad_split(int M, int* rpw, int* wgs) {
  const int target = std::max(1, std::min(512, (M + 255) / 256));
  *rpw = ((M + target - 1) / target + 63) / 64 * 64;
  *wgs = (M + *rpw - 1) / *rpw;
}

}  // namespace
}  // namespace ctr

using namespace ctr;

extern "C" int ctr_rowgemm_bf_supported(int K, int N) { return bf_shape(K, N) ? 1 : 0; }

extern "C" int ctr_rowgemm_bf(int M, int K, int N, const float* A, int lda, const float* W, int tb, float* C, int ldc,
                              const float* bias, const float* add, int ld_add, const float* resid, int ld_resid,
                              const float* norm_w, float* norm_h, float* norm_r, float eps, void* stream) {
  CTR_REQUIRE(bf_shape(K, N), "unsupported (K, N)");
  CTR_REQUIRE((lda & 3) == 0 && (((uintptr_t)A) & 15) == 0, "A rows must be 16-byte aligned");
  CTR_REQUIRE(!norm_w || resid, "the fused RMSNorm needs the residual");
  if (M <= 0) return 0;
  RowGemmBfArgs a{M, A, lda, W, tb, C, ldc, bias, add, ld_add, resid, ld_resid, norm_w, norm_h, norm_r, eps};
  hipStream_t s = (hipStream_t)stream;
  if (K == 64 && N == 64) launch_bf<64, 64>(a, s);
  else if (K == 64) launch_bf<64, 192>(a, s);
  else launch_bf<192, 64>(a, s);
  return check_launch("rowgemm_bf");
}

extern "C" int ctr_rowgemm_bf_wgrad_rows(int M) {
  int rpw, wgs;
  bf_wgrad_split(std::max(M, 1), &rpw, &wgs);
  return wgs;
}

extern "C" int ctr_rowgemm_bf_wgrad(const float* dY, int ldy, const float* X, int ldx, int M, int NO, int NIN,
                                    float* slab, long ld_slab, int o_db, void* stream) {
  CTR_REQUIRE(bf_wgrad_shape(NO, NIN), "unsupported (NO, NIN)");
  CTR_REQUIRE(o_db >= NO * NIN && ld_slab >= (long)o_db + NO, "slab layout");
  if (M <= 0) return 0;
  int rpw, grid;
  bf_wgrad_split(M, &rpw, &grid);
  hipStream_t s = (hipStream_t)stream;
  if (NO == 64) rowgemm_bf_wgrad_kernel<64, 64><<<grid, 256, 0, s>>>(dY, ldy, X, ldx, M, rpw, slab, ld_slab, o_db);
  else rowgemm_bf_wgrad_kernel<192, 64><<<grid, 256, 0, s>>>(dY, ldy, X, ldx, M, rpw, slab, ld_slab, o_db);
  return check_launch("rowgemm_bf_wgrad");
}

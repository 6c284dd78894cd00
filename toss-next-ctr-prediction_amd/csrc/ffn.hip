// Fused position-wise FFN of the DARE encoder layer (src/models/dare.py:53-70, the ffn Sequential
// Linear(D, FF) -> GELU -> Dropout -> Linear(FF, D), then residual + RMSNorm), forward and backward.
//
// Unfused, each layer writes and re-reads two M x FF fp32 activations (pre-GELU and post-dropout:
// 2 x 377 MB at M = 245,760, FF = 384) and the backward writes/reads a third (dact) -- ~2.3 GB of HBM
// traffic per layer.  Here a workgroup owns RT rows; the FF-wide values live only in registers (plus a
// 16-column wave-private LDS tile).  Forward: each wave RW = RT/4 rows, all waves walk FF in 16-column
// chunks and store the dropout keep bits.  Backward (recomputes pre = x1 W1^T + b1, reads the keep
// bits): for D <= 32 the column-owner form (ffn_bwd_cols_kernel: wave w takes chunks w, w+4, ... over
// all the tile's rows), otherwise the rows-per-wave form (ffn_bwd_kernel).
//
// All products are v_mfma_f32_16x16x4_f32 (exact fp32).  Operand layouts (lane l, g = l>>4, c = l&15):
//   A[i][k] -> lane holds A[c][g],  B[k][j] -> lane holds B[g][c],  C[i][j] -> reg r holds C[4g+r][c].
// A contraction may visit its k index in any order, which removes transposes:
//   * D-contractions (x1 W1^T, dh W2) give lane group g the k range [g*D/4, (g+1)*D/4), so each lane
//     reads its A row segment with ds_read_b128 and its B row segment with 16-byte global loads;
//   * row-contractions (dW1, dW2) use the C-layout register r of a 16-row block directly as the A / B
//     operand whose k-set is the rows {4g + r}.
// Only the FF-contractions (fo W2^T forward, dact W1 backward) stage the chunk through LDS.
// Weight / bias grads go to a per-workgroup slab row (rows-per-wave form: the four waves' partials summed
// in a fixed order per chunk; column-owner form: complete per wave); ctr_colsum (rowops.hip) reduces the
// slabs in a fixed order -- deterministic.
#include <cstdlib>

#include "common.h"
#include "ctr_hip.h"

namespace ctr {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 buf_ld4(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
}

struct FfnArgs {
  int M, FF;
  const float* x;      // (M, D) layer input x1 (post-norm1)
  const float* W1;     // (FF, D)
  const float* b1;     // (FF)
  const float* W2;     // (D, FF)
  const float* b2;     // (D)
  const float* nw;     // (D) norm2 weight
  float eps;
  Drop drop;
  uint16_t* mask;      // dropout keep bits (layout: FfnTile::LW), written by the forward, read by the backward
  // forward outputs
  float* y;            // (M, D) = norm2(x + ffn(x))
  float* h;            // (M, D) pre-norm sum (saved for the norm backward)
  float* r;            // (M) 1/rms
  // backward
  const float* dh;     // (M, D) grad wrt the pre-norm sum (from ctr_rmsnorm_bwd)
  float* dx;           // (M, D) grad wrt x1 (ffn path + residual)
  float* slab;         // (gridDim.x, ld_slab): [dW1 at o_w1 | db1 at o_b1 | dW2 at o_w2] per workgroup
  long ld_slab;
  int o_b1, o_w2;
  // norm-fused backward (ctr_ffn_bwd_norms): the layer's two RMSNorm backwards around the FFN
  int o_w1, o_b2, o_n1, o_n2;   // slab offsets of dW1, db2, d norm1.w, d norm2.w
  const float* dy;     // (M, D) grad wrt the layer output x2 = norm2(h2)
  const float* h2;     // (M, D) pre-norm2 sum, r2 (M) its rsqrt, nw2 norm2.w
  const float* r2;
  const float* nw2;
  const float* h1;     // (M, D) pre-norm1 sum (x + attn(x)), r1 (M), nw1 norm1.w
  const float* r1;
  const float* nw1;
  float* dh1;          // (M, D) output: grad wrt h1
  __bf16* wbf;         // amp bf16: W1 (FF, D) | W2^T (FF, D) | W1^T (D, FF) in bf16, written by the forward
};

template <int D>
struct FfnTile {
  static constexpr int RT = D >= 64 ? 64 : 128;   // rows per workgroup
  static constexpr int RW = RT / 4;               // rows per wave
  static constexpr int NI = RW / 16;              // 16-row blocks per wave
  static constexpr int NJ = D / 16;               // 16-col blocks of D
  static constexpr int KQ = D / 4;                // k-steps of a D-contraction
  static constexpr int S = D + 4;                 // LDS row stride of x / dh tiles (16 B aligned)
  static constexpr int SS = 20;                   // staging row stride (16 cols + pad)
  static constexpr int TILE = RT * S;             // floats of one x / dh tile
  static constexpr int STG = RW * SS;             // one wave's staging tile
  static constexpr int PW = 32 * D + 16;          // one wave's per-chunk weight-grad partial
  static constexpr int RG = PW > STG ? PW : STG;  // backward: per-wave region (staging, then partial)
  // backward: double-buffered regions (one barrier per chunk) when two workgroups still fit a CU
  static constexpr int NBUF = (2 * TILE + 8 * RG) * 4 <= 80 * 1024 ? 2 : 1;
  // keep-bit layout.  LW ("lane words", D <= 32, RT = 128): for 16-column chunk ci and 128-row tile t,
  // dword ((ci * T128 + t) * 4 + g) * 16 + c holds the bits of column 16 ci + c for the rows
  // 128 t + 16 i + 4 g + rr at bit 4 i + rr -- exactly what lane (g, c) of a kernel whose 16-row blocks
  // start on a tile boundary needs (one dword per chunk).  Otherwise (D = 64): chunk-major (FF/16, M)
  // uint16 row words.
  static constexpr bool LW = D <= 32;
};

// dword index of lane (g, c)'s keep bits for chunk ci, 128-row tile t (LW layout)
__device__ __forceinline__ uint32_t lw_word(int ci, int t, int T128, int g, int c) {
  return ((uint32_t)(ci * T128 + t) * 4 + g) * 16 + c;
}
__host__ __device__ __forceinline__ long lw_words(long M, int FF) { return (long)(FF / 16) * ((M + 127) / 128) * 64; }

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// Column position of d in a PERM tile (column-owner backward): the NJ values 16j + c of lane column c
// sit next to each other, so a lane reads them with one ds_read_b64 at a per-row immediate offset.
template <int D>
__device__ __forceinline__ constexpr int pcol(int d) { return (d % 16) * (D / 16) + d / 16; }

// store a row segment (columns c4..c4+3) into an LDS tile row, permuted (pcol) or not
template <int D, bool PERM>
__device__ __forceinline__ void put4(float* row, int c4, f32x4 v) {
  if (PERM) {
#pragma unroll
    for (int t = 0; t < 4; ++t) row[pcol<D>(c4 + t)] = v[t];
  } else {
    *(f32x4*)(row + c4) = v;
  }
}

// rows [m0, m0+RT) of a (M, D) matrix -> LDS tile with stride S (zero rows past M)
template <int D, bool PERM = false>
__device__ __forceinline__ void load_tile(const float* __restrict__ src, int M, int m0, float* dst) {
  using T = FfnTile<D>;
  for (int q = threadIdx.x; q < T::RT * D / 4; q += 256) {
    const int i = q / (D / 4), c4 = (q % (D / 4)) * 4;
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (m0 + i < M) v = *(const f32x4*)(src + (long)(m0 + i) * D + c4);
    put4<D, PERM>(dst + i * T::S, c4, v);
  }
}

// acc[i] (C[row][ff], rows 16i.. of the wave's tile rows, ff = this lane's column) += rows x D @ B over
// D, lane group g covering d in [g*KQ, (g+1)*KQ); bv[kk] = this lane's B value for d = g*KQ + kk.
template <int D>
__device__ __forceinline__ void dcontract(const float* tile, const float (&bv)[FfnTile<D>::KQ],
                                          f32x4 (&acc)[FfnTile<D>::NI], int g, int c) {
  using T = FfnTile<D>;
#pragma unroll
  for (int i = 0; i < T::NI; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  // k-step outer, row blocks inner: the NI accumulation chains interleave (no dependent-MFMA stall)
#pragma unroll
  for (int kq = 0; kq < T::KQ; kq += 4) {
    f32x4 av[T::NI];
#pragma unroll
    for (int i = 0; i < T::NI; ++i) av[i] = *(const f32x4*)(tile + (16 * i + c) * T::S + g * T::KQ + kq);
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int i = 0; i < T::NI; ++i) acc[i] = mfma4(av[i][t], bv[kq + t], acc[i]);
  }
}

// acc[i][j] += st(rows x 16) @ Wslice(16 x D): A from the staging tile, bw[j][t] = B[f0 + 4g + t][16j + c]
template <int D>
__device__ __forceinline__ void fcontract(const float* st, const float (&bw)[FfnTile<D>::NJ][4],
                                          f32x4 (&acc)[FfnTile<D>::NI][FfnTile<D>::NJ], int g, int c) {
  using T = FfnTile<D>;
#pragma unroll
  for (int i = 0; i < T::NI; ++i) {
    const f32x4 av = *(const f32x4*)(st + (16 * i + c) * T::SS + 4 * g);
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int j = 0; j < T::NJ; ++j) acc[i][j] = mfma4(av[t], bw[j][t], acc[i][j]);
  }
}

// ---------------------------------------------------------------- forward
// h = x + (y + b2); RMSNorm over the row (the row's D values sit in the 16 lanes of one lane group).
// yacc[i][j][rr]: row 16i + 4g + rr of this wave's rows (first row mw, LDS rows xw), column 16j + c.
template <int D, class T>
__device__ __forceinline__ void ffn_fwd_epilogue(const FfnArgs& a, const f32x4 (&yacc)[T::NI][T::NJ], const float* xw,
                                                 int mw) {
  const int lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
#pragma unroll
  for (int i = 0; i < T::NI; ++i)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int row = 16 * i + 4 * g + rr, m = mw + row;
      float hv[T::NJ];
      float ss = 0.f;
#pragma unroll
      for (int j = 0; j < T::NJ; ++j) {
        const int d = 16 * j + c;
        hv[j] = xw[row * T::S + d] + (yacc[i][j][rr] + a.b2[d]);
        ss += hv[j] * hv[j];
      }
      ss = group_sum<16>(ss);
      const float rs = 1.0f / sqrtf(ss / (float)D + a.eps);
      if (m < a.M) {
        if (c == 0) a.r[m] = rs;
#pragma unroll
        for (int j = 0; j < T::NJ; ++j) {
          const int d = 16 * j + c;
          a.h[(long)m * D + d] = hv[j];
          a.y[(long)m * D + d] = a.nw[d] * hv[j] * rs;
        }
      }
    }
}

template <int D>
__global__ __launch_bounds__(256) void ffn_fwd_kernel(FfnArgs a) {
  using T = FfnTile<D>;
  __shared__ __attribute__((aligned(16))) float smem[T::TILE + 4 * T::STG];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, c = lane & 15;
  const int m0 = blockIdx.x * T::RT;
  load_tile<D>(a.x, a.M, m0, smem);
  __syncthreads();
  const float* xw = smem + w * T::RW * T::S;     // this wave's rows
  float* st = smem + T::TILE + w * T::STG;

  f32x4 yacc[T::NI][T::NJ];
#pragma unroll
  for (int i = 0; i < T::NI; ++i)
#pragma unroll
    for (int j = 0; j < T::NJ; ++j) yacc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // W slices of chunk f0 are prefetched one chunk ahead into the other of two register sets (the chunk
  // loop is unrolled by two, so no copies and no wait on the prefetch until its chunk); buffer loads keep
  // the per-lane offsets fixed and move the chunk offset to an SGPR
  const auto rW1 = buf_rsrc(a.W1, (uint32_t)a.FF * D * 4);
  const auto rW2 = buf_rsrc(a.W2, (uint32_t)a.FF * D * 4);
  const auto rb1 = buf_rsrc(a.b1, (uint32_t)a.FF * 4);
  const uint32_t mask_bytes = !a.mask ? 0u : T::LW ? (uint32_t)lw_words(a.M, a.FF) * 4 : (uint32_t)(a.FF / 16) * a.M * 2;
  const auto rmask = buf_rsrc(a.mask, mask_bytes);
  const int T128 = (a.M + 127) / 128;
  struct Wc {
    float v1[T::KQ], v2[T::NJ][4], b;
  };
  auto load_w = [&](int f0, Wc& W) {
    // the chunk offsets are wave-uniform: readfirstlane puts them in SGPRs (a VGPR soffset would make
    // the compiler emit a waterfall loop per load)
    const uint32_t s1 = __builtin_amdgcn_readfirstlane((uint32_t)f0 * D * 4);
    const uint32_t s2 = __builtin_amdgcn_readfirstlane((uint32_t)f0 * 4);
#pragma unroll
    for (int kq = 0; kq < T::KQ; kq += 4)
      *(f32x4*)&W.v1[kq] = buf_ld4(rW1, (uint32_t)(c * D + g * T::KQ + kq) * 4, s1);
#pragma unroll
    for (int j = 0; j < T::NJ; ++j) {
      const f32x4 v = buf_ld4(rW2, ((uint32_t)(16 * j + c) * a.FF + 4 * g) * 4, s2);
#pragma unroll
      for (int t = 0; t < 4; ++t) W.v2[j][t] = v[t];
    }
    W.b = buf_ld(rb1, (uint32_t)c * 4, s2);
  };
  auto chunk = [&](int f0, const Wc& W) {
    f32x4 pre[T::NI];
    dcontract<D>(xw, W.v1, pre, g, c);
    // fo = dropout(gelu(pre + b1)) -> staging tile [row][16]; keep bits -> mask (layout FfnTile::LW)
    uint32_t kbyte = 0;
#pragma unroll
    for (int i = 0; i < T::NI; ++i) {
      // columns (ff even, ff + 1) of a row are one RNG pair held by lanes c, c^1: each lane hashes two
      // of the block's four rows and swaps the results with its neighbour (DPP quad_perm [1,0,3,2])
      uint32_t pb[4] = {0u, 0u, 0u, 0u};
      const uint32_t odd = c & 1;
      if (a.drop.thresh) {
        const uint32_t mb = (uint32_t)(m0 + w * T::RW + 16 * i + 4 * g + 2 * odd), ffe = (uint32_t)(f0 + (c & ~1));
        const uint32_t h0 = drop_pair_bits(a.drop, (mb * (uint32_t)a.FF + ffe) >> 1);
        const uint32_t h1 = drop_pair_bits(a.drop, ((mb + 1) * (uint32_t)a.FF + ffe) >> 1);
        const uint32_t o0 = (uint32_t)__builtin_amdgcn_mov_dpp((int)h0, 0xB1, 0xF, 0xF, true);
        const uint32_t o1 = (uint32_t)__builtin_amdgcn_mov_dpp((int)h1, 0xB1, 0xF, 0xF, true);
        pb[0] = odd ? o0 : h0;
        pb[1] = odd ? o1 : h1;
        pb[2] = odd ? h0 : o0;
        pb[3] = odd ? h1 : o1;
      }
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int row = 16 * i + 4 * g + rr, m = m0 + w * T::RW + row;
        float v = gelu_f(pre[i][rr] + W.b);
        if (a.drop.thresh) {
          const bool keep = drop_pair_keep(a.drop, pb[rr], odd);
          v = keep ? v * a.drop.scale : 0.f;
          if (T::LW) {
            kbyte |= (keep ? 1u : 0u) << (4 * i + rr);
          } else {
            const unsigned long long bal = __ballot(keep);
            buf_st_u16((uint32_t)(bal >> (16 * g)), rmask,
                       (c == 0 && m < a.M) ? ((uint32_t)(f0 >> 4) * a.M + m) * 2 : BUF_OOB);
          }
        }
        st[row * T::SS + c] = v;
      }
    }
    // this wave's rows are bits 8w .. 8w+7 of the lane word: one byte store
    if (T::LW && a.drop.thresh) buf_st_u8(kbyte, rmask, lw_word(f0 >> 4, blockIdx.x, T128, g, c) * 4 + w);
    __builtin_amdgcn_wave_barrier();
    fcontract<D>(st, W.v2, yacc, g, c);
    __builtin_amdgcn_wave_barrier();
  };
  Wc wa, wb;
  load_w(0, wa);
  int f0 = 0;
  for (; f0 + 32 <= a.FF; f0 += 32) {      // sched_barrier: see the backward
    load_w(f0 + 16, wb);
    chunk(f0, wa);
    __builtin_amdgcn_sched_barrier(0);
    load_w(min(f0 + 32, a.FF - 16), wa);     // past the end: a harmless reload of the last chunk
    chunk(f0 + 16, wb);
    __builtin_amdgcn_sched_barrier(0);
  }
  if (f0 < a.FF) chunk(f0, wa);               // odd chunk count: wa holds chunk FF-16

  ffn_fwd_epilogue<D, T>(a, yacc, xw, m0 + w * T::RW);
}

// ---------------------------------------------------------------- backward
// Norm-fused loader: dh2 = RMSNorm-backward(dy; h2, r2, nw2) for the tile's rows, written as the dh
// tile (rmsnorm_bwd_small's formula: dh = w dy r - h r^3/D sum_k w_k dy_k h_k); the workgroup's
// column sums of dh2 (ffn.3.bias grad) and of dy h2 r2 (norm2.w grad) go to the slab.  `red` holds
// 2 * 256 * 4 floats of scratch.
template <int D, bool PERM = false, class T = FfnTile<D>>
__device__ void load_dh_norm2(const FfnArgs& a, int m0, float* dst, float* red, float* slab, bool acc = false) {
  constexpr int TPR = D / 4;                  // threads per row (one float4 each)
  float cb[4] = {0.f, 0.f, 0.f, 0.f}, cn[4] = {0.f, 0.f, 0.f, 0.f};
  const int c4 = (threadIdx.x % TPR) * 4;
  f32x4 w2 = *(const f32x4*)(a.nw2 + c4);
  for (int q = threadIdx.x; q < T::RT * TPR; q += 256) {
    const int i = q / TPR, m = m0 + i;
    f32x4 gy = {0.f, 0.f, 0.f, 0.f}, hv = {0.f, 0.f, 0.f, 0.f};
    float rm = 0.f;
    if (m < a.M) {
      gy = *(const f32x4*)(a.dy + (long)m * D + c4);
      hv = *(const f32x4*)(a.h2 + (long)m * D + c4);
      rm = a.r2[m];
    }
    float dot = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t) dot = fmaf(w2[t] * gy[t], hv[t], dot);
#pragma unroll
    for (int o = 1; o < TPR; o <<= 1) dot += __shfl_xor(dot, o, 64);
    const float coef = rm * rm * rm / (float)D * dot;
    f32x4 g;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      g[t] = w2[t] * gy[t] * rm - hv[t] * coef;
      cb[t] += g[t];
      cn[t] = fmaf(gy[t] * hv[t], rm, cn[t]);
    }
    put4<D, PERM>(dst + i * T::S, c4, g);
  }
  // column sums over the tile rows: threads with the same c4 hold disjoint row sets; fixed-order sum
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    red[threadIdx.x * 4 + t] = cb[t];
    red[1024 + threadIdx.x * 4 + t] = cn[t];
  }
  __syncthreads();
  if (threadIdx.x < 2 * D) {
    const int which = threadIdx.x / D, col = threadIdx.x % D;
    const int sub = col / 4 % TPR, t = col % 4;
    float sum = 0.f;
    for (int u = sub; u < 256; u += TPR) sum += red[which * 1024 + u * 4 + t];
    float* dstp = slab + (which ? a.o_n2 : a.o_b2) + col;
    *dstp = acc ? *dstp + sum : sum;
  }
  __syncthreads();
}

// dx = dact W1 (complete over FF) + dh (residual path) for this wave's RW rows (dx[i][j][rr]: row
// 16i+4g+rr, col 16j+c; dw = the wave's rows of the dh tile); NORMS: the norm1 backward.  `scratch`:
// 4*D floats of LDS no wave still reads.
template <int D, bool NORMS, bool PERM = false, class T = FfnTile<D>>
__device__ __forceinline__ void ffn_bwd_epilogue(const FfnArgs& a, const f32x4 (&dxacc)[T::NI][T::NJ],
                                                 const float* dw, int m0, float* slab, float* scratch,
                                                 bool acc = false) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, c = lane & 15;
  if (!NORMS) {
#pragma unroll
    for (int i = 0; i < T::NI; ++i)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int row = 16 * i + 4 * g + rr, m = m0 + w * T::RW + row;
        const auto rdx = buf_rsrc(a.dx, (uint32_t)a.M * D * 4);     // rows past M: dropped
#pragma unroll
        for (int j = 0; j < T::NJ; ++j) {
          const int d = 16 * j + c;
          buf_st(dxacc[i][j][rr] + dw[row * T::S + (PERM ? pcol<D>(d) : d)], rdx, (uint32_t)(m * D + d) * 4);
        }
      }
    return;
  }
  // norm-fused: dh1 = RMSNorm-backward(dx1; h1, r1, nw1) per row (a row's D values sit in the 16 lanes
  // of one lane group, NJ per lane), and this workgroup's norm1.w grad partial sum_rows dx1 h1 r1
  // h1 / r1 rows past M read 0 and their dh1 stores are dropped (buffer bounds): no branches, so all
  // the row loads are in flight together
  const auto rh1 = buf_rsrc(a.h1, (uint32_t)a.M * D * 4), rr1 = buf_rsrc(a.r1, (uint32_t)a.M * 4);
  const auto rdh1 = buf_rsrc(a.dh1, (uint32_t)a.M * D * 4);
  float nw[T::NJ], cn1[T::NJ];
#pragma unroll
  for (int j = 0; j < T::NJ; ++j) {
    nw[j] = a.nw1[16 * j + c];
    cn1[j] = 0.f;
  }
  float hv[T::NI][4][T::NJ], rmv[T::NI][4];
#pragma unroll
  for (int i = 0; i < T::NI; ++i)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int m = m0 + w * T::RW + 16 * i + 4 * g + rr;
      rmv[i][rr] = buf_ld(rr1, (uint32_t)m * 4);
#pragma unroll
      for (int j = 0; j < T::NJ; ++j) hv[i][rr][j] = buf_ld(rh1, (uint32_t)(m * D + 16 * j + c) * 4);
    }
#pragma unroll
  for (int i = 0; i < T::NI; ++i)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int row = 16 * i + 4 * g + rr, m = m0 + w * T::RW + row;
      float dx1[T::NJ];
      float dot = 0.f;
      const float rm = rmv[i][rr];
#pragma unroll
      for (int j = 0; j < T::NJ; ++j) {
        const int d = 16 * j + c;
        dx1[j] = dxacc[i][j][rr] + dw[row * T::S + (PERM ? pcol<D>(d) : d)];
        dot = fmaf(nw[j] * dx1[j], hv[i][rr][j], dot);
      }
      dot = group_sum<16>(dot);
      const float coef = rm * rm * rm / (float)D * dot;
#pragma unroll
      for (int j = 0; j < T::NJ; ++j) {
        buf_st(nw[j] * dx1[j] * rm - hv[i][rr][j] * coef, rdh1, (uint32_t)(m * D + 16 * j + c) * 4);
        cn1[j] = fmaf(dx1[j] * hv[i][rr][j], rm, cn1[j]);
      }
    }
  // sum the norm1.w partials over the lane groups, then over the waves (fixed order)
#pragma unroll
  for (int j = 0; j < T::NJ; ++j) {
    cn1[j] += __shfl_xor(cn1[j], 16, 64);
    cn1[j] += __shfl_xor(cn1[j], 32, 64);
  }
  __syncthreads();                         // the last chunk's sum has read the regions
  float* red = scratch;
  if (g == 0)
#pragma unroll
    for (int j = 0; j < T::NJ; ++j) red[w * D + 16 * j + c] = cn1[j];
  __syncthreads();
  if (tid < D) {
    const float v = ((red[tid] + red[D + tid]) + red[2 * D + tid]) + red[3 * D + tid];
    slab[a.o_n1 + tid] = acc ? slab[a.o_n1 + tid] + v : v;
  }
}

template <int D, bool NORMS>
__global__ __launch_bounds__(256) void ffn_bwd_kernel(FfnArgs a) {
  using T = FfnTile<D>;
  // [x tile | dh tile | two buffers of 4 per-wave regions]; chunk k uses buffer k & 1 for its dact
  // staging tile and then (same wave, same region) its weight-grad partial, so one barrier per chunk
  // separates the partial writes from the cross-wave sum, and the alternate buffer keeps the next
  // chunk's writes clear of a slower wave's sum.
  __shared__ __attribute__((aligned(16))) float smem[2 * T::TILE + 4 * T::NBUF * T::RG];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, c = lane & 15;
  const int m0 = blockIdx.x * T::RT;
  float* slab = a.slab + (long)blockIdx.x * a.ld_slab;
  load_tile<D>(a.x, a.M, m0, smem);
  if (NORMS) load_dh_norm2<D>(a, m0, smem + T::TILE, smem + 2 * T::TILE, slab);
  else load_tile<D>(a.dh, a.M, m0, smem + T::TILE);
  __syncthreads();
  const float* xw = smem + w * T::RW * T::S;
  const float* dw = smem + T::TILE + w * T::RW * T::S;

  f32x4 dxacc[T::NI][T::NJ];
#pragma unroll
  for (int i = 0; i < T::NI; ++i)
#pragma unroll
    for (int j = 0; j < T::NJ; ++j) dxacc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // W slices and dropout keep words of chunk f0 are prefetched one chunk ahead into the other of two
  // register sets (chunk loop unrolled by two: no copies, no early wait); buffer loads, the chunk offset
  // in an SGPR, the keep words' row bound checked by the buffer (no branches)
  constexpr int NR = 4 * T::NI;         // rows of this lane: 16 i + 4 g + rr
  const bool drop = a.drop.thresh != 0;
  const auto rW1 = buf_rsrc(a.W1, (uint32_t)a.FF * D * 4);
  const auto rW2 = buf_rsrc(a.W2, (uint32_t)a.FF * D * 4);
  const auto rb1 = buf_rsrc(a.b1, (uint32_t)a.FF * 4);
  const uint32_t mask_bytes = !drop ? 0u : T::LW ? (uint32_t)lw_words(a.M, a.FF) * 4 : (uint32_t)(a.FF / 16) * a.M * 2;
  const auto rmask = buf_rsrc(a.mask, mask_bytes);
  const uint32_t mrow = (uint32_t)(m0 + w * T::RW + 4 * g);
  const int T128 = (a.M + 127) / 128;
  struct Wc {
    float v1[T::KQ], v2[T::KQ], v3[T::NJ][4], b;
    uint32_t mk[T::LW ? 1 : NR];
  };
  auto load_w = [&](int f0, Wc& W) {
    // the chunk offsets are wave-uniform: readfirstlane puts them in SGPRs (a VGPR soffset would make
    // the compiler emit a waterfall loop per load)
    const uint32_t s1 = __builtin_amdgcn_readfirstlane((uint32_t)f0 * D * 4);
    const uint32_t s2 = __builtin_amdgcn_readfirstlane((uint32_t)f0 * 4);
#pragma unroll
    for (int kq = 0; kq < T::KQ; kq += 4)
      *(f32x4*)&W.v1[kq] = buf_ld4(rW1, (uint32_t)(c * D + g * T::KQ + kq) * 4, s1);
#pragma unroll
    for (int kk = 0; kk < T::KQ; ++kk) W.v2[kk] = buf_ld(rW2, ((uint32_t)(g * T::KQ + kk) * a.FF + c) * 4, s2);
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int j = 0; j < T::NJ; ++j) W.v3[j][t] = buf_ld(rW1, (uint32_t)((4 * g + t) * D + 16 * j + c) * 4, s1);
    W.b = buf_ld(rb1, (uint32_t)c * 4, s2);
    // rows past M read the next chunk's words (their dact and fo are 0 anyway) or, in the last chunk,
    // fall off the buffer (0)
    if (T::LW) {             // one lane word: this wave's rows at bits 8w + 4i + rr
      const uint32_t word = __builtin_bit_cast(uint32_t, buf_ld(rmask, lw_word(f0 >> 4, blockIdx.x, T128, g, c) * 4));
      W.mk[0] = word >> (8 * w);
    } else {
      const uint32_t mb = ((uint32_t)(f0 >> 4) * a.M + mrow) * 2;
#pragma unroll
      for (int q = 0; q < NR; ++q) W.mk[q] = buf_ld_u16(rmask, mb + (16 * (q >> 2) + (q & 3)) * 2);
    }
  };
  auto chunk = [&](int f0, int buf, const Wc& W) {
    float* rg = smem + 2 * T::TILE + (buf * 4 + w) * T::RG;
    f32x4 pre[T::NI], dact[T::NI];
    dcontract<D>(xw, W.v1, pre, g, c);
    dcontract<D>(dw, W.v2, dact, g, c);
    f32x4 dw2[T::NJ], dw1[T::NJ];
#pragma unroll
    for (int j = 0; j < T::NJ; ++j) dw2[j] = dw1[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    float db = 0.f;
#pragma unroll
    for (int i = 0; i < T::NI; ++i)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int row = 16 * i + 4 * g + rr, m = m0 + w * T::RW + row;
        const float z = pre[i][rr] + W.b;
        // gelu and gelu' share Phi (branch-free norm_cdf); exp on the hardware exp2
        const float cdf = norm_cdf(z);
        const float gz = z * cdf;
        const float gg = cdf + z * (__builtin_amdgcn_exp2f(-0.72134752044448170f * z * z) * 0.39894228040143268f);
        const bool keep = !drop || (T::LW ? (W.mk[0] >> (4 * i + rr)) & 1u : (W.mk[4 * i + rr] >> c) & 1u);
        const float sc = drop ? (keep ? a.drop.scale : 0.f) : 1.f;
        const float fo = (m < a.M) ? gz * sc : 0.f;
        const float da = dact[i][rr] * sc * gg;
        dact[i][rr] = da;
        db += da;
        // dW2[d][ff] += dh[row][d] fo[row][ff];  dW1[ff][d] += dact[row][ff] x[row][d]   (k-set rows {4g+rr})
#pragma unroll
        for (int j = 0; j < T::NJ; ++j) {
          dw2[j] = mfma4(dw[row * T::S + 16 * j + c], fo, dw2[j]);
          dw1[j] = mfma4(da, xw[row * T::S + 16 * j + c], dw1[j]);
        }
      }
    db += __shfl_xor(db, 16);
    db += __shfl_xor(db, 32);
    // dx += dact W1 over this chunk (stage dact as [row][16] in this wave's region)
#pragma unroll
    for (int i = 0; i < T::NI; ++i)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) rg[(16 * i + 4 * g + rr) * T::SS + c] = dact[i][rr];
    __builtin_amdgcn_wave_barrier();
    fcontract<D>(rg, W.v3, dxacc, g, c);
    __builtin_amdgcn_wave_barrier();
    // this wave's weight-grad partial over its rows -> the same region; fixed-order 4-wave sum -> slab
#pragma unroll
    for (int j = 0; j < T::NJ; ++j)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        rg[(4 * g + rr) * D + 16 * j + c] = dw1[j][rr];                 // C[ff = 4g+rr][d = 16j+c]
        rg[16 * D + (16 * j + 4 * g + rr) * 16 + c] = dw2[j][rr];       // C[d = 16j+4g+rr][ff = c]
      }
    if (g == 0) rg[32 * D + c] = db;
    __syncthreads();
    const float* red = smem + 2 * T::TILE + buf * 4 * T::RG;
    auto sum4 = [&](int q) { return ((red[q] + red[T::RG + q]) + red[2 * T::RG + q]) + red[3 * T::RG + q]; };
    static_assert((16 * D) % 256 == 0, "dW1 / dW2 partial rows split evenly over the workgroup");
#pragma unroll
    for (int it = 0; it < 16 * D / 256; ++it) {
      const int q = it * 256 + tid;
      slab[a.o_w1 + (long)f0 * D + q] = sum4(q);
    }
#pragma unroll
    for (int it = 0; it < 16 * D / 256; ++it) {
      const int u = it * 256 + tid;
      slab[a.o_w2 + (long)(u >> 4) * a.FF + f0 + (u & 15)] = sum4(16 * D + u);
    }
    if (tid < 16) slab[a.o_b1 + f0 + tid] = sum4(32 * D + tid);
    if (T::NBUF == 1) __syncthreads();     // single buffer: the sum must finish before the next staging
  };
  Wc wa, wb;
  load_w(0, wa);
  int f0 = 0;
  // sched_barrier: a set's reload stays after its chunk's last use, so the two sets keep their registers
  // across the back edge (no copies, which would wait for the in-flight prefetch)
  for (; f0 + 32 <= a.FF; f0 += 32) {
    load_w(f0 + 16, wb);
    chunk(f0, 0, wa);
    __builtin_amdgcn_sched_barrier(0);
    load_w(min(f0 + 32, a.FF - 16), wa);     // past the end: a harmless reload of the last chunk
    chunk(f0 + 16, T::NBUF == 2 ? 1 : 0, wb);
    __builtin_amdgcn_sched_barrier(0);
  }
  if (f0 < a.FF) chunk(f0, 0, wa);            // odd chunk count: wa holds chunk FF-16

  ffn_bwd_epilogue<D, NORMS>(a, dxacc, dw, m0, slab, smem + 2 * T::TILE);
}

// ---------------------------------------------------------------- backward, column-owner form
// D <= 32 with FF/16 a multiple of 4: wave w walks chunks w, w+4, w+8, ... over ALL 128 rows of the
// tile, so each chunk's dW1 / dW2 / db1 slices are complete over the tile in one wave's registers (no
// per-chunk cross-wave sum, no workgroup barrier in the chunk loop) and go straight to the slab.  The
// price is a per-wave dx accumulator over all 128 rows (its FF quarter), exchanged once at the end:
// each wave writes the three row groups it does not own, then sums its own 32 rows in the fixed order
// of the source waves -- deterministic like the rows-per-wave kernel (different summation order).
template <int D>
struct FfnCols {
  using T = FfnTile<D>;
  static_assert(T::RT == 128 && T::LW, "column-owner backward: 128-row tiles with lane-word keep bits");
  static constexpr int NB = 8;                      // 16-row blocks of the tile
  static constexpr int STG = 16 * T::SS;            // one wave's dact staging block
  static constexpr int XCH = 12 * 32 * D;           // dx exchange: (source wave, other group) slots
  static constexpr int LOAD = T::TILE + 2048;       // x tile + the norm loader's scratch
  static constexpr int MAIN = T::TILE + 4 * STG;    // x tile + staging
  static constexpr int UNION = XCH > LOAD ? (XCH > MAIN ? XCH : MAIN) : (LOAD > MAIN ? LOAD : MAIN);
};

template <int D, bool NORMS>
__global__ __launch_bounds__(256) void ffn_bwd_cols_kernel(FfnArgs a) {
  using T = FfnTile<D>;
  using C = FfnCols<D>;
  // [dh tile | union { x tile, 4 staging blocks } / { norm loader scratch } / { dx exchange }]
  __shared__ __attribute__((aligned(16))) float smem[T::TILE + C::UNION];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, c = lane & 15;
  const int m0 = blockIdx.x * T::RT;
  float* slab = a.slab + (long)blockIdx.x * a.ld_slab;
  float* dht = smem;
  float* xt = smem + T::TILE;
  load_tile<D, true>(a.x, a.M, m0, xt);
  if (NORMS) load_dh_norm2<D, true>(a, m0, dht, xt + T::TILE, slab);
  else load_tile<D, true>(a.dh, a.M, m0, dht);
  __syncthreads();
  float* st = xt + T::TILE + w * C::STG;

  f32x4 dxacc[C::NB][T::NJ];
#pragma unroll
  for (int i = 0; i < C::NB; ++i)
#pragma unroll
    for (int j = 0; j < T::NJ; ++j) dxacc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const bool drop = a.drop.thresh != 0;
  const auto rW1 = buf_rsrc(a.W1, (uint32_t)a.FF * D * 4);
  const auto rW2 = buf_rsrc(a.W2, (uint32_t)a.FF * D * 4);
  const auto rb1 = buf_rsrc(a.b1, (uint32_t)a.FF * 4);
  const auto rmask = buf_rsrc(a.mask, drop ? (uint32_t)lw_words(a.M, a.FF) * 4 : 0u);
  const int T128 = (a.M + 127) / 128;
  struct Wc {
    float v1[T::KQ], v2[T::KQ], v3[T::NJ][4], b;
    uint32_t mk;
  };
  // per-lane buffer offsets: one VGPR base per operand, everything chunk- or k-dependent is uniform
  // (SGPR soffset).  The D-contraction's k order follows the permuted tile: tile position g*KQ + q holds
  // d = 16 (q % NJ) + 4g + q / NJ.
  const uint32_t vo1 = (uint32_t)(c * D + 4 * g) * 4, vo2 = (uint32_t)(4 * g * a.FF + c) * 4;
  const uint32_t vo3 = (uint32_t)(4 * g * D + c) * 4, vob = (uint32_t)c * 4;
  auto load_w = [&](int ci, Wc& W) {
    const int f0 = 16 * ci;
    const uint32_t s1 = __builtin_amdgcn_readfirstlane((uint32_t)f0 * D * 4);
    const uint32_t s2 = __builtin_amdgcn_readfirstlane((uint32_t)f0 * 4);
#pragma unroll
    for (int j = 0; j < T::NJ; ++j) {
      const f32x4 v = buf_ld4(rW1, vo1, s1 + 64 * j);                // W1[ff][16j + 4g .. +3]
#pragma unroll
      for (int t = 0; t < 4; ++t) W.v1[t * T::NJ + j] = v[t];
    }
#pragma unroll
    for (int q = 0; q < T::KQ; ++q)
      W.v2[q] = buf_ld(rW2, vo2, s2 + (uint32_t)((16 * (q % T::NJ) + q / T::NJ) * a.FF) * 4);
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int j = 0; j < T::NJ; ++j) W.v3[j][t] = buf_ld(rW1, vo3, s1 + (uint32_t)(t * D + 16 * j) * 4);
    W.b = buf_ld(rb1, vob, s2);
    W.mk = __builtin_bit_cast(uint32_t, buf_ld(rmask, lw_word(ci, blockIdx.x, T128, g, c) * 4));
  };
  auto chunk = [&](int ci, const Wc& W) {
    const int f0 = 16 * ci;
    // the x / dh tiles are loop-invariant: without this the compiler hoists all 8 blocks' tile reads out
    // of the chunk loop and keeps them in ~200 VGPRs (one wave per SIMD)
    asm volatile("" ::: "memory");
    f32x4 dw2[T::NJ], dw1[T::NJ];
#pragma unroll
    for (int j = 0; j < T::NJ; ++j) dw2[j] = dw1[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    float db = 0.f;
#pragma unroll
    for (int i = 0; i < C::NB; ++i) {
      // pre = x W1^T and dfo = dh W2 for rows 16i.. (two interleaved chains over the D-contraction)
      f32x4 pre = {0.f, 0.f, 0.f, 0.f}, dact = {0.f, 0.f, 0.f, 0.f};
      const float* xr = xt + (16 * i + c) * T::S + g * T::KQ;
      const float* hr = dht + (16 * i + c) * T::S + g * T::KQ;
#pragma unroll
      for (int kq = 0; kq < T::KQ; kq += 4) {
        const f32x4 ax = *(const f32x4*)(xr + kq), ah = *(const f32x4*)(hr + kq);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          pre = mfma4(ax[t], W.v1[kq + t], pre);
          dact = mfma4(ah[t], W.v2[kq + t], dact);
        }
      }
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int row = 16 * i + 4 * g + rr, m = m0 + row;
        const float z = pre[rr] + W.b;
        const float cdf = norm_cdf(z);
        const float gz = z * cdf;
        const float gg = cdf + z * (__builtin_amdgcn_exp2f(-0.72134752044448170f * z * z) * 0.39894228040143268f);
        const bool keep = !drop || ((W.mk >> (4 * i + rr)) & 1u);
        const float sc = drop ? (keep ? a.drop.scale : 0.f) : 1.f;
        const float fo = (m < a.M) ? gz * sc : 0.f;
        const float da = dact[rr] * sc * gg;
        dact[rr] = da;
        db += da;
        float hd[T::NJ], xd[T::NJ];                  // columns 16j + c: adjacent in the permuted tiles
#pragma unroll
        for (int j = 0; j < T::NJ; ++j) {
          hd[j] = dht[row * T::S + c * T::NJ + j];
          xd[j] = xt[row * T::S + c * T::NJ + j];
        }
#pragma unroll
        for (int j = 0; j < T::NJ; ++j) {
          dw2[j] = mfma4(hd[j], fo, dw2[j]);
          dw1[j] = mfma4(da, xd[j], dw1[j]);
        }
      }
      // dx[rows 16i..] += dact W1 over this chunk: the dact block through this wave's staging tile
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) st[(4 * g + rr) * T::SS + c] = dact[rr];
      __builtin_amdgcn_wave_barrier();
      const f32x4 av = *(const f32x4*)(st + c * T::SS + 4 * g);
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int j = 0; j < T::NJ; ++j) dxacc[i][j] = mfma4(av[t], W.v3[j][t], dxacc[i][j]);
      __builtin_amdgcn_sched_barrier(0);      // keep the next block's tile reads from piling up registers
    }
    db += __shfl_xor(db, 16);
    db += __shfl_xor(db, 32);
    // the chunk's weight-grad slices, complete over the tile: C[ff = 4g+rr][d = 16j+c], C[d = 16j+4g+rr][ff = c]
#pragma unroll
    for (int j = 0; j < T::NJ; ++j)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        slab[a.o_w1 + (long)(f0 + 4 * g + rr) * D + 16 * j + c] = dw1[j][rr];
        slab[a.o_w2 + (long)(16 * j + 4 * g + rr) * a.FF + f0 + c] = dw2[j][rr];
      }
    if (g == 0) slab[a.o_b1 + f0 + c] = db;
  };
  // chunks w, w+4, ...: ping-pong prefetch as in the rows-per-wave kernel
  const int nk = a.FF / 64;
  for (int k = 0; k < nk; ++k) {
    Wc wa;
    load_w(w + 4 * k, wa);
    chunk(w + 4 * k, wa);
  }

  // dx exchange: slot (src, grp) for grp != src holds src's partial of group grp's 32 rows, lane-major
  __syncthreads();                                  // x tile / staging no longer read
  float* xch = xt;
  auto slot = [&](int src, int grp) { return xch + (src * 3 + (grp < src ? grp : grp - 1)) * 32 * D; };
#pragma unroll
  for (int grp = 0; grp < 4; ++grp) {
    if (grp == w) continue;
    float* dst = slot(w, grp);
#pragma unroll
    for (int ii = 0; ii < 2; ++ii)
#pragma unroll
      for (int j = 0; j < T::NJ; ++j)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) dst[((ii * T::NJ + j) * 4 + rr) * 64 + lane] = dxacc[2 * grp + ii][j][rr];
  }
  __syncthreads();
  f32x4 own[2][T::NJ], dxs[2][T::NJ];
#pragma unroll
  for (int ii = 0; ii < 2; ++ii)
#pragma unroll
    for (int j = 0; j < T::NJ; ++j) {
      own[ii][j] = dxacc[ii][j];
#pragma unroll
      for (int grp = 1; grp < 4; ++grp)
        if (grp == w) own[ii][j] = dxacc[2 * grp + ii][j];
    }
#pragma unroll
  for (int ii = 0; ii < 2; ++ii)
#pragma unroll
    for (int j = 0; j < T::NJ; ++j)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        float sum = 0.f;
#pragma unroll
        for (int src = 0; src < 4; ++src) {
          const float v = src == w ? own[ii][j][rr]
                                   : slot(src, w == src ? 0 : w)[((ii * T::NJ + j) * 4 + rr) * 64 + lane];
          sum += v;
        }
        dxs[ii][j][rr] = sum;
      }
  static_assert(T::NI == 2 && T::RW == 32, "the epilogue takes 32 rows per wave");
  ffn_bwd_epilogue<D, NORMS, true>(a, dxs, dht + w * T::RW * T::S, m0, slab, xt);
}

// ---------------------------------------------------------------- amp: bf16
// The reference under autocast(bfloat16) runs both FFN Linears as bf16 matmuls (src/train.py:158-164).
// Here every product is v_mfma_f32_16x16x32_bf16 (bf16-rounded operands, fp32 accumulation); GELU, the
// dropout, the residual and both RMSNorms stay fp32.  At bf16 MFMA rates the products cost ~1/16 of the
// fp32 form, so these kernels are bound by the element-wise GELU / dropout VALU work: it runs on packed
// fp32 pairs (v_pk_fma_f32 / v_pk_mul_f32: two elements per issue) with a 5-term erfc (cdf_as2).  The
// layouts are chosen so no product needs a transpose except the backward's dact W1:
//   * forward, pre^T = W1 x^T (A = W1 rows, B = x rows: both 8 contiguous d per lane) leaves ff on the
//     accumulator's row axis, so fo feeds y = fo W2^T as the A operand directly (k-set of lane group g:
//     ff {4g..4g+3} of the chunk's first 16 columns, then of its second 16);
//   * backward, pre = x W1^T / dfo = dh W2 leave the rows on the accumulator's row axis, so fo and dact of
//     two 16-row blocks feed the row contractions dW2^T = fo^T dh and dW1 = dact^T x directly (k-set:
//     rows {4g..4g+3} of block 0, then of block 1); dact goes through a wave-private LDS staging block
//     for dx = dact W1.
// The forward also writes the bf16 weight images the backward's operands read with one 16-byte load each
// (wbf: W1 (FF, D) | W2^T (FF, D) | W1^T (D, FF)); the weights do not change between the two.
// Keep bits (layout "row words"): word (chunk * nb16 + blk) * 16 + row16 holds bit f of 32-column chunk
// `chunk`, column f, of row 16 blk + row16 -- the forward assembles a row's word across the four lane
// groups, the backward reads the words of its rows.  The dropout decisions themselves are the fp32
// path's (drop_pair_bits of the element pair), so both modes drop the same elements.
// Backward weight grads: persistent workgroups (ctr_ffn_slab_rows: <= 512, two per CU) walk row tiles
// t = blockIdx.x, + gridDim.x, ...; per 32-column chunk the four waves' partials are summed in a fixed
// order and added into the workgroup's own slab row (first tile: stored), so the slab has one row per
// workgroup instead of one per tile -- deterministic.
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

template <int D>
struct FfnBf {
  static_assert(D == 32 || D == 64, "bf16 FFN: D in {32, 64}");
  static constexpr int RT = 128, RW = 32, NI = 2;   // rows per tile / per wave, 16-row blocks per wave
  static constexpr int KH = D / 32;                 // k steps of a D-contraction
  static constexpr int NJ = D / 16;                 // 16-col blocks of D
  static constexpr int S = D + 4;                   // fp32 tile row stride
  static constexpr int TILE = RT * S;
  static constexpr int SST = 32;                    // dact staging: [32 rows][32 cols] bf16, 16-B chunks swizzled
  static constexpr int STG = 2 * 16 * SST;          // bf16 elements per wave
  static constexpr int ES = D + 4;                  // exchange, dW1 half: [32 ff][ES] (+ 32 db1)
  static constexpr int E2S = 36;                    // exchange, dW2 half: [D][E2S]
  static constexpr int XCH = (32 * ES + 32) > (D * E2S) ? (32 * ES + 32) : (D * E2S);   // floats per wave
  // two exchange buffers (one barrier per half) while two workgroups still fit a CU's 160 KB
  static constexpr int NBUF = D <= 32 ? 2 : 1;
};

__device__ __forceinline__ f32x4 mfma_bf(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ bf16x8 pack8(f32x4 lo, f32x4 hi) {
  const bf16x4 l = __builtin_convertvector(lo, bf16x4), h = __builtin_convertvector(hi, bf16x4);
  return bf16x8{l[0], l[1], l[2], l[3], h[0], h[1], h[2], h[3]};
}
__device__ __forceinline__ bf16x8 cat8(bf16x4 lo, bf16x4 hi) {
  return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}
__device__ __forceinline__ bf16x8 buf_ld_bf8(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
  return __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
}
__device__ __forceinline__ void buf_st_u32(uint32_t v, __amdgpu_buffer_rsrc_t r, uint32_t voff) {
  __builtin_amdgcn_raw_buffer_store_b32(v, r, voff, 0, 0);
}
// workgroup barrier ordering LDS only (the exchange's global slab updates need no cross-wave order)
__device__ __forceinline__ void lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// Phi(z) and exp(-z^2/2) of two elements for the bf16 path: Abramowitz-Stegun 7.1.26 (|erf error| <=
// 1.5e-7, so Phi to 7.5e-8 absolute -- far below the 2^-9 relative rounding the bf16 product applies to
// the activation); 5 coefficients instead of norm_cdf's 9, packed, and the exponential doubles as the
// GELU derivative's pdf.
__device__ __forceinline__ f32x2 cdf_as2(f32x2 z, f32x2& e) {
  const f32x2 x = f32x2{fabsf(z.x), fabsf(z.y)} * 0.70710678118654752f;
  const f32x2 d = x * 0.3275911f + 1.0f;
  const f32x2 t = {__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
  f32x2 p = t * (0.5f * 1.061405429f) + (0.5f * -1.453152027f);
  p = p * t + (0.5f * 1.421413741f);
  p = p * t + (0.5f * -0.284496736f);
  p = p * t + (0.5f * 0.254829592f);
  const f32x2 ar = z * z * -0.72134752044448170f;
  e = f32x2{__builtin_amdgcn_exp2f(ar.x), __builtin_amdgcn_exp2f(ar.y)};
  const f32x2 h = p * t * e;
  const f32x2 q = 1.0f - h;
  return f32x2{z.x < 0.f ? h.x : q.x, z.y < 0.f ? h.y : q.y};
}

// GELU of two elements for the forward (cdf_as2's erfc fit): z Phi(z) = max(z, 0) - |z| h with
// h = erfc(|z| / sqrt 2) / 2 -- one fused multiply-add where z * (z < 0 ? h : 1 - h) took a subtract, two
// compares, two selects and a multiply; the backward recomputes its fo as z * cdf_as2(z), the same value to
// within fp32 rounding (both are rounded to bf16 for the products)
__device__ __forceinline__ f32x2 gelu_as2(f32x2 z) {
  const f32x2 az = {fabsf(z.x), fabsf(z.y)};
  const f32x2 d = az * (0.70710678118654752f * 0.3275911f) + 1.0f;
  const f32x2 t = {__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
  f32x2 p = t * (0.5f * 1.061405429f) + (0.5f * -1.453152027f);
  p = p * t + (0.5f * 1.421413741f);
  p = p * t + (0.5f * -0.284496736f);
  p = p * t + (0.5f * 0.254829592f);
  const f32x2 ar = z * z * -0.72134752044448170f;
  const f32x2 e = {__builtin_amdgcn_exp2f(ar.x), __builtin_amdgcn_exp2f(ar.y)};
  const f32x2 h = p * t * e;
  return __builtin_elementwise_fma(-az, h, f32x2{fmaxf(z.x, 0.f), fmaxf(z.y, 0.f)});
}

// rows [m0, m0 + RT) of a (M, D) matrix -> fp32 LDS tile, row stride D + 4 (zero rows past M)
template <int D, int RT>
__device__ __forceinline__ void load_rows(const float* __restrict__ src, int M, int m0, float* dst) {
  for (int q = threadIdx.x; q < RT * D / 4; q += 256) {
    const int i = q / (D / 4), c4 = (q % (D / 4)) * 4;
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (m0 + i < M) v = *(const f32x4*)(src + (long)(m0 + i) * D + c4);
    *(f32x4*)(dst + i * (D + 4) + c4) = v;
  }
}

__device__ __forceinline__ uint32_t rw_word(int chunk, int nb16, int blk, int row16) {
  return ((uint32_t)(chunk * nb16 + blk) * 16 + row16);
}

template <int D, bool DROP>
__global__ __launch_bounds__(256) void ffn_fwd_bf_kernel(FfnArgs a) {
  using T = FfnBf<D>;
  __shared__ __attribute__((aligned(16))) float xt[T::TILE];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, c = lane & 15;
  const int m0 = blockIdx.x * T::RT, rb = w * T::RW;
  // bf16 weight images for the backward: W1 (FF, D) | W2^T (FF, D) | W1^T (D, FF)
  if (a.wbf) {
    const int n = a.FF * D;
    for (int e = blockIdx.x * 256 + tid; e < 3 * n; e += gridDim.x * 256) {
      float v;
      if (e < n) {
        v = a.W1[e];
      } else if (e < 2 * n) {
        const int q = e - n;
        v = a.W2[(q % D) * a.FF + q / D];
      } else {
        const int q = e - 2 * n;
        v = a.W1[(q % a.FF) * D + q / a.FF];
      }
      a.wbf[e] = (__bf16)v;
    }
  }
  load_rows<D, T::RT>(a.x, a.M, m0, xt);
  __syncthreads();
  const float* xw = xt + rb * T::S;
  // B operand of pre^T = W1 x^T: x[row 16i + c][32kh + 8g .. +7]
  bf16x8 xf[T::NI][T::KH];
#pragma unroll
  for (int i = 0; i < T::NI; ++i)
#pragma unroll
    for (int kh = 0; kh < T::KH; ++kh) {
      const float* p = xw + (16 * i + c) * T::S + 32 * kh + 8 * g;
      xf[i][kh] = pack8(*(const f32x4*)p, *(const f32x4*)(p + 4));
    }
  f32x4 yacc[T::NI][T::NJ];
#pragma unroll
  for (int i = 0; i < T::NI; ++i)
#pragma unroll
    for (int j = 0; j < T::NJ; ++j) yacc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nb16 = (a.M + 15) / 16;
  const auto rW1 = buf_rsrc(a.W1, (uint32_t)a.FF * D * 4);
  const auto rW2 = buf_rsrc(a.W2, (uint32_t)a.FF * D * 4);
  const auto rb1 = buf_rsrc(a.b1, (uint32_t)a.FF * 4);
  const auto rmask = buf_rsrc(a.mask, DROP ? (uint32_t)nb16 * 16 * (a.FF / 32) * 4 : 0u);
  const uint32_t thr = a.drop.thresh;
  const float dsc = a.drop.scale;
  struct Wc {
    bf16x8 w1[2][T::KH], w2[T::NJ];
    f32x4 b[2];
  };
  auto load_w = [&](int f0, Wc& W) {
    const uint32_t s1 = __builtin_amdgcn_readfirstlane((uint32_t)f0 * D * 4);
    const uint32_t s2 = __builtin_amdgcn_readfirstlane((uint32_t)f0 * 4);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int kh = 0; kh < T::KH; ++kh) {      // A of pre^T: W1[f0 + 16s + c][32kh + 8g .. +7]
        const uint32_t vo = (uint32_t)((16 * s + c) * D + 32 * kh + 8 * g) * 4;
        W.w1[s][kh] = pack8(buf_ld4(rW1, vo, s1), buf_ld4(rW1, vo + 16, s1));
      }
#pragma unroll
    for (int j = 0; j < T::NJ; ++j) {          // B of y: W2[16j + c][f0 + 4g .. +3], [f0 + 16 + 4g .. +3]
      const uint32_t vo = (uint32_t)((16 * j + c) * a.FF + 4 * g) * 4;
      W.w2[j] = pack8(buf_ld4(rW2, vo, s2), buf_ld4(rW2, vo + 64, s2));
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) W.b[s] = buf_ld4(rb1, (uint32_t)(16 * s + 4 * g) * 4, s2);
  };
  auto chunk = [&](int f0, const Wc& W) {
    // all of the chunk's pre^T products first: the element-wise work of block 0 covers their latency
    f32x4 p[T::NI][2];
#pragma unroll
    for (int i = 0; i < T::NI; ++i)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        p[i][s] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kh = 0; kh < T::KH; ++kh) p[i][s] = mfma_bf(W.w1[s][kh], xf[i][kh], p[i][s]);
      }
#pragma unroll
    for (int i = 0; i < T::NI; ++i) {
      // p[i][s][r] = pre[row 16i + c][ff f0 + 16s + 4g + r]; elements (r = 0,1), (2,3) share a hash
      const uint32_t m = (uint32_t)(m0 + rb + 16 * i + c);
      uint32_t kb = 0;              // keep bit of element (s, r) at 4s + r
      f32x4 fo[2];
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const f32x2 z = {p[i][s][2 * q] + W.b[s][2 * q], p[i][s][2 * q + 1] + W.b[s][2 * q + 1]};
          f32x2 e;
          f32x2 v = z * cdf_as2(z, e);
          if (DROP) {
            const uint32_t hb = drop_pair_bits(a.drop, (m * (uint32_t)a.FF + f0 + 16 * s + 4 * g + 2 * q) >> 1);
            const bool k0 = (hb & 0xFFFFu) >= thr, k1 = (hb >> 16) >= thr;
            v = v * f32x2{k0 ? dsc : 0.f, k1 ? dsc : 0.f};
            kb |= (k0 ? 1u : 0u) << (4 * s + 2 * q);
            kb |= (k1 ? 1u : 0u) << (4 * s + 2 * q + 1);
          }
          fo[s][2 * q] = v.x;
          fo[s][2 * q + 1] = v.y;
        }
      const bf16x8 af = pack8(fo[0], fo[1]);
#pragma unroll
      for (int j = 0; j < T::NJ; ++j) yacc[i][j] = mfma_bf(af, W.w2[j], yacc[i][j]);
      if (DROP) {     // the row's word: bits 4g .. 4g+3 and 16+4g .. +3 from each lane group, stored by group 0
        uint32_t kw = ((kb & 0xFu) << (4 * g)) | ((kb >> 4) << (16 + 4 * g));
        kw |= (uint32_t)__shfl_xor((int)kw, 16, 64);
        kw |= (uint32_t)__shfl_xor((int)kw, 32, 64);
        const uint32_t wi = rw_word(f0 >> 5, nb16, (m0 + rb) / 16 + i, c);
        buf_st_u32(kw, rmask, (g == 0 && (int)m < a.M) ? wi * 4 : BUF_OOB);
      }
    }
  };
  Wc wa, wb;
  load_w(0, wa);
  int f0 = 0;
  for (; f0 + 64 <= a.FF; f0 += 64) {
    load_w(f0 + 32, wb);
    chunk(f0, wa);
    __builtin_amdgcn_sched_barrier(0);
    load_w(min(f0 + 64, a.FF - 32), wa);     // past the end: a harmless reload of the last chunk
    chunk(f0 + 32, wb);
    __builtin_amdgcn_sched_barrier(0);
  }
  if (f0 < a.FF) chunk(f0, wa);
  ffn_fwd_epilogue<D, T>(a, yacc, xw, m0 + rb);
}

// Wave-independent forward (D = 32, round 5): no x tile in LDS and no barrier after the weight staging, so a
// workgroup's eight waves run free of each other and two workgroups (51 KB of weight images each) fit a CU at four
// waves per SIMD (<= 128 registers).  A wave owns 32-row tiles t = wave, + total waves, ...; its x rows are read
// straight into registers in the k order the products use -- lane (g, c) holds x[row 16 i + c][4g .. 4g+3] and
// [16 + 4g .. 16 + 4g+3] -- which is both the B operand of pre^T = W1 x^T (the staged W1 image carries the same d
// order) and, because the output is formed TRANSPOSED (y^T = W2 fo^T: A = the W2 image, B = fo straight from the
// pre^T accumulators), exactly the fp32 residual the epilogue adds to lane (g, c)'s outputs y[row 16 i + c][16 j +
// 4g + r]: a row's 32 outputs sit in its four lane groups, the RMSNorm sum takes two lane swaps, h and y go out as
// 16-byte stores of whole rows.  The next tile's rows are loaded while the current one computes.  Keep bits, their
// "row words" layout, the weight images for the backward: as the per-tile kernels.
// D = 64 (round 5): the same with 16-row tiles (NI = 1; 99 KB of weight images) and one workgroup of sixteen waves
// per CU (four per SIMD); the d order of step kh of a D-contraction is {32 kh + 4g .. +3} u {32 kh + 16 + 4g .. +3}.
template <int D_>
struct FfnFw {
  static constexpr int D = D_, NI = D == 32 ? 2 : 1, RW = 16 * NI, NWAVE = D == 32 ? 8 : 16;
  static constexpr int KH = D / 32, NJ = D / 16;
};

template <int D, bool DROP>
__global__ __launch_bounds__(FfnFw<D>::NWAVE * 64) __attribute__((amdgpu_waves_per_eu(4))) void ffn_fwd_bfw_kernel(
    FfnArgs a) {
  using T = FfnFw<D>;
  constexpr int NI = T::NI, KH = T::KH, NJ = T::NJ, NT = T::NWAVE * 64;
  extern __shared__ __attribute__((aligned(16))) char fsm[];
  const int FF = a.FF, NCH = FF / 32;
  bf16x8* iw1 = (bf16x8*)fsm;                 // [NCH][2][KH][64]: W1[32 ch + 16 s + c][32 kh + 4g .. +3 | 32 kh + 16 + 4g ..]
  bf16x8* iw2 = iw1 + NCH * 2 * KH * 64;      // [NCH][NJ][64]: W2[16 j + c][32 ch + 4g .. +3 | 32 ch + 16 + 4g ..]
  float* sb1 = (float*)(iw2 + NCH * NJ * 64);  // [FF]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, c = lane & 15;
  if (a.wbf) {     // bf16 weight images for the backward: W1 (FF, D) | W2^T (FF, D) | W1^T (D, FF)
    const int n = FF * D;
    for (int e = blockIdx.x * NT + tid; e < 3 * n; e += gridDim.x * NT) {
      float v;
      if (e < n) {
        v = a.W1[e];
      } else if (e < 2 * n) {
        const int q = e - n;
        v = a.W2[(q % D) * FF + q / D];
      } else {
        const int q = e - 2 * n;
        v = a.W1[(q % FF) * D + q / FF];
      }
      a.wbf[e] = (__bf16)v;
    }
  }
  for (int u = tid; u < NCH * 2 * KH * 64; u += NT) {
    const int l = u & 63, q = u >> 6, kh = q % KH, sc = q / KH, s2 = sc & 1, ch = sc >> 1, lg = l >> 4;
    const float* p = a.W1 + (long)(32 * ch + 16 * s2 + (l & 15)) * D + 32 * kh + 4 * lg;
    iw1[u] = pack8(*(const f32x4*)p, *(const f32x4*)(p + 16));
  }
  for (int u = tid; u < NCH * NJ * 64; u += NT) {
    const int l = u & 63, q = u >> 6, j = q % NJ, ch = q / NJ;
    const float* p = a.W2 + (long)(16 * j + (l & 15)) * FF + 32 * ch + 4 * (l >> 4);
    iw2[u] = pack8(*(const f32x4*)p, *(const f32x4*)(p + 16));
  }
  for (int u = tid; u < FF; u += NT) sb1[u] = a.b1[u];
  __syncthreads();

  const int nb16 = (a.M + 15) / 16;
  const auto rmask = buf_rsrc(a.mask, DROP ? (uint32_t)nb16 * 16 * (FF / 32) * 4 : 0u);
  const uint32_t xbytes = (uint32_t)a.M * D * 4;
  const auto rx = buf_rsrc(a.x, xbytes);
  const auto rh = buf_rsrc(a.h, xbytes);
  const auto ry = buf_rsrc(a.y, xbytes);
  const auto rr = buf_rsrc(a.r, (uint32_t)a.M * 4);
  const uint32_t thr = a.drop.thresh;
  const float dsc = a.drop.scale;
  // x rows of a tile: xr[i][j] = x[m0 + 16 i + c][16 j + 4g .. +3] (0 past M)
  f32x4 xr[NI][NJ];
  auto fetch_x = [&](int t) {
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        xr[i][j] = buf_ld4(rx, (uint32_t)(((t * T::RW + 16 * i + c) * D) + 16 * j + 4 * g) * 4, 0);
  };
  struct Wc {
    bf16x8 w1[2][KH], w2[NJ];
    f32x4 b[2];
  };
  auto load_w = [&](int ch, Wc& W) {
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
#pragma unroll
      for (int kh = 0; kh < KH; ++kh) W.w1[s2][kh] = iw1[((ch * 2 + s2) * KH + kh) * 64 + lane];
      W.b[s2] = *(const f32x4*)(sb1 + 32 * ch + 16 * s2 + 4 * g);
    }
#pragma unroll
    for (int j = 0; j < NJ; ++j) W.w2[j] = iw2[(ch * NJ + j) * 64 + lane];
  };
  const int ntiles = (a.M + T::RW - 1) / T::RW;
  const int gw = blockIdx.x * T::NWAVE + w, nw = gridDim.x * T::NWAVE;
  if (gw < ntiles) fetch_x(gw);
  for (int tile = gw; tile < ntiles; tile += nw) {
    const int m0 = tile * T::RW;
    bf16x8 xf[NI][KH];
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int kh = 0; kh < KH; ++kh) xf[i][kh] = pack8(xr[i][2 * kh], xr[i][2 * kh + 1]);
    if (tile + nw < ntiles) fetch_x(tile + nw);
    f32x4 yacc[NI][NJ];
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) yacc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int ch = 0; ch < NCH; ++ch) {
      Wc W;
      load_w(ch, W);
      const int f0 = 32 * ch;
      f32x4 p[NI][2];
#pragma unroll
      for (int i = 0; i < NI; ++i)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          p[i][s2] = mfma_bf(W.w1[s2][0], xf[i][0], W.b[s2]);                            // pre^T [ff][row], + b1
#pragma unroll
          for (int kh = 1; kh < KH; ++kh) p[i][s2] = mfma_bf(W.w1[s2][kh], xf[i][kh], p[i][s2]);
        }
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        const uint32_t m = (uint32_t)(m0 + 16 * i + c);
        uint32_t kb = 0;
        f32x4 fo[2];
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            const f32x2 z = {p[i][s2][2 * q], p[i][s2][2 * q + 1]};
            f32x2 v = gelu_as2(z);
            if (DROP) {
              const uint32_t hb = drop_pair_bits(a.drop, (m * (uint32_t)FF + f0 + 16 * s2 + 4 * g + 2 * q) >> 1);
              const bool k0 = (hb & 0xFFFFu) >= thr, k1 = (hb >> 16) >= thr;
              v = v * f32x2{k0 ? dsc : 0.f, k1 ? dsc : 0.f};
              kb |= (k0 ? 1u : 0u) << (4 * s2 + 2 * q);
              kb |= (k1 ? 1u : 0u) << (4 * s2 + 2 * q + 1);
            }
            fo[s2][2 * q] = v.x;
            fo[s2][2 * q + 1] = v.y;
          }
        const bf16x8 bf = pack8(fo[0], fo[1]);
#pragma unroll
        for (int j = 0; j < NJ; ++j) yacc[i][j] = mfma_bf(W.w2[j], bf, yacc[i][j]);         // y^T [d][row]
        if (DROP) {
          uint32_t kw = ((kb & 0xFu) << (4 * g)) | ((kb >> 4) << (16 + 4 * g));
          kw |= (uint32_t)__shfl_xor((int)kw, 16, 64);
          kw |= (uint32_t)__shfl_xor((int)kw, 32, 64);
          const uint32_t wi = rw_word(ch, nb16, m0 / 16 + i, c);
          buf_st_u32(kw, rmask, (g == 0 && (int)m < a.M) ? wi * 4 : BUF_OOB);
        }
      }
    }
    // epilogue: h = x + (y + b2), r = 1 / rms(h), y = nw h r -- row 16 i + c over the four lane groups; the x rows
    // (this wave's own, read at the tile's start) are read again rather than held across the chunk loop
    f32x4 xc[NI][NJ], bb[NJ], nn[NJ];
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        xc[i][j] = buf_ld4(rx, (uint32_t)(((m0 + 16 * i + c) * D) + 16 * j + 4 * g) * 4, 0);
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      bb[j] = *(const f32x4*)(a.b2 + 16 * j + 4 * g);
      nn[j] = *(const f32x4*)(a.nw + 16 * j + 4 * g);
    }
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      f32x4 hv[NJ];
      float ss = 0.f;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        hv[j] = xc[i][j] + (yacc[i][j] + bb[j]);
#pragma unroll
        for (int r = 0; r < 4; ++r) ss = fmaf(hv[j][r], hv[j][r], ss);
      }
      ss += __shfl_xor(ss, 16, 64);
      ss += __shfl_xor(ss, 32, 64);
      const float rs = 1.0f / sqrtf(ss / (float)D + a.eps);
      const uint32_t row = (uint32_t)(m0 + 16 * i + c);
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const uint32_t off = (row * D + 16 * j + 4 * g) * 4;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, hv[j]), rh, off, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, nn[j] * hv[j] * rs), ry, off, 0, 0);
      }
      buf_st(rs, rr, g == 0 ? row * 4 : BUF_OOB);
    }
  }
}

template <int D>
static size_t ffn_fwdw_lds(int FF) { return (size_t)FF * D * 2 * 2 + (size_t)FF * 4; }

// Backward tile: D = 32 takes 128-row tiles (32 rows per wave), D = 64 64-row tiles (16 per wave) so two
// workgroups fit a CU's LDS.  Per 32-column chunk every wave writes its fo / dact rows as bf16 [ff][rows]
// images; after one barrier each wave reads its dact rows back transposed (ds_read_b64_tr_b16) for
// dx = dact W1 and computes its share of the chunk's weight-grad tiles over ALL the tile's rows (K = RT)
// from the images and the tile's x^T / dh^T images -- complete tiles, no cross-wave partial sums -- and
// adds them into the workgroup's slab row.  The images alternate between two buffers: one barrier a chunk.
template <int D>
struct FfnBb {
  static_assert(D == 32 || D == 64, "bf16 FFN: D in {32, 64}");
  static constexpr int RT = D <= 32 ? 128 : 64;
  static constexpr int RW = RT / 4, NI = RW / 16;
  static constexpr int KH = D / 32, NJ = D / 16;
  static constexpr int S = D + 4;                   // fp32 tile row stride
  static constexpr int TILE = RT * S;
  static constexpr int RS = RT + 8;                 // bf16 image row stride (rows of a [col][row] image)
  static constexpr int IMG = 32 * RS;               // one [32 ff][RT] image, bf16 elements
  static constexpr int CIMG = D * RS;               // one [D][RT] image, bf16 elements
  static constexpr int NT = 2 * NJ / 4;             // dW1 (and dW2^T) 16x16 tiles per wave and chunk
  // the fo / dact image buffers (2 x 2 images) share their LDS with the x tile + the norm loader scratch
  static constexpr int RREG = 2 * IMG > TILE + 2048 ? 2 * IMG : TILE + 2048;   // floats
};

typedef short s16x4 __attribute__((ext_vector_type(4)));
// 4 rows x 16 columns of 16-bit elements, delivered transposed (MI355X ds_read_b64_tr_b16): lane 4q + p of
// each 16-lane group addresses row q, columns 4p .. 4p+3; lane i receives column i, row q in element q
__device__ __forceinline__ bf16x4 lds_tr4(const __bf16* p) {
  return __builtin_bit_cast(bf16x4, __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)p));
}

template <int D, bool NORMS, bool DROP>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void ffn_bwd_bf_kernel(FfnArgs a) {
  using T = FfnBb<D>;
  // [H: dh tile (fp32; residual / norm1 epilogue) | R: x tile + loader scratch, then 2 x {fo, dact} images |
  //  XC, HC: x^T and dh^T images of the tile (bf16)]
  __shared__ __attribute__((aligned(16))) float smem[T::TILE + T::RREG + T::CIMG];
  float* H = smem;
  float* X = smem + T::TILE;
  __bf16* IM = (__bf16*)X;
  __bf16* XC = (__bf16*)(smem + T::TILE + T::RREG);
  __bf16* HC = XC + T::CIMG;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, c = lane & 15;
  const int rb = w * T::RW;
  float* slab = a.slab + (long)blockIdx.x * a.ld_slab;
  const int nb16 = (a.M + 15) / 16;
  const int ntiles = (a.M + T::RT - 1) / T::RT;
  const int FF = a.FF;
  const auto rw = buf_rsrc(a.wbf, (uint32_t)(3 * FF * D) * 2);
  const auto rb1 = buf_rsrc(a.b1, (uint32_t)FF * 4);
  const auto rmask = buf_rsrc(a.mask, DROP ? (uint32_t)nb16 * 16 * (FF / 32) * 4 : 0u);
  const float dsc = a.drop.scale;
  const uint32_t vw1 = (uint32_t)(c * D + 8 * g) * 2;          // W1 / W2^T rows f0 + c (+16s), d 8g..
  const uint32_t vw1t = (uint32_t)(c * FF + 8 * g) * 2;         // W1^T rows d = c (+16j), ff f0 + 8g..
  // this wave's weight-grad tiles of each chunk: (s, j) for j in js0 .. js0 + NT - 1; db1 with the j = 0 tile
  const int ts = w >> 1, js0 = (w & 1) * T::NT;
  const bool has_db = js0 == 0;
  bf16x8 ones;
#pragma unroll
  for (int e = 0; e < 8; ++e) ones[e] = (__bf16)1.0f;
  struct Wc {
    bf16x8 w1[2][T::KH], w2[2][T::KH];
    float b[2];
    uint32_t mk[T::NI][4];
  };

  for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const bool acc = t != (int)blockIdx.x;      // later tiles add into the workgroup's slab row
    const int m0 = t * T::RT;
    const int blk0 = (m0 + rb) / 16;
    __syncthreads();                            // the previous tile is done with every region
    load_rows<D, T::RT>(a.x, a.M, m0, X);
    if (NORMS) load_dh_norm2<D, false, T>(a, m0, H, X + T::TILE, slab, acc);
    else load_rows<D, T::RT>(a.dh, a.M, m0, H);
    __syncthreads();
    // row fragments (A of pre / dfo: 8 contiguous d of row 16i + c) and the x^T / dh^T images
    bf16x8 xr[T::NI][T::KH], hr[T::NI][T::KH];
#pragma unroll
    for (int i = 0; i < T::NI; ++i)
#pragma unroll
      for (int kh = 0; kh < T::KH; ++kh) {
        const int o = (rb + 16 * i + c) * T::S + 32 * kh + 8 * g;
        xr[i][kh] = pack8(*(const f32x4*)(X + o), *(const f32x4*)(X + o + 4));
        hr[i][kh] = pack8(*(const f32x4*)(H + o), *(const f32x4*)(H + o + 4));
      }
    for (int q = tid; q < T::RT * D / 4; q += 256) {
      const int row = q % T::RT, d4 = (q / T::RT) * 4;
      const f32x4 vx = *(const f32x4*)(X + row * T::S + d4), vh = *(const f32x4*)(H + row * T::S + d4);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        XC[(d4 + k) * T::RS + row] = (__bf16)vx[k];
        HC[(d4 + k) * T::RS + row] = (__bf16)vh[k];
      }
    }
    __syncthreads();                            // X becomes the image buffers

    f32x4 dxacc[T::NI][T::NJ];
#pragma unroll
    for (int i = 0; i < T::NI; ++i)
#pragma unroll
      for (int j = 0; j < T::NJ; ++j) dxacc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    auto load_w = [&](int f0, Wc& W) {
      const uint32_t s1 = __builtin_amdgcn_readfirstlane((uint32_t)f0 * D * 2);
      const uint32_t s2 = __builtin_amdgcn_readfirstlane((uint32_t)(FF * D + f0 * D) * 2);
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int kh = 0; kh < T::KH; ++kh) {
          // B of pre: W1[f0 + 16s + c][32kh + 8g .. +7];  B of dfo: W2^T[f0 + 16s + c][32kh + 8g .. +7]
          const uint32_t vo = vw1 + (uint32_t)(16 * s * D + 32 * kh) * 2;
          W.w1[s][kh] = buf_ld_bf8(rw, vo, s1);
          W.w2[s][kh] = buf_ld_bf8(rw, vo, s2);
        }
      const uint32_t sb = __builtin_amdgcn_readfirstlane((uint32_t)f0 * 4);
#pragma unroll
      for (int s = 0; s < 2; ++s) W.b[s] = buf_ld(rb1, (uint32_t)(16 * s + c) * 4, sb);
      if (DROP) {
        // keep words of rows 16i + 4g + r, pre-shifted to this lane's column; rows past M read 0 (their dh
        // is 0 anyway)
        const uint32_t sm = __builtin_amdgcn_readfirstlane((uint32_t)(f0 >> 5) * nb16 * 16 * 4);
#pragma unroll
        for (int i = 0; i < T::NI; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            W.mk[i][r] = __builtin_bit_cast(uint32_t, buf_ld(rmask, (uint32_t)((blk0 + i) * 16 + 4 * g + r) * 4, sm)) >> c;
      }
    };

    // slab entries this lane owns in a chunk (fixed over tiles, so a later tile's read-modify-write sees
    // this lane's own earlier store): dW1 rows f0 + 16 ts + 4g + r, column 16j + c; dW2 row 16j + c,
    // columns f0 + 16 ts + 4g + r; db1 f0 + 16 ts + 4g + r (lanes c = 0 of the db owners)
    auto p_w1 = [&](int f0, int jj, int r) { return slab + a.o_w1 + (long)(f0 + 16 * ts + 4 * g + r) * D + 16 * (js0 + jj) + c; };
    auto p_w2 = [&](int f0, int jj, int r) { return slab + a.o_w2 + (long)(16 * (js0 + jj) + c) * FF + f0 + 16 * ts + 4 * g + r; };
    auto p_b1 = [&](int f0, int r) { return slab + a.o_b1 + f0 + 16 * ts + 4 * g + r; };

    // the slab values a chunk's tiles add to (later tiles only); loaded one chunk ahead, so a chunk's wait
    // for them does not also wait for the previous chunk's slab stores (loads and stores retire in order)
    struct Os {
      float o1[T::NT][4], o2[T::NT][4], ob[4];
    };
    auto load_o = [&](int f0, Os& O) {
#pragma unroll
      for (int jj = 0; jj < T::NT; ++jj)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          O.o1[jj][r] = acc ? *p_w1(f0, jj, r) : 0.f;
          O.o2[jj][r] = acc ? *p_w2(f0, jj, r) : 0.f;
        }
#pragma unroll
      for (int r = 0; r < 4; ++r) O.ob[r] = (acc && has_db && c == 0) ? *p_b1(f0, r) : 0.f;
    };

    auto chunk = [&](int f0, int bsel, const Wc& W, const Os& O, Os& On, int fn) {
      __bf16* FO = IM + bsel * 2 * T::IMG;
      __bf16* DA = FO + T::IMG;
      // B of dx: W1^T[16j + c][f0 + 8g .. +7] (first used after the element-wise work)
      bf16x8 w1d[T::NJ];
      const uint32_t s3 = __builtin_amdgcn_readfirstlane((uint32_t)(2 * FF * D + f0) * 2);
#pragma unroll
      for (int j = 0; j < T::NJ; ++j) w1d[j] = buf_ld_bf8(rw, vw1t + (uint32_t)(16 * j * FF) * 2, s3);
      if (fn >= 0) load_o(fn, On);
      // the chunk's D-contractions (their latency under the element-wise work)
      f32x4 pre[T::NI][2], dfo[T::NI][2];
#pragma unroll
      for (int i = 0; i < T::NI; ++i)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          pre[i][s] = dfo[i][s] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int kh = 0; kh < T::KH; ++kh) {
            pre[i][s] = mfma_bf(xr[i][kh], W.w1[s][kh], pre[i][s]);
            dfo[i][s] = mfma_bf(hr[i][kh], W.w2[s][kh], dfo[i][s]);
          }
        }
#pragma unroll
      for (int i = 0; i < T::NI; ++i)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          // pre[i][s][r], dfo[i][s][r]: row rb + 16i + 4g + r, column f0 + 16s + c
          f32x4 fv, dv;
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            const f32x2 z = f32x2{pre[i][s][2 * q], pre[i][s][2 * q + 1]} + W.b[s];
            f32x2 e;
            const f32x2 cdf = cdf_as2(z, e);
            const f32x2 gg = z * e * 0.39894228040143268f + cdf;
            f32x2 sc = {1.f, 1.f};
            if (DROP)
              sc = f32x2{((W.mk[i][2 * q] >> (16 * s)) & 1u) ? dsc : 0.f, ((W.mk[i][2 * q + 1] >> (16 * s)) & 1u) ? dsc : 0.f};
            const f32x2 fo = z * cdf * sc;
            const f32x2 da = f32x2{dfo[i][s][2 * q], dfo[i][s][2 * q + 1]} * sc * gg;
            fv[2 * q] = fo.x;
            fv[2 * q + 1] = fo.y;
            dv[2 * q] = da.x;
            dv[2 * q + 1] = da.y;
          }
          // the [ff][rows] images: 4 consecutive rows of column 16s + c
          const int o = (16 * s + c) * T::RS + rb + 16 * i + 4 * g;
          *(bf16x4*)(FO + o) = __builtin_convertvector(fv, bf16x4);
          *(bf16x4*)(DA + o) = __builtin_convertvector(dv, bf16x4);
        }
      lds_sync();
      // dx[rows 16i..] += dact W1 over the chunk: A = dact[row 16i + c][ff 8g .. +7], transposed reads
#pragma unroll
      for (int i = 0; i < T::NI; ++i) {
        const __bf16* base = DA + (8 * g + (lane & 15) / 4) * T::RS + rb + 16 * i + 4 * (lane & 3);
        const bf16x8 av = cat8(lds_tr4(base), lds_tr4(base + 4 * T::RS));
#pragma unroll
        for (int j = 0; j < T::NJ; ++j) dxacc[i][j] = mfma_bf(av, w1d[j], dxacc[i][j]);
      }
      // this wave's weight-grad tiles over the tile's RT rows (C[ff 16 ts + 4g + r][d 16j + c])
      f32x4 t1[T::NT], t2[T::NT], tb = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int jj = 0; jj < T::NT; ++jj) t1[jj] = t2[jj] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < T::RT / 32; ++kk) {
        const bf16x8 ad = *(const bf16x8*)(DA + (16 * ts + c) * T::RS + 32 * kk + 8 * g);
        const bf16x8 af = *(const bf16x8*)(FO + (16 * ts + c) * T::RS + 32 * kk + 8 * g);
#pragma unroll
        for (int jj = 0; jj < T::NT; ++jj) {
          const int o = (16 * (js0 + jj) + c) * T::RS + 32 * kk + 8 * g;
          t1[jj] = mfma_bf(ad, *(const bf16x8*)(XC + o), t1[jj]);
          t2[jj] = mfma_bf(af, *(const bf16x8*)(HC + o), t2[jj]);
        }
        if (has_db) tb = mfma_bf(ad, ones, tb);
      }
#pragma unroll
      for (int jj = 0; jj < T::NT; ++jj)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          *p_w1(f0, jj, r) = O.o1[jj][r] + t1[jj][r];
          *p_w2(f0, jj, r) = O.o2[jj][r] + t2[jj][r];
        }
      if (has_db && c == 0)
#pragma unroll
        for (int r = 0; r < 4; ++r) *p_b1(f0, r) = O.ob[r] + tb[r];
    };

    Os oa, ob;
    load_o(0, oa);
    if constexpr (D <= 32) {     // weights of the next chunk prefetched into the other register set
      Wc wa, wb;
      load_w(0, wa);
      int f0 = 0;
      for (; f0 + 64 <= FF; f0 += 64) {
        load_w(f0 + 32, wb);
        chunk(f0, 0, wa, oa, ob, f0 + 32);
        __builtin_amdgcn_sched_barrier(0);
        load_w(min(f0 + 64, FF - 32), wa);
        chunk(f0 + 32, 1, wb, ob, oa, f0 + 64 < FF ? f0 + 64 : -1);
        __builtin_amdgcn_sched_barrier(0);
      }
      if (f0 < FF) chunk(f0, 0, wa, oa, ob, -1);
    } else {
      for (int f0 = 0; f0 < FF; f0 += 32) {     // D = 64: no register room for a second slab set
        Wc wa;
        load_w(f0, wa);
        if (f0 > 0) load_o(f0, oa);
        chunk(f0, (f0 >> 5) & 1, wa, oa, ob, -1);
      }
    }
    ffn_bwd_epilogue<D, NORMS, false, T>(a, dxacc, H + rb * T::S, m0, slab, X, acc);
  }
}

// ---------------------------------------------------------------- amp: bf16, column-owner persistent backward
// One 512-thread workgroup per CU walks a contiguous range of 32-row steps.  Wave w OWNS the FF columns
// [16 NT w, 16 NT (w + 1)) (FF = 128 NT) for the whole launch: its dW1 / dW2 / db1 slices are complete over
// every row the workgroup visits in that wave's registers and are written ONCE, at the end, to the
// workgroup's slab row (no per-tile slab read-modify-write), and its weight operands stay in registers.
// The price is the dx = dact W1 contraction over FF, split over the eight waves: each writes its partial
// for the step's 32 rows to an LDS exchange slot and, after the step's single barrier, every wave sums
// the eight partials of its own four rows in a fixed order (deterministic) and runs the norm1 backward.
// Per step a wave loads / prepares four rows of the NEXT step (norm2 backward of dy, bf16 images of x and
// dh, keep words) while the current step's images are read: images triple-buffered, exchange double-
// buffered, so one barrier per step orders everything.
// Products (v_mfma_f32_16x16x32_bf16; the odd tile of the dx contraction on 16x16x16):
//   pre / dfo = x W1^T / dh W2 (rows on the accumulator's row axis, ff on its column axis);
//   dW1[ff][d] += dact^T x and dW2[d][ff] += dh^T fo over the step's rows, the row k-set of lane group g
//   being rows {4g..4g+3} of both 16-row blocks -- dact / fo straight from the accumulator registers,
//   x / dh from the images by transposed reads (ds_read_b64_tr_b16);
//   dx += dact W1: dact through a wave-private [ff][row] staging image, read back transposed.
template <int D, int NT>
struct FfnOwn {
  static constexpr int NW = 8;                  // waves per workgroup
  static constexpr int SR = 32;                 // rows per step
  static constexpr int KH = D / 32, NJ = D / 16, NP = NT / 2;
  static constexpr int VPL = D / 16;            // loader / epilogue: floats of a row per lane (16 lanes a row)
  static constexpr int FF = 128 * NT;
  static constexpr int NCH = FF / 32;           // 32-column keep-word chunks (<= 16: one word per lane)
  static constexpr int XRS = D == 32 ? 96 : 160;   // bytes per row of the bf16 x / dh images (conflict-free
                                                   // ds_read_b128 rows and transposed 4-row reads)
  static constexpr int O_XB = 0, O_HB = SR * XRS, O_KB = 2 * SR * XRS;
  static constexpr int IMG = 2 * SR * XRS + NCH * SR * 4;
  static constexpr int XCS = D + 4;             // floats per exchange row: 4 XCS = 16 mod 32 banks
  static constexpr int XSLOT = SR * XCS * 4;
  static constexpr int XCH = NW * XSLOT;
  static constexpr int S4 = 24;                 // dwords per staging row ([ff][32 rows] bf16, swizzled)
  static constexpr int STG = 16 * NT * S4 * 4;
  static constexpr int O_XCH = 3 * IMG, O_STG = O_XCH + 2 * XCH;
  static constexpr int LDS = O_STG + NW * STG;
  static_assert(NCH <= 16 && LDS <= 160 * 1024, "FfnOwn: shape");
};

// staging image byte offset of (ff row, 4 rows from rowM): dword (rowM / 2) ^ f(ff) -- 8-byte stores of
// four rows and the transposed reads of the dx A operand without bank conflicts on the stores and <= 2-way
// on the reads
__device__ __forceinline__ int own_stg(int ffl, int rowM) {
  const int f = (((ffl >> 2) & 1) << 1) ^ (((ffl >> 3) & 1) << 2);
  return ffl * (24 * 4) + ((((rowM >> 1)) ^ f) << 2);
}

__device__ __forceinline__ f32x4 mfma_bf16k(bf16x4 a, bf16x4 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(__builtin_bit_cast(s16x4, a), __builtin_bit_cast(s16x4, b), c,
                                                   0, 0, 0);
}

template <int N>
struct fvec {
  float v[N];
};
// Row segments are read with plain global loads behind a row bound.  Not raw buffer loads: ROCm 7.2's backend
// miscompiles a buffer load whose result vector is then taken apart element by element (the 8-byte form and
// a 16-byte load of which two elements are used alike): it shrinks the load to ONE dword and hands that
// dword out for every element (reproduced stand-alone: buffer_load_dword + v_cvt_pk_bf16_f32 v, v, v).
template <int N>
__device__ __forceinline__ fvec<N> ld_row(const float* __restrict__ p, bool ok) {
  typedef float fv __attribute__((ext_vector_type(N)));
  fv u = {};
  if (ok) u = *(const fv*)p;
  fvec<N> o;
#pragma unroll
  for (int i = 0; i < N; ++i) o.v[i] = u[i];
  return o;
}

template <int D, int NT, bool NORMS, bool DROP>
__global__ __launch_bounds__(512) void ffn_bwd_own_kernel(FfnArgs a, int steps_per_wg) {
  using T = FfnOwn<D, NT>;
  constexpr int VPL = T::VPL, KH = T::KH, NJ = T::NJ, NP = T::NP, FF = T::FF;
  __shared__ __attribute__((aligned(16))) char lds[T::LDS];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, c = lane & 15;
  const int M = a.M;
  const int nsteps = (M + T::SR - 1) / T::SR;
  const int s0 = blockIdx.x * steps_per_wg, s1 = min(nsteps, s0 + steps_per_wg);
  const int nb16 = (M + 15) / 16;
  const int fw = 16 * NT * w;                   // this wave's first FF column
  const float dsc = a.drop.scale;

  // ---- resident weights (bf16 images written by the forward: W1 (FF, D) | W2^T (FF, D) | W1^T (D, FF))
  const auto rw = buf_rsrc(a.wbf, (uint32_t)(3 * FF * D) * 2);
  bf16x8 w1b[NT][KH], w2b[NT][KH];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int kh = 0; kh < KH; ++kh) {
      const uint32_t o = (uint32_t)((fw + 16 * t + c) * D + 32 * kh + 8 * g) * 2;
      w1b[t][kh] = buf_ld_bf8(rw, o, 0);
      w2b[t][kh] = buf_ld_bf8(rw, o + (uint32_t)(FF * D) * 2, 0);
    }
  bf16x8 w1t32[NP > 0 ? NP : 1][NJ];
  bf16x4 w1t16[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const uint32_t row = (uint32_t)(2 * FF * D + (16 * j + c) * FF + fw) * 2;
#pragma unroll
    for (int p = 0; p < NP; ++p) w1t32[p][j] = buf_ld_bf8(rw, row + (uint32_t)(32 * p + 8 * g) * 2, 0);
    if constexpr (NT & 1)
      w1t16[j] = *(const bf16x4*)(a.wbf + 2 * FF * D + (16 * j + c) * FF + fw + 32 * NP + 4 * g);
  }
  float b1v[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) b1v[t] = a.b1[fw + 16 * t + c];

  // ---- accumulators over the whole launch
  f32x4 dw1[NT][NJ], dw2[NT][NJ];
  float db1[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    db1[t] = 0.f;
#pragma unroll
    for (int j = 0; j < NJ; ++j) dw1[t][j] = dw2[t][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  float cb2[VPL], cn2[VPL], cn1[VPL];
#pragma unroll
  for (int v = 0; v < VPL; ++v) cb2[v] = cn2[v] = cn1[v] = 0.f;

  // ---- loader / epilogue lane map: row 4w + g of the step, columns c0 .. c0 + VPL - 1
  const int rl = 4 * w + g, c0 = VPL * c;
  const uint32_t mbytes = (uint32_t)M * D * 4;
  const auto rr2 = buf_rsrc(a.r2, NORMS ? (uint32_t)M * 4 : 0u);
  const auto rr1 = buf_rsrc(a.r1, NORMS ? (uint32_t)M * 4 : 0u);
  const auto rout = buf_rsrc(NORMS ? a.dh1 : a.dx, mbytes);
  const auto rmask = buf_rsrc(a.mask, DROP ? (uint32_t)nb16 * 16 * (FF / 32) * 4 : 0u);
  float nw2[VPL], nw1[VPL];
#pragma unroll
  for (int v = 0; v < VPL; ++v) {
    nw2[v] = NORMS ? a.nw2[c0 + v] : 0.f;
    nw1[v] = NORMS ? a.nw1[c0 + v] : 0.f;
  }
  struct Raw {
    fvec<VPL> x, dy, h2, h1;
    float r2, r1;
    uint32_t kw;
  };
  auto issue = [&](int s, Raw& R) {
    const int m = T::SR * s + rl;
    const bool ok = m < M;
    const long e = (long)m * D + c0;
    const uint32_t offr = ok ? (uint32_t)m * 4 : BUF_OOB;
    R.x = ld_row<VPL>(a.x + e, ok);
    R.dy = ld_row<VPL>((NORMS ? a.dy : a.dh) + e, ok);
    if (NORMS) {
      R.h2 = ld_row<VPL>(a.h2 + e, ok);
      R.h1 = ld_row<VPL>(a.h1 + e, ok);
      R.r2 = buf_ld(rr2, offr);
      R.r1 = buf_ld(rr1, offr);
    }
    if (DROP) {      // keep word of chunk lane / 4, row 4w + lane % 4 (lanes >= 4 NCH idle)
      const int row = T::SR * s + 4 * w + (lane & 3), ch = lane >> 2;
      const bool ok = lane < 4 * T::NCH && row < M;
      R.kw = __builtin_bit_cast(uint32_t, buf_ld(rmask, ok ? rw_word(ch, nb16, row >> 4, row & 15) * 4 : BUF_OOB));
    }
  };
  // norm2 backward of the loaded rows -> dh2 (kept for this row's epilogue) + the images of step s
  auto prepare = [&](int s, const Raw& R, float (&dh2)[VPL]) {
    char* img = lds + (s % 3) * T::IMG;
    if (NORMS) {
      float dot = 0.f;
#pragma unroll
      for (int v = 0; v < VPL; ++v) dot = fmaf(nw2[v] * R.dy.v[v], R.h2.v[v], dot);
      dot = group_sum<16>(dot);
      const float rm = R.r2;
      const float coef = rm * rm * rm / (float)D * dot;
#pragma unroll
      for (int v = 0; v < VPL; ++v) {
        dh2[v] = nw2[v] * R.dy.v[v] * rm - R.h2.v[v] * coef;
        cb2[v] += dh2[v];
        cn2[v] = fmaf(R.dy.v[v] * R.h2.v[v], rm, cn2[v]);
      }
    } else {
#pragma unroll
      for (int v = 0; v < VPL; ++v) dh2[v] = R.dy.v[v];
    }
    if constexpr (VPL == 2) {
      *(bf16x2*)(img + T::O_XB + rl * T::XRS + c0 * 2) = bf16x2{(__bf16)R.x.v[0], (__bf16)R.x.v[1]};
      *(bf16x2*)(img + T::O_HB + rl * T::XRS + c0 * 2) = bf16x2{(__bf16)dh2[0], (__bf16)dh2[1]};
    } else {
      *(bf16x4*)(img + T::O_XB + rl * T::XRS + c0 * 2) =
          bf16x4{(__bf16)R.x.v[0], (__bf16)R.x.v[1], (__bf16)R.x.v[2], (__bf16)R.x.v[3]};
      *(bf16x4*)(img + T::O_HB + rl * T::XRS + c0 * 2) =
          bf16x4{(__bf16)dh2[0], (__bf16)dh2[1], (__bf16)dh2[2], (__bf16)dh2[3]};
    }
    if (DROP && lane < 4 * T::NCH) *(uint32_t*)(img + T::O_KB + ((lane >> 2) * T::SR + 4 * w + (lane & 3)) * 4) = R.kw;
  };

  char* stg = lds + T::O_STG + w * T::STG;
  // the step's products; the dx partial of the step's 32 rows -> exchange slot (s & 1, w)
  auto compute = [&](int s) {
    const char* img = lds + (s % 3) * T::IMG;
    bf16x8 xa[2][KH], ha[2][KH], xt[NJ], ht[NJ];
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int kh = 0; kh < KH; ++kh) {
        const int o = (16 * b + c) * T::XRS + (32 * kh + 8 * g) * 2;
        xa[b][kh] = *(const bf16x8*)(img + T::O_XB + o);
        ha[b][kh] = *(const bf16x8*)(img + T::O_HB + o);
      }
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      // lane 4q + p of group g: row 16b + 4g + q, columns 16j + 4p .. +3 -> lane c gets column 16j + c
      const int o0 = (4 * g + (c >> 2)) * T::XRS + (16 * j + 4 * (c & 3)) * 2, o1 = o0 + 16 * T::XRS;
      xt[j] = cat8(lds_tr4((const __bf16*)(img + T::O_XB + o0)), lds_tr4((const __bf16*)(img + T::O_XB + o1)));
      ht[j] = cat8(lds_tr4((const __bf16*)(img + T::O_HB + o0)), lds_tr4((const __bf16*)(img + T::O_HB + o1)));
    }
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int f0 = fw + 16 * t;
      f32x4 pre[2], dfo[2];
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        pre[b] = dfo[b] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kh = 0; kh < KH; ++kh) {
          pre[b] = mfma_bf(xa[b][kh], w1b[t][kh], pre[b]);
          dfo[b] = mfma_bf(ha[b][kh], w2b[t][kh], dfo[b]);
        }
      }
      f32x4 fo[2], da[2];
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        u32x4 kw = {0u, 0u, 0u, 0u};
        if (DROP) kw = *(const u32x4*)(img + T::O_KB + ((f0 >> 5) * T::SR + 16 * b + 4 * g) * 4);
        const int bit = (f0 & 31) + c;
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          // pre[b][r]: row 16b + 4g + r, column f0 + c
          const f32x2 z = f32x2{pre[b][2 * q], pre[b][2 * q + 1]} + b1v[t];
          f32x2 e;
          const f32x2 cdf = cdf_as2(z, e);
          const f32x2 gg = z * e * 0.39894228040143268f + cdf;
          f32x2 sc = {1.f, 1.f};
          if (DROP) sc = f32x2{((kw[2 * q] >> bit) & 1u) ? dsc : 0.f, ((kw[2 * q + 1] >> bit) & 1u) ? dsc : 0.f};
          const f32x2 fv = z * cdf * sc;
          const f32x2 dv = f32x2{dfo[b][2 * q], dfo[b][2 * q + 1]} * sc * gg;
          fo[b][2 * q] = fv.x;
          fo[b][2 * q + 1] = fv.y;
          da[b][2 * q] = dv.x;
          da[b][2 * q + 1] = dv.y;
        }
        db1[t] += (da[b][0] + da[b][1]) + (da[b][2] + da[b][3]);
      }
      const bf16x8 afo = pack8(fo[0], fo[1]), ada = pack8(da[0], da[1]);
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        dw1[t][j] = mfma_bf(ada, xt[j], dw1[t][j]);      // C[ff f0 + 4g + r][d 16j + c]
        dw2[t][j] = mfma_bf(ht[j], afo, dw2[t][j]);      // C[d 16j + 4g + r][ff f0 + c]
      }
#pragma unroll
      for (int b = 0; b < 2; ++b)
        *(bf16x4*)(stg + own_stg(16 * t + c, 16 * b + 4 * g)) = __builtin_convertvector(da[b], bf16x4);
    }
    __builtin_amdgcn_wave_barrier();
    // dx partial over this wave's FF columns: A = dact[row 16b + c][ff k-set of group g] (transposed reads)
    float* xs = (float*)(lds + T::O_XCH + (s & 1) * T::XCH + w * T::XSLOT);
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      f32x4 dxp[NJ];
#pragma unroll
      for (int j = 0; j < NJ; ++j) dxp[j] = f32x4{0.f, 0.f, 0.f, 0.f};
      const int rm = 16 * b + 4 * (c & 3);
#pragma unroll
      for (int p = 0; p < NP; ++p) {
        const int fl = 32 * p + 8 * g + (c >> 2);
        const bf16x8 av = cat8(lds_tr4((const __bf16*)(stg + own_stg(fl, rm))),
                               lds_tr4((const __bf16*)(stg + own_stg(fl + 4, rm))));
#pragma unroll
        for (int j = 0; j < NJ; ++j) dxp[j] = mfma_bf(av, w1t32[p][j], dxp[j]);
      }
      if constexpr (NT & 1) {
        const bf16x4 av = lds_tr4((const __bf16*)(stg + own_stg(32 * NP + 4 * g + (c >> 2), rm)));
#pragma unroll
        for (int j = 0; j < NJ; ++j) dxp[j] = mfma_bf16k(av, w1t16[j], dxp[j]);
      }
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) xs[(16 * b + 4 * g + r) * T::XCS + 16 * j + c] = dxp[j][r];
    }
    __builtin_amdgcn_wave_barrier();     // the staging image is rewritten by the next step
  };

  // the eight partials of this lane's row (fixed source order) + the residual -> norm1 backward
  auto epilogue = [&](int s, const float (&dh2)[VPL], const Raw& R) {
    const float* xs = (const float*)(lds + T::O_XCH + (s & 1) * T::XCH);
    float dx1[VPL];
#pragma unroll
    for (int v = 0; v < VPL; ++v) dx1[v] = 0.f;
#pragma unroll
    for (int src = 0; src < T::NW; ++src) {
      const fvec<VPL> pv = *(const fvec<VPL>*)(xs + src * (T::XSLOT / 4) + rl * T::XCS + c0);
#pragma unroll
      for (int v = 0; v < VPL; ++v) dx1[v] += pv.v[v];
    }
    const int m = T::SR * s + rl;
    const uint32_t off = m < M ? (uint32_t)(m * D + c0) * 4 : BUF_OOB;
#pragma unroll
    for (int v = 0; v < VPL; ++v) dx1[v] += dh2[v];
    if (!NORMS) {
#pragma unroll
      for (int v = 0; v < VPL; ++v) buf_st(dx1[v], rout, off + 4 * v);
      return;
    }
    float dot = 0.f;
#pragma unroll
    for (int v = 0; v < VPL; ++v) dot = fmaf(nw1[v] * dx1[v], R.h1.v[v], dot);
    dot = group_sum<16>(dot);
    const float rm = R.r1;
    const float coef = rm * rm * rm / (float)D * dot;
#pragma unroll
    for (int v = 0; v < VPL; ++v) {
      buf_st(nw1[v] * dx1[v] * rm - R.h1.v[v] * coef, rout, off + 4 * v);
      cn1[v] = fmaf(dx1[v] * R.h1.v[v], rm, cn1[v]);
    }
  };

  // ---- the step pipeline
  // static priority for the second-dispatched half of the workgroup (MI355X_MICROARCH.md, two waves per SIMD item 4):
  // the SIMD partners run the same step in lockstep and the younger half loses every arbitration (128.1 / 129.5 /
  // 132.4 -> 127.4 / 126.0 / 131.6 us, profiles/r06/ab_ffn_bwd_prio.log)
  if (w >= 4) __builtin_amdgcn_s_setprio(1);
  Raw rc, rn;
  float dh2c[VPL], dh2n[VPL];
  if (s0 < s1) {
    issue(s0, rc);
    prepare(s0, rc, dh2c);
  }
  __syncthreads();
  for (int s = s0; s < s1; ++s) {
    const bool more = s + 1 < s1;
    if (more) issue(s + 1, rn);
    compute(s);
    if (more) prepare(s + 1, rn, dh2n);
    __syncthreads();
    epilogue(s, dh2c, rc);
#pragma unroll
    for (int v = 0; v < VPL; ++v) dh2c[v] = dh2n[v];
    rc = rn;
  }

  // ---- the workgroup's slab row, written once
  float* slab = a.slab + (long)blockIdx.x * a.ld_slab;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int f0 = fw + 16 * t;
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        slab[a.o_w1 + (long)(f0 + 4 * g + r) * D + 16 * j + c] = dw1[t][j][r];
        slab[a.o_w2 + (long)(16 * j + 4 * g + r) * FF + f0 + c] = dw2[t][j][r];
      }
    float v = db1[t];
    v += __shfl_xor(v, 16, 64);
    v += __shfl_xor(v, 32, 64);
    if (g == 0) slab[a.o_b1 + f0 + c] = v;
  }
  // column sums of the norm weights / db2: lanes of one column (4 per wave, 8 waves), fixed order
  __syncthreads();                       // the exchange buffers are free
  float* red = (float*)(lds + T::O_XCH);   // [wave][3][D]
#pragma unroll
  for (int v = 0; v < VPL; ++v) {
    float q[3] = {cb2[v], cn2[v], cn1[v]};
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      q[k] += __shfl_xor(q[k], 16, 64);
      q[k] += __shfl_xor(q[k], 32, 64);
      if (g == 0) red[(w * 3 + k) * D + c0 + v] = q[k];
    }
  }
  __syncthreads();
  if (NORMS && tid < 3 * D) {
    const int k = tid / D, col = tid % D;
    float sum = 0.f;
#pragma unroll
    for (int src = 0; src < T::NW; ++src) sum += red[(src * 3 + k) * D + col];
    slab[(k == 0 ? a.o_b2 : k == 1 ? a.o_n2 : a.o_n1) + col] = sum;
  }
}

// ---------------------------------------------------------------- amp: bf16, D = 64 column-owner backward, two passes
// D = 64 (cfgs/v3_k148_s1.yaml) in the owner form above: a wave's dW1 AND dW2 slices (2 x 16 NT x 64 floats) plus its
// resident weights need more registers than two waves per SIMD hold, so the weight grads are split over two passes
// over the rows, each with its own accumulators in registers and ONE slab write per workgroup at the end:
//   PASS 1: pre / dfo -> dact -> dW1, db1 (owner registers) and dx = dact W1 + dh2 -> norm1 backward, the norm
//           weights' / db2 column sums.  The dx contraction over FF is NOT split over the waves (an 8-way fp32
//           partial exchange of 32 x 64 rows per wave would need 140 KB of LDS): every wave writes its dact columns
//           into a shared [FF][32 rows] bf16 image, and after one barrier wave w computes the whole 16 x 16 dx tile
//           (row block w / 4, column block w % 4) over all FF from that image and W1^T (LDS-resident, bf16), so
//           each dx element is one fixed-order MFMA chain (deterministic).  Two barriers per 32-row step.
//   PASS 2: pre -> fo -> dW2 = dh2^T fo (owner registers).  Recomputes pre and the norm2 backward of dy.
// The pass-2 re-read of x / dy / h2 (3 x 4 B x M x 64) replaces the per-tile slab read-modify-writes of the
// rows-per-wave kernel (ffn_bwd_bf_kernel<64>: 2 GB written per launch at cfg4).
template <int NT>
struct FfnOwn64 {
  static constexpr int D = 64, NW = 8, SR = 32, KH = 2, NJ = 4, VPL = 4;
  static constexpr int FF = 128 * NT, NCH = FF / 32, NP = FF / 32;
  static constexpr int XRS = 160;                                  // bytes per bf16 image row (as FfnOwn<64>)
  static constexpr int O_XB = 0, O_HB = SR * XRS, O_KB = 2 * SR * XRS;
  static constexpr int IMG = 2 * SR * XRS + NCH * SR * 4;          // one step's images; two of them
  static constexpr int O_DA = 2 * IMG;                             // pass 1: dact [FF][32 rows] bf16 (own_stg)
  static constexpr int DA = FF * 24 * 4;
  static constexpr int XCS = D + 4;                                // pass 1: dx tiles [32 rows][XCS] fp32
  static constexpr int O_DX = O_DA + DA, DXB = SR * XCS * 4;
  static constexpr int W1S = FF * 2 + 16;                          // pass 1: W1^T [64 d][FF] bf16, row bytes
  static constexpr int O_W1T = O_DX + DXB;
  static constexpr int LDS1 = O_W1T + D * W1S;
  static constexpr int LDS2 = 2 * IMG;
  static_assert(NCH <= 16 && LDS1 <= 160 * 1024, "FfnOwn64: shape");
};

template <int NT, int PASS, bool NORMS, bool DROP>
__global__ __launch_bounds__(512) void ffn_bwd_own64_kernel(FfnArgs a, int steps_per_wg) {
  using T = FfnOwn64<NT>;
  constexpr int D = 64, VPL = T::VPL, KH = T::KH, NJ = T::NJ, FF = T::FF;
  __shared__ __attribute__((aligned(16))) char lds[PASS == 1 ? T::LDS1 : T::LDS2];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, c = lane & 15;
  const int M = a.M;
  const int nsteps = (M + T::SR - 1) / T::SR;
  const int s0 = blockIdx.x * steps_per_wg, s1 = min(nsteps, s0 + steps_per_wg);
  const int nb16 = (M + 15) / 16;
  const int fw = 16 * NT * w;                   // this wave's first FF column
  const float dsc = a.drop.scale;

  // ---- resident weights: W1 slice (pre) in registers; W2^T slice (dfo) and W1^T (dx, LDS) in pass 1
  const auto rw = buf_rsrc(a.wbf, (uint32_t)(3 * FF * D) * 2);
  bf16x8 w1b[NT][KH], w2b[PASS == 1 ? NT : 1][KH];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int kh = 0; kh < KH; ++kh) {
      const uint32_t o = (uint32_t)((fw + 16 * t + c) * D + 32 * kh + 8 * g) * 2;
      w1b[t][kh] = buf_ld_bf8(rw, o, 0);
      if constexpr (PASS == 1) w2b[t][kh] = buf_ld_bf8(rw, o + (uint32_t)(FF * D) * 2, 0);
    }
  if constexpr (PASS == 1) {
    for (int q = tid; q < D * FF / 8; q += 512) {      // W1^T rows d, 8 ff per 16-byte chunk
      const int d = q / (FF / 8), f8 = (q % (FF / 8)) * 8;
      *(bf16x8*)(lds + T::O_W1T + d * T::W1S + f8 * 2) = buf_ld_bf8(rw, (uint32_t)(2 * FF * D + d * FF + f8) * 2, 0);
    }
  }
  float b1v[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) b1v[t] = a.b1[fw + 16 * t + c];

  // ---- accumulators over the whole launch: dW1 + db1 (pass 1) or dW2 (pass 2)
  f32x4 dwa[NT][NJ];
  float db1[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    db1[t] = 0.f;
#pragma unroll
    for (int j = 0; j < NJ; ++j) dwa[t][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  float cb2[VPL], cn2[VPL], cn1[VPL];
#pragma unroll
  for (int v = 0; v < VPL; ++v) cb2[v] = cn2[v] = cn1[v] = 0.f;

  // ---- loader / epilogue lane map: row 4w + g of the step, columns c0 .. c0 + 3
  const int rl = 4 * w + g, c0 = VPL * c;
  const uint32_t mbytes = (uint32_t)M * D * 4;
  const auto rr2 = buf_rsrc(a.r2, NORMS ? (uint32_t)M * 4 : 0u);
  const auto rr1 = buf_rsrc(a.r1, NORMS && PASS == 1 ? (uint32_t)M * 4 : 0u);
  const auto rout = buf_rsrc(NORMS ? a.dh1 : a.dx, PASS == 1 ? mbytes : 0u);
  const auto rmask = buf_rsrc(a.mask, DROP ? (uint32_t)nb16 * 16 * (FF / 32) * 4 : 0u);
  float nw2[VPL], nw1[VPL];
#pragma unroll
  for (int v = 0; v < VPL; ++v) {
    nw2[v] = NORMS ? a.nw2[c0 + v] : 0.f;
    nw1[v] = NORMS && PASS == 1 ? a.nw1[c0 + v] : 0.f;
  }
  struct Raw {
    fvec<VPL> x, dy, h2;
    float r2;
    uint32_t kw;
  };
  struct Nr1 {        // the norm1 backward's operands of the step's epilogue row (pass 1)
    fvec<VPL> h1;
    float r1;
  };
  auto issue = [&](int s, Raw& R) {
    const int m = T::SR * s + rl;
    const bool ok = m < M;
    const long e = (long)m * D + c0;
    R.x = ld_row<VPL>(a.x + e, ok);
    R.dy = ld_row<VPL>((NORMS ? a.dy : a.dh) + e, ok);
    if (NORMS) {
      R.h2 = ld_row<VPL>(a.h2 + e, ok);
      R.r2 = buf_ld(rr2, ok ? (uint32_t)m * 4 : BUF_OOB);
    }
    if (DROP) {      // keep word of chunk lane / 4, row 4w + lane % 4 (lanes >= 4 NCH idle)
      const int row = T::SR * s + 4 * w + (lane & 3), ch = lane >> 2;
      const bool okk = lane < 4 * T::NCH && row < M;
      R.kw = __builtin_bit_cast(uint32_t, buf_ld(rmask, okk ? rw_word(ch, nb16, row >> 4, row & 15) * 4 : BUF_OOB));
    }
  };
  auto issue_n1 = [&](int s, Nr1& N) {
    const int m = T::SR * s + rl;
    const bool ok = m < M;
    N.h1 = ld_row<VPL>(a.h1 + (long)m * D + c0, ok);
    N.r1 = buf_ld(rr1, ok ? (uint32_t)m * 4 : BUF_OOB);
  };
  // norm2 backward of the loaded rows -> dh2 (pass 1 keeps it for the row's epilogue) + the images of step s
  auto prepare = [&](int s, const Raw& R, float (&dh2)[VPL]) {
    char* img = lds + (s & 1) * T::IMG;
    if (NORMS) {
      float dot = 0.f;
#pragma unroll
      for (int v = 0; v < VPL; ++v) dot = fmaf(nw2[v] * R.dy.v[v], R.h2.v[v], dot);
      dot = group_sum<16>(dot);
      const float rm = R.r2;
      const float coef = rm * rm * rm / (float)D * dot;
#pragma unroll
      for (int v = 0; v < VPL; ++v) {
        dh2[v] = nw2[v] * R.dy.v[v] * rm - R.h2.v[v] * coef;
        if constexpr (PASS == 1) {
          cb2[v] += dh2[v];
          cn2[v] = fmaf(R.dy.v[v] * R.h2.v[v], rm, cn2[v]);
        }
      }
    } else {
#pragma unroll
      for (int v = 0; v < VPL; ++v) dh2[v] = R.dy.v[v];
    }
    *(bf16x4*)(img + T::O_XB + rl * T::XRS + c0 * 2) =
        bf16x4{(__bf16)R.x.v[0], (__bf16)R.x.v[1], (__bf16)R.x.v[2], (__bf16)R.x.v[3]};
    *(bf16x4*)(img + T::O_HB + rl * T::XRS + c0 * 2) = bf16x4{(__bf16)dh2[0], (__bf16)dh2[1], (__bf16)dh2[2], (__bf16)dh2[3]};
    if (DROP && lane < 4 * T::NCH) *(uint32_t*)(img + T::O_KB + ((lane >> 2) * T::SR + 4 * w + (lane & 3)) * 4) = R.kw;
  };

  // transposed image reads: lane 4q + p of group g -> row 16b + 4g + q, columns 16j + 4p .. +3, so lane c gets
  // column 16j + c at the rows {4g .. 4g + 3} of both 16-row blocks (the k-set of the row contractions)
  auto tr_cols = [&](const char* base, int j) {
    const int o0 = (4 * g + (c >> 2)) * T::XRS + (16 * j + 4 * (c & 3)) * 2, o1 = o0 + 16 * T::XRS;
    return cat8(lds_tr4((const __bf16*)(base + o0)), lds_tr4((const __bf16*)(base + o1)));
  };

  // the step's products: pass 1 -> dW1 / db1 and the dact image; pass 2 -> dW2
  auto compute = [&](int s) {
    const char* img = lds + (s & 1) * T::IMG;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int f0 = fw + 16 * t;
      // the A rows are re-read per column tile (registers: a wave holds its W1 / W2^T slices and dW1)
      bf16x8 xa[2][KH], ha[PASS == 1 ? 2 : 1][KH];
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int kh = 0; kh < KH; ++kh) {
          const int o = (16 * b + c) * T::XRS + (32 * kh + 8 * g) * 2;
          xa[b][kh] = *(const bf16x8*)(img + T::O_XB + o);
          if constexpr (PASS == 1) ha[b][kh] = *(const bf16x8*)(img + T::O_HB + o);
        }
      f32x4 pre[2], dfo[2];
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        pre[b] = dfo[b] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kh = 0; kh < KH; ++kh) {
          pre[b] = mfma_bf(xa[b][kh], w1b[t][kh], pre[b]);
          if constexpr (PASS == 1) dfo[b] = mfma_bf(ha[b][kh], w2b[t][kh], dfo[b]);
        }
      }
      f32x4 out[2];       // pass 1: dact; pass 2: fo
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        u32x4 kw = {0u, 0u, 0u, 0u};
        if (DROP) kw = *(const u32x4*)(img + T::O_KB + ((f0 >> 5) * T::SR + 16 * b + 4 * g) * 4);
        const int bit = (f0 & 31) + c;
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          // pre[b][r]: row 16b + 4g + r, column f0 + c
          const f32x2 z = f32x2{pre[b][2 * q], pre[b][2 * q + 1]} + b1v[t];
          f32x2 e;
          const f32x2 cdf = cdf_as2(z, e);
          f32x2 sc = {1.f, 1.f};
          if (DROP) sc = f32x2{((kw[2 * q] >> bit) & 1u) ? dsc : 0.f, ((kw[2 * q + 1] >> bit) & 1u) ? dsc : 0.f};
          f32x2 v;
          if constexpr (PASS == 1) {
            const f32x2 gg = z * e * 0.39894228040143268f + cdf;
            v = f32x2{dfo[b][2 * q], dfo[b][2 * q + 1]} * sc * gg;
          } else {
            v = z * cdf * sc;
          }
          out[b][2 * q] = v.x;
          out[b][2 * q + 1] = v.y;
        }
        if constexpr (PASS == 1) db1[t] += (out[b][0] + out[b][1]) + (out[b][2] + out[b][3]);
      }
      const bf16x8 ao = pack8(out[0], out[1]);
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        if constexpr (PASS == 1) dwa[t][j] = mfma_bf(ao, tr_cols(img + T::O_XB, j), dwa[t][j]);   // C[ff f0+4g+r][d 16j+c]
        else dwa[t][j] = mfma_bf(tr_cols(img + T::O_HB, j), ao, dwa[t][j]);                     // C[d 16j+4g+r][ff f0+c]
      }
      if constexpr (PASS == 1) {
#pragma unroll
        for (int b = 0; b < 2; ++b)
          *(bf16x4*)(lds + T::O_DA + own_stg(f0 + c, 16 * b + 4 * g)) = __builtin_convertvector(out[b], bf16x4);
      }
    }
  };

  // pass 1: wave w's dx tile (rows 16 (w / 4) .., columns 16 (w % 4) ..) over all FF from the dact image
  auto dx_tile = [&]() {
    const int rb = w >> 2, dj = w & 3;
    const int rm = 16 * rb + 4 * (c & 3);
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int p = 0; p < T::NP; ++p) {
      const int fl = 32 * p + 8 * g + (c >> 2);
      const bf16x8 av = cat8(lds_tr4((const __bf16*)(lds + T::O_DA + own_stg(fl, rm))),
                             lds_tr4((const __bf16*)(lds + T::O_DA + own_stg(fl + 4, rm))));
      const bf16x8 bv = *(const bf16x8*)(lds + T::O_W1T + (16 * dj + c) * T::W1S + (32 * p + 8 * g) * 2);
      acc = mfma_bf(av, bv, acc);
    }
    float* xs = (float*)(lds + T::O_DX);
#pragma unroll
    for (int r = 0; r < 4; ++r) xs[(16 * rb + 4 * g + r) * T::XCS + 16 * dj + c] = acc[r];
  };

  // pass 1: dx1 = dact W1 + dh2 of this lane's row -> norm1 backward (or dx)
  auto epilogue = [&](int s, const float (&dh2)[VPL], const Nr1& N) {
    const fvec<VPL> pv = *(const fvec<VPL>*)((const float*)(lds + T::O_DX) + rl * T::XCS + c0);
    float dx1[VPL];
#pragma unroll
    for (int v = 0; v < VPL; ++v) dx1[v] = pv.v[v] + dh2[v];
    const int m = T::SR * s + rl;
    const uint32_t off = m < M ? (uint32_t)(m * D + c0) * 4 : BUF_OOB;
    if (!NORMS) {
#pragma unroll
      for (int v = 0; v < VPL; ++v) buf_st(dx1[v], rout, off + 4 * v);
      return;
    }
    float dot = 0.f;
#pragma unroll
    for (int v = 0; v < VPL; ++v) dot = fmaf(nw1[v] * dx1[v], N.h1.v[v], dot);
    dot = group_sum<16>(dot);
    const float rm = N.r1;
    const float coef = rm * rm * rm / (float)D * dot;
#pragma unroll
    for (int v = 0; v < VPL; ++v) {
      buf_st(nw1[v] * dx1[v] * rm - N.h1.v[v] * coef, rout, off + 4 * v);
      cn1[v] = fmaf(dx1[v] * N.h1.v[v], rm, cn1[v]);
    }
  };

  // ---- the step pipeline (images double-buffered; pass 1: dact image and dx tiles single, two barriers a step)
  Raw rn;
  Nr1 n1;
  float dh2c[VPL], dh2n[VPL];
  if (s0 < s1) {
    Raw r0;
    issue(s0, r0);
    prepare(s0, r0, dh2c);
  }
  __syncthreads();       // W1^T and the first images
  for (int s = s0; s < s1; ++s) {
    const bool more = s + 1 < s1;
    if (more) issue(s + 1, rn);
    if constexpr (PASS == 1) {
      if (NORMS) issue_n1(s, n1);
      compute(s);
      lds_sync();        // every wave's dact columns are in the image
      dx_tile();
      if (more) prepare(s + 1, rn, dh2n);
      lds_sync();        // the dx tiles and the next images are complete
      epilogue(s, dh2c, n1);
#pragma unroll
      for (int v = 0; v < VPL; ++v) dh2c[v] = dh2n[v];
    } else {
      compute(s);
      if (more) prepare(s + 1, rn, dh2n);
      lds_sync();        // the next images are complete; this step's are free
    }
  }

  // ---- the workgroup's slab row, written once
  float* slab = a.slab + (long)blockIdx.x * a.ld_slab;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int f0 = fw + 16 * t;
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if constexpr (PASS == 1) slab[a.o_w1 + (long)(f0 + 4 * g + r) * D + 16 * j + c] = dwa[t][j][r];
        else slab[a.o_w2 + (long)(16 * j + 4 * g + r) * FF + f0 + c] = dwa[t][j][r];
      }
    if constexpr (PASS == 1) {
      float v = db1[t];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      if (g == 0) slab[a.o_b1 + f0 + c] = v;
    }
  }
  if constexpr (PASS == 1 && NORMS) {
    // column sums of the norm weights / db2: lanes of one column (4 per wave, 8 waves), fixed order
    __syncthreads();
    float* red = (float*)(lds + T::O_DA);   // [wave][3][D]
#pragma unroll
    for (int v = 0; v < VPL; ++v) {
      float q[3] = {cb2[v], cn2[v], cn1[v]};
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        q[k] += __shfl_xor(q[k], 16, 64);
        q[k] += __shfl_xor(q[k], 32, 64);
        if (g == 0) red[(w * 3 + k) * D + c0 + v] = q[k];
      }
    }
    __syncthreads();
    if (tid < 3 * D) {
      const int k = tid / D, col = tid % D;
      float sum = 0.f;
#pragma unroll
      for (int src = 0; src < T::NW; ++src) sum += red[(src * 3 + k) * D + col];
      slab[(k == 0 ? a.o_b2 : k == 1 ? a.o_n2 : a.o_n1) + col] = sum;
    }
  }
}

// the owner-form shapes: D = 32 (one pass) and D = 64 (two passes, ffn_bwd_own64_kernel), FF = 128 NT, NT <= 3
static int ffn_own_nt(int D, int FF) {
  if ((D != 32 && D != 64) || FF % 128 != 0) return 0;
  const int nt = FF / 128;
  return nt >= 1 && nt <= 3 ? nt : 0;     // NT = 4 spills at 256 VGPRs
}
static int ffn_own_steps_per_wg(long M) {
  const long ns = (M + 31) / 32;
  const long grid = ns < 256 ? ns : 256;
  return (int)((ns + grid - 1) / grid);
}
static int ffn_own_grid(long M) {
  const long ns = (M + 31) / 32;
  const long per = ffn_own_steps_per_wg(M);
  return (int)((ns + per - 1) / per);
}

template <int D, int NT>
static void launch_ffn_own(const FfnArgs& a, hipStream_t s) {
  const int per = ffn_own_steps_per_wg(a.M), grid = ffn_own_grid(a.M);
  const bool drop = a.drop.thresh != 0;
  if constexpr (D == 32) {
    if (a.dy) {
      if (drop) ffn_bwd_own_kernel<D, NT, true, true><<<grid, 512, 0, s>>>(a, per);
      else ffn_bwd_own_kernel<D, NT, true, false><<<grid, 512, 0, s>>>(a, per);
    } else {
      if (drop) ffn_bwd_own_kernel<D, NT, false, true><<<grid, 512, 0, s>>>(a, per);
      else ffn_bwd_own_kernel<D, NT, false, false><<<grid, 512, 0, s>>>(a, per);
    }
  } else {      // D = 64: pass 1 (dW1, db1, dx / dh1, norm columns), then pass 2 (dW2) into the same slab rows
    if (a.dy) {
      if (drop) {
        ffn_bwd_own64_kernel<NT, 1, true, true><<<grid, 512, 0, s>>>(a, per);
        ffn_bwd_own64_kernel<NT, 2, true, true><<<grid, 512, 0, s>>>(a, per);
      } else {
        ffn_bwd_own64_kernel<NT, 1, true, false><<<grid, 512, 0, s>>>(a, per);
        ffn_bwd_own64_kernel<NT, 2, true, false><<<grid, 512, 0, s>>>(a, per);
      }
    } else {
      if (drop) {
        ffn_bwd_own64_kernel<NT, 1, false, true><<<grid, 512, 0, s>>>(a, per);
        ffn_bwd_own64_kernel<NT, 2, false, true><<<grid, 512, 0, s>>>(a, per);
      } else {
        ffn_bwd_own64_kernel<NT, 1, false, false><<<grid, 512, 0, s>>>(a, per);
        ffn_bwd_own64_kernel<NT, 2, false, false><<<grid, 512, 0, s>>>(a, per);
      }
    }
  }
}

// persistent backward grid: at most 512 workgroups (two per CU), tiles split as evenly as possible
static int ffn_bf_grid(long M, int D) {
  const long rt = D <= 32 ? 128 : 64;
  const long nt = (M + rt - 1) / rt;
  const long per = (nt + 511) / 512;
  return (int)((nt + per - 1) / per);
}

template <int D>
static void launch_ffn(const FfnArgs& a, bool bwd, hipStream_t s) {
  const int blocks = cdiv(a.M, FfnTile<D>::RT);
  if (!bwd) {
    ffn_fwd_kernel<D><<<blocks, 256, 0, s>>>(a);
    return;
  }
  if constexpr (D <= 32) {
    if ((a.FF / 16) % 4 == 0) {       // column-owner backward: chunks split evenly over the four waves
      if (a.dy) ffn_bwd_cols_kernel<D, true><<<blocks, 256, 0, s>>>(a);
      else ffn_bwd_cols_kernel<D, false><<<blocks, 256, 0, s>>>(a);
      return;
    }
  }
  if (a.dy) ffn_bwd_kernel<D, true><<<blocks, 256, 0, s>>>(a);
  else ffn_bwd_kernel<D, false><<<blocks, 256, 0, s>>>(a);
}

static bool ffn_shape_ok(int D, int FF) { return (D == 16 || D == 32 || D == 64) && FF > 0 && FF % 16 == 0; }
static bool ffn_bf_shape_ok(int D, int FF) { return (D == 32 || D == 64) && FF > 0 && FF % 32 == 0; }

// buffer resources carry 32-bit byte extents: (M, D) activations, (FF, D) weights, the keep-bit words
static bool ffn_extent_ok(long M, int D, int FF) {
  const long lim = 1L << 31;
  return M * D * 4 < lim && (long)FF * D * 4 < lim && M * (FF / 16) * 2 < lim;
}

template <int D>
static void launch_ffn_bf(const FfnArgs& a, bool bwd, hipStream_t s) {
  const bool drop = a.drop.thresh != 0;
  if (!bwd) {
    {
      // D = 32: two workgroups of eight waves per CU; D = 64: one of sixteen
      constexpr size_t lim = D == 32 ? 76 * 1024 : 150 * 1024;
      const size_t sm = ffn_fwdw_lds<D>(a.FF);
      if (sm <= lim) {
        static bool attr = false;
        if (!attr) {
          (void)hipFuncSetAttribute((const void*)ffn_fwd_bfw_kernel<D, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)lim);
          (void)hipFuncSetAttribute((const void*)ffn_fwd_bfw_kernel<D, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)lim);
          attr = true;
        }
        using T = FfnFw<D>;
        const int grid = std::min(cdiv(a.M, T::RW * T::NWAVE), (D == 32 ? 2 : 1) * 256);
        if (drop) ffn_fwd_bfw_kernel<D, true><<<grid, T::NWAVE * 64, sm, s>>>(a);
        else ffn_fwd_bfw_kernel<D, false><<<grid, T::NWAVE * 64, sm, s>>>(a);
        return;
      }
    }
    if (drop) ffn_fwd_bf_kernel<D, true><<<cdiv(a.M, 128), 256, 0, s>>>(a);
    else ffn_fwd_bf_kernel<D, false><<<cdiv(a.M, 128), 256, 0, s>>>(a);
    return;
  }
  if (const int nt = ffn_own_nt(D, a.FF)) {
    switch (nt) {
      case 1: launch_ffn_own<D, 1>(a, s); return;
      case 2: launch_ffn_own<D, 2>(a, s); return;
      default: launch_ffn_own<D, 3>(a, s); return;
    }
  }
  const int grid = ffn_bf_grid(a.M, D);
  if (a.dy) {
    if (drop) ffn_bwd_bf_kernel<D, true, true><<<grid, 256, 0, s>>>(a);
    else ffn_bwd_bf_kernel<D, true, false><<<grid, 256, 0, s>>>(a);
  } else {
    if (drop) ffn_bwd_bf_kernel<D, false, true><<<grid, 256, 0, s>>>(a);
    else ffn_bwd_bf_kernel<D, false, false><<<grid, 256, 0, s>>>(a);
  }
}

static int ffn_dispatch(const FfnArgs& a, int D, bool bwd, int flags, hipStream_t s) {
  if (flags & CTR_FFN_BF16) {
    if (D == 32) launch_ffn_bf<32>(a, bwd, s);
    else launch_ffn_bf<64>(a, bwd, s);
    return check_launch(bwd ? "ffn_bwd_bf16" : "ffn_fwd_bf16");
  }
  switch (D) {
    case 16: launch_ffn<16>(a, bwd, s); break;
    case 32: launch_ffn<32>(a, bwd, s); break;
    default: launch_ffn<64>(a, bwd, s); break;
  }
  return check_launch(bwd ? "ffn_bwd" : "ffn_fwd");
}

}  // namespace ctr

using namespace ctr;

extern "C" int ctr_ffn_supported(int D, int FF, int flags) {
  return ((flags & CTR_FFN_BF16) ? ffn_bf_shape_ok(D, FF) : ffn_shape_ok(D, FF)) ? 1 : 0;
}

extern "C" int ctr_ffn_slab_rows(int M, int D, int FF, int flags) {
  if (flags & CTR_FFN_BF16) return ffn_own_nt(D, FF) ? ffn_own_grid(M) : ffn_bf_grid(M, D);
  return cdiv(M, D >= 64 ? 64 : 128);
}

// enough for either keep-bit layout (FfnTile::LW)
extern "C" int ctr_ffn_mask_words(int M, int FF) {
  const long rowwords = ((long)M * (FF / 16) + 1) / 2;
  return (int)(lw_words(M, FF) > rowwords ? lw_words(M, FF) : rowwords);
}

extern "C" int ctr_ffn_fwd(const float* x, int M, int D, int FF, const float* W1, const float* b1, const float* W2,
                           const float* b2, const float* norm_w, float eps, uint32_t drop_key, uint32_t drop_thresh,
                           float drop_scale, uint32_t* mask, float* y, float* h, float* r, void* wbf, int flags,
                           void* stream) {
  CTR_REQUIRE(ffn_shape_ok(D, FF), "ctr_ffn_fwd: needs D in {16,32,64} and FF % 16 == 0");
  CTR_REQUIRE(!(flags & CTR_FFN_BF16) || ffn_bf_shape_ok(D, FF), "ctr_ffn_fwd bf16: needs D in {32,64} and FF % 32 == 0");
  CTR_REQUIRE(ffn_extent_ok(M, D, FF), "ctr_ffn_fwd: M x D too large for 32-bit buffer offsets");
  if (M <= 0) return 0;
  FfnArgs a = {};
  a.M = M; a.FF = FF; a.x = x; a.W1 = W1; a.b1 = b1; a.W2 = W2; a.b2 = b2; a.nw = norm_w; a.eps = eps;
  a.drop = Drop{drop_key, drop_thresh, drop_scale};
  a.mask = (uint16_t*)mask;
  a.y = y; a.h = h; a.r = r;
  a.wbf = (flags & CTR_FFN_BF16) ? (__bf16*)wbf : nullptr;
  return ffn_dispatch(a, D, false, flags, (hipStream_t)stream);
}

extern "C" int ctr_ffn_bwd(const float* x, const float* dh, int M, int D, int FF, const float* W1, const float* b1,
                           const float* W2, uint32_t drop_key, uint32_t drop_thresh, float drop_scale,
                           const uint32_t* mask, float* dx, float* slab, long ld_slab, int o_b1, int o_w2,
                           const void* wbf, int flags, void* stream) {
  CTR_REQUIRE(!(flags & CTR_FFN_BF16) || wbf, "ctr_ffn_bwd bf16 needs the forward's bf16 weight images (wbf)");
  CTR_REQUIRE(!drop_thresh || mask, "ctr_ffn_bwd with dropout needs the forward's keep bits");
  CTR_REQUIRE(ffn_shape_ok(D, FF), "ctr_ffn_bwd: needs D in {16,32,64} and FF % 16 == 0");
  CTR_REQUIRE(!(flags & CTR_FFN_BF16) || ffn_bf_shape_ok(D, FF), "ctr_ffn_bwd bf16: needs D in {32,64} and FF % 32 == 0");
  CTR_REQUIRE(ffn_extent_ok(M, D, FF), "ctr_ffn_bwd: M x D too large for 32-bit buffer offsets");
  CTR_REQUIRE(o_b1 >= FF * D && o_w2 >= o_b1 + FF && ld_slab >= (long)o_w2 + (long)D * FF, "ctr_ffn_bwd: slab layout");
  if (M <= 0) return 0;
  FfnArgs a = {};
  a.M = M; a.FF = FF; a.x = x; a.W1 = W1; a.b1 = b1; a.W2 = W2;
  a.drop = Drop{drop_key, drop_thresh, drop_scale};
  a.mask = (uint16_t*)const_cast<uint32_t*>(mask);
  a.dh = dh; a.dx = dx; a.slab = slab; a.ld_slab = ld_slab; a.o_b1 = o_b1; a.o_w2 = o_w2;
  a.wbf = (__bf16*)const_cast<void*>(wbf);
  return ffn_dispatch(a, D, true, flags, (hipStream_t)stream);
}

extern "C" int ctr_ffn_bwd_norms(const float* x, const float* dy, const float* h2, const float* r2, const float* nw2,
                                 const float* h1, const float* r1, const float* nw1, int M, int D, int FF,
                                 const float* W1, const float* b1, const float* W2, uint32_t drop_key,
                                 uint32_t drop_thresh, float drop_scale, const uint32_t* mask, float* dh1,
                                 float* slab, long ld_slab, int o_n1, int o_w1, int o_b1, int o_w2, int o_b2, int o_n2,
                                 const void* wbf, int flags, void* stream) {
  CTR_REQUIRE(!(flags & CTR_FFN_BF16) || wbf, "ctr_ffn_bwd_norms bf16 needs the forward's bf16 weight images (wbf)");
  CTR_REQUIRE(!drop_thresh || mask, "ctr_ffn_bwd_norms with dropout needs the forward's keep bits");
  CTR_REQUIRE(ffn_shape_ok(D, FF), "ctr_ffn_bwd_norms: needs D in {16,32,64} and FF % 16 == 0");
  CTR_REQUIRE(!(flags & CTR_FFN_BF16) || ffn_bf_shape_ok(D, FF),
              "ctr_ffn_bwd_norms bf16: needs D in {32,64} and FF % 32 == 0");
  CTR_REQUIRE(ffn_extent_ok(M, D, FF), "ctr_ffn_bwd_norms: M x D too large for 32-bit buffer offsets");
  CTR_REQUIRE(dy && h2 && r2 && nw2 && h1 && r1 && nw1 && dh1, "ctr_ffn_bwd_norms: missing norm operands");
  CTR_REQUIRE(o_n1 + D <= o_w1 && o_w1 + FF * D <= o_b1 && o_b1 + FF <= o_w2 && o_w2 + D * FF <= o_b2 &&
                  o_b2 + D <= o_n2 && ld_slab >= (long)o_n2 + D,
              "ctr_ffn_bwd_norms: slab layout");
  if (M <= 0) return 0;
  FfnArgs a = {};
  a.M = M; a.FF = FF; a.x = x; a.W1 = W1; a.b1 = b1; a.W2 = W2;
  a.drop = Drop{drop_key, drop_thresh, drop_scale};
  a.mask = (uint16_t*)const_cast<uint32_t*>(mask);
  a.slab = slab; a.ld_slab = ld_slab; a.o_b1 = o_b1; a.o_w2 = o_w2;
  a.o_w1 = o_w1; a.o_b2 = o_b2; a.o_n1 = o_n1; a.o_n2 = o_n2;
  a.dy = dy; a.h2 = h2; a.r2 = r2; a.nw2 = nw2; a.h1 = h1; a.r1 = r1; a.nw1 = nw1; a.dh1 = dh1;
  a.wbf = (__bf16*)const_cast<void*>(wbf);
  return ffn_dispatch(a, D, true, flags, (hipStream_t)stream);
}

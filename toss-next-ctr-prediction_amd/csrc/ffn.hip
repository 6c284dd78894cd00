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

  // h = x + (y + b2); RMSNorm over the row (the row's D values sit in the 16 lanes of one lane group)
#pragma unroll
  for (int i = 0; i < T::NI; ++i)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int row = 16 * i + 4 * g + rr, m = m0 + w * T::RW + row;
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

// ---------------------------------------------------------------- backward
// Norm-fused loader: dh2 = RMSNorm-backward(dy; h2, r2, nw2) for the tile's rows, written as the dh
// tile (rmsnorm_bwd_small's formula: dh = w dy r - h r^3/D sum_k w_k dy_k h_k); the workgroup's
// column sums of dh2 (ffn.3.bias grad) and of dy h2 r2 (norm2.w grad) go to the slab.  `red` holds
// 2 * 256 * 4 floats of scratch.
template <int D, bool PERM = false>
__device__ void load_dh_norm2(const FfnArgs& a, int m0, float* dst, float* red, float* slab) {
  using T = FfnTile<D>;
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
    slab[(which ? a.o_n2 : a.o_b2) + col] = sum;
  }
  __syncthreads();
}

// dx = dact W1 (complete over FF) + dh (residual path) for this wave's RW rows (dx[i][j][rr]: row
// 16i+4g+rr, col 16j+c; dw = the wave's rows of the dh tile); NORMS: the norm1 backward.  `scratch`:
// 4*D floats of LDS no wave still reads.
template <int D, bool NORMS, bool PERM = false>
__device__ __forceinline__ void ffn_bwd_epilogue(const FfnArgs& a, const f32x4 (&dxacc)[FfnTile<D>::NI][FfnTile<D>::NJ],
                                                 const float* dw, int m0, float* slab, float* scratch) {
  using T = FfnTile<D>;
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
  if (tid < D) slab[a.o_n1 + tid] = ((red[tid] + red[D + tid]) + red[2 * D + tid]) + red[3 * D + tid];
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

// buffer resources carry 32-bit byte extents: (M, D) activations, (FF, D) weights, the keep-bit words
static bool ffn_extent_ok(long M, int D, int FF) {
  const long lim = 1L << 31;
  return M * D * 4 < lim && (long)FF * D * 4 < lim && M * (FF / 16) * 2 < lim;
}

static int ffn_dispatch(const FfnArgs& a, int D, bool bwd, hipStream_t s) {
  switch (D) {
    case 16: launch_ffn<16>(a, bwd, s); break;
    case 32: launch_ffn<32>(a, bwd, s); break;
    default: launch_ffn<64>(a, bwd, s); break;
  }
  return check_launch(bwd ? "ffn_bwd" : "ffn_fwd");
}

}  // namespace ctr

using namespace ctr;

extern "C" int ctr_ffn_supported(int D, int FF) { return ffn_shape_ok(D, FF) ? 1 : 0; }

extern "C" int ctr_ffn_slab_rows(int M, int D) { return cdiv(M, D >= 64 ? 64 : 128); }

// enough for either keep-bit layout (FfnTile::LW)
extern "C" int ctr_ffn_mask_words(int M, int FF) {
  const long rowwords = ((long)M * (FF / 16) + 1) / 2;
  return (int)(lw_words(M, FF) > rowwords ? lw_words(M, FF) : rowwords);
}

extern "C" int ctr_ffn_fwd(const float* x, int M, int D, int FF, const float* W1, const float* b1, const float* W2,
                           const float* b2, const float* norm_w, float eps, uint32_t drop_key, uint32_t drop_thresh,
                           float drop_scale, uint32_t* mask, float* y, float* h, float* r, void* stream) {
  CTR_REQUIRE(ffn_shape_ok(D, FF), "ctr_ffn_fwd: needs D in {16,32,64} and FF % 16 == 0");
  CTR_REQUIRE(ffn_extent_ok(M, D, FF), "ctr_ffn_fwd: M x D too large for 32-bit buffer offsets");
  if (M <= 0) return 0;
  FfnArgs a = {};
  a.M = M; a.FF = FF; a.x = x; a.W1 = W1; a.b1 = b1; a.W2 = W2; a.b2 = b2; a.nw = norm_w; a.eps = eps;
  a.drop = Drop{drop_key, drop_thresh, drop_scale};
  a.mask = (uint16_t*)mask;
  a.y = y; a.h = h; a.r = r;
  return ffn_dispatch(a, D, false, (hipStream_t)stream);
}

extern "C" int ctr_ffn_bwd(const float* x, const float* dh, int M, int D, int FF, const float* W1, const float* b1,
                           const float* W2, uint32_t drop_key, uint32_t drop_thresh, float drop_scale,
                           const uint32_t* mask, float* dx, float* slab, long ld_slab, int o_b1, int o_w2,
                           void* stream) {
  CTR_REQUIRE(!drop_thresh || mask, "ctr_ffn_bwd with dropout needs the forward's keep bits");
  CTR_REQUIRE(ffn_shape_ok(D, FF), "ctr_ffn_bwd: needs D in {16,32,64} and FF % 16 == 0");
  CTR_REQUIRE(ffn_extent_ok(M, D, FF), "ctr_ffn_bwd: M x D too large for 32-bit buffer offsets");
  CTR_REQUIRE(o_b1 >= FF * D && o_w2 >= o_b1 + FF && ld_slab >= (long)o_w2 + (long)D * FF, "ctr_ffn_bwd: slab layout");
  if (M <= 0) return 0;
  FfnArgs a = {};
  a.M = M; a.FF = FF; a.x = x; a.W1 = W1; a.b1 = b1; a.W2 = W2;
  a.drop = Drop{drop_key, drop_thresh, drop_scale};
  a.mask = (uint16_t*)const_cast<uint32_t*>(mask);
  a.dh = dh; a.dx = dx; a.slab = slab; a.ld_slab = ld_slab; a.o_b1 = o_b1; a.o_w2 = o_w2;
  return ffn_dispatch(a, D, true, (hipStream_t)stream);
}

extern "C" int ctr_ffn_bwd_norms(const float* x, const float* dy, const float* h2, const float* r2, const float* nw2,
                                 const float* h1, const float* r1, const float* nw1, int M, int D, int FF,
                                 const float* W1, const float* b1, const float* W2, uint32_t drop_key,
                                 uint32_t drop_thresh, float drop_scale, const uint32_t* mask, float* dh1,
                                 float* slab, long ld_slab, int o_n1, int o_w1, int o_b1, int o_w2, int o_b2, int o_n2,
                                 void* stream) {
  CTR_REQUIRE(!drop_thresh || mask, "ctr_ffn_bwd_norms with dropout needs the forward's keep bits");
  CTR_REQUIRE(ffn_shape_ok(D, FF), "ctr_ffn_bwd_norms: needs D in {16,32,64} and FF % 16 == 0");
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
  return ffn_dispatch(a, D, true, (hipStream_t)stream);
}

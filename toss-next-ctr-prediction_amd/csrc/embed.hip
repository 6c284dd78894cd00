// Feature-embedding kernels: numeric/binary slope embeddings, hashed categorical gather +
// per-column projection, and the context / query vector.
//
//   feat_embed  : src/models/feature_embed.py:19-27, 42-48   out = (x*W + b) @ P^T
//   cat_embed   : src/models/wrapper.py:106-112, 149-150      e_c = T_c[X_cat[:,c]] @ P_c^T (+ emb dropout)
//   context     : src/models/wrapper.py:114-136               ctx means, ctx_mlp, S1 / S2 / concat query
#include "common.h"
#include "ctr_hip.h"

namespace ctr {

// ------------------------------------------------------------------------------------------------
// numeric / binary feature embedding
// ------------------------------------------------------------------------------------------------
// out[b, f, d] = sum_k (x[b,f] W[f,k] + bias[f,k]) P[d,k] = x[b,f] * A[f,d] + Bv[f,d] with
// A[f,d] = W[f,:].P[d,:], Bv[f,d] = bias[f,:].P[d,:] formed once per workgroup: the stream is then one
// FMA per output (the reference's per-k rounding differs by a few ulp).  Workgroup = (feature f, chunk
// of fe_rows(D) samples); lanes = d, so each sample's D outputs are one contiguous store.  A thread takes 32
// samples (one round trip for their x values; the per-workgroup projection staging amortised over 32 x 256 / D
// samples -- 64 per workgroup before, 5,248 workgroups a call at cfg2, ~21 us for 43 MB).
constexpr int FE_NB = 32;                           // samples per thread
__host__ __device__ __forceinline__ int fe_rows_d(int D) { return FE_NB * (256 / D); }

// One or two feature groups (numeric, binary) in one launch: the groups' workgroups side by side in the grid
// (group 1's after group 0's), each with its own x, weights and output -- one launch and one boundary fewer per
// direction than a launch per group.
struct FeGrp {
  const float* x;
  int F;
  const float* W;
  const float* bias;      // nullable
  const float* P;
  float* out;             // forward output (row stride ld) / backward: the incoming grad dout
  float* dW;
  float* dbias;           // nullable
  float* dP;
  float* ws;              // backward chunk partials (ctr_feat_embed_bwd_ws)
};
struct FeGrps {
  FeGrp g[2];
  int n;
  long ld;                // out / dout row stride
};
// block index along the groups' concatenation -> (group, index inside it)
__device__ __forceinline__ const FeGrp& fe_pick(const FeGrps& a, int& i, int per0) {
  if (a.n > 1 && i >= per0) {
    i -= per0;
    return a.g[1];
  }
  return a.g[0];
}

__global__ __launch_bounds__(256) void feat_embed_fwd_kernel(FeGrps ga, int B, int fe, int D) {
  extern __shared__ float sfe[];         // P [D][fe+1] | W row [fe] | bias row [fe]
  int f = blockIdx.y;
  const FeGrp& gr = fe_pick(ga, f, ga.g[0].F);
  const float* __restrict__ x = gr.x;
  const float* __restrict__ W = gr.W;
  const float* __restrict__ bias = gr.bias;
  const float* __restrict__ P = gr.P;
  float* __restrict__ out = gr.out;
  const int F = gr.F;
  const long out_ld = ga.ld;
  const int b0 = blockIdx.x * fe_rows_d(D);
  const int RG = 256 / D, d = threadIdx.x % D, rg = threadIdx.x / D;
  const int FP = fe + 1;
  float* sP = sfe;
  float* sW = sfe + D * FP;
  float* sB = sW + fe;
  for (int q = threadIdx.x; q < D * fe; q += 256) sP[(q / fe) * FP + q % fe] = P[q];
  for (int q = threadIdx.x; q < fe; q += 256) {
    sW[q] = W[(long)f * fe + q];
    sB[q] = bias ? bias[(long)f * fe + q] : 0.f;
  }
  __syncthreads();
  if (rg >= RG) return;
  float A = 0.f, Bv = 0.f;
  for (int k = 0; k < fe; ++k) {
    const float pk = sP[d * FP + k];
    A = fmaf(sW[k], pk, A);
    Bv = fmaf(sB[k], pk, Bv);
  }
  // the group's samples b0 + rg + RG i (i < FE_NB): every x load issued before the stores
  float xv[FE_NB];
#pragma unroll
  for (int i = 0; i < FE_NB; ++i) xv[i] = x[(long)min(b0 + rg + RG * i, B - 1) * F + f];
#pragma unroll
  for (int i = 0; i < FE_NB; ++i) {
    const int b = b0 + rg + RG * i;
    if (b < B) out[(long)b * out_ld + (long)f * D + d] = fmaf(xv[i], A, Bv);
  }
}

// per (feature f, sample chunk): S1[f,d] = sum_b x[b,f] dout[b,f,d], S0[f,d] = sum_b dout[b,f,d]
// lanes = d, 256/D row groups stride the chunk, combined in fixed order -> part[chunk][2][F][D]
__global__ __launch_bounds__(256) void feat_embed_bwd_sums(FeGrps ga, int B, int D, int rows_per_chunk) {
  __shared__ float r1[256], r0[256];
  int f = blockIdx.x;
  const FeGrp& gr = fe_pick(ga, f, ga.g[0].F);
  const float* __restrict__ x = gr.x;
  const float* __restrict__ dout = gr.out;
  float* __restrict__ part = gr.ws;
  const int F = gr.F;
  const long dout_ld = ga.ld;
  const int chunk = blockIdx.y, t = threadIdx.x;
  const int RG = 256 / D;
  const int d = t % D, rg = t / D;
  const int b0 = chunk * rows_per_chunk, b1 = min(B, b0 + rows_per_chunk);
  float s1 = 0.f, s0 = 0.f;
  if (rg < RG)
    for (int bb = b0 + rg; bb < b1; bb += 32 * RG) {    // 32 rows' loads issued together (a chunk's rows at D = 32),
      float gv[32], xv[32];                             // summed in row order
#pragma unroll
      for (int i = 0; i < 32; ++i) {
        const int b = min(bb + RG * i, b1 - 1);
        gv[i] = dout[(long)b * dout_ld + (long)f * D + d];
        xv[i] = x[(long)b * F + f];
      }
#pragma unroll
      for (int i = 0; i < 32; ++i) {
        if (bb + RG * i >= b1) break;
        s1 = fmaf(xv[i], gv[i], s1);
        s0 += gv[i];
      }
    }
  r1[t] = s1;
  r0[t] = s0;
  __syncthreads();
  if (t < D) {
    float a = 0.f, c = 0.f;
    for (int g = 0; g < RG; ++g) {
      a += r1[g * D + t];
      c += r0[g * D + t];
    }
    float* o = part + (long)chunk * 2 * F * D;
    o[(long)f * D + t] = a;
    o[(long)F * D + (long)f * D + t] = c;
  }
}

// F + D workgroups (one per output row; one workgroup for all of it took ~19 us, a chain of round trips):
// workgroup f < F sums the chunk partials of S1[f, :], S0[f, :] (fixed chunk order) and forms dW[f, :] = S1[f] @ P,
// dbias[f, :] = S0[f] @ P; workgroup F + d sums those of S1[:, d], S0[:, d] and forms dP[d, :] = sum_f (S1[f, d]
// W[f, :] + S0[f, d] bias[f, :]) in feature order -- the same sums, products and orders as the one-workgroup form
__global__ __launch_bounds__(256) void feat_embed_bwd_final(FeGrps ga, int nchunk, int D, int fe) {
  extern __shared__ float sfb[];       // row f: S [2][D] | P [D][fe];  column d: S [2][F] | W [F][fe] | bias [F][fe]
  int blk = blockIdx.x;
  const FeGrp& gr = fe_pick(ga, blk, ga.g[0].F + D);
  const float* __restrict__ part = gr.ws;
  const float* __restrict__ W = gr.W;
  const float* __restrict__ bias = gr.bias;
  const float* __restrict__ P = gr.P;
  float* __restrict__ dW = gr.dW;
  float* __restrict__ dbias = gr.dbias;
  float* __restrict__ dP = gr.dP;
  const int F = gr.F;
  const int tid = threadIdx.x;
  const long n2 = 2L * F * D;
  const bool rowf = blk < F;
  const int f = blk, dd = blk - F;
  const int nS = rowf ? 2 * D : 2 * F;
  for (int q = tid; q < nS; q += 256) {
    // element of S (S1 then S0): row f -> (h, d) = (q / D, q % D); column d -> (h, f) = (q / F, q % F)
    const long idx = rowf ? (long)(q / D) * F * D + (long)f * D + q % D : (long)(q / F) * F * D + (long)(q % F) * D + dd;
    float v[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) v[c] = part[(long)min(c, nchunk - 1) * n2 + idx];
    float t = 0.f;
#pragma unroll
    for (int c = 0; c < 16; ++c)
      if (c < nchunk) t += v[c];
    sfb[q] = t;
  }
  float* sw = sfb + nS;
  if (rowf) {
    for (int q = tid; q < D * fe; q += 256) sw[q] = P[q];
  } else {
    for (int q = tid; q < F * fe; q += 256) {
      sw[q] = W[q];
      sw[F * fe + q] = bias ? bias[q] : 0.f;
    }
  }
  __syncthreads();
  if (rowf) {
    const float* S1 = sfb;
    const float* S0 = sfb + D;
    for (int k = tid; k < fe; k += 256) {
      float a = 0.f, c = 0.f;
      for (int d = 0; d < D; ++d) {
        a = fmaf(S1[d], sw[d * fe + k], a);
        c = fmaf(S0[d], sw[d * fe + k], c);
      }
      dW[(long)f * fe + k] = a;
      if (dbias) dbias[(long)f * fe + k] = c;
    }
  } else {
    const float* S1 = sfb;
    const float* S0 = sfb + F;
    const float* sb = sw + F * fe;
    for (int k = tid; k < fe; k += 256) {
      float a = 0.f;
      for (int ff = 0; ff < F; ++ff) {
        a = fmaf(S1[ff], sw[ff * fe + k], a);
        if (bias) a = fmaf(S0[ff], sb[ff * fe + k], a);
      }
      dP[(long)dd * fe + k] = a;
    }
  }
}

// ------------------------------------------------------------------------------------------------
// hashed categorical embeddings: one thread per (b, c, d); the D threads of a (b, c) share the row
// ------------------------------------------------------------------------------------------------
struct CatMeta {
  const float* tabs;      // table storage: the arena, or (row-sharded tables) the batch's fetched rows
  const long* tab_off;    // element offset of table c in tabs
  const long* proj_off;   // element offset of proj c ([D][d_c]) in the arena
  const int* dims;        // d_c
  int row_ld;             // row stride of every table in tabs (0: d_c)
};

// Workgroup = (categorical c, 64 samples): the projection P_c (D x d_c) and the block's gathered table
// rows are staged in LDS once, then thread (sample i, dim d) forms sum_k T[i][k] P_c[d][k] from LDS
// (row values broadcast across the D lanes of a sample, P_c rows at a 65-float stride: no bank conflicts).
// The per-output arithmetic (fmaf over k in order) is unchanged from a thread-per-output form, whose
// strided P_c reads (32 cache lines per load instruction) bounded it.
constexpr int CE_SPB = 64;     // samples per workgroup
constexpr int CE_LD = 65;      // LDS row stride (floats)

__global__ __launch_bounds__(256) void cat_embed_fwd_kernel(const int* __restrict__ xcat, int B, int Fc,
                                                            const float* __restrict__ arena, CatMeta cm, int D,
                                                            float* __restrict__ cat_e, float* __restrict__ xf,
                                                            long xf_ld, Drop drop) {
  __shared__ float sP[64 * CE_LD];
  __shared__ float sT[CE_SPB * CE_LD];
  const int c = blockIdx.x, tid = threadIdx.x;
  const int dc = cm.dims[c];
  const int b0 = blockIdx.y * CE_SPB, nb = min(CE_SPB, B - b0);
  const float* P = arena + cm.proj_off[c];
  for (int e = tid; e < D * dc; e += 256) {
    const int d = e / dc, k = e - d * dc;
    sP[d * CE_LD + k] = P[e];
  }
  const float* T = cm.tabs + cm.tab_off[c];
  const long tld = cm.row_ld ? cm.row_ld : dc;
  __shared__ int sidx[CE_SPB];
  if (tid < nb) sidx[tid] = xcat[(long)(b0 + tid) * Fc + c];
  __syncthreads();
  // (sample, element) items over the table's dc elements only, the row ids from LDS and a thread's (up to 16)
  // gathers issued together (an id -> row load chain per item left the staging latency-bound)
  {
    constexpr int EPT = CE_SPB * 64 / 256;
    float tv[EPT];
#pragma unroll
    for (int u = 0; u < EPT; ++u) {
      const int e = tid + 256 * u;
      if (e < nb * dc) {
        const int i = e / dc, k = e - i * dc;
        tv[u] = T[(long)sidx[i] * tld + k];
      }
    }
#pragma unroll
    for (int u = 0; u < EPT; ++u) {
      const int e = tid + 256 * u;
      if (e < nb * dc) {
        const int i = e / dc, k = e - i * dc;
        sT[i * CE_LD + k] = tv[u];
      }
    }
  }
  __syncthreads();
  for (int e = tid; e < nb * D; e += 256) {
    const int i = e / D, d = e - i * D;
    const float* t = sT + i * CE_LD;
    const float* pp = sP + d * CE_LD;
    float acc = 0.f;
#pragma unroll 8
    for (int k = 0; k < dc; ++k) acc = fmaf(t[k], pp[k], acc);
    const uint32_t q = ((uint32_t)(b0 + i) * Fc + c) * D + d;
    cat_e[q] = acc;
    if (xf) xf[(long)(b0 + i) * xf_ld + (long)c * D + d] = drop_apply(drop, q, acc);
  }
}

// row-grad contributions: contrib[(b*Fc+c)*64 + k] = sum_d dcat[b,c,d] P_c[d,k]  (zero-padded to 64)
// keys[b*Fc+c] = row_base[c] + X_cat[b,c].  Same (c, 64 samples) workgroups and LDS staging as the forward.
__global__ __launch_bounds__(256) void cat_embed_bwd_rows(const int* __restrict__ xcat, int B, int Fc,
                                                          const float* __restrict__ arena, CatMeta cm, int D,
                                                          const float* __restrict__ dcat,
                                                          const uint32_t* __restrict__ row_base,
                                                          float* __restrict__ contrib, uint32_t* __restrict__ keys) {
  __shared__ float sP[64 * CE_LD];
  __shared__ float sG[CE_SPB * CE_LD];
  const int c = blockIdx.x, tid = threadIdx.x;
  const int dc = cm.dims[c];
  const int b0 = blockIdx.y * CE_SPB, nb = min(CE_SPB, B - b0);
  const float* P = arena + cm.proj_off[c];
  for (int e = tid; e < D * dc; e += 256) {
    const int d = e / dc, k = e - d * dc;
    sP[d * CE_LD + k] = P[e];
  }
  for (int e = tid; e < nb * D; e += 256) {
    const int i = e / D, d = e - i * D;
    sG[i * CE_LD + d] = dcat[((long)(b0 + i) * Fc + c) * D + d];
  }
  __syncthreads();
  // items (sample, k < dc) only: the columns past d_c of a contribution row stay zero from the buffer's first fill
  // (a slot (b, c) always holds table c), so the 64-wide rows' padding is not rewritten every step
  for (int e = tid; e < nb * dc; e += 256) {
    const int i = e / dc, k = e - i * dc;
    const long bc = (long)(b0 + i) * Fc + c;
    const float* g = sG + i * CE_LD;
    float acc = 0.f;
#pragma unroll 8
    for (int d = 0; d < D; ++d) acc = fmaf(g[d], sP[d * CE_LD + k], acc);
    contrib[bc * 64 + k] = acc;
  }
  if (tid < nb) {
    const long bc = (long)(b0 + tid) * Fc + c;
    keys[bc] = row_base[c] + (uint32_t)xcat[bc];
  }
}

// dP_c[d,k] = sum_b dcat[b,c,d] * T_c[row_b, k]   -- block (c, chunk) partials over a row chunk.
// The chunk's gathered table rows and dcat rows are staged in LDS 64 samples at a time (the gather is
// the latency-bound part).  Each thread owns a 4x4 (d, k) register tile and reads its operands as two
// 16-byte LDS loads per row; when D x dc has fewer than 256/4x4 tiles the block's threads split the rows
// into groups (row i -> group i % ngrp), whose tiles are summed in fixed group order at the end.
constexpr int CP_SUB = 64;
constexpr int CP_LD = 68;        // LDS row stride (floats): 16-byte aligned, rows offset by 4 banks

__global__ __launch_bounds__(256) void cat_embed_bwd_proj_partial(const int* __restrict__ xcat, int B, int Fc,
                                                                  const float* __restrict__ arena, CatMeta cm,
                                                                  int D, const float* __restrict__ dcat,
                                                                  int rows_per_chunk, float* __restrict__ part) {
  __shared__ __attribute__((aligned(16))) float sT[CP_SUB * CP_LD];
  __shared__ __attribute__((aligned(16))) float sG[CP_SUB * CP_LD];
  const int c = blockIdx.x, chunk = blockIdx.y;
  const int dc = cm.dims[c];
  const int b0 = chunk * rows_per_chunk, b1 = min(B, b0 + rows_per_chunk);
  const float* T = cm.tabs + cm.tab_off[c];
  const long tld = cm.row_ld ? cm.row_ld : dc;
  float* out = part + ((long)chunk * Fc + c) * (64 * 64);
  const int nd4 = (D + 3) >> 2, nk4 = (dc + 3) >> 2;
  const int ntile = nd4 * nk4;                       // <= 256
  const int ngrp = 256 / ntile;
  const int tile = threadIdx.x % ntile, grp = threadIdx.x / ntile;
  const bool active = grp < ngrp;
  const int d0 = (tile / nk4) * 4, k0 = (tile % nk4) * 4;
  float acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = 0.f;
  __shared__ int sidx[CP_SUB];
  for (int s0 = b0; s0 < b1; s0 += CP_SUB) {
    const int ns = min(CP_SUB, b1 - s0);
    __syncthreads();
    // the sub-chunk's row ids first (one load each), then every thread's 16 gathers in flight at once: the
    // per-element id -> row load chain left the staging latency-bound (wait-mem 0.81)
    if (threadIdx.x < CP_SUB) sidx[threadIdx.x] = threadIdx.x < ns ? xcat[(long)(s0 + threadIdx.x) * Fc + c] : 0;
    __syncthreads();
    constexpr int EPT = CP_SUB * 64 / 256;
    float tv[EPT], gv[EPT];
#pragma unroll
    for (int u = 0; u < EPT; ++u) {
      const int e = threadIdx.x + 256 * u, i = e >> 6, k = e & 63;
      tv[u] = 0.f;
      gv[u] = 0.f;
      if (i < ns) {
        const long b = s0 + i;
        if (k < dc) tv[u] = T[(long)sidx[i] * tld + k];
        if (k < D) gv[u] = dcat[(b * Fc + c) * D + k];
      }
    }
#pragma unroll
    for (int u = 0; u < EPT; ++u) {
      const int e = threadIdx.x + 256 * u, i = e >> 6, k = e & 63;
      sT[i * CP_LD + k] = tv[u];
      sG[i * CP_LD + k] = gv[u];
    }
    __syncthreads();
    if (active) {
      for (int i = grp; i < ns; i += ngrp) {
        const float4 g = *reinterpret_cast<const float4*>(&sG[i * CP_LD + d0]);
        const float4 tv = *reinterpret_cast<const float4*>(&sT[i * CP_LD + k0]);
        const float gg[4] = {g.x, g.y, g.z, g.w};
        const float tt[4] = {tv.x, tv.y, tv.z, tv.w};
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int v = 0; v < 4; ++v) acc[u][v] = fmaf(gg[u], tt[v], acc[u][v]);
      }
    }
  }
  // fixed-order sum over the row groups (through LDS), then the (d, k) tile store
  __syncthreads();
  float* red = sT;                                   // ngrp * ntile * 16 <= 4096 floats
  if (active && grp > 0) {
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int v = 0; v < 4; ++v) red[((grp * ntile) + tile) * 16 + u * 4 + v] = acc[u][v];
  }
  __syncthreads();
  if (active && grp == 0) {
    for (int g2 = 1; g2 < ngrp; ++g2)
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int v = 0; v < 4; ++v) acc[u][v] += red[((g2 * ntile) + tile) * 16 + u * 4 + v];
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int d = d0 + u, k = k0 + v;
        if (d < D && k < dc) out[d * dc + k] = acc[u][v];
      }
  }
}

// one thread per (c, output q): the nchunk partials summed in chunk order, eight loads in flight
__global__ __launch_bounds__(256) void cat_embed_bwd_proj_final(int nchunk, int Fc, int D, CatMeta cm,
                                                                const long* __restrict__ proj_goff,
                                                                const float* __restrict__ part,
                                                                float* __restrict__ grad) {
  const int c = blockIdx.x;
  const int dc = cm.dims[c];
  const int q = blockIdx.y * 256 + threadIdx.x;
  if (q >= D * dc) return;
  const float* pc = part + (long)c * (64 * 64) + q;
  const long cs = (long)Fc * (64 * 64);
  float s = 0.f;
  int ch = 0;
  for (; ch + 8 <= nchunk; ch += 8) {
    float a[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] = pc[(ch + j) * cs];
#pragma unroll
    for (int j = 0; j < 8; ++j) s += a[j];
  }
  for (; ch < nchunk; ++ch) s += pc[ch * cs];
  grad[proj_goff[c] + q] = s;
}

// ------------------------------------------------------------------------------------------------
// context + query: one wave per sample; lane = output dim d (D <= 64)
// ------------------------------------------------------------------------------------------------
struct CtxArgs {
  const float* num_e; long num_ld; int Fn;    // (B, Fn, D) rows at stride num_ld
  const float* mask_e; long mask_ld; int Fm;
  const float* cat_e; int Fc;                 // (B, Fc, D) contiguous, pre-dropout
  int D, B, mode, qi;                         // mode 0 S1, 1 S2, 2 concat
  const float* Wc; const float* bc;           // ctx_mlp.0 (D, nctx*D), (D)
  float* ctx;                                 // (B, nctx*D)
  float* hq;                                  // (B, D) relu(ctx_mlp) output
  float* query;                               // (B, D)
};

// One wave per sample (4 per workgroup): lane = (part pp = lane / D, dim d = lane % D), P = 64 / D parts;
// part pp sums features pp, pp + P, ... and the parts combine in fixed order through the wave's LDS row.
// Then the ctx_mlp row and the query (lane = d).
__device__ __forceinline__ float ctx_wave_mean(const float* __restrict__ x, int F, int D, float* sp) {
  const int lane = threadIdx.x & 63;
  if ((D & 3) == 0 && (((uintptr_t)x) & 15) == 0) {
    // 16-byte loads: lane = (part pp, column quad dq), P = 64 / (D/4) parts; sp holds 4 floats per lane, so
    // element d of part pp sits at sp[pp * D + d]
    typedef float f4 __attribute__((ext_vector_type(4)));
    const int Dq = D >> 2, P = 64 / Dq;
    const int dq = lane % Dq, pp = lane / Dq;
    f4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = {0.f, 0.f, 0.f, 0.f};
    if (pp < P) {
      // the part's features i = 0, 1, ... (f = pp + i P): even i into a0, odd into a1, eight loads issued before
      // their adds (two per iteration left one round trip per pair of loads)
      const f4* x4 = (const f4*)x;
      const int nf = F > pp ? (F - pp + P - 1) / P : 0;
      for (int i0 = 0; i0 < nf; i0 += 8) {
        f4 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int i = i0 + u < nf ? i0 + u : nf - 1;
          v[u] = x4[(long)(pp + i * P) * Dq + dq];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          if (i0 + u < nf) {
            if (u & 1) a1 += v[u];
            else a0 += v[u];
          }
        }
      }
    }
    const f4 v = a0 + a1;
    if (pp < P) *(f4*)&sp[(pp * Dq + dq) * 4] = v;
    __builtin_amdgcn_wave_barrier();
    float m = 0.f;
    if (lane < D) {
      for (int q = 0; q < P; ++q) m += sp[q * D + lane];
      m = m / (float)F;
    }
    __builtin_amdgcn_wave_barrier();
    return m;
  }
  const int P = 64 / D;
  const int d = lane % D, pp = lane / D;
  float s0 = 0.f, s1 = 0.f;
  if (pp < P) {
    int f = pp;
    for (; f + P < F; f += 2 * P) {
      s0 += x[(long)f * D + d];
      s1 += x[(long)(f + P) * D + d];
    }
    if (f < F) s0 += x[(long)f * D + d];
  }
  sp[lane] = s0 + s1;
  __builtin_amdgcn_wave_barrier();
  float m = 0.f;
  if (lane < D) {
    for (int q = 0; q < P; ++q) m += sp[q * D + lane];
    m = m / (float)F;
  }
  __builtin_amdgcn_wave_barrier();
  return m;
}

__global__ __launch_bounds__(256) void context_fwd_kernel(CtxArgs a) {
  __shared__ float sctx_all[4][3 * 64];
  __shared__ __attribute__((aligned(16))) float sp_all[4][256];
  const int w = threadIdx.x >> 6, t = threadIdx.x & 63;
  const int b = blockIdx.x * 4 + w;
  if (b >= a.B) return;
  float* sctx = sctx_all[w];
  float* sp = sp_all[w];
  const int D = a.D;
  int nctx = 0;
  if (a.Fn > 0) {
    const float m = ctx_wave_mean(a.num_e + (long)b * a.num_ld, a.Fn, D, sp);
    if (t < D) sctx[nctx * D + t] = m;
    ++nctx;
  }
  if (a.Fm > 0) {
    const float m = ctx_wave_mean(a.mask_e + (long)b * a.mask_ld, a.Fm, D, sp);
    if (t < D) sctx[nctx * D + t] = m;
    ++nctx;
  }
  if (a.Fc > 0) {
    const float m = ctx_wave_mean(a.cat_e + (long)b * a.Fc * D, a.Fc, D, sp);
    if (t < D) sctx[nctx * D + t] = m;
  } else if (t < D) {
    sctx[nctx * D + t] = 0.f;
  }
  ++nctx;
  __builtin_amdgcn_wave_barrier();
  const int W = nctx * D;
  for (int j = t; j < W; j += 64) a.ctx[(long)b * W + j] = sctx[j];
  if (t < D) {
    const int d = t;
    float q;
    float h = 0.f;
    if (a.mode != 0) {
      float acc = 0.f;
#pragma unroll 8
      for (int j = 0; j < W; ++j) acc = fmaf(sctx[j], a.Wc[(long)d * W + j], acc);
      h = acc + a.bc[d];
      h = h > 0.f ? h : 0.f;
      a.hq[(long)b * D + d] = h;
    }
    const float qc = a.mode != 1 ? a.cat_e[((long)b * a.Fc + a.qi) * D + d] : 0.f;
    if (a.mode == 0) q = qc;
    else if (a.mode == 1) q = h;
    else q = 0.5f * (qc + h);
    a.query[(long)b * D + d] = q;
  }
}

struct CtxBwdArgs {
  CtxArgs f;
  const float* dquery;      // (B, D)
  const float* dxf_cat;     // (B, Fc*D) slice of dxF at row stride dxf_ld (nullable)
  long dxf_ld;
  Drop emb_drop;            // dropout applied on the xF cat slot
  const float* dfc;         // fc-head input grad (B, nfc*D) (nullable): [u | num_mean | mask_mean | cat...]
  long dfc_ld;
  float* dnum;              // (B, Fn, D) rows at stride num_ld: += dctx_num / Fn (+ fc mean grad)
  float* dmask;             // (B, Fm, D) rows at stride mask_ld
  float* dcat;              // (B, Fc, D) written
  float* dpre;              // (B, D) grad of ctx_mlp pre-activation (for dWc, dbc); nullable in S1
};

// One 256-thread block per sample: the small dpre / dctx products first, then the three per-feature
// broadcasts (dnum += g_num[d], dmask += g_mask[d], dcat = ...) as flat element loops over the sample's
// contiguous F*D slices, so every wave instruction moves 256 contiguous bytes (the earlier one-wave form
// left half of its lanes idle at D = 32 and walked F serially).
constexpr int CTXB_T = 256;

__global__ __launch_bounds__(CTXB_T) void context_bwd_kernel(CtxBwdArgs a) {
  __shared__ float sdp[64];
  __shared__ float sdctx[3 * 64];
  __shared__ float sg[3][64];        // per-slot broadcast grads: num / Fn, mask / Fm, cat / Fc
  __shared__ float sq[64];           // the query's grad on the query cat slot
  const CtxArgs& f = a.f;
  const int b = blockIdx.x, t = threadIdx.x, D = f.D;
  const int nctx = (f.Fn > 0) + (f.Fm > 0) + 1;
  const int W = nctx * D;
  if (t < 64) {
    float dqv = t < D ? a.dquery[(long)b * D + t] : 0.f;
    float dh = 0.f;
    if (t < D && f.mode != 0) {
      dh = f.mode == 2 ? 0.5f * dqv : dqv;
      dh = f.hq[(long)b * D + t] > 0.f ? dh : 0.f;
      if (a.dpre) a.dpre[(long)b * D + t] = dh;
    }
    sdp[t] = dh;
    sq[t] = f.mode == 1 ? 0.f : (f.mode == 2 ? 0.5f * dqv : dqv);
  }
  __syncthreads();
  // dctx[j] = sum_d dpre[d] * Wc[d, j]   (W <= 192 < 256)
  if (t < W) {
    float acc = 0.f;
    if (f.mode != 0)
#pragma unroll 8
      for (int i = 0; i < D; ++i) acc = fmaf(sdp[i], f.Wc[(long)i * W + t], acc);
    sdctx[t] = acc;
  }
  __syncthreads();
  // fc layout: [u, num_mean?, mask_mean?, cat_0 .. cat_{Fc-1}]
  if (t < D) {
    int slot = 0, fcslot = 1;
    if (f.Fn > 0) {
      float g = sdctx[slot * D + t];
      if (a.dfc) g += a.dfc[(long)b * a.dfc_ld + (long)fcslot * D + t];
      sg[0][t] = g / (float)f.Fn;
      ++slot;
      ++fcslot;
    }
    if (f.Fm > 0) {
      float g = sdctx[slot * D + t];
      if (a.dfc) g += a.dfc[(long)b * a.dfc_ld + (long)fcslot * D + t];
      sg[1][t] = g / (float)f.Fm;
      ++slot;
    }
    sg[2][t] = f.Fc > 0 ? sdctx[slot * D + t] / (float)f.Fc : 0.f;
  }
  __syncthreads();
  // dnum += g_num[d], dmask += g_mask[d]: 16-byte read-modify-writes when the rows allow it
  // (each thread's read-modify-writes in groups of four: the group's loads issued before its stores -- in a plain
  // loop every load followed the previous store to the same array, one round trip per element)
  auto bcast_add = [&](float* dst, int F, const float* g) {
    const int n = F * D;
    if ((D & 3) == 0 && (((uintptr_t)dst) & 15) == 0) {
      typedef float f4 __attribute__((ext_vector_type(4)));
      f4* d4 = (f4*)dst;
      const int n4 = n >> 2;
      for (int e0 = t; e0 < n4; e0 += 4 * CTXB_T) {
        f4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = d4[min(e0 + u * CTXB_T, n4 - 1)];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int e4 = e0 + u * CTXB_T;
          if (e4 < n4) {
            const int d = (e4 << 2) % D;
            d4[e4] = v[u] + f4{g[d], g[d + 1], g[d + 2], g[d + 3]};
          }
        }
      }
    } else {
      for (int e = t; e < n; e += CTXB_T) dst[e] += g[e % D];
    }
  };
  if (f.Fn > 0) bcast_add(a.dnum + (long)b * f.num_ld, f.Fn, sg[0]);
  if (f.Fm > 0) bcast_add(a.dmask + (long)b * f.mask_ld, f.Fm, sg[1]);
  const int fc0 = 1 + (f.Fn > 0) + (f.Fm > 0);
  const int n = f.Fc * D;
  for (int e0 = t; e0 < n; e0 += 8 * CTXB_T) {      // eight elements' loads per thread issued together
    float gx[8], gf[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = min(e0 + u * CTXB_T, n - 1);
      gx[u] = a.dxf_cat ? a.dxf_cat[(long)b * a.dxf_ld + e] : 0.f;
      gf[u] = a.dfc ? a.dfc[(long)b * a.dfc_ld + (long)fc0 * D + e] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = e0 + u * CTXB_T;
      if (e >= n) break;
      const int c = e / D, d = e - c * D;
      const long q = (long)b * n + e;
      float g = 0.f;
      if (a.dxf_cat) g = a.emb_drop.thresh ? (drop_keep(a.emb_drop, (uint32_t)q) ? gx[u] * a.emb_drop.scale : 0.f) : gx[u];
      if (a.dfc) g += gf[u];
      if (c == f.qi) g += sq[d];
      g += sg[2][d];
      a.dcat[q] = g;
    }
  }
}

}  // namespace ctr

using namespace ctr;

static int fe_fwd(const FeGrps& ga, int B, int fe, int D, hipStream_t s) {
  const int Ft = ga.g[0].F + (ga.n > 1 ? ga.g[1].F : 0);
  if (B == 0 || Ft == 0) return 0;
  CTR_REQUIRE(D <= 256, "D > 256");
  const size_t sm = ((size_t)D * (fe + 1) + 2 * fe) * sizeof(float);
  CTR_REQUIRE(sm <= 64 * 1024, "feat_embed: D x fe projection exceeds LDS");
  feat_embed_fwd_kernel<<<dim3(cdiv(B, fe_rows_d(D)), Ft), 256, sm, s>>>(ga, B, fe, D);
  return check_launch("feat_embed_fwd");
}

extern "C" int ctr_feat_embed_fwd(const float* x, int B, int F, const float* W, const float* bias, const float* P,
                                  int fe, int D, float* out, long out_ld, void* stream) {
  FeGrps ga{};
  ga.g[0] = FeGrp{x, F, W, bias, P, out, nullptr, nullptr, nullptr, nullptr};
  ga.n = 1;
  ga.ld = out_ld;
  return fe_fwd(ga, B, fe, D, (hipStream_t)stream);
}

extern "C" int ctr_feat_embed_fwd2(const float* x0, int F0, const float* W0, const float* bias0, const float* P0,
                                   float* out0, const float* x1, int F1, const float* W1, const float* bias1,
                                   const float* P1, float* out1, int B, int fe, int D, long out_ld, void* stream) {
  FeGrps ga{};
  ga.g[0] = FeGrp{x0, F0, W0, bias0, P0, out0, nullptr, nullptr, nullptr, nullptr};
  ga.g[1] = FeGrp{x1, F1, W1, bias1, P1, out1, nullptr, nullptr, nullptr, nullptr};
  ga.n = 2;
  ga.ld = out_ld;
  CTR_REQUIRE(F0 > 0 && F1 > 0, "ctr_feat_embed_fwd2: both groups need features");
  return fe_fwd(ga, B, fe, D, (hipStream_t)stream);
}

static int fe_chunks(int B) { return std::max(1, std::min(16, cdiv(B, 256))); }   // <= 16: feat_embed_bwd_final

extern "C" size_t ctr_feat_embed_bwd_ws(int B, int F, int D) {
  return (size_t)fe_chunks(B) * 2 * F * D * sizeof(float);
}

static int fe_bwd(const FeGrps& ga, int B, int fe, int D, hipStream_t s) {
  const int F0 = ga.g[0].F, F1 = ga.n > 1 ? ga.g[1].F : 0, Fmax = std::max(F0, F1);
  if (F0 + F1 == 0) return 0;
  CTR_REQUIRE(D <= 256, "D > 256");
  const size_t sm_row = ((size_t)2 * D + (size_t)D * fe) * sizeof(float);
  const size_t sm_col = ((size_t)2 * Fmax + (size_t)2 * Fmax * fe) * sizeof(float);
  const size_t sm = sm_row > sm_col ? sm_row : sm_col;
  CTR_REQUIRE(sm <= 160 * 1024, "feat_embed_bwd: sums + weights exceed LDS");
  const int nch = fe_chunks(B);
  const int rpc = cdiv(B, nch);
  feat_embed_bwd_sums<<<dim3(F0 + F1, nch), 256, 0, s>>>(ga, B, D, rpc);
  if (sm > 64 * 1024)
    (void)hipFuncSetAttribute((const void*)feat_embed_bwd_final, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm);
  feat_embed_bwd_final<<<F0 + D + (ga.n > 1 ? F1 + D : 0), 256, sm, s>>>(ga, nch, D, fe);
  return check_launch("feat_embed_bwd");
}

extern "C" int ctr_feat_embed_bwd(const float* x, int B, int F, const float* W, const float* bias, const float* P,
                                  int fe, int D, const float* dout, long dout_ld, float* dW, float* dbias,
                                  float* dP, float* ws, void* stream) {
  if (F == 0) return 0;
  FeGrps ga{};
  ga.g[0] = FeGrp{x, F, W, bias, P, const_cast<float*>(dout), dW, dbias, dP, ws};
  ga.n = 1;
  ga.ld = dout_ld;
  return fe_bwd(ga, B, fe, D, (hipStream_t)stream);
}

extern "C" int ctr_feat_embed_bwd2(const float* x0, int F0, const float* W0, const float* bias0, const float* P0,
                                   const float* dout0, float* dW0, float* dbias0, float* dP0, float* ws0,
                                   const float* x1, int F1, const float* W1, const float* bias1, const float* P1,
                                   const float* dout1, float* dW1, float* dbias1, float* dP1, float* ws1, int B, int fe,
                                   int D, long dout_ld, void* stream) {
  CTR_REQUIRE(F0 > 0 && F1 > 0, "ctr_feat_embed_bwd2: both groups need features");
  FeGrps ga{};
  ga.g[0] = FeGrp{x0, F0, W0, bias0, P0, const_cast<float*>(dout0), dW0, dbias0, dP0, ws0};
  ga.g[1] = FeGrp{x1, F1, W1, bias1, P1, const_cast<float*>(dout1), dW1, dbias1, dP1, ws1};
  ga.n = 2;
  ga.ld = dout_ld;
  return fe_bwd(ga, B, fe, D, (hipStream_t)stream);
}

extern "C" int ctr_cat_embed_fwd(const int* xcat, int B, int Fc, const float* arena, const float* tab_base,
                                 const long* tab_off, const long* proj_off, const int* dims, int row_ld, int D,
                                 float* cat_e, float* xf, long xf_ld,
                                 uint32_t drop_key, uint32_t drop_thresh, float drop_scale, void* stream) {
  if (B == 0 || Fc == 0) return 0;
  CTR_REQUIRE((long)B * Fc * 64 < (1L << 32), "cat_embed: B*Fc*64 must fit 32-bit indexing");
  CTR_REQUIRE(row_ld >= 0 && row_ld <= 64, "cat_embed: row_ld must be in [0, 64]");
  CatMeta cm{tab_base ? tab_base : arena, tab_off, proj_off, dims, row_ld};
  CTR_REQUIRE(D <= 64, "cat_embed: D > 64");
  cat_embed_fwd_kernel<<<dim3(Fc, cdiv(B, CE_SPB)), 256, 0, (hipStream_t)stream>>>(
      xcat, B, Fc, arena, cm, D, cat_e, xf, xf_ld, Drop{drop_key, drop_thresh, drop_scale});
  return check_launch("cat_embed_fwd");
}

constexpr int CP_RPC = 64;     // rows per projection-grad partial (one LDS sub-chunk per workgroup)

extern "C" size_t ctr_cat_embed_bwd_ws(int B, int Fc) {
  int nchunk = (B + CP_RPC - 1) / CP_RPC;
  return (size_t)nchunk * Fc * 64 * 64 * sizeof(float);
}

extern "C" int ctr_cat_embed_bwd(const int* xcat, int B, int Fc, const float* arena, const float* tab_base,
                                 const long* tab_off, const long* proj_off, const int* dims, int row_ld, int D,
                                 const float* dcat,
                                 const uint32_t* row_base, float* contrib, uint32_t* keys, float* grad_arena,
                                 const long* proj_goff, float* ws, void* stream) {
  if (B == 0 || Fc == 0) return 0;
  CTR_REQUIRE(D <= 64, "D > 64");
  CTR_REQUIRE((long)B * Fc * 64 < (1L << 32), "cat_embed: B*Fc*64 must fit 32-bit indexing");
  CTR_REQUIRE(row_ld >= 0 && row_ld <= 64, "cat_embed: row_ld must be in [0, 64]");
  hipStream_t s = (hipStream_t)stream;
  CatMeta cm{tab_base ? tab_base : arena, tab_off, proj_off, dims, row_ld};
  cat_embed_bwd_rows<<<dim3(Fc, cdiv(B, CE_SPB)), 256, 0, s>>>(xcat, B, Fc, arena, cm, D, dcat, row_base, contrib,
                                                                keys);
  const int rpc = CP_RPC;
  const int nchunk = (B + rpc - 1) / rpc;
  cat_embed_bwd_proj_partial<<<dim3(Fc, nchunk), 256, 0, s>>>(xcat, B, Fc, arena, cm, D, dcat, rpc, ws);
  cat_embed_bwd_proj_final<<<dim3(Fc, cdiv(D * 64, 256)), 256, 0, s>>>(nchunk, Fc, D, cm, proj_goff, ws,
                                                                        grad_arena);
  return check_launch("cat_embed_bwd");
}

extern "C" int ctr_context_fwd(const float* num_e, long num_ld, int Fn, const float* mask_e, long mask_ld, int Fm,
                               const float* cat_e, int Fc, int D, int B, int mode, int qi, const float* Wc,
                               const float* bc, float* ctx, float* hq, float* query, void* stream) {
  if (B == 0) return 0;
  CTR_REQUIRE(D <= 64, "D > 64");
  CtxArgs a{num_e, num_ld, Fn, mask_e, mask_ld, Fm, cat_e, Fc, D, B, mode, qi, Wc, bc, ctx, hq, query};
  context_fwd_kernel<<<cdiv(B, 4), 256, 0, (hipStream_t)stream>>>(a);
  return check_launch("context_fwd");
}

extern "C" int ctr_context_bwd(const float* num_e, long num_ld, int Fn, const float* mask_e, long mask_ld, int Fm,
                               const float* cat_e, int Fc, int D, int B, int mode, int qi, const float* Wc,
                               const float* hq, const float* dquery, const float* dxf_cat, long dxf_ld,
                               uint32_t drop_key, uint32_t drop_thresh, float drop_scale, const float* dfc,
                               long dfc_ld, float* dnum, float* dmask, float* dcat, float* dpre, void* stream) {
  if (B == 0) return 0;
  CtxBwdArgs a;
  a.f = CtxArgs{num_e, num_ld, Fn, mask_e, mask_ld, Fm, cat_e, Fc, D, B, mode, qi, Wc, nullptr, nullptr,
                const_cast<float*>(hq), nullptr};
  a.dquery = dquery;
  a.dxf_cat = dxf_cat;
  a.dxf_ld = dxf_ld;
  a.emb_drop = Drop{drop_key, drop_thresh, drop_scale};
  a.dfc = dfc;
  a.dfc_ld = dfc_ld;
  a.dnum = dnum;
  a.dmask = dmask;
  a.dcat = dcat;
  a.dpre = dpre;
  CTR_REQUIRE(D <= 64, "D > 64");
  context_bwd_kernel<<<B, CTXB_T, 0, (hipStream_t)stream>>>(a);
  return check_launch("context_bwd");
}

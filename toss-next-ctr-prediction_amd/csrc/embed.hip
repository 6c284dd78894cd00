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
__global__ __launch_bounds__(256) void feat_embed_fwd_kernel(const float* __restrict__ x, int B, int F,
                                                             const float* __restrict__ W,
                                                             const float* __restrict__ bias,
                                                             const float* __restrict__ P, int fe, int D,
                                                             float* __restrict__ out, long out_ld) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* sP = sm;               // [fe][D]: lanes (consecutive d) read consecutive banks
  float* sW = sm + D * fe;      // [F][fe] (broadcast across the d lanes)
  float* sB = sW + F * fe;      // [F][fe]
  for (int i = threadIdx.x; i < D * fe; i += blockDim.x) sP[(i % fe) * D + i / fe] = P[i];
  for (int i = threadIdx.x; i < F * fe; i += blockDim.x) {
    sW[i] = W[i];
    sB[i] = bias ? bias[i] : 0.f;
  }
  __syncthreads();
  const long total = (long)B * F * D;
  for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q < total; q += (long)gridDim.x * blockDim.x) {
    const int d = (int)(q % D);
    const long bf = q / D;
    const int f = (int)(bf % F);
    const long b = bf / F;
    const float xv = x[b * F + f];
    float acc = 0.f;
    for (int k = 0; k < fe; ++k) {
      float e = xv * sW[f * fe + k];
      if (bias) e = e + sB[f * fe + k];
      acc = fmaf(e, sP[k * D + d], acc);
    }
    out[b * out_ld + (long)f * D + d] = acc;
  }
}

// S1[f,d] = sum_b x[b,f] dout[b,f,d],  S0[f,d] = sum_b dout[b,f,d]: one workgroup per feature f;
// lanes = d (coalesced dout rows), 256/D row groups stride the batch, combined in fixed order.
__global__ __launch_bounds__(256) void feat_embed_bwd_sums(const float* __restrict__ x, int B, int F, int D,
                                                          const float* __restrict__ dout, long dout_ld,
                                                          float* __restrict__ S) {
  __shared__ float r1[256], r0[256];
  const int f = blockIdx.x, t = threadIdx.x;
  const int RG = 256 / D;
  const int d = t % D, rg = t / D;
  float s1 = 0.f, s0 = 0.f;
  if (rg < RG)
    for (int b = rg; b < B; b += RG) {
      const float g = dout[(long)b * dout_ld + (long)f * D + d];
      s1 = fmaf(x[(long)b * F + f], g, s1);
      s0 += g;
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
    S[(long)f * D + t] = a;
    S[(long)F * D + (long)f * D + t] = c;
  }
}

// dW = S1 @ P, dbias = S0 @ P, dP = sum_f S1^T W + S0^T bias   (one thread per output element)
__global__ __launch_bounds__(256) void feat_embed_bwd_final(int F, int D, int fe, const float* __restrict__ S,
                                                           const float* __restrict__ W,
                                                           const float* __restrict__ bias,
                                                           const float* __restrict__ P,
                                                           float* __restrict__ dW, float* __restrict__ dbias,
                                                           float* __restrict__ dP) {
  const float* S1 = S;
  const float* S0 = S + F * D;
  const int q = blockIdx.x * 256 + threadIdx.x;
  if (q < F * fe) {
    const int f = q / fe, k = q % fe;
    float a = 0.f, c = 0.f;
    for (int d = 0; d < D; ++d) {
      a = fmaf(S1[f * D + d], P[d * fe + k], a);
      c = fmaf(S0[f * D + d], P[d * fe + k], c);
    }
    dW[q] = a;
    if (dbias) dbias[q] = c;
  } else if (q < F * fe + D * fe) {
    const int r = q - F * fe;
    const int d = r / fe, k = r % fe;
    float a = 0.f;
    for (int f = 0; f < F; ++f) {
      a = fmaf(S1[f * D + d], W[f * fe + k], a);
      if (bias) a = fmaf(S0[f * D + d], bias[f * fe + k], a);
    }
    dP[r] = a;
  }
}

// ------------------------------------------------------------------------------------------------
// hashed categorical embeddings: one thread per (b, c, d); the D threads of a (b, c) share the row
// ------------------------------------------------------------------------------------------------
struct CatMeta {
  const long* tab_off;    // element offset of table c in the arena
  const long* proj_off;   // element offset of proj c ([D][d_c]) in the arena
  const int* dims;        // d_c
};

__global__ __launch_bounds__(256) void cat_embed_fwd_kernel(const int* __restrict__ xcat, int B, int Fc,
                                                            const float* __restrict__ arena, CatMeta cm, int D,
                                                            float* __restrict__ cat_e, float* __restrict__ xf,
                                                            long xf_ld, Drop drop) {
  const long total = (long)B * Fc * D;
  for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q < total; q += (long)gridDim.x * blockDim.x) {
    const int d = (int)(q % D);
    const long bc = q / D;
    const int c = (int)(bc % Fc);
    const long b = bc / Fc;
    const int dc = cm.dims[c];
    const long row = xcat[b * Fc + c];
    const float* t = arena + cm.tab_off[c] + row * dc;
    const float* p = arena + cm.proj_off[c] + (long)d * dc;
    float acc = 0.f;
    for (int k = 0; k < dc; ++k) acc = fmaf(t[k], p[k], acc);
    cat_e[q] = acc;
    if (xf) xf[b * xf_ld + (long)c * D + d] = drop_apply(drop, (uint32_t)q, acc);
  }
}

// row-grad contributions: contrib[(b*Fc+c)*64 + k] = sum_d dcat[b,c,d] P_c[d,k]  (zero-padded to 64)
// keys[b*Fc+c] = row_base[c] + X_cat[b,c]
__global__ __launch_bounds__(256) void cat_embed_bwd_rows(const int* __restrict__ xcat, int B, int Fc,
                                                          const float* __restrict__ arena, CatMeta cm, int D,
                                                          const float* __restrict__ dcat,
                                                          const uint32_t* __restrict__ row_base,
                                                          float* __restrict__ contrib, uint32_t* __restrict__ keys) {
  const long total = (long)B * Fc * 64;
  for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q < total; q += (long)gridDim.x * blockDim.x) {
    const int k = (int)(q & 63);
    const long bc = q >> 6;
    const int c = (int)(bc % Fc);
    const long b = bc / Fc;
    const int dc = cm.dims[c];
    float acc = 0.f;
    if (k < dc) {
      const float* p = arena + cm.proj_off[c] + k;
      const float* g = dcat + bc * D;
      for (int d = 0; d < D; ++d) acc = fmaf(g[d], p[(long)d * dc], acc);
    }
    contrib[q] = acc;
    if (k == 0) keys[bc] = row_base[c] + (uint32_t)xcat[b * Fc + c];
  }
}

// dP_c[d,k] = sum_b dcat[b,c,d] * T_c[row_b, k]   -- block (c, chunk) partials over a row chunk
__global__ __launch_bounds__(256) void cat_embed_bwd_proj_partial(const int* __restrict__ xcat, int B, int Fc,
                                                                  const float* __restrict__ arena, CatMeta cm,
                                                                  int D, const float* __restrict__ dcat,
                                                                  int rows_per_chunk, float* __restrict__ part) {
  const int c = blockIdx.x, chunk = blockIdx.y;
  const int dc = cm.dims[c];
  const int b0 = chunk * rows_per_chunk, b1 = min(B, b0 + rows_per_chunk);
  const float* T = arena + cm.tab_off[c];
  float* out = part + ((long)chunk * Fc + c) * (64 * 64);
  for (int q = threadIdx.x; q < D * dc; q += blockDim.x) {
    const int d = q / dc, k = q % dc;
    float acc = 0.f;
    for (int b = b0; b < b1; ++b) {
      const long row = xcat[(long)b * Fc + c];
      acc = fmaf(dcat[((long)b * Fc + c) * D + d], T[row * dc + k], acc);
    }
    out[q] = acc;
  }
}

__global__ __launch_bounds__(256) void cat_embed_bwd_proj_final(int nchunk, int Fc, int D, CatMeta cm,
                                                                const long* __restrict__ proj_goff,
                                                                const float* __restrict__ part,
                                                                float* __restrict__ grad) {
  const int c = blockIdx.x;
  const int dc = cm.dims[c];
  for (int q = threadIdx.x; q < D * dc; q += blockDim.x) {
    float s = 0.f;
    for (int ch = 0; ch < nchunk; ++ch) s += part[((long)ch * Fc + c) * (64 * 64) + q];
    grad[proj_goff[c] + q] = s;
  }
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

__global__ __launch_bounds__(64) void context_fwd_kernel(CtxArgs a) {
  __shared__ float sctx[3 * 64];
  const int b = blockIdx.x, d = threadIdx.x;
  const int D = a.D;
  int nctx = 0;
  if (d < D) {
    if (a.Fn > 0) {
      float s = 0.f;
      for (int f = 0; f < a.Fn; ++f) s += a.num_e[(long)b * a.num_ld + (long)f * D + d];
      sctx[nctx * D + d] = s / (float)a.Fn;
    }
  }
  if (a.Fn > 0) ++nctx;
  if (d < D && a.Fm > 0) {
    float s = 0.f;
    for (int f = 0; f < a.Fm; ++f) s += a.mask_e[(long)b * a.mask_ld + (long)f * D + d];
    sctx[nctx * D + d] = s / (float)a.Fm;
  }
  if (a.Fm > 0) ++nctx;
  if (d < D) {
    float s = 0.f;
    for (int c = 0; c < a.Fc; ++c) s += a.cat_e[((long)b * a.Fc + c) * D + d];
    sctx[nctx * D + d] = a.Fc > 0 ? s / (float)a.Fc : 0.f;
  }
  ++nctx;
  __syncthreads();
  const int W = nctx * D;
  if (d < D) {
    for (int j = d; j < W; j += D) a.ctx[(long)b * W + j] = sctx[j];
    float q;
    float h = 0.f;
    if (a.mode != 0) {
      float acc = 0.f;
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

__global__ __launch_bounds__(64) void context_bwd_kernel(CtxBwdArgs a) {
  __shared__ float sdp[64];
  __shared__ float sdctx[3 * 64];
  const CtxArgs& f = a.f;
  const int b = blockIdx.x, d = threadIdx.x, D = f.D;
  const int nctx = (f.Fn > 0) + (f.Fm > 0) + 1;
  const int W = nctx * D;
  float dqv = d < D ? a.dquery[(long)b * D + d] : 0.f;
  float dh = 0.f;
  if (d < D && f.mode != 0) {
    dh = f.mode == 2 ? 0.5f * dqv : dqv;
    dh = f.hq[(long)b * D + d] > 0.f ? dh : 0.f;
    if (a.dpre) a.dpre[(long)b * D + d] = dh;
  }
  if (d < 64) sdp[d] = dh;
  __syncthreads();
  // dctx[j] = sum_d dpre[d] * Wc[d, j]
  for (int j = d; j < W; j += 64) {
    float acc = 0.f;
    if (f.mode != 0)
      for (int i = 0; i < D; ++i) acc = fmaf(sdp[i], f.Wc[(long)i * W + j], acc);
    sdctx[j] = acc;
  }
  __syncthreads();
  if (d >= D) return;
  int slot = 0;
  const int fcbase = 1;  // fc layout: [u, num_mean?, mask_mean?, cat_0.. cat_{Fc-1}]
  int fcslot = fcbase;
  if (f.Fn > 0) {
    float g = sdctx[slot * D + d];
    if (a.dfc) g += a.dfc[(long)b * a.dfc_ld + (long)fcslot * D + d];
    g = g / (float)f.Fn;
    for (int k = 0; k < f.Fn; ++k) a.dnum[(long)b * f.num_ld + (long)k * D + d] += g;
    ++slot;
    ++fcslot;
  }
  if (f.Fm > 0) {
    float g = sdctx[slot * D + d];
    if (a.dfc) g += a.dfc[(long)b * a.dfc_ld + (long)fcslot * D + d];
    g = g / (float)f.Fm;
    for (int k = 0; k < f.Fm; ++k) a.dmask[(long)b * f.mask_ld + (long)k * D + d] += g;
    ++slot;
    ++fcslot;
  }
  const float gc = f.Fc > 0 ? sdctx[slot * D + d] / (float)f.Fc : 0.f;
  for (int c = 0; c < f.Fc; ++c) {
    const long q = ((long)b * f.Fc + c) * D + d;
    float g = 0.f;
    if (a.dxf_cat) {
      const float gx = a.dxf_cat[(long)b * a.dxf_ld + (long)c * D + d];
      g = a.emb_drop.thresh ? (drop_keep(a.emb_drop, (uint32_t)q) ? gx * a.emb_drop.scale : 0.f) : gx;
    }
    if (a.dfc) g += a.dfc[(long)b * a.dfc_ld + (long)(fcslot + c) * D + d];
    if (c == f.qi && f.mode != 1) g += f.mode == 2 ? 0.5f * dqv : dqv;
    g += gc;
    a.dcat[q] = g;
  }
}

}  // namespace ctr

using namespace ctr;

extern "C" int ctr_feat_embed_fwd(const float* x, int B, int F, const float* W, const float* bias, const float* P,
                                  int fe, int D, float* out, long out_ld, void* stream) {
  if (B == 0 || F == 0) return 0;
  size_t sm = (size_t)(D * fe + 2 * F * fe) * sizeof(float);
  CTR_REQUIRE(sm <= 64 * 1024, "feat_embed weights exceed 64 KB LDS staging");
  long total = (long)B * F * D;
  int blocks = (int)std::min<long>((total + 255) / 256, 8192);
  feat_embed_fwd_kernel<<<blocks, 256, sm, (hipStream_t)stream>>>(x, B, F, W, bias, P, fe, D, out, out_ld);
  return check_launch("feat_embed_fwd");
}

extern "C" size_t ctr_feat_embed_bwd_ws(int B, int F, int D) { return (size_t)2 * F * D * sizeof(float); }

extern "C" int ctr_feat_embed_bwd(const float* x, int B, int F, const float* W, const float* bias, const float* P,
                                  int fe, int D, const float* dout, long dout_ld, float* dW, float* dbias,
                                  float* dP, float* ws, void* stream) {
  if (F == 0) return 0;
  CTR_REQUIRE(D <= 256, "D > 256");
  hipStream_t s = (hipStream_t)stream;
  feat_embed_bwd_sums<<<F, 256, 0, s>>>(x, B, F, D, dout, dout_ld, ws);
  feat_embed_bwd_final<<<cdiv((long)(F + D) * fe, 256), 256, 0, s>>>(F, D, fe, ws, W, bias, P, dW, dbias, dP);
  return check_launch("feat_embed_bwd");
}

extern "C" int ctr_cat_embed_fwd(const int* xcat, int B, int Fc, const float* arena, const long* tab_off,
                                 const long* proj_off, const int* dims, int D, float* cat_e, float* xf, long xf_ld,
                                 uint32_t drop_key, uint32_t drop_thresh, float drop_scale, void* stream) {
  if (B == 0 || Fc == 0) return 0;
  CatMeta cm{tab_off, proj_off, dims};
  long total = (long)B * Fc * D;
  int blocks = (int)std::min<long>((total + 255) / 256, 16384);
  cat_embed_fwd_kernel<<<blocks, 256, 0, (hipStream_t)stream>>>(xcat, B, Fc, arena, cm, D, cat_e, xf, xf_ld,
                                                                 Drop{drop_key, drop_thresh, drop_scale});
  return check_launch("cat_embed_fwd");
}

extern "C" size_t ctr_cat_embed_bwd_ws(int B, int Fc) {
  int nchunk = (B + 127) / 128;
  return (size_t)nchunk * Fc * 64 * 64 * sizeof(float);
}

extern "C" int ctr_cat_embed_bwd(const int* xcat, int B, int Fc, const float* arena, const long* tab_off,
                                 const long* proj_off, const int* dims, int D, const float* dcat,
                                 const uint32_t* row_base, float* contrib, uint32_t* keys, float* grad_arena,
                                 const long* proj_goff, float* ws, void* stream) {
  if (B == 0 || Fc == 0) return 0;
  CTR_REQUIRE(D <= 64, "D > 64");
  hipStream_t s = (hipStream_t)stream;
  CatMeta cm{tab_off, proj_off, dims};
  long total = (long)B * Fc * 64;
  int blocks = (int)std::min<long>((total + 255) / 256, 16384);
  cat_embed_bwd_rows<<<blocks, 256, 0, s>>>(xcat, B, Fc, arena, cm, D, dcat, row_base, contrib, keys);
  const int rpc = 128;
  const int nchunk = (B + rpc - 1) / rpc;
  cat_embed_bwd_proj_partial<<<dim3(Fc, nchunk), 256, 0, s>>>(xcat, B, Fc, arena, cm, D, dcat, rpc, ws);
  cat_embed_bwd_proj_final<<<Fc, 256, 0, s>>>(nchunk, Fc, D, cm, proj_goff, ws, grad_arena);
  return check_launch("cat_embed_bwd");
}

extern "C" int ctr_context_fwd(const float* num_e, long num_ld, int Fn, const float* mask_e, long mask_ld, int Fm,
                               const float* cat_e, int Fc, int D, int B, int mode, int qi, const float* Wc,
                               const float* bc, float* ctx, float* hq, float* query, void* stream) {
  if (B == 0) return 0;
  CTR_REQUIRE(D <= 64, "D > 64");
  CtxArgs a{num_e, num_ld, Fn, mask_e, mask_ld, Fm, cat_e, Fc, D, B, mode, qi, Wc, bc, ctx, hq, query};
  context_fwd_kernel<<<B, 64, 0, (hipStream_t)stream>>>(a);
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
  context_bwd_kernel<<<B, 64, 0, (hipStream_t)stream>>>(a);
  return check_launch("context_bwd");
}

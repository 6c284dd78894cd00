// DARE sequence path: recency-decayed dot-product top-K selection and the gating pool.
//
//   topk_select : src/models/dare.py:116-138   gather att rows, score = <att,q> + log(decay+1e-8),
//                                               pads -> -1e9, sorted top-K, gather only the K rep rows
//   pool        : src/models/dare.py:150-162   softmax / relu gating, weighted sum, dropout, aux head
//
// top-K: one workgroup per sequence row; scores land in LDS and a bitonic network sorts
// (score desc, position asc) pairs of next_pow2(L) <= 1024.  Backward emits row-grad contributions
// (key = token id, or INVALID for pads, whose grads nn.Embedding(padding_idx) drops) that the
// deterministic dedup (rowgrad.hip) folds into the tables.
#include "common.h"
#include "ctr_hip.h"

namespace ctr {

constexpr uint32_t INVALID_KEY = 0xFFFFFFFFu;

__device__ __forceinline__ bool pair_before(float sa, int ia, float sb, int ib) {
  return sa > sb || (sa == sb && ia < ib);
}

template <int NT>
__global__ __launch_bounds__(NT) void topk_fwd_kernel(const int* __restrict__ seq, int L, const float* __restrict__ q,
                                                      const float* __restrict__ E_att,
                                                      const float* __restrict__ E_rep, int D,
                                                      const float* __restrict__ decay_log, int K, int pad_id, int N,
                                                      int* __restrict__ idx_out, int* __restrict__ tok_out,
                                                      float* __restrict__ vals, float* __restrict__ sel) {
  __shared__ float ss[1024];
  __shared__ int si[1024];
  __shared__ float sq[64];
  const int b = blockIdx.x, t = threadIdx.x;
  if (t < D) sq[t] = q[(long)b * D + t];
  __syncthreads();
  const int* srow = seq + (long)b * L;
  for (int l = t; l < N; l += NT) {
    float s = -INFINITY;
    if (l < L) {
      const int tok = srow[l];
      if (tok == pad_id) {
        s = -1e9f;
      } else {
        const float* a = E_att + (long)tok * D;
        float acc = 0.f;
        for (int d = 0; d < D; d += 4) {
          const float4 v = *(const float4*)(a + d);
          acc += v.x * sq[d];
          acc += v.y * sq[d + 1];
          acc += v.z * sq[d + 2];
          acc += v.w * sq[d + 3];
        }
        s = acc + decay_log[l];
      }
    }
    ss[l] = s;
    si[l] = l;
  }
  __syncthreads();
  // bitonic sort, descending by score, ascending by position on ties
  for (int size = 2; size <= N; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = t; i < N / 2; i += NT) {
        const int lo = 2 * i - (i & (stride - 1));
        const int hi = lo + stride;
        const bool desc = ((lo & size) == 0);
        const float a = ss[lo], c = ss[hi];
        const int ia = si[lo], ic = si[hi];
        const bool swap = desc ? pair_before(c, ic, a, ia) : pair_before(a, ia, c, ic);
        if (swap) {
          ss[lo] = c; ss[hi] = a;
          si[lo] = ic; si[hi] = ia;
        }
      }
      __syncthreads();
    }
  }
  int* stok = si;        // (in place: entry k is read and rewritten by the same thread)
  for (int k = t; k < K; k += NT) {
    const int l = si[k];
    const int tk = srow[l];
    idx_out[(long)b * K + k] = l;
    tok_out[(long)b * K + k] = tk;
    vals[(long)b * K + k] = ss[k];
    stok[k] = tk;
  }
  __syncthreads();
  // the selected rep rows: tokens from LDS (a token -> row load chain per element before), 16-byte copies
  if ((D & 3) == 0 && ((((uintptr_t)E_rep) | ((uintptr_t)sel)) & 15) == 0) {
    const int D4 = D >> 2;
#pragma unroll 4
    for (int e = t; e < K * D4; e += NT) {
      const int k = e / D4, d4 = e - k * D4;
      *(float4*)(sel + ((long)b * K + k) * D + 4 * d4) = *(const float4*)(E_rep + (long)stok[k] * D + 4 * d4);
    }
  } else {
#pragma unroll 4
    for (int e = t; e < K * D; e += NT) {
      const int k = e / D, d = e % D;
      sel[((long)b * K + k) * D + d] = E_rep[(long)stok[k] * D + d];
    }
  }
}

// dq[b] = sum_k dvals[b,k] * E_att[tok]; att contributions dvals*q keyed by token; rep keys.
__global__ __launch_bounds__(256) void topk_bwd_kernel(const int* __restrict__ tok, int B, int K,
                                                       const float* __restrict__ q,
                                                       const float* __restrict__ E_att, int D,
                                                       const float* __restrict__ dvals, int pad_id,
                                                       float* __restrict__ dq, float* __restrict__ att_contrib,
                                                       uint32_t* __restrict__ att_keys,
                                                       uint32_t* __restrict__ rep_keys) {
  // one wave per sample b: lane = d for dq; then (k, d) pairs for contributions
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int b = blockIdx.x * 4 + wid;
  if (b >= B) return;
  const int* tb = tok + (long)b * K;
  const float* dv = dvals + (long)b * K;
  // keys in chunks of TB_CH: the chunk's token / weight loads, then its row gathers, all independent (one memory
  // round trip each per chunk instead of a token -> row dependency per key); summed in ascending k as before.
  // The att contributions dvals * q and the keys are written from the same chunk registers (a separate pass
  // re-loaded the token and weight of every (k, d) one dependent round trip after another), and the gathers are
  // unconditional -- the padding token reads row 0, its term dropped at the add (a conditional load put its use,
  // and a wait, inside a branch per key)
  constexpr int TB_CH = 16;
  float* ac = att_contrib + (long)b * K * D;
  uint32_t* ak = att_keys + (long)b * K;
  uint32_t* rk = rep_keys + (long)b * K;
  if (D <= 32) {    // two half-waves take the even / odd k, combined in a fixed order
    const int d = lane & 31, h = lane >> 5;
    float acc = 0.f;
    if (d < D) {
      const float qd = q[(long)b * D + d];
      for (int k0 = h; k0 < K; k0 += 2 * TB_CH) {
        int t[TB_CH];
        float w[TB_CH], e[TB_CH];
#pragma unroll
        for (int u = 0; u < TB_CH; ++u) {
          const int k = k0 + 2 * u;
          t[u] = k < K ? tb[k] : pad_id;
          w[u] = k < K ? dv[k] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < TB_CH; ++u) e[u] = E_att[(long)(t[u] != pad_id ? t[u] : 0) * D + d];
#pragma unroll
        for (int u = 0; u < TB_CH; ++u) {
          const int k = k0 + 2 * u;
          if (t[u] != pad_id) acc = fmaf(w[u], e[u], acc);
          if (k < K) {
            ac[(long)k * D + d] = t[u] != pad_id ? w[u] * qd : 0.f;
            if (d == 0) {
              const uint32_t key = t[u] != pad_id ? (uint32_t)t[u] : INVALID_KEY;
              ak[k] = key;
              rk[k] = key;
            }
          }
        }
      }
    }
    const float other = __shfl_down(acc, 32);
    if (h == 0 && d < D) dq[(long)b * D + d] = acc + other;
  } else if (lane < D) {
    float acc = 0.f;
    const float qd = q[(long)b * D + lane];
    for (int k0 = 0; k0 < K; k0 += TB_CH) {
      int t[TB_CH];
      float w[TB_CH], e[TB_CH];
#pragma unroll
      for (int u = 0; u < TB_CH; ++u) {
        const int k = k0 + u;
        t[u] = k < K ? tb[k] : pad_id;
        w[u] = k < K ? dv[k] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < TB_CH; ++u) e[u] = E_att[(long)(t[u] != pad_id ? t[u] : 0) * D + lane];
#pragma unroll
      for (int u = 0; u < TB_CH; ++u) {
        const int k = k0 + u;
        if (t[u] != pad_id) acc = fmaf(w[u], e[u], acc);
        if (k < K) {
          ac[(long)k * D + lane] = t[u] != pad_id ? w[u] * qd : 0.f;
          if (lane == 0) {
            const uint32_t key = t[u] != pad_id ? (uint32_t)t[u] : INVALID_KEY;
            ak[k] = key;
            rk[k] = key;
          }
        }
      }
    }
    dq[(long)b * D + lane] = acc;
  }
}

// ------------------------------------------------------------------------------------------------
// gating pool: one wave per sample
// ------------------------------------------------------------------------------------------------
struct PoolArgs {
  const float* x;       // (B, K, D) encoder output
  const float* vals;    // (B, K)
  int B, K, D, gating;  // gating 0 softmax, 1 relu-normalised
  Drop drop;            // dare dropout on u (B, D)
  const float* waux;    // (D)
  const float* baux;    // (1)
  float* w;             // (B, K) saved gate weights
  float* u;             // (B, D) post-dropout u (saved)
  float* xf_u;          // xF slot 0 (row stride xf_ld), nullable
  long xf_ld;
  float* aux;           // (B)
};

__global__ __launch_bounds__(64) void pool_fwd_kernel(PoolArgs a) {
  __shared__ float sw[256];
  const int b = blockIdx.x, lane = threadIdx.x;
  const int K = a.K, D = a.D;
  const float* v = a.vals + (long)b * K;
  if (a.gating == 0) {
    float m = -INFINITY;
    for (int k = lane; k < K; k += 64) m = fmaxf(m, v[k]);
    m = wave_max(m);
    float s = 0.f;
    for (int k = lane; k < K; k += 64) {
      const float e = expf(v[k] - m);
      sw[k] = e;
      s += e;
    }
    s = wave_sum(s);
    __syncthreads();
    for (int k = lane; k < K; k += 64) sw[k] = sw[k] / s;
  } else {
    float s = 0.f;
    for (int k = lane; k < K; k += 64) {
      const float r = fmaxf(v[k], 0.f);
      sw[k] = r;
      s += r;
    }
    s = wave_sum(s);
    __syncthreads();
    for (int k = lane; k < K; k += 64) sw[k] = sw[k] / (s + 1e-12f);
  }
  __syncthreads();
  for (int k = lane; k < K; k += 64) a.w[(long)b * K + k] = sw[k];
  float ud = 0.f;
  if (lane < D) {
    const float* xb = a.x + (long)b * K * D;
    float acc = 0.f;
    for (int k = 0; k < K; ++k) acc += xb[(long)k * D + lane] * sw[k];
    ud = drop_apply(a.drop, (uint32_t)((long)b * D + lane), acc);
    a.u[(long)b * D + lane] = ud;
    if (a.xf_u) a.xf_u[(long)b * a.xf_ld + lane] = ud;
  }
  const float z = wave_sum(lane < D ? ud * a.waux[lane] : 0.f);
  if (lane == 0) a.aux[b] = z + a.baux[0];
}

struct PoolBwdArgs {
  PoolArgs f;
  const float* du;      // grad wrt post-dropout u: (B, D) at row stride du_ld (nullable)
  long du_ld;
  const float* daux;    // (B) (nullable)
  float* dx;            // (B, K, D)
  float* dvals;         // (B, K)
};

__global__ __launch_bounds__(64) void pool_bwd_kernel(PoolBwdArgs a) {
  __shared__ float sdu[64];
  __shared__ float sdw[256];
  __shared__ float swk[256];
  const PoolArgs& f = a.f;
  const int b = blockIdx.x, lane = threadIdx.x;
  const int K = f.K, D = f.D;
  float g = 0.f;
  if (lane < D) {
    if (a.du) g = a.du[(long)b * a.du_ld + lane];
    if (a.daux) g += a.daux[b] * f.waux[lane];
    if (f.drop.thresh) g = drop_keep(f.drop, (uint32_t)((long)b * D + lane)) ? g * f.drop.scale : 0.f;
  }
  sdu[lane] = g;
  const float* xb = f.x + (long)b * K * D;
  const float* wb = f.w + (long)b * K;
  // the sample's gate weights staged in LDS: read from global inside the dx loop they were re-loaded after every
  // dx store (the pointers may alias), one round trip per element group
  for (int k = lane; k < K; k += 64) swk[k] = wb[k];
  __syncthreads();
  for (int e = lane; e < K * D; e += 64) {
    const int k = e / D, d = e % D;
    a.dx[(long)b * K * D + e] = swk[k] * sdu[d];
  }
  float dot = 0.f;
  for (int k = lane; k < K; k += 64) {
    float s = 0.f;
    for (int d = 0; d < D; ++d) s = fmaf(xb[(long)k * D + d], sdu[d], s);
    sdw[k] = s;
    dot += (f.gating == 0 ? swk[k] * s : s * fmaxf(f.vals[(long)b * K + k], 0.f));
  }
  dot = wave_sum(dot);
  __syncthreads();
  if (f.gating == 0) {
    for (int k = lane; k < K; k += 64) a.dvals[(long)b * K + k] = swk[k] * (sdw[k] - dot);
  } else {
    // w = r / (S + eps), r = relu(v): dv_k = [v_k>0] (dw_k/(S+eps) - sum_j dw_j r_j/(S+eps)^2)
    float S = 0.f;
    for (int k = lane; k < K; k += 64) S += fmaxf(f.vals[(long)b * K + k], 0.f);
    S = wave_sum(S) + 1e-12f;
    for (int k = lane; k < K; k += 64) {
      const float v = f.vals[(long)b * K + k];
      a.dvals[(long)b * K + k] = v > 0.f ? (sdw[k] / S - dot / (S * S)) : 0.f;
    }
  }
}

// mean over heads of the relative position bias: out[d] = mean_h rel[d, h]  (src/models/dare.py:56-60)
__global__ void pos_bias_mean_kernel(const float* __restrict__ rel, int H, int n, float* __restrict__ out) {
  for (int d = blockIdx.x * blockDim.x + threadIdx.x; d < n; d += gridDim.x * blockDim.x) {
    float s = 0.f;
    for (int h = 0; h < H; ++h) s += rel[(long)d * H + h];
    out[d] = s / (float)H;
  }
}

// drel[d, h] = (sum_p part[p, d]) / H for every head h (the head-mean bias), in two passes over the
// (nparts, n) partials: pass 1, block s sums its PB_ROWS consecutive rows, a thread per column (coalesced row
// reads, the rows' loads issued together, summed in row order) and writes the sums over the block's first row
// (that block is the only reader / writer of those rows: the partials are scratch); pass 2, a block per column d
// sums the blocks' rows in a fixed-order block reduction.  (A block per column over all rows read the column
// at a 4n-byte stride: 25 us per call at cfg2.)
constexpr int PB_ROWS = 32;
__global__ __launch_bounds__(128) void pos_bias_grad_part(float* __restrict__ part, int nparts, int n) {
  const int p0 = blockIdx.x * PB_ROWS, np = min(nparts - p0, PB_ROWS);
  for (int d = threadIdx.x; d < n; d += 128) {
    float v[PB_ROWS];
#pragma unroll
    for (int k = 0; k < PB_ROWS; ++k) v[k] = k < np ? part[(long)(p0 + k) * n + d] : 0.f;
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < PB_ROWS; ++k) s += v[k];
    part[(long)p0 * n + d] = s;
  }
}

__global__ __launch_bounds__(256) void pos_bias_grad_kernel(const float* __restrict__ part, int nsplit, int H, int n,
                                                            float* __restrict__ drel) {
  __shared__ float red[4];
  const int d = blockIdx.x;
  float s = 0.f;
  for (int k = threadIdx.x; k < nsplit; k += 256) s += part[(long)k * PB_ROWS * n + d];
  s = block_sum(s, red);
  if (threadIdx.x < H) drel[(long)d * H + threadIdx.x] = s / (float)H;
}

}  // namespace ctr

using namespace ctr;

extern "C" int ctr_dare_topk_fwd(const int* seq, int B, int L, const float* q, const float* E_att,
                                 const float* E_rep, int D, const float* decay_log, int K, int pad_id, int* idx,
                                 int* tok, float* vals, float* sel, void* stream) {
  if (B == 0) return 0;
  CTR_REQUIRE(L >= 1 && L <= 1024, "L must be in [1, 1024]");
  CTR_REQUIRE(K >= 1 && K <= L, "K must be in [1, L]");
  CTR_REQUIRE(D % 4 == 0 && D <= 64, "D must be a multiple of 4 and <= 64");
  int N = 1;
  while (N < L) N <<= 1;
  if (N < 2) N = 2;
  if (N <= 128)
    topk_fwd_kernel<64><<<B, 64, 0, (hipStream_t)stream>>>(seq, L, q, E_att, E_rep, D, decay_log, K, pad_id, N, idx,
                                                          tok, vals, sel);
  else
    topk_fwd_kernel<256><<<B, 256, 0, (hipStream_t)stream>>>(seq, L, q, E_att, E_rep, D, decay_log, K, pad_id, N,
                                                            idx, tok, vals, sel);
  return check_launch("dare_topk_fwd");
}

extern "C" int ctr_dare_topk_bwd(const int* tok, int B, int K, const float* q, const float* E_att, int D,
                                 const float* dvals, int pad_id, float* dq, float* att_contrib, uint32_t* att_keys,
                                 uint32_t* rep_keys, void* stream) {
  if (B == 0) return 0;
  CTR_REQUIRE(D <= 64, "D > 64");
  topk_bwd_kernel<<<cdiv(B, 4), 256, 0, (hipStream_t)stream>>>(tok, B, K, q, E_att, D, dvals, pad_id, dq,
                                                               att_contrib, att_keys, rep_keys);
  return check_launch("dare_topk_bwd");
}

extern "C" int ctr_pool_fwd(const float* x, const float* vals, int B, int K, int D, int gating, uint32_t drop_key,
                            uint32_t drop_thresh, float drop_scale, const float* waux, const float* baux, float* w,
                            float* u, float* xf_u, long xf_ld, float* aux, void* stream) {
  if (B == 0) return 0;
  CTR_REQUIRE(K <= 256 && D <= 64, "pool needs K <= 256, D <= 64");
  PoolArgs a{x, vals, B, K, D, gating, Drop{drop_key, drop_thresh, drop_scale}, waux, baux, w, u, xf_u, xf_ld, aux};
  pool_fwd_kernel<<<B, 64, 0, (hipStream_t)stream>>>(a);
  return check_launch("pool_fwd");
}

extern "C" int ctr_pool_bwd(const float* x, const float* vals, const float* w, int B, int K, int D, int gating,
                            uint32_t drop_key, uint32_t drop_thresh, float drop_scale, const float* waux,
                            const float* du, long du_ld, const float* daux, float* dx, float* dvals, void* stream) {
  if (B == 0) return 0;
  CTR_REQUIRE(K <= 256 && D <= 64, "pool needs K <= 256, D <= 64");
  PoolBwdArgs a;
  a.f = PoolArgs{x, vals, B, K, D, gating, Drop{drop_key, drop_thresh, drop_scale}, waux, nullptr,
                 const_cast<float*>(w), nullptr, nullptr, 0, nullptr};
  a.du = du;
  a.du_ld = du_ld;
  a.daux = daux;
  a.dx = dx;
  a.dvals = dvals;
  pool_bwd_kernel<<<B, 64, 0, (hipStream_t)stream>>>(a);
  return check_launch("pool_bwd");
}

extern "C" int ctr_pos_bias_mean(const float* rel, int H, int n, float* out, void* stream) {
  pos_bias_mean_kernel<<<cdiv(n, 256), 256, 0, (hipStream_t)stream>>>(rel, H, n, out);
  return check_launch("pos_bias_mean");
}

extern "C" int ctr_pos_bias_grad(float* part, int nparts, int H, int n, float* drel, void* stream) {
  CTR_REQUIRE(H <= 256, "H > 256");
  if (n <= 0) return 0;
  const int nsplit = std::max(1, cdiv(nparts, PB_ROWS));
  // the partials are the attention backward's per-(sample, head group) scratch: reduced in place
  if (nparts > 0) pos_bias_grad_part<<<nsplit, 128, 0, (hipStream_t)stream>>>(part, nparts, n);
  pos_bias_grad_kernel<<<n, 256, 0, (hipStream_t)stream>>>(part, nparts > 0 ? nsplit : 0, H, n, drel);
  return check_launch("pos_bias_grad");
}

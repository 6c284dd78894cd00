// Fused gradient clip + AdamW + EMA over the whole parameter arena -- the HBM-bound stream that
// dominates a training step.
//
// Replaces, per step: nn.utils.clip_grad_norm_ (src/train.py:194), torch.optim.AdamW.step
// (src/train.py:138,195; torch/optim/adam.py _single_tensor_adam, decoupled weight decay) and
// ModelEMA.update (src/utils/ema.py:92-131).  Semantics are the dense reference ones: EVERY
// element of every table is decayed / moment-updated each step, rows that no sample touched see
// grad = 0.  What differs is that no dense table gradient ever exists: table grads arrive as the
// compact (sorted unique keys, summed rows) produced by rowgrad.hip, and each workgroup maps the
// touched rows of its chunk into an LDS slot table (binary search + forward scan of the sorted keys).
// Per element: read p, m, v, ema (+ g) and write p, m, v, ema once -- 32 B/param of HBM traffic.
#include "common.h"
#include "ctr_hip.h"

namespace ctr {

constexpr int OPT_CHUNK = 8192;                 // elements per workgroup
constexpr int OPT_MAXROWS = OPT_CHUNK / 4 + 2;  // sparse segments need width >= 4

struct OptScalars {
  float decay_mul;    // 1 - lr*wd
  float b1w;          // 1 - beta1 (lerp weight)
  float b2, omb2;     // beta2, 1 - beta2
  float eps;
  float step_size;    // lr / (1 - beta1^t)
  float bc2_sqrt;     // sqrt(1 - beta2^t)
  float ema_d, ema_omd;
  int do_adam, do_ema;
};

__device__ __forceinline__ void adam_ema_elem(const OptScalars& s, float& p, float& m, float& v, float& e, float g,
                                              bool adam) {
  if (adam) {
    p = p * s.decay_mul;                                  // param.mul_(1 - lr*wd)
    m = m + s.b1w * (g - m);                              // exp_avg.lerp_(grad, 1-beta1)
    v = v * s.b2 + s.omb2 * g * g;                        // exp_avg_sq.mul_(b2).addcmul_(g, g, 1-b2)
    const float denom = sqrtf(v) / s.bc2_sqrt + s.eps;    // (sqrt(v) / bc2_sqrt).add_(eps)
    p = p + (-s.step_size) * (m / denom);                 // param.addcdiv_(m, denom, -step_size)
  }
  if (s.do_ema) e = e * s.ema_d + s.ema_omd * p;          // shadow.mul_(d).add_(p, alpha=1-d)
}

__global__ __launch_bounds__(256) void adamw_ema_kernel(const ctr_opt_chunk_t* __restrict__ chunks,
                                                        const ctr_opt_seg_t* __restrict__ segs,
                                                        float* __restrict__ P, float* __restrict__ M,
                                                        float* __restrict__ V, float* __restrict__ E,
                                                        const float* __restrict__ dgrad,
                                                        const float* __restrict__ coef_ptr, OptScalars s) {
  __shared__ int map[OPT_MAXROWS];
  __shared__ uint32_t lo_s;
  const ctr_opt_chunk_t ch = chunks[blockIdx.x];
  const ctr_opt_seg_t sg = segs[ch.seg];
  const float coef = coef_ptr ? *coef_ptr : 1.0f;
  const bool adam = s.do_adam && sg.kind != 2;
  const int tid = threadIdx.x;
  long r0 = 0;
  if (sg.kind == 1 && adam) {
    r0 = ch.e0 / sg.width;
    const long r1 = (ch.e1 - 1) / sg.width;
    const int nrows = (int)(r1 - r0 + 1);
    for (int i = tid; i < nrows; i += 256) map[i] = -1;
    const uint32_t nu = *sg.n_uniq;
    const uint32_t k0 = sg.key_base + (uint32_t)r0, k1 = sg.key_base + (uint32_t)r1;
    if (tid == 0) {
      uint32_t lo = 0, hi = nu;   // first index with key >= k0
      while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (sg.keys[mid] < k0) lo = mid + 1;
        else hi = mid;
      }
      lo_s = lo;
    }
    __syncthreads();
    for (uint32_t i = lo_s + tid; i < nu; i += 256) {
      const uint32_t k = sg.keys[i];
      if (k > k1) break;
      map[k - k0] = (int)i;
    }
    __syncthreads();
  }
  float* p = P + sg.p_off;
  float* m = M + sg.p_off;
  float* v = V + sg.p_off;
  float* e = E + sg.p_off;
  for (long q = ch.e0 + (long)tid * 4; q < ch.e1; q += 1024) {
    const int cnt = (int)min((long)4, ch.e1 - q);
    float4 pv = {0, 0, 0, 0}, mv = {0, 0, 0, 0}, vv = {0, 0, 0, 0}, ev = {0, 0, 0, 0};
    const bool full = cnt == 4;
    if (full) {
      pv = *(const float4*)(p + q);
      if (adam) {
        mv = *(const float4*)(m + q);
        vv = *(const float4*)(v + q);
      }
      if (s.do_ema) ev = *(const float4*)(e + q);
    } else {
      float* pp = (float*)&pv;
      float* mp = (float*)&mv;
      float* vp = (float*)&vv;
      float* ep = (float*)&ev;
      for (int j = 0; j < cnt; ++j) {
        pp[j] = p[q + j];
        if (adam) {
          mp[j] = m[q + j];
          vp[j] = v[q + j];
        }
        if (s.do_ema) ep[j] = e[q + j];
      }
    }
    float g[4] = {0.f, 0.f, 0.f, 0.f};
    if (adam) {
      if (sg.kind == 0) {
        const float* gp = dgrad + sg.g_off + q;
        for (int j = 0; j < cnt; ++j) g[j] = gp[j] * coef;
      } else {
        for (int j = 0; j < cnt; ++j) {
          const long el = q + j;
          const long row = el / sg.width;
          const int slot = map[row - r0];
          if (slot >= 0) g[j] = sg.G[(long)slot * sg.g_ld + (el - row * sg.width)] * coef;
        }
      }
    }
    float* pp = (float*)&pv;
    float* mp = (float*)&mv;
    float* vp = (float*)&vv;
    float* ep = (float*)&ev;
#pragma unroll
    for (int j = 0; j < 4; ++j) adam_ema_elem(s, pp[j], mp[j], vp[j], ep[j], g[j], adam);
    if (full) {
      if (adam) {
        *(float4*)(p + q) = pv;
        *(float4*)(m + q) = mv;
        *(float4*)(v + q) = vv;
      }
      if (s.do_ema) *(float4*)(e + q) = ev;
    } else {
      for (int j = 0; j < cnt; ++j) {
        if (adam) {
          p[q + j] = pp[j];
          m[q + j] = mp[j];
          v[q + j] = vp[j];
        }
        if (s.do_ema) e[q + j] = ep[j];
      }
    }
  }
}

// ---------------- global grad norm (clip_grad_norm_) ----------------
constexpr int NORM_BLOCKS = 256;

__global__ __launch_bounds__(256) void sqnorm_dense_kernel(const float* __restrict__ x, long n,
                                                           float* __restrict__ part) {
  __shared__ float red[4];
  float s = 0.f;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) s = fmaf(x[i], x[i], s);
  s = block_sum(s, red);
  if (threadIdx.x == 0) part[blockIdx.x] = s;
}

__global__ __launch_bounds__(256) void sqnorm_rows_kernel(const uint32_t* __restrict__ keys,
                                                          const float* __restrict__ G,
                                                          const uint32_t* __restrict__ n_uniq, int width, int ld,
                                                          uint32_t invalid_key, float* __restrict__ part) {
  __shared__ float red[4];
  const uint32_t nu = *n_uniq;
  float s = 0.f;
  const long total = (long)nu * width;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const long u = i / width;
    if (keys[u] == invalid_key) continue;
    const float g = G[u * ld + (i - u * width)];
    s = fmaf(g, g, s);
  }
  s = block_sum(s, red);
  if (threadIdx.x == 0) part[blockIdx.x] = s;
}

__global__ __launch_bounds__(256) void clip_finalize_kernel(const float* __restrict__ part, int nparts, float max_norm,
                                                            float* __restrict__ out) {
  __shared__ float red[4];
  float s = 0.f;
  for (int i = threadIdx.x; i < nparts; i += 256) s += part[i];
  s = block_sum(s, red);
  if (threadIdx.x == 0) {
    const float norm = sqrtf(s);
    out[0] = norm;
    out[1] = max_norm > 0.f ? fminf(max_norm / (norm + 1e-6f), 1.0f) : 1.0f;
  }
}

}  // namespace ctr

using namespace ctr;

extern "C" int ctr_opt_chunk_elems(void) { return OPT_CHUNK; }

extern "C" int ctr_adamw_ema(const ctr_opt_chunk_t* chunks, int nchunks, const ctr_opt_seg_t* segs, float* P, float* M,
                             float* V, float* E, const float* dgrad, const float* coef, float lr, float wd,
                             float beta1, float beta2, float eps, int step, float ema_decay, int do_adam, int do_ema,
                             void* stream) {
  if (nchunks == 0) return 0;
  OptScalars s;
  // host-side scalar math in double, exactly as torch/optim/adam.py computes it in Python floats
  const double bc1 = 1.0 - std::pow((double)beta1, step), bc2 = 1.0 - std::pow((double)beta2, step);
  s.decay_mul = (float)(1.0 - (double)lr * (double)wd);
  s.b1w = (float)(1.0 - (double)beta1);
  s.b2 = beta2;
  s.omb2 = (float)(1.0 - (double)beta2);
  s.eps = eps;
  s.step_size = (float)((double)lr / bc1);
  s.bc2_sqrt = (float)std::sqrt(bc2);
  s.ema_d = ema_decay;
  s.ema_omd = (float)(1.0 - (double)ema_decay);
  s.do_adam = do_adam;
  s.do_ema = do_ema;
  adamw_ema_kernel<<<nchunks, 256, 0, (hipStream_t)stream>>>(chunks, segs, P, M, V, E, dgrad, coef, s);
  return check_launch("adamw_ema");
}

extern "C" int ctr_norm_nparts_per_call(void) { return NORM_BLOCKS; }

extern "C" int ctr_sqnorm_dense(const float* x, long n, float* part, void* stream) {
  sqnorm_dense_kernel<<<NORM_BLOCKS, 256, 0, (hipStream_t)stream>>>(x, n, part);
  return check_launch("sqnorm_dense");
}

extern "C" int ctr_sqnorm_rows(const uint32_t* keys, const float* G, const uint32_t* n_uniq, int width, int ld,
                               uint32_t invalid_key, float* part, void* stream) {
  sqnorm_rows_kernel<<<NORM_BLOCKS, 256, 0, (hipStream_t)stream>>>(keys, G, n_uniq, width, ld, invalid_key, part);
  return check_launch("sqnorm_rows");
}

extern "C" int ctr_clip_finalize(const float* part, int nparts, float max_norm, float* out, void* stream) {
  clip_finalize_kernel<<<1, 256, 0, (hipStream_t)stream>>>(part, nparts, max_norm, out);
  return check_launch("clip_finalize");
}

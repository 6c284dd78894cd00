// Validation metrics and temperature-calibration objective of the K-fold loop, on device
// (src/utils/metrics.py:5-29, src/utils/calibration.py:23-52; src/train.py:226-240 runs them on the CPU
// between epochs over ~N/5 rows).
//
//   ctr_val_prob     p = sigmoid(z) in f64 (the loop's raw probabilities), or the calibrator's
//                    p = clip(sigmoid(clip(z/T, +-50)), 1e-7, 1-1e-7), all in f32 as the reference's
//                    predict_proba computes it (calibration.py:102-110)
//   ctr_ap_wll       sklearn average_precision_score on clip(nan_to_num(p), 1e-12, 1-1e-12) and the 50:50
//                    weighted logloss: descending radix sort of the f64 probabilities (order-preserving
//                    u64 keys) with the labels, tp = scan(labels), run-length groups of equal scores
//                    (sklearn's distinct thresholds), AP = sum_groups (tp_e - tp_prev) * tp_e / (e+1) / P
//   ctr_temp_nll     the LBFGS closure of fit_temperature at one T: sums of y log p, (1-y) log(1-p) and
//                    their d/dT (p = clamp(sigmoid(z/T), 1e-7, 1-1e-7); clamped elements have zero grad)
// All sums are f64 with a fixed reduction tree (fixed grid, fixed-order second pass): deterministic.
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_run_length_encode.hpp>
#include <rocprim/device/device_scan.hpp>

#include "common.h"
#include "ctr_hip.h"

namespace ctr {

constexpr int RED_BLOCKS = 1024, RED_THREADS = 256;   // 4 blocks per CU

__device__ __forceinline__ double block_sum_f64(double v, double* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) red[w] = v;
  __syncthreads();
  double s = 0.0;
  for (int i = 0; i < (int)(blockDim.x >> 6); ++i) s += red[i];
  return s;
}

// sum of NQ quantities: partial[b * NQ + q] per block (grid-stride in a fixed order), then one block
template <int NQ>
__global__ void reduce_final_kernel(const double* __restrict__ partial, int nb, double* __restrict__ out) {
  __shared__ double red[16];
  for (int q = 0; q < NQ; ++q) {
    double v = 0.0;
    for (int b = threadIdx.x; b < nb; b += blockDim.x) v += partial[b * NQ + q];
    v = block_sum_f64(v, red);
    if (threadIdx.x == 0) out[q] = v;
  }
}

__device__ __forceinline__ double sanitize(double p) {       // np.nan_to_num(nan=0.5, posinf=1, neginf=0)
  if (p != p) return 0.5;
  if (p == INFINITY) return 1.0;
  if (p == -INFINITY) return 0.0;
  return p;
}

__device__ __forceinline__ uint64_t order_key(double x) {    // u64 order == double order (no NaN here)
  const uint64_t b = __double_as_longlong(x);
  return (b >> 63) ? ~b : (b | 0x8000000000000000ULL);
}

__global__ void val_prob_kernel(const float* __restrict__ z, int n, float T, int calibrated, double* __restrict__ p) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    if (calibrated) {
      // the reference's predict_proba path is float32 end to end: TemperatureScaler on a float32 tensor,
      // then _sigmoid_stable_numpy and np.clip on the float32 array (src/utils/calibration.py:104-110)
      const float zt = fminf(fmaxf(z[i] / T, -50.f), 50.f);
      const float v = 1.0f / (1.0f + expf(-zt));
      p[i] = (double)fminf(fmaxf(v, 1e-7f), 1.0f - 1e-7f);
    } else {
      p[i] = 1.0 / (1.0 + exp(-(double)z[i]));
    }
  }
}

// keys for the AP sort + the WLL / label partial sums {sum -log p (pos), sum -log(1-p) (neg), n_pos}
__global__ void ap_prep_kernel(const double* __restrict__ p, const float* __restrict__ y, int n,
                               uint64_t* __restrict__ keys, uint32_t* __restrict__ labels, double* __restrict__ partial) {
  __shared__ double red[16];
  double lp = 0.0, ln = 0.0, np_ = 0.0;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const double q = fmin(fmax(sanitize(p[i]), 1e-12), 1.0 - 1e-12);
    const bool pos = y[i] == 1.0f;
    keys[i] = order_key(q);
    labels[i] = pos ? 1u : 0u;
    if (pos) {
      lp -= log(q);
      np_ += 1.0;
    } else {
      ln -= log(1.0 - q);
    }
  }
  lp = block_sum_f64(lp, red);
  ln = block_sum_f64(ln, red);
  np_ = block_sum_f64(np_, red);
  if (threadIdx.x == 0) {
    partial[blockIdx.x * 3 + 0] = lp;
    partial[blockIdx.x * 3 + 1] = ln;
    partial[blockIdx.x * 3 + 2] = np_;
  }
}

// AP contribution of each group of equal scores (sklearn's distinct thresholds), summed per block
__global__ void ap_groups_kernel(const uint32_t* __restrict__ tp, const uint32_t* __restrict__ counts,
                                 const uint32_t* __restrict__ starts, const uint32_t* __restrict__ n_groups,
                                 double* __restrict__ partial) {
  __shared__ double red[16];
  const uint32_t ng = *n_groups;
  double acc = 0.0;
  for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < ng; j += gridDim.x * blockDim.x) {
    const uint32_t s = starts[j], e = s + counts[j] - 1;
    const double te = (double)tp[e], tprev = s ? (double)tp[s - 1] : 0.0;
    acc += (te - tprev) * te / (double)(e + 1);
  }
  acc = block_sum_f64(acc, red);
  if (threadIdx.x == 0) partial[blockIdx.x] = acc;
}

__global__ void ap_final_kernel(const double* __restrict__ sums3, const double* __restrict__ apsum, int n,
                                double* __restrict__ out) {
  const double npos = sums3[2], nneg = (double)n - npos;
  // ap_score: 0.0 when y is all one class (metrics.py:19-20); WLL NaN then (:11-13)
  out[0] = (npos == 0.0 || nneg == 0.0) ? 0.0 : apsum[0] / npos;
  out[1] = (npos == 0.0 || nneg == 0.0) ? NAN : 0.5 * (sums3[0] / npos + sums3[1] / nneg);
  out[2] = npos;
}

// per-element math in f32 as the reference's closure (torch f32 on CPU), sums in f64
__global__ void temp_nll_kernel(const float* __restrict__ z, const float* __restrict__ y, int n, float T,
                                double* __restrict__ partial) {
  __shared__ double red[16];
  double s_pos = 0.0, s_neg = 0.0, g_pos = 0.0, g_neg = 0.0;
  const float invT2 = 1.0f / (T * T);
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const float zt = z[i] / T;
    const float v = 1.0f / (1.0f + expf(-zt));
    const bool clip = v < 1e-7f || v > 1.0f - 1e-7f;
    const float p = fminf(fmaxf(v, 1e-7f), 1.0f - 1e-7f);
    const float dzt = -z[i] * invT2;                       // d(z/T)/dT
    if (y[i] == 1.0f) {
      s_pos += (double)logf(p);
      if (!clip) g_pos += (double)((1.0f - p) * dzt);      // d log p / dT
    } else {
      s_neg += (double)logf(1.0f - p);
      if (!clip) g_neg -= (double)(p * dzt);               // d log(1-p) / dT
    }
  }
  s_pos = block_sum_f64(s_pos, red);
  s_neg = block_sum_f64(s_neg, red);
  g_pos = block_sum_f64(g_pos, red);
  g_neg = block_sum_f64(g_neg, red);
  if (threadIdx.x == 0) {
    partial[blockIdx.x * 4 + 0] = s_pos;
    partial[blockIdx.x * 4 + 1] = s_neg;
    partial[blockIdx.x * 4 + 2] = g_pos;
    partial[blockIdx.x * 4 + 3] = g_neg;
  }
}

struct MetricsWs {
  size_t keys, skeys, labels, slabels, tp, ukeys, counts, starts, ngroups, partial, sums, temp, total, temp_bytes;
};

static MetricsWs metrics_layout(int n) {
  MetricsWs w{};
  size_t t1 = 0, t2 = 0, t3 = 0, t4 = 0;
  (void)rocprim::radix_sort_pairs_desc(nullptr, t1, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                                       (const uint32_t*)nullptr, (uint32_t*)nullptr, (size_t)n);
  (void)rocprim::inclusive_scan(nullptr, t2, (const uint32_t*)nullptr, (uint32_t*)nullptr, (size_t)n,
                                rocprim::plus<uint32_t>());
  (void)rocprim::run_length_encode(nullptr, t3, (const uint64_t*)nullptr, (unsigned)n, (uint64_t*)nullptr,
                                   (uint32_t*)nullptr, (uint32_t*)nullptr);
  (void)rocprim::exclusive_scan(nullptr, t4, (const uint32_t*)nullptr, (uint32_t*)nullptr, 0u, (size_t)n,
                                rocprim::plus<uint32_t>());
  size_t tb = t1;
  if (t2 > tb) tb = t2;
  if (t3 > tb) tb = t3;
  if (t4 > tb) tb = t4;
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  size_t off = 0;
  w.keys = off; off += al(8 * (size_t)n);
  w.skeys = off; off += al(8 * (size_t)n);
  w.ukeys = off; off += al(8 * (size_t)n);
  w.labels = off; off += al(4 * (size_t)n);
  w.slabels = off; off += al(4 * (size_t)n);
  w.tp = off; off += al(4 * (size_t)n);
  w.counts = off; off += al(4 * (size_t)n);
  w.starts = off; off += al(4 * (size_t)n);
  w.ngroups = off; off += al(4);
  w.partial = off; off += al(8 * 4 * RED_BLOCKS);
  w.sums = off; off += al(8 * 8);
  w.temp = off; off += al(tb);
  w.temp_bytes = tb;
  w.total = off;
  return w;
}

}  // namespace ctr

using namespace ctr;

extern "C" size_t ctr_metrics_ws_size(int n) { return n > 0 ? metrics_layout(n).total : 4096; }

extern "C" int ctr_val_prob(const float* z, int n, float T, int calibrated, double* p, void* stream) {
  CTR_REQUIRE(!calibrated || T > 0.f, "ctr_val_prob: temperature must be positive");
  if (n <= 0) return 0;
  const int g = cdiv(n, 256) < 4096 ? cdiv(n, 256) : 4096;
  val_prob_kernel<<<g, 256, 0, (hipStream_t)stream>>>(z, n, T, calibrated, p);
  return check_launch("val_prob");
}

extern "C" int ctr_ap_wll(const double* p, const float* y, int n, double* out, void* ws, size_t ws_bytes,
                          void* stream) {
  hipStream_t s = (hipStream_t)stream;
  CTR_REQUIRE(n >= 0, "ctr_ap_wll: n < 0");
  const MetricsWs w = metrics_layout(n > 0 ? n : 1);
  CTR_REQUIRE(ws && ws_bytes >= w.total, "ctr_ap_wll: workspace too small (ctr_metrics_ws_size)");
  char* b = (char*)ws;
  double* partial = (double*)(b + w.partial);
  double* sums = (double*)(b + w.sums);
  if (n == 0) {
    (void)hipMemsetAsync(sums, 0, 8 * 8, s);
    ap_final_kernel<<<1, 1, 0, s>>>(sums, sums + 4, 0, out);
    return check_launch("ap_wll");
  }
  uint64_t* keys = (uint64_t*)(b + w.keys);
  uint64_t* skeys = (uint64_t*)(b + w.skeys);
  uint32_t* labels = (uint32_t*)(b + w.labels);
  uint32_t* slabels = (uint32_t*)(b + w.slabels);
  uint32_t* tp = (uint32_t*)(b + w.tp);
  uint32_t* counts = (uint32_t*)(b + w.counts);
  uint32_t* starts = (uint32_t*)(b + w.starts);
  uint32_t* ng = (uint32_t*)(b + w.ngroups);
  void* temp = b + w.temp;
  size_t tb = w.temp_bytes;
  ap_prep_kernel<<<RED_BLOCKS, RED_THREADS, 0, s>>>(p, y, n, keys, labels, partial);
  reduce_final_kernel<3><<<1, 256, 0, s>>>(partial, RED_BLOCKS, sums);
  hipError_t e = rocprim::radix_sort_pairs_desc(temp, tb, keys, skeys, labels, slabels, (size_t)n, 0, 64, s);
  CTR_REQUIRE(e == hipSuccess, "ctr_ap_wll: radix sort failed");
  tb = w.temp_bytes;
  e = rocprim::inclusive_scan(temp, tb, slabels, tp, (size_t)n, rocprim::plus<uint32_t>(), s);
  CTR_REQUIRE(e == hipSuccess, "ctr_ap_wll: scan failed");
  tb = w.temp_bytes;
  e = rocprim::run_length_encode(temp, tb, skeys, (unsigned)n, keys /* unique keys: scratch */, counts, ng, s);
  CTR_REQUIRE(e == hipSuccess, "ctr_ap_wll: run-length encode failed");
  tb = w.temp_bytes;
  e = rocprim::exclusive_scan(temp, tb, counts, starts, 0u, (size_t)n, rocprim::plus<uint32_t>(), s);
  CTR_REQUIRE(e == hipSuccess, "ctr_ap_wll: offsets scan failed");
  ap_groups_kernel<<<RED_BLOCKS, RED_THREADS, 0, s>>>(tp, counts, starts, ng, partial);
  reduce_final_kernel<1><<<1, 256, 0, s>>>(partial, RED_BLOCKS, sums + 4);
  ap_final_kernel<<<1, 1, 0, s>>>(sums, sums + 4, n, out);
  return check_launch("ap_wll");
}

extern "C" int ctr_temp_nll(const float* z, const float* y, int n, float T, double* out, void* ws, size_t ws_bytes,
                            void* stream) {
  hipStream_t s = (hipStream_t)stream;
  CTR_REQUIRE(T > 0.f, "ctr_temp_nll: temperature must be positive");
  CTR_REQUIRE(ws && ws_bytes >= 8 * 4 * RED_BLOCKS, "ctr_temp_nll: workspace too small (ctr_metrics_ws_size)");
  double* partial = (double*)ws;
  temp_nll_kernel<<<RED_BLOCKS, RED_THREADS, 0, s>>>(z, y, n, T, partial);
  reduce_final_kernel<4><<<1, 256, 0, s>>>(partial, RED_BLOCKS, out);
  return check_launch("temp_nll");
}

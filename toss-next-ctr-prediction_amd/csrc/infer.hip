// Fold-ensemble inference tail (src/infer.py:102-158): per-model calibration of the logits and the
// ensemble over models, on device -- the reference round-trips every batch's logits to the CPU for the
// calibrator (src/infer.py:112-116) and stacks the per-model probabilities with torch ops.
//
//   ctr_calibrate  p = clip(iso(clip(sigmoid(clip(z / T, -50, 50)))))  (src/utils/calibration.py:102-110
//                  with the temperature scaler and, if present, the isotonic map as its thresholds);
//                  without a calibrator p = clip(sigmoid(z)) (the model's prob, src/infer.py:108,122)
//   ctr_ensemble   src/utils/metrics.py:48-86: mean / geom_mean / logit_mean / median / trim_mean /
//                  weighted over M <= 32 models, one thread per sample
#include "common.h"
#include "ctr_hip.h"

namespace ctr {

constexpr float P_LO = 1e-7f, P_HI = 1.0f - 1e-7f;

__device__ __forceinline__ float clampf(float x, float lo, float hi) { return fminf(fmaxf(x, lo), hi); }

// np.interp over the isotonic thresholds (out_of_bounds="clip": ends extend flat)
__device__ float iso_interp(float x, const float* __restrict__ xs, const float* __restrict__ ys, int n) {
  if (x <= xs[0]) return ys[0];
  if (x >= xs[n - 1]) return ys[n - 1];
  int lo = 0, hi = n - 1;
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (xs[mid] <= x) lo = mid; else hi = mid;
  }
  const float dx = xs[hi] - xs[lo];
  return dx > 0.f ? ys[lo] + (x - xs[lo]) * (ys[hi] - ys[lo]) / dx : ys[hi];
}

__global__ void calibrate_kernel(const float* __restrict__ z, int n, float T, int has_T,
                                 const float* __restrict__ iso_x, const float* __restrict__ iso_y, int n_iso,
                                 float* __restrict__ p) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    float v;
    if (has_T || n_iso > 0) {
      const float zt = has_T ? z[i] / T : z[i];
      v = 1.0f / (1.0f + expf(-clampf(zt, -50.f, 50.f)));
      if (n_iso > 0) v = iso_interp(clampf(v, P_LO, P_HI), iso_x, iso_y, n_iso);
    } else {
      v = sigmoid_f(z[i]);
    }
    p[i] = clampf(v, P_LO, P_HI);
  }
}

__device__ __forceinline__ float logit_safe(float p) {
  p = clampf(p, P_LO, P_HI);
  return logf(p) - log1pf(-p);
}

// method: 0 mean, 1 geom_mean, 2 logit_mean, 3 median, 4 trim_mean (k models cut each side), 5 weighted
__global__ void ensemble_kernel(const float* __restrict__ P, int M, int B, int method, const float* __restrict__ w,
                                int k, float* __restrict__ out) {
  for (int b = blockIdx.x * blockDim.x + threadIdx.x; b < B; b += gridDim.x * blockDim.x) {
    float wsum = 0.f;
    if (w)
      for (int m = 0; m < M; ++m) wsum += w[m];
    float r;
    if (method == 0 || method == 5) {
      float s = 0.f;
      for (int m = 0; m < M; ++m) s += w ? P[(long)m * B + b] * (w[m] / wsum) : P[(long)m * B + b];
      r = w ? s : s / (float)M;
    } else if (method == 1) {
      float s = 0.f;
      for (int m = 0; m < M; ++m) {
        const float l = logf(clampf(P[(long)m * B + b], P_LO, P_HI));
        s += w ? l * (w[m] / wsum) : l;
      }
      r = expf(w ? s : s / (float)M);
    } else if (method == 2) {
      float s = 0.f;
      for (int m = 0; m < M; ++m) {
        const float l = logit_safe(P[(long)m * B + b]);
        s += w ? l * (w[m] / wsum) : l;
      }
      r = sigmoid_f(w ? s : s / (float)M);
    } else {    // median / trim_mean: sort the M values (M <= 32)
      float v[32];
      for (int m = 0; m < M; ++m) v[m] = P[(long)m * B + b];
      for (int i = 1; i < M; ++i) {
        const float x = v[i];
        int j = i - 1;
        while (j >= 0 && v[j] > x) {
          v[j + 1] = v[j];
          --j;
        }
        v[j + 1] = x;
      }
      if (method == 3) {
        r = v[(M - 1) / 2];                 // torch.median: the lower of the two middle values
      } else {
        float s = 0.f;
        for (int m = k; m < M - k; ++m) s += v[m];
        r = s / (float)(M - 2 * k);
      }
    }
    out[b] = r;
  }
}

}  // namespace ctr

using namespace ctr;

extern "C" int ctr_calibrate(const float* z, int n, float T, int has_T, const float* iso_x, const float* iso_y,
                             int n_iso, float* p, void* stream) {
  CTR_REQUIRE(!has_T || T > 0.f, "ctr_calibrate: temperature must be positive");
  CTR_REQUIRE(n_iso == 0 || (iso_x && iso_y), "ctr_calibrate: isotonic thresholds missing");
  if (n <= 0) return 0;
  calibrate_kernel<<<cdiv(n, 256) < 4096 ? cdiv(n, 256) : 4096, 256, 0, (hipStream_t)stream>>>(z, n, T, has_T, iso_x,
                                                                                              iso_y, n_iso, p);
  return check_launch("calibrate");
}

extern "C" int ctr_ensemble(const float* P, int M, int B, int method, const float* w, int k, float* out, void* stream) {
  CTR_REQUIRE(M >= 1 && M <= 32, "ctr_ensemble: 1..32 models");
  CTR_REQUIRE(method >= 0 && method <= 5, "ctr_ensemble: unknown method");
  CTR_REQUIRE(method != 5 || w, "ctr_ensemble: weighted needs weights");
  CTR_REQUIRE(method != 4 || (k >= 0 && 2 * k < M), "ctr_ensemble: trim k out of range");
  if (B <= 0) return 0;
  ensemble_kernel<<<cdiv(B, 256) < 4096 ? cdiv(B, 256) : 4096, 256, 0, (hipStream_t)stream>>>(P, M, B, method, w, k,
                                                                                             out);
  return check_launch("ensemble");
}

// AdamW + EMA element update shared by the dense arena stream (optim.hip) and the lazy table rows
// (lazy.hip).  Both must produce the same bits for the same sequence of ticks, so the arithmetic is
// spelled out with explicit fmaf (no reliance on the compiler's contraction choices) and lives in
// one place.
//
// torch/optim/adam.py _single_tensor_adam with decoupled weight decay (AdamW), then
// ModelEMA.update (src/utils/ema.py:92-131):
//   p *= 1 - lr*wd;  m.lerp_(g, 1-b1);  v = v*b2 + (1-b2) g^2;
//   p -= lr/bc1 * m / (sqrt(v)/sqrt(bc2) + eps);   e = e*d + (1-d) p
#pragma once
#include <cmath>

#include "common.h"

namespace ctr {

// One optimizer tick's scalars; also the layout of one entry of the lazy-update tick history.
// The per-element math uses the hardware sqrt / reciprocal (v_sqrt_f32, v_rcp_f32, ~1 ulp) and a
// multiply by 1/sqrt(bc2) where torch divides: a few ulp on the update term (itself ~lr relative to
// the parameter), far inside the parity tolerance, and ~3x fewer VALU cycles per element-tick --
// which is what bounds the lazy replay (the dense stream is HBM-bound either way).
struct OptScalars {
  float decay_mul;    // 1 - lr*wd
  float b1w;          // 1 - beta1 (lerp weight)
  float b2, omb2;     // beta2, 1 - beta2
  float eps;
  float step_size;    // lr / (1 - beta1^t)
  float rbc2;         // 1 / sqrt(1 - beta2^t)
  float ema_d, ema_omd;
  int do_adam, do_ema;
  int pad;
};
static_assert(sizeof(OptScalars) == 48, "history entry is 48 bytes");

// host-side scalar math in double, exactly as torch/optim/adam.py computes it in Python floats
inline OptScalars make_opt_scalars(float lr, float wd, float beta1, float beta2, float eps, int step,
                                   float ema_decay, int do_adam, int do_ema) {
  OptScalars s;
  const double bc1 = 1.0 - std::pow((double)beta1, step), bc2 = 1.0 - std::pow((double)beta2, step);
  s.decay_mul = (float)(1.0 - (double)lr * (double)wd);
  s.b1w = (float)(1.0 - (double)beta1);
  s.b2 = beta2;
  s.omb2 = (float)(1.0 - (double)beta2);
  s.eps = eps;
  s.step_size = (float)((double)lr / bc1);
  s.rbc2 = (float)(1.0 / std::sqrt(bc2));
  s.ema_d = ema_decay;
  s.ema_omd = (float)(1.0 - (double)ema_decay);
  s.do_adam = do_adam;
  s.do_ema = do_ema;
  s.pad = 0;
  return s;
}

// `#pragma clang fp contract(off)` in every element function: a caller's g = grad * coef would otherwise be
// fused into `g - m` after inlining (fma(grad, coef, -m)) in one caller and not in another, and the dense
// stream and the lazy replay would round m differently -- the explicit fmaf calls are the only fusions.
__device__ __forceinline__ void adam_elem(const OptScalars& s, float& p, float& m, float& v, float g) {
#pragma clang fp contract(off)
  p = p * s.decay_mul;                                  // param.mul_(1 - lr*wd)
  m = fmaf(s.b1w, g - m, m);                            // exp_avg.lerp_(grad, 1-beta1)
  v = fmaf(s.omb2 * g, g, v * s.b2);                    // exp_avg_sq.mul_(b2).addcmul_(g, g, 1-b2)
  const float denom = fmaf(__builtin_amdgcn_sqrtf(v), s.rbc2, s.eps);   // (sqrt(v) / bc2_sqrt).add_(eps)
  p = fmaf(-s.step_size, m * __builtin_amdgcn_rcpf(denom), p);          // param.addcdiv_(m, denom, -step)
}

__device__ __forceinline__ void ema_elem(const OptScalars& s, float p, float& e) {
#pragma clang fp contract(off)
  e = fmaf(e, s.ema_d, s.ema_omd * p);                  // shadow.mul_(d).add_(p, alpha=1-d)
}

__device__ __forceinline__ void adam_ema_elem(const OptScalars& s, float& p, float& m, float& v, float& e, float g,
                                              bool adam) {
  if (adam) adam_elem(s, p, m, v, g);
  if (s.do_ema) ema_elem(s, p, e);
}

// A tick with grad 0 (a table row no sample touched), bit-identical to adam_elem(.., g = 0):
// fmaf(b1w, 0 - m, m) == fmaf(b1w, -m, m) (the two differ only in the sign of a zero product, which
// the addend absorbs) and fmaf(omb2 * 0, 0, v * b2) == v * b2 (v >= 0).
__device__ __forceinline__ void idle_adam_elem(const OptScalars& s, float& p, float& m, float& v) {
#pragma clang fp contract(off)
  p = p * s.decay_mul;
  m = fmaf(s.b1w, -m, m);
  v = v * s.b2;
  const float denom = fmaf(__builtin_amdgcn_sqrtf(v), s.rbc2, s.eps);
  p = fmaf(-s.step_size, m * __builtin_amdgcn_rcpf(denom), p);
}

// Two elements of idle_adam_elem / ema_elem at once on packed f32 pairs (v_pk_mul_f32 / v_pk_fma_f32:
// each half is the same IEEE multiply / fused multiply-add as the scalar form, so the bits are equal);
// the square root and reciprocal stay per element.  For the VALU-bound replay of stepped rows.
typedef float f32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f32x2 splat2(float a) { return f32x2{a, a}; }

__device__ __forceinline__ void idle_adam_pk(const OptScalars& s, f32x2& p, f32x2& m, f32x2& v) {
#pragma clang fp contract(off)
  p = p * splat2(s.decay_mul);
  m = __builtin_elementwise_fma(splat2(s.b1w), -m, m);
  v = v * splat2(s.b2);
  const f32x2 sq = {__builtin_amdgcn_sqrtf(v.x), __builtin_amdgcn_sqrtf(v.y)};
  const f32x2 denom = __builtin_elementwise_fma(sq, splat2(s.rbc2), splat2(s.eps));
  const f32x2 r = {__builtin_amdgcn_rcpf(denom.x), __builtin_amdgcn_rcpf(denom.y)};
  p = __builtin_elementwise_fma(splat2(-s.step_size), m * r, p);
}

__device__ __forceinline__ void ema_pk(const OptScalars& s, f32x2 p, f32x2& e) {
#pragma clang fp contract(off)
  e = __builtin_elementwise_fma(e, splat2(s.ema_d), splat2(s.ema_omd) * p);
}

}  // namespace ctr

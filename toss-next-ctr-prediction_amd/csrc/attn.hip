// Self-attention core of DAREEncoderLayer over the K selected candidates (src/models/dare.py:53-62,
// MHA explicit path of torch.nn.functional.multi_head_attention_forward):
//   s_ij = mean_h rel[j-i+tk] + (q_i * sqrt(1/dh)) . k_j ;  p = softmax_j(s) ; p~ = dropout(p) ;
//   o_i = sum_j p~_ij v_j
// One workgroup per (sample, group of G heads); one thread per query row.  Heads are only dh = D/H
// = 4..8 wide -- far too thin for an MFMA tile -- so scores are VALU dot products against K/V rows
// broadcast from LDS.  The backward recomputes P from the saved row max / row sum (no K x K tensor
// ever reaches HBM), keeps one K x K tile per head in LDS, and reduces the positional-bias grad
// along diagonals in a fixed order (deterministic).
#include "common.h"
#include "ctr_hip.h"

namespace ctr {

constexpr int MAX_DH = 16;

struct AttnArgs {
  const float* qkv;     // (B*K, 3D)
  int B, K, H, dh, D, G;
  const float* relmean; // (2*tk+1) or null
  int tk;
  float scale;          // sqrt(1/dh) as the reference's python float -> fp32
  Drop drop;            // over ((b*H + h)*K + i)*K + j
  float* o;             // (B*K, D)
  float* mrow;          // (B*H*K)
  float* lrow;          // (B*H*K)
  // backward
  const float* dO;      // (B*K, D)
  float* dqkv;          // (B*K, 3D)
  float* drel_part;     // (B * H/G, 2*tk+1)
};

__device__ __forceinline__ float attn_bias(const AttnArgs& a, const float* srel, int i, int j) {
  return a.relmean ? srel[j - i + a.tk] : 0.f;
}

__global__ __launch_bounds__(256) void attn_fwd_kernel(AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int K = a.K, dh = a.dh, D = a.D, G = a.G;
  const int b = blockIdx.x, hg = blockIdx.y;
  float* sk = sm;                       // [G][K][dh]
  float* sv = sk + G * K * dh;          // [G][K][dh]
  float* srel = sv + G * K * dh;        // [2tk+1]
  const int nrel = 2 * a.tk + 1;
  const float* base = a.qkv + (long)b * K * 3 * D;
  for (int e = threadIdx.x; e < G * K * dh; e += blockDim.x) {
    const int g = e / (K * dh), r = e % (K * dh), j = r / dh, c = r % dh;
    const int h = hg * G + g;
    sk[e] = base[(long)j * 3 * D + D + h * dh + c];
    sv[e] = base[(long)j * 3 * D + 2 * D + h * dh + c];
  }
  if (a.relmean)
    for (int e = threadIdx.x; e < nrel; e += blockDim.x) srel[e] = a.relmean[e];
  __syncthreads();
  const int t = threadIdx.x;
  if (t >= G * K) return;
  const int g = t / K, i = t % K, h = hg * G + g;
  float qs[MAX_DH];
#pragma unroll
  for (int c = 0; c < MAX_DH; ++c) qs[c] = c < dh ? base[(long)i * 3 * D + h * dh + c] * a.scale : 0.f;
  const float* kg = sk + g * K * dh;
  const float* vg = sv + g * K * dh;
  float m = -INFINITY;
  for (int j = 0; j < K; ++j) {
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < MAX_DH; ++c)
      if (c < dh) s = fmaf(qs[c], kg[j * dh + c], s);
    s = attn_bias(a, srel, i, j) + s;
    m = fmaxf(m, s);
  }
  float l = 0.f;
  for (int j = 0; j < K; ++j) {
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < MAX_DH; ++c)
      if (c < dh) s = fmaf(qs[c], kg[j * dh + c], s);
    s = attn_bias(a, srel, i, j) + s;
    l += expf(s - m);
  }
  float acc[MAX_DH];
#pragma unroll
  for (int c = 0; c < MAX_DH; ++c) acc[c] = 0.f;
  const uint32_t rowbase = (uint32_t)((((long)b * a.H + h) * K + i) * K);
  for (int j = 0; j < K; ++j) {
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < MAX_DH; ++c)
      if (c < dh) s = fmaf(qs[c], kg[j * dh + c], s);
    s = attn_bias(a, srel, i, j) + s;
    float p = expf(s - m) / l;
    p = drop_apply(a.drop, rowbase + j, p);
#pragma unroll
    for (int c = 0; c < MAX_DH; ++c)
      if (c < dh) acc[c] = fmaf(p, vg[j * dh + c], acc[c]);
  }
#pragma unroll
  for (int c = 0; c < MAX_DH; ++c)
    if (c < dh) a.o[((long)b * K + i) * D + h * dh + c] = acc[c];
  const long r = ((long)b * a.H + h) * K + i;
  a.mrow[r] = m;
  a.lrow[r] = l;
}

__global__ __launch_bounds__(256) void attn_bwd_kernel(AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int K = a.K, dh = a.dh, D = a.D, G = a.G;
  const int b = blockIdx.x, hg = blockIdx.y;
  const int nrel = 2 * a.tk + 1;
  float* P = sm;                        // [G][K][K]
  float* sq = P + G * K * K;            // [G][K][dh] scaled q
  float* sk = sq + G * K * dh;
  float* sv = sk + G * K * dh;
  float* sdo = sv + G * K * dh;
  float* sD = sdo + G * K * dh;         // [G][K]
  float* srel = sD + G * K;             // [nrel]
  const float* base = a.qkv + (long)b * K * 3 * D;
  for (int e = threadIdx.x; e < G * K * dh; e += blockDim.x) {
    const int g = e / (K * dh), r = e % (K * dh), j = r / dh, c = r % dh;
    const int h = hg * G + g;
    sq[e] = base[(long)j * 3 * D + h * dh + c] * a.scale;
    sk[e] = base[(long)j * 3 * D + D + h * dh + c];
    sv[e] = base[(long)j * 3 * D + 2 * D + h * dh + c];
    sdo[e] = a.dO[((long)b * K + j) * D + h * dh + c];
  }
  if (a.relmean)
    for (int e = threadIdx.x; e < nrel; e += blockDim.x) srel[e] = a.relmean[e];
  __syncthreads();
  const int t = threadIdx.x;
  const bool act = t < G * K;
  const int g = act ? t / K : 0, i = act ? t % K : 0, h = hg * G + g;
  float* Pg = P + g * K * K;
  const float* qg = sq + g * K * dh;
  const float* kg = sk + g * K * dh;
  const float* vg = sv + g * K * dh;
  const float* dog = sdo + g * K * dh;
  // phase A: recompute P rows, D_i = do_i . o_i
  if (act) {
    const long r = ((long)b * a.H + h) * K + i;
    const float m = a.mrow[r], l = a.lrow[r];
    for (int j = 0; j < K; ++j) {
      float s = 0.f;
      for (int c = 0; c < dh; ++c) s = fmaf(qg[i * dh + c], kg[j * dh + c], s);
      s = attn_bias(a, srel, i, j) + s;
      Pg[i * K + j] = expf(s - m) / l;
    }
    float dd = 0.f;
    for (int c = 0; c < dh; ++c) dd = fmaf(dog[i * dh + c], a.o[((long)b * K + i) * D + h * dh + c], dd);
    sD[g * K + i] = dd;
  }
  __syncthreads();
  // phase B (thread = key column j): dv_j = sum_i p~_ij do_i
  if (act) {
    const int j = i;
    float acc[MAX_DH];
    for (int c = 0; c < MAX_DH; ++c) acc[c] = 0.f;
    for (int ii = 0; ii < K; ++ii) {
      const uint32_t idx = (uint32_t)((((long)b * a.H + h) * K + ii) * K + j);
      const float p = drop_apply(a.drop, idx, Pg[ii * K + j]);
#pragma unroll
      for (int c = 0; c < MAX_DH; ++c)
        if (c < dh) acc[c] = fmaf(p, dog[ii * dh + c], acc[c]);
    }
    for (int c = 0; c < dh; ++c) a.dqkv[((long)b * K + j) * 3 * D + 2 * D + h * dh + c] = acc[c];
  }
  __syncthreads();
  // phase C (row i): dS_ij = P_ij (dp~_ij * mask - D_i) ; dq_i = scale * sum_j dS_ij k_j
  if (act) {
    float acc[MAX_DH];
    for (int c = 0; c < MAX_DH; ++c) acc[c] = 0.f;
    const float Di = sD[g * K + i];
    const uint32_t rowbase = (uint32_t)((((long)b * a.H + h) * K + i) * K);
    for (int j = 0; j < K; ++j) {
      float dp = 0.f;
      for (int c = 0; c < dh; ++c) dp = fmaf(dog[i * dh + c], vg[j * dh + c], dp);
      if (a.drop.thresh) dp = drop_keep(a.drop, rowbase + j) ? dp * a.drop.scale : 0.f;
      const float ds = Pg[i * K + j] * (dp - Di);
      Pg[i * K + j] = ds;
#pragma unroll
      for (int c = 0; c < MAX_DH; ++c)
        if (c < dh) acc[c] = fmaf(ds, kg[j * dh + c], acc[c]);
    }
    for (int c = 0; c < dh; ++c) a.dqkv[((long)b * K + i) * 3 * D + h * dh + c] = acc[c] * a.scale;
  }
  __syncthreads();
  // phase D (column j): dk_j = sum_i dS_ij qs_i
  if (act) {
    const int j = i;
    float acc[MAX_DH];
    for (int c = 0; c < MAX_DH; ++c) acc[c] = 0.f;
    for (int ii = 0; ii < K; ++ii) {
      const float ds = Pg[ii * K + j];
#pragma unroll
      for (int c = 0; c < MAX_DH; ++c)
        if (c < dh) acc[c] = fmaf(ds, qg[ii * dh + c], acc[c]);
    }
    for (int c = 0; c < dh; ++c) a.dqkv[((long)b * K + j) * 3 * D + D + h * dh + c] = acc[c];
  }
  // phase E: positional-bias grad, summed along diagonals j - i = o, heads in order
  if (a.relmean) {
    for (int e = threadIdx.x; e < nrel; e += blockDim.x) {
      const int o = e - a.tk;
      float s = 0.f;
      if (o > -K && o < K) {
        for (int gg = 0; gg < G; ++gg) {
          const float* Pq = P + gg * K * K;
          const int i0 = o >= 0 ? 0 : -o, i1 = o >= 0 ? K - o : K;
          for (int ii = i0; ii < i1; ++ii) s += Pq[ii * K + ii + o];
        }
      }
      a.drel_part[((long)b * gridDim.y + hg) * nrel + e] = s;
    }
  }
}

static int pick_group(int H, int K, size_t per_head_lds, size_t lds_cap) {
  int best = 1;
  for (int g = 1; g <= H; ++g)
    if (H % g == 0 && g * K <= 256 && g * per_head_lds <= lds_cap) best = g;
  return best;
}

}  // namespace ctr

using namespace ctr;

extern "C" int ctr_attn_fwd(const float* qkv, int B, int K, int H, int D, const float* relmean, int tk, float scale,
                            uint32_t drop_key, uint32_t drop_thresh, float drop_scale, float* o, float* mrow,
                            float* lrow, void* stream) {
  if (B == 0) return 0;
  const int dh = D / H;
  CTR_REQUIRE(D % H == 0 && dh <= MAX_DH, "head dim must divide D and be <= 16");
  CTR_REQUIRE(K <= 256, "K > 256");
  CTR_REQUIRE(!relmean || tk >= K - 1, "positional-bias table shorter than K");
  const int G = pick_group(H, K, (size_t)2 * K * dh * 4, 64 * 1024);
  AttnArgs a{};
  a.qkv = qkv; a.B = B; a.K = K; a.H = H; a.dh = dh; a.D = D; a.G = G;
  a.relmean = relmean; a.tk = tk; a.scale = scale; a.drop = Drop{drop_key, drop_thresh, drop_scale};
  a.o = o; a.mrow = mrow; a.lrow = lrow;
  size_t sm = ((size_t)2 * G * K * dh + 2 * tk + 1) * sizeof(float);
  attn_fwd_kernel<<<dim3(B, H / G), 256, sm, (hipStream_t)stream>>>(a);
  return check_launch("attn_fwd");
}

extern "C" int ctr_attn_bwd_nparts(int H, int K, int D) {
  const int dh = D / H;
  const int G = pick_group(H, K, (size_t)(K * K + 4 * K * dh + K) * 4, 100 * 1024);
  return H / G;
}

extern "C" int ctr_attn_bwd(const float* qkv, const float* o, const float* dO, int B, int K, int H, int D,
                            const float* relmean, int tk, float scale, uint32_t drop_key, uint32_t drop_thresh,
                            float drop_scale, const float* mrow, const float* lrow, float* dqkv, float* drel_part,
                            void* stream) {
  if (B == 0) return 0;
  const int dh = D / H;
  CTR_REQUIRE(D % H == 0 && dh <= MAX_DH, "head dim must divide D and be <= 16");
  CTR_REQUIRE(K <= 256, "K > 256");
  const int G = pick_group(H, K, (size_t)(K * K + 4 * K * dh + K) * 4, 100 * 1024);
  AttnArgs a{};
  a.qkv = qkv; a.B = B; a.K = K; a.H = H; a.dh = dh; a.D = D; a.G = G;
  a.relmean = relmean; a.tk = tk; a.scale = scale; a.drop = Drop{drop_key, drop_thresh, drop_scale};
  a.o = const_cast<float*>(o); a.mrow = const_cast<float*>(mrow); a.lrow = const_cast<float*>(lrow);
  a.dO = dO; a.dqkv = dqkv; a.drel_part = drel_part;
  size_t sm = ((size_t)G * K * K + 4 * (size_t)G * K * dh + G * K + 2 * tk + 1) * sizeof(float);
  CTR_REQUIRE(sm <= 160 * 1024, "attention backward tile exceeds LDS");
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)attn_bwd_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr_set = true;
  }
  attn_bwd_kernel<<<dim3(B, H / G), 256, sm, (hipStream_t)stream>>>(a);
  return check_launch("attn_bwd");
}

// Self-attention core of DAREEncoderLayer over the K selected candidates (src/models/dare.py:53-62,
// MHA explicit path of torch.nn.functional.multi_head_attention_forward):
//   s_ij = mean_h rel[j-i+tk] + (q_i * sqrt(1/dh)) . k_j ;  p = softmax_j(s) ; p~ = dropout(p) ;
//   o_i = sum_j p~_ij v_j
// One workgroup per (sample, group of G heads); one thread per query row (forward, backward row pass)
// or key column (backward column pass).  Heads are only dh = D/H = 4..8 wide -- far too thin for an
// MFMA tile -- so scores are VALU dot products against K/V rows that every lane of a wave reads at
// the same LDS address (broadcast).  The backward recomputes P from the saved row max / row sum; only
// dS (K x (K+1), odd stride: conflict-free row reads) is kept in LDS, no K x K tensor reaches HBM.
// The positional-bias grad is reduced along diagonals in a fixed order (deterministic).
#include "common.h"
#include "ctr_hip.h"

namespace ctr {

struct AttnArgs {
  const float* qkv;     // (B*K, 3D)
  int B, K, H, D, G;
  const float* relmean; // (2*tk+1) or null
  int tk;
  float scale;          // sqrt(1/dh) as the reference's python float -> fp32
  Drop drop;            // over ((b*H + h)*K + i)*K + j
  float* o;             // (B*K, D)
  float* mrow;          // (B*H*K) row max of s
  float* lrow;          // (B*H*K) row sum of exp(s - max)
  const float* dO;      // (B*K, D)
  float* dqkv;          // (B*K, 3D)
  float* drel_part;     // (B * H/G, 2*tk+1)
};

template <int DH>
__device__ __forceinline__ float dotv(const float (&a)[DH], const float* b) {
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < DH; ++c) s = fmaf(a[c], b[c], s);
  return s;
}

template <int DH>
__global__ __launch_bounds__(256) void attn_fwd_kernel(AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int K = a.K, D = a.D, G = a.G;
  const int b = blockIdx.x, hg = blockIdx.y;
  float* sk = sm;                       // [G][K][DH]
  float* sv = sk + G * K * DH;          // [G][K][DH]
  float* srel = sv + G * K * DH;        // [2tk+1]
  const float* base = a.qkv + (long)b * K * 3 * D;
  for (int e = threadIdx.x; e < G * K * DH; e += blockDim.x) {
    const int g = e / (K * DH), r = e % (K * DH), j = r / DH, c = r % DH;
    const int col = (hg * G + g) * DH + c;
    sk[e] = base[(long)j * 3 * D + D + col];
    sv[e] = base[(long)j * 3 * D + 2 * D + col];
  }
  if (a.relmean)
    for (int e = threadIdx.x; e < 2 * a.tk + 1; e += blockDim.x) srel[e] = a.relmean[e];
  __syncthreads();
  const int t = threadIdx.x;
  if (t >= G * K) return;
  const int g = t / K, i = t % K, h = hg * G + g;
  float qs[DH];
#pragma unroll
  for (int c = 0; c < DH; ++c) qs[c] = base[(long)i * 3 * D + h * DH + c] * a.scale;
  const float* kg = sk + g * K * DH;
  const float* vg = sv + g * K * DH;
  const float* rb = srel + a.tk - i;     // rb[j] = relmean[j - i + tk]
  const bool bias = a.relmean != nullptr;
  float m = -INFINITY;
  for (int j = 0; j < K; ++j) {
    const float s = (bias ? rb[j] : 0.f) + dotv<DH>(qs, kg + j * DH);
    m = fmaxf(m, s);
  }
  float l = 0.f;
  float acc[DH];
#pragma unroll
  for (int c = 0; c < DH; ++c) acc[c] = 0.f;
  const uint32_t rowbase = (uint32_t)((((long)b * a.H + h) * K + i) * K);
  for (int j = 0; j < K; ++j) {
    const float s = (bias ? rb[j] : 0.f) + dotv<DH>(qs, kg + j * DH);
    const float e = expf(s - m);
    l += e;
    const float w = a.drop.thresh ? (drop_keep(a.drop, rowbase + j) ? e * a.drop.scale : 0.f) : e;
#pragma unroll
    for (int c = 0; c < DH; ++c) acc[c] = fmaf(w, vg[j * DH + c], acc[c]);
  }
  const float inv = 1.0f / l;
#pragma unroll
  for (int c = 0; c < DH; ++c) a.o[((long)b * K + i) * D + h * DH + c] = acc[c] * inv;
  const long r = ((long)b * a.H + h) * K + i;
  a.mrow[r] = m;
  a.lrow[r] = l;
}

template <int DH>
__global__ __launch_bounds__(256) void attn_bwd_kernel(AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int K = a.K, D = a.D, G = a.G;
  const int KP = K + 1;                    // odd row stride
  const int b = blockIdx.x, hg = blockIdx.y;
  const int nrel = 2 * a.tk + 1;
  float* sq = sm;                          // [G][K][DH] scaled q
  float* sk = sq + G * K * DH;
  float* sv = sk + G * K * DH;
  float* sdo = sv + G * K * DH;
  float* sm_ = sdo + G * K * DH;           // [G][K] row max
  float* sl = sm_ + G * K;                 // [G][K] row sum
  float* srel = sl + G * K;                // [nrel]
  float* dS = srel + ((nrel + 3) & ~3);    // [G][K][KP]
  const float* base = a.qkv + (long)b * K * 3 * D;
  for (int e = threadIdx.x; e < G * K * DH; e += blockDim.x) {
    const int g = e / (K * DH), r = e % (K * DH), j = r / DH, c = r % DH;
    const int col = (hg * G + g) * DH + c;
    sq[e] = base[(long)j * 3 * D + col] * a.scale;
    sk[e] = base[(long)j * 3 * D + D + col];
    sv[e] = base[(long)j * 3 * D + 2 * D + col];
    sdo[e] = a.dO[((long)b * K + j) * D + col];
  }
  for (int e = threadIdx.x; e < G * K; e += blockDim.x) {
    const int g = e / K, i = e % K;
    const long r = ((long)b * a.H + hg * G + g) * K + i;
    sm_[e] = a.mrow[r];
    sl[e] = a.lrow[r];
  }
  if (a.relmean)
    for (int e = threadIdx.x; e < nrel; e += blockDim.x) srel[e] = a.relmean[e];
  __syncthreads();
  const int t = threadIdx.x;
  const bool act = t < G * K;
  const bool bias = a.relmean != nullptr;
  const int g = act ? t / K : 0, i = act ? t % K : 0, h = hg * G + g;
  const float* qg = sq + g * K * DH;
  const float* kg = sk + g * K * DH;
  const float* vg = sv + g * K * DH;
  const float* dog = sdo + g * K * DH;
  float* dSg = dS + g * K * KP;
  const uint32_t hbase = (uint32_t)(((long)b * a.H + h) * K * K);
  // ---- row pass (thread = query row i): P, dP~, dS, dq
  if (act) {
    float qi[DH], di[DH], oi[DH];
#pragma unroll
    for (int c = 0; c < DH; ++c) {
      qi[c] = qg[i * DH + c];
      di[c] = dog[i * DH + c];
      oi[c] = a.o[((long)b * K + i) * D + h * DH + c];
    }
    const float Di = dotv<DH>(di, oi);
    const float mi = sm_[g * K + i], li = 1.0f / sl[g * K + i];
    const float* rb = srel + a.tk - i;
    float dq[DH];
#pragma unroll
    for (int c = 0; c < DH; ++c) dq[c] = 0.f;
    for (int j = 0; j < K; ++j) {
      const float s = (bias ? rb[j] : 0.f) + dotv<DH>(qi, kg + j * DH);
      const float p = expf(s - mi) * li;
      float dp = dotv<DH>(di, vg + j * DH);
      if (a.drop.thresh) dp = drop_keep(a.drop, hbase + (uint32_t)(i * K + j)) ? dp * a.drop.scale : 0.f;
      const float ds = p * (dp - Di);
      dSg[i * KP + j] = ds;
#pragma unroll
      for (int c = 0; c < DH; ++c) dq[c] = fmaf(ds, kg[j * DH + c], dq[c]);
    }
#pragma unroll
    for (int c = 0; c < DH; ++c) a.dqkv[((long)b * K + i) * 3 * D + h * DH + c] = dq[c] * a.scale;
  }
  __syncthreads();
  // ---- column pass (thread = key column j): dk_j = sum_i dS_ij qs_i ; dv_j = sum_i p~_ij do_i
  if (act) {
    const int j = i;
    float kj[DH], dk[DH], dv[DH];
#pragma unroll
    for (int c = 0; c < DH; ++c) {
      kj[c] = kg[j * DH + c];
      dk[c] = 0.f;
      dv[c] = 0.f;
    }
    for (int ii = 0; ii < K; ++ii) {
      const float ds = dSg[ii * KP + j];
      const float s = (bias ? srel[a.tk + j - ii] : 0.f) + dotv<DH>(kj, qg + ii * DH);
      float p = expf(s - sm_[g * K + ii]) / sl[g * K + ii];
      if (a.drop.thresh) p = drop_keep(a.drop, hbase + (uint32_t)(ii * K + j)) ? p * a.drop.scale : 0.f;
#pragma unroll
      for (int c = 0; c < DH; ++c) {
        dk[c] = fmaf(ds, qg[ii * DH + c], dk[c]);
        dv[c] = fmaf(p, dog[ii * DH + c], dv[c]);
      }
    }
#pragma unroll
    for (int c = 0; c < DH; ++c) {
      a.dqkv[((long)b * K + j) * 3 * D + D + h * DH + c] = dk[c];
      a.dqkv[((long)b * K + j) * 3 * D + 2 * D + h * DH + c] = dv[c];
    }
  }
  // ---- positional-bias grad: sum of dS along diagonals j - i = o, heads of the group in order
  if (bias) {
    for (int e = threadIdx.x; e < nrel; e += blockDim.x) {
      const int o = e - a.tk;
      float s = 0.f;
      if (o > -K && o < K) {
        const int i0 = o >= 0 ? 0 : -o, i1 = o >= 0 ? K - o : K;
        for (int gg = 0; gg < G; ++gg) {
          const float* Pq = dS + gg * K * KP;
          for (int ii = i0; ii < i1; ++ii) s += Pq[ii * KP + ii + o];
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

static size_t bwd_lds(int G, int K, int dh, int tk) {
  const int nrel = 2 * tk + 1;
  return ((size_t)4 * G * K * dh + 2 * G * K + ((nrel + 3) & ~3) + (size_t)G * K * (K + 1)) * sizeof(float);
}

static int bwd_group(int H, int K, int dh) {
  return pick_group(H, K, (size_t)(K * (K + 1) + 4 * K * dh + 2 * K) * 4, 80 * 1024);
}

template <int DH>
static void launch_fwd(const AttnArgs& a, size_t sm, hipStream_t s) {
  attn_fwd_kernel<DH><<<dim3(a.B, a.H / a.G), (a.G * a.K + 63) / 64 * 64, sm, s>>>(a);
}

template <int DH>
static void launch_bwd(const AttnArgs& a, size_t sm, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)attn_bwd_kernel<DH>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024);
    attr = true;
  }
  attn_bwd_kernel<DH><<<dim3(a.B, a.H / a.G), (a.G * a.K + 63) / 64 * 64, sm, s>>>(a);
}

}  // namespace ctr

using namespace ctr;

extern "C" int ctr_attn_fwd(const float* qkv, int B, int K, int H, int D, const float* relmean, int tk, float scale,
                            uint32_t drop_key, uint32_t drop_thresh, float drop_scale, float* o, float* mrow,
                            float* lrow, void* stream) {
  if (B == 0) return 0;
  const int dh = D / H;
  CTR_REQUIRE(D % H == 0 && (dh == 2 || dh == 4 || dh == 8 || dh == 16), "head dim must be 2, 4, 8 or 16");
  CTR_REQUIRE(K <= 256, "K > 256");
  CTR_REQUIRE(!relmean || tk >= K - 1, "positional-bias table shorter than K");
  const int G = pick_group(H, K, (size_t)2 * K * dh * 4, 64 * 1024);
  AttnArgs a{};
  a.qkv = qkv; a.B = B; a.K = K; a.H = H; a.D = D; a.G = G;
  a.relmean = relmean; a.tk = tk; a.scale = scale; a.drop = Drop{drop_key, drop_thresh, drop_scale};
  a.o = o; a.mrow = mrow; a.lrow = lrow;
  const size_t sm = ((size_t)2 * G * K * dh + 2 * tk + 1) * sizeof(float);
  hipStream_t s = (hipStream_t)stream;
  switch (dh) {
    case 2: launch_fwd<2>(a, sm, s); break;
    case 4: launch_fwd<4>(a, sm, s); break;
    case 8: launch_fwd<8>(a, sm, s); break;
    default: launch_fwd<16>(a, sm, s); break;
  }
  return check_launch("attn_fwd");
}

extern "C" int ctr_attn_bwd_nparts(int H, int K, int D) { return H / bwd_group(H, K, D / H); }

extern "C" int ctr_attn_bwd(const float* qkv, const float* o, const float* dO, int B, int K, int H, int D,
                            const float* relmean, int tk, float scale, uint32_t drop_key, uint32_t drop_thresh,
                            float drop_scale, const float* mrow, const float* lrow, float* dqkv, float* drel_part,
                            void* stream) {
  if (B == 0) return 0;
  const int dh = D / H;
  CTR_REQUIRE(D % H == 0 && (dh == 2 || dh == 4 || dh == 8 || dh == 16), "head dim must be 2, 4, 8 or 16");
  CTR_REQUIRE(K <= 256, "K > 256");
  const int G = bwd_group(H, K, dh);
  AttnArgs a{};
  a.qkv = qkv; a.B = B; a.K = K; a.H = H; a.D = D; a.G = G;
  a.relmean = relmean; a.tk = tk; a.scale = scale; a.drop = Drop{drop_key, drop_thresh, drop_scale};
  a.o = const_cast<float*>(o); a.mrow = const_cast<float*>(mrow); a.lrow = const_cast<float*>(lrow);
  a.dO = dO; a.dqkv = dqkv; a.drel_part = drel_part;
  const size_t sm = bwd_lds(G, K, dh, tk);
  CTR_REQUIRE(sm <= 160 * 1024, "attention backward tile exceeds LDS");
  hipStream_t s = (hipStream_t)stream;
  switch (dh) {
    case 2: launch_bwd<2>(a, sm, s); break;
    case 4: launch_bwd<4>(a, sm, s); break;
    case 8: launch_bwd<8>(a, sm, s); break;
    default: launch_bwd<16>(a, sm, s); break;
  }
  return check_launch("attn_bwd");
}

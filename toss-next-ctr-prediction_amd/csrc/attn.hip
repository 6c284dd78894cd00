// Self-attention core of DAREEncoderLayer over the K selected candidates (src/models/dare.py:53-62,
// MHA explicit path of torch.nn.functional.multi_head_attention_forward):
//   s_ij = mean_h rel[j-i+tk] + (q_i * sqrt(1/dh)) . k_j ;  p = softmax_j(s) ; p~ = dropout(p) ;
//   o_i = sum_j p~_ij v_j
// One workgroup per (sample, group of G heads).  Heads are only dh = D/H = 2..16 wide -- far too thin
// for an MFMA tile (a 16x16x4 f32 MFMA would waste 3/4 of its N on a dh = 4 PV product) -- so scores
// are VALU dot products against K/V/Q rows that a whole wave reads at one LDS address (broadcast).
// The per-element costs that matter are exp and the counter-hash dropout, so:
//   * the forward evaluates the hash once and stores the keep bits (B*H*K*ceil(K/32) words: ~15 MB
//     per layer at the benchmark shape) -- the backward reads bits instead of re-hashing;
//   * the backward is one pass per key column j (thread = j) that recomputes p_ij once, writes dS_ij
//     to LDS and accumulates dk_j, dv_j; a second, cheap pass per query row i sums dq_i = dS_i. k.
// Nothing K x K reaches HBM.  The positional-bias grad is reduced along diagonals in a fixed order.
#include "common.h"
#include "ctr_hip.h"

namespace ctr {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

struct AttnArgs {
  const float* qkv;     // (B*K, 3D)
  int B, K, H, D, G;
  const float* relmean; // (2*tk+1) or null
  int tk;
  float scale;          // sqrt(1/dh) as the reference's python float -> fp32
  Drop drop;            // over ((b*H + h)*K + i)*K + j
  uint32_t* mask;       // (B*H*K, KW) keep bits of p~ (dropout only)
  int KW;               // words per mask row = ceil(K/32)
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

// exp(x) on the hardware exp2 (v_exp_f32, ~1 ulp); forward and backward use the same formula
__device__ __forceinline__ float fexp(float x) { return __builtin_amdgcn_exp2f(x * 1.4426950408889634f); }

template <int DH, bool BIAS, bool DROP>
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
  if (BIAS)
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
  float m = -INFINITY;
#pragma unroll 4
  for (int j = 0; j < K; ++j) {
    const float s = (BIAS ? rb[j] : 0.f) + dotv<DH>(qs, kg + j * DH);
    m = fmaxf(m, s);
  }
  float l = 0.f;
  float acc[DH];
#pragma unroll
  for (int c = 0; c < DH; ++c) acc[c] = 0.f;
  const long r = ((long)b * a.H + h) * K + i;
  const uint32_t rowbase = (uint32_t)(r * K);
  uint32_t* mrow_bits = a.mask + r * a.KW;
  for (int j0 = 0; j0 < K; j0 += 32) {          // one keep-bit word per 32 keys
    const int j1 = min(K, j0 + 32);
    uint32_t word = 0;
    auto elem = [&](int j, bool keep) {
      const float s = (BIAS ? rb[j] : 0.f) + dotv<DH>(qs, kg + j * DH);
      const float e = fexp(s - m);
      l += e;
      float w = e;
      if (DROP) {
        word |= (uint32_t)keep << (j - j0);
        w = keep ? e * a.drop.scale : 0.f;
      }
#pragma unroll
      for (int c = 0; c < DH; ++c) acc[c] = fmaf(w, vg[j * DH + c], acc[c]);
    };
    if (DROP && (K & 1) == 0) {
      // even K: every row starts on an even element index, so keys (j, j+1) share one pair hash
#pragma unroll 2
      for (int j = j0; j < j1; j += 2) {
        const uint32_t bits = drop_pair_bits(a.drop, (rowbase + j) >> 1);
        elem(j, drop_pair_keep(a.drop, bits, 0));
        elem(j + 1, drop_pair_keep(a.drop, bits, 1));
      }
    } else {
#pragma unroll 4
      for (int j = j0; j < j1; ++j) elem(j, DROP ? drop_keep(a.drop, rowbase + j) : true);
    }
    if (DROP) mrow_bits[j0 >> 5] = word;
  }
  const float inv = 1.0f / l;
#pragma unroll
  for (int c = 0; c < DH; ++c) a.o[((long)b * K + i) * D + h * DH + c] = acc[c] * inv;
  a.mrow[r] = m;
  a.lrow[r] = l;
}

// Packed forward for K <= 64, K even, dh in {4, 8} (cfg2: K = 60, dh = 4).  Same thread mapping as
// attn_fwd_kernel (thread = query row i of one head), but every per-element step runs on key PAIRS in
// packed f32 (v_pk_fma / v_pk_add / v_pk_mul: two scores per instruction): K is stored pair-interleaved
// ([j/2][c][2]) so one ds_read_b128 yields (k_j,c, k_j+1,c) pairs; the scores stay in registers between
// the max and the exp pass (no second QK product); scores live in log2 units (q pre-scaled by
// sqrt(1/dh) log2(e), the bias by log2(e)), so p = exp2(s - m) is one subtract and one v_exp; the pair's
// dropout hash is the pair's own (K even: element 2k of a row is always even); 1/(1-p) and 1/l are applied
// once per row.  mrow is stored in natural units (m ln 2) for the backward's recompute.
template <int DH, bool BIAS, bool DROP>
__global__ __launch_bounds__(256) void attn_fwd_pk_kernel(AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  constexpr float L2E = 1.4426950408889634f;
  const int K = a.K, D = a.D, G = a.G, KP = K >> 1;
  const int b = blockIdx.x, hg = blockIdx.y;
  const int nrel = 2 * a.tk + 1, nr2 = (nrel + 2) & ~1;
  float* sk = sm;                       // [G][K/2][DH][2]
  float* sv = sk + G * K * DH;          // [G][K][DH]
  float* s0 = sv + G * K * DH;          // [nr2] rel * log2e
  float* s1 = s0 + nr2;                 // [nr2] shifted by one: s1[e] = rel[e + 1] * log2e
  const float* base = a.qkv + (long)b * K * 3 * D;
  for (int e = threadIdx.x; e < G * K * DH; e += blockDim.x) {
    const int g = e / (K * DH), r = e % (K * DH), j = r / DH, c = r % DH;
    const int col = (hg * G + g) * DH + c;
    sk[g * K * DH + (j >> 1) * 2 * DH + 2 * c + (j & 1)] = base[(long)j * 3 * D + D + col];
    sv[e] = base[(long)j * 3 * D + 2 * D + col];
  }
  if (BIAS)
    for (int e = threadIdx.x; e < nr2; e += blockDim.x) {
      s0[e] = e < nrel ? a.relmean[e] * L2E : 0.f;
      s1[e] = e + 1 < nrel ? a.relmean[e + 1] * L2E : 0.f;
    }
  __syncthreads();
  const int t = threadIdx.x;
  if (t >= G * K) return;
  const int g = t / K, i = t % K, h = hg * G + g;
  const float qsc = a.scale * L2E;
  f32x2 q2[DH];
#pragma unroll
  for (int c = 0; c < DH; ++c) {
    const float v = base[(long)i * 3 * D + h * DH + c] * qsc;
    q2[c] = f32x2{v, v};
  }
  const float* kg = sk + g * K * DH;
  const float* vg = sv + g * K * DH;
  const int bi = a.tk - i;                               // bias index of key 0
  const float* rbp = (bi & 1) ? s1 + (bi - 1) : s0 + bi;  // pair jp: rbp[2 jp], rbp[2 jp + 1], 8-byte aligned
  f32x2 sc[32];
  f32x2 mx = {-INFINITY, -INFINITY};
#pragma unroll
  for (int jp = 0; jp < 32; ++jp) {
    if (jp < KP) {
      const f32x4* kp = (const f32x4*)(kg + jp * 2 * DH);
      f32x2 acc = BIAS ? *(const f32x2*)(rbp + 2 * jp) : f32x2{0.f, 0.f};
#pragma unroll
      for (int c2 = 0; c2 < DH / 2; ++c2) {
        const f32x4 kk = kp[c2];
        acc = q2[2 * c2] * f32x2{kk[0], kk[1]} + acc;
        acc = q2[2 * c2 + 1] * f32x2{kk[2], kk[3]} + acc;
      }
      sc[jp] = acc;
      mx = f32x2{fmaxf(mx.x, acc.x), fmaxf(mx.y, acc.y)};
    }
  }
  const float m = fmaxf(mx.x, mx.y);
  f32x2 l2 = {0.f, 0.f};
  f32x2 acc[DH / 2];
#pragma unroll
  for (int c2 = 0; c2 < DH / 2; ++c2) acc[c2] = f32x2{0.f, 0.f};
  const long r = ((long)b * a.H + h) * K + i;
  const uint32_t pair0 = (uint32_t)(r * K) >> 1;
  uint32_t w0 = 0, w1 = 0;
  const uint32_t thr = a.drop.thresh;
#pragma unroll
  for (int jp = 0; jp < 32; ++jp) {
    if (jp < KP) {
      const f32x2 e = {__builtin_amdgcn_exp2f(sc[jp].x - m), __builtin_amdgcn_exp2f(sc[jp].y - m)};
      l2 += e;
      f32x2 w = e;
      if (DROP) {
        const uint32_t hb = drop_pair_bits(a.drop, pair0 + jp);
        const bool k0 = (hb & 0xFFFFu) >= thr, k1 = (hb >> 16) >= thr;
        w = f32x2{k0 ? e.x : 0.f, k1 ? e.y : 0.f};
        const uint32_t bits = (k0 ? 1u : 0u) | (k1 ? 2u : 0u);
        if (jp < 16) w0 |= bits << (2 * jp);
        else w1 |= bits << (2 * jp - 32);
      }
      const f32x4* v0 = (const f32x4*)(vg + 2 * jp * DH);
      const f32x4* v1 = (const f32x4*)(vg + (2 * jp + 1) * DH);
#pragma unroll
      for (int c4 = 0; c4 < DH / 4; ++c4) {
        const f32x4 a0 = v0[c4], a1 = v1[c4];
        acc[2 * c4] = f32x2{w.x, w.x} * f32x2{a0[0], a0[1]} + acc[2 * c4];
        acc[2 * c4 + 1] = f32x2{w.x, w.x} * f32x2{a0[2], a0[3]} + acc[2 * c4 + 1];
        acc[2 * c4] = f32x2{w.y, w.y} * f32x2{a1[0], a1[1]} + acc[2 * c4];
        acc[2 * c4 + 1] = f32x2{w.y, w.y} * f32x2{a1[2], a1[3]} + acc[2 * c4 + 1];
      }
    }
  }
  const float l = l2.x + l2.y;
  const float inv = (DROP ? a.drop.scale : 1.0f) / l;
  float* op = a.o + ((long)b * K + i) * D + h * DH;
#pragma unroll
  for (int c4 = 0; c4 < DH / 4; ++c4)
    *(f32x4*)(op + 4 * c4) = f32x4{acc[2 * c4].x * inv, acc[2 * c4].y * inv, acc[2 * c4 + 1].x * inv,
                                   acc[2 * c4 + 1].y * inv};
  if (DROP) {
    uint32_t* mb = a.mask + r * a.KW;
    mb[0] = w0;
    if (K > 32) mb[1] = w1;
  }
  a.mrow[r] = m * 0.69314718055994531f;
  a.lrow[r] = l;
}

// KC > 0: K <= KC with compile-time LDS strides (dS rows of KC + 1, two keep-bit words per row), so the
// row batches' LDS addresses are immediate offsets of one base; KC = 0: strides from K.
template <int DH, bool BIAS, bool DROP, int KC>
__global__ __launch_bounds__(256) void attn_bwd_kernel(AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int K = a.K, D = a.D, G = a.G, KW = a.KW;
  const int KP = KC ? KC + 1 : K + 1;      // odd row stride
  const int MKW = KC ? (KC + 31) / 32 : KW;   // keep-bit words per row in LDS
  const int b = blockIdx.x, hg = blockIdx.y;
  const int nrel = 2 * a.tk + 1;
  float* sq = sm;                          // [G][K][DH] scaled q
  float* sk = sq + G * K * DH;
  float* sv = sk + G * K * DH;
  float* sdo = sv + G * K * DH;
  f32x4* sst = (f32x4*)(sdo + G * K * DH); // [G][K] {row max, 1 / row sum, do_i . o_i, 0}: one b128 read
  float* srel = (float*)(sst + G * K);     // [nrel]
  uint32_t* smask = (uint32_t*)(srel + nrel);   // [G][K][MKW]
  float* dS = (float*)(smask + G * K * MKW);    // [G][K][KP]
  const float* base = a.qkv + (long)b * K * 3 * D;
  for (int e = threadIdx.x; e < G * K * DH; e += blockDim.x) {
    const int g = e / (K * DH), r = e % (K * DH), j = r / DH, c = r % DH;
    const int col = (hg * G + g) * DH + c;
    sq[e] = base[(long)j * 3 * D + col] * a.scale;
    sk[e] = base[(long)j * 3 * D + D + col];
    sv[e] = base[(long)j * 3 * D + 2 * D + col];
    sdo[e] = a.dO[((long)b * K + j) * D + col];
  }
  const long r0 = ((long)b * a.H + hg * G) * K;     // first (head, row) of the group
  if (DROP)
    for (int e = threadIdx.x; e < G * K * MKW; e += blockDim.x) {
      const int rw = e / MKW, wd = e - rw * MKW;
      smask[e] = wd < KW ? a.mask[(r0 + rw) * KW + wd] : 0u;
    }
  if (BIAS)
    for (int e = threadIdx.x; e < nrel; e += blockDim.x) srel[e] = a.relmean[e];
  const int t = threadIdx.x;
  const bool act = t < G * K;
  const int g = act ? t / K : 0, i = act ? t % K : 0, h = hg * G + g;
  if (act) {
    float di = 0.f;
#pragma unroll
    for (int c = 0; c < DH; ++c)
      di = fmaf(a.dO[((long)b * K + i) * D + h * DH + c], a.o[((long)b * K + i) * D + h * DH + c], di);
    sst[t] = f32x4{a.mrow[r0 + t], 1.0f / a.lrow[r0 + t], di, 0.f};
  }
  __syncthreads();
  const float* qg = sq + g * K * DH;
  const float* kg = sk + g * K * DH;
  const float* vg = sv + g * K * DH;
  const float* dog = sdo + g * K * DH;
  const f32x4* stg = sst + g * K;
  const uint32_t* mk = smask + g * K * MKW;
  float* dSg = dS + g * K * KP;
  // ---- column pass (thread = key column j): p_ij, dS_ij -> LDS; dk_j = sum_i dS_ij qs_i, dv_j = sum_i p~_ij do_i
  // Rows are taken NB at a time: every LDS operand of the NB rows is loaded before any dS store, so the
  // loads of a batch issue back to back (one latency per batch, not per row).
  if (act) {
    constexpr int NB = 4;
    const int j = i;
    float kj[DH], vj[DH], dk[DH], dv[DH];
#pragma unroll
    for (int c = 0; c < DH; ++c) {
      kj[c] = kg[j * DH + c];
      vj[c] = vg[j * DH + c];
      dk[c] = 0.f;
      dv[c] = 0.f;
    }
    const float* rb = srel + a.tk + j;   // rb[-ii] = relmean[j - ii + tk]
    const int jw = j >> 5, jb = j & 31;
    const float dscale = a.drop.scale;
    auto row = [&](int ii, const float* qi, const float* doi, f32x4 st, float rel, uint32_t mw, float& ds_out) {
      const float s = rel + dotv<DH>(kj, qi);
      const float p = fexp(s - st[0]) * st[1];
      float dp = dotv<DH>(vj, doi);
      float pt = p;
      if (DROP) {            // keep ? x * scale : 0 as one multiply by a selected factor
        const float ks = ((mw >> jb) & 1u) ? dscale : 0.f;
        dp *= ks;
        pt = p * ks;
      }
      const float ds = p * (dp - st[2]);
      ds_out = ds;
#pragma unroll
      for (int c = 0; c < DH; ++c) {
        dk[c] = fmaf(ds, qi[c], dk[c]);
        dv[c] = fmaf(pt, doi[c], dv[c]);
      }
    };
    int ii = 0;
    for (; ii + NB <= K; ii += NB) {
      float q[NB][DH], dov[NB][DH], rel[NB], ds[NB];
      f32x4 st[NB];
      uint32_t mw[NB];
#pragma unroll
      for (int u = 0; u < NB; ++u) {
#pragma unroll
        for (int c = 0; c < DH; ++c) {
          q[u][c] = qg[(ii + u) * DH + c];
          dov[u][c] = dog[(ii + u) * DH + c];
        }
        st[u] = stg[ii + u];
        rel[u] = BIAS ? rb[-(ii + u)] : 0.f;
        mw[u] = DROP ? mk[(ii + u) * MKW + jw] : 0u;
      }
#pragma unroll
      for (int u = 0; u < NB; ++u) row(ii + u, q[u], dov[u], st[u], rel[u], mw[u], ds[u]);
#pragma unroll
      for (int u = 0; u < NB; ++u) dSg[(ii + u) * KP + j] = ds[u];
    }
    for (; ii < K; ++ii) {
      float q[DH], dov[DH], ds;
#pragma unroll
      for (int c = 0; c < DH; ++c) {
        q[c] = qg[ii * DH + c];
        dov[c] = dog[ii * DH + c];
      }
      row(ii, q, dov, stg[ii], BIAS ? rb[-ii] : 0.f, DROP ? mk[ii * MKW + jw] : 0u, ds);
      dSg[ii * KP + j] = ds;
    }
#pragma unroll
    for (int c = 0; c < DH; ++c) {
      a.dqkv[((long)b * K + j) * 3 * D + D + h * DH + c] = dk[c];
      a.dqkv[((long)b * K + j) * 3 * D + 2 * D + h * DH + c] = dv[c];
    }
  }
  __syncthreads();
  // ---- row pass (thread = query row i): dq_i = scale * sum_j dS_ij k_j
  if (act) {
    float dq[DH];
#pragma unroll
    for (int c = 0; c < DH; ++c) dq[c] = 0.f;
    const float* dsr = dSg + i * KP;
#pragma unroll 4
    for (int j = 0; j < K; ++j) {
      const float ds = dsr[j];
#pragma unroll
      for (int c = 0; c < DH; ++c) dq[c] = fmaf(ds, kg[j * DH + c], dq[c]);
    }
#pragma unroll
    for (int c = 0; c < DH; ++c) a.dqkv[((long)b * K + i) * 3 * D + h * DH + c] = dq[c] * a.scale;
  }
  // ---- positional-bias grad: sum of dS along diagonals j - i = o.  Each (diagonal, head, half of the
  // diagonal) is one work item (2G items per diagonal spread over the block instead of one thread
  // walking all G heads), the 2G partials are then added in a fixed order.
  if (BIAS) {
    __syncthreads();                               // row pass done: the tiles before dS are free
    const int per = 2 * G;
    const long prefix = (long)4 * G * K * DH + 4 * G * K + nrel + (long)G * K * MKW;
    float* part = prefix >= (long)nrel * per ? sq : dS + G * K * KP;   // [nrel][2G] (ctr_attn_bwd sizes LDS)
    for (int q = threadIdx.x; q < nrel * per; q += blockDim.x) {
      const int e = q / per, gg = (q % per) >> 1, half = q & 1;
      const int o = e - a.tk;
      float s = 0.f;
      if (o > -K && o < K) {
        const int i0 = o >= 0 ? 0 : -o, i1 = o >= 0 ? K - o : K;
        const int im = (i0 + i1) >> 1;
        const int lo = half ? im : i0, hi = half ? i1 : im;
        const float* Pq = dS + gg * K * KP;
#pragma unroll 4
        for (int ii = lo; ii < hi; ++ii) s += Pq[ii * KP + ii + o];
      }
      part[q] = s;
    }
    __syncthreads();
    for (int e = threadIdx.x; e < nrel; e += blockDim.x) {
      float s = 0.f;
      for (int u = 0; u < per; ++u) s += part[e * per + u];
      a.drel_part[((long)b * gridDim.y + hg) * nrel + e] = s;
    }
  }
}

// K <= 64: one head per WAVE (lane = key column j in the column pass, query row i in the row pass), G heads
// per workgroup, and no K x K dS tile in LDS: the row pass recomputes p_ij / dS_ij (the same arithmetic as
// the column pass, so dS and dq are bit-identical to a stored tile) instead of reading it back.  That cuts
// the LDS per head from ~20 KB to ~6 KB, so six workgroups (24 waves) share a CU instead of two -- the
// kernel is latency-bound on its LDS broadcasts and exp, and occupancy is what hides that.
// Positional-bias grad without a dS tile: at row step ii lane j adds dS_ij to diagonal j - ii, so a
// diagonal's running sum moves one lane right per step -- a DPP wave_shr:1 of one accumulator register.
// Lane K-1 holds a finished diagonal after every step (stored to LDS); the negative diagonals finish in
// lanes 0..K-2 after the last step.  Each head sums its diagonals in row order, heads add in fixed order.
template <int DH, bool BIAS, bool DROP>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(6))) void attn_bwd_wave_kernel(AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int K = a.K, D = a.D, G = a.G, KW = a.KW;
  const int b = blockIdx.x, hg = blockIdx.y;
  const int nrel = 2 * a.tk + 1, ND = 2 * K - 1;
  float* sq = sm;                          // [G][K][DH] scaled q
  float* sk = sq + G * K * DH;
  float* sv = sk + G * K * DH;
  float* sdo = sv + G * K * DH;
  f32x4* sst = (f32x4*)(sdo + G * K * DH); // [G][K] {row max, 1 / row sum, do_i . o_i, 0}
  float* srel = (float*)(sst + G * K);     // [nrel]
  uint32_t* smask = (uint32_t*)(srel + nrel);   // [G][K][KW]
  float* sdiag = (float*)(smask + G * K * KW);  // [G][2K-1] diagonal sums of dS, o + K - 1
  const float* base = a.qkv + (long)b * K * 3 * D;
  for (int e = threadIdx.x; e < G * K * DH; e += blockDim.x) {
    const int g = e / (K * DH), r = e % (K * DH), j = r / DH, c = r % DH;
    const int col = (hg * G + g) * DH + c;
    sq[e] = base[(long)j * 3 * D + col] * a.scale;
    sk[e] = base[(long)j * 3 * D + D + col];
    sv[e] = base[(long)j * 3 * D + 2 * D + col];
    sdo[e] = a.dO[((long)b * K + j) * D + col];
  }
  const long r0 = ((long)b * a.H + hg * G) * K;     // first (head, row) of the group
  if (DROP)
    for (int e = threadIdx.x; e < G * K * KW; e += blockDim.x) smask[e] = a.mask[r0 * KW + e];
  if (BIAS)
    for (int e = threadIdx.x; e < nrel; e += blockDim.x) srel[e] = a.relmean[e];
  const int g = threadIdx.x >> 6, lane = threadIdx.x & 63, h = hg * G + g;
  const bool act = lane < K;
  const int li = act ? lane : K - 1;                // inactive lanes mirror the last column / row
  if (act) {
    float di = 0.f;
#pragma unroll
    for (int c = 0; c < DH; ++c)
      di = fmaf(a.dO[((long)b * K + lane) * D + h * DH + c], a.o[((long)b * K + lane) * D + h * DH + c], di);
    sst[g * K + lane] = f32x4{a.mrow[r0 + g * K + lane], 1.0f / a.lrow[r0 + g * K + lane], di, 0.f};
  }
  __syncthreads();
  const float* qg = sq + g * K * DH;
  const float* kg = sk + g * K * DH;
  const float* vg = sv + g * K * DH;
  const float* dog = sdo + g * K * DH;
  const f32x4* stg = sst + g * K;
  const uint32_t* mk = smask + g * K * KW;
  float* dg = sdiag + g * ND;
  const float dscale = a.drop.scale;
  const float live = act ? 1.0f : 0.0f;
  // ---- column pass (lane = key column j): dk_j = sum_i dS_ij qs_i, dv_j = sum_i p~_ij do_i
  {
    constexpr int NB = DH <= 4 ? 2 : 1;   // row batch (all LDS operands loaded first); fits 80 VGPRs
    const int j = li;
    float kj[DH], vj[DH], dk[DH], dv[DH];
#pragma unroll
    for (int c = 0; c < DH; ++c) {
      kj[c] = kg[j * DH + c];
      vj[c] = vg[j * DH + c];
      dk[c] = 0.f;
      dv[c] = 0.f;
    }
    const float* rb = srel + a.tk + j;
    const int jw = j >> 5, jb = j & 31;
    float diag = 0.f;
    for (int ii = 0; ii < K; ii += NB) {
      float q[NB][DH], dov[NB][DH], rel[NB];
      f32x4 st[NB];
      uint32_t mw[NB];
#pragma unroll
      for (int u = 0; u < NB; ++u) {
        const int r = ii + u < K ? ii + u : K - 1;
#pragma unroll
        for (int c = 0; c < DH; ++c) {
          q[u][c] = qg[r * DH + c];
          dov[u][c] = dog[r * DH + c];
        }
        st[u] = stg[r];
        rel[u] = BIAS ? rb[-r] : 0.f;
        mw[u] = DROP ? mk[r * KW + jw] : 0u;
      }
#pragma unroll
      for (int u = 0; u < NB; ++u) {
        if (ii + u < K) {                               // wave-uniform
          const float sc = rel[u] + dotv<DH>(kj, q[u]);
          const float p = fexp(sc - st[u][0]) * st[u][1];
          float dp = dotv<DH>(vj, dov[u]);
          float pt = p;
          if (DROP) {
            const float ks = ((mw[u] >> jb) & 1u) ? dscale : 0.f;
            dp *= ks;
            pt = p * ks;
          }
          const float ds = p * (dp - st[u][2]) * live;
          pt *= live;
#pragma unroll
          for (int c = 0; c < DH; ++c) {
            dk[c] = fmaf(ds, q[u][c], dk[c]);
            dv[c] = fmaf(pt, dov[u][c], dv[c]);
          }
          if (BIAS) {
            if (ii + u > 0) diag = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(
                0, __builtin_bit_cast(int, diag), 0x138 /* wave_shr:1 */, 0xF, 0xF, false));
            diag += ds;
            if (lane == K - 1) dg[2 * K - 2 - (ii + u)] = diag;   // diagonal K-1-(ii+u) is complete
          }
        }
      }
    }
    if (BIAS && lane < K - 1) dg[lane] = diag;         // diagonals lane - (K-1) < 0
    if (act) {
#pragma unroll
      for (int c = 0; c < DH; ++c) {
        a.dqkv[((long)b * K + j) * 3 * D + D + h * DH + c] = dk[c];
        a.dqkv[((long)b * K + j) * 3 * D + 2 * D + h * DH + c] = dv[c];
      }
    }
  }
  // ---- row pass (lane = query row i): dq_i = scale * sum_j dS_ij k_j, dS recomputed as above
  {
    const int i = li;
    float qi[DH], doi[DH], dq[DH];
#pragma unroll
    for (int c = 0; c < DH; ++c) {
      qi[c] = qg[i * DH + c];
      doi[c] = dog[i * DH + c];
      dq[c] = 0.f;
    }
    const f32x4 st = stg[i];
    const float* rb = srel + a.tk - i;                  // rb[j] = relmean[j - i + tk]
    for (int j0 = 0; j0 < K; j0 += 32) {
      const uint32_t mw = DROP ? mk[i * KW + (j0 >> 5)] : 0u;
      const int j1 = j0 + 32 < K ? j0 + 32 : K;
#pragma unroll 4
      for (int j = j0; j < j1; ++j) {
        float kj[DH], vj[DH];
#pragma unroll
        for (int c = 0; c < DH; ++c) {
          kj[c] = kg[j * DH + c];
          vj[c] = vg[j * DH + c];
        }
        const float sc = (BIAS ? rb[j] : 0.f) + dotv<DH>(kj, qi);
        const float p = fexp(sc - st[0]) * st[1];
        float dp = dotv<DH>(vj, doi);
        if (DROP) dp *= ((mw >> (j - j0)) & 1u) ? dscale : 0.f;
        const float ds = p * (dp - st[2]);
#pragma unroll
        for (int c = 0; c < DH; ++c) dq[c] = fmaf(ds, kj[c], dq[c]);
      }
    }
    if (act) {
#pragma unroll
      for (int c = 0; c < DH; ++c) a.dqkv[((long)b * K + i) * 3 * D + h * DH + c] = dq[c] * a.scale;
    }
  }
  if (BIAS) {
    __syncthreads();
    for (int e = threadIdx.x; e < nrel; e += blockDim.x) {
      const int o = e - a.tk;
      float s = 0.f;
      if (o > -K && o < K)
        for (int gg = 0; gg < G; ++gg) s += sdiag[gg * ND + o + K - 1];
      a.drel_part[((long)b * gridDim.y + hg) * nrel + e] = s;
    }
  }
}

// 64 < K <= 256: one head per workgroup of NW = ceil(K/64) waves, every wave a 64-column segment of the
// head in the column pass (lane = key column j = 64w + lane) and a 64-row segment in the row pass (lane =
// query row i), dS recomputed in the row pass as in attn_bwd_wave_kernel -- no K x K tile in LDS.  The
// stored-tile form (attn_bwd_kernel) needs K (K+1) floats of LDS per head (87 KB at K = 148): one
// 3-wave workgroup per CU, so nothing hides its LDS and exp latencies; this form takes ~29 KB per head.
// Positional-bias grad: the DPP diagonal shift of attn_bwd_wave_kernel per wave; a diagonal leaving a
// wave's last column (lane 63, or the last live lane) is a finished PARTIAL sum over that wave's columns,
// stored to [wave][diagonal]; the waves' partials are added in wave order at the end (deterministic).
template <int DH, bool BIAS, bool DROP>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void attn_bwd_multi_kernel(AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int K = a.K, D = a.D, KW = a.KW;
  const int b = blockIdx.x, h = blockIdx.y;
  const int nrel = 2 * a.tk + 1, ND = 2 * K - 1;
  const int NW = (K + 63) >> 6;
  float* sq = sm;                          // [K][DH] scaled q
  float* sk = sq + K * DH;
  float* sv = sk + K * DH;
  float* sdo = sv + K * DH;
  f32x4* sst = (f32x4*)(sdo + K * DH);     // [K] {row max, 1 / row sum, do_i . o_i, 0}
  float* srel = (float*)(sst + K);         // [nrel]
  uint32_t* smask = (uint32_t*)(srel + nrel);   // [K][KW]
  float* sdiag = (float*)(smask + K * KW); // [NW][2K-1] per-wave partial diagonal sums
  const float* base = a.qkv + (long)b * K * 3 * D;
  for (int e = threadIdx.x; e < K * DH; e += blockDim.x) {
    const int j = e / DH, c = e % DH;
    const int col = h * DH + c;
    sq[e] = base[(long)j * 3 * D + col] * a.scale;
    sk[e] = base[(long)j * 3 * D + D + col];
    sv[e] = base[(long)j * 3 * D + 2 * D + col];
    sdo[e] = a.dO[((long)b * K + j) * D + col];
  }
  const long r0 = ((long)b * a.H + h) * K;     // first row of the head
  if (DROP)
    for (int e = threadIdx.x; e < K * KW; e += blockDim.x) smask[e] = a.mask[r0 * KW + e];
  if (BIAS) {
    for (int e = threadIdx.x; e < nrel; e += blockDim.x) srel[e] = a.relmean[e];
    for (int e = threadIdx.x; e < NW * ND; e += blockDim.x) sdiag[e] = 0.f;
  }
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int t = threadIdx.x;                        // column j (column pass) / row i (row pass)
  const bool act = t < K;
  const int li = act ? t : K - 1;                   // dead lanes mirror the last column / row
  if (act) {
    float di = 0.f;
#pragma unroll
    for (int c = 0; c < DH; ++c)
      di = fmaf(a.dO[((long)b * K + t) * D + h * DH + c], a.o[((long)b * K + t) * D + h * DH + c], di);
    sst[t] = f32x4{a.mrow[r0 + t], 1.0f / a.lrow[r0 + t], di, 0.f};
  }
  __syncthreads();
  const float dscale = a.drop.scale;
  const float live = act ? 1.0f : 0.0f;
  const int last_lane = min(63, K - 1 - 64 * w);    // the wave's last live column
  // ---- column pass (lane = key column j): dk_j = sum_i dS_ij qs_i, dv_j = sum_i p~_ij do_i
  {
    const int j = li;
    float kj[DH], vj[DH], dk[DH], dv[DH];
#pragma unroll
    for (int c = 0; c < DH; ++c) {
      kj[c] = sk[j * DH + c];
      vj[c] = sv[j * DH + c];
      dk[c] = 0.f;
      dv[c] = 0.f;
    }
    const float* rb = srel + a.tk + j;
    const int jw = j >> 5, jb = j & 31;
    float diag = 0.f;
    float* dgw = sdiag + w * ND + (K - 1);          // dgw[o] = partial of diagonal o = j - i over this wave
    for (int ii = 0; ii < K; ++ii) {
      float q[DH], dov[DH];
#pragma unroll
      for (int c = 0; c < DH; ++c) {
        q[c] = sq[ii * DH + c];
        dov[c] = sdo[ii * DH + c];
      }
      const f32x4 st = sst[ii];
      const float rel = BIAS ? rb[-ii] : 0.f;
      const uint32_t mw = DROP ? smask[ii * KW + jw] : 0u;
      const float sc = rel + dotv<DH>(kj, q);
      const float p = fexp(sc - st[0]) * st[1];
      float dp = dotv<DH>(vj, dov);
      float pt = p;
      if (DROP) {
        const float ks = ((mw >> jb) & 1u) ? dscale : 0.f;
        dp *= ks;
        pt = p * ks;
      }
      const float ds = p * (dp - st[2]) * live;
      pt *= live;
#pragma unroll
      for (int c = 0; c < DH; ++c) {
        dk[c] = fmaf(ds, q[c], dk[c]);
        dv[c] = fmaf(pt, dov[c], dv[c]);
      }
      if (BIAS) {
        if (ii > 0) diag = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(
            0, __builtin_bit_cast(int, diag), 0x138 /* wave_shr:1 */, 0xF, 0xF, false));
        diag += ds;
        // the diagonal in the wave's last live column leaves the wave's columns at the next step
        if (lane == last_lane) dgw[64 * w + lane - ii] = diag;
      }
    }
    if (BIAS && lane < last_lane) dgw[64 * w + lane - (K - 1)] = diag;   // diagonals still inside at the end
    if (act) {
#pragma unroll
      for (int c = 0; c < DH; ++c) {
        a.dqkv[((long)b * K + j) * 3 * D + D + h * DH + c] = dk[c];
        a.dqkv[((long)b * K + j) * 3 * D + 2 * D + h * DH + c] = dv[c];
      }
    }
  }
  // ---- row pass (lane = query row i): dq_i = scale * sum_j dS_ij k_j, dS recomputed as above
  {
    const int i = li;
    float qi[DH], doi[DH], dq[DH];
#pragma unroll
    for (int c = 0; c < DH; ++c) {
      qi[c] = sq[i * DH + c];
      doi[c] = sdo[i * DH + c];
      dq[c] = 0.f;
    }
    const f32x4 st = sst[i];
    const float* rb = srel + a.tk - i;                  // rb[j] = relmean[j - i + tk]
    for (int j0 = 0; j0 < K; j0 += 32) {
      const uint32_t mw = DROP ? smask[i * KW + (j0 >> 5)] : 0u;
      const int j1 = j0 + 32 < K ? j0 + 32 : K;
#pragma unroll 4
      for (int j = j0; j < j1; ++j) {
        float kj[DH], vj[DH];
#pragma unroll
        for (int c = 0; c < DH; ++c) {
          kj[c] = sk[j * DH + c];
          vj[c] = sv[j * DH + c];
        }
        const float sc = (BIAS ? rb[j] : 0.f) + dotv<DH>(kj, qi);
        const float p = fexp(sc - st[0]) * st[1];
        float dp = dotv<DH>(vj, doi);
        if (DROP) dp *= ((mw >> (j - j0)) & 1u) ? dscale : 0.f;
        const float ds = p * (dp - st[2]);
#pragma unroll
        for (int c = 0; c < DH; ++c) dq[c] = fmaf(ds, kj[c], dq[c]);
      }
    }
    if (act) {
#pragma unroll
      for (int c = 0; c < DH; ++c) a.dqkv[((long)b * K + i) * 3 * D + h * DH + c] = dq[c] * a.scale;
    }
  }
  if (BIAS) {
    __syncthreads();
    for (int e = threadIdx.x; e < nrel; e += blockDim.x) {
      const int o = e - a.tk;
      float s = 0.f;
      if (o > -K && o < K)
        for (int ww = 0; ww < NW; ++ww) s += sdiag[ww * ND + o + K - 1];
      a.drel_part[((long)b * gridDim.y + h) * nrel + e] = s;
    }
  }
}

static int pick_group(int H, int K, size_t per_head_lds, size_t lds_cap) {
  int best = 1;
  for (int g = 1; g <= H; ++g)
    if (H % g == 0 && g * K <= 256 && g * per_head_lds <= lds_cap) best = g;
  return best;
}

// compile-time-stride variants of the backward (attn_bwd_kernel KC): K <= 60 (the benchmark's K; a dS
// stride of 61 keeps four heads per workgroup within 80 KB), K <= 64
static int bwd_kc(int K) { return K <= 60 ? 60 : K <= 64 ? 64 : 0; }
static int bwd_kp(int K) { return bwd_kc(K) ? bwd_kc(K) + 1 : K + 1; }
static int bwd_mkw(int K) { return bwd_kc(K) ? (bwd_kc(K) + 31) / 32 : (K + 31) / 32; }

static size_t bwd_lds(int G, int K, int dh, int tk) {
  const int nrel = 2 * tk + 1;
  const size_t prefix = (size_t)4 * G * K * dh + 4 * G * K + nrel + (size_t)G * K * bwd_mkw(K);
  const size_t part = (size_t)2 * G * nrel;     // positional-bias partials: in the prefix when they fit
  return (prefix + (size_t)G * K * bwd_kp(K) + (prefix >= part ? 0 : part)) * sizeof(float);
}

static int bwd_group(int H, int K, int dh) {
  return pick_group(H, K, (size_t)(K * bwd_kp(K) + 4 * K * dh + 4 * K + K * bwd_mkw(K)) * 4, 80 * 1024);
}

// the wave-per-head backward (K <= 64, dh <= 8): G = the largest divisor of H up to 4 (one wave per head)
static bool bwd_use_wave(int K, int dh) { return K <= 64 && dh <= 8; }
// the multi-wave recompute backward (64 < K <= 256, dh <= 8): one head per workgroup
static bool bwd_use_multi(int K, int dh) { return K > 64 && K <= 256 && dh <= 8; }

static size_t bwd_multi_lds(int K, int dh, int tk) {
  return ((size_t)4 * K * dh + 4 * K + (2 * tk + 1) + (size_t)K * ((K + 31) / 32) +
          (size_t)((K + 63) / 64) * (2 * K - 1)) * sizeof(float);
}

template <int DH>
static void launch_bwd_multi(const AttnArgs& a, size_t sm, hipStream_t s) {
  const bool bias = a.relmean != nullptr, drop = a.drop.thresh != 0;
  const dim3 grid(a.B, a.H), blk((a.K + 63) / 64 * 64);
  if (bias && drop) attn_bwd_multi_kernel<DH, true, true><<<grid, blk, sm, s>>>(a);
  else if (bias) attn_bwd_multi_kernel<DH, true, false><<<grid, blk, sm, s>>>(a);
  else if (drop) attn_bwd_multi_kernel<DH, false, true><<<grid, blk, sm, s>>>(a);
  else attn_bwd_multi_kernel<DH, false, false><<<grid, blk, sm, s>>>(a);
}

static int bwd_wave_group(int H) {
  int g = 1;
  for (int c = 1; c <= 4; ++c)
    if (H % c == 0) g = c;
  return g;
}

static size_t bwd_wave_lds(int G, int K, int dh, int tk) {
  return ((size_t)4 * G * K * dh + 4 * G * K + (2 * tk + 1) + (size_t)G * K * ((K + 31) / 32) +
          (size_t)G * (2 * K - 1)) * sizeof(float);
}

template <int DH, bool BIAS, bool DROP>
static void launch_bwd_wave3(const AttnArgs& a, size_t sm, hipStream_t s) {
  attn_bwd_wave_kernel<DH, BIAS, DROP><<<dim3(a.B, a.H / a.G), a.G * 64, sm, s>>>(a);
}

template <int DH>
static void launch_bwd_wave(const AttnArgs& a, size_t sm, hipStream_t s) {
  const bool bias = a.relmean != nullptr, drop = a.drop.thresh != 0;
  if (bias && drop) launch_bwd_wave3<DH, true, true>(a, sm, s);
  else if (bias) launch_bwd_wave3<DH, true, false>(a, sm, s);
  else if (drop) launch_bwd_wave3<DH, false, true>(a, sm, s);
  else launch_bwd_wave3<DH, false, false>(a, sm, s);
}

template <int DH, bool BIAS, bool DROP>
static void launch_fwd3(const AttnArgs& a, size_t sm, hipStream_t s) {
  attn_fwd_kernel<DH, BIAS, DROP><<<dim3(a.B, a.H / a.G), (a.G * a.K + 63) / 64 * 64, sm, s>>>(a);
}

// the packed forward: K <= 64 and even, dh in {4, 8}, the output rows 16-byte aligned
static bool fwd_use_pk(int K, int dh, int D) { return K <= 64 && (K & 1) == 0 && (dh == 4 || dh == 8) && D % 4 == 0; }

template <int DH, bool BIAS, bool DROP>
static void launch_fwd_pk3(const AttnArgs& a, hipStream_t s) {
  const size_t sm = ((size_t)2 * a.G * a.K * DH + 2 * (size_t)((2 * a.tk + 3) & ~1)) * sizeof(float);
  attn_fwd_pk_kernel<DH, BIAS, DROP><<<dim3(a.B, a.H / a.G), (a.G * a.K + 63) / 64 * 64, sm, s>>>(a);
}

template <int DH>
static void launch_fwd_pk(const AttnArgs& a, hipStream_t s) {
  const bool bias = a.relmean != nullptr, drop = a.drop.thresh != 0;
  if (bias && drop) launch_fwd_pk3<DH, true, true>(a, s);
  else if (bias) launch_fwd_pk3<DH, true, false>(a, s);
  else if (drop) launch_fwd_pk3<DH, false, true>(a, s);
  else launch_fwd_pk3<DH, false, false>(a, s);
}

template <int DH>
static void launch_fwd(const AttnArgs& a, size_t sm, hipStream_t s) {
  const bool bias = a.relmean != nullptr, drop = a.drop.thresh != 0;
  if (bias && drop) launch_fwd3<DH, true, true>(a, sm, s);
  else if (bias) launch_fwd3<DH, true, false>(a, sm, s);
  else if (drop) launch_fwd3<DH, false, true>(a, sm, s);
  else launch_fwd3<DH, false, false>(a, sm, s);
}

template <int DH, bool BIAS, bool DROP, int KC>
static void launch_bwd4(const AttnArgs& a, size_t sm, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)attn_bwd_kernel<DH, BIAS, DROP, KC>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  attn_bwd_kernel<DH, BIAS, DROP, KC><<<dim3(a.B, a.H / a.G), (a.G * a.K + 63) / 64 * 64, sm, s>>>(a);
}

template <int DH, bool BIAS, bool DROP>
static void launch_bwd3(const AttnArgs& a, size_t sm, hipStream_t s) {
  if (bwd_kc(a.K) == 60) launch_bwd4<DH, BIAS, DROP, 60>(a, sm, s);
  else if (bwd_kc(a.K) == 64) launch_bwd4<DH, BIAS, DROP, 64>(a, sm, s);
  else launch_bwd4<DH, BIAS, DROP, 0>(a, sm, s);
}

template <int DH>
static void launch_bwd(const AttnArgs& a, size_t sm, hipStream_t s) {
  const bool bias = a.relmean != nullptr, drop = a.drop.thresh != 0;
  if (bias && drop) launch_bwd3<DH, true, true>(a, sm, s);
  else if (bias) launch_bwd3<DH, true, false>(a, sm, s);
  else if (drop) launch_bwd3<DH, false, true>(a, sm, s);
  else launch_bwd3<DH, false, false>(a, sm, s);
}

}  // namespace ctr

using namespace ctr;

// test hook: 1 = always the generic (unpacked) forward, so tests can compare the two forms
static int ctr_attn_force_generic = 0;
extern "C" void ctr_attn_set_generic(int on) { ctr_attn_force_generic = on; }

// row layout (this file) or the bf16-MFMA kernels' lane layout (attn_mf.hip: 128 words per head), whichever is larger
extern "C" int ctr_attn_mask_words(int B, int K, int H) {
  // per head: the fp32 kernels' K rows of ceil(K / 32) words, or the bf16-MFMA kernels' lane layout
  // (attn_mf.hip: 64 lanes x NW words, NW = 2 for nt = ceil(K / 16) <= 4, ceil(4 nt^2 / 32) beyond)
  const int row = K * ((K + 31) / 32), nt = (K + 15) / 16;
  const int lanes = 64 * (nt <= 4 ? 2 : (4 * nt * nt + 31) / 32);
  return B * H * std::max(row, lanes);
}

extern "C" int ctr_attn_fwd(const float* qkv, int B, int K, int H, int D, const float* relmean, int tk, float scale,
                            uint32_t drop_key, uint32_t drop_thresh, float drop_scale, uint32_t* mask, float* o,
                            float* mrow, float* lrow, void* stream) {
  if (B == 0) return 0;
  const int dh = D / H;
  CTR_REQUIRE(D % H == 0 && (dh == 2 || dh == 4 || dh == 8 || dh == 16), "head dim must be 2, 4, 8 or 16");
  CTR_REQUIRE(K <= 256, "K > 256");
  CTR_REQUIRE(!relmean || tk >= K - 1, "positional-bias table shorter than K");
  const int G = pick_group(H, K, (size_t)2 * K * dh * 4, 64 * 1024);
  AttnArgs a{};
  a.qkv = qkv; a.B = B; a.K = K; a.H = H; a.D = D; a.G = G;
  a.relmean = relmean; a.tk = tk; a.scale = scale; a.drop = Drop{drop_key, drop_thresh, drop_scale};
  a.mask = mask; a.KW = (K + 31) / 32;
  CTR_REQUIRE(!drop_thresh || mask, "attention forward with dropout needs a keep-bit buffer");
  a.o = o; a.mrow = mrow; a.lrow = lrow;
  const size_t sm = ((size_t)2 * G * K * dh + 2 * tk + 1) * sizeof(float);
  hipStream_t s = (hipStream_t)stream;
  if (fwd_use_pk(K, dh, D) && !ctr_attn_force_generic) {
    if (dh == 4) launch_fwd_pk<4>(a, s);
    else launch_fwd_pk<8>(a, s);
    return check_launch("attn_fwd");
  }
  switch (dh) {
    case 2: launch_fwd<2>(a, sm, s); break;
    case 4: launch_fwd<4>(a, sm, s); break;
    case 8: launch_fwd<8>(a, sm, s); break;
    default: launch_fwd<16>(a, sm, s); break;
  }
  return check_launch("attn_fwd");
}

extern "C" int ctr_attn_bwd_nparts(int H, int K, int D) {
  const int dh = D / H;
  return H / (bwd_use_wave(K, dh) ? bwd_wave_group(H) : bwd_use_multi(K, dh) ? 1 : bwd_group(H, K, dh));
}

extern "C" int ctr_attn_bwd(const float* qkv, const float* o, const float* dO, int B, int K, int H, int D,
                            const float* relmean, int tk, float scale, uint32_t drop_key, uint32_t drop_thresh,
                            float drop_scale, const uint32_t* mask, const float* mrow, const float* lrow, float* dqkv,
                            float* drel_part, void* stream) {
  if (B == 0) return 0;
  const int dh = D / H;
  CTR_REQUIRE(D % H == 0 && (dh == 2 || dh == 4 || dh == 8 || dh == 16), "head dim must be 2, 4, 8 or 16");
  CTR_REQUIRE(K <= 256, "K > 256");
  CTR_REQUIRE(!drop_thresh || mask, "attention backward with dropout needs the forward's keep bits");
  const bool wave = bwd_use_wave(K, dh), multi = !wave && bwd_use_multi(K, dh);
  const int G = wave ? bwd_wave_group(H) : multi ? 1 : bwd_group(H, K, dh);
  AttnArgs a{};
  a.qkv = qkv; a.B = B; a.K = K; a.H = H; a.D = D; a.G = G;
  a.relmean = relmean; a.tk = tk; a.scale = scale; a.drop = Drop{drop_key, drop_thresh, drop_scale};
  a.mask = const_cast<uint32_t*>(mask); a.KW = (K + 31) / 32;
  a.o = const_cast<float*>(o); a.mrow = const_cast<float*>(mrow); a.lrow = const_cast<float*>(lrow);
  a.dO = dO; a.dqkv = dqkv; a.drel_part = drel_part;
  const size_t sm = wave ? bwd_wave_lds(G, K, dh, tk) : multi ? bwd_multi_lds(K, dh, tk) : bwd_lds(G, K, dh, tk);
  CTR_REQUIRE(sm <= 160 * 1024, "attention backward tile exceeds LDS");
  hipStream_t s = (hipStream_t)stream;
  if (multi) {
    CTR_REQUIRE(sm <= 64 * 1024, "attention backward (multi-wave form) tile exceeds 64 KB");
    switch (dh) {
      case 2: launch_bwd_multi<2>(a, sm, s); break;
      case 4: launch_bwd_multi<4>(a, sm, s); break;
      default: launch_bwd_multi<8>(a, sm, s); break;
    }
    return check_launch("attn_bwd");
  }
  if (wave) {
    CTR_REQUIRE(sm <= 64 * 1024, "attention backward (wave form) tile exceeds 64 KB");
    switch (dh) {
      case 2: launch_bwd_wave<2>(a, sm, s); break;
      case 4: launch_bwd_wave<4>(a, sm, s); break;
      default: launch_bwd_wave<8>(a, sm, s); break;
    }
    return check_launch("attn_bwd");
  }
  switch (dh) {
    case 2: launch_bwd<2>(a, sm, s); break;
    case 4: launch_bwd<4>(a, sm, s); break;
    case 8: launch_bwd<8>(a, sm, s); break;
    default: launch_bwd<16>(a, sm, s); break;
  }
  return check_launch("attn_bwd");
}

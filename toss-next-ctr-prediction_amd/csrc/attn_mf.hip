// Attention core of DAREEncoderLayer on bf16 MFMA (amp: bf16), K <= 64, head dim dh in {4, 8}.
// Same algorithm as attn.hip (src/models/dare.py:53-62, torch's MHA explicit path): s_ij = mean_h rel[j-i+tk]
// + (q_i sqrt(1/dh)) . k_j ; p = softmax_j(s) ; p~ = dropout(p) ; o_i = sum_j p~_ij v_j ; and its backward.
// Under torch.autocast(bfloat16) the reference runs both attention products (baddbmm(q, k^T) and bmm(p~, v))
// and their autograd products on bf16 operands with fp32 accumulation; here every product is a
// v_mfma_f32_16x16x16_bf16 over bf16-rounded q*scale, k, v, dO, p~ and dS, while the softmax, the dropout
// and dS = p (dp - do.o) stay fp32 (the scores are not rounded to bf16 -- the reference rounds them; ours is
// the more precise side of that difference).
//
// One wave per head, the whole K x K head in registers as 16 x 16 tiles (nt = ceil(K/16) tiles a side, K <= 160:
// staged operands padded to KT = 64 rows for nt <= 4, 16 nt rows beyond; the forward holds one query tile's
// row of score tiles at a time, the backward one key tile's column).  Every elementwise step works on the TRANSPOSED score tile S^T = K Q^T, whose MFMA
// accumulator layout puts key j = 16 tj + 4g + r in register r of lane (g, c) and query i = 16 ti + c in the
// lane: a softmax row (fixed i) is the lane's registers plus the four lane groups (two permlane swaps), and
// the tile's registers ARE the B operand of the products that reduce over keys (o^T = v^T p~^T,
// dq^T = k^T dS^T) -- no data movement.  The products that reduce over queries (dk^T = q^T dS,
// dv^T = do^T p~) take dS / p~ through a per-wave 16 x 64 LDS image read back with ds_read_b64_tr_b16.
// Per head: 32 MFMAs forward, 80 backward; per score element ~12 VALU operations (exp, dropout, dS)
// instead of the ~50 of the VALU kernels (which recompute p in a second pass for dq).
//
// Keep bits of p~ (the backward reads them instead of re-hashing) are stored in the lane layout: per head
// NW words x 64 lanes; element (i = 16 ti + c, j = 16 tj + 4g + r) is bit pos % 32 of word pos / 32 of lane (g, c),
// pos = 16 ti + 4 tj + r for nt <= 4 (NW = 2: bit 16 (ti & 1) + 4 tj + r of word ti >> 1) and key-tile major
// pos = 4 nt tj + 4 ti + r beyond (NW = ceil(4 nt^2 / 32)), where the backward walks key tiles in a loop.  The keep decision is the same counter hash as every other dropout site (common.h).
// mrow holds the row max in log2 units (the forward's and backward's exp2 argument), lrow the row sum.
#include <type_traits>

#include "common.h"
#include "ctr_hip.h"

namespace ctr {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));

constexpr int NT_MAX = 10;                  // K <= 160
constexpr float L2E = 1.4426950408889634f;
// per tile count: staged rows, keep-bit stride per query tile, keep words per lane
template <int NT>
struct Kt {
  static constexpr int KT = NT <= 4 ? 64 : 16 * NT;
  static constexpr int NW = NT <= 4 ? 2 : (4 * NT * NT + 31) / 32;
};

struct AttnBfArgs {
  const float* qkv;      // (B*K, 3D)
  int B, K, H, D, G, nt, tk;
  const float* relmean;  // (2tk+1) or null
  float scale;           // sqrt(1/dh) (the reference's python float in fp32)
  Drop drop;
  uint32_t* mask;        // (B*H, 2, 64) keep bits, lane layout
  float* o;              // (B*K, D)
  float* mrow;           // (B*H*K) row max, log2 units
  float* lrow;           // (B*H*K) row sum of exp2(t - max)
  const float* dO;       // (B*K, D)
  float* dqkv;           // (B*K, 3D)
  float* drel_part;      // (B * H/G, 2tk+1)
  int ngrp;              // head groups per sample (H / G)
  const float* dh1;      // backward with the out-projection fused (nt <= 4, D = 32): dO = dh1 W_out computed in
  const float* w_out;    // the kernel from the (B*K, 32) rows dh1 and W_out (32, 32); dO is then unused
  // amp: the bf16 forms of the saved projections (null: the fp32 ones above).  qkv16 (B*K, 3D) holds the staged
  // operands themselves -- bf16(q * scale), bf16(k), bf16(v), the values both attention products take -- so the
  // backward stages them as they are; dqkv16 (B*K, 3D) receives bf16(dq), bf16(dk), bf16(dv) (RNE), the dtype of
  // the reference's autocast in-projection output grad
  const __bf16* qkv16;
  __bf16* dqkv16;
  // the layer backward (ctr_attn_bwd_bf_layer16: one workgroup holds every head of a sample): the in-projection's
  // input grad dx = dqkv W_in + dh1 from the workgroup's own dqkv16 rows, W_in = in_proj_weight (3D, D)
  const float* w_in;
  float* dx;
  int dx_lds;            // byte offset of the workgroup's LDS dqkv copy
};

// workgroup -> (sample, head group), 1-D grid: with ngrp > 1 head groups a sample's workgroups are 8 apart in
// dispatch order -- on the same XCD (workgroups are dealt round-robin to the 8 XCDs) and close in time -- so the
// second one finds the sample's qkv / o / dO lines in that XCD's L2.  (As a (B, ngrp) grid the head groups of a
// sample ran B workgroups apart on different XCDs and each fetched whole 128-byte lines for its half rows.)
__device__ __forceinline__ int wg_sample(const AttnBfArgs& a) {
  if (a.ngrp == 1) return blockIdx.x;
  const int span = 8 * a.ngrp, q = blockIdx.x / span;
  return 8 * q + (blockIdx.x - q * span) % 8;
}
__device__ __forceinline__ int wg_group(const AttnBfArgs& a) { return a.ngrp == 1 ? 0 : (blockIdx.x % (8 * a.ngrp)) / 8; }
__host__ __forceinline__ int wg_grid(const AttnBfArgs& a) { return a.ngrp == 1 ? a.B : (a.B + 7) / 8 * 8 * a.ngrp; }

__device__ __forceinline__ f32x4 mma(bf16x4 a, bf16x4 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(__builtin_bit_cast(s16x4, a), __builtin_bit_cast(s16x4, b), c,
                                                   0, 0, 0);
}

// 4 rows x 16 columns of 16-bit elements, transposed (ds_read_b64_tr_b16): lane 4q + p of each 16-lane group
// addresses row q, columns 4p .. 4p+3; lane i of the group receives column i, row q in element q
__device__ __forceinline__ bf16x4 tr4(const __bf16* p) {
  return __builtin_bit_cast(bf16x4,
                            __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)p));
}
__device__ __forceinline__ bf16x4 ld4(const __bf16* p) { return *(const bf16x4*)p; }

__device__ __forceinline__ bf16x4 to_bf4(f32x4 v) { return __builtin_convertvector(v, bf16x4); }
__device__ __forceinline__ f32x4 to_f4(bf16x4 v) { return __builtin_convertvector(v, f32x4); }
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
// all ones where x's sign bit is set (v_ashrrev_i32 in asm: as C the compiler turns it back into a compare +
// select, which keeps the lane masks in SGPRs)
__device__ __forceinline__ uint32_t sign_mask(uint32_t x) {
  uint32_t m;
  asm("v_ashrrev_i32 %0, 31, %1" : "=v"(m) : "v"(x));
  return m;
}
// all ones where bit B of x is set, one v_bfe_i32 (as C, sbfe & constant became and + compare + select: three
// VALU per keep bit instead of one)
__device__ __forceinline__ uint32_t bit_mask(uint32_t x, int b) {
  uint32_t m;
  asm("v_bfe_i32 %0, %1, %2, 1" : "=v"(m) : "v"(x), "i"(b));
  return m;
}
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
// RNE bf16 pairs (v_cvt_pk_bf16_f32 each), as two dwords: one conversion for both the MFMA operand and the
// LDS image (through to_bf4 the compiler converted twice, differently packed)
__device__ __forceinline__ u32x2 pk_bf4(f32x4 v) {
  const bf16x2 lo = __builtin_convertvector(f32x2{v[0], v[1]}, bf16x2), hi = __builtin_convertvector(f32x2{v[2], v[3]}, bf16x2);
  return u32x2{__builtin_bit_cast(uint32_t, lo), __builtin_bit_cast(uint32_t, hi)};
}

// one 4-column piece of a dq / dk / dv row at element offset off of the (B*K, 3D) gradient: fp32, or bf16 (RNE)
__device__ __forceinline__ void store_dqkv(const AttnBfArgs& a, long off, f32x4 v) {
  if (a.dqkv16) *(u32x2*)(a.dqkv16 + off) = pk_bf4(v);
  else *(f32x4*)(a.dqkv + off) = v;
}

// The forward's P V product at K > 64 on a two-term bf16 split of p: hi = bf16(p) (the operand autocast's bf16 bmm
// takes) and lo = bf16(p - hi) (the difference is exact in fp32), both against the same bf16 v, so o carries p to ~16
// bits (K <= 64: bf16(p) alone, attn_fwd_mf_kernel).  The
// backward's softmax statistic D_i = bf16(dO_i) . o_i is then the row sum of p_ij dP_ij (dP = bf16(dO) bf16(v)^T, the
// MFMA product) to within that: the two sides of dS = p (dP - D) agree, as in the reference's fp32 softmax backward
// (torch: p * (dP - sum(p * dP))).  With o from bf16(p) alone, D differed from sum p dP by the rounding of p (and,
// with fp32 dO in D, of dO), and rows whose value vectors are all equal (a history of pads only: exact dS = 0) got a
// dS of that rounding's size -- amplified by 1 / rms of the zero rows at the first layer's norm (cfg4 at B = 1024:
// 11 % on the layer-0 MHA bias grads against the reference's own 0.8 %).
__device__ __forceinline__ bf16x4 lo_bf4(const float (&pe)[4], bf16x4 hi) {
  f32x4 d;
#pragma unroll
  for (int r = 0; r < 4; ++r) d[r] = pe[r] - (float)hi[r];
  return __builtin_bit_cast(bf16x4, pk_bf4(d));
}

// four fp32 values rounded to bf16 (RNE) and back
__device__ __forceinline__ f32x4 bfr4(f32x4 v) {
  const bf16x4 b = __builtin_bit_cast(bf16x4, pk_bf4(v));
  return f32x4{(float)b[0], (float)b[1], (float)b[2], (float)b[3]};
}

// all-reduce over the four 16-lane groups (lanes c, c+16, c+32, c+48) by two permlane swaps of two copies of
// the value: v_permlane16_swap leaves rows (r0 r0 r2 r2) in one copy and (r1 r1 r3 r3) in the other,
// v_permlane32_swap (lo lo) / (hi hi).  In asm: through __builtin_amdgcn_permlane16/32_swap the compiler
// (ROCm 7.2) stored the FIRST result for both (measured on gfx950); the s_nop covers the VALU-write ->
// permlane-read hazard the compiler does not see inside asm.  Same bits in all four lanes (op commutative).
__device__ __forceinline__ void swap16(float& x, float& y) {
  asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(x), "+v"(y));
}
__device__ __forceinline__ void swap32(float& x, float& y) {
  asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(x), "+v"(y));
}
template <class Op>
__device__ __forceinline__ float grp_reduce(float v, Op op) {
  float x = v, y = v;
  swap16(x, y);
  v = op(x, y);
  x = v;
  y = v;
  swap32(x, y);
  return op(x, y);
}
__device__ __forceinline__ float grp_max(float v) {
  return grp_reduce(v, [](float p, float q) { return fmaxf(p, q); });
}
__device__ __forceinline__ float grp_sum(float v) {
  return grp_reduce(v, [](float p, float q) { return p + q; });
}

// Workgroup barrier ordering LDS only.  __syncthreads() also waits for every outstanding global load and store
// (its release fence is for all address spaces): the prologue's early loads and the dqkv stores of the backward
// would be waited for at each barrier instead of draining behind the following work.
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// Workgroup staging: q * scale, k, v (and dO) of the group's G heads as bf16 [KT][RS] images; rows >= K are zero.
// The mask chunk's first slot carries the padded-key mask through the score product (k: 1 on padded keys j >= K,
// q: -3e38), so S^T = K Q^T carries -3e38 (-> -inf after the log2 scale) on every padded key and an exact +-0
// elsewhere: no per-element masking.  Compact rows: the four heads' dims back to back, then ONE mask chunk (slot 4 dh) and one zero chunk (slot
// 4 dh + 4) shared by the heads of the row; a head's operand read of lane group g takes dims 4g .. 4g+3 while
// 4g < dh, the row's mask chunk at 4g == dh, the zero chunk beyond.  Column (transposed) reads take 16 slots from
// the head's first dim: the slots past its dims land in output rows d >= dh of the product, which are never
// stored.  (A mask chunk per head took 52 instead of 40 slots per row at dh = 8.)
// HG: the heads a row holds (4; 8 for the layer backward at dh = 4, which stages all of D = 32 in one workgroup)
template <int DH, int NT, int HG = 4>
struct Stg {
  static constexpr int KT = Kt<NT>::KT;
  static constexpr int HS = DH;                     // slots per head
  static constexpr int RS = HG * DH + 8;            // row stride (bf16 elements), <= HG heads
  static constexpr int IM = KT * RS;                // elements per staged operand
  static constexpr int PAD = 16;                    // transposed reads past the last head of the last row
  static constexpr int MOFF = HG * DH;              // the row's mask chunk
  static constexpr int ZOFF = HG * DH + 4;          // the row's zero chunk
};
constexpr float NEG_BIG = -3.0e38f;

template <int DH, int NT, bool WITH_DO, int HG = 4>
__device__ __forceinline__ void stage(const AttnBfArgs& a, int b, int hg, __bf16* sq, __bf16* sk, __bf16* sv, __bf16* sdo) {
  using S = Stg<DH, NT, HG>;
  constexpr int KT = S::KT;
  const int K = a.K, D = a.D, G = a.G;
  const float* base = a.qkv + (long)b * K * 3 * D + hg * G * DH;
  const float* dob = WITH_DO ? a.dO + (long)b * K * D + hg * G * DH : nullptr;
  constexpr int NCD = DH / 4, NCR = HG * NCD + 2;  // chunks per row: HG heads' dims, mask, zero
  for (int e = threadIdx.x; e < KT * NCR; e += blockDim.x) {
    const int j = e / NCR, ch = e - j * NCR;
    f32x4 q = {0.f, 0.f, 0.f, 0.f}, k = q, v = q, d = q;
    int o;
    if (ch < HG * NCD) {
      const int u = ch / NCD, dc = ch - u * NCD;
      o = j * S::RS + u * DH + 4 * dc;
      if (u < G && j < K) {
        const long e0 = (long)j * 3 * D + u * DH + 4 * dc;
        if (a.qkv16) {      // the forward's staged values (q already scaled): converted back exactly
          const __bf16* r = a.qkv16 + (long)b * K * 3 * D + hg * G * DH + e0;
          q = to_f4(*(const bf16x4*)r);
          k = to_f4(*(const bf16x4*)(r + D));
          v = to_f4(*(const bf16x4*)(r + 2 * D));
        } else {
          const float* r = base + e0;
          q = *(const f32x4*)r * a.scale;
          k = *(const f32x4*)(r + D);
          v = *(const f32x4*)(r + 2 * D);
        }
        if (WITH_DO) d = *(const f32x4*)(dob + (long)j * D + u * DH + 4 * dc);
      }
    } else if (ch == HG * NCD) {                  // the row's mask chunk
      o = j * S::RS + S::MOFF;
      q[0] = NEG_BIG;
      k[0] = j >= K ? 1.f : 0.f;
    } else {                                      // the row's zero chunk
      o = j * S::RS + S::ZOFF;
    }
    *(bf16x4*)(sq + o) = to_bf4(q);
    *(bf16x4*)(sk + o) = to_bf4(k);
    *(bf16x4*)(sv + o) = to_bf4(v);
    if (WITH_DO) *(bf16x4*)(sdo + o) = to_bf4(d);
  }
}

// positional bias table in LDS, log2 units, padded by RPAD zeros on both sides: the score element
// (i = 16 ti + c, j = 16 tj + 4g + r) takes rel[j - i + tk] = srel[RPAD + 16 (tj - ti) + 4g + r - c + tk]; the
// index stays inside the padded table for every padded row / key (whose values are discarded), so each
// tile's four values are loads at one per-lane base + immediate offsets, no clamping
// (RPAD = the staged rows KT: 16 (nt - 1) + 15 < KT)
template <int NT>
__device__ __forceinline__ void stage_rel(const AttnBfArgs& a, float* srel) {
  constexpr int RPAD = Kt<NT>::KT;
  const int nrel = 2 * a.tk + 1;
  for (int e = threadIdx.x; e < nrel + 2 * RPAD; e += blockDim.x) {
    const int x = e - RPAD;
    srel[e] = (x >= 0 && x < nrel) ? a.relmean[x] * L2E : 0.f;
  }
}
template <int NT>
__host__ __device__ __forceinline__ int rel_floats(int tk) { return (2 * tk + 1 + 2 * Kt<NT>::KT + 3) & ~3; }   // 16-B multiple

// dS / p~ image of one key tile: 64 query rows x 16 keys, bf16, row stride 16; the 4-key chunk ch of row rw
// stored at chunk ch ^ ((rw >> 2) & 3): the ds_write_b64 of a score tile (16 lanes: rows 16 ti + 0..15, one
// chunk) and the ds_read_b64_tr_b16 (32 lanes: rows 16 ti + 4g + q, chunks p) are both bank-conflict free
__device__ __forceinline__ int swz(int rw, int ch) { return rw * 16 + 4 * (ch ^ ((rw >> 2) & 3)); }
template <int NT>
__host__ __device__ constexpr int img_elems() { return Kt<NT>::KT * 16; }   // bf16 elements per image

// operand reads: row access (lane (g, c) <- slots 4g .. 4g+3 of row `row`; zeros past the head's slots) and
// transposed column access (lane (g, c) <- column c of rows row0 + 4g .. row0 + 4g + 3)
// (the row read is unconditional: lanes past the head's slots read the zero chunk at ZOFF of the image)
template <int DH, int NT, int HG = 4>
__device__ __forceinline__ bf16x4 op_row(const __bf16* img, int row, int hs, int g) {
  using S = Stg<DH, NT, HG>;
  return ld4(img + row * S::RS + (4 * g < DH ? hs + 4 * g : 4 * g == DH ? S::MOFF : S::ZOFF));
}
template <int DH, int NT, int HG = 4>
__device__ __forceinline__ bf16x4 op_col(const __bf16* img, int row0, int hs, int g, int c) {
  return tr4(img + (row0 + 4 * g + (c >> 2)) * Stg<DH, NT, HG>::RS + hs + 4 * (c & 3));
}

// ------------------------------------------------------------------------------------------------
// forward.  NT = the tiles a side (ceil(K / 16)); DROPK: 0 none, 1 K even (pair hashes), 2 K odd
template <int NT, int DH, bool BIAS, int DROPK>
__global__ __launch_bounds__(256) void attn_fwd_mf_kernel(AttnBfArgs a) {
  const int b = wg_sample(a), hgrp = wg_group(a);
  if (b >= a.B) return;      // the grid's tail past the last sample
  using S = Stg<DH, NT>;
  using KB = Kt<NT>;
  extern __shared__ __attribute__((aligned(16))) __bf16 smb[];
  const int K = a.K, D = a.D, G = a.G;
  __bf16* sq = smb;
  __bf16* sk = sq + S::IM;
  __bf16* sv = sk + S::IM;
  float* srel = (float*)(sv + S::IM + S::PAD);
  stage<DH, NT, false>(a, b, hgrp, sq, sk, sv, nullptr);
  if (BIAS) stage_rel<NT>(a, srel);
  __syncthreads();
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
  const int h = hgrp * G + w, hs = w * S::HS;
  bf16x4 kop[NT], vtop[NT];
#pragma unroll
  for (int tj = 0; tj < NT; ++tj) {
    kop[tj] = op_row<DH, NT>(sk, 16 * tj + c, hs, g);          // A = k [j][d]
    vtop[tj] = op_col<DH, NT>(sv, 16 * tj, hs, g, c);          // A = v^T [d][j]
  }
  const float* rb = srel + KB::KT + a.tk + 4 * g - c;      // + 16 (tj - ti) + r
  const long hr = ((long)b * a.H + h) * K;                 // (head, row 0)
  uint32_t words[KB::NW];
#pragma unroll
  for (int q = 0; q < KB::NW; ++q) words[q] = 0u;
  const float dsc = DROPK ? a.drop.scale : 1.0f;
#pragma unroll
  for (int ti = 0; ti < NT; ++ti) {
    __builtin_amdgcn_sched_barrier(0);
    const bf16x4 qop = op_row<DH, NT>(sq, 16 * ti + c, hs, g); // B = q^T [d][i]
    const int i = 16 * ti + c;
    const uint32_t rowbase = (uint32_t)((hr + i) * K);
    // nt > 4: this query tile's keep bits first (bit 4 tj + r of kbw), so the hash chains die before the exp
    // pass instead of being interleaved with it (the interleaved form needed ~450 registers at nt = 10)
    uint32_t kbw[2] = {0u, 0u};
    if constexpr (DROPK != 0 && NT > 4) {
#pragma unroll
      for (int tj = 0; tj < NT; ++tj) {
        const uint32_t j0 = 16 * tj + 4 * g;
        uint32_t half[4];
        if (DROPK == 1) {
          const uint32_t h0 = drop_pair_bits(a.drop, (rowbase + j0) >> 1);
          const uint32_t h1 = drop_pair_bits(a.drop, (rowbase + j0 + 2) >> 1);
          half[0] = h0 & 0xFFFFu;
          half[1] = h0 >> 16;
          half[2] = h1 & 0xFFFFu;
          half[3] = h1 >> 16;
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const uint32_t idx = rowbase + j0 + r;
            const uint32_t hb = mix32((idx >> 1) ^ a.drop.key);
            half[r] = (idx & 1u) ? hb >> 16 : hb & 0xFFFFu;
          }
        }
        uint32_t nib = 0u;
#pragma unroll
        for (int r = 0; r < 4; ++r) nib |= (~sign_mask(half[r] - a.drop.thresh) & 1u) << r;
        const int p = 4 * tj;
        kbw[p >> 5] |= nib << (p & 31);
      }
    }
    f32x4 t[NT];
    float mx = -INFINITY;
#pragma unroll
    for (int tj = 0; tj < NT; ++tj) {
      const f32x4 s = mma(kop[tj], qop, f32x4{0.f, 0.f, 0.f, 0.f});                    // S^T [j][i]
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        t[tj][r] = BIAS ? fmaf(s[r], L2E, rb[16 * (tj - ti) + r]) : s[r] * L2E;
        mx = fmaxf(mx, t[tj][r]);
      }
    }
    mx = grp_max(mx);
    float l = 0.f;
    uint32_t dropped = 0u;
    f32x4 oacc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int tj = 0; tj < NT; ++tj) {
      float pe[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        pe[r] = __builtin_amdgcn_exp2f(t[tj][r] - mx);
        l += pe[r];
      }
      if (DROPK != 0 && NT > 4) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {      // all ones where kept
          const int p = 4 * tj + r;
          const uint32_t km = (uint32_t)__builtin_amdgcn_sbfe((int)kbw[p >> 5], p & 31, 1);
          pe[r] = __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, pe[r]) & km);
        }
      } else if (DROPK) {
        // keep iff the element's 16-bit hash half >= thresh; drop mask m = (half - thresh) >> 31 (arithmetic:
        // all ones = dropped), p~ = p & ~m, and the dropped-bit word collects m's bit (one v_and_or each) --
        // integer arithmetic throughout: compares would leave 64 lane masks in SGPRs (spilled).  The masked
        // values live in a float array: the same and-not on f32x4 elements was miscompiled (ROCm 7.2: every
        // element masked from element 0's value, found on gfx950 against the torch reference)
        const uint32_t j0 = 16 * tj + 4 * g;
        uint32_t half[4];
        if (DROPK == 1) {     // K even: (j, j+1) for even j is one pair hash
          const uint32_t h0 = drop_pair_bits(a.drop, (rowbase + j0) >> 1);
          const uint32_t h1 = drop_pair_bits(a.drop, (rowbase + j0 + 2) >> 1);
          half[0] = h0 & 0xFFFFu;
          half[1] = h0 >> 16;
          half[2] = h1 & 0xFFFFu;
          half[3] = h1 >> 16;
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const uint32_t idx = rowbase + j0 + r;
            const uint32_t hb = mix32((idx >> 1) ^ a.drop.key);
            half[r] = (idx & 1u) ? hb >> 16 : hb & 0xFFFFu;
          }
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const uint32_t m = sign_mask(half[r] - a.drop.thresh);
          pe[r] = __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, pe[r]) & ~m);
          dropped |= m & (1u << (4 * tj + r));
        }
      }
      const bf16x4 pb = __builtin_bit_cast(bf16x4, pk_bf4(f32x4{pe[0], pe[1], pe[2], pe[3]}));
      oacc = mma(vtop[tj], pb, oacc);                                                  // o^T [d][i]
      // K > 64: p as hi + lo (lo_bf4); K <= 64 keeps bf16(p) alone -- the bits of attn_layer_fwd_kernel, whose
      // registers (64 at eight waves per SIMD) hold no lo term
      if constexpr (NT > 4) oacc = mma(vtop[tj], lo_bf4(pe, pb), oacc);
    }
    l = grp_sum(l);
    if (i < K) {
      const float inv = dsc / l;
      if (4 * g < DH) *(f32x4*)(a.o + ((long)b * K + i) * D + h * DH + 4 * g) = oacc * inv;
      if (g == 0) {
        a.mrow[hr + i] = mx;
        a.lrow[hr + i] = l;
      }
    }
    if (DROPK && NT <= 4) words[ti >> 1] |= (~dropped & 0xFFFFu) << (16 * (ti & 1));
    if constexpr (DROPK != 0 && NT > 4) {     // stored layout: key-tile major (a nibble never straddles words)
#pragma unroll
      for (int tj = 0; tj < NT; ++tj) {
        const int p = 4 * tj, q = 4 * NT * tj + 4 * ti;
        words[q >> 5] |= ((kbw[p >> 5] >> (p & 31)) & 0xFu) << (q & 31);
      }
    }

  }
  if (DROPK) {
    uint32_t* mk = a.mask + ((long)b * a.H + h) * (64 * KB::NW);
#pragma unroll
    for (int q = 0; q < KB::NW; ++q) mk[64 * q + lane] = words[q];
  }
}

// ------------------------------------------------------------------------------------------------
// backward: dq, dk, dv into dqkv; positional-bias grad partials (diagonal sums of dS over the group's heads).
// Key tiles outer (dk, dv of a key tile complete in its iteration), query tiles inner (dq accumulates).
// four waves per SIMD (128 registers, no spill; with the compact rows four workgroups fit a CU's LDS): 141 -> 126 us
// at cfg2 against three
// start of tile diagonal ee = a - c (-15 .. 15) in a 16 x 16 tile stored diagonal-major, rows of 16 - |ee| floats
__device__ __forceinline__ int diag_off(int ee) {
  const int n = ee + 15;
  return n <= 16 ? n * (n + 1) / 2 : 256 - (31 - n) * (32 - n) / 2;
}

template <int NT, int DH, bool BIAS, bool DROP, int HG = 4, bool DX = false>
__global__ __launch_bounds__(64 * HG) __attribute__((amdgpu_waves_per_eu(4))) void attn_bwd_mf_kernel(AttnBfArgs a) {
  const int b = wg_sample(a), hgrp = wg_group(a);
  if (b >= a.B) return;      // the grid's tail past the last sample
  using S = Stg<DH, NT, HG>;
  using KB = Kt<NT>;
  constexpr int ND = 2 * NT - 1, IMG = img_elems<NT>(), KT = KB::KT;
  extern __shared__ __attribute__((aligned(16))) __bf16 smb[];
  const int K = a.K, D = a.D, G = a.G;
  __bf16* sq = smb;
  __bf16* sk = sq + S::IM;
  __bf16* sv = sk + S::IM;
  __bf16* sdo = sv + S::IM;
  __bf16* simg = sdo + S::IM + S::PAD;              // per wave: dS image, p~ image
  float* srel = (float*)(simg + HG * 2 * IMG);
  // DX: the bf16 dqkv rows [KT][DXS] past the staging / epilogue space (a.dx_lds bytes from the base)
  constexpr int DXS = 104;                  // 208-byte rows: the tail's 16-byte row reads hit distinct banks
  __bf16* sdx = (__bf16*)((char*)smb + (DX ? a.dx_lds : 0));
  const bool opj = a.dh1 != nullptr;      // block-uniform
  const int GD = G * DH;                    // the workgroup's columns of dO
  float* dot = (float*)simg;                // opj: the dO tile [KT][GD] (fp32), in the image space until the loop
  // the row statistics' operands (this lane's query row: o, the forward's row max / sum, dO without opj) and the
  // keep words, loaded first: their round trips overlap the staging's instead of following its barrier
  static_assert(KT == 64, "one query row per lane");
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
  const int h = hgrp * G + w, hs = w * S::HS;
  const long hr = ((long)b * a.H + h) * K;
  f32x4 o_row[DH / 4], do_row[DH / 4];
  float m_row = 0.f, l_row = 1.f;
  if (lane < K) {
    const float* op = a.o + ((long)b * K + lane) * D + h * DH;
#pragma unroll
    for (int q = 0; q < DH / 4; ++q) {
      o_row[q] = *(const f32x4*)(op + 4 * q);
      do_row[q] = opj ? f32x4{0.f, 0.f, 0.f, 0.f} : *(const f32x4*)(a.dO + ((long)b * K + lane) * D + h * DH + 4 * q);
    }
    m_row = a.mrow[hr + lane];
    l_row = a.lrow[hr + lane];
  }
  uint32_t words[KB::NW];
#pragma unroll
  for (int q = 0; q < KB::NW; ++q) words[q] = 0u;
  if (DROP) {
    const uint32_t* mk = a.mask + ((long)b * a.H + h) * (64 * KB::NW);
#pragma unroll
    for (int q = 0; q < KB::NW; ++q) words[q] = mk[64 * q + lane];
  }
  if (opj) {
    // dO = dh1 W_out on v_mfma_f32_16x16x4f32 in rowgemm.hip's k order (lane group g: k = 8g + kk; + 0.f as its
    // bias-less epilogue): the same bits as the ctr_rowgemm launch it replaces.  Tiles: 4 row blocks x ncb column
    // blocks of the workgroup's GD columns, at most two per wave; operands straight from global (a lane's dh1
    // row segment is two 16-byte loads), issued before the q / k / v staging so the round trips overlap.
    const int w0 = threadIdx.x >> 6, l0 = threadIdx.x & 63, g0 = l0 >> 4, c0 = l0 & 15;
    const int ncb = (GD + 15) >> 4, cbase = hgrp * GD;   // 1 or 2 (GD <= 32): tile t = (rb = t >> nsh, t & nm)
    const int nsh = ncb - 1, nm = ncb - 1;
    const long r0 = (long)b * K;
    f32x4 acc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    int tiles[2] = {-1, -1};
    for (int t = w0, q = 0; t < 4 * ncb && q < 2; t += G, ++q) {
      tiles[q] = t;
      const int rb = t >> nsh, i = 16 * rb + c0, n = cbase + 16 * (t & nm) + c0;
      const bool nin = 16 * (t & nm) + c0 < GD;
      f32x4 x0 = {0.f, 0.f, 0.f, 0.f}, x1 = x0;
      if (i < K) {
        x0 = *(const f32x4*)(a.dh1 + (r0 + i) * 32 + 8 * g0);
        x1 = *(const f32x4*)(a.dh1 + (r0 + i) * 32 + 8 * g0 + 4);
      }
      float wv[8];
#pragma unroll
      for (int kk = 0; kk < 8; ++kk) wv[kk] = nin ? a.w_out[(8 * g0 + kk) * 32 + n] : 0.f;
#pragma unroll
      for (int kk = 0; kk < 8; ++kk)
        acc[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(kk < 4 ? x0[kk] : x1[kk - 4], wv[kk], acc[q], 0, 0, 0);
    }
    stage<DH, NT, false, HG>(a, b, hgrp, sq, sk, sv, nullptr);
    for (int j = threadIdx.x; j < KT; j += blockDim.x) {   // sdo's mask / zero chunks
      *(bf16x4*)(sdo + j * S::RS + S::MOFF) = bf16x4{};
      *(bf16x4*)(sdo + j * S::RS + S::ZOFF) = bf16x4{};
    }
    if (BIAS) stage_rel<NT>(a, srel);
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      if (tiles[q] < 0) continue;
      const int rb = tiles[q] >> nsh, col = 16 * (tiles[q] & nm) + c0;
      if (col >= GD) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = 16 * rb + 4 * g0 + r;
        const float v = i < K ? acc[q][r] + 0.f : 0.f;
        dot[i * GD + col] = v;
        sdo[i * S::RS + col] = (__bf16)v;
      }
    }
  } else {
    stage<DH, NT, true, HG>(a, b, hgrp, sq, sk, sv, sdo);
    if (BIAS) stage_rel<NT>(a, srel);
  }
  lds_barrier();
  __bf16* ids = simg + w * 2 * IMG;
  __bf16* ipt = ids + IMG;
  const float* rb = srel + KT + a.tk + 4 * g - c;
  // per query row i (lane): {max (log2), 1 / sum, D_i = do_i . o_i} in the wave's LDS row table, read back
  // per score tile (padded rows: p = 0, D = 0)
  f32x4* stw = (f32x4*)(srel + rel_floats<NT>(BIAS ? a.tk : 0)) + w * KT;
  {
    f32x4 st = {0.f, 0.f, 0.f, 0.f};
    if (lane < K) {
      float s = 0.f;
#pragma unroll
      for (int q = 0; q < DH / 4; ++q) {
        // D_i from bf16(dO): the dO operand the dP product takes (lo_bf4 above)
        const f32x4 x = bfr4(opj ? *(const f32x4*)(dot + lane * GD + w * DH + 4 * q) : do_row[q]), y = o_row[q];
        s = fmaf(x[0], y[0], s);
        s = fmaf(x[1], y[1], s);
        s = fmaf(x[2], y[2], s);
        s = fmaf(x[3], y[3], s);
      }
      st = f32x4{m_row, 1.0f / l_row, s, 0.f};
    }
    stw[lane] = st;
  }
  __builtin_amdgcn_wave_barrier();
  if (opj) lds_barrier();                 // every wave's dO-tile reads before the images overwrite it
  const uint32_t dsc_bits = __builtin_bit_cast(uint32_t, DROP ? a.drop.scale : 1.0f);
  f32x4 dq[NT];
  float dg[ND][4];
#pragma unroll
  for (int ti = 0; ti < NT; ++ti) dq[ti] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int dt = 0; dt < ND; ++dt)
#pragma unroll
    for (int r = 0; r < 4; ++r) dg[dt][r] = 0.f;
#pragma unroll
  for (int tj = 0; tj < NT; ++tj) {
    __builtin_amdgcn_sched_barrier(0);     // one key tile at a time: bounds the live registers
    const int j = 16 * tj + c;
    const bf16x4 kop = op_row<DH, NT, HG>(sk, j, hs, g);                                       // A = k [j][d]
    const bf16x4 vop = op_row<DH, NT, HG>(sv, j, hs, g);                                       // A = v [j][d]
    const bf16x4 ktop = op_col<DH, NT, HG>(sk, 16 * tj, hs, g, c);                             // A = k^T [d][j]
#pragma unroll
    for (int ti = 0; ti < NT; ++ti) {
      const int i = 16 * ti + c;
      const bf16x4 qop = op_row<DH, NT, HG>(sq, i, hs, g);                                     // B = q^T [d][i]
      const bf16x4 doop = op_row<DH, NT, HG>(sdo, i, hs, g);                                   // B = do^T [d][i]
      const f32x4 s = mma(kop, qop, f32x4{0.f, 0.f, 0.f, 0.f});                       // S^T [j][i]
      const f32x4 dp = mma(vop, doop, f32x4{0.f, 0.f, 0.f, 0.f});                     // dP~^T [j][i]
      const f32x4 st = stw[i];
      f32x4 dsv, ptv;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float x = BIAS ? fmaf(s[r], L2E, rb[16 * (tj - ti) + r]) : s[r] * L2E;
        const float p = __builtin_amdgcn_exp2f(x - st[0]) * st[1];
        float dpk = dp[r], pt = p;
        if (DROP) {   // keep ? 1 / (1 - p) : 0, from the bit's sign-extension
          const int pos = 16 * ti + 4 * tj + r;
          const float kf = __builtin_bit_cast(float, bit_mask(words[pos >> 5], pos & 31) & dsc_bits);
          dpk *= kf;
          pt *= kf;
        }
        const float ds = p * (dpk - st[2]);
        if (BIAS) dg[tj - ti + NT - 1][r] += ds;
        dsv[r] = ds;
        ptv[r] = pt;
      }
      const u32x2 dsu = pk_bf4(dsv), ptu = pk_bf4(ptv);
      dq[ti] = mma(ktop, __builtin_bit_cast(bf16x4, dsu), dq[ti]);                      // dq^T [d][i]
      *(u32x2*)(ids + swz(i, g)) = dsu;
      *(u32x2*)(ipt + swz(i, g)) = ptu;
    }
    __builtin_amdgcn_wave_barrier();
    // dk^T [d][j] = sum_i q^T [d][i] dS [i][j], dv^T [d][j] = sum_i do^T [d][i] p~ [i][j]
    f32x4 dk = {0.f, 0.f, 0.f, 0.f}, dv = dk;
#pragma unroll
    for (int ti = 0; ti < NT; ++ti) {
      const int rw = 16 * ti + 4 * g + (c >> 2);
      dk = mma(op_col<DH, NT, HG>(sq, 16 * ti, hs, g, c), tr4(ids + swz(rw, c & 3)), dk);      // B = dS [i][j]
      dv = mma(op_col<DH, NT, HG>(sdo, 16 * ti, hs, g, c), tr4(ipt + swz(rw, c & 3)), dv);     // B = p~ [i][j]
    }
    __builtin_amdgcn_wave_barrier();
    if (4 * g < DH && j < K) {
      const long off = ((long)b * K + j) * 3 * D + h * DH + 4 * g;
      store_dqkv(a, off + D, dk);
      store_dqkv(a, off + 2 * D, dv);
      if constexpr (DX) {      // the workgroup's copy of its bf16 dqkv rows for the in-projection product below
        *(u32x2*)(sdx + j * DXS + D + h * DH + 4 * g) = pk_bf4(dk);
        *(u32x2*)(sdx + j * DXS + 2 * D + h * DH + 4 * g) = pk_bf4(dv);
      }
    }
  }
  if (4 * g < DH) {
#pragma unroll
    for (int ti = 0; ti < NT; ++ti) {
      const int i = 16 * ti + c;
      if (i < K) {
        store_dqkv(a, ((long)b * K + i) * 3 * D + h * DH + 4 * g, dq[ti] * a.scale);
        if constexpr (DX) *(u32x2*)(sdx + i * DXS + h * DH + 4 * g) = pk_bf4(dq[ti] * a.scale);
      }
    }
  }
  // DX: the in-projection product's operands that do not come from this kernel, issued before the bias epilogue
  // (wave w: column block w & 1, row blocks w / 2 (+ 2 with four waves); W_in (96, 32) row-major, tb = 0)
  const long r0 = (long)b * K;
  float wv[DX ? 24 : 1], res[DX ? 8 / HG : 1][4];
  if constexpr (DX) {
    const int n = 16 * (w & 1) + c;
#pragma unroll
    for (int kk = 0; kk < 24; ++kk) wv[kk] = a.w_in[(24 * g + kk) * 32 + n];
#pragma unroll
    for (int q = 0; q < 8 / HG; ++q)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) res[q][rr] = a.dh1[(r0 + min(16 * ((w >> 1) + 2 * q) + 4 * g + rr, K - 1)) * 32 + n];
  }
  if (BIAS) {
    // diagonal sums of dS: register (dt, r) of lane (g, c) holds the sum over the tiles of diagonal dt of
    // element (a = 4g + r, c) = diagonal 16 (dt - (NT-1)) + a - c.  Heads first (fixed order), then diagonals.
    lds_barrier();                                    // staging / image space is reused
    float* sd = (float*)smb;                            // [G][ND][16 a][16 c]
#pragma unroll
    for (int dt = 0; dt < ND; ++dt)
#pragma unroll
      for (int r = 0; r < 4; ++r) sd[((w * ND + dt) * 16 + 4 * g + r) * 16 + c] = dg[dt][r];
    lds_barrier();
    // head sums (fixed order), stored diagonal-major: tile diagonal ee = a - c of tile-diagonal dt is a packed row
    // of 16 - |ee| floats at dt * 256 + diag_off(ee), element min(a, c) -- a diagonal's sum then reads one row at
    // immediate offsets (the [a][c] layout took a computed address per element).  A thread's loads are issued
    // together (heads clamped in range, unused values dropped): the chains of dependent LDS round trips were this
    // epilogue's cost.
    float* sh = sd + G * ND * 256;                      // [ND][256] (+ 16 floats of read padding)
    for (int p = threadIdx.x; p < 256; p += blockDim.x) {
      const int aa = p >> 4, cc = p & 15;
      const int o = diag_off(aa - cc) + (aa < cc ? aa : cc);
      float v[ND][HG];
#pragma unroll
      for (int dt = 0; dt < ND; ++dt)
#pragma unroll
        for (int u = 0; u < HG; ++u) v[dt][u] = sd[((u < G ? u : 0) * ND + dt) * 256 + p];
#pragma unroll
      for (int dt = 0; dt < ND; ++dt) {
        float s = 0.f;
#pragma unroll
        for (int u = 0; u < HG; ++u)
          if (u < G) s += v[dt][u];
        sh[dt * 256 + o] = s;
      }
    }
    lds_barrier();
    // thread 2 x + half: diagonal d = x - (16 NT - 1); half 0 the tile diagonal with 0 <= d - 16 dt' <= 15,
    // half 1 the one above it (-16 <= d - 16 dt' <= -1; -16 is no diagonal of a tile).  Element order along a
    // row = ascending a, the order of the sum it replaces.
    constexpr int NDG = 2 * 16 * NT - 1;
    const int nrel = 2 * a.tk + 1;
    float* out = a.drel_part + ((long)b * a.ngrp + hgrp) * nrel;
    for (int t0 = 0; t0 < 2 * NDG; t0 += blockDim.x) {
      const int t = t0 + threadIdx.x;
      const int x = t >> 1, half = t & 1;
      const int d = x - (16 * NT - 1);
      float s = 0.f;
      if (x < NDG) {
        const int dth = (d >= 0 ? d : d - 15) / 16;      // floor(d / 16)
        const int dtp = dth + half;
        const int e = d - 16 * dtp;
        const int dtx = dtp + NT - 1;
        const bool tin = dtx >= 0 && dtx < ND && e > -16;
        const int len = 16 - (e < 0 ? -e : e);
        const float* row = sh + (tin ? dtx * 256 + diag_off(e) : 0);
        float vv[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) vv[k] = row[k];
#pragma unroll
        for (int k = 0; k < 16; ++k)
          if (tin && k < len) s += vv[k];
      }
      // the pair (half 0, half 1) is lanes (2x, 2x+1): half 0 adds its neighbour's sum
      const float o = __shfl_xor(s, 1);
      if (half == 0 && x < NDG) {
        const int ei = d + a.tk;
        if (ei >= 0 && ei < nrel) out[ei] = (d > -K && d < K) ? s + o : 0.f;
      }
    }
    // offsets outside [-(16 NT - 1), 16 NT - 1]: zero
    for (int e = threadIdx.x; e < nrel; e += blockDim.x) {
      const int d = e - a.tk;
      if (d < -(16 * NT - 1) || d > 16 * NT - 1) out[e] = 0.f;
    }
  }
  if constexpr (DX) {
    // The in-projection's input grad of the sample's rows plus the residual, dx = dqkv W_in + dh1 (dare.py:53-70:
    // the in_proj backward of MHA and the skip connection around it), from the workgroup's LDS copy of the bf16 dqkv
    // rows it stored: rowgemm_kernel<96, 32, true, true>'s products in its k order and its epilogue -- lane group g
    // holds k = 24 g .. 24 g + 23 of row 16 rb + c, one v_mfma_f32_16x16x4f32 per k step, (acc + 0) + dh1 -- so the
    // bits of the ctr_rowgemm_a16 launch this replaces.  Tiles (row block rb, column block cb) of the K x 32 result.
    if (!BIAS) lds_barrier();                         // (the bias epilogue's barriers order the copy otherwise)
    typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
    const int cb = w & 1, n = 16 * cb + c;
#pragma unroll
    for (int q = 0; q < 8 / HG; ++q) {
      const int rb = (w >> 1) + 2 * q;
      if (16 * rb >= K) break;                        // wave-uniform
      const __bf16* ap = sdx + min(16 * rb + c, K - 1) * DXS + 24 * g;
      const bf16x8 v0 = *(const bf16x8*)ap, v1 = *(const bf16x8*)(ap + 8), v2 = *(const bf16x8*)(ap + 16);
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < 24; ++kk) {
        const float av = kk < 8 ? (float)v0[kk] : kk < 16 ? (float)v1[kk - 8] : (float)v2[kk - 16];
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av, wv[kk], acc, 0, 0, 0);
      }
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int i = 16 * rb + 4 * g + rr;
        if (i < K) {
          float v = acc[rr] + 0.f;
          v += res[q][rr];
          a.dx[(r0 + i) * 32 + n] = v;
        }
      }
    }
  }
}
// ------------------------------------------------------------------------------------------------
// backward for K > 64 (nt > 4).  The nt <= 4 kernel's per-wave [KT][16] dS / p~ images and its (2 nt - 1) x 4
// diagonal registers would take ~120 KB of LDS and ~500 registers per wave at nt = 10; here
//   * dk, dv of the key tile accumulate per query tile through a 16 x 16 image pair (dS, p~ of tile (ti, tj)
//     written, read back transposed, consumed) -- 1 KB per wave;
//   * the positional-bias diagonal sums run in a window of nt tile diagonals: diagonal tile dt = tj - ti + nt - 1
//     sits in window slot nt - 1 - ti while key tile tj runs, and slot 0 (dt = tj) is final after it (later
//     key tiles only reach dt > tj), so it is folded into the wave's per-diagonal sums in LDS (a 16 x 16 scratch,
//     31 lanes each summing one diagonal in a fixed order) and the window moves on -- with tj unrolled the move
//     is register renaming.  The heads of the workgroup are summed in a fixed order at the end.
#ifndef ATT_DB
#define ATT_DB 1
#endif
#ifndef ATT_WPE
#define ATT_WPE 0
#endif
#ifndef ATT_SB
#define ATT_SB 0
#endif
template <int NT, int DH, bool BIAS, bool DROP>
__global__ __launch_bounds__(256)
#if ATT_WPE
__attribute__((amdgpu_waves_per_eu(ATT_WPE)))
#endif
void attn_bwd_mfl_kernel(AttnBfArgs a) {
  const int b = wg_sample(a), hgrp = wg_group(a);
  if (b >= a.B) return;      // the grid's tail past the last sample
  using S = Stg<DH, NT>;
  using KB = Kt<NT>;
  constexpr int KT = KB::KT, NDG = 32 * NT - 1, NDGP = (NDG + 3) & ~3;
  extern __shared__ __attribute__((aligned(16))) __bf16 smb[];
  const int K = a.K, D = a.D, G = a.G;
  __bf16* sq = smb;
  __bf16* sk = sq + S::IM;
  __bf16* sv = sk + S::IM;
  __bf16* sdo = sv + S::IM;
  __bf16* simg = sdo + S::IM + S::PAD;              // per wave: 16 x 16 dS image, 16 x 16 p~ image (x2)
  float* srel = (float*)(simg + 4 * 4 * 256);
  // keep words: key tile tj's 4 nt bits start at bit 4 nt tj of the lane's word row and span up to three words;
  // the next tile's words are loaded while the current one runs (tile 0's during the staging)
  const uint32_t* mk = a.mask + ((long)b * a.H + hgrp * G + (threadIdx.x >> 6)) * (64 * KB::NW) + (threadIdx.x & 63);
  auto fetch_kw = [&](int t, uint32_t (&kw)[3]) {
    const int w0 = (4 * NT * t) >> 5;
#pragma unroll
    for (int u = 0; u < 3; ++u) kw[u] = mk[64 * min(w0 + u, KB::NW - 1)];
  };
  uint32_t kwn[3] = {0u, 0u, 0u};
  if (DROP) fetch_kw(0, kwn);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
  const int h = hgrp * G + w, hs = w * S::HS;
  const long hr = ((long)b * a.H + h) * K;
  // the row statistics' operands (dO, o, the forward's row max / sum of the lane's rows) loaded before the
  // staging, all of them at once: their round trips overlap the staging's instead of following it one row at a time
  constexpr int NR = (KT + 63) / 64;
  f32x4 rdo[NR][DH / 4], ro[NR][DH / 4];
  float rm[NR], rl[NR];
#pragma unroll
  for (int u = 0; u < NR; ++u) {
    const int row = min(lane + 64 * u, K - 1);     // clamped (rows past K are zeroed below)
    const float* dp = a.dO + ((long)b * K + row) * D + h * DH;
    const float* op = a.o + ((long)b * K + row) * D + h * DH;
#pragma unroll
    for (int q = 0; q < DH / 4; ++q) {
      rdo[u][q] = *(const f32x4*)(dp + 4 * q);
      ro[u][q] = *(const f32x4*)(op + 4 * q);
    }
    rm[u] = a.mrow[hr + row];
    rl[u] = a.lrow[hr + row];
  }
  stage<DH, NT, true>(a, b, hgrp, sq, sk, sv, sdo);
  if (BIAS) stage_rel<NT>(a, srel);
  __bf16* ids0 = simg + w * 4 * 256;
  const float* rb = srel + KT + a.tk + 4 * g - c;
  f32x4* stw = (f32x4*)(srel + rel_floats<NT>(BIAS ? a.tk : 0)) + w * KT;
  float* sdg = (float*)(stw + (4 - w) * KT) + w * (256 + NDGP);   // per wave: [16][16] scratch, NDG diagonal sums
  float* dsum = sdg + 256;
#pragma unroll
  for (int u = 0; u < NR; ++u) {
    const int row = lane + 64 * u;
    float s = 0.f;
#pragma unroll
    for (int q = 0; q < DH / 4; ++q) {     // D_i from bf16(dO), as attn_bwd_mf_kernel
      const f32x4 x = bfr4(rdo[u][q]);
      s = fmaf(x[0], ro[u][q][0], s);
      s = fmaf(x[1], ro[u][q][1], s);
      s = fmaf(x[2], ro[u][q][2], s);
      s = fmaf(x[3], ro[u][q][3], s);
    }
    if (row < KT) stw[row] = row < K ? f32x4{rm[u], 1.0f / rl[u], s, 0.f} : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  if (BIAS)
    for (int e = lane; e < NDGP; e += 64) dsum[e] = 0.f;
  __syncthreads();
  const uint32_t dsc_bits = __builtin_bit_cast(uint32_t, DROP ? a.drop.scale : 1.0f);
  // fold the finished tile diagonal dt (values v[r] of element (a = 4g + r, c): diagonal 16 (dt - nt + 1) + a - c)
  // into dsum: lane e + 15 (e = a - c in [-15, 15]) sums its diagonal over a, ascending
  auto fold = [&](int dt, const float (&v)[4]) {
#pragma unroll
    for (int r = 0; r < 4; ++r) sdg[(4 * g + r) * 16 + c] = v[r];
    __builtin_amdgcn_wave_barrier();
    if (lane < 31) {
      const int e = lane - 15;
      float sum = 0.f;
      const int a0 = e > 0 ? e : 0, a1 = e < 0 ? 15 + e : 15;
      for (int aa = a0; aa <= a1; ++aa) sum += sdg[aa * 16 + (aa - e)];
      dsum[16 * dt + lane] += sum;          // diagonal 16 (dt - nt + 1) + e  ->  index 16 dt + e + 15
    }
    __builtin_amdgcn_wave_barrier();
  };
  f32x4 dq[NT];
  float win[NT][4];            // window slot k = tile diagonal tj + k
#pragma unroll
  for (int ti = 0; ti < NT; ++ti) dq[ti] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 0; k < NT; ++k)
#pragma unroll
    for (int r = 0; r < 4; ++r) win[k][r] = 0.f;
  // key tiles in a loop (unrolled, the per-query-tile operands of every key tile were hoisted and kept live:
  // ~340 registers at nt = 10); this tile's 4 nt keep bits (bit 4 ti + r) from the mask in global memory
#pragma unroll 1
  for (int tj = 0; tj < NT; ++tj) {
    const int j = 16 * tj + c;
    const bf16x4 kop = op_row<DH, NT>(sk, j, hs, g);                                   // A = k [j][d]
    const bf16x4 vop = op_row<DH, NT>(sv, j, hs, g);                                   // A = v [j][d]
    const bf16x4 ktop = op_col<DH, NT>(sk, 16 * tj, hs, g, c);                         // A = k^T [d][j]
    uint64_t kb = 0;
    if (DROP) {
      const uint32_t kw[3] = {kwn[0], kwn[1], kwn[2]};
      fetch_kw(min(tj + 1, NT - 1), kwn);
      const int p0 = 4 * NT * tj, w0 = p0 >> 5;
      const uint64_t lo = kw[0], hi = w0 + 1 < KB::NW ? kw[1] : 0u;
      kb = ((hi << 32) | lo) >> (p0 & 31);
      if ((p0 & 31) + 4 * NT > 64) kb |= (uint64_t)kw[2] << (64 - (p0 & 31));
    }
    const float* rbt = rb + 16 * tj;
    f32x4 dk = {0.f, 0.f, 0.f, 0.f}, dv = dk;
#pragma unroll
    for (int ti = 0; ti < NT; ++ti) {
#if ATT_SB
      __builtin_amdgcn_sched_barrier(0);
#endif
      __bf16* ids = ids0 + (ATT_DB ? (ti & 1) * 512 : 0);
      __bf16* ipt = ids + 256;
      const int i = 16 * ti + c;
      const bf16x4 qop = op_row<DH, NT>(sq, i, hs, g);                                 // B = q^T [d][i]
      const bf16x4 doop = op_row<DH, NT>(sdo, i, hs, g);                               // B = do^T [d][i]
      const f32x4 s = mma(kop, qop, f32x4{0.f, 0.f, 0.f, 0.f});                       // S^T [j][i]
      const f32x4 dp = mma(vop, doop, f32x4{0.f, 0.f, 0.f, 0.f});                     // dP~^T [j][i]
      const f32x4 st = stw[i];
      f32x4 dsv, ptv;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float x = BIAS ? fmaf(s[r], L2E, rbt[r - 16 * ti]) : s[r] * L2E;
        const float p = __builtin_amdgcn_exp2f(x - st[0]) * st[1];
        float dpk = dp[r], pt = p;
        if (DROP) {
          const int pos = 4 * ti + r;
          const uint32_t wsel = pos < 32 ? (uint32_t)kb : (uint32_t)(kb >> 32);
          const float kf = __builtin_bit_cast(float, (uint32_t)__builtin_amdgcn_sbfe((int)wsel, pos & 31, 1) & dsc_bits);
          dpk *= kf;
          pt *= kf;
        }
        const float ds = p * (dpk - st[2]);
        if (BIAS) win[NT - 1 - ti][r] += ds;
        dsv[r] = ds;
        ptv[r] = pt;
      }
      const u32x2 dsu = pk_bf4(dsv), ptu = pk_bf4(ptv);
      dq[ti] = mma(ktop, __builtin_bit_cast(bf16x4, dsu), dq[ti]);                      // dq^T [d][i]
      // dk^T [d][j] += q^T [d][i] dS [i][j], dv^T [d][j] += do^T [d][i] p~ [i][j] over this tile's 16 queries
      *(u32x2*)(ids + swz(c, g)) = dsu;
      *(u32x2*)(ipt + swz(c, g)) = ptu;
#if !ATT_DB
      __builtin_amdgcn_wave_barrier();
#endif
      const int rw = 4 * g + (c >> 2);
      dk = mma(op_col<DH, NT>(sq, 16 * ti, hs, g, c), tr4(ids + swz(rw, c & 3)), dk);   // B = dS [i][j]
      dv = mma(op_col<DH, NT>(sdo, 16 * ti, hs, g, c), tr4(ipt + swz(rw, c & 3)), dv);  // B = p~ [i][j]
#if !ATT_DB
      __builtin_amdgcn_wave_barrier();
#endif
    }
    if (4 * g < DH && j < K) {
      const long off = ((long)b * K + j) * 3 * D + h * DH + 4 * g;
      store_dqkv(a, off + D, dk);
      store_dqkv(a, off + 2 * D, dv);
    }
    if (BIAS) {
      fold(tj, win[0]);
#pragma unroll
      for (int k = 0; k + 1 < NT; ++k)
#pragma unroll
        for (int r = 0; r < 4; ++r) win[k][r] = win[k + 1][r];
#pragma unroll
      for (int r = 0; r < 4; ++r) win[NT - 1][r] = 0.f;
    }
  }
  if (4 * g < DH) {
#pragma unroll
    for (int ti = 0; ti < NT; ++ti) {
      const int i = 16 * ti + c;
      if (i < K) store_dqkv(a, ((long)b * K + i) * 3 * D + h * DH + 4 * g, dq[ti] * a.scale);
    }
  }
  if (BIAS) {
#pragma unroll
    for (int k = 0; k + 1 < NT; ++k) fold(NT + k, win[k]);     // tile diagonals nt .. 2 nt - 2
    __syncthreads();
    // heads of the group summed in a fixed order; diagonal d = x - (16 nt - 1) of the x-th sum
    const int nrel = 2 * a.tk + 1;
    float* out = a.drel_part + ((long)b * a.ngrp + hgrp) * nrel;
    const float* base = (const float*)(stw + (4 - w) * KT);     // wave 0's scratch
    for (int e = threadIdx.x; e < nrel; e += blockDim.x) {
      const int d = e - a.tk, x = d + 16 * NT - 1;
      float sum = 0.f;
      if (d > -K && d < K) {
        for (int u = 0; u < G; ++u) sum += base[u * (256 + NDGP) + 256 + x];
      }
      out[e] = sum;
    }
  }
}

// ------------------------------------------------------------------------------------------------
// Fused first half of an encoder layer (amp: bf16, D = 32, every head of a sample in one workgroup, K <= 64):
//   qkv = x W_in^T + b_in  ->  attention (the forward above, one wave per head)  ->
//   x1 = norm1(x + o W_out^T + b_out)   (src/models/dare.py:53-62: MultiheadAttention + residual + RMSNorm)
// One workgroup per sample.  The projections run on v_mfma_f32_16x16x4f32 (exact fp32 fmaf chains, as the row
// kernels they replace): the x rows, the attention output o and the out-projection result pass through LDS, and
// qkv / o / h1 / r1 / x1 are written for the backward and the next kernel -- two launches (in_proj, out_proj +
// norm) and their boundaries fewer per layer, and qkv / o are not read back from HBM by the forward.
namespace lf {
constexpr int D = 32, RS = 40, MOFF = 32, ZOFF = 36;     // staged bf16 rows: 8 x 4 or 4 x 8 head dims, mask, zero
constexpr int XS = D + 4;                                // fp32 x / o / y tile rows
}  // namespace lf

template <int DH>
__device__ __forceinline__ bf16x4 lf_row(const __bf16* img, int row, int hs, int g) {
  return ld4(img + row * lf::RS + (4 * g < DH ? hs + 4 * g : 4 * g == DH ? lf::MOFF : lf::ZOFF));
}
__device__ __forceinline__ bf16x4 lf_col(const __bf16* img, int row0, int hs, int g, int c) {
  return tr4(img + (row0 + 4 * g + (c >> 2)) * lf::RS + hs + 4 * (c & 3));
}

struct LayerFwdArgs {
  AttnBfArgs at;          // qkv (output), K, H, relmean, scale, drop, mask, o, mrow, lrow (B = samples)
  const float* x;         // (B*K, 32) layer input
  const float* w_in;      // (96, 32), b_in (96)
  const float* b_in;
  const float* w_out;     // (32, 32), b_out (32)
  const float* b_out;
  const float* nw1;       // (32) norm1 weight
  const float* rel_w;     // pbias.rel.weight (2tk+1, H): the head-mean bias formed here (null: no bias) ...
  float* relmean;         // ... and written by workgroup 0 for the backward (ctr_pos_bias_mean's bits)
  float eps;
  float* qkv;             // (B*K, 96) saved for the backward, or (qkv16, amp) its bf16 staged form:
  __bf16* qkv16;          // bf16(q * scale) | bf16(k) | bf16(v), copied from the LDS images
  float* h1;              // (B*K, 32) pre-norm sum, r1 (B*K) its rsqrt, x1 (B*K, 32) the layer's next input
  float* r1;
  float* x1;
};

template <int DH, bool BIAS, int DROPK>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(8))) void attn_layer_fwd_kernel(LayerFwdArgs L) {
  constexpr int NT = 4, KT = 64, G = lf::D / DH;     // all heads of the sample
  const AttnBfArgs& a = L.at;
  __shared__ __attribute__((aligned(16))) __bf16 sq[KT * lf::RS + 16];
  __shared__ __attribute__((aligned(16))) __bf16 sk[KT * lf::RS + 16];
  __shared__ __attribute__((aligned(16))) __bf16 sv[KT * lf::RS + 16];
  __shared__ __attribute__((aligned(16))) float xt[KT * lf::XS];      // x rows, then the out-projection result
  __shared__ __attribute__((aligned(16))) float ot[KT * lf::XS];      // attention output o
  __shared__ float srel[2 * 64 + 2 * KT + 4];
  const int K = a.K, b = blockIdx.x, tid = threadIdx.x;
  const int w = tid >> 6, lane = tid & 63, g = lane >> 4, c = lane & 15;
  const long row0 = (long)b * K;
  // ---- x rows -> LDS (zero rows >= K); mask / zero chunks; positional bias (log2 units)
  for (int e = tid; e < KT * lf::D / 4; e += 64 * G) {
    const int i = e / (lf::D / 4), c4 = (e % (lf::D / 4)) * 4;
    const f32x4 v = i < K ? *(const f32x4*)(L.x + (row0 + i) * lf::D + c4) : f32x4{0.f, 0.f, 0.f, 0.f};
    *(f32x4*)(xt + i * lf::XS + c4) = v;
  }
  for (int j = tid; j < KT; j += 64 * G) {
    const bf16x4 z4 = {};
    bf16x4 mq = z4, mk = z4;
    mq[0] = (__bf16)NEG_BIG;
    mk[0] = (__bf16)(j >= K ? 1.f : 0.f);
    *(bf16x4*)(sq + j * lf::RS + lf::MOFF) = mq;
    *(bf16x4*)(sk + j * lf::RS + lf::MOFF) = mk;
    *(bf16x4*)(sv + j * lf::RS + lf::MOFF) = z4;
    *(bf16x4*)(sq + j * lf::RS + lf::ZOFF) = z4;
    *(bf16x4*)(sk + j * lf::RS + lf::ZOFF) = z4;
    *(bf16x4*)(sv + j * lf::RS + lf::ZOFF) = z4;
  }
  if (BIAS) {   // stage_rel of the head-mean table, each entry summed over the heads as pos_bias_mean_kernel does
    const int nrel = 2 * a.tk + 1;
    for (int e = tid; e < nrel + 2 * KT; e += 64 * G) {
      const int x = e - KT;
      float v = 0.f;
      if (x >= 0 && x < nrel) {
        float sm = 0.f;
        for (int hh = 0; hh < a.H; ++hh) sm += L.rel_w[(long)x * a.H + hh];
        const float mean = sm / (float)a.H;
        if (b == 0) L.relmean[x] = mean;
        v = mean * L2E;
      }
      srel[e] = v;
    }
  }
  lds_barrier();
  // ---- in-projection: 4 row blocks x 6 column blocks of 16, K = 32 (8 MFMA k-steps of 4); tile t -> (rb, cb)
  for (int t = w; t < 24; t += G) {
    const int rb = t / 6, cb = t % 6;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {       // lane group g takes k = 8g + kk: rowgemm.hip's order, the same bits
      const float av = xt[(16 * rb + c) * lf::XS + 8 * g + kk];                 // A[i = c][k]
      const float bv = L.w_in[(16 * cb + c) * lf::D + 8 * g + kk];              // B[k][n = c] = W_in[n][k]
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc, 0, 0, 0);
    }
    const int n = 16 * cb + c, sec = n >> 5, col = n & 31;                      // q | k | v section, column
    const float bias = L.b_in[n];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = 16 * rb + 4 * g + r;
      const float v = acc[r] + bias;
      if (i < K && !L.qkv16) L.qkv[(row0 + i) * (3 * lf::D) + n] = v;
      __bf16* dst = sec == 0 ? sq : sec == 1 ? sk : sv;
      dst[i * lf::RS + col] = (__bf16)(i < K ? (sec == 0 ? v * a.scale : v) : 0.f);
    }
  }
  lds_barrier();
  if (L.qkv16) {    // amp: the staged images are what the backward stages -- 16-byte row pieces, 12 a row
    for (int e = tid; e < K * 12; e += 64 * G) {
      const int i = e / 12, ch = e - 12 * i, sec = ch >> 2, c8 = 8 * (ch & 3);
      const __bf16* src = (sec == 0 ? sq : sec == 1 ? sk : sv) + i * lf::RS + c8;
      *(uint4*)(L.qkv16 + (row0 + i) * (3 * lf::D) + 32 * sec + c8) = *(const uint4*)src;
    }
  }
  // ---- attention, wave w = head h (attn_fwd_mf_kernel's per-head body at nt = 4)
  {
    const int h = w, hs = h * DH;
    bf16x4 kop[NT], vtop[NT];
#pragma unroll
    for (int tj = 0; tj < NT; ++tj) {
      kop[tj] = lf_row<DH>(sk, 16 * tj + c, hs, g);
      vtop[tj] = lf_col(sv, 16 * tj, hs, g, c);
    }
    const float* rb = srel + KT + a.tk + 4 * g - c;
    const long hr = ((long)b * a.H + h) * K;
    const float dsc = DROPK ? a.drop.scale : 1.0f;
    const int nt = (K + 15) >> 4;
    const uint32_t dmask = nt >= 4 ? 0xFFFFu : (1u << (4 * nt)) - 1u;
    // the dropout decisions of all four query tiles first, as 64 bits (query tile ti: bits 16 (ti & 1) .. of
    // word ti >> 1, bit 4 tj + r = key 16 tj + 4 g + r): the hashes' temporaries are then not live beside the
    // score tiles (104 registers otherwise, two workgroups per CU instead of four)
    uint32_t dbits[2] = {0u, 0u};
    if (DROPK) {
#pragma unroll
      for (int ti = 0; ti < NT; ++ti) {
        const uint32_t rowbase = (uint32_t)((hr + 16 * ti + c) * K);
        uint32_t dropped = 0u;
#pragma unroll
        for (int tj = 0; tj < NT; ++tj) {
          const uint32_t j0 = 16 * tj + 4 * g;
          uint32_t half[4];
          if (DROPK == 1) {
            const uint32_t h0 = drop_pair_bits(a.drop, (rowbase + j0) >> 1);
            const uint32_t h1v = drop_pair_bits(a.drop, (rowbase + j0 + 2) >> 1);
            half[0] = h0 & 0xFFFFu;
            half[1] = h0 >> 16;
            half[2] = h1v & 0xFFFFu;
            half[3] = h1v >> 16;
          } else {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const uint32_t idx = rowbase + j0 + r;
              const uint32_t hb = mix32((idx >> 1) ^ a.drop.key);
              half[r] = (idx & 1u) ? hb >> 16 : hb & 0xFFFFu;
            }
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) dropped |= (half[r] < a.drop.thresh ? 1u : 0u) << (4 * tj + r);
        }
        dbits[ti >> 1] |= dropped << (16 * (ti & 1));
      }
    }
#pragma unroll
    for (int ti = 0; ti < NT; ++ti) {
      __builtin_amdgcn_sched_barrier(0);
      const bf16x4 qop = lf_row<DH>(sq, 16 * ti + c, hs, g);
      const int i = 16 * ti + c;
      f32x4 t[NT];
      float mx = -INFINITY;
#pragma unroll
      for (int tj = 0; tj < NT; ++tj) {
        const f32x4 sc = mma(kop[tj], qop, f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          t[tj][r] = BIAS ? fmaf(sc[r], L2E, rb[16 * (tj - ti) + r]) : sc[r] * L2E;
          mx = fmaxf(mx, t[tj][r]);
        }
      }
      mx = grp_max(mx);
      float l = 0.f;
      const uint32_t dropped = dbits[ti >> 1] >> (16 * (ti & 1));
      bf16x4 pb[NT];
#pragma unroll
      for (int tj = 0; tj < NT; ++tj) {
        float pe[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          pe[r] = __builtin_amdgcn_exp2f(t[tj][r] - mx);
          l += pe[r];
          if (DROPK && ((dropped >> (4 * tj + r)) & 1u)) pe[r] = 0.f;
        }
        pb[tj] = __builtin_bit_cast(bf16x4, pk_bf4(f32x4{pe[0], pe[1], pe[2], pe[3]}));
      }
      l = grp_sum(l);
      f32x4 oacc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int tj = 0; tj < NT; ++tj) oacc = mma(vtop[tj], pb[tj], oacc);
      const float inv = dsc / l;
      if (4 * g < DH) {
        const f32x4 ov = oacc * inv;
        *(f32x4*)(ot + i * lf::XS + h * DH + 4 * g) = i < K ? ov : f32x4{0.f, 0.f, 0.f, 0.f};
        if (i < K) *(f32x4*)(a.o + (row0 + i) * lf::D + h * DH + 4 * g) = ov;
      }
      if (i < K && g == 0) {
        a.mrow[hr + i] = mx;
        a.lrow[hr + i] = l;
      }
    }
    if (DROPK) {   // the keep words attn_fwd_mf_kernel writes at nt = ceil(K / 16): key tiles >= nt kept, query tiles >= nt none
      uint32_t* mk = a.mask + ((long)b * a.H + h) * 128;
      uint32_t words[2] = {0u, 0u};
#pragma unroll
      for (int ti = 0; ti < NT; ++ti)
        if (ti < nt) words[ti >> 1] |= (~((dbits[ti >> 1] >> (16 * (ti & 1))) & dmask) & 0xFFFFu) << (16 * (ti & 1));
      mk[lane] = words[0];
      mk[64 + lane] = words[1];
    }
  }
  lds_barrier();
  // ---- out-projection + bias + residual + RMSNorm: wave w < 4 takes row block w, both 16-column blocks, and
  // finishes it as rowgemm.hip's epilogue does (same k order, same per-row sum and 16-lane reduction: same bits)
  if (w < 4) {
    const int rb = w;
    f32x4 acc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
      const float av = ot[(16 * rb + c) * lf::XS + 8 * g + kk];
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, L.w_out[(16 * j + c) * lf::D + 8 * g + kk], acc[j], 0, 0, 0);
    }
    float bj[2], nw[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      bj[j] = L.b_out[16 * j + c];
      nw[j] = L.nw1[16 * j + c];
    }
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int i = 16 * rb + 4 * g + rr;
      float v[2], ss = 0.f;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        v[j] = acc[j][rr] + bj[j];
        v[j] = xt[i * lf::XS + 16 * j + c] + v[j];
        ss += v[j] * v[j];
      }
      ss = group_sum<16>(ss);
      const float r = 1.0f / sqrtf(ss / (float)lf::D + L.eps);
      if (i < K) {
        const long row = row0 + i;
        if (c == 0) L.r1[row] = r;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          L.h1[row * lf::D + 16 * j + c] = v[j];
          L.x1[row * lf::D + 16 * j + c] = nw[j] * v[j] * r;
        }
      }
    }
  }
}

int pick_g(int H) {
  int g = 1;
  for (int c = 1; c <= 4; ++c)
    if (H % c == 0) g = c;
  return g;
}

template <int DH, int NT>
size_t fwd_lds(int tk) { return ((size_t)3 * Stg<DH, NT>::IM + Stg<DH, NT>::PAD) * 2 + (size_t)rel_floats<NT>(tk) * 4; }

template <int DH, int NT, int HG = 4>
size_t bwd_lds(int G, int tk) {
  using S = Stg<DH, NT, HG>;
  const size_t main = ((size_t)4 * S::IM + S::PAD) * 2 + (size_t)HG * 2 * img_elems<NT>() * 2 +
                      (size_t)rel_floats<NT>(tk) * 4 + (size_t)HG * Kt<NT>::KT * 16;
  const size_t ND = 2 * NT - 1, diag = ((size_t)G * ND * 256 + ND * 256 + 16) * 4;
  return main > diag ? main : diag;
}

// nt > 4: operands, the four waves' 16 x 16 image pairs, bias table, stats rows, per-wave diagonal scratch + sums
template <int DH, int NT>
size_t bwdl_lds(int tk) {
  constexpr int NDGP = (32 * NT - 1 + 3) & ~3;
  return ((size_t)4 * Stg<DH, NT>::IM + Stg<DH, NT>::PAD) * 2 + (size_t)4 * 4 * 256 * 2 + (size_t)rel_floats<NT>(tk) * 4 +
         (size_t)4 * Kt<NT>::KT * 16 + (size_t)4 * (256 + NDGP) * 4;
}

// more than 64 KB of dynamic LDS (nt > 4) has to be allowed per kernel
template <class F>
void allow_lds(F* kern, size_t sm) {
  if (sm > 64 * 1024) (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm);
}

template <int NT, int DH, bool BIAS, int DROPK>
void launch_fwd5(const AttnBfArgs& a, size_t sm, hipStream_t s) {
  allow_lds(attn_fwd_mf_kernel<NT, DH, BIAS, DROPK>, sm);
  attn_fwd_mf_kernel<NT, DH, BIAS, DROPK><<<wg_grid(a), dim3(64 * a.G), sm, s>>>(a);
}

template <int NT, int DH, bool BIAS>
void launch_fwd4(const AttnBfArgs& a, size_t sm, hipStream_t s) {
  if (a.drop.thresh == 0) launch_fwd5<NT, DH, BIAS, 0>(a, sm, s);
  else if (a.K & 1) launch_fwd5<NT, DH, BIAS, 2>(a, sm, s);
  else launch_fwd5<NT, DH, BIAS, 1>(a, sm, s);
}

template <int NT, int DH>
void launch_fwd3(const AttnBfArgs& a, hipStream_t s) {
  const size_t sm = fwd_lds<DH, NT>(a.relmean ? a.tk : 0);
  if (a.relmean) launch_fwd4<NT, DH, true>(a, sm, s);
  else launch_fwd4<NT, DH, false>(a, sm, s);
}

template <int DH>
void launch_fwd2(const AttnBfArgs& a, hipStream_t s) {
  switch (a.nt) {
    case 1: launch_fwd3<1, DH>(a, s); break;
    case 2: launch_fwd3<2, DH>(a, s); break;
    case 3: launch_fwd3<3, DH>(a, s); break;
    case 4: launch_fwd3<4, DH>(a, s); break;
    case 5: launch_fwd3<5, DH>(a, s); break;
    case 6: launch_fwd3<6, DH>(a, s); break;
    case 7: launch_fwd3<7, DH>(a, s); break;
    case 8: launch_fwd3<8, DH>(a, s); break;
    case 9: launch_fwd3<9, DH>(a, s); break;
    default: launch_fwd3<10, DH>(a, s); break;
  }
}

template <int NT, int DH, bool BIAS, bool DROP>
void launch_bwd4(const AttnBfArgs& a, size_t sm, hipStream_t s) {
  if constexpr (NT > 4) {
    allow_lds(attn_bwd_mfl_kernel<NT, DH, BIAS, DROP>, sm);
    attn_bwd_mfl_kernel<NT, DH, BIAS, DROP><<<wg_grid(a), dim3(64 * a.G), sm, s>>>(a);
  } else {
    allow_lds(attn_bwd_mf_kernel<NT, DH, BIAS, DROP>, sm);
    attn_bwd_mf_kernel<NT, DH, BIAS, DROP><<<wg_grid(a), dim3(64 * a.G), sm, s>>>(a);
  }
}

template <int NT, int DH>
void launch_bwd3(const AttnBfArgs& a, hipStream_t s) {
  const size_t sm = NT > 4 ? bwdl_lds<DH, NT>(a.relmean ? a.tk : 0) : bwd_lds<DH, NT>(a.G, a.relmean ? a.tk : 0);
  const bool bias = a.relmean != nullptr, drop = a.drop.thresh != 0;
  if (bias && drop) launch_bwd4<NT, DH, true, true>(a, sm, s);
  else if (bias) launch_bwd4<NT, DH, true, false>(a, sm, s);
  else if (drop) launch_bwd4<NT, DH, false, true>(a, sm, s);
  else launch_bwd4<NT, DH, false, false>(a, sm, s);
}

template <int DH>
void launch_bwd2(const AttnBfArgs& a, hipStream_t s) {
  switch (a.nt) {
    case 1: launch_bwd3<1, DH>(a, s); break;
    case 2: launch_bwd3<2, DH>(a, s); break;
    case 3: launch_bwd3<3, DH>(a, s); break;
    case 4: launch_bwd3<4, DH>(a, s); break;
    case 5: launch_bwd3<5, DH>(a, s); break;
    case 6: launch_bwd3<6, DH>(a, s); break;
    case 7: launch_bwd3<7, DH>(a, s); break;
    case 8: launch_bwd3<8, DH>(a, s); break;
    case 9: launch_bwd3<9, DH>(a, s); break;
    default: launch_bwd3<10, DH>(a, s); break;
  }
}

// the layer backward: one workgroup of H waves per sample, every head staged in its rows (HG = H = D / dh)
template <int NT, int DH, bool BIAS, bool DROP>
void launch_bwd_layer4(const AttnBfArgs& a, hipStream_t s) {
  constexpr int HG = 32 / DH;
  AttnBfArgs b = a;
  b.dx_lds = (int)bwd_lds<DH, NT, HG>(a.G, BIAS ? a.tk : 0);
  const size_t sm = (size_t)b.dx_lds + (size_t)Kt<NT>::KT * 104 * 2;
  allow_lds(attn_bwd_mf_kernel<NT, DH, BIAS, DROP, HG, true>, sm);
  attn_bwd_mf_kernel<NT, DH, BIAS, DROP, HG, true><<<a.B, dim3(64 * HG), sm, s>>>(b);
}
template <int NT, int DH>
void launch_bwd_layer3(const AttnBfArgs& a, hipStream_t s) {
  const bool bias = a.relmean != nullptr, drop = a.drop.thresh != 0;
  if (bias && drop) launch_bwd_layer4<NT, DH, true, true>(a, s);
  else if (bias) launch_bwd_layer4<NT, DH, true, false>(a, s);
  else if (drop) launch_bwd_layer4<NT, DH, false, true>(a, s);
  else launch_bwd_layer4<NT, DH, false, false>(a, s);
}
template <int DH>
void launch_bwd_layer2(const AttnBfArgs& a, hipStream_t s) {
  switch (a.nt) {
    case 1: launch_bwd_layer3<1, DH>(a, s); break;
    case 2: launch_bwd_layer3<2, DH>(a, s); break;
    case 3: launch_bwd_layer3<3, DH>(a, s); break;
    default: launch_bwd_layer3<4, DH>(a, s); break;
  }
}

bool bf_ok(int K, int H, int D) {
  if (K < 1 || K > 16 * NT_MAX || H < 1 || D % H) return false;
  const int dh = D / H;
  return dh == 4 || dh == 8;
}

}  // namespace
}  // namespace ctr

using namespace ctr;

extern "C" int ctr_attn_bf_ok(int K, int H, int D) { return bf_ok(K, H, D) ? 1 : 0; }

extern "C" int ctr_attn_fwd_bf(const float* qkv, int B, int K, int H, int D, const float* relmean, int tk, float scale,
                               uint32_t drop_key, uint32_t drop_thresh, float drop_scale, uint32_t* mask, float* o,
                               float* mrow, float* lrow, void* stream) {
  if (B == 0) return 0;
  CTR_REQUIRE(bf_ok(K, H, D), "ctr_attn_fwd_bf: K <= 160 and head dim 4 or 8");
  CTR_REQUIRE(!relmean || tk >= K - 1, "positional-bias table shorter than K");
  CTR_REQUIRE(!drop_thresh || mask, "attention forward with dropout needs a keep-bit buffer");
  AttnBfArgs a{};
  a.qkv = qkv; a.B = B; a.K = K; a.H = H; a.D = D; a.G = pick_g(H); a.ngrp = H / a.G; a.nt = (K + 15) / 16; a.tk = tk;
  a.relmean = relmean; a.scale = scale; a.drop = Drop{drop_key, drop_thresh, drop_scale};
  a.mask = mask; a.o = o; a.mrow = mrow; a.lrow = lrow;
  hipStream_t s = (hipStream_t)stream;
  if (D / H == 4) launch_fwd2<4>(a, s);
  else launch_fwd2<8>(a, s);
  return check_launch("attn_fwd_bf");
}

extern "C" int ctr_attn_bwd_bf_nparts(int H) { return H / pick_g(H); }

extern "C" int ctr_attn_bwd_bf(const float* qkv, const float* o, const float* dO, int B, int K, int H, int D,
                               const float* relmean, int tk, float scale, uint32_t drop_key, uint32_t drop_thresh,
                               float drop_scale, const uint32_t* mask, const float* mrow, const float* lrow,
                               float* dqkv, float* drel_part, void* stream) {
  if (B == 0) return 0;
  CTR_REQUIRE(bf_ok(K, H, D), "ctr_attn_bwd_bf: K <= 160 and head dim 4 or 8");
  CTR_REQUIRE(!relmean || tk >= K - 1, "positional-bias table shorter than K");
  CTR_REQUIRE(!drop_thresh || mask, "attention backward with dropout needs the forward's keep bits");
  AttnBfArgs a{};
  a.qkv = qkv; a.B = B; a.K = K; a.H = H; a.D = D; a.G = pick_g(H); a.ngrp = H / a.G; a.nt = (K + 15) / 16; a.tk = tk;
  a.relmean = relmean; a.scale = scale; a.drop = Drop{drop_key, drop_thresh, drop_scale};
  a.mask = const_cast<uint32_t*>(mask); a.o = const_cast<float*>(o); a.mrow = const_cast<float*>(mrow);
  a.lrow = const_cast<float*>(lrow); a.dO = dO; a.dqkv = dqkv; a.drel_part = drel_part;
  hipStream_t s = (hipStream_t)stream;
  if (D / H == 4) launch_bwd2<4>(a, s);
  else launch_bwd2<8>(a, s);
  return check_launch("attn_bwd_bf");
}

extern "C" int ctr_attn_bwd_bf_oproj_ok(int K, int H, int D) {
  return (bf_ok(K, H, D) && K <= 64 && D == 32 && pick_g(H) == 4 && (4 * (D / H)) % 16 == 0) ? 1 : 0;
}

static int attn_bwd_oproj(const float* qkv, const __bf16* qkv16, const float* o, const float* dh1, const float* w_out,
                          int B, int K, int H, int D, const float* relmean, int tk, float scale, uint32_t drop_key,
                          uint32_t drop_thresh, float drop_scale, const uint32_t* mask, const float* mrow,
                          const float* lrow, float* dqkv, __bf16* dqkv16, float* drel_part, void* stream) {
  if (B == 0) return 0;
  CTR_REQUIRE(ctr_attn_bwd_bf_oproj_ok(K, H, D), "ctr_attn_bwd_bf_oproj: K <= 64, D = 32, 4 or 8 heads");
  CTR_REQUIRE(!relmean || tk >= K - 1, "positional-bias table shorter than K");
  CTR_REQUIRE(!drop_thresh || mask, "attention backward with dropout needs the forward's keep bits");
  AttnBfArgs a{};
  a.qkv = qkv; a.B = B; a.K = K; a.H = H; a.D = D; a.G = pick_g(H); a.ngrp = H / a.G; a.nt = (K + 15) / 16; a.tk = tk;
  a.relmean = relmean; a.scale = scale; a.drop = Drop{drop_key, drop_thresh, drop_scale};
  a.mask = const_cast<uint32_t*>(mask); a.o = const_cast<float*>(o); a.mrow = const_cast<float*>(mrow);
  a.lrow = const_cast<float*>(lrow); a.dO = nullptr; a.dqkv = dqkv; a.drel_part = drel_part;
  a.dh1 = dh1; a.w_out = w_out; a.qkv16 = qkv16; a.dqkv16 = dqkv16;
  hipStream_t s = (hipStream_t)stream;
  if (D / H == 4) launch_bwd2<4>(a, s);
  else launch_bwd2<8>(a, s);
  return check_launch("attn_bwd_bf_oproj");
}

extern "C" int ctr_attn_bwd_bf_oproj(const float* qkv, const float* o, const float* dh1, const float* w_out, int B, int K,
                                     int H, int D, const float* relmean, int tk, float scale, uint32_t drop_key,
                                     uint32_t drop_thresh, float drop_scale, const uint32_t* mask, const float* mrow,
                                     const float* lrow, float* dqkv, float* drel_part, void* stream) {
  return attn_bwd_oproj(qkv, nullptr, o, dh1, w_out, B, K, H, D, relmean, tk, scale, drop_key, drop_thresh, drop_scale,
                        mask, mrow, lrow, dqkv, nullptr, drel_part, stream);
}

extern "C" int ctr_attn_bwd_bf_oproj16(const uint16_t* qkv16, const float* o, const float* dh1, const float* w_out, int B,
                                       int K, int H, int D, const float* relmean, int tk, float scale, uint32_t drop_key,
                                       uint32_t drop_thresh, float drop_scale, const uint32_t* mask, const float* mrow,
                                       const float* lrow, uint16_t* dqkv16, float* drel_part, void* stream) {
  CTR_REQUIRE(B == 0 || (qkv16 && dqkv16), "ctr_attn_bwd_bf_oproj16: qkv16 and dqkv16 are required");
  return attn_bwd_oproj(nullptr, (const __bf16*)qkv16, o, dh1, w_out, B, K, H, D, relmean, tk, scale, drop_key,
                        drop_thresh, drop_scale, mask, mrow, lrow, nullptr, (__bf16*)dqkv16, drel_part, stream);
}

extern "C" int ctr_attn_bwd_bf_layer_ok(int K, int H, int D) {
  return (bf_ok(K, H, D) && K <= 64 && D == 32 && (H == 8 || H == 4)) ? 1 : 0;
}

extern "C" int ctr_attn_bwd_bf_layer16(const uint16_t* qkv16, const float* o, const float* dh1, const float* w_out,
                                       const float* w_in, int B, int K, int H, int D, const float* relmean, int tk,
                                       float scale, uint32_t drop_key, uint32_t drop_thresh, float drop_scale,
                                       const uint32_t* mask, const float* mrow, const float* lrow, uint16_t* dqkv16,
                                       float* drel_part, float* dx, void* stream) {
  if (B == 0) return 0;
  CTR_REQUIRE(ctr_attn_bwd_bf_layer_ok(K, H, D), "ctr_attn_bwd_bf_layer16: K <= 64, D = 32, 4 or 8 heads");
  CTR_REQUIRE(qkv16 && dqkv16 && dh1 && w_out && w_in && dx, "ctr_attn_bwd_bf_layer16: null operand");
  CTR_REQUIRE(!relmean || tk >= K - 1, "positional-bias table shorter than K");
  CTR_REQUIRE(!drop_thresh || mask, "attention backward with dropout needs the forward's keep bits");
  AttnBfArgs a{};
  a.B = B; a.K = K; a.H = H; a.D = D; a.G = H; a.ngrp = 1; a.nt = (K + 15) / 16; a.tk = tk;
  a.relmean = relmean; a.scale = scale; a.drop = Drop{drop_key, drop_thresh, drop_scale};
  a.mask = const_cast<uint32_t*>(mask); a.o = const_cast<float*>(o); a.mrow = const_cast<float*>(mrow);
  a.lrow = const_cast<float*>(lrow); a.drel_part = drel_part;
  a.dh1 = dh1; a.w_out = w_out; a.qkv16 = (const __bf16*)qkv16; a.dqkv16 = (__bf16*)dqkv16;
  a.w_in = w_in; a.dx = dx;
  hipStream_t s = (hipStream_t)stream;
  if (D / H == 4) launch_bwd_layer2<4>(a, s);
  else launch_bwd_layer2<8>(a, s);
  return check_launch("attn_bwd_bf_layer16");
}

extern "C" int ctr_attn_layer_fwd_ok(int K, int H, int D) {
  return (K >= 1 && K <= 64 && D == 32 && (H == 8 || H == 4)) ? 1 : 0;
}

static int attn_layer_fwd(const float* x, int B, int K, int H, int D, const float* w_in, const float* b_in,
                          const float* rel_w, float* relmean, int tk, float scale, uint32_t drop_key, uint32_t drop_thresh,
                          float drop_scale, uint32_t* mask, const float* w_out, const float* b_out, const float* nw1,
                          float eps, float* qkv, __bf16* qkv16, float* o, float* mrow, float* lrow, float* h1, float* r1,
                          float* x1, void* stream) {
  if (B == 0) return 0;
  CTR_REQUIRE(ctr_attn_layer_fwd_ok(K, H, D), "ctr_attn_layer_fwd_bf: K <= 64, D = 32, 4 or 8 heads");
  CTR_REQUIRE(!rel_w || (relmean && tk >= K - 1 && tk <= 64),
              "positional bias: needs the relmean output, tk >= K - 1 and tk <= 64");
  CTR_REQUIRE(!drop_thresh || mask, "attention forward with dropout needs a keep-bit buffer");
  LayerFwdArgs L{};
  AttnBfArgs& a = L.at;
  a.qkv = qkv; a.B = B; a.K = K; a.H = H; a.D = D; a.G = H; a.ngrp = 1; a.nt = (K + 15) / 16; a.tk = tk;
  a.relmean = relmean; a.scale = scale; a.drop = Drop{drop_key, drop_thresh, drop_scale};
  a.mask = mask; a.o = o; a.mrow = mrow; a.lrow = lrow;
  L.rel_w = rel_w; L.relmean = relmean;
  L.x = x; L.w_in = w_in; L.b_in = b_in; L.w_out = w_out; L.b_out = b_out; L.nw1 = nw1; L.eps = eps;
  L.qkv = qkv; L.qkv16 = qkv16; L.h1 = h1; L.r1 = r1; L.x1 = x1;
  hipStream_t s = (hipStream_t)stream;
  const int nth = 64 * H;
  const int dk = drop_thresh == 0 ? 0 : (K & 1) ? 2 : 1;
  auto go = [&](auto dh_tag, auto bias_tag) {
    constexpr int DH = decltype(dh_tag)::value;
    constexpr bool BS = decltype(bias_tag)::value;
    if (dk == 0) attn_layer_fwd_kernel<DH, BS, 0><<<B, nth, 0, s>>>(L);
    else if (dk == 1) attn_layer_fwd_kernel<DH, BS, 1><<<B, nth, 0, s>>>(L);
    else attn_layer_fwd_kernel<DH, BS, 2><<<B, nth, 0, s>>>(L);
  };
  using I4 = std::integral_constant<int, 4>;
  using I8 = std::integral_constant<int, 8>;
  using BT = std::true_type;
  using BF = std::false_type;
  if (H == 8) {
    if (rel_w) go(I4{}, BT{}); else go(I4{}, BF{});
  } else {
    if (rel_w) go(I8{}, BT{}); else go(I8{}, BF{});
  }
  return check_launch("attn_layer_fwd_bf");
}

extern "C" int ctr_attn_layer_fwd_bf(const float* x, int B, int K, int H, int D, const float* w_in, const float* b_in,
                                     const float* rel_w, float* relmean, int tk, float scale, uint32_t drop_key, uint32_t drop_thresh,
                                     float drop_scale, uint32_t* mask, const float* w_out, const float* b_out,
                                     const float* nw1, float eps, float* qkv, float* o, float* mrow, float* lrow,
                                     float* h1, float* r1, float* x1, void* stream) {
  return attn_layer_fwd(x, B, K, H, D, w_in, b_in, rel_w, relmean, tk, scale, drop_key, drop_thresh, drop_scale, mask,
                        w_out, b_out, nw1, eps, qkv, nullptr, o, mrow, lrow, h1, r1, x1, stream);
}

extern "C" int ctr_attn_layer_fwd_bf16(const float* x, int B, int K, int H, int D, const float* w_in, const float* b_in,
                                       const float* rel_w, float* relmean, int tk, float scale, uint32_t drop_key,
                                       uint32_t drop_thresh, float drop_scale, uint32_t* mask, const float* w_out,
                                       const float* b_out, const float* nw1, float eps, uint16_t* qkv16, float* o,
                                       float* mrow, float* lrow, float* h1, float* r1, float* x1, void* stream) {
  CTR_REQUIRE(B == 0 || qkv16, "ctr_attn_layer_fwd_bf16: qkv16 is required");
  return attn_layer_fwd(x, B, K, H, D, w_in, b_in, rel_w, relmean, tk, scale, drop_key, drop_thresh, drop_scale, mask,
                        w_out, b_out, nw1, eps, nullptr, (__bf16*)qkv16, o, mrow, lrow, h1, r1, x1, stream);
}

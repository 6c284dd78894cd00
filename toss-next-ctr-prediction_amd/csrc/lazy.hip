// Exact lazy AdamW + EMA for the embedding tables.
//
// The reference steps every element of every table each step (torch.optim.AdamW over dense
// nn.Embedding grads, src/train.py:195; ModelEMA.update, src/utils/ema.py:92-131): with 1.24 B
// table elements that is ~40 GB of HBM traffic per step although a batch touches well under 1% of
// the rows.  Here a row is only brought up to date when something needs it:
//   * ctr_lazy_touch   -- rows a batch reads in the forward (hashed categoricals, sequence tokens),
//   * ctr_lazy_update  -- rows that receive a gradient this tick (replay, then the real tick),
//   * ctr_lazy_flush   -- all rows, before parameters / moments / EMA are read as a whole.
// "Brought up to date" = the ticks the row missed are replayed from the device tick history with
// grad 0, through the same adam.h arithmetic as the dense stream, so the result is bit-identical to
// stepping the row densely every tick (tests/test_gpu_lazy.py checks that bitwise).
//
// Work mapping: a group of lg lanes per row; lane l holds elements l, l+lg, ... (<= 8 per lane, rows
// are <= 64 wide) in registers across the whole replay, the tick loop wave-uniform (one scalar load of
// a tick's history entry per wave), and the row's p, m, v, ema read and written once.
//
// Row state word last[row]: bits 0..30 the last tick applied, bit 31 (LAST_NZ) set once the row has
// taken a gradient tick.  A row without it has zero moments (fresh optimizer state; idle ticks keep
// them +0), so its replay reads and writes only p and the EMA shadow -- half the bytes of a stepped
// row.  At the benchmark config over 90 % of the categorical rows are in that state at a flush.
#include "adam.h"
#include "common.h"
#include "ctr_hip.h"

namespace ctr {

constexpr int LQ = 8;           // row elements held per lane (rows are <= 64 wide)
constexpr int LG = 8;           // lanes per row in touch / update (any table width)
constexpr int FLUSH_MAXTABS = 64;
constexpr uint32_t LAZY_INVALID = 0xFFFFFFFFu;
constexpr int LAST_NZ = (int)0x80000000u;
__device__ __forceinline__ int ltick(int w) { return w & 0x7FFFFFFF; }

__global__ void opt_hist_record_kernel(OptScalars* hist, int tick, OptScalars s) { hist[tick] = s; }

typedef float f32x4 __attribute__((ext_vector_type(4)));

// Ticks k0..k1 of the history, four per step: the four entries' scalar loads go out together (one wait)
// and the loop overhead is paid once per four ticks; f(sc, k) applies one tick.
template <class F>
__device__ __forceinline__ void for_ticks(const OptScalars* __restrict__ hist, int k0, int k1, F&& f) {
  int k = k0;
  for (; k + 3 <= k1; k += 4) {
    const OptScalars* h = hist + k;
    const OptScalars a = h[0], b = h[1], c = h[2], d = h[3];
    f(a, k);
    f(b, k + 1);
    f(c, k + 2);
    f(d, k + 3);
  }
  for (; k <= k1; ++k) f(hist[k], k);
}

// Brings rows from their last tick s to tick t_idle with grad 0, then (grow != null) applies tick
// t_idle+1 with grad grow*coef.  A row is spread over lg lanes.  Element of register slot q in lane l:
//   strided (any width):          j = l + lg*q, q < nq
//   contiguous (width % 8 == 0):  j = 8l + q   -- two 16-byte loads / stores per array per lane
// Every lane of the wave takes part (dead lanes: live = false) and the tick loop runs over the
// wave-uniform range (min over the wave's rows of s, t_idle], each tick's scalars one scalar load; a lane
// applies tick k only when k > its own s (exec-masked).  (A per-lane form that walked each row's own
// range with a per-lane history load every tick was bound on that load, and a wave holding both
// zero-moment and stepped rows ran both loops.)
// A row whose moments are all zero (never stepped with a non-zero grad) stays zero under idle ticks:
// only the decay multiply and the EMA remain.  With m == v == 0, adam_elem(g = 0) gives m = v = +0,
// denom = eps and p = fmaf(-step, +0, p * decay) == p * decay: bit for bit the same -- so a wave with
// any stepped row runs the full idle-tick arithmetic on all its rows, and an all-zero wave the short form.
template <bool VEC>
__device__ __forceinline__ void replay_rows_wave(float* __restrict__ p_row, float* __restrict__ m_row,
                                                 float* __restrict__ v_row, float* __restrict__ e_row, int width,
                                                 int l, int lg, int nq, bool live, int s, bool nzr,
                                                 const OptScalars* __restrict__ hist, int t_idle,
                                                 const float* __restrict__ grow = nullptr, float coef = 1.0f) {
  float p[LQ], m[LQ], v[LQ], e[LQ];
  const bool vlane = live && (!VEC || 8 * l < width);
#pragma unroll
  for (int q = 0; q < LQ; ++q) p[q] = m[q] = v[q] = e[q] = 0.0f;
  if (VEC) {
    if (vlane) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const f32x4 z4 = {0.f, 0.f, 0.f, 0.f};
        const f32x4 pv = *(const f32x4*)(p_row + 8 * l + 4 * h);
        const f32x4 mv = nzr ? *(const f32x4*)(m_row + 8 * l + 4 * h) : z4;
        const f32x4 vv = nzr ? *(const f32x4*)(v_row + 8 * l + 4 * h) : z4;
        const f32x4 ev = e_row ? *(const f32x4*)(e_row + 8 * l + 4 * h) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          p[4 * h + t] = pv[t];
          m[4 * h + t] = mv[t];
          v[4 * h + t] = vv[t];
          e[4 * h + t] = ev[t];
        }
      }
    }
    nq = LQ;
  } else if (live) {
#pragma unroll
    for (int q = 0; q < LQ; ++q) {
      const int j = l + lg * q;
      if (q < nq && j < width) {
        p[q] = p_row[j];
        if (nzr) {
          m[q] = m_row[j];
          v[q] = v_row[j];
        }
        if (e_row) e[q] = e_row[j];
      }
    }
  }
  bool zero = true;
#pragma unroll
  for (int q = 0; q < LQ; ++q) zero = zero && m[q] == 0.0f && v[q] == 0.0f;
  const bool any_stepped = __ballot(!zero) != 0ull;
  if (!live) s = t_idle;
  int smin = s;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) smin = min(smin, __shfl_xor(smin, o));
  smin = __builtin_amdgcn_readfirstlane(smin);
  if (smin >= t_idle && grow == nullptr) return;
  if (smin >= t_idle) {
    // nothing to replay (the gradient tick below only)
  } else if (!any_stepped) {
    bool stepped = false;
    for_ticks(hist, smin + 1, t_idle, [&](const OptScalars& sc, int k) {
      if (k > s) {
        if (sc.do_adam) {
          stepped = true;
#pragma unroll
          for (int q = 0; q < LQ; ++q)
            if (q < nq) p[q] = p[q] * sc.decay_mul;
        }
        if (sc.do_ema) {
#pragma unroll
          for (int q = 0; q < LQ; ++q)
            if (q < nq) ema_elem(sc, p[q], e[q]);
        }
      }
    });
    if (stepped) {
#pragma unroll
      for (int q = 0; q < LQ; ++q) m[q] = v[q] = 0.0f;    // a dense idle tick leaves +0 moments
    }
  } else {
    // element pairs (q, q+1) in packed f32 (slots past nq hold zeros and are never stored)
    f32x2 pp[LQ / 2], mm[LQ / 2], vv[LQ / 2], ee[LQ / 2];
#pragma unroll
    for (int h = 0; h < LQ / 2; ++h) {
      pp[h] = f32x2{p[2 * h], p[2 * h + 1]};
      mm[h] = f32x2{m[2 * h], m[2 * h + 1]};
      vv[h] = f32x2{v[2 * h], v[2 * h + 1]};
      ee[h] = f32x2{e[2 * h], e[2 * h + 1]};
    }
    for_ticks(hist, smin + 1, t_idle, [&](const OptScalars& sc, int k) {
      if (k > s) {
#pragma unroll
        for (int h = 0; h < LQ / 2; ++h) {
          if (2 * h < nq) {
            if (sc.do_adam) idle_adam_pk(sc, pp[h], mm[h], vv[h]);
            if (sc.do_ema) ema_pk(sc, pp[h], ee[h]);
          }
        }
      }
    });
#pragma unroll
    for (int h = 0; h < LQ / 2; ++h) {
      p[2 * h] = pp[h].x;
      p[2 * h + 1] = pp[h].y;
      m[2 * h] = mm[h].x;
      m[2 * h + 1] = mm[h].y;
      v[2 * h] = vv[h].x;
      v[2 * h + 1] = vv[h].y;
      e[2 * h] = ee[h].x;
      e[2 * h + 1] = ee[h].y;
    }
  }
  if (grow) {
    const OptScalars sc = hist[t_idle + 1];
#pragma unroll
    for (int q = 0; q < LQ; ++q) {
      const int j = VEC ? 8 * l + q : l + lg * q;
      const bool lv = VEC ? vlane : (live && q < nq && j < width);
      if (lv) adam_ema_elem(sc, p[q], m[q], v[q], e[q], grow[j] * coef, sc.do_adam != 0);
    }
  } else if (s >= t_idle) {
    return;
  }
  // moments of a row without a gradient tick stay the +0 already in memory
  const bool st_mv = nzr || grow != nullptr;
  if (VEC) {
    if (vlane) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        *(f32x4*)(p_row + 8 * l + 4 * h) = f32x4{p[4 * h], p[4 * h + 1], p[4 * h + 2], p[4 * h + 3]};
        if (st_mv) {
          *(f32x4*)(m_row + 8 * l + 4 * h) = f32x4{m[4 * h], m[4 * h + 1], m[4 * h + 2], m[4 * h + 3]};
          *(f32x4*)(v_row + 8 * l + 4 * h) = f32x4{v[4 * h], v[4 * h + 1], v[4 * h + 2], v[4 * h + 3]};
        }
        if (e_row) *(f32x4*)(e_row + 8 * l + 4 * h) = f32x4{e[4 * h], e[4 * h + 1], e[4 * h + 2], e[4 * h + 3]};
      }
    }
  } else if (live) {
#pragma unroll
    for (int q = 0; q < LQ; ++q) {
      const int j = l + lg * q;
      if (q < nq && j < width) {
        p_row[j] = p[q];
        if (st_mv) {
          m_row[j] = m[q];
          v_row[j] = v[q];
        }
        if (e_row) e_row[j] = e[q];
      }
    }
  }
}

struct RowPtrs {
  float *p, *m, *v, *e;
};

__device__ __forceinline__ RowPtrs row_ptrs(const ctr_lazy_tab_t& tb, long row, float* P, float* M, float* V,
                                            float* E) {
  const long o = tb.p_off + row * (long)tb.width;
  return {P + o, M + o, V + o, E ? E + o : nullptr};
}

// One 8-lane group per (id, table) item.  The group leader claims the row with a CAS on last[row]
// (s -> tick); only the winner replays, so a row read many times in a batch is caught up once.
// STAGED (ntabs <= FLUSH_MAXTABS): the table descriptors are copied to LDS first -- the key -> table binary search
// and the descriptor reads were a chain of dependent global loads ahead of every row's own loads
template <bool STAGED>
__global__ __launch_bounds__(256) void lazy_touch_kernel(const ctr_lazy_tab_t* __restrict__ gtabs, int ntabs,
                                                         const int32_t* __restrict__ X, long nitems, int ncols,
                                                         int per_column, float* P, float* M, float* V, float* E,
                                                         const OptScalars* __restrict__ hist, int tick) {
  __shared__ ctr_lazy_tab_t stabs[STAGED ? FLUSH_MAXTABS : 1];
  if (STAGED) {
    for (int i = threadIdx.x; i < ntabs; i += 256) stabs[i] = gtabs[i];
    __syncthreads();
  }
  const ctr_lazy_tab_t* tabs = STAGED ? stabs : gtabs;
  const long item = (blockIdx.x * 256L + threadIdx.x) / LG;
  const int l8 = threadIdx.x & (LG - 1);
  int s = tick, win = 0, ti = 0, nz = 0;
  long row = -1;
  if (item < nitems) {
    long xi;
    if (per_column == 1) {
      xi = item;
      ti = (int)(item % ncols);
    } else if (per_column == 2) {
      xi = item;
    } else {
      xi = item / ntabs;
      ti = (int)(item % ntabs);
    }
    row = X[xi];
    if (per_column == 2 && row >= 0) {   // X holds keys: the last table with key_base <= key
      int a = 0, b = ntabs;
      while (b - a > 1) {
        const int mid = (a + b) >> 1;
        if (tabs[mid].key_base <= (uint32_t)row) a = mid; else b = mid;
      }
      ti = a;
      row -= (long)tabs[a].key_base;
    }
  }
  if (item < nitems && l8 == 0 && row >= 0 && row < tabs[ti].rows) {
    int* lp = tabs[ti].last + row;
    const int w = __hip_atomic_load(lp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s = ltick(w);
    nz = w & LAST_NZ;
    if (s < tick) win = atomicCAS(lp, w, tick | nz) == w;
  }
  const int leader = (threadIdx.x & 63) & ~(LG - 1);
  win = __shfl(win, leader);
  s = __shfl(s, leader);
  nz = __shfl(nz, leader);
  const ctr_lazy_tab_t tb = tabs[win ? ti : 0];
  const RowPtrs r = row_ptrs(tb, win ? row : 0, P, M, V, E);
  replay_rows_wave<false>(r.p, r.m, r.v, r.e, tb.width, l8, LG, cdiv(tb.width, LG), win != 0, s, nz != 0, hist,
                          tick);
}

// One 8-lane group per compact grad slot: keys are unique, so no claim is needed.
template <bool STAGED>
__global__ __launch_bounds__(256) void lazy_update_kernel(const ctr_lazy_tab_t* __restrict__ gtabs, int ntabs,
                                                          const uint32_t* __restrict__ keys,
                                                          const float* __restrict__ G, int g_ld,
                                                          const uint32_t* __restrict__ n_uniq, long cap,
                                                          const float* __restrict__ coef_ptr, float* P, float* M,
                                                          float* V, float* E, const OptScalars* __restrict__ hist,
                                                          int tick) {
  __shared__ ctr_lazy_tab_t stabs[STAGED ? FLUSH_MAXTABS : 1];
  const long item = (blockIdx.x * 256L + threadIdx.x) / LG;
  const int l8 = threadIdx.x & (LG - 1);
  // the slot's key and the unique count load side by side (the key was loaded after the count)
  uint32_t key = item < cap ? keys[item] : LAZY_INVALID;
  const long nu = min(cap, (long)*n_uniq);
  if (STAGED) {
    for (int i = threadIdx.x; i < ntabs; i += 256) stabs[i] = gtabs[i];
    __syncthreads();
  }
  const ctr_lazy_tab_t* tabs = STAGED ? stabs : gtabs;
  bool live = item < nu && key != LAZY_INVALID;
  if (!live) key = LAZY_INVALID;
  int a = 0;
  long row = 0;
  int s = tick - 1, w = 0;
  if (live) {
    int b = ntabs;   // last table with key_base <= key
    while (b - a > 1) {
      const int mid = (a + b) >> 1;
      if (tabs[mid].key_base <= key) a = mid; else b = mid;
    }
    row = (long)(key - tabs[a].key_base);
    live = row < tabs[a].rows;
    if (live) {
      w = tabs[a].last[row];
      s = ltick(w);
    }
  }
  const ctr_lazy_tab_t tb = tabs[live ? a : 0];
  const RowPtrs r = row_ptrs(tb, live ? row : 0, P, M, V, E);
  const float coef = coef_ptr ? *coef_ptr : 1.0f;
  replay_rows_wave<false>(r.p, r.m, r.v, r.e, tb.width, l8, LG, cdiv(tb.width, LG), live, s, (w & LAST_NZ) != 0,
                          hist, tick - 1, G + (live ? item : 0) * (long)g_ld, coef);
  if (live && l8 == 0) tb.last[row] = tick | LAST_NZ;
}

// ------------------------------------------------------------------------------------------------
// DARE table pair (emb_att, emb_rep): both are read for the same tokens and get gradients for the
// same keys, so a token's att row and rep row always share their last-applied tick.  One WAVE per
// token: lanes [0, W) hold the att row's elements, [W, 2W) the rep row's (2 per lane when W = 64),
// so every lane replays the same tick range -- no divergence between row groups -- and each tick's
// scalars are a wave-uniform (scalar) load.

// EPL = elements per lane: 1 for W <= 32 (no dead lane slot replayed), 2 for W <= 64
template <int EPL>
struct PairRow {
  float p[EPL], m[EPL], v[EPL], e[EPL];
  long o[EPL];             // arena offsets; -1 = lane slot unused
};

template <int EPL>
__device__ __forceinline__ void pair_load(PairRow<EPL>& r, const ctr_lazy_tab_t& ta, const ctr_lazy_tab_t& tb, long row,
                                          const float* P, const float* M, const float* V, const float* E, bool nz) {
  const int W = ta.width, lane = threadIdx.x & 63;
#pragma unroll
  for (int q = 0; q < EPL; ++q) {
    const int el = lane + 64 * q;
    r.o[q] = el < W ? ta.p_off + row * W + el : el < 2 * W ? tb.p_off + row * W + (el - W) : -1;
    r.p[q] = r.m[q] = r.v[q] = r.e[q] = 0.f;
    if (r.o[q] >= 0) {
      r.p[q] = P[r.o[q]];
      if (nz) {     // moments of a row without a gradient tick are +0
        r.m[q] = M[r.o[q]];
        r.v[q] = V[r.o[q]];
      }
      if (E) r.e[q] = E[r.o[q]];
    }
  }
}

template <int EPL>
__device__ __forceinline__ void pair_store(const PairRow<EPL>& r, float* P, float* M, float* V, float* E, bool st_mv) {
#pragma unroll
  for (int q = 0; q < EPL; ++q)
    if (r.o[q] >= 0) {
      P[r.o[q]] = r.p[q];
      if (st_mv) {
        M[r.o[q]] = r.m[q];
        V[r.o[q]] = r.v[q];
      }
      if (E) E[r.o[q]] = r.e[q];
    }
}

// ticks (s, t_idle] with grad 0, then (g != null) tick t_idle + 1 with grad g[q] * coef; same
// arithmetic as replay_rows_wave (adam.h), decided per wave (s and the zero test are wave-uniform)
template <int EPL>
__device__ __forceinline__ void pair_replay(PairRow<EPL>& r, bool has_e, const OptScalars* __restrict__ hist, int s,
                                            int t_idle, const float* g, float coef) {
  bool nz = false;
#pragma unroll
  for (int q = 0; q < EPL; ++q) nz = nz || r.m[q] != 0.0f || r.v[q] != 0.0f;
  const bool zero = __ballot(nz) == 0;      // every element of both rows never stepped with a grad
  if (zero) {
    bool stepped = false;
    for_ticks(hist, s + 1, t_idle, [&](const OptScalars& sc, int) {
      if (sc.do_adam) {
        stepped = true;
#pragma unroll
        for (int q = 0; q < EPL; ++q) r.p[q] = r.p[q] * sc.decay_mul;
      }
      if (sc.do_ema) {
#pragma unroll
        for (int q = 0; q < EPL; ++q) ema_elem(sc, r.p[q], r.e[q]);
      }
    });
    if (stepped) {
#pragma unroll
      for (int q = 0; q < EPL; ++q) r.m[q] = r.v[q] = 0.0f;
    }
  } else {
    for_ticks(hist, s + 1, t_idle, [&](const OptScalars& sc, int) {
#pragma unroll
      for (int q = 0; q < EPL; ++q) {
        if (sc.do_adam) idle_adam_elem(sc, r.p[q], r.m[q], r.v[q]);
        if (sc.do_ema) ema_elem(sc, r.p[q], r.e[q]);
      }
    });
  }
  if (g) {
    const OptScalars sc = hist[t_idle + 1];
#pragma unroll
    for (int q = 0; q < EPL; ++q)
      if (r.o[q] >= 0) adam_ema_elem(sc, r.p[q], r.m[q], r.v[q], r.e[q], g[q] * coef, sc.do_adam != 0);
  }
  (void)has_e;
}

// The pair kernels take NT tokens per wave iteration: the NT claims / tick reads go out together (lane u
// handles token u), then all NT rows' loads, then the NT replays, then the stores -- one memory latency per
// NT rows instead of one per row (a wave per token was latency-bound on the CAS -> load -> store chain).
constexpr int PAIR_NT = 4;

// forward read of tokens X[0, n): lane u of a wave claims token u's att-row tick with a CAS (a token read
// many times in the batch is caught up once) and the rep row's tick follows it
template <int EPL>
__global__ __launch_bounds__(256) void lazy_touch_pair_kernel(const ctr_lazy_tab_t* __restrict__ tabs,
                                                              const int32_t* __restrict__ X, long n, float* P,
                                                              float* M, float* V, float* E,
                                                              const OptScalars* __restrict__ hist, int tick) {
  const ctr_lazy_tab_t ta = tabs[0], tb = tabs[1];
  const long wave = (blockIdx.x * 256L + threadIdx.x) >> 6, nwaves = (long)gridDim.x * 4;
  const int lane = threadIdx.x & 63;
  for (long t0 = wave * PAIR_NT; t0 < n; t0 += nwaves * PAIR_NT) {
    int my_row = -1, my_s = tick, my_nz = 0;
    if (lane < PAIR_NT && t0 + lane < n) {
      const long row = X[t0 + lane];
      // a token equal to its predecessor's is that position's job: runs of one token (the left padding of
      // every sequence: ~half the batch is the pad row) claim once instead of hammering one tick word
      const bool dup = t0 + lane > 0 && X[t0 + lane - 1] == row;
      if (!dup && row >= 0 && row < ta.rows) {
        int* lp = ta.last + row;
        const int w = __hip_atomic_load(lp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (ltick(w) < tick && atomicCAS(lp, w, tick | (w & LAST_NZ)) == w) {
          my_row = (int)row;
          my_s = ltick(w);
          my_nz = w & LAST_NZ;
        }
      }
    }
    int rows[PAIR_NT], ss[PAIR_NT], nzs[PAIR_NT];
    PairRow<EPL> r[PAIR_NT];
#pragma unroll
    for (int u = 0; u < PAIR_NT; ++u) {
      rows[u] = __builtin_amdgcn_readlane(my_row, u);
      ss[u] = __builtin_amdgcn_readlane(my_s, u);
      nzs[u] = __builtin_amdgcn_readlane(my_nz, u);
      if (rows[u] >= 0) pair_load(r[u], ta, tb, rows[u], P, M, V, E, nzs[u] != 0);
    }
#pragma unroll
    for (int u = 0; u < PAIR_NT; ++u)
      if (rows[u] >= 0) pair_replay(r[u], E != nullptr, hist, ss[u], tick, nullptr, 0.f);
#pragma unroll
    for (int u = 0; u < PAIR_NT; ++u)
      if (rows[u] >= 0) {
        pair_store(r[u], P, M, V, E, nzs[u] != 0);
        if (lane == 0) tb.last[rows[u]] = tick | nzs[u];
      }
  }
}

// one optimizer tick for the unique keys [0, *n_uniq) shared by the att grads Ga and the rep grads Gb
template <int EPL>
__global__ __launch_bounds__(256) void lazy_update_pair_kernel(const ctr_lazy_tab_t* __restrict__ tabs,
                                                               const uint32_t* __restrict__ keys,
                                                               const float* __restrict__ Ga,
                                                               const float* __restrict__ Gb, int g_ld,
                                                               const uint32_t* __restrict__ n_uniq, long cap,
                                                               const float* __restrict__ coef_ptr, float* P,
                                                               float* M, float* V, float* E,
                                                               const OptScalars* __restrict__ hist, int tick) {
  const ctr_lazy_tab_t ta = tabs[0], tb = tabs[1];
  const long wave = (blockIdx.x * 256L + threadIdx.x) >> 6, nwaves = (long)gridDim.x * 4;
  const int lane = threadIdx.x & 63, W = ta.width;
  const long nu = min(cap, (long)*n_uniq);
  const float coef = coef_ptr ? *coef_ptr : 1.0f;
  for (long it0 = wave * PAIR_NT; it0 < nu; it0 += nwaves * PAIR_NT) {
    int my_row = -1, my_s = 0;
    if (lane < PAIR_NT && it0 + lane < nu) {
      const uint32_t key = keys[it0 + lane];
      if (key != LAZY_INVALID && (long)(key - ta.key_base) < ta.rows) {
        my_row = (int)(key - ta.key_base);
        my_s = ta.last[my_row];       // state word: tick and LAST_NZ
      }
    }
    int rows[PAIR_NT], ss[PAIR_NT];
    PairRow<EPL> r[PAIR_NT];
    float g[PAIR_NT][EPL];
#pragma unroll
    for (int u = 0; u < PAIR_NT; ++u) {
      rows[u] = __builtin_amdgcn_readlane(my_row, u);
      ss[u] = __builtin_amdgcn_readlane(my_s, u);
      if (rows[u] >= 0) {
        pair_load(r[u], ta, tb, rows[u], P, M, V, E, (ss[u] & LAST_NZ) != 0);
        ss[u] = ltick(ss[u]);
        const long it = it0 + u;
#pragma unroll
        for (int q = 0; q < EPL; ++q) {
          const int el = lane + 64 * q;
          g[u][q] = el < W ? Ga[it * (long)g_ld + el] : el < 2 * W ? Gb[it * (long)g_ld + (el - W)] : 0.f;
        }
      }
    }
#pragma unroll
    for (int u = 0; u < PAIR_NT; ++u)
      if (rows[u] >= 0) pair_replay(r[u], E != nullptr, hist, ss[u], tick - 1, g[u], coef);
#pragma unroll
    for (int u = 0; u < PAIR_NT; ++u)
      if (rows[u] >= 0) {
        pair_store(r[u], P, M, V, E, true);
        if (lane == 0) {
          ta.last[rows[u]] = tick | LAST_NZ;
          tb.last[rows[u]] = tick | LAST_NZ;
        }
      }
  }
}

// every row pair not yet at tick (flush of the DARE tables)
template <int EPL>
__global__ __launch_bounds__(256) void lazy_flush_pair_kernel(const ctr_lazy_tab_t* __restrict__ tabs, float* P,
                                                              float* M, float* V, float* E,
                                                              const OptScalars* __restrict__ hist, int tick) {
  const ctr_lazy_tab_t ta = tabs[0], tb = tabs[1];
  const long wave = (blockIdx.x * 256L + threadIdx.x) >> 6, nwaves = (long)gridDim.x * 4;
  const int lane = threadIdx.x & 63;
  for (long r0 = wave * PAIR_NT; r0 < ta.rows; r0 += nwaves * PAIR_NT) {
    int my_w = tick;
    if (lane < PAIR_NT && r0 + lane < ta.rows) my_w = ta.last[r0 + lane];
    int ss[PAIR_NT], nzs[PAIR_NT];
    PairRow<EPL> r[PAIR_NT];
#pragma unroll
    for (int u = 0; u < PAIR_NT; ++u) {
      const int w = __builtin_amdgcn_readlane(my_w, u);
      ss[u] = ltick(w);
      nzs[u] = w & LAST_NZ;
      if (ss[u] < tick) pair_load(r[u], ta, tb, r0 + u, P, M, V, E, nzs[u] != 0);
    }
#pragma unroll
    for (int u = 0; u < PAIR_NT; ++u)
      if (ss[u] < tick) pair_replay(r[u], E != nullptr, hist, ss[u], tick, nullptr, 0.f);
#pragma unroll
    for (int u = 0; u < PAIR_NT; ++u)
      if (ss[u] < tick) {
        pair_store(r[u], P, M, V, E, nzs[u] != 0);
        if (lane == 0) {
          ta.last[r0 + u] = tick | nzs[u];
          tb.last[r0 + u] = tick | nzs[u];
        }
      }
  }
}

// Classified replay of DARE table-pair rows (W % 4 == 0, 128 % W == 0).  The rows to bring current sit in a
// zero-moment and a stepped list in LDS (absolute row, last tick); each wave replays list entries in groups
// of 2 x (128 / W) row pairs: W / 4 lanes hold a table row (a float4 each, element pairs in packed f32), one
// tick loop for the whole group, a lane applying tick k only past its own row's tick.  A wave's rows all take
// the short (zero-moment: decay + EMA) or all the full replay, and the per-tick scalar work (history loads,
// flag branches) is shared by 2 x (128 / W) row pairs instead of being paid per pair: the one-wave-per-pair
// kernels spent ~0.17 ms per replayed tick of a cfg2 flush whatever the rows' class.  Same adam.h arithmetic
// per element (packed halves are the same IEEE operations): bit-identical to the dense stream.  List order is
// arbitrary; rows are independent.  Rows end at `tick`; both tables' state words are written when write_a,
// else only the rep table's (the att word was claimed by CAS).
template <int W, int CL>
__device__ __forceinline__ void replay_pair_list(const ctr_lazy_tab_t& ta, const ctr_lazy_tab_t& tb,
                                                 const int* lrow, const int* ls, int n, float* P, float* M,
                                                 float* V, float* E, const OptScalars* __restrict__ hist, int tick,
                                                 bool write_a) {
  constexpr int LPT = W / 4;               // lanes per table row
  constexpr int LPP = 2 * LPT;             // lanes per row pair
  constexpr int PPS = 64 / LPP;            // row pairs per slot
#ifndef PAIR_NS0
#define PAIR_NS0 4
#endif
#ifndef PAIR_NS1
#define PAIR_NS1 2
#endif
  constexpr int NS = CL ? PAIR_NS1 : PAIR_NS0;   // slots per lane
  constexpr int GRP = PPS * NS;            // row pairs per wave group
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int u = lane / LPP, c = lane % LPP;
  const bool is_b = c >= LPT;
  const long tab_off = is_b ? tb.p_off : ta.p_off;
  const int e0 = 4 * (is_b ? c - LPT : c);
  for (int g0 = wv * GRP; g0 < n; g0 += nw * GRP) {
    long off[NS], row[NS];
    int s[NS];
    bool live[NS];
    f32x2 p[NS][2], m[NS][2], v[NS][2], e[NS][2];
    int smin = tick;
#pragma unroll
    for (int q = 0; q < NS; ++q) {
      const int idx = g0 + q * PPS + u;
      live[q] = idx < n;
      row[q] = live[q] ? lrow[idx] : 0;
      s[q] = live[q] ? ls[idx] : tick;
      off[q] = tab_off + row[q] * W + e0;
      const f32x4 z4 = {0.f, 0.f, 0.f, 0.f};
      f32x4 pv = z4, mv = z4, vv = z4, ev = z4;
      if (live[q]) {
        pv = *(const f32x4*)(P + off[q]);
        if (CL) {
          mv = *(const f32x4*)(M + off[q]);
          vv = *(const f32x4*)(V + off[q]);
        }
        if (E) ev = *(const f32x4*)(E + off[q]);
      }
      p[q][0] = f32x2{pv[0], pv[1]}; p[q][1] = f32x2{pv[2], pv[3]};
      m[q][0] = f32x2{mv[0], mv[1]}; m[q][1] = f32x2{mv[2], mv[3]};
      v[q][0] = f32x2{vv[0], vv[1]}; v[q][1] = f32x2{vv[2], vv[3]};
      e[q][0] = f32x2{ev[0], ev[1]}; e[q][1] = f32x2{ev[2], ev[3]};
      smin = min(smin, s[q]);
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) smin = min(smin, __shfl_xor(smin, o));
    smin = __builtin_amdgcn_readfirstlane(smin);
    for_ticks(hist, smin + 1, tick, [&](const OptScalars& sc, int k) {
#pragma unroll
      for (int q = 0; q < NS; ++q) {
        if (k > s[q]) {
          if (sc.do_adam) {
            if (CL) {
              idle_adam_pk(sc, p[q][0], m[q][0], v[q][0]);
              idle_adam_pk(sc, p[q][1], m[q][1], v[q][1]);
            } else {
              p[q][0] = p[q][0] * splat2(sc.decay_mul);
              p[q][1] = p[q][1] * splat2(sc.decay_mul);
            }
          }
          if (sc.do_ema) {
            ema_pk(sc, p[q][0], e[q][0]);
            ema_pk(sc, p[q][1], e[q][1]);
          }
        }
      }
    });
#pragma unroll
    for (int q = 0; q < NS; ++q) {
      if (!live[q]) continue;
      *(f32x4*)(P + off[q]) = f32x4{p[q][0].x, p[q][0].y, p[q][1].x, p[q][1].y};
      if (CL) {
        *(f32x4*)(M + off[q]) = f32x4{m[q][0].x, m[q][0].y, m[q][1].x, m[q][1].y};
        *(f32x4*)(V + off[q]) = f32x4{v[q][0].x, v[q][0].y, v[q][1].x, v[q][1].y};
      }
      if (E) *(f32x4*)(E + off[q]) = f32x4{e[q][0].x, e[q][0].y, e[q][1].x, e[q][1].y};
      if (c == 0) {
        if (write_a) ta.last[row[q]] = tick | (CL ? LAST_NZ : 0);
        tb.last[row[q]] = tick | (CL ? LAST_NZ : 0);
      }
    }
  }
}

constexpr int CLS_CH = 1024;     // rows per workgroup iteration of the flush
// token positions per workgroup of the touch: its claims (a load and a CAS per position) and its row gathers
// are dependent memory round trips, so many small workgroups beat few large ones (one of 1024 positions per
// workgroup: 400 workgroups at cfg2, 141 us; 256: 1600 workgroups)
constexpr int TOUCH_CH = 256;

// flush of the DARE table pair: a workgroup sorts CLS_CH consecutive row pairs behind `tick` into a zero-moment
// and a stepped list (CL < 0) and replays both, or lists only class CL (one kernel per class, as
// lazy_flush_cls_kernel: the zero-moment pass at the short replay's register count)
template <int W, int CL>
__global__ __launch_bounds__(256) void lazy_flush_pair_cls_kernel(const ctr_lazy_tab_t* __restrict__ tabs, float* P,
                                                                  float* M, float* V, float* E,
                                                                  const OptScalars* __restrict__ hist, int tick) {
  constexpr int NL = CL < 0 ? 2 : 1;
  __shared__ int lrow[NL][CLS_CH];
  __shared__ int ls[NL][CLS_CH];
  __shared__ int cnt[NL];
  const ctr_lazy_tab_t ta = tabs[0], tb = tabs[1];
  const int tid = threadIdx.x;
  const long rows = ta.rows;
  const long step = (long)gridDim.x * CLS_CH;
  // the state words of a chunk are loaded while the previous chunk replays (a memory round trip per chunk
  // otherwise sat between the list barriers with nothing else in flight)
  int wv[CLS_CH / 256];
  auto load_words = [&](long r0) {
#pragma unroll
    for (int q = 0; q < CLS_CH / 256; ++q) {
      const long r = r0 + tid + 256 * q;
      wv[q] = r < rows ? ta.last[r] : tick;
    }
  };
  load_words((long)blockIdx.x * CLS_CH);
  for (long r0 = (long)blockIdx.x * CLS_CH; r0 < rows; r0 += step) {
    if (tid < NL) cnt[tid] = 0;
    __syncthreads();
#pragma unroll
    for (int q = 0; q < CLS_CH / 256; ++q) {
      const int st = ltick(wv[q]);
      const int cl = (wv[q] & LAST_NZ) ? 1 : 0;
      if (st < tick && (CL < 0 || cl == CL)) {
        const int li = CL < 0 ? cl : 0;
        const int pos = atomicAdd(&cnt[li], 1);
        lrow[li][pos] = (int)(r0 + tid + 256 * q);
        ls[li][pos] = st;
      }
    }
    __syncthreads();
    if (r0 + step < rows) load_words(r0 + step);
    if (CL <= 0) replay_pair_list<W, 0>(ta, tb, lrow[0], ls[0], cnt[0], P, M, V, E, hist, tick, true);
    if (CL != 0) replay_pair_list<W, 1>(ta, tb, lrow[NL - 1], ls[NL - 1], cnt[NL - 1], P, M, V, E, hist, tick, true);
    __syncthreads();      // the lists are refilled by the next iteration
  }
}

// ------------------------------------------------------------------------------------------------
// Classified flush of the categorical tables (any width <= 64): the pair kernel's scheme for one table
// at a time.  A workgroup iteration takes CLS_CH consecutive rows of one table (the chunk grid is
// table-major), lists those behind `tick` of its class in LDS (one state-word load per row, four in flight
// per thread), and the waves replay the list in groups: LPR lanes hold a row, four elements each (float4
// when the table's rows are 16-byte aligned, else elements c + LPR t), NS rows per lane -- 64 / LPR x NS
// rows per group, one wave-uniform tick loop, a lane applying tick k only past its row's own tick.  (The
// per-row-group kernel before it, lazy_flush_kernel, sorted 256 / lg rows per iteration and replayed one row
// per lane group: two barriers and two memory round trips per 64 rows.)  Same adam.h arithmetic per element
// as every other replay: bit-identical to the dense stream.
template <int LPR, bool VEC, int CL, int NS>
__device__ __forceinline__ void replay_tab_list(const ctr_lazy_tab_t& tb, const int* lrow, const int* ls, int n,
                                                float* P, float* M, float* V, float* E,
                                                const OptScalars* __restrict__ hist, int tick) {
  constexpr int RPS = 64 / LPR;            // rows per slot
  constexpr int GRP = RPS * NS;            // rows per wave group
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int u = lane / LPR, c = lane % LPR;
  const int W = tb.width;
  for (int g0 = wv * GRP; g0 < n; g0 += nw * GRP) {
    long base[NS];
    int row[NS], s[NS];
    bool live[NS];
    f32x2 p[NS][2], m[NS][2], v[NS][2], e[NS][2];
    int smin = tick;
#pragma unroll
    for (int q = 0; q < NS; ++q) {
      const int idx = g0 + q * RPS + u;
      live[q] = idx < n;
      row[q] = live[q] ? lrow[idx] : 0;
      s[q] = live[q] ? ls[idx] : tick;
      base[q] = tb.p_off + (long)row[q] * W;
      float pv[4] = {0.f, 0.f, 0.f, 0.f}, mv[4] = {0.f, 0.f, 0.f, 0.f}, vv[4] = {0.f, 0.f, 0.f, 0.f},
            ev[4] = {0.f, 0.f, 0.f, 0.f};
      if (VEC) {
        if (live[q] && 4 * c < W) {
          const long o = base[q] + 4 * c;
          const f32x4 a = *(const f32x4*)(P + o);
#pragma unroll
          for (int t = 0; t < 4; ++t) pv[t] = a[t];
          if (CL) {
            const f32x4 b = *(const f32x4*)(M + o), d = *(const f32x4*)(V + o);
#pragma unroll
            for (int t = 0; t < 4; ++t) {
              mv[t] = b[t];
              vv[t] = d[t];
            }
          }
          if (E) {
            const f32x4 b = *(const f32x4*)(E + o);
#pragma unroll
            for (int t = 0; t < 4; ++t) ev[t] = b[t];
          }
        }
      } else if (live[q]) {
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const int j = c + LPR * t;
          if (j < W) {
            const long o = base[q] + j;
            pv[t] = P[o];
            if (CL) {
              mv[t] = M[o];
              vv[t] = V[o];
            }
            if (E) ev[t] = E[o];
          }
        }
      }
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        p[q][h] = f32x2{pv[2 * h], pv[2 * h + 1]};
        m[q][h] = f32x2{mv[2 * h], mv[2 * h + 1]};
        v[q][h] = f32x2{vv[2 * h], vv[2 * h + 1]};
        e[q][h] = f32x2{ev[2 * h], ev[2 * h + 1]};
      }
      smin = min(smin, s[q]);
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) smin = min(smin, __shfl_xor(smin, o));
    smin = __builtin_amdgcn_readfirstlane(smin);
    for_ticks(hist, smin + 1, tick, [&](const OptScalars& sc, int k) {
#pragma unroll
      for (int q = 0; q < NS; ++q) {
        if (k > s[q]) {
          if (sc.do_adam) {
            if (CL) {
              idle_adam_pk(sc, p[q][0], m[q][0], v[q][0]);
              idle_adam_pk(sc, p[q][1], m[q][1], v[q][1]);
            } else {
              p[q][0] = p[q][0] * splat2(sc.decay_mul);
              p[q][1] = p[q][1] * splat2(sc.decay_mul);
            }
          }
          if (sc.do_ema) {
            ema_pk(sc, p[q][0], e[q][0]);
            ema_pk(sc, p[q][1], e[q][1]);
          }
        }
      }
    });
#pragma unroll
    for (int q = 0; q < NS; ++q) {
      if (!live[q]) continue;
      const float pv[4] = {p[q][0].x, p[q][0].y, p[q][1].x, p[q][1].y};
      const float mv[4] = {m[q][0].x, m[q][0].y, m[q][1].x, m[q][1].y};
      const float vv[4] = {v[q][0].x, v[q][0].y, v[q][1].x, v[q][1].y};
      const float ev[4] = {e[q][0].x, e[q][0].y, e[q][1].x, e[q][1].y};
      if (VEC) {
        if (4 * c < W) {
          const long o = base[q] + 4 * c;
          *(f32x4*)(P + o) = f32x4{pv[0], pv[1], pv[2], pv[3]};
          if (CL) {
            *(f32x4*)(M + o) = f32x4{mv[0], mv[1], mv[2], mv[3]};
            *(f32x4*)(V + o) = f32x4{vv[0], vv[1], vv[2], vv[3]};
          }
          if (E) *(f32x4*)(E + o) = f32x4{ev[0], ev[1], ev[2], ev[3]};
        }
      } else {
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const int j = c + LPR * t;
          if (j < W) {
            const long o = base[q] + j;
            P[o] = pv[t];
            if (CL) {
              M[o] = mv[t];
              V[o] = vv[t];
            }
            if (E) E[o] = ev[t];
          }
        }
      }
      if (c == 0) tb.last[row[q]] = tick | (CL ? LAST_NZ : 0);
    }
  }
}

// lanes per row of the classified flush: four elements per lane
__device__ __forceinline__ int cls_lpr(int width) {
  const int need = (width + 3) / 4;
  return need <= 1 ? 1 : need <= 2 ? 2 : need <= 4 ? 4 : need <= 8 ? 8 : 16;
}

#ifndef FLUSH_NS0
#define FLUSH_NS0 4
#endif
#ifndef FLUSH_NS1
#define FLUSH_NS1 2
#endif
// One kernel per class (zero-moment rows first, then the stepped rows): the short replay alone needs far fewer
// registers than the full one (one kernel holding both ran at the full replay's 112 VGPRs, four waves per SIMD),
// so the zero-moment pass runs at a higher occupancy.  Each pass reads the
// state words of every row (140 MB at cfg2, a few percent of the row bytes) and lists its own class.
template <int CL>
__global__ __launch_bounds__(256) void lazy_flush_cls_kernel(const ctr_lazy_tab_t* __restrict__ tabs, int ntabs,
                                                             float* P, float* M, float* V, float* E,
                                                             const OptScalars* __restrict__ hist, int tick) {
  __shared__ long chunk0[FLUSH_MAXTABS + 1];
  __shared__ int lrow[CLS_CH];
  __shared__ int ls[CLS_CH];
  __shared__ int cnt;
  const int tid = threadIdx.x;
  if (tid == 0) {
    long c = 0;
    for (int t = 0; t < ntabs; ++t) {
      chunk0[t] = c;
      c += cdiv(tabs[t].rows, (long)CLS_CH);
    }
    chunk0[ntabs] = c;
  }
  __syncthreads();
  const long nchunks = chunk0[ntabs];
  // chunk -> (table, first row); the state words of a chunk are loaded while the previous chunk replays
  auto locate = [&](long ch, int& ti, long& r0) {
    int a = 0, b = ntabs;
    while (b - a > 1) {
      const int mid = (a + b) >> 1;
      if (chunk0[mid] <= ch) a = mid; else b = mid;
    }
    ti = a;
    r0 = (ch - chunk0[a]) * CLS_CH;
  };
  int wv[CLS_CH / 256];
  auto load_words = [&](long ch) {
    int ti;
    long r0;
    locate(ch, ti, r0);
    const long trows = tabs[ti].rows;
    const int* last = tabs[ti].last;
#pragma unroll
    for (int q = 0; q < CLS_CH / 256; ++q) {
      const long r = r0 + tid + 256 * q;
      wv[q] = r < trows ? last[r] : tick;
    }
  };
  if (blockIdx.x < nchunks) load_words(blockIdx.x);
  for (long ch = blockIdx.x; ch < nchunks; ch += gridDim.x) {
    int ti;
    long r0;
    locate(ch, ti, r0);
    const ctr_lazy_tab_t tb = tabs[ti];
    if (tid == 0) cnt = 0;
    __syncthreads();
#pragma unroll
    for (int q = 0; q < CLS_CH / 256; ++q) {
      const int st = ltick(wv[q]);
      if (st < tick && ((wv[q] & LAST_NZ) ? 1 : 0) == CL) {
        const int pos = atomicAdd(&cnt, 1);
        lrow[pos] = (int)(r0 + tid + 256 * q);
        ls[pos] = st;
      }
    }
    __syncthreads();
    const int n = cnt;
    if (ch + gridDim.x < nchunks) load_words(ch + gridDim.x);
    if (n > 0) {
      constexpr int NS = CL ? FLUSH_NS1 : FLUSH_NS0;
      const bool vec = (tb.width & 3) == 0 && (tb.p_off & 3) == 0;    // block-uniform
      switch (cls_lpr(tb.width)) {
        case 1:
          if (vec) replay_tab_list<1, true, CL, NS>(tb, lrow, ls, n, P, M, V, E, hist, tick);
          else replay_tab_list<1, false, CL, NS>(tb, lrow, ls, n, P, M, V, E, hist, tick);
          break;
        case 2:
          if (vec) replay_tab_list<2, true, CL, NS>(tb, lrow, ls, n, P, M, V, E, hist, tick);
          else replay_tab_list<2, false, CL, NS>(tb, lrow, ls, n, P, M, V, E, hist, tick);
          break;
        case 4:
          if (vec) replay_tab_list<4, true, CL, NS>(tb, lrow, ls, n, P, M, V, E, hist, tick);
          else replay_tab_list<4, false, CL, NS>(tb, lrow, ls, n, P, M, V, E, hist, tick);
          break;
        case 8:
          if (vec) replay_tab_list<8, true, CL, NS>(tb, lrow, ls, n, P, M, V, E, hist, tick);
          else replay_tab_list<8, false, CL, NS>(tb, lrow, ls, n, P, M, V, E, hist, tick);
          break;
        default:
          if (vec) replay_tab_list<16, true, CL, NS>(tb, lrow, ls, n, P, M, V, E, hist, tick);
          else replay_tab_list<16, false, CL, NS>(tb, lrow, ls, n, P, M, V, E, hist, tick);
          break;
      }
    }
    __syncthreads();      // the list is refilled by the next iteration
  }
}

// forward read of tokens X[0, n): a workgroup claims the rows of CLS_CH token positions (CAS on the att
// row's state word: a token read many times is caught up once; a token equal to its predecessor is that
// position's job) into the lists, then replays them
// hot (>= 0): a row most sequences hold (the padding token of the left-padded histories): claimed once,
// by the first workgroup, and skipped at every position -- 4096 CAS attempts on one word per step otherwise
// serialise at its L2 channel (~40 us of the touch at cfg2)
template <int W>
__global__ __launch_bounds__(256) void lazy_touch_pair_cls_kernel(const ctr_lazy_tab_t* __restrict__ tabs,
                                                                  const int32_t* __restrict__ X, long n, int hot,
                                                                  float* P, float* M, float* V, float* E,
                                                                  const OptScalars* __restrict__ hist, int tick) {
  // TOUCH_CH + 1: in the first chunk the hot row can join TOUCH_CH distinct claimed rows of the same class
  __shared__ int lrow[2][TOUCH_CH + 1];
  __shared__ int ls[2][TOUCH_CH + 1];
  __shared__ int cnt[2];
  const ctr_lazy_tab_t ta = tabs[0], tb = tabs[1];
  const int tid = threadIdx.x;
  for (long p0 = (long)blockIdx.x * TOUCH_CH; p0 < n; p0 += (long)gridDim.x * TOUCH_CH) {
    if (tid < 2) cnt[tid] = 0;
    __syncthreads();
    if (p0 == 0 && tid == 0 && hot >= 0 && hot < ta.rows) {
      int* lp = ta.last + hot;
      const int w = __hip_atomic_load(lp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (ltick(w) < tick && atomicCAS(lp, w, tick | (w & LAST_NZ)) == w) {
        const int cl = (w & LAST_NZ) ? 1 : 0;
        const int q = atomicAdd(&cnt[cl], 1);
        lrow[cl][q] = hot;
        ls[cl][q] = ltick(w);
      }
    }
    for (int i = tid; i < TOUCH_CH; i += 256) {
      const long pos = p0 + i;
      if (pos < n) {
        const long row = X[pos];
        const bool dup = (pos > 0 && X[pos - 1] == row) || row == hot;
        if (!dup && row >= 0 && row < ta.rows) {
          int* lp = ta.last + row;
          const int w = __hip_atomic_load(lp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (ltick(w) < tick && atomicCAS(lp, w, tick | (w & LAST_NZ)) == w) {
            const int cl = (w & LAST_NZ) ? 1 : 0;
            const int q = atomicAdd(&cnt[cl], 1);
            lrow[cl][q] = (int)row;
            ls[cl][q] = ltick(w);
          }
        }
      }
    }
    __syncthreads();
    replay_pair_list<W, 0>(ta, tb, lrow[0], ls[0], cnt[0], P, M, V, E, hist, tick, false);
    replay_pair_list<W, 1>(ta, tb, lrow[1], ls[1], cnt[1], P, M, V, E, hist, tick, false);
    __syncthreads();
  }
}

}  // namespace ctr

using namespace ctr;

extern "C" int ctr_opt_hist_entry_bytes(void) { return (int)sizeof(OptScalars); }

extern "C" int ctr_opt_hist_record(void* hist, int tick, float lr, float wd, float beta1, float beta2, float eps,
                                   int step, float ema_decay, int do_adam, int do_ema, void* stream) {
  CTR_REQUIRE(hist != nullptr && tick > 0, "ctr_opt_hist_record: bad history / tick");
  const OptScalars s = make_opt_scalars(lr, wd, beta1, beta2, eps, step, ema_decay, do_adam, do_ema);
  opt_hist_record_kernel<<<1, 1, 0, (hipStream_t)stream>>>((OptScalars*)hist, tick, s);
  return check_launch("opt_hist_record");
}

extern "C" int ctr_lazy_touch(const ctr_lazy_tab_t* tabs, int ntabs, const int32_t* X, long nx, int ncols,
                              int per_column, float* P, float* M, float* V, float* E, const void* hist, int tick,
                              void* stream) {
  CTR_REQUIRE(per_column >= 0 && per_column <= 2, "ctr_lazy_touch: per_column must be 0, 1 or 2");
  CTR_REQUIRE(ntabs > 0 && (per_column != 1 || ntabs == ncols), "ctr_lazy_touch: per_column needs ntabs == ncols");
  if (tick <= 0 || nx <= 0 || ncols <= 0) return 0;
  const long nitems = per_column ? nx * ncols : nx * ncols * ntabs;
  const unsigned grid = (unsigned)cdiv(nitems * LG, 256L);
  if (ntabs <= FLUSH_MAXTABS)
    lazy_touch_kernel<true><<<grid, 256, 0, (hipStream_t)stream>>>(tabs, ntabs, X, nitems, ncols, per_column, P, M, V,
                                                                   E, (const OptScalars*)hist, tick);
  else
    lazy_touch_kernel<false><<<grid, 256, 0, (hipStream_t)stream>>>(tabs, ntabs, X, nitems, ncols, per_column, P, M,
                                                                    V, E, (const OptScalars*)hist, tick);
  return check_launch("lazy_touch");
}

extern "C" int ctr_lazy_update(const ctr_lazy_tab_t* tabs, int ntabs, const uint32_t* keys, const float* G, int g_ld,
                               const uint32_t* n_uniq, long cap, const float* coef, float* P, float* M, float* V,
                               float* E, const void* hist, int tick, void* stream) {
  CTR_REQUIRE(ntabs > 0 && tick > 0, "ctr_lazy_update: bad tables / tick");
  if (cap <= 0) return 0;
  const unsigned grid = (unsigned)cdiv(cap * LG, 256L);
  if (ntabs <= FLUSH_MAXTABS)
    lazy_update_kernel<true><<<grid, 256, 0, (hipStream_t)stream>>>(tabs, ntabs, keys, G, g_ld, n_uniq, cap, coef, P,
                                                                    M, V, E, (const OptScalars*)hist, tick);
  else
    lazy_update_kernel<false><<<grid, 256, 0, (hipStream_t)stream>>>(tabs, ntabs, keys, G, g_ld, n_uniq, cap, coef,
                                                                     P, M, V, E, (const OptScalars*)hist, tick);
  return check_launch("lazy_update");
}

extern "C" int ctr_lazy_flush(const ctr_lazy_tab_t* tabs, int ntabs, long max_rows, float* P, float* M, float* V,
                              float* E, const void* hist, int tick, void* stream) {
  CTR_REQUIRE(ntabs <= FLUSH_MAXTABS, "ctr_lazy_flush: too many tables");
  if (ntabs <= 0 || tick <= 0 || max_rows <= 0) return 0;
  lazy_flush_cls_kernel<0><<<2048, 256, 0, (hipStream_t)stream>>>(tabs, ntabs, P, M, V, E, (const OptScalars*)hist,
                                                                  tick);
  lazy_flush_cls_kernel<1><<<2048, 256, 0, (hipStream_t)stream>>>(tabs, ntabs, P, M, V, E, (const OptScalars*)hist,
                                                                  tick);
  return check_launch("lazy_flush");
}

static int pair_grid(long n) {   // 4 waves per block, PAIR_NT rows per wave iteration
  return (int)std::max<long>(1, std::min<long>((n + 4 * PAIR_NT - 1) / (4 * PAIR_NT), 256L * 16));
}

static bool pair_ok(const ctr_lazy_tab_t* tabs_host_view) { return tabs_host_view != nullptr; }

extern "C" int ctr_lazy_touch_pair(const ctr_lazy_tab_t* tabs, int width, const int32_t* X, long n, float* P,
                                   float* M, float* V, float* E, const void* hist, int tick, void* stream) {
  return ctr_lazy_touch_pair_hot(tabs, width, X, n, -1, P, M, V, E, hist, tick, stream);
}

extern "C" int ctr_lazy_touch_pair_hot(const ctr_lazy_tab_t* tabs, int width, const int32_t* X, long n, int hot_row,
                                       float* P, float* M, float* V, float* E, const void* hist, int tick,
                                       void* stream) {
  CTR_REQUIRE(pair_ok(tabs) && width >= 1 && width <= 64, "ctr_lazy_touch_pair: two tables of width <= 64");
  if (tick <= 0 || n <= 0) return 0;
  {
    const int cgrid = (int)std::max<long>(1, std::min<long>((n + TOUCH_CH - 1) / TOUCH_CH, 256L * 16));
    const OptScalars* h = (const OptScalars*)hist;
    hipStream_t s = (hipStream_t)stream;
    switch (width) {      // the classified touch for the widths whose rows split into float4 lanes
      case 4: lazy_touch_pair_cls_kernel<4><<<cgrid, 256, 0, s>>>(tabs, X, n, hot_row, P, M, V, E, h, tick); return check_launch("lazy_touch_pair");
      case 8: lazy_touch_pair_cls_kernel<8><<<cgrid, 256, 0, s>>>(tabs, X, n, hot_row, P, M, V, E, h, tick); return check_launch("lazy_touch_pair");
      case 16: lazy_touch_pair_cls_kernel<16><<<cgrid, 256, 0, s>>>(tabs, X, n, hot_row, P, M, V, E, h, tick); return check_launch("lazy_touch_pair");
      case 32: lazy_touch_pair_cls_kernel<32><<<cgrid, 256, 0, s>>>(tabs, X, n, hot_row, P, M, V, E, h, tick); return check_launch("lazy_touch_pair");
      case 64: lazy_touch_pair_cls_kernel<64><<<cgrid, 256, 0, s>>>(tabs, X, n, hot_row, P, M, V, E, h, tick); return check_launch("lazy_touch_pair");
      default: break;
    }
  }
  if (width <= 32)
    lazy_touch_pair_kernel<1><<<pair_grid(n), 256, 0, (hipStream_t)stream>>>(tabs, X, n, P, M, V, E,
                                                                             (const OptScalars*)hist, tick);
  else
    lazy_touch_pair_kernel<2><<<pair_grid(n), 256, 0, (hipStream_t)stream>>>(tabs, X, n, P, M, V, E,
                                                                             (const OptScalars*)hist, tick);
  return check_launch("lazy_touch_pair");
}

extern "C" int ctr_lazy_update_pair(const ctr_lazy_tab_t* tabs, int width, const uint32_t* keys, const float* Ga,
                                    const float* Gb, int g_ld, const uint32_t* n_uniq, long cap, const float* coef,
                                    float* P, float* M, float* V, float* E, const void* hist, int tick, void* stream) {
  CTR_REQUIRE(pair_ok(tabs) && width >= 1 && width <= 64 && tick > 0, "ctr_lazy_update_pair: bad tables / tick");
  if (cap <= 0) return 0;
  if (width <= 32)
    lazy_update_pair_kernel<1><<<pair_grid(cap), 256, 0, (hipStream_t)stream>>>(
        tabs, keys, Ga, Gb, g_ld, n_uniq, cap, coef, P, M, V, E, (const OptScalars*)hist, tick);
  else
    lazy_update_pair_kernel<2><<<pair_grid(cap), 256, 0, (hipStream_t)stream>>>(
        tabs, keys, Ga, Gb, g_ld, n_uniq, cap, coef, P, M, V, E, (const OptScalars*)hist, tick);
  return check_launch("lazy_update_pair");
}

extern "C" int ctr_lazy_flush_pair(const ctr_lazy_tab_t* tabs, int width, long rows, float* P, float* M, float* V,
                                   float* E, const void* hist, int tick, void* stream) {
  CTR_REQUIRE(pair_ok(tabs) && width >= 1 && width <= 64, "ctr_lazy_flush_pair: two tables of width <= 64");
  if (tick <= 0 || rows <= 0) return 0;
  const int cgrid = (int)std::max<long>(1, std::min<long>((rows + CLS_CH - 1) / CLS_CH, 256L * 8));
  const OptScalars* h = (const OptScalars*)hist;
  hipStream_t s = (hipStream_t)stream;
  switch (width) {      // the classified flush for the widths whose rows split into float4 lanes
    case 4: lazy_flush_pair_cls_kernel<4, -1><<<cgrid, 256, 0, s>>>(tabs, P, M, V, E, h, tick); return check_launch("lazy_flush_pair");
    case 8: lazy_flush_pair_cls_kernel<8, -1><<<cgrid, 256, 0, s>>>(tabs, P, M, V, E, h, tick); return check_launch("lazy_flush_pair");
    case 16: lazy_flush_pair_cls_kernel<16, -1><<<cgrid, 256, 0, s>>>(tabs, P, M, V, E, h, tick); return check_launch("lazy_flush_pair");
    case 32: lazy_flush_pair_cls_kernel<32, -1><<<cgrid, 256, 0, s>>>(tabs, P, M, V, E, h, tick); return check_launch("lazy_flush_pair");
    case 64: lazy_flush_pair_cls_kernel<64, -1><<<cgrid, 256, 0, s>>>(tabs, P, M, V, E, h, tick); return check_launch("lazy_flush_pair");
    default: break;
  }
  if (width <= 32)
    lazy_flush_pair_kernel<1><<<pair_grid(rows), 256, 0, (hipStream_t)stream>>>(tabs, P, M, V, E,
                                                                                 (const OptScalars*)hist, tick);
  else
    lazy_flush_pair_kernel<2><<<pair_grid(rows), 256, 0, (hipStream_t)stream>>>(tabs, P, M, V, E,
                                                                                 (const OptScalars*)hist, tick);
  return check_launch("lazy_flush_pair");
}

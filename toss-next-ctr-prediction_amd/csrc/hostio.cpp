// Host-side hot loops of the Parquet -> NPY shard cache builder (tossctr/build_cache.py, the drop-in for
// src/data/build_cache_v1.py).  Both run over Arrow string columns (int32 offsets + UTF-8 bytes):
//
//   ctr_hash_utf8  XXH64(bytes, seed) per string -- the build's stable replacement for polars'
//                  `Series.hash(seed=2025, seed_1=0)` (build_cache_v1.py:104-111, 128-129), whose value
//                  is polars-version specific and not reproducible without polars.  XXH64 is restated
//                  from its published specification; tests check it against the `xxhash` package.
//   ctr_parse_seq  the per-row Python loop of build_cache_v1.py:149-156: split on ',', drop empty
//                  tokens, int() each, keep the last L, right-align into a pad-filled (n, L) int32 row.
#include <cstdint>
#include <cstring>

#include "ctr_hip.h"

namespace {

constexpr uint64_t P1 = 0x9E3779B185EBCA87ULL, P2 = 0xC2B2AE3D27D4EB4FULL, P3 = 0x165667B19E3779F9ULL,
                   P4 = 0x85EBCA77C2B2AE63ULL, P5 = 0x27D4EB2F165667C5ULL;

inline uint64_t rotl(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
inline uint64_t rd64(const uint8_t* p) {
  uint64_t v;
  std::memcpy(&v, p, 8);   // little-endian host
  return v;
}
inline uint32_t rd32(const uint8_t* p) {
  uint32_t v;
  std::memcpy(&v, p, 4);
  return v;
}
inline uint64_t round64(uint64_t acc, uint64_t in) {
  acc += in * P2;
  acc = rotl(acc, 31);
  return acc * P1;
}
inline uint64_t merge64(uint64_t acc, uint64_t v) {
  acc ^= round64(0, v);
  return acc * P1 + P4;
}

uint64_t xxh64(const uint8_t* p, size_t len, uint64_t seed) {
  const uint8_t* end = p + len;
  uint64_t h;
  if (len >= 32) {
    uint64_t v1 = seed + P1 + P2, v2 = seed + P2, v3 = seed, v4 = seed - P1;
    const uint8_t* limit = end - 32;
    do {
      v1 = round64(v1, rd64(p));
      v2 = round64(v2, rd64(p + 8));
      v3 = round64(v3, rd64(p + 16));
      v4 = round64(v4, rd64(p + 24));
      p += 32;
    } while (p <= limit);
    h = rotl(v1, 1) + rotl(v2, 7) + rotl(v3, 12) + rotl(v4, 18);
    h = merge64(h, v1);
    h = merge64(h, v2);
    h = merge64(h, v3);
    h = merge64(h, v4);
  } else {
    h = seed + P5;
  }
  h += (uint64_t)len;
  while (p + 8 <= end) {
    h ^= round64(0, rd64(p));
    h = rotl(h, 27) * P1 + P4;
    p += 8;
  }
  if (p + 4 <= end) {
    h ^= (uint64_t)rd32(p) * P1;
    h = rotl(h, 23) * P2 + P3;
    p += 4;
  }
  while (p < end) {
    h ^= (uint64_t)(*p) * P5;
    h = rotl(h, 11) * P1;
    ++p;
  }
  h ^= h >> 33;
  h *= P2;
  h ^= h >> 29;
  h *= P3;
  h ^= h >> 32;
  return h;
}

inline bool is_space(uint8_t ch) { return ch == ' ' || ch == '\t' || ch == '\n' || ch == '\r' || ch == '\v' || ch == '\f'; }

// Python int(token) for an ASCII decimal token (surrounding whitespace allowed); false where int() raises
// or the value does not fit the int32 the reference casts to
bool parse_int(const uint8_t* a, const uint8_t* b, int32_t* v) {
  while (a < b && is_space(*a)) ++a;
  while (b > a && is_space(b[-1])) --b;
  bool neg = false;
  if (a < b && (*a == '+' || *a == '-')) {
    neg = *a == '-';
    ++a;
  }
  if (a == b) return false;
  int64_t x = 0;
  for (; a < b; ++a) {
    if (*a < '0' || *a > '9') return false;
    x = x * 10 + (*a - '0');
    if (x > ((int64_t)1 << 31)) return false;
  }
  x = neg ? -x : x;
  if (x > INT32_MAX || x < INT32_MIN) return false;
  *v = (int32_t)x;
  return true;
}

}  // namespace

extern "C" int ctr_hash_utf8(const int32_t* offsets, const uint8_t* data, long n, uint64_t seed, uint64_t* out) {
  if (n < 0 || (n > 0 && (!offsets || !out))) return -1;
  for (long i = 0; i < n; ++i) {
    const int32_t a = offsets[i], b = offsets[i + 1];
    if (b < a) return -1;
    out[i] = xxh64(data + a, (size_t)(b - a), seed);
  }
  return 0;
}

extern "C" long ctr_parse_seq(const int32_t* offsets, const uint8_t* data, const uint8_t* valid, long n, int L,
                              int pad_id, int32_t* out) {
  if (n < 0 || L <= 0 || (n > 0 && (!offsets || !out))) return -1;
  for (long i = 0; i < n; ++i) {
    int32_t* row = out + (size_t)i * L;
    for (int t = 0; t < L; ++t) row[t] = pad_id;
    if (valid && !valid[i]) continue;                // null -> "" -> all pad
    const uint8_t* s = data + offsets[i];
    const uint8_t* e = data + offsets[i + 1];
    long ntok = 0;                                   // non-empty tokens (the reference's `if x`)
    for (const uint8_t* q = s; q <= e;) {
      const uint8_t* t = q;
      while (t < e && *t != ',') ++t;
      ntok += t > q;
      q = t + 1;
    }
    long k = 0;
    for (const uint8_t* q = s; q <= e;) {
      const uint8_t* t = q;
      while (t < e && *t != ',') ++t;
      if (t > q) {
        int32_t v;
        if (!parse_int(q, t, &v)) return -(2 + i);   // int(x) raises: report the row
        if (k >= ntok - L) row[L - ntok + k] = v;
        ++k;
      }
      q = t + 1;
    }
  }
  return 0;
}

// ---------------------------------------------------------------------------------------------------------
// Co-visitation features (tossctr/covis.py, the drop-in for src/features/covis.py): the seq column exploded
// the way _parse_seq_topk + explode + cum_count do it (covis.py:60-80, :174-183):
//   pieces = str.split(",") (empty pieces kept; a null seq is the empty list), each cast to Int32 non-strictly
//   (null unless [+-]digits within int32), the LAST top_k pieces kept; an empty list explodes to one null;
//   pos = (# non-null tokens so far in the row) - 1.
// ctr_covis_explode_count fills row_ptr (n + 1) and returns the exploded length; ctr_covis_explode fills
// tok / pos / ok (ok = 1 for a non-null token).  Rows are split over threads (disjoint output ranges).
// ---------------------------------------------------------------------------------------------------------
#include <algorithm>
#include <thread>
#include <vector>

namespace {

bool parse_i32_strict(const uint8_t* a, const uint8_t* b, int32_t* v) {
  bool neg = false;
  if (a < b && (*a == '+' || *a == '-')) neg = *a++ == '-';
  if (a == b) return false;
  int64_t x = 0;
  for (; a < b; ++a) {
    if (*a < '0' || *a > '9') return false;
    x = x * 10 + (*a - '0');
    if (x > ((int64_t)1 << 31)) return false;
  }
  x = neg ? -x : x;
  if (x > INT32_MAX || x < INT32_MIN) return false;
  *v = (int32_t)x;
  return true;
}

inline long covis_pieces(const int32_t* off, const uint8_t* data, const uint8_t* valid, long i) {
  if (valid && !valid[i]) return 0;
  return 1 + (long)std::count(data + off[i], data + off[i + 1], (uint8_t)',');
}

template <class F>
void parallel_rows(long n, F&& f) {
  unsigned nt = std::thread::hardware_concurrency();
  nt = std::max(1u, std::min(nt, 16u));
  if (n < 65536) nt = 1;
  std::vector<std::thread> th;
  const long chunk = (n + nt - 1) / nt;
  for (unsigned t = 0; t < nt; ++t) {
    const long a = t * chunk, b = std::min(n, a + chunk);
    if (a >= b) break;
    th.emplace_back([&f, a, b] { f(a, b); });
  }
  for (auto& x : th) x.join();
}

}  // namespace

extern "C" long ctr_covis_explode_count(const int32_t* offsets, const uint8_t* data, const uint8_t* valid, long n,
                                        int top_k, int64_t* row_ptr) {
  if (n < 0 || !row_ptr || (n > 0 && !offsets)) return -1;
  row_ptr[0] = 0;
  for (long i = 0; i < n; ++i) {
    const long m = std::min<long>(covis_pieces(offsets, data, valid, i), top_k > 0 ? top_k : 0);
    row_ptr[i + 1] = row_ptr[i] + std::max<long>(m, 1);
  }
  return (long)row_ptr[n];
}

extern "C" int ctr_covis_explode(const int32_t* offsets, const uint8_t* data, const uint8_t* valid, long n, int top_k,
                                 const int64_t* row_ptr, int32_t* tok, int32_t* pos, uint8_t* ok) {
  if (n < 0 || (n > 0 && (!offsets || !row_ptr || !tok || !pos || !ok))) return -1;
  parallel_rows(n, [&](long a, long b) {
    for (long i = a; i < b; ++i) {
      const int64_t o = row_ptr[i];
      const long pieces = covis_pieces(offsets, data, valid, i);
      const long m = std::min<long>(pieces, top_k > 0 ? top_k : 0);
      if (m == 0) {                                   // [] explodes to one null
        tok[o] = 0;
        pos[o] = -1;
        ok[o] = 0;
        continue;
      }
      const uint8_t* s = data + offsets[i];
      const uint8_t* e = data + offsets[i + 1];
      long skip = pieces - m, k = 0;
      int32_t cnt = 0;
      for (const uint8_t* q = s; q <= e;) {
        const uint8_t* t = q;
        while (t < e && *t != ',') ++t;
        if (skip > 0) {
          --skip;
        } else {
          int32_t v = 0;
          const bool good = parse_i32_strict(q, t, &v);
          cnt += good;
          tok[o + k] = good ? v : 0;
          ok[o + k] = good;
          pos[o + k] = cnt - 1;
          ++k;
        }
        q = t + 1;
      }
    }
  });
  return 0;
}

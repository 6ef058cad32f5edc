// ingest_parse.h — scalar parsing primitives of the JSON ingest codec (ingest.hip), shared by the device
// kernel and the host (the host uses them for fd_hash64 and the CPU unit tests of the primitives).
//
//   fd::hash_bytes        card / device / merchant / vocabulary identity: fmix64(FNV-1a-64(utf-8 bytes))
//   fd::scan_number       RFC 8259 number grammar -> (significand w <= 19 digits, exponent q, sign)
//   fd::decimal_to_double correctly rounded decimal -> binary64: Clinger's exact fast path, else the
//                         Eisel-Lemire 128-bit product (pow5_table.h); w+1 cross-check for > 19 digits
//   fd::decimal_to_cents  exact amount in cents (round half to even below a cent, flagged inexact)
//   fd::parse_iso_instant ISO-8601 date-time -> epoch ms (UTC when no offset; fraction truncated, as
//                         java.time.Instant.toEpochMilli)
#pragma once

#include <cstdint>

#include "pow5_table.h"

#if defined(__HIPCC__)
#define FD_HD __host__ __device__ __forceinline__
#else
#define FD_HD inline
#endif

namespace fd {

constexpr uint64_t kFnvBasis = 0xcbf29ce484222325ull;
constexpr uint64_t kFnvPrime = 0x100000001b3ull;

FD_HD uint64_t fnv_step(uint64_t h, unsigned char c) { return (h ^ c) * kFnvPrime; }

FD_HD uint64_t fmix64_hd(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdULL;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ULL;
  k ^= k >> 33;
  return k;
}

FD_HD uint64_t hash_finish(uint64_t fnv) { return fmix64_hd(fnv); }

FD_HD uint64_t hash_bytes(const unsigned char* s, int64_t n) {
  uint64_t h = kFnvBasis;
  for (int64_t i = 0; i < n; ++i) h = fnv_step(h, s[i]);
  return hash_finish(h);
}

// compile-time FNV-1a of a key name (no finaliser): the kernel's key dispatch
constexpr uint64_t key_hash(const char* s, uint64_t h = kFnvBasis) {
  return *s ? key_hash(s + 1, (h ^ (unsigned char)*s) * kFnvPrime) : h;
}

FD_HD void mul64x64(uint64_t a, uint64_t b, uint64_t& hi, uint64_t& lo) {
#if defined(__HIP_DEVICE_COMPILE__)
  lo = a * b;
  hi = __umul64hi(a, b);
#else
  const unsigned __int128 p = (unsigned __int128)a * b;
  lo = (uint64_t)p;
  hi = (uint64_t)(p >> 64);
#endif
}

// Eisel-Lemire: w * 10^q (w != 0, no sign) -> binary64 bits; exact for w < 2^64 with the 128-bit table
FD_HD uint64_t eisel_lemire_bits(int64_t q, uint64_t w) {
  if (w == 0 || q < kPow5Min) return 0ull;
  if (q > kPow5Max) return 0x7FFull << 52;
  const int lz = __builtin_clzll(w);
  w <<= lz;
  const int idx = 2 * (int)(q - kPow5Min);
  uint64_t hi, lo;
  mul64x64(w, kPow5Table[idx], hi, lo);
  const uint64_t precision_mask = 0xFFFFFFFFFFFFFFFFull >> 55;  // mantissa bits + 3
  if ((hi & precision_mask) == precision_mask) {
    uint64_t hi2, lo2;
    mul64x64(w, kPow5Table[idx + 1], hi2, lo2);
    lo += hi2;
    if (hi2 > lo) ++hi;
  }
  const int upperbit = (int)(hi >> 63);
  const int shift = upperbit + 64 - 52 - 3;
  uint64_t mantissa = hi >> shift;
  int32_t power2 = (int32_t)(((((152170 + 65536) * (int32_t)q) >> 16) + 63) + upperbit - lz + 1023);
  if (power2 <= 0) {  // subnormal
    if (-power2 + 1 >= 64) return 0ull;
    mantissa >>= -power2 + 1;
    mantissa += (mantissa & 1);
    mantissa >>= 1;
    power2 = (mantissa < (1ull << 52)) ? 0 : 1;
    return (mantissa & ((1ull << 52) - 1)) | ((uint64_t)power2 << 52);
  }
  if (lo <= 1 && q >= -4 && q <= 23 && (mantissa & 3) == 1) {  // exactly halfway: round to even
    if ((mantissa << shift) == hi) mantissa &= ~1ull;
  }
  mantissa += (mantissa & 1);
  mantissa >>= 1;
  if (mantissa >= (2ull << 52)) {
    mantissa = 1ull << 52;
    ++power2;
  }
  mantissa &= ~(1ull << 52);
  if (power2 >= 0x7FF) return 0x7FFull << 52;
  return mantissa | ((uint64_t)power2 << 52);
}

FD_HD double bits_to_double(uint64_t b) {
  union {
    uint64_t u;
    double d;
  } x;
  x.u = b;
  return x.d;
}

FD_HD double pow10_exact(int e) {  // 10^e, e in [0, 22]: exact binary64 values
  // by the bits of e: 10^1, 10^2, 10^4, 10^8, 10^16 and every product of them are exact (5^22 < 2^53), so the
  // result is the same exact value as a running product, in at most five multiplies instead of e
  double p = (e & 1) ? 10.0 : 1.0;
  if (e & 2) p *= 100.0;
  if (e & 4) p *= 1e4;
  if (e & 8) p *= 1e8;
  if (e & 16) p *= 1e16;
  return p;
}

// decimal value (-1)^neg * w * 10^q -> nearest binary64 (ties to even); *ambiguous set when digits beyond
// the 19th changed the rounding (many = true and w, w+1 round differently)
FD_HD double decimal_to_double(uint64_t w, int64_t q, bool neg, bool many, bool* ambiguous) {
  double d;
  if (!many && w <= (1ull << 53) && q >= -22 && q <= 22) {  // Clinger: both operands exact, one rounding
    d = (double)w;
    d = q < 0 ? d / pow10_exact((int)-q) : d * pow10_exact((int)q);
  } else {
    const uint64_t b = eisel_lemire_bits(q, w);
    if (many && ambiguous && eisel_lemire_bits(q, w + 1) != b) *ambiguous = true;
    d = bits_to_double(b);
  }
  return neg ? -d : d;
}

struct Decimal {
  uint64_t w = 0;   // first <= 19 significant digits
  int64_t q = 0;    // value = w * 10^q (digits beyond the 19th dropped)
  bool neg = false;
  bool many = false;  // > 19 significant digits
  bool frac_or_exp = false;
};

// RFC 8259 number at s[pos..end); returns the index after it, or -1 on a grammar error
template <class Bytes>
FD_HD int scan_number(const Bytes& s, int pos, int end, Decimal& d) {
  d = Decimal{};
  int i = pos;
  if (i < end && s[i] == '-') {
    d.neg = true;
    ++i;
  }
  if (i >= end) return -1;
  int nd = 0;  // significant digits taken
  if (s[i] == '0') {
    ++i;
  } else if (s[i] >= '1' && s[i] <= '9') {
    while (i < end && s[i] >= '0' && s[i] <= '9') {
      if (nd < 19) {
        d.w = d.w * 10 + (uint64_t)(s[i] - '0');
        ++nd;
      } else {
        if (s[i] != '0') d.many = true;  // a dropped non-zero digit: the value is truncated
        ++d.q;
      }
      ++i;
    }
  } else {
    return -1;
  }
  if (i < end && s[i] == '.') {
    d.frac_or_exp = true;
    ++i;
    if (i >= end || s[i] < '0' || s[i] > '9') return -1;
    while (i < end && s[i] >= '0' && s[i] <= '9') {
      if (nd == 0 && s[i] == '0') {
        --d.q;  // leading zero of the fraction: not significant
      } else if (nd < 19) {
        d.w = d.w * 10 + (uint64_t)(s[i] - '0');
        ++nd;
        --d.q;
      } else if (s[i] != '0') {
        d.many = true;
      }
      ++i;
    }
  }
  if (i < end && (s[i] == 'e' || s[i] == 'E')) {
    d.frac_or_exp = true;
    ++i;
    bool eneg = false;
    if (i < end && (s[i] == '+' || s[i] == '-')) {
      eneg = s[i] == '-';
      ++i;
    }
    if (i >= end || s[i] < '0' || s[i] > '9') return -1;
    int64_t e = 0;
    while (i < end && s[i] >= '0' && s[i] <= '9') {
      if (e < 100000) e = e * 10 + (s[i] - '0');
      ++i;
    }
    d.q += eneg ? -e : e;
  }
  if (d.w == 0) d.many = false;  // zero (any digits): exact
  return i;
}

// exact cents of a decimal amount; *inexact when it had sub-cent digits (rounded half to even) or more than
// 19 significant digits; false on overflow of int64
FD_HD bool decimal_to_cents(const Decimal& d, int64_t* cents, bool* inexact) {
  const int64_t e = d.q + 2;
  uint64_t c;
  if (d.many) *inexact = true;
  if (d.w == 0) {
    *cents = 0;
    return true;
  }
  if (e >= 0) {
    if (e > 18) return false;
    uint64_t p = 1;
    for (int k = 0; k < e; ++k) p *= 10;
    if (d.w > 0x7FFFFFFFFFFFFFFFull / p) return false;
    c = d.w * p;
  } else if (-e > 19) {
    c = 0;
    *inexact = true;
  } else {
    uint64_t p = 1;
    for (int k = 0; k < -e; ++k) p *= 10;
    c = d.w / p;
    const uint64_t r = d.w - c * p;
    if (r) {
      *inexact = true;
      const uint64_t half = p / 2;  // p is even (a power of ten >= 10)
      if (r > half || (r == half && (c & 1))) ++c;
    }
    if (c > 0x7FFFFFFFFFFFFFFFull) return false;
  }
  *cents = d.neg ? -(int64_t)c : (int64_t)c;
  return true;
}

FD_HD int64_t days_from_civil(int64_t y, unsigned m, unsigned d) {  // proleptic Gregorian -> days since 1970-01-01
  y -= m <= 2;
  const int64_t era = (y >= 0 ? y : y - 399) / 400;
  const unsigned yoe = (unsigned)(y - era * 400);
  const unsigned doy = (153 * (m + (m > 2 ? -3 : 9)) + 2) / 5 + d - 1;
  const unsigned doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
  return era * 146097 + (int64_t)doe - 719468;
}

template <class Bytes>
FD_HD bool digits_at(const Bytes& s, int i, int n, int end, int* v) {
  if (i + n > end) return false;
  int x = 0;
  for (int k = 0; k < n; ++k) {
    const int c = s[i + k];
    if (c < '0' || c > '9') return false;
    x = x * 10 + (c - '0');
  }
  *v = x;
  return true;
}

// "YYYY-MM-DDTHH:MM:SS[.f{1,9}][Z|(+|-)HH:MM]" occupying exactly s[pos..end) -> epoch ms
template <class Bytes>
FD_HD bool parse_iso_instant(const Bytes& s, int pos, int end, int64_t* ms) {
  int Y, M, D, h, mi, sec;
  if (!digits_at(s, pos, 4, end, &Y) || pos + 19 > end || s[pos + 4] != '-' || !digits_at(s, pos + 5, 2, end, &M) ||
      s[pos + 7] != '-' || !digits_at(s, pos + 8, 2, end, &D) || s[pos + 10] != 'T' ||
      !digits_at(s, pos + 11, 2, end, &h) || s[pos + 13] != ':' || !digits_at(s, pos + 14, 2, end, &mi) ||
      s[pos + 16] != ':' || !digits_at(s, pos + 17, 2, end, &sec))
    return false;
  if (M < 1 || M > 12 || D < 1 || h > 23 || mi > 59 || sec > 59) return false;
  const bool leap = (Y % 4 == 0 && Y % 100 != 0) || Y % 400 == 0;
  // month lengths - 28, two bits per month (Jan .. Dec: 3 0 3 2 3 2 3 3 2 3 2 3); no array (no scratch)
  const int mdays = 28 + (int)((0xeefbb3u >> (2 * (M - 1))) & 3u) + ((M == 2 && leap) ? 1 : 0);
  if (D > mdays) return false;
  int i = pos + 19;
  int frac_ms = 0;
  if (i < end && s[i] == '.') {
    ++i;
    int nd = 0;
    while (i < end && s[i] >= '0' && s[i] <= '9') {
      if (nd < 3) frac_ms = frac_ms * 10 + (s[i] - '0');
      ++nd;
      ++i;
    }
    if (nd == 0 || nd > 9) return false;
    for (int k = nd; k < 3; ++k) frac_ms *= 10;
  }
  int off_min = 0;
  if (i < end && (s[i] == 'Z' || s[i] == 'z')) {
    ++i;
  } else if (i < end && (s[i] == '+' || s[i] == '-')) {
    int oh, om;
    const bool neg = s[i] == '-';
    if (!digits_at(s, i + 1, 2, end, &oh) || i + 6 > end || s[i + 3] != ':' || !digits_at(s, i + 4, 2, end, &om) ||
        oh > 18 || om > 59)
      return false;
    off_min = (neg ? -1 : 1) * (oh * 60 + om);
    i += 6;
  }
  if (i != end) return false;
  const int64_t days = days_from_civil(Y, (unsigned)M, (unsigned)D);
  const int64_t secs = days * 86400 + h * 3600 + mi * 60 + sec - (int64_t)off_min * 60;
  *ms = secs * 1000 + frac_ms;
  return true;
}

}  // namespace fd

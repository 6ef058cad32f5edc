// ingest.hip — the Kafka JSON codec on the device: a micro-batch of raw transaction
// messages -> the engine's SoA batch (fd_txn_batch + fd_txn_context + window inputs), in HBM.
//
// Reference: the simulator writes each transaction as json.dumps(asdict(Transaction), default=str)
// (services/data-simulator/src/main/python/simulator.py:77-101 fields, :186 serializer, :376-385 send); the
// Flink job reads it with TransactionDeserializationSchema.deserialize (fl/serialization/
// TransactionDeserializationSchema.java:28-49: Jackson ObjectMapper + JavaTimeModule; on any exception an
// ERROR placeholder transaction goes downstream). The derived codes follow FeatureExtractor
// (fl/features/FeatureExtractor.java:300-325 device / IP / user agent, :434-451 isPrivateIP /
// analyzeSuspiciousUserAgent, :366-381 payment / type / card). Declared semantics: DESIGN.md "Ingest".
//
// One wavefront per message (two messages per wave in the member phase), two waves per workgroup:
//   stage      : 16-B coalesced loads of the message into LDS (<= 4 KiB; longer -> FD_INGEST_TOO_LONG)
//   structure  : lane i owns bytes [64i, 64i+64): unescaped-quote parity -> wave prefix XOR (ballot) gives
//                the in-string state at every segment start; bracket depth deltas -> wave prefix sum; the
//                depth-1 ':' of every top-level member is recorded; balance / closure validated
//   members    : lane j parses member j sequentially from LDS: key (decoded, FNV-1a -> field), value by the
//                field's type (strings streamed through the hash / IP-prefix / user-agent matchers without
//                materialising them, numbers by the exact decimal -> binary64 conversion of
//                ingest_parse.h, ISO-8601 instants, the nested geolocation objects)
//   resolve    : duplicate keys -> the last one wins (Jackson); missing / null fields -> defaults; lane f
//                writes output column f for the message
// HBM traffic per message: its bytes + 16 B of offsets in, ~100 B of SoA out.
#include <cstring>

#include "fd_internal.h"
#include "ingest_parse.h"

namespace fd {
namespace {

// two waves per workgroup (4 messages, ~19 KB of LDS): a workgroup fits beside the fused ensemble kernel's
// compact-layout workgroup (132 KB) on one CU, so a codec running on its own stream overlaps the scoring (config 3j)
constexpr int kWaves = 2;
constexpr int kSlots = 2 * kWaves;  // messages per workgroup
constexpr int kMaxMsg = 4080;      // bytes per message: 64 lanes x 64-byte segments minus the 16-B alignment shift
constexpr int kMaxMembers = 64;    // top-level members per message (one per lane; more -> malformed)
constexpr int kStage = 4096;

enum Field : int {
  F_TXN_ID, F_USER_ID, F_MERCHANT_ID, F_AMOUNT, F_TIMESTAMP, F_IP, F_DEVICE_FP, F_UA, F_GEO, F_MLOC,
  F_WEEKEND, F_HOUR, F_FRAUD, F_SCORE, F_PAY, F_TTYPE, F_CTYPE, F_COUNT
};

// simulator (snake_case, simulator.py:77-101) and Java bean (camelCase) property names, as compile-time
// FNV-1a constants (namespace-scope constexpr: never evaluated on the device)
struct KeyName {
  uint64_t h;
  int field;
};
constexpr KeyName kKeys[] = {
    {key_hash("transaction_id"), F_TXN_ID},
    {key_hash("transactionId"), F_TXN_ID},
    {key_hash("user_id"), F_USER_ID},
    {key_hash("userId"), F_USER_ID},
    {key_hash("merchant_id"), F_MERCHANT_ID},
    {key_hash("merchantId"), F_MERCHANT_ID},
    {key_hash("amount"), F_AMOUNT},
    {key_hash("timestamp"), F_TIMESTAMP},
    {key_hash("ip_address"), F_IP},
    {key_hash("ipAddress"), F_IP},
    {key_hash("device_fingerprint"), F_DEVICE_FP},
    {key_hash("deviceFingerprint"), F_DEVICE_FP},
    {key_hash("user_agent"), F_UA},
    {key_hash("userAgent"), F_UA},
    {key_hash("geolocation"), F_GEO},
    {key_hash("merchant_location"), F_MLOC},
    {key_hash("merchantLocation"), F_MLOC},
    {key_hash("is_weekend"), F_WEEKEND},
    {key_hash("isWeekend"), F_WEEKEND},
    {key_hash("hour_of_day"), F_HOUR},
    {key_hash("hourOfDay"), F_HOUR},
    {key_hash("is_fraud"), F_FRAUD},
    {key_hash("isFraud"), F_FRAUD},
    {key_hash("fraud_score"), F_SCORE},
    {key_hash("fraudScore"), F_SCORE},
    {key_hash("payment_method"), F_PAY},
    {key_hash("paymentMethod"), F_PAY},
    {key_hash("transaction_type"), F_TTYPE},
    {key_hash("transactionType"), F_TTYPE},
    {key_hash("card_type"), F_CTYPE},
    {key_hash("cardType"), F_CTYPE},
};
constexpr int kNumKeys = 31;

__device__ __forceinline__ int field_of_key(uint64_t h) {
  int f = -1;
#pragma unroll
  for (int k = 0; k < kNumKeys; ++k)
    if (h == kKeys[k].h) f = kKeys[k].field;
  return f;
}

// byte view of a wave's staged message (message byte i = stage[shift + i]); one ds_read_u8 per access keeps
// every access site a single instruction (the kernel must stay small enough for the instruction cache)
struct Reader {
  const unsigned char* st;
  int shift;
  __device__ __forceinline__ int operator[](int i) const { return st[shift + i]; }
  // message bytes i .. i+3 (little-endian) from two dword reads and one v_alignbyte (i >= 0; the stage slot is
  // padded so the second dword of the last byte stays inside it)
  __device__ __forceinline__ unsigned word(int i) const {
    const int p = shift + i;
    const unsigned* w = reinterpret_cast<const unsigned*>(st) + (p >> 2);
    return __builtin_amdgcn_alignbyte(w[1], w[0], (unsigned)(p & 3));
  }
};

// SWAR byte masks over one dword (bit 7 of each byte): the lowest flagged byte of the borrow form is exact
__device__ __forceinline__ unsigned first_zero_mask(unsigned x) { return (x - 0x01010101u) & ~x & 0x80808080u; }
__device__ __forceinline__ unsigned exact_zero_mask(unsigned x) {  // every byte exact (no borrow)
  return ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x | 0x7F7F7F7Fu);
}
// bytes that end a raw string run: '"', '\\' or a control character
__device__ __forceinline__ unsigned string_stop_mask(unsigned w) {
  return first_zero_mask(w ^ 0x22222222u) | first_zero_mask(w ^ 0x5C5C5C5Cu) | ((w - 0x20202020u) & ~w & 0x80808080u);
}

__device__ __forceinline__ bool is_ws(int c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r'; }

__device__ __forceinline__ int hexval(int c) {
  if (c >= '0' && c <= '9') return c - '0';
  if (c >= 'a' && c <= 'f') return c - 'a' + 10;
  if (c >= 'A' && c <= 'F') return c - 'A' + 10;
  return -1;
}

// streaming view of one decoded JSON string: FNV-1a, the first 8 decoded bytes and the byte count; with UA
// also the UTF-16 length (Java String.length()) and the "bot" / "crawler" substring matchers
// (FeatureExtractor.java:447-451) — only the user-agent fallback decoder needs those, every other member scans
// with the lean form
template <bool UA>
struct StrStats {
  uint64_t fnv = kFnvBasis;
  uint64_t head = 0;  // first 8 decoded bytes, little-endian
  uint64_t roll = 0;  // UA: last 8 decoded bytes
  int nbytes = 0;
  int units = 0;  // UA
  bool bot = false, crawler = false;  // UA
  bool escaped = false;
  __device__ __forceinline__ void byte(unsigned c) {  // branchless: selects, no divergent branches per byte
    fnv = fnv_step(fnv, (unsigned char)c);
    const uint64_t sh = (uint64_t)c << (8 * (nbytes & 7));
    head |= (nbytes < 8) ? sh : 0ull;
    ++nbytes;
    if constexpr (UA) {
      roll = (roll << 8) | c;
      bot = bot | ((roll & 0xFFFFFFull) == 0x626F74ull);                     // "bot"
      crawler = crawler | ((roll & 0xFFFFFFFFFFFFFFull) == 0x637261776C6572ull);  // "crawler"
    }
  }
  __device__ __forceinline__ void add_units(int n) {
    if constexpr (UA) units += n;
  }
  __device__ __forceinline__ void utf8(unsigned cp) {
    if (cp < 0x80) {
      byte(cp);
    } else if (cp < 0x800) {
      byte(0xC0 | (cp >> 6));
      byte(0x80 | (cp & 0x3F));
    } else if (cp < 0x10000) {
      byte(0xE0 | (cp >> 12));
      byte(0x80 | ((cp >> 6) & 0x3F));
      byte(0x80 | (cp & 0x3F));
    } else {
      byte(0xF0 | (cp >> 18));
      byte(0x80 | ((cp >> 12) & 0x3F));
      byte(0x80 | ((cp >> 6) & 0x3F));
      byte(0x80 | (cp & 0x3F));
    }
  }
};

// decode the string whose opening quote is at s[pos]; returns the index after the closing quote, -1 if malformed
template <class S>
__device__ __forceinline__ int scan_string(const Reader& s, int pos, int end, S& st) {
  int i = pos + 1;
  while (i < end) {
    // the raw run, four bytes per LDS access: the first stop byte ('"', '\\', control) from the SWAR masks, the
    // bytes before it fed to the stats (predicated, no per-byte branches)
    int c;
    for (;;) {
      const unsigned w = s.word(i);
      const unsigned stop = string_stop_mask(w);
      const int nb = min(stop ? (__builtin_ctz(stop) >> 3) : 4, end - i);
  #pragma unroll
      for (int k = 0; k < 4; ++k) {
        if (k < nb) {
          const unsigned b = (w >> (8 * k)) & 0xFFu;
          st.byte(b);
          // UTF-16 units of raw UTF-8: one per lead byte, two for a 4-byte sequence
          st.add_units((int)((b & 0xC0u) != 0x80u) + (int)(b >= 0xF0u));
        }
      }
      i += nb;
      if (nb < 4) {
        c = i < end ? (int)((w >> (8 * nb)) & 0xFFu) : -1;
        break;
      }
    }
    if (c == '"') return i + 1;
    if (c != '\\') return -1;  // unescaped control character, or the end
    st.escaped = true;
    if (i + 1 >= end) return -1;
    const int e = s[i + 1];
    i += 2;
    unsigned cp;
    switch (e) {
      case '"': cp = '"'; break;
      case '\\': cp = '\\'; break;
      case '/': cp = '/'; break;
      case 'b': cp = 8; break;
      case 'f': cp = 12; break;
      case 'n': cp = 10; break;
      case 'r': cp = 13; break;
      case 't': cp = 9; break;
      case 'u': {
        if (i + 4 > end) return -1;
        int v = 0;
        for (int k = 0; k < 4; ++k) {
          const int h = hexval(s[i + k]);
          if (h < 0) return -1;
          v = v * 16 + h;
        }
        i += 4;
        st.add_units(1);
        if (v >= 0xD800 && v <= 0xDBFF && i + 6 <= end && s[i] == '\\' && s[i + 1] == 'u') {
          int lo = 0;
          bool ok = true;
          for (int k = 0; k < 4; ++k) {
            const int h = hexval(s[i + 2 + k]);
            ok = ok && h >= 0;
            lo = lo * 16 + (h < 0 ? 0 : h);
          }
          if (ok && lo >= 0xDC00 && lo <= 0xDFFF) {
            i += 6;
            st.add_units(1);
            st.utf8(0x10000u + (((unsigned)v - 0xD800u) << 10) + ((unsigned)lo - 0xDC00u));
            continue;
          }
        }
        // lone surrogates: Java keeps them; their UTF-8 (CESU) bytes are hashed as is
        st.utf8((unsigned)v);
        continue;
      }
      default: return -1;
    }
    st.add_units(1);
    st.byte(cp);
  }
  return -1;
}

// a run of decimal digits from s[i] (at least i < end), four bytes per LDS access: per-byte digit test on the
// dword (t = byte ^ '0' is a digit iff its high nibble is 0 and its low nibble + 6 stays below 16), the digits
// before the first other byte fed to `digit` in order; returns the index after the run
template <class F>
__device__ __forceinline__ int digit_run(const Reader& s, int i, int end, F&& digit) {
  for (;;) {
    const unsigned t = s.word(i) ^ 0x30303030u;
    const unsigned other = (t & 0xF0F0F0F0u) | (((t & 0x0F0F0F0Fu) + 0x06060606u) & 0x10101010u);
    const int nb = min(other ? (__builtin_ctz(other) >> 3) : 4, end - i);
  #pragma unroll
    for (int k = 0; k < 4; ++k)
      if (k < nb) digit((int)((t >> (8 * k)) & 0xFu));
    i += nb;
    if (nb < 4) return i;
  }
}

// scan_number (ingest_parse.h, the RFC 8259 grammar and the same Decimal) with the integer and fraction digit runs
// read a dword at a time; the exponent (rare) byte by byte
__device__ __forceinline__ int scan_number_w(const Reader& s, int pos, int end, Decimal& d) {
  d = Decimal{};
  int i = pos;
  if (i < end && s[i] == '-') {
    d.neg = true;
    ++i;
  }
  if (i >= end) return -1;
  int nd = 0;  // significant digits taken
  const int c0 = s[i];
  if (c0 == '0') {
    ++i;
  } else if (c0 >= '1' && c0 <= '9') {
    i = digit_run(s, i, end, [&](int g) {
      if (nd < 19) {
        d.w = d.w * 10 + (uint64_t)g;
        ++nd;
      } else {
        d.many = d.many || g != 0;  // a dropped non-zero digit: the value is truncated
        ++d.q;
      }
    });
  } else {
    return -1;
  }
  if (i < end && s[i] == '.') {
    d.frac_or_exp = true;
    ++i;
    if (i >= end || s[i] < '0' || s[i] > '9') return -1;
    i = digit_run(s, i, end, [&](int g) {
      if (nd == 0 && g == 0) {
        --d.q;  // leading zero of the fraction: not significant
      } else if (nd < 19) {
        d.w = d.w * 10 + (uint64_t)g;
        ++nd;
        --d.q;
      } else {
        d.many = d.many || g != 0;
      }
    });
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

__device__ __forceinline__ bool lit_at(const Reader& s, int i, int end, const char* w, int n);
// parse_iso_instant (ingest_parse.h, same grammar and result) with the fixed 19-byte prefix read as five dwords and
// the fraction as a digit run: "YYYY-MM-DDTHH:MM:SS[.f{1,9}][Z|(+|-)HH:MM]" occupying exactly s[pos..end)
__device__ __forceinline__ bool parse_iso_w(const Reader& s, int pos, int end, int64_t* ms) {
  if (pos + 19 > end) return false;
  unsigned w[5];
#pragma unroll
  for (int q = 0; q < 5; ++q) w[q] = s.word(pos + 4 * q);
  auto B = [&](int i) { return (int)((w[i >> 2] >> (8 * (i & 3))) & 0xFFu); };
  bool ok = B(4) == '-' && B(7) == '-' && B(10) == 'T' && B(13) == ':' && B(16) == ':';
  auto num = [&](int i, int nd) {  // nd digits from byte i (ok cleared on a non-digit)
    int v = 0;
#pragma unroll
    for (int k = 0; k < nd; ++k) {
      const int g = B(i + k) - '0';
      ok = ok && (unsigned)g <= 9u;
      v = v * 10 + g;
    }
    return v;
  };
  const int Y = num(0, 4), M = num(5, 2), D = num(8, 2), h = num(11, 2), mi = num(14, 2), sec = num(17, 2);
  if (!ok) return false;
  if (M < 1 || M > 12 || D < 1 || h > 23 || mi > 59 || sec > 59) return false;
  const bool leap = (Y % 4 == 0 && Y % 100 != 0) || Y % 400 == 0;
  const int mdays = 28 + (int)((0xeefbb3u >> (2 * (M - 1))) & 3u) + ((M == 2 && leap) ? 1 : 0);
  if (D > mdays) return false;
  int i = pos + 19;
  int frac_ms = 0;
  if (i < end && s[i] == '.') {
    ++i;
    int nd = 0;
    if (i < end && s[i] >= '0' && s[i] <= '9')
      i = digit_run(s, i, end, [&](int g) {
        if (nd < 3) frac_ms = frac_ms * 10 + g;
        ++nd;
      });
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


// the end of the string whose opening quote is at s[pos] (escapes validated, nothing decoded); -1 if malformed
__device__ __forceinline__ int skip_string(const Reader& s, int pos, int end) {
  int i = pos + 1;
  while (i < end) {
    const int c = s[i];
    if (c == '"') return i + 1;
    if (c < 0x20) return -1;
    if (c == '\\') {
      if (i + 1 >= end) return -1;
      const int e = s[i + 1];
      if (e == 'u') {
        if (i + 6 > end) return -1;
        for (int k = 2; k < 6; ++k)
          if (hexval(s[i + k]) < 0) return -1;
        i += 6;
        continue;
      }
      if (e != '"' && e != '\\' && e != '/' && e != 'b' && e != 'f' && e != 'n' && e != 'r' && e != 't') return -1;
      i += 2;
      continue;
    }
    ++i;
  }
  return -1;
}

// skip one JSON value at s[pos], validated by the RFC 8259 grammar (nesting <= 64); returns the index after
// it, -1 if malformed
__device__ __forceinline__ int skip_value(const Reader& s, int pos, int end) {
  enum { VALUE, VALUE_OR_CLOSE, KEY, KEY_OR_CLOSE, COLON, COMMA_OR_CLOSE };
  unsigned long long objects = 0ull;  // bit d: level d+1 is an object (else an array)
  int depth = 0, state = VALUE, i = pos;
  for (;;) {
    while (i < end && is_ws(s[i])) ++i;
    if (i >= end) return -1;
    const int c = s[i];
    bool value_done = false;
    if (state == VALUE || state == VALUE_OR_CLOSE) {
      if (state == VALUE_OR_CLOSE && c == ']') {
        --depth;
        ++i;
        value_done = true;
      } else if (c == '{' || c == '[') {
        if (depth == 64) return -1;
        if (c == '{') objects |= 1ull << depth; else objects &= ~(1ull << depth);
        ++depth;
        ++i;
        state = c == '{' ? KEY_OR_CLOSE : VALUE_OR_CLOSE;
        continue;
      } else if (c == '"') {
        i = skip_string(s, i, end);
        if (i < 0) return -1;
        value_done = true;
      } else if (c == 't' || c == 'f' || c == 'n') {
        const int n = c == 'f' ? 5 : 4;
        if (!lit_at(s, i, end, c == 't' ? "true" : (c == 'f' ? "false" : "null"), n)) return -1;
        i += n;
        value_done = true;
      } else {
        Decimal d;
        i = scan_number_w(s, i, end, d);
        if (i < 0) return -1;
        value_done = true;
      }
    } else if (state == KEY || state == KEY_OR_CLOSE) {
      if (state == KEY_OR_CLOSE && c == '}') {
        --depth;
        ++i;
        value_done = true;
      } else {
        if (c != '"') return -1;
        i = skip_string(s, i, end);
        if (i < 0) return -1;
        state = COLON;
        continue;
      }
    } else if (state == COLON) {
      if (c != ':') return -1;
      ++i;
      state = VALUE;
      continue;
    } else {  // COMMA_OR_CLOSE
      const bool obj = (objects >> (depth - 1)) & 1ull;
      if (c == ',') {
        ++i;
        state = obj ? KEY : VALUE;
        continue;
      }
      if (c != (obj ? '}' : ']')) return -1;
      --depth;
      ++i;
      value_done = true;
    }
    if (value_done) {
      if (depth == 0) return i;
      state = COMMA_OR_CLOSE;
    }
  }
}

__device__ __forceinline__ bool lit_at(const Reader& s, int i, int end, const char* w, int n) {  // NOLINT
  if (i + n > end) return false;
  for (int k = 0; k < n; ++k)
    if (s[i + k] != w[k]) return false;
  return true;
}

__device__ __forceinline__ double nan_d() { return __builtin_nan(""); }

// a location value: {"lat": x, "lon": y, ...} or null, x / y numbers, numeric strings or null. The decimals are
// returned (conversion happens at the caller's single decimal -> binary64 site); has[t] = 0 absent/null, 1 set.
__device__ __forceinline__ int scan_latlon(const Reader& s, int pos, int end, Decimal& d0, Decimal& d1, int& has0,
                                           int& has1) {
  // fast path: the simulator's shape {"lat": x, "lon": y} (numbers or numeric strings, one space after ':' and
  // ','), recognised by dword compares; any other shape -> the general walk below from the start
  if (pos + 8 <= end && s.word(pos) == 0x616C227Bu && s.word(pos + 4) == 0x203A2274u) {  // {"la  t":_
    int i = pos + 8;
    for (int t = 0; t < 2; ++t) {  // one number-scan site for both coordinates
      const bool q = s[i] == '"';
      Decimal tmp;
      int e = scan_number_w(s, q ? i + 1 : i, end, tmp);
      if (e >= 0 && q) e = (e < end && s[e] == '"') ? e + 1 : -1;
      if (e < 0) break;
      if (t == 0) {
        d0 = tmp;
        if (!(e + 9 <= end && s.word(e) == 0x6C22202Cu && s.word(e + 4) == 0x3A226E6Fu && s[e + 8] == ' ')) break;
        i = e + 9;  // ,_"l  on":  _
      } else {
        d1 = tmp;
        if (e >= end || s[e] != '}') break;
        has0 = has1 = 1;
        return e + 1;
      }
    }
  }
  has0 = has1 = 0;
  if (lit_at(s, pos, end, "null", 4)) return pos + 4;
  if (s[pos] != '{') return -1;
  int i = pos + 1;
  while (i < end && is_ws(s[i])) ++i;
  if (i < end && s[i] == '}') return i + 1;
  while (i < end) {
    if (s[i] != '"') return -1;
    const int ks = i;
    i = skip_string(s, i, end);
    if (i < 0) return -1;
    // "lat" / "lon" (unescaped spelling)
    const int t = (i - ks == 5 && s[ks + 1] == 'l' && ((s[ks + 2] == 'a' && s[ks + 3] == 't') ||
                                                         (s[ks + 2] == 'o' && s[ks + 3] == 'n')))
                      ? (s[ks + 2] == 'a' ? 0 : 1)
                      : -1;
    while (i < end && is_ws(s[i])) ++i;
    if (i >= end || s[i] != ':') return -1;
    ++i;
    while (i < end && is_ws(s[i])) ++i;
    if (i >= end) return -1;
    if (t >= 0) {
      if (lit_at(s, i, end, "null", 4)) {
        if (t == 0) has0 = 0; else has1 = 0;
        i += 4;
      } else {
        // a numeric string: the number must end at the closing quote (its characters are never '"' or '\\')
        const bool quoted = s[i] == '"';
        Decimal tmp;
        const int e = scan_number_w(s, quoted ? i + 1 : i, end, tmp);
        if (e < 0 || (quoted && (e >= end || s[e] != '"'))) return -1;
        i = quoted ? e + 1 : e;
        if (t == 0) {
          d0 = tmp;
          has0 = 1;
        } else {
          d1 = tmp;
          has1 = 1;
        }
      }
    } else {
      i = skip_value(s, i, end);
      if (i < 0) return -1;
    }
    while (i < end && is_ws(s[i])) ++i;
    if (i >= end) return -1;
    if (s[i] == '}') return i + 1;
    if (s[i] != ',') return -1;
    ++i;
    while (i < end && is_ws(s[i])) ++i;
  }
  return -1;
}

struct Table {  // open addressing: hash -> value (key 0 = empty)
  const unsigned long long* keys;
  const int* vals;
  unsigned long long mask;
};

__device__ __forceinline__ int table_find(const Table& t, uint64_t h, int miss) {
  if (!t.keys) return miss;
  if (h == 0) h = 1;
  unsigned long long s = fmix64_hd(h ^ 0x9E3779B97F4A7C15ull) & t.mask;
  for (unsigned long long p = 0; p <= t.mask; ++p) {
    const unsigned long long k = t.keys[s];
    if (k == h) return t.vals[s];
    if (k == 0) return miss;
    s = (s + 1) & t.mask;
  }
  return miss;
}

struct Tables {
  Table merchants, vocab[3];
};

// a parsed field value (the lane's member)
struct Val {
  uint64_t u = 0;                // hashes, cents, ts, codes
  double a = 0.0, b = 0.0;       // f64 values (score, lat, lon)
  bool null = true;
};

// 4 waves per SIMD (128 VGPRs, no spills to memory): the members phase is latency-bound per lane, so occupancy
// is the lever (142 VGPRs gave 3 waves per SIMD)
__global__ void __launch_bounds__(64 * kWaves) __attribute__((amdgpu_waves_per_eu(4))) ingest_json_kernel(const unsigned char* __restrict__ buf,
                                                          const int64_t* __restrict__ offsets, int64_t n, Tables T,
                                                          fd_ingest_out out, int stop_after) {
  __shared__ __attribute__((aligned(16))) unsigned char stage[kSlots][kStage + 16];  // + the word reads' tail
  __shared__ int colon[kSlots][kMaxMembers];
  __shared__ int nmem[kSlots], ncomma[kSlots], shift_s[kSlots], len_s[kSlots];
  __shared__ unsigned status_s[kSlots];
  __shared__ int win[kSlots][F_COUNT];

  const int wv = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  // ---- staging: wave w stages messages 2w and 2w+1 of the block's, the first 1 KiB of both loaded before either
  //      is stored (both loads in flight), the rest (messages > 1 KiB) after; one barrier
  const int64_t total_bytes = offsets[n];
  int64_t a0h[2];
  int spanh[2];
  auto load16 = [&](int64_t g) {
    if (g + 16 <= total_bytes) return *reinterpret_cast<const uint4*>(buf + g);
    unsigned wq[4] = {0u, 0u, 0u, 0u};  // the buffer's last partial chunk, byte by byte (no read past its end)
  #pragma unroll
    for (int q = 0; q < 16; ++q)
      if (g + q < total_bytes) wq[q >> 2] |= (unsigned)buf[g + q] << (8 * (q & 3));
    return make_uint4(wq[0], wq[1], wq[2], wq[3]);
  };
  uint4 first[2];
  #pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int ms = 2 * wv + h;
    const int64_t m = (int64_t)blockIdx.x * kSlots + ms;
    const bool live = m < n;
    int64_t off = 0, len = 0;
    if (live) {
      off = offsets[m];
      len = offsets[m + 1] - off;
    }
    if (lane == 0) {
      nmem[ms] = 0;
      ncomma[ms] = 0;
      status_s[ms] = (live && (len > kMaxMsg || len < 0)) ? FD_INGEST_TOO_LONG : 0u;
    }
    if (lane < F_COUNT) win[ms][lane] = -1;
    const bool go = live && len >= 0 && len <= kMaxMsg;
    a0h[h] = off & ~15ll;
    spanh[h] = (int)(off - a0h[h]) + (go ? (int)len : 0);
    if (lane * 16 < spanh[h]) first[h] = load16(a0h[h] + 16ll * lane);
  }
  #pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int ms = 2 * wv + h;
    if (lane * 16 < spanh[h]) *reinterpret_cast<uint4*>(&stage[ms][16 * lane]) = first[h];
    for (int k = lane + 64; k * 16 < spanh[h]; k += 64)
      *reinterpret_cast<uint4*>(&stage[ms][16 * k]) = load16(a0h[h] + 16ll * k);
  }
  __syncthreads();
  // ---- structure: the wave's two messages one after the other
  for (int h = 0; h < 2 && stop_after != 1; ++h) {
    const int ms = 2 * wv + h;
    const int64_t m = (int64_t)blockIdx.x * kSlots + ms;
    const bool live = m < n;
    int64_t off = 0, len = 0;
    if (live) {
      off = offsets[m];
      len = offsets[m + 1] - off;
    }
    const bool go = live && len >= 0 && len <= kMaxMsg;
    const int L = go ? (int)len : 0;
    const int shift = (int)(off & 15ll);
    const Reader s{&stage[ms][0], shift};

    // ---- structure, from registers: lane i owns stage bytes [64i, 64i + 64) (16-B aligned) = message bytes
    //      [q0, q0 + 64) with q0 = 64i - shift, valid where 0 <= q0 + k < L
    // segment width: the staged bytes [0, shift + L) over 64 lanes, a multiple of 4 (4..64); a 750-B message
    // costs 12 bytes per lane instead of a fixed 64
    const int seg_words = max(1, (shift + L + 255) / 256);
    const unsigned* seg = reinterpret_cast<const unsigned*>(&stage[ms][lane * 4 * seg_words]);
    const int q0 = lane * 4 * seg_words - shift;
    // pass 1, the only per-byte pass: the segment's bytes classified into bit masks (bit k = segment byte k; only
    // bytes of the message): quotes, backslashes, opening / closing brackets, colons, commas, non-whitespace
    // message bytes of the segment: k in [klo, khi)
    const int klo = max(0, -q0), khi = min(4 * seg_words, L - q0);
    const unsigned long long vm =
        khi > klo ? ((khi - klo == 64 ? ~0ull : ((1ull << (khi - klo)) - 1ull)) << klo) : 0ull;
    unsigned long long qm = 0, bm = 0, om = 0, cm = 0, km = 0, mm = 0;
    int first_nw = L, last_nw = -1;
  #pragma unroll 2
    for (int j = 0; j < seg_words; ++j) {
      const unsigned w = seg[j];
      unsigned nq = 0, nb = 0, no = 0, nc = 0, nk = 0, nm4 = 0, nn = 0;
  #pragma unroll
      for (int b = 0; b < 4; ++b) {
        const int c = (int)((w >> (8 * b)) & 0xFFu);
        const bool v = (unsigned)(q0 + 4 * j + b) < (unsigned)L;
        const int c20 = c | 0x20;  // '[' -> '{', ']' -> '}'
        nq |= (v && c == '"' ? 1u : 0u) << b;
        nb |= (v && c == '\\' ? 1u : 0u) << b;
        no |= (v && c20 == '{' ? 1u : 0u) << b;
        nc |= (v && c20 == '}' ? 1u : 0u) << b;
        nk |= (v && c == ':' ? 1u : 0u) << b;
        nm4 |= (v && c == ',' ? 1u : 0u) << b;
        nn |= (v && !is_ws(c) ? 1u : 0u) << b;
      }
      const int sh = 4 * j;
      if (nn) {
        first_nw = min(first_nw, q0 + sh + (__ffs((int)nn) - 1));
        last_nw = q0 + sh + (31 - __clz((int)nn));
      }
      qm |= (unsigned long long)nq << sh;
      bm |= (unsigned long long)nb << sh;
      om |= (unsigned long long)no << sh;
      cm |= (unsigned long long)nc << sh;
      km |= (unsigned long long)nk << sh;
      mm |= (unsigned long long)nm4 << sh;
    }
    // escape carry into the next lane: the backslash run ending at the segment's last message byte
    int run = 0;
    if (vm) {
      const int top = 63 - __clzll(vm);
      const unsigned long long below = (top == 63) ? ~0ull : ((2ull << top) - 1ull);
      const unsigned long long nonbs = vm & ~bm & below;
      run = nonbs ? top - (63 - __clzll(nonbs)) : __popcll(vm);
    }
    int bs0 = __shfl_up(run, 1);
    if (lane == 0) bs0 = 0;
    if (__ballot(vm != 0ull && bm == vm) != 0ull) {  // a segment of only backslashes: exact carry from LDS
      int b2 = 0;
      for (int p = q0 - 1; p >= 0 && q0 < L && s[p] == '\\'; --p) ++b2;
      bs0 = b2;
    }
    // escaped bytes (after an odd backslash run, the carry included): only lanes with a backslash or an odd carry
    unsigned long long esc = 0;
    if (bm != 0ull || (bs0 & 1)) {
      int r = bs0;
      for (unsigned long long x = vm; x; x &= x - 1) {
        const int k = __ffsll((long long)x) - 1;
        if (r & 1) esc |= 1ull << k;
        r = ((bm >> k) & 1ull) ? r + 1 : 0;
      }
    }
    const unsigned long long uq = qm & ~esc;  // string delimiters
    const int par = __popcll(uq) & 1;
    for (int d = 32; d >= 1; d >>= 1) {
      first_nw = min(first_nw, __shfl_xor(first_nw, d));
      last_nw = max(last_nw, __shfl_xor(last_nw, d));
    }
    const unsigned long long pb = __ballot(par);
    const unsigned long long lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    const int in0 = __popcll(pb & lt) & 1;
    const int total_par = __popcll(pb) & 1;
    // inside a string: the inclusive prefix XOR of the delimiters, flipped by the state at the segment start
    unsigned long long instr = uq;
    instr ^= instr << 1;
    instr ^= instr << 2;
    instr ^= instr << 4;
    instr ^= instr << 8;
    instr ^= instr << 16;
    instr ^= instr << 32;
    if (in0) instr = ~instr;
    const unsigned long long oo = om & ~instr, oc = cm & ~instr;  // brackets outside strings
    // pass 2: the bracket depth delta -> wave prefix sum
    const int delta = __popcll(oo) - __popcll(oc);
    int depth0 = delta;  // inclusive prefix sum over lanes
    for (int d = 1; d < 64; d <<= 1) {
      const int v = __shfl_up(depth0, d);
      if (lane >= d) depth0 += v;
    }
    const int total_depth = __shfl(depth0, 63);
    depth0 -= delta;
    // pass 3, over the structural bytes outside strings only: depth-1 colons (members), depth-1 commas, the first
    // return to depth 0, and a depth below 0 anywhere (malformed)
    bool bad = false;
    int depth = depth0, zero_at = L;
    for (unsigned long long x = (oo | oc | km | mm) & ~instr; x; x &= x - 1) {
      const int k = __ffsll((long long)x) - 1;
      const unsigned long long bit = 1ull << k;
      const int p = q0 + k;
      if (km & bit) {
        if (depth == 1) {
          const int slot = atomicAdd(&nmem[ms], 1);
          if (slot < kMaxMembers) colon[ms][slot] = p;
        }
      } else if (mm & bit) {
        if (depth == 1) atomicAdd(&ncomma[ms], 1);
      } else if (oo & bit) {
        ++depth;
      } else {
        --depth;
        bad = bad || depth < 0;
        if (depth == 0) zero_at = min(zero_at, p);
      }
    }
    for (int d = 32; d >= 1; d >>= 1) zero_at = min(zero_at, __shfl_xor(zero_at, d));
    bad = bad || (__ballot(bad) != 0ull);
    if (go && lane == 0) {
      const bool ok = !bad && L > 0 && total_par == 0 && total_depth == 0 && first_nw < L && s[first_nw] == '{' &&
                      zero_at == last_nw;
      if (!ok) status_s[ms] |= FD_INGEST_MALFORMED;
    }
    __syncthreads();
    const int nm = go ? nmem[ms] : 0;
    if (go && lane == 0 && status_s[ms] == 0u) {
      // member skeleton: n members <-> n-1 depth-1 commas; an empty object holds only whitespace
      bool bad_skel = nm > kMaxMembers || (nm > 0 && ncomma[ms] != nm - 1) || (nm == 0 && ncomma[ms] != 0);
      if (nm == 0) {
        int q = first_nw + 1;
        while (q < L && is_ws(s[q])) ++q;
        bad_skel = bad_skel || q != zero_at;
      }
      if (bad_skel) status_s[ms] |= FD_INGEST_MALFORMED;
    }
    __syncthreads();
    const bool structural_ok = go && status_s[ms] == 0u;
    if (lane == 0) {
      shift_s[ms] = shift;
      len_s[ms] = go ? L : -1;
    }
  }
  __syncthreads();
  if (stop_after == 2) return;

  // ---- members: two messages per wave — half h = lane >> 5 parses message 2w+h, lane j = lane & 31 its members
  //      j and j + 32 (the divergent member code is paid once for both messages)
  const int ms = 2 * wv + (lane >> 5);
  const int64_t m = (int64_t)blockIdx.x * kSlots + ms;
  const bool live = m < n;
  const int L = len_s[ms] < 0 ? 0 : len_s[ms];
  const bool go = live && len_s[ms] >= 0;
  const Reader s{&stage[ms][0], shift_s[ms]};
  const int nm = go ? min(nmem[ms], kMaxMembers) : 0;
  const bool structural_ok = go && status_s[ms] == 0u;
  int my_field0 = -1, my_colon0 = -1, my_field1 = -1, my_colon1 = -1;
  Val my0, my1;
  unsigned my_status = 0;
  // user-agent string members are deferred to the cooperative scan below (r = 0 / 1: member j / j + 32)
  bool ua_pend0 = false, ua_pend1 = false;
  int ua_v0 = 0, ua_v1 = 0, ua_c0 = 0, ua_c1 = 0;
  for (int r = 0; r < 2; ++r) {
  const int mi = 32 * r + (lane & 31);
  for (int once = 0; once < 1 && structural_ok && mi < nm; ++once) {  // `continue` = member rejected
    const int c = colon[ms][mi];
    // key: the string ending right before the colon
    int kc = c - 1;
    while (kc >= 0 && is_ws(s[kc])) --kc;
    if (kc < 1 || s[kc] != '"') {
      my_status |= FD_INGEST_MALFORMED;
      continue;
    }
    // the key's opening quote: the last unescaped '"' before kc, four bytes per LDS access
    int ko = kc - 1;
    while (ko >= 0) {
      const int lo = max(ko - 3, 0);
      const unsigned z = exact_zero_mask(s.word(lo) ^ 0x22222222u) & (0xFFFFFFFFu >> (8 * (3 - (ko - lo))));
      if (!z) {
        ko = lo - 1;
        continue;
      }
      const int q = lo + ((31 - __builtin_clz(z)) >> 3);
      int r = 0;
      for (int b = q - 1; b >= 0 && s[b] == '\\'; --b) ++r;
      ko = q;
      if (!(r & 1)) break;
      --ko;
    }
    int pre = ko - 1;
    while (pre >= 0 && is_ws(s[pre])) --pre;
    if (ko < 0 || pre < 0 || (s[pre] != '{' && s[pre] != ',')) {
      my_status |= FD_INGEST_MALFORMED;
      continue;
    }
    StrStats<false> key;
    if (scan_string(s, ko, L, key) != kc + 1) {
      my_status |= FD_INGEST_MALFORMED;
      continue;
    }
    const int f = field_of_key(key.fnv);
    int v = c + 1;
    while (v < L && is_ws(s[v])) ++v;
    if (v >= L) {
      my_status |= FD_INGEST_MALFORMED;
      continue;
    }
    int e = -1;
    if (f == F_UA && s[v] == '"') {  // the message's longest string: scanned by the whole wave below
      if (r == 0) {
        ua_pend0 = true;
        ua_v0 = v;
        ua_c0 = c;
      } else {
        ua_pend1 = true;
        ua_v1 = v;
        ua_c1 = c;
      }
      continue;
    }
    // ---- one token scan per member: string / literal / number / location object. An unknown property
    //      (f < 0: validated, then ignored — @JsonIgnoreProperties(ignoreUnknown = true)) shares the scalar
    //      scans; only an object / array value takes the generic skip_value walk.
    Val val;
    val.null = false;
    const int ch = s[v];
    int kind = -1;  // 0 null, 1 string, 2 number, 3 true, 4 false, 5 location, 6 skipped structure
    StrStats<false> st;
    Decimal dec0, dec1;
    int has0 = 0, has1 = 0;
    int num_a = -1, num_b = L;
    if (f == F_GEO || f == F_MLOC) {
      e = scan_latlon(s, v, L, dec0, dec1, has0, has1);
      kind = 5;
    } else if (ch == '"') {
      e = scan_string(s, v, L, st);
      kind = 1;
      if (e >= 0 && (f == F_AMOUNT || f == F_SCORE || f == F_HOUR)) {  // numeric string
        if (st.escaped) e = -1;
        num_a = v + 1;
        num_b = e - 1;
      }
    } else if (lit_at(s, v, L, "null", 4)) {
      e = v + 4;
      kind = 0;
    } else if (lit_at(s, v, L, "true", 4)) {
      e = v + 4;
      kind = 3;
    } else if (lit_at(s, v, L, "false", 5)) {
      e = v + 5;
      kind = 4;
    } else if (ch == '-' || (ch >= '0' && ch <= '9')) {
      kind = 2;
      num_a = v;
    } else if (f < 0 && (ch == '{' || ch == '[')) {
      e = skip_value(s, v, L);
      kind = 6;
    }
    if (e < 0 && kind != 2) {
      my_status |= FD_INGEST_MALFORMED;
      continue;
    }
    if (num_a >= 0 && e >= -1) {  // the single number scan
      const int ne = scan_number_w(s, num_a, num_b, dec0);
      if (kind == 2) e = ne;
      else if (ne != num_b) e = -1;
      has0 = e >= 0 ? 1 : 0;
    }
    if (e < 0) {
      my_status |= FD_INGEST_MALFORMED;
      continue;
    }
    if (kind == 0) val.null = true;
    // literal text of a scalar bound to a String property (Jackson's scalar -> String coercion)
    if ((kind == 2 || kind == 3 || kind == 4) && f >= 0 && f != F_AMOUNT && f != F_SCORE && f != F_HOUR &&
        f != F_WEEKEND && f != F_FRAUD) {
      for (int q = v; q < e; ++q) st.byte((unsigned)s[q]);
      kind = 1;
    }
    bool bad = false;
    switch (f) {
      case F_TXN_ID: case F_USER_ID: case F_MERCHANT_ID: case F_IP: case F_DEVICE_FP: case F_UA:
      case F_PAY: case F_TTYPE: case F_CTYPE: {
        if (kind != 1) break;  // null
        const uint64_t h = hash_finish(st.fnv);
        if (f == F_IP) {
          const bool priv = (st.nbytes >= 8 && st.head == 0x2E3836312E323931ull) ||            // "192.168."
                            (st.nbytes >= 3 && (st.head & 0xFFFFFFull) == 0x2E3031ull) ||       // "10."
                            (st.nbytes >= 7 && (st.head & 0xFFFFFFFFFFFFFFull) == 0x2E36312E323731ull);  // "172.16."
          val.u = priv ? 1 : 2;
        } else if (f == F_UA) {  // literal text only (strings are deferred): ASCII, no "bot" / "crawler"
          val.u = st.nbytes < 20 ? 1 : 0;
        } else if (f == F_MERCHANT_ID) {
          val.u = (uint64_t)(int64_t)table_find(T.merchants, h, -1);
        } else if (f == F_PAY || f == F_TTYPE || f == F_CTYPE) {
          const int code = table_find(T.vocab[f - F_PAY], h, FD_VOCAB_OTHER);
          if (code == FD_VOCAB_OTHER) my_status |= FD_INGEST_UNKNOWN_VOCAB;
          val.u = (uint64_t)code;
        } else {
          val.u = h;
        }
        break;
      }
      case F_AMOUNT: {
        if (kind == 0) break;
        if (!has0) {
          bad = true;
          break;
        }
        bool inexact = false;
        int64_t cents;
        if (!decimal_to_cents(dec0, &cents, &inexact)) {
          bad = true;
          break;
        }
        if (inexact) my_status |= FD_INGEST_INEXACT;
        val.u = (uint64_t)cents;
        break;
      }
      case F_SCORE: case F_GEO: case F_MLOC:
        if (f == F_SCORE && kind != 0 && !has0) bad = true;
        break;  // decimals converted below
      case F_TIMESTAMP: {
        if (kind == 0) break;
        int64_t ms;
        if (kind != 1 || st.escaped || !parse_iso_w(s, v + 1, e - 1, &ms)) {
          bad = true;
          break;
        }
        val.u = (uint64_t)ms;
        break;
      }
      case F_WEEKEND: case F_FRAUD: {
        if (kind == 3 || kind == 4) {
          val.u = kind == 3 ? 1 : 0;
        } else if (kind == 1 && !st.escaped && st.nbytes == 4 && st.head == 0x65757274ull) {  // "true"
          val.u = 1;
        } else if (kind == 1 && !st.escaped && st.nbytes == 5 && st.head == 0x65736C6166ull) {  // "false"
          val.u = 0;
        } else if (kind == 2 && !dec0.frac_or_exp) {  // integer coercion: 0 -> false, other -> true
          val.u = dec0.w != 0 ? 1 : 0;
        } else if (kind != 0) {
          bad = true;
        }
        break;
      }
      case F_HOUR: {
        if (kind == 0) break;
        const Decimal& d = dec0;
        if (!has0) {
          bad = true;
          break;
        }
        // integer value (a fraction truncates toward zero, Jackson ACCEPT_FLOAT_AS_INT); hours 0..254
        int64_t iv = 0;
        bool ok = !d.neg || d.w == 0;
        if (ok && d.w) {
          if (d.q >= 0) {
            ok = d.w <= 254 && d.q <= 3;
            iv = (int64_t)d.w;
            for (int k = 0; ok && k < d.q; ++k) iv *= 10;
          } else if (-d.q <= 19) {
            uint64_t p = 1;
            for (int k = 0; k < -d.q; ++k) p *= 10;
            iv = (int64_t)(d.w / p);
          }
        }
        if (!ok || iv > 254) {
          bad = true;
          break;
        }
        val.u = (uint64_t)iv;
        break;
      }
      default: break;
    }
    // the single decimal -> binary64 site: fraud score, or the two coordinates of a location
    if (!bad && (f == F_SCORE || f == F_GEO || f == F_MLOC)) {
      val.a = val.b = nan_d();
      for (int t = 0; t < 2; ++t) {
        const bool h = t == 0 ? has0 : (f != F_SCORE && has1);
        if (!h) continue;
        const Decimal d = t == 0 ? dec0 : dec1;
        bool amb = false;
        const double x = decimal_to_double(d.w, d.q, d.neg, d.many, &amb);
        if (amb) my_status |= FD_INGEST_INEXACT;
        if (t == 0) val.a = x; else val.b = x;
      }
    }
    if (bad) {
      my_status |= FD_INGEST_MALFORMED;
      continue;
    }
    while (e < L && is_ws(s[e])) ++e;
    if (e >= L || (s[e] != ',' && s[e] != '}')) {
      my_status |= FD_INGEST_MALFORMED;
      continue;
    }
    if (f < 0) continue;  // an ignored property, validated
    if (r == 0) {
      my_field0 = f;
      my_colon0 = c;
      my0 = val;
    } else {
      my_field1 = f;
      my_colon1 = c;
      my1 = val;
    }
    atomicMax(&win[ms][f], c);
  }
  }
  // ---- deferred user-agent strings (FeatureExtractor.analyzeSuspiciousUserAgent needs only the "bot" /
  //      "crawler" substrings of the decoded string and its UTF-16 length): the whole wave walks each one 64
  //      bytes per step. Lane p's backslash-run parity (read backwards) marks escape starts and escaped
  //      characters, the escaped 'u's mark their 4 hex digits; the end is the first unescaped quote or
  //      control byte (ballot). UTF-16 units = raw lead bytes (+1 for 4-byte leads) + one per escape; a
  //      substring match starts on a raw byte (escapes decode to non-letters, so they only break matches).
  //      Escapes the scan cannot price exactly — \u00XX below 0x80 (an ASCII letter could join a match) or
  //      invalid ones — send the string back to its lane's serial decoder.
  int ua_e0 = -1, ua_e1 = -1;
  unsigned ua_f0 = 0, ua_f1 = 0;
  bool ua_serial0 = false, ua_serial1 = false;
  for (int r = 0; r < 2; ++r) {
    unsigned long long pend = __ballot(r == 0 ? ua_pend0 : ua_pend1);
    while (pend) {
      const int owner = __ffsll((long long)pend) - 1;
      pend &= pend - 1;
      const int vpos = __shfl(r == 0 ? ua_v0 : ua_v1, owner);
      const int oms = 2 * wv + (owner >> 5);
      const Reader so{&stage[oms][0], shift_s[oms]};
      const int oL = len_s[oms];
      int units = 0, endq = -1, how = 0;  // how: 1 closing quote, 2 serial fallback, 3 control byte / end
      bool hit = false;
      unsigned long long u_prev = 0ull;
      for (int base = vpos + 1;; base += 64) {
        const int p = base + lane;
        const int ch = p < oL ? so[p] : 0;
        int run = 0;  // backslashes right before p, inside the string
        for (int q = p - 1; q > vpos && so[q] == '\\'; --q) ++run;
        const bool escaped = run & 1;
        const bool esc_start = ch == '\\' && !escaped;
        const unsigned long long U = __ballot(escaped && ch == 'u');
        const unsigned long long hexcov_m = (U << 1) | (U << 2) | (U << 3) | (U << 4) | (u_prev >> 63) |
                                            (u_prev >> 62) | (u_prev >> 61) | (u_prev >> 60);
        u_prev = U;
        const bool hexcov = (hexcov_m >> lane) & 1ull;
        const bool covered = escaped || esc_start || hexcov;
        const bool is_hex = (ch >= '0' && ch <= '9') || (ch >= 'a' && ch <= 'f') || (ch >= 'A' && ch <= 'F');
        bool odd = hexcov && !is_hex;
        if (escaped && !hexcov)
          odd = odd || !(ch == '"' || ch == '\\' || ch == '/' || ch == 'b' || ch == 'f' || ch == 'n' ||
                         ch == 'r' || ch == 't' || ch == 'u');
        if (escaped && ch == 'u' && p + 3 < oL)  // \u00XX with XX < 0x80: decodes to ASCII
          odd = odd || (so[p + 1] == '0' && so[p + 2] == '0' && so[p + 3] >= '0' && so[p + 3] <= '7');
        const unsigned long long stop = __ballot(ch < 0x20 || (ch == '"' && !escaped && !hexcov));
        const int first = stop ? __ffsll((long long)stop) - 1 : 64;
        const bool content = lane < first;
        if (__ballot(odd && lane <= first) != 0ull) {
          how = 2;
          break;
        }
        const bool raw = content && !covered;
        units += __popcll(__ballot(raw && (ch & 0xC0) != 0x80)) + __popcll(__ballot(raw && ch >= 0xF0)) +
                 __popcll(__ballot(content && esc_start));
        bool m = false;
        if (raw && ch == 'b' && p + 2 < oL) m = so[p + 1] == 'o' && so[p + 2] == 't';
        if (raw && ch == 'c' && p + 6 < oL) {
          const int c1 = so[p + 1], c2 = so[p + 2], c3 = so[p + 3], c4 = so[p + 4], c5 = so[p + 5], c6 = so[p + 6];
          m = c1 == 'r' && c2 == 'a' && c3 == 'w' && c4 == 'l' && c5 == 'e' && c6 == 'r';
        }
        hit = hit || __ballot(m) != 0ull;
        if (stop) {
          endq = base + first;
          how = __shfl(ch, first) == '"' ? 1 : 3;
          break;
        }
      }
      if (lane == owner) {
        const int e = how == 1 ? endq + 1 : -1;
        const unsigned flag = (hit || units < 20) ? 1u : 0u;
        if (r == 0) {
          ua_e0 = e;
          ua_f0 = flag;
          ua_serial0 = how == 2;
        } else {
          ua_e1 = e;
          ua_f1 = flag;
          ua_serial1 = how == 2;
        }
      }
    }
  }
  for (int r = 0; r < 2; ++r) {  // each owner finishes its user-agent members as the member loop would
    if (!(r == 0 ? ua_pend0 : ua_pend1)) continue;
    const int v = r == 0 ? ua_v0 : ua_v1, c = r == 0 ? ua_c0 : ua_c1;
    int e = r == 0 ? ua_e0 : ua_e1;
    unsigned flag = r == 0 ? ua_f0 : ua_f1;
    if (r == 0 ? ua_serial0 : ua_serial1) {
      StrStats<true> st;
      e = scan_string(s, v, L, st);
      flag = (st.bot || st.crawler || st.units < 20) ? 1u : 0u;
    }
    if (e < 0) {
      my_status |= FD_INGEST_MALFORMED;
      continue;
    }
    while (e < L && is_ws(s[e])) ++e;
    if (e >= L || (s[e] != ',' && s[e] != '}')) {
      my_status |= FD_INGEST_MALFORMED;
      continue;
    }
    Val val;
    val.null = false;
    val.u = flag;
    if (r == 0) {
      my_field0 = F_UA;
      my_colon0 = c;
      my0 = val;
    } else {
      my_field1 = F_UA;
      my_colon1 = c;
      my1 = val;
    }
    atomicMax(&win[ms][F_UA], c);
  }
  if (my_status) atomicOr(&status_s[ms], my_status);
  __syncthreads();
  if (stop_after == 3) {
    if (live && (lane & 31) == 0 && out.status) out.status[m] = (unsigned char)(my_field0 + my_colon1);  // keep the work
    return;
  }
  // ---- resolve: the winner of each field publishes its value to LDS, then lane f writes column f
  __shared__ unsigned long long vu[kSlots][F_COUNT];
  __shared__ double va[kSlots][F_COUNT], vb[kSlots][F_COUNT];
  __shared__ unsigned char vnull[kSlots][F_COUNT];
  if (go && my_field0 >= 0 && win[ms][my_field0] == my_colon0) {
    vu[ms][my_field0] = my0.u;
    va[ms][my_field0] = my0.a;
    vb[ms][my_field0] = my0.b;
    vnull[ms][my_field0] = my0.null ? 1 : 0;
  }
  if (go && my_field1 >= 0 && win[ms][my_field1] == my_colon1) {
    vu[ms][my_field1] = my1.u;
    va[ms][my_field1] = my1.a;
    vb[ms][my_field1] = my1.b;
    vnull[ms][my_field1] = my1.null ? 1 : 0;
  }
  __syncthreads();
  if (!live) return;
  unsigned st = status_s[ms];
  const bool valid_struct = (st & (FD_INGEST_MALFORMED | FD_INGEST_TOO_LONG)) == 0;
  auto present = [&](int f) { return valid_struct && win[ms][f] >= 0 && !vnull[ms][f]; };
  if (valid_struct && (!present(F_USER_ID) || !present(F_AMOUNT) || !present(F_TIMESTAMP))) st |= FD_INGEST_MISSING;
  const bool ok = (st & (FD_INGEST_MALFORMED | FD_INGEST_TOO_LONG | FD_INGEST_MISSING)) == 0;
  if (!ok) st &= (FD_INGEST_MALFORMED | FD_INGEST_TOO_LONG | FD_INGEST_MISSING);  // an invalid row: its class only
  const int f = lane & 31;
  if (f < F_COUNT) {
    const bool p = ok && present(f);
    const unsigned long long u = p ? vu[ms][f] : 0ull;
    const double A = p ? va[ms][f] : nan_d(), B = p ? vb[ms][f] : nan_d();
    switch (f) {
      case F_TXN_ID: if (out.txn_hash) out.txn_hash[m] = u; break;
      case F_USER_ID: if (out.card_key) out.card_key[m] = u; break;
      case F_MERCHANT_ID: if (out.merchant) out.merchant[m] = p ? (int)(long long)u : -1; break;
      case F_AMOUNT: if (out.amount_cents) out.amount_cents[m] = (long long)u; break;
      case F_TIMESTAMP: if (out.ts_ms) out.ts_ms[m] = (long long)u; break;
      case F_IP: if (out.ip_class) out.ip_class[m] = p ? (unsigned char)u : 0; break;
      case F_DEVICE_FP: if (out.device_fp) out.device_fp[m] = u; break;
      case F_UA: if (out.user_agent_flag) out.user_agent_flag[m] = p ? (unsigned char)u : 255; break;
      case F_GEO:
        if (out.geo_lat) out.geo_lat[m] = A;
        if (out.geo_lon) out.geo_lon[m] = B;
        break;
      case F_MLOC:
        if (out.merchant_lat) out.merchant_lat[m] = A;
        if (out.merchant_lon) out.merchant_lon[m] = B;
        break;
      case F_WEEKEND: if (out.weekend) out.weekend[m] = p ? (unsigned char)u : 255; break;
      case F_HOUR: if (out.hour) out.hour[m] = p ? (unsigned char)u : 255; break;
      case F_FRAUD: if (out.is_fraud) out.is_fraud[m] = p ? (unsigned char)u : 0; break;
      case F_SCORE: if (out.fraud_score) out.fraud_score[m] = A; break;
      case F_PAY: if (out.payment_method) out.payment_method[m] = p ? (unsigned char)u : 255; break;
      case F_TTYPE: if (out.transaction_type) out.transaction_type[m] = p ? (unsigned char)u : 255; break;
      case F_CTYPE: if (out.card_type) out.card_type[m] = p ? (unsigned char)u : 255; break;
      default: break;
    }
  } else if (f == 31 && out.status) {
    out.status[m] = (unsigned char)st;
  }
}

}  // namespace

// ---------------------------------------------------------------- host side

namespace {

void build_table(DeviceBuffer& keys, DeviceBuffer& vals, unsigned long long* mask, const uint8_t* bytes,
                 const int64_t* offsets, int64_t n, hipStream_t stream) {
  uint64_t cap = 16;
  while (cap < (uint64_t)std::max<int64_t>(n, 1) * 2) cap <<= 1;
  std::vector<unsigned long long> k(cap, 0ull);
  std::vector<int> v(cap, -1);
  for (int64_t i = 0; i < n; ++i) {
    FD_REQUIRE(offsets[i + 1] >= offsets[i], FD_ERR_INVALID_ARG, "vocabulary offsets must be non-decreasing");
    uint64_t h = hash_bytes(bytes + offsets[i], offsets[i + 1] - offsets[i]);
    if (h == 0) h = 1;
    uint64_t s = fmix64_hd(h ^ 0x9E3779B97F4A7C15ull) & (cap - 1);
    while (k[s] != 0ull && k[s] != h) s = (s + 1) & (cap - 1);
    if (k[s] == h) continue;  // duplicate string: the first position keeps its index
    k[s] = h;
    v[s] = (int)i;
  }
  keys.ensure(cap * 8);
  vals.ensure(cap * 4);
  FD_HIP(hipMemcpyAsync(keys.ptr, k.data(), cap * 8, hipMemcpyHostToDevice, stream));
  FD_HIP(hipMemcpyAsync(vals.ptr, v.data(), cap * 4, hipMemcpyHostToDevice, stream));
  FD_HIP(hipStreamSynchronize(stream));
  *mask = cap - 1;
}

}  // namespace

void ingest_set_vocab(Engine& e, int which, const uint8_t* bytes, const int64_t* offsets, int64_t n) {
  FD_REQUIRE(which >= 0 && which < 3, FD_ERR_INVALID_ARG, "unknown vocabulary");
  FD_REQUIRE(n >= 0 && n <= FD_VOCAB_OTHER, FD_ERR_INVALID_ARG, "a vocabulary holds at most 254 strings");
  FD_REQUIRE(n == 0 || (bytes && offsets), FD_ERR_INVALID_ARG, "null vocabulary");
  IngestTables& t = e.ingest;
  build_table(t.vkeys[which], t.vvals[which], &t.vmask[which], bytes, offsets, n, e.stream);
  t.vloaded[which] = true;
}

void ingest_set_merchants(Engine& e, const uint8_t* bytes, const int64_t* offsets, int64_t n) {
  FD_REQUIRE(n >= 0 && n < (1ll << 31), FD_ERR_INVALID_ARG, "merchant count out of range");
  FD_REQUIRE(n == 0 || (bytes && offsets), FD_ERR_INVALID_ARG, "null merchant ids");
  IngestTables& t = e.ingest;
  build_table(t.mkeys, t.mvals, &t.mmask, bytes, offsets, n, e.stream);
  t.mloaded = true;
}

void launch_ingest(Engine& e, const uint8_t* d_bytes, const int64_t* d_offsets, int64_t n, const fd_ingest_out& out) {
  FD_REQUIRE(n >= 0 && n <= (1ll << 30), FD_ERR_INVALID_ARG, "message count out of range (<= 2^30 per call)");
  FD_REQUIRE(d_offsets, FD_ERR_INVALID_ARG, "null offsets");
  if (n == 0) return;
  FD_REQUIRE(d_bytes, FD_ERR_INVALID_ARG, "null message bytes");
  IngestTables& t = e.ingest;
  Tables T{};
  if (t.mloaded) T.merchants = Table{t.mkeys.as<const unsigned long long>(), t.mvals.as<const int>(), t.mmask};
  for (int w = 0; w < 3; ++w)
    if (t.vloaded[w]) T.vocab[w] = Table{t.vkeys[w].as<const unsigned long long>(), t.vvals[w].as<const int>(), t.vmask[w]};
  Engine::Timed* ev = e.timing ? e.next_event_pair(FD_TIMING_INGEST) : nullptr;
  if (ev) FD_HIP(hipEventRecord(ev->a, e.stream));
  const int64_t blocks = (n + kSlots - 1) / kSlots;
  hipLaunchKernelGGL(ingest_json_kernel, dim3((unsigned)blocks), dim3(64 * kWaves), 0, e.stream, d_bytes, d_offsets, n, T, out,
                     t.stop_after);
  FD_HIP(hipGetLastError());
  if (ev) FD_HIP(hipEventRecord(ev->b, e.stream));
}

}  // namespace fd

// Bulk JSON encoding of the streaming classifier's output records (N-09, output side).
//
// For record i the bytes are exactly what Python's json.dumps produces (default settings:
// ensure_ascii=True, ", " / ": " separators, float repr) for
//   {"prediction": p, "confidence": c, "analysis": null, "historical_insight": null,
//    "original_text": text_i}
// (the Kafka output contract of /root/reference/app_ui.py:218-225), so the engine can hand the
// producer ready-made values instead of building a dict and calling json.dumps per message.
// status[i]: 0 ok, 1 text is not valid UTF-8 (the caller encodes that record itself), 2 skipped.
// Two multi-threaded passes: exact lengths, then prefix offsets + write.
#include <charconv>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "parallel_for.h"
#include "swar.h"

namespace fdx {

namespace {

// Python float repr ('r' mode, float_repr_style 'short'): shortest round-trip digits, fixed
// notation when -4 <= exponent < 16, else d[.ddd]e[+-]XX. json.dumps spells nan/inf as
// NaN/Infinity/-Infinity.
int py_float_repr(double v, char* out) {
  if (std::isnan(v)) { std::memcpy(out, "NaN", 3); return 3; }
  if (std::isinf(v)) {
    if (v < 0) { std::memcpy(out, "-Infinity", 9); return 9; }
    std::memcpy(out, "Infinity", 8);
    return 8;
  }
  char* o = out;
  if (std::signbit(v)) { *o++ = '-'; v = -v; }
  if (v == 0.0) { std::memcpy(o, "0.0", 3); return (int)(o - out) + 3; }
  char sci[40];
  const auto r = std::to_chars(sci, sci + sizeof(sci) - 1, v, std::chars_format::scientific);
  *r.ptr = '\0';
  const char* e = sci;
  while (e < r.ptr && *e != 'e') ++e;
  char digits[24];
  int nd = 0;
  for (const char* p = sci; p < e; ++p) if (*p != '.') digits[nd++] = *p;
  const int exp10 = std::atoi(e + 1);
  if (exp10 >= -4 && exp10 < 16) {
    if (exp10 >= 0) {
      const int ip = exp10 + 1;
      for (int i = 0; i < ip; ++i) *o++ = i < nd ? digits[i] : '0';
      *o++ = '.';
      if (nd > ip) for (int i = ip; i < nd; ++i) *o++ = digits[i];
      else *o++ = '0';
    } else {
      *o++ = '0';
      *o++ = '.';
      for (int i = 0; i < -exp10 - 1; ++i) *o++ = '0';
      for (int i = 0; i < nd; ++i) *o++ = digits[i];
    }
  } else {
    *o++ = digits[0];
    if (nd > 1) {
      *o++ = '.';
      for (int i = 1; i < nd; ++i) *o++ = digits[i];
    }
    *o++ = 'e';
    *o++ = exp10 < 0 ? '-' : '+';
    const int ax = exp10 < 0 ? -exp10 : exp10;
    if (ax < 10) *o++ = '0';
    char eb[8];
    const auto er = std::to_chars(eb, eb + sizeof(eb), ax);
    for (const char* p = eb; p < er.ptr; ++p) *o++ = *p;
  }
  return (int)(o - out);
}

const char kHex[] = "0123456789abcdef";

inline void put_u16(uint8_t*& o, uint32_t u) {
  o[0] = '\\'; o[1] = 'u';
  o[2] = kHex[(u >> 12) & 15]; o[3] = kHex[(u >> 8) & 15]; o[4] = kHex[(u >> 4) & 15]; o[5] = kHex[u & 15];
  o += 6;
}

// Decode one UTF-8 code point at s[i]; returns bytes consumed or 0 if invalid (overlong forms,
// surrogates, > U+10FFFF and truncated sequences are invalid, as in Python's strict decoder).
inline int utf8_next(const uint8_t* s, int64_t n, int64_t i, uint32_t* cp) {
  const uint8_t c = s[i];
  if (c < 0x80) { *cp = c; return 1; }
  int len;
  uint32_t v, lo;
  if (c >= 0xC2 && c <= 0xDF) { len = 2; v = c & 0x1F; lo = 0x80; }
  else if (c >= 0xE0 && c <= 0xEF) { len = 3; v = c & 0x0F; lo = 0x800; }
  else if (c >= 0xF0 && c <= 0xF4) { len = 4; v = c & 0x07; lo = 0x10000; }
  else return 0;
  if (i + len > n) return 0;
  for (int k = 1; k < len; ++k) {
    const uint8_t t = s[i + k];
    if ((t & 0xC0) != 0x80) return 0;
    v = (v << 6) | (t & 0x3F);
  }
  if (v < lo || v > 0x10FFFF || (v >= 0xD800 && v <= 0xDFFF)) return 0;
  *cp = v;
  return len;
}

// JSON string body (without quotes) with ensure_ascii escapes; out == nullptr -> length only.
// Returns -1 on invalid UTF-8.
int64_t escape_ascii(const uint8_t* s, int64_t n, uint8_t* out) {
  int64_t len = 0;
  uint8_t* o = out;
  for (int64_t i = 0; i < n;) {
    while (n - i >= 8) {             // printable ASCII without quote / backslash: 8 at a time
      const uint64_t w = swar_load(s + i);
      if (swar_has_less(w, 0x20) || swar_has_byte(w, '"') || swar_has_byte(w, '\\') || swar_has_7f_or_high(w)) break;
      if (o) { std::memcpy(o, s + i, 8); o += 8; }
      len += 8;
      i += 8;
    }
    if (i >= n) break;
    uint32_t cp;
    const int k = utf8_next(s, n, i, &cp);
    if (k == 0) return -1;
    i += k;
    if (cp >= 0x20 && cp <= 0x7E && cp != '"' && cp != '\\') {
      if (o) *o++ = (uint8_t)cp;
      len += 1;
      continue;
    }
    const char* esc = nullptr;
    switch (cp) {
      case '"': esc = "\\\""; break;
      case '\\': esc = "\\\\"; break;
      case '\n': esc = "\\n"; break;
      case '\r': esc = "\\r"; break;
      case '\t': esc = "\\t"; break;
      case '\b': esc = "\\b"; break;
      case '\f': esc = "\\f"; break;
      default: break;
    }
    if (esc) {
      if (o) { o[0] = (uint8_t)esc[0]; o[1] = (uint8_t)esc[1]; o += 2; }
      len += 2;
    } else if (cp < 0x10000) {
      if (o) put_u16(o, cp);
      len += 6;
    } else {
      const uint32_t u = cp - 0x10000;
      if (o) { put_u16(o, 0xD800 | (u >> 10)); put_u16(o, 0xDC00 | (u & 0x3FF)); }
      len += 12;
    }
  }
  return len;
}

const char kHead1[] = "{\"prediction\": ";
const char kHead2[] = ", \"confidence\": ";
const char kHead3[] = ", \"analysis\": null, \"historical_insight\": null, \"original_text\": \"";
const char kTail[] = "\"}";

}  // namespace

int64_t encode_records(const double* pred, const double* conf, const uint8_t* text, const int64_t* off,
                       const int32_t* skip, int64_t n, uint8_t* out, int64_t cap, int64_t* out_off, int32_t* status,
                       int threads) {
  std::vector<int64_t> lens((size_t)n, 0);
  parallel_for(n, threads, 64, [&](int64_t lo, int64_t hi) {
    char num[64];
    for (int64_t i = lo; i < hi; ++i) {
      if (skip && skip[i]) { status[i] = 2; lens[i] = 0; continue; }
      const int64_t body = escape_ascii(text + off[i], off[i + 1] - off[i], nullptr);
      if (body < 0) { status[i] = 1; lens[i] = 0; continue; }
      status[i] = 0;
      lens[i] = (int64_t)(sizeof(kHead1) - 1 + sizeof(kHead2) - 1 + sizeof(kHead3) - 1 + sizeof(kTail) - 1) +
                py_float_repr(pred[i], num) + py_float_repr(conf[i], num) + body;
    }
  });
  out_off[0] = 0;
  for (int64_t i = 0; i < n; ++i) out_off[i + 1] = out_off[i] + lens[(size_t)i];
  if (out_off[n] > cap) return -out_off[n];   // caller grows the buffer and retries
  parallel_for(n, threads, 64, [&](int64_t lo, int64_t hi) {
    for (int64_t i = lo; i < hi; ++i) {
      if (status[i] != 0) continue;
      uint8_t* o = out + out_off[i];
      auto put = [&](const char* s, size_t k) { std::memcpy(o, s, k); o += k; };
      put(kHead1, sizeof(kHead1) - 1);
      o += py_float_repr(pred[i], reinterpret_cast<char*>(o));
      put(kHead2, sizeof(kHead2) - 1);
      o += py_float_repr(conf[i], reinterpret_cast<char*>(o));
      put(kHead3, sizeof(kHead3) - 1);
      o += escape_ascii(text + off[i], off[i + 1] - off[i], o);
      put(kTail, sizeof(kTail) - 1);
    }
  });
  return out_off[n];
}

}  // namespace fdx

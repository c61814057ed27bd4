// Bulk extraction of one string field (e.g. "text") from Kafka JSON message values (N-09).
//
// Input: N JSON objects packed back-to-back (bytes + int64 offsets). For each object the value of
// the first top-level key equal to `field` must be a JSON string; it is unescaped (\" \\ \/ \b \f
// \n \r \t \uXXXX with surrogate pairs -> UTF-8) and appended to the output buffer, which is laid
// out exactly like a PackedText (so it can be written straight into a pinned ring slot).
// status[i]: 0 ok, 1 malformed JSON / field missing / not a string, 2 output buffer full.
// Multi-threaded in two passes: (1) per-message unescaped lengths, (2) prefix offsets + copy.
#include <cstdint>
#include <cstring>
#include <vector>

#include "parallel_for.h"
#include "swar.h"

namespace fdx {

namespace {

inline const uint8_t* skip_ws(const uint8_t* p, const uint8_t* e) {
  while (p < e && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) ++p;
  return p;
}

inline int hexv(uint8_t c) {
  if (c >= '0' && c <= '9') return c - '0';
  if (c >= 'a' && c <= 'f') return c - 'a' + 10;
  if (c >= 'A' && c <= 'F') return c - 'A' + 10;
  return -1;
}

// Parse a JSON string starting at p (pointing at the opening quote). If out != nullptr the
// unescaped UTF-8 is written there. Returns pointer past the closing quote or nullptr on error;
// *len receives the unescaped byte length.
const uint8_t* parse_string(const uint8_t* p, const uint8_t* e, uint8_t* out, int64_t* len) {
  if (p >= e || *p != '"') return nullptr;
  ++p;
  int64_t n = 0;
  while (p < e) {
    while (e - p >= 8) {             // runs of plain bytes: 8 at a time
      const uint64_t w = swar_load(p);
      if (swar_has_byte(w, '"') || swar_has_byte(w, '\\')) break;
      if (out) std::memcpy(out + n, p, 8);
      p += 8;
      n += 8;
    }
    if (p >= e) break;
    uint8_t c = *p++;
    if (c == '"') { *len = n; return p; }
    if (c != '\\') {
      if (out) out[n] = c;
      ++n;
      continue;
    }
    if (p >= e) return nullptr;
    c = *p++;
    uint32_t cp;
    switch (c) {
      case '"': cp = '"'; break;
      case '\\': cp = '\\'; break;
      case '/': cp = '/'; break;
      case 'b': cp = 8; break;
      case 'f': cp = 12; break;
      case 'n': cp = 10; break;
      case 'r': cp = 13; break;
      case 't': cp = 9; break;
      case 'u': {
        if (e - p < 4) return nullptr;
        int a = hexv(p[0]), b = hexv(p[1]), cc = hexv(p[2]), d = hexv(p[3]);
        if ((a | b | cc | d) < 0) return nullptr;
        cp = (uint32_t)((a << 12) | (b << 8) | (cc << 4) | d);
        p += 4;
        if (cp >= 0xD800 && cp <= 0xDBFF && e - p >= 6 && p[0] == '\\' && p[1] == 'u') {
          int a2 = hexv(p[2]), b2 = hexv(p[3]), c2 = hexv(p[4]), d2 = hexv(p[5]);
          if ((a2 | b2 | c2 | d2) >= 0) {
            const uint32_t lo = (uint32_t)((a2 << 12) | (b2 << 8) | (c2 << 4) | d2);
            if (lo >= 0xDC00 && lo <= 0xDFFF) {
              cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
              p += 6;
            }
          }
        }
        if (cp >= 0xD800 && cp <= 0xDFFF) cp = 0xFFFD;   // lone surrogate
        break;
      }
      default: return nullptr;
    }
    uint8_t buf[4];
    int k;
    if (cp < 0x80) { buf[0] = (uint8_t)cp; k = 1; }
    else if (cp < 0x800) { buf[0] = 0xC0 | (cp >> 6); buf[1] = 0x80 | (cp & 0x3F); k = 2; }
    else if (cp < 0x10000) { buf[0] = 0xE0 | (cp >> 12); buf[1] = 0x80 | ((cp >> 6) & 0x3F); buf[2] = 0x80 | (cp & 0x3F); k = 3; }
    else { buf[0] = 0xF0 | (cp >> 18); buf[1] = 0x80 | ((cp >> 12) & 0x3F); buf[2] = 0x80 | ((cp >> 6) & 0x3F); buf[3] = 0x80 | (cp & 0x3F); k = 4; }
    if (out) std::memcpy(out + n, buf, k);
    n += k;
  }
  return nullptr;
}

// Skip any JSON value; returns pointer past it or nullptr.
const uint8_t* skip_value(const uint8_t* p, const uint8_t* e, int depth = 0) {
  p = skip_ws(p, e);
  if (p >= e || depth > 64) return nullptr;
  if (*p == '"') { int64_t l; return parse_string(p, e, nullptr, &l); }
  if (*p == '{' || *p == '[') {
    const uint8_t close = (*p == '{') ? '}' : ']';
    const bool obj = *p == '{';
    ++p;
    p = skip_ws(p, e);
    if (p < e && *p == close) return p + 1;
    while (p && p < e) {
      if (obj) {
        int64_t l;
        p = parse_string(skip_ws(p, e), e, nullptr, &l);
        if (!p) return nullptr;
        p = skip_ws(p, e);
        if (p >= e || *p != ':') return nullptr;
        ++p;
      }
      p = skip_value(p, e, depth + 1);
      if (!p) return nullptr;
      p = skip_ws(p, e);
      if (p >= e) return nullptr;
      if (*p == ',') { ++p; continue; }
      if (*p == close) return p + 1;
      return nullptr;
    }
    return nullptr;
  }
  // literal / number
  while (p < e && *p != ',' && *p != '}' && *p != ']' && *p != ' ' && *p != '\n' && *p != '\t' && *p != '\r') ++p;
  return p;
}

// Locate the string value of `field` in the top-level object; returns pointer to its opening quote.
const uint8_t* find_field(const uint8_t* p, const uint8_t* e, const uint8_t* field, int64_t flen) {
  p = skip_ws(p, e);
  if (p >= e || *p != '{') return nullptr;
  ++p;
  std::vector<uint8_t> key;
  while (p < e) {
    p = skip_ws(p, e);
    if (p < e && *p == '}') return nullptr;
    int64_t klen;
    const uint8_t* after = parse_string(p, e, nullptr, &klen);
    if (!after) return nullptr;
    key.resize((size_t)klen);
    parse_string(p, e, key.data(), &klen);
    p = skip_ws(after, e);
    if (p >= e || *p != ':') return nullptr;
    p = skip_ws(p + 1, e);
    if (klen == flen && std::memcmp(key.data(), field, (size_t)flen) == 0) return (p < e && *p == '"') ? p : nullptr;
    p = skip_value(p, e);
    if (!p) return nullptr;
    p = skip_ws(p, e);
    if (p < e && *p == ',') { ++p; continue; }
    return nullptr;
  }
  return nullptr;
}

}  // namespace

namespace {

// record i = bytes [begin(i), end(i)); a null begin is a missing value (status 1)
template <class Begin, class End>
int64_t extract_impl(Begin begin, End end, int64_t n, const uint8_t* field, int64_t flen, uint8_t* out,
                     int64_t out_cap, int64_t* out_off, int32_t* status, int threads) {
  std::vector<int64_t> lens((size_t)n, 0);
  std::vector<const uint8_t*> where((size_t)n, nullptr);
  parallel_for(n, threads, 512, [&](int64_t lo, int64_t hi) {
    for (int64_t i = lo; i < hi; ++i) {
      const uint8_t* s = begin(i);
      const uint8_t* e = end(i);
      const uint8_t* q = s ? find_field(s, e, field, flen) : nullptr;
      int64_t l = 0;
      if (q && parse_string(q, e, nullptr, &l)) { where[i] = q; lens[i] = l; status[i] = 0; }
      else { status[i] = 1; lens[i] = 0; }
    }
  });
  out_off[0] = 0;
  for (int64_t i = 0; i < n; ++i) {
    int64_t l = lens[i];
    if (out_off[i] + l > out_cap) { status[i] = 2; l = 0; where[i] = nullptr; lens[i] = 0; }
    out_off[i + 1] = out_off[i] + l;
  }
  parallel_for(n, threads, 512, [&](int64_t lo, int64_t hi) {
    for (int64_t i = lo; i < hi; ++i) {
      if (!where[i]) continue;
      int64_t l;
      parse_string(where[i], end(i), out + out_off[i], &l);
    }
  });
  return out_off[n];
}

}  // namespace

// Returns total bytes written. out_off must have n+1 entries.
int64_t extract_json_field(const uint8_t* in, const int64_t* in_off, int64_t n, const uint8_t* field, int64_t flen,
                           uint8_t* out, int64_t out_cap, int64_t* out_off, int32_t* status, int threads) {
  return extract_impl([&](int64_t i) { return in + in_off[i]; }, [&](int64_t i) { return in + in_off[i + 1]; }, n,
                      field, flen, out, out_cap, out_off, status, threads);
}

// The same over n separate buffers (begin[i], len[i]); begin[i] == nullptr: a missing value.
int64_t extract_json_field_ptrs(const uint8_t* const* begin, const int64_t* len, int64_t n, const uint8_t* field,
                                int64_t flen, uint8_t* out, int64_t out_cap, int64_t* out_off, int32_t* status,
                                int threads) {
  return extract_impl([&](int64_t i) { return begin[i]; }, [&](int64_t i) { return begin[i] + len[i]; }, n, field,
                      flen, out, out_cap, out_off, status, threads);
}

}  // namespace fdx

// 8-bytes-at-a-time byte-class tests for the host JSON paths (json_text.cpp, json_encode.cpp).
#pragma once
#include <cstdint>
#include <cstring>

namespace fdx {

constexpr uint64_t kSwarOnes = 0x0101010101010101ull;
constexpr uint64_t kSwarHigh = 0x8080808080808080ull;

inline uint64_t swar_load(const uint8_t* p) {
  uint64_t w;
  std::memcpy(&w, p, 8);
  return w;
}
// any byte == 0
inline bool swar_has_zero(uint64_t v) { return ((v - kSwarOnes) & ~v & kSwarHigh) != 0; }
// any byte == b
inline bool swar_has_byte(uint64_t w, uint8_t b) { return swar_has_zero(w ^ (kSwarOnes * b)); }
// any byte < n (n <= 128)
inline bool swar_has_less(uint64_t w, uint8_t n) { return ((w - kSwarOnes * n) & ~w & kSwarHigh) != 0; }
// any byte >= 0x7f (0x7f + 1 sets the high bit; carries only leave bytes that are >= 0x80)
inline bool swar_has_7f_or_high(uint64_t w) { return ((w | (w + kSwarOnes)) & kSwarHigh) != 0; }

}  // namespace fdx

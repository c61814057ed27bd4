// Shared host/device definitions for the MI355X (gfx950) native core.
//
// Text semantics reproduce the reference pipeline exactly:
//   clean_text = regexp_replace(lower(dialogue), "[^a-zA-Z ]", "")
//       (/root/reference/fraud_detection_spark.py:42-45, utils/agent_api.py:139-145)
//   Tokenizer  = lower().split("\\s") with Java split semantics (stage R-31)
//   StopWordsRemover (stage R-32), HashingTF = MurmurHash3_x86_32(utf8, seed 42)
//       -> nonNegativeMod(numFeatures) (stage R-33)
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define FDX_HD __host__ __device__ __forceinline__
#else
#define FDX_HD inline
#endif

namespace fdx {

// ---------------------------------------------------------------- murmur3
FDX_HD uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

FDX_HD uint32_t murmur_mix_k(uint32_t k) {
  k *= 0xcc9e2d51u;
  k = rotl32(k, 15);
  k *= 0x1b873593u;
  return k;
}

FDX_HD uint32_t murmur_mix_h(uint32_t h, uint32_t k) {
  h ^= murmur_mix_k(k);
  h = rotl32(h, 13);
  return h * 5u + 0xe6546b64u;
}

FDX_HD uint32_t murmur_fmix(uint32_t h, uint32_t len) {
  h ^= len;
  h ^= h >> 16;
  h *= 0x85ebca6bu;
  h ^= h >> 13;
  h *= 0xc2b2ae35u;
  h ^= h >> 16;
  return h;
}

// Streaming murmur3_x86_32 (Spark hashUnsafeBytes2): feed bytes one at a time.
struct Murmur3 {
  uint32_t h, k, n;
  FDX_HD void init(uint32_t seed) { h = seed; k = 0; n = 0; }
  FDX_HD void push(uint8_t b) {
    k |= (uint32_t)b << (8 * (n & 3));
    ++n;
    if ((n & 3) == 0) { h = murmur_mix_h(h, k); k = 0; }
  }
  FDX_HD uint32_t finish() const {
    uint32_t hh = h;
    if (n & 3) hh ^= murmur_mix_k(k);
    return murmur_fmix(hh, n);
  }
};

// second seed of the 64-bit token key (murmur3 seed 42 in the high word, this in the low word)
constexpr uint32_t kKeySeed2 = 0x9747b28cu;

FDX_HD uint32_t murmur3_bytes(const uint8_t* p, uint32_t len, uint32_t seed) {
  Murmur3 m; m.init(seed);
  for (uint32_t i = 0; i < len; ++i) m.push(p[i]);
  return m.finish();
}

// Spark Utils.nonNegativeMod on the signed 32-bit hash.
FDX_HD int32_t non_negative_mod(uint32_t h, int32_t mod) {
  int32_t s = (int32_t)h;
  int32_t r = s % mod;
  return r < 0 ? r + mod : r;
}

// ---------------------------------------------------------------- text rules
// Java \s = [ \t\n\x0B\f\r]
FDX_HD bool is_java_space(uint8_t c) {
  return c == ' ' || c == '\t' || c == '\n' || c == 0x0B || c == '\f' || c == '\r';
}

// Cleaning of one byte position in the raw UTF-8 stream (lower() then strip [^a-zA-Z ]).
// Returns the output byte or 0 for "deleted". The only non-ASCII code points whose Java
// lowercase lands in [a-z] are U+0130 (-> "i" + U+0307, the combining dot is stripped) and
// U+212A KELVIN SIGN (-> "k"). `b1`/`b2` are the following bytes (0 past the end).
FDX_HD uint8_t clean_byte(uint8_t b0, uint8_t b1, uint8_t b2) {
  if (b0 < 0x80) {
    if (b0 >= 'A' && b0 <= 'Z') return b0 + 32;
    if ((b0 >= 'a' && b0 <= 'z') || b0 == ' ') return b0;
    return 0;
  }
  if (b0 == 0xC4 && b1 == 0xB0) return 'i';                 // U+0130
  if (b0 == 0xE2 && b1 == 0x84 && b2 == 0xAA) return 'k';   // U+212A
  return 0;
}

// Flags of the fused text pipeline (bit field shared by host and device code).
enum : int {
  kFlagClean = 1 << 0,        // apply lower + [^a-zA-Z ] strip before tokenizing
  kFlagBinary = 1 << 1,       // HashingTF/CountVectorizer binary=true
  kFlagWriteCsr = 1 << 2,     // materialise the per-doc sparse vector
  kFlagIdf = 1 << 3,          // scale values by idf[]
  kFlagLR = 1 << 4,           // binary logistic-regression margin
  kFlagTrees = 1 << 5,        // tree-ensemble raw prediction
  kFlagVocab = 1 << 6,        // CountVectorizerModel lookup instead of hashing
  kFlagStopwords = 1 << 7,    // apply stop-word filtering
  kFlagCmpLess = 1 << 8,      // tree split: go left iff x < thr (XGBoost); else x <= thr (Spark)
  kFlagPreLowered = 1 << 9,   // text already Unicode-lowercased by the host: pass UTF-8 through
  kFlagKeys = 1 << 10,        // CountVectorizer fit: emit a 64-bit key per kept token (no vectors)
};

// Status codes written per document.
enum : int { kStatusOk = 0, kStatusTooLong = 1, kStatusNeedsHost = 2 };

// Open-addressing string set/map keyed by murmur3(seed 42); slot -> entry index or -1.
// Entries are verified byte-for-byte, so hash collisions never change semantics.
struct StrTable {
  const int32_t* slots;     // [mask + 1]
  const uint32_t* hashes;   // [n] murmur3 seed 42 of each entry
  const int64_t* offs;      // [n + 1] into bytes
  const uint8_t* bytes;
  int32_t mask;             // table size - 1 (power of two); -1 => empty table
};

}  // namespace fdx

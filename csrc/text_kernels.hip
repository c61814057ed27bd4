// Fused text featurization + scoring for gfx950 (K-01..K-04, K-06, K-07, K-16 of SURVEY.md §2.5).
//
// One 64-lane wavefront owns one dialogue end to end; a 256-thread workgroup holds four
// independent dialogues. Everything between the raw UTF-8 bytes and the score stays in LDS:
//   1. clean   : dword loads (4 bytes/lane, 256 B per wave-step), lower + [^a-zA-Z ] strip,
//                wave prefix-scan compaction into an LDS byte buffer        (X-01)
//   2. tokens  : Java split("\\s") segment starts via ballot, queued 64 at a
//                time so every lane hashes one token (murmur3, seed 42)      (X-02, X-04)
//   3. filter  : stop-word open-addressing table, verified byte-for-byte    (X-03)
//   4. bucket  : nonNegativeMod(h, F) (HashingTF) or vocab lookup (CountVectorizerModel)
//   5. sort    : in-LDS bitonic sort of the bucket list, run-length encode  (sparse vector)
//   6. value   : tf (or 1 if binary) * idf                                  (X-06)
//   7. score   : LR margin (fp64 wave reduction) or tree-ensemble traversal
//                with binary search over the LDS-resident sorted indices     (X-07, X-11)
// Only the score (and optionally the sparse vector) is written back to HBM.
// Two instantiations: the streaming one (4 dialogues per 256-thread workgroup, 4 KB of cleaned
// text / 1024 kept tokens per dialogue, ~34 KB LDS per workgroup) and a long-dialogue one (one
// dialogue per single-wave workgroup, 64 KB / 16384 tokens, ~128 KB LDS -- CDNA4 lets one
// workgroup take up to 160 KB) that runs only on the documents the first launch flags as too
// long (long transcripts stay on the GPU). Longer ones are finished by the host.
#include "scoring.h"
#include "ops.h"

// Spark (JVM) never fuses multiply-add; keep fp64 scores bit-comparable with the host path.
#pragma clang fp contract(off)

namespace fdx {

constexpr int kWave = 64;
constexpr int kCapB = 4096;       // streaming variant: cleaned bytes per dialogue held in LDS
constexpr int kCapT = 1024;       //                    kept tokens per dialogue held in LDS
constexpr int kWavesPerBlock = 4;
constexpr int kLongCapB = 65536;  // long-dialogue variant
constexpr int kLongCapT = 16384;

__device__ __forceinline__ void lds_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ int lane_id() { return threadIdx.x & (kWave - 1); }

__device__ __forceinline__ int wave_incl_scan(int v) {
  const int lane = lane_id();
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const int t = __shfl_up(v, o, kWave);
    if (lane >= o) v += t;
  }
  return v;
}

__device__ __forceinline__ double wave_sum_f64(double v) {
#pragma unroll
  for (int o = kWave / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

__device__ __forceinline__ int popc_below(unsigned long long m) {
  return __popcll(m & ((1ull << lane_id()) - 1ull));
}

__device__ __forceinline__ bool is_delim(uint8_t c, bool cleaned) {
  return cleaned ? (c == ' ') : is_java_space(c);
}

// Hash one token starting at `p` of the cleaned buffer; returns length in *len.
__device__ __forceinline__ uint32_t hash_token(const uint8_t* s_clean, int p, int n, bool cleaned,
                                               int* len) {
  Murmur3 m;
  m.init(42u);
  for (int i = p; i < n; ++i) {
    const uint8_t c = s_clean[i];
    if (is_delim(c, cleaned)) break;
    m.push(c);
  }
  *len = (int)m.n;
  return m.finish();
}

template <int CAPB, int CAPT, int WAVES>
__global__ __launch_bounds__(kWave * WAVES) void featurize_score_kernel(FeatArgs a) {
  static_assert(CAPB / 4 >= CAPT && CAPB <= 65536, "counts reuse the byte buffer; token starts are 16-bit");
  __shared__ __attribute__((aligned(16))) uint8_t s_clean_all[WAVES][CAPB];
  __shared__ uint32_t s_tok_all[WAVES][CAPT];
  __shared__ uint16_t s_q_all[WAVES][2 * kWave];

  const int wid = threadIdx.x / kWave;
  const int lane = lane_id();
  const int slot = blockIdx.x * WAVES + wid;
  if (slot >= (a.doc_list ? a.n_list : a.num_docs)) return;
  const int d = a.doc_list ? a.doc_list[slot] : slot;
  if (d < 0 || d >= a.num_docs) return;      // a stale / foreign doc list never indexes out of range

  uint8_t* s_clean = s_clean_all[wid];
  uint32_t* s_tok = s_tok_all[wid];
  uint32_t* s_cnt = reinterpret_cast<uint32_t*>(s_clean);   // reused after hashing
  uint16_t* s_q = s_q_all[wid];

  const bool cleaned = (a.flags & kFlagClean) != 0;
  const bool prelowered = (a.flags & kFlagPreLowered) != 0;
  const int64_t s = a.doc_off[d], e = a.doc_off[d + 1];
  const int K = (a.flags & kFlagTrees) ? a.trees.K : 1;
  if (e - s > CAPB) {
    if (lane == 0) a.out_status[d] = kStatusTooLong;
    return;
  }

  // ------------------------------------------------------------------ 1. clean
  int n = 0;
  bool host = false;
  for (int64_t base = s & ~3ll; base < e; base += 4 * kWave) {
    const int64_t p0 = base + 4 * lane;
    uint32_t w = 0;
    if (p0 < e) w = *reinterpret_cast<const uint32_t*>(a.text + p0);
    uint32_t packed = 0;
    int c = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int64_t p = p0 + k;
      const uint8_t b = (w >> (8 * k)) & 0xffu;
      if (p >= s && p < e) {
        int o;
        if (cleaned) {
          if (b < 0x80) {
            o = clean_byte(b, 0, 0);
          } else {
            const uint8_t b1 = (p + 1 < e) ? a.text[p + 1] : 0;
            const uint8_t b2 = (p + 2 < e) ? a.text[p + 2] : 0;
            o = clean_byte(b, b1, b2);
          }
          o = o ? o : -1;
        } else if (prelowered) {
          o = b;
        } else {
          host = host || (b >= 0x80);
          o = (b >= 'A' && b <= 'Z') ? b + 32 : b;
        }
        if (o >= 0) {
          packed |= (uint32_t)o << (8 * c);
          ++c;
        }
      }
    }
    const int incl = wave_incl_scan(c);
    const int pos = n + incl - c;
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (k < c) s_clean[pos + k] = (packed >> (8 * k)) & 0xffu;
    n += __shfl(incl, kWave - 1, kWave);
  }
  if (__ballot(host)) {
    if (lane == 0) a.out_status[d] = kStatusNeedsHost;
    return;
  }
  lds_sync();

  // ------------------------------------------------------------------ 2-4. tokens
  // q = last non-delimiter position; segments starting at p <= q are the kept tokens.
  int q = -1;
  for (int base = 0; base < n; base += kWave) {
    const int p = base + lane;
    const unsigned long long m = __ballot(p < n && !is_delim(s_clean[p], cleaned));
    if (m) q = base + 63 - __clzll(m);
  }

  int ntok = 0;      // kept tokens in s_tok
  int nall = 0;      // tokens after stop-word removal (CountVectorizer minTF denominator)
  const bool use_vocab = (a.flags & kFlagVocab) != 0;
  const bool use_stop = (a.flags & kFlagStopwords) != 0;

  const bool keys_mode = (a.flags & kFlagKeys) != 0;
  auto emit = [&](int start, bool valid) {
    int len = 0;
    bool keep_sw = false;   // survived stop-word removal
    int32_t bucket = -1;
    uint32_t h = 0;
    if (valid) {
      h = hash_token(s_clean, start, n, cleaned, &len);
      keep_sw = !(use_stop && table_find(a.stop, h, s_clean + start, len) >= 0);
      if (keep_sw && !keys_mode)
        bucket = use_vocab ? table_find(a.vocab, h, s_clean + start, len)
                           : non_negative_mod(h, a.num_features);
    }
    const unsigned long long sm = __ballot(keep_sw);
    if (keys_mode && keep_sw && a.out_keys)
      a.out_keys[a.key_off[d] + nall + popc_below(sm)] =
          ((uint64_t)h << 32) | murmur3_bytes(s_clean + start, (uint32_t)len, kKeySeed2);
    nall += __popcll(sm);
    const bool keep = keep_sw && bucket >= 0;
    const unsigned long long km = __ballot(keep);
    const int slot = ntok + popc_below(km);
    if (keep && slot < CAPT) s_tok[slot] = (uint32_t)bucket;
    ntok += __popcll(km);
  };

  if (q < 0) {
    if (n == 0) emit(0, lane == 0);   // "" -> one empty token
  } else {
    int qn = 0;
    for (int base = 0; base <= q; base += kWave) {
      const int p = base + lane;
      const bool st = p <= q && (p == 0 || is_delim(s_clean[p - 1], cleaned));
      const unsigned long long m = __ballot(st);
      if (st) s_q[qn + popc_below(m)] = (uint16_t)p;
      qn += __popcll(m);
      if (qn >= kWave) {
        lds_sync();
        const int start = s_q[lane];
        const int rest = (lane < qn - kWave) ? s_q[kWave + lane] : 0;
        lds_sync();
        if (lane < qn - kWave) s_q[lane] = (uint16_t)rest;
        emit(start, true);
        qn -= kWave;
      }
    }
    lds_sync();
    if (qn > 0) {
      const int start = (lane < qn) ? s_q[lane] : 0;
      emit(start, lane < qn);
    }
  }
  if (keys_mode) {
    if (lane == 0) {
      if (a.out_ntok) a.out_ntok[d] = nall;
      a.out_status[d] = kStatusOk;
    }
    return;
  }
  if (ntok > CAPT) {
    if (lane == 0) a.out_status[d] = kStatusTooLong;
    return;
  }
  lds_sync();

  // ------------------------------------------------------------------ 5. sort + RLE
  int P = 1;
  while (P < ntok) P <<= 1;
  for (int i = ntok + lane; i < P; i += kWave) s_tok[i] = 0xffffffffu;
  lds_sync();
  for (int k = 2; k <= P; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = lane; i < P; i += kWave) {
        const int ixj = i ^ j;
        if (ixj > i) {
          const uint32_t x = s_tok[i], y = s_tok[ixj];
          const bool up = (i & k) == 0;
          if ((x > y) == up) { s_tok[i] = y; s_tok[ixj] = x; }
        }
      }
      lds_sync();
    }
  }

  // heads of equal runs -> unique ids (in place into s_tok) and run starts (s_cnt)
  int nu = 0;
  uint32_t prev_last = 0xffffffffu;
  for (int base = 0; base < ntok; base += kWave) {
    const int i = base + lane;
    const uint32_t cur = (i < ntok) ? s_tok[i] : 0u;
    uint32_t prv = __shfl_up(cur, 1, kWave);
    if (lane == 0) prv = prev_last;
    const bool head = i < ntok && (i == 0 || cur != prv);
    prev_last = __shfl(cur, kWave - 1, kWave);
    const unsigned long long m = __ballot(head);
    lds_sync();
    if (head) {
      const int j = nu + popc_below(m);
      s_tok[j] = cur;
      s_cnt[j] = (uint32_t)i;
    }
    nu += __popcll(m);
    lds_sync();
  }
  // counts = next head - head
  for (int base = 0; base < nu; base += kWave) {
    const int j = base + lane;
    uint32_t c = 0;
    if (j < nu) {
      const uint32_t nxt = (j + 1 < nu) ? s_cnt[j + 1] : (uint32_t)ntok;
      c = nxt - s_cnt[j];
    }
    lds_sync();
    if (j < nu) s_cnt[j] = c;
    lds_sync();
  }

  // CountVectorizerModel minTF: keep count >= minTF (absolute) or >= minTF * tokens (fraction).
  if (use_vocab && (a.min_tf > 1.0 || (a.min_tf > 0.0 && a.min_tf < 1.0))) {
    const double thr = a.min_tf >= 1.0 ? a.min_tf : a.min_tf * nall;
    int nk = 0;
    for (int base = 0; base < nu; base += kWave) {
      const int j = base + lane;
      const bool keep = j < nu && (double)s_cnt[j] >= thr;
      const uint32_t u = keep ? s_tok[j] : 0u, c = keep ? s_cnt[j] : 0u;
      const unsigned long long m = __ballot(keep);
      lds_sync();
      if (keep) { const int t = nk + popc_below(m); s_tok[t] = u; s_cnt[t] = c; }
      nk += __popcll(m);
      lds_sync();
    }
    nu = nk;
  }

  // ------------------------------------------------------------------ 6-7. values + score
  const bool binary = (a.flags & kFlagBinary) != 0;
  const bool use_idf = (a.flags & kFlagIdf) != 0;
  const int64_t ob = csr_slot(s, d);   // CSR scratch base (scoring.h)
  double lr_part = 0.0;
  for (int j = lane; j < nu; j += kWave) {
    const uint32_t u = s_tok[j];
    double v = binary ? 1.0 : (double)s_cnt[j];
    if (use_idf) v *= a.idf[u];
    if (a.flags & kFlagWriteCsr) {
      a.out_idx[ob + j] = (int32_t)u;
      a.out_val[ob + j] = (float)v;
    }
    if (a.flags & kFlagLR) lr_part += v * a.lr_w[u];
  }
  if (lane == 0) {
    a.out_nnz[d] = nu;
    if (a.out_ntok) a.out_ntok[d] = nall;
    a.out_status[d] = kStatusOk;
  }
  if (a.flags & kFlagLR) {
    const double m = wave_sum_f64(lr_part);
    if (lane == 0) a.out_raw[d] = m + a.lr_b;
  }
  if (a.flags & kFlagTrees) {
    const TreeEnsemble& te = a.trees;
    const bool cmp_less = (a.flags & kFlagCmpLess) != 0;
    auto lookup = [&](int32_t f) -> double {
      const int32_t j = sorted_find<uint32_t>(s_tok, nu, (uint32_t)f);
      if (j < 0) return 0.0;
      double v = binary ? 1.0 : (double)s_cnt[j];
      if (use_idf) v *= a.idf[f];
      return v;
    };
    double acc0 = 0.0, acc1 = 0.0;
    for (int t = lane; t < te.num_trees; t += kWave) {
      const int32_t leaf = tree_find_leaf(te, te.roots[t], cmp_less, lookup);
      const double w = te.weights[t];
      acc0 += w * te.leaf[(int64_t)leaf * te.K];
      if (te.K > 1) acc1 += w * te.leaf[(int64_t)leaf * te.K + 1];
    }
    acc0 = wave_sum_f64(acc0);
    acc1 = wave_sum_f64(acc1);
    if (lane == 0) {
      a.out_raw[(int64_t)d * K] = acc0;
      if (K > 1) a.out_raw[(int64_t)d * K + 1] = acc1;
    }
  }
}

void launch_featurize_score(const FeatArgs& a, hipStream_t stream) {
  if (a.doc_list) {          // long dialogues: one per single-wave workgroup
    if (a.n_list > 0)
      hipLaunchKernelGGL((featurize_score_kernel<kLongCapB, kLongCapT, 1>), dim3(a.n_list), dim3(kWave), 0, stream, a);
    return;
  }
  if (a.num_docs <= 0) return;
  const int blocks = (a.num_docs + kWavesPerBlock - 1) / kWavesPerBlock;
  hipLaunchKernelGGL((featurize_score_kernel<kCapB, kCapT, kWavesPerBlock>), dim3(blocks), dim3(kWave * kWavesPerBlock),
                     0, stream, a);
}

}  // namespace fdx

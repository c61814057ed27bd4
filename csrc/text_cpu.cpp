// Host implementation of the fused featurize+score pipeline (same contract as
// featurize_score_kernel in text_kernels.hip). Used for CPU-only execution, for documents the
// GPU kernel flags kStatusTooLong/kStatusNeedsHost, and as a native cross-check in tests.
// Multi-threaded over documents with std::thread; no GPU dependency.
#include <algorithm>
#include <cmath>
#include <string>
#include <thread>
#include <vector>

#include "scoring.h"

namespace fdx {

namespace {

// Java String.toLowerCase for the code points we must handle exactly in non-clean mode is
// delegated to Python (kStatusNeedsHost); here only ASCII lowercase is applied.
void clean_doc(const uint8_t* p, int64_t len, bool cleaned, bool prelowered, std::string* out,
               bool* needs_host) {
  out->clear();
  out->reserve(len);
  for (int64_t i = 0; i < len; ++i) {
    const uint8_t b = p[i];
    if (cleaned) {
      const uint8_t b1 = i + 1 < len ? p[i + 1] : 0;
      const uint8_t b2 = i + 2 < len ? p[i + 2] : 0;
      const uint8_t o = clean_byte(b, b1, b2);
      if (o) out->push_back((char)o);
    } else if (prelowered) {
      out->push_back((char)b);
    } else {
      if (b >= 0x80) *needs_host = true;
      out->push_back((char)((b >= 'A' && b <= 'Z') ? b + 32 : b));
    }
  }
}

void process_doc(const FeatArgs& a, int32_t d, std::string& clean, std::vector<uint32_t>& toks,
                 std::vector<std::pair<uint32_t, uint32_t>>& runs) {
  const bool cleaned = (a.flags & kFlagClean) != 0;
  const int64_t s = a.doc_off[d], e = a.doc_off[d + 1];
  const int K = (a.flags & kFlagTrees) ? a.trees.K : 1;
  bool needs_host = false;
  clean_doc(a.text + s, e - s, cleaned, (a.flags & kFlagPreLowered) != 0, &clean, &needs_host);
  if (needs_host) { a.out_status[d] = kStatusNeedsHost; return; }
  auto delim = [&](uint8_t c) { return cleaned ? c == ' ' : is_java_space(c); };
  const int64_t n = (int64_t)clean.size();
  const uint8_t* cb = reinterpret_cast<const uint8_t*>(clean.data());

  // Java split("\\s"): segments up to the last non-delimiter; "" -> [""]
  int64_t q = -1;
  for (int64_t i = n - 1; i >= 0; --i) if (!delim(cb[i])) { q = i; break; }
  toks.clear();
  int32_t nall = 0;
  const bool use_vocab = (a.flags & kFlagVocab) != 0;
  const bool use_stop = (a.flags & kFlagStopwords) != 0;
  const bool keys_mode = (a.flags & kFlagKeys) != 0;
  auto emit = [&](int64_t start, int64_t len) {
    const uint32_t h = murmur3_bytes(cb + start, (uint32_t)len, 42u);
    if (use_stop && table_find(a.stop, h, cb + start, (int32_t)len) >= 0) return;
    if (keys_mode) {
      if (a.out_keys)
        a.out_keys[a.key_off[d] + nall] = ((uint64_t)h << 32) | murmur3_bytes(cb + start, (uint32_t)len, kKeySeed2);
      ++nall;
      return;
    }
    ++nall;
    int32_t bucket = use_vocab ? table_find(a.vocab, h, cb + start, (int32_t)len)
                               : non_negative_mod(h, a.num_features);
    if (bucket >= 0) toks.push_back((uint32_t)bucket);
  };
  if (q < 0) {
    if (n == 0) emit(0, 0);
  } else {
    int64_t start = 0;
    for (int64_t i = 0; i <= q; ++i) {
      if (delim(cb[i])) { emit(start, i - start); start = i + 1; }
    }
    int64_t end = start;
    while (end < n && !delim(cb[end])) ++end;
    emit(start, end - start);
  }
  if (keys_mode) {
    if (a.out_ntok) a.out_ntok[d] = nall;
    a.out_status[d] = kStatusOk;
    return;
  }
  std::sort(toks.begin(), toks.end());
  runs.clear();
  for (size_t i = 0; i < toks.size();) {
    size_t j = i;
    while (j < toks.size() && toks[j] == toks[i]) ++j;
    runs.emplace_back(toks[i], (uint32_t)(j - i));
    i = j;
  }
  if (use_vocab && (a.min_tf > 1.0 || (a.min_tf > 0.0 && a.min_tf < 1.0))) {
    const double thr = a.min_tf >= 1.0 ? a.min_tf : a.min_tf * nall;
    std::vector<std::pair<uint32_t, uint32_t>> kept;
    for (auto& r : runs) if ((double)r.second >= thr) kept.push_back(r);
    runs.swap(kept);
  }
  const bool binary = (a.flags & kFlagBinary) != 0;
  const bool use_idf = (a.flags & kFlagIdf) != 0;
  const int64_t ob = csr_slot(s, d);
  double lr = 0.0;
  const int32_t nu = (int32_t)runs.size();
  std::vector<double> vals(nu);
  for (int32_t j = 0; j < nu; ++j) {
    double v = binary ? 1.0 : (double)runs[j].second;
    if (use_idf) v *= a.idf[runs[j].first];
    vals[j] = v;
    if (a.flags & kFlagWriteCsr) {
      a.out_idx[ob + j] = (int32_t)runs[j].first;
      a.out_val[ob + j] = (float)v;
    }
  }
  if (a.flags & kFlagLR) {
    // Same summation order as the 64-lane wave reduction: lane-strided partials, xor-tree.
    double part[64] = {0};
    for (int32_t j = 0; j < nu; ++j) part[j & 63] += vals[j] * a.lr_w[runs[j].first];
    for (int o = 32; o > 0; o >>= 1)
      for (int l = 0; l < 64; ++l) if (l < (l ^ o)) { const double t = part[l] + part[l ^ o]; part[l] = t; part[l ^ o] = t; }
    lr = part[0];
    a.out_raw[d] = lr + a.lr_b;
  }
  if (a.flags & kFlagTrees) {
    const TreeEnsemble& te = a.trees;
    const bool cmp_less = (a.flags & kFlagCmpLess) != 0;
    auto lookup = [&](int32_t f) -> double {
      int32_t lo = 0, hi = nu - 1;
      while (lo <= hi) {
        const int32_t mid = (lo + hi) >> 1;
        if ((int32_t)runs[mid].first == f) return vals[mid];
        if ((int32_t)runs[mid].first < f) lo = mid + 1; else hi = mid - 1;
      }
      return 0.0;
    };
    double p0[64] = {0}, p1[64] = {0};
    for (int32_t t = 0; t < te.num_trees; ++t) {
      const int32_t leaf = tree_find_leaf(te, te.roots[t], cmp_less, lookup);
      p0[t & 63] += te.weights[t] * te.leaf[(int64_t)leaf * te.K];
      if (te.K > 1) p1[t & 63] += te.weights[t] * te.leaf[(int64_t)leaf * te.K + 1];
    }
    for (int o = 32; o > 0; o >>= 1)
      for (int l = 0; l < 64; ++l) if (l < (l ^ o)) {
        double t = p0[l] + p0[l ^ o]; p0[l] = t; p0[l ^ o] = t;
        t = p1[l] + p1[l ^ o]; p1[l] = t; p1[l ^ o] = t;
      }
    a.out_raw[(int64_t)d * K] = p0[0];
    if (K > 1) a.out_raw[(int64_t)d * K + 1] = p1[0];
  }
  a.out_nnz[d] = nu;
  if (a.out_ntok) a.out_ntok[d] = nall;
  a.out_status[d] = kStatusOk;
}

}  // namespace

void featurize_score_cpu(const FeatArgs& a, const int32_t* only_docs, int32_t n_only, int threads) {
  const int32_t total = only_docs ? n_only : a.num_docs;
  if (total <= 0) return;
  if (threads <= 0) threads = (int)std::max(1u, std::thread::hardware_concurrency());
  threads = std::min<int>(threads, std::max<int32_t>(1, total / 64));
  auto work = [&](int32_t lo, int32_t hi) {
    std::string clean;
    std::vector<uint32_t> toks;
    std::vector<std::pair<uint32_t, uint32_t>> runs;
    for (int32_t i = lo; i < hi; ++i) process_doc(a, only_docs ? only_docs[i] : i, clean, toks, runs);
  };
  if (threads <= 1) { work(0, total); return; }
  std::vector<std::thread> pool;
  const int32_t chunk = (total + threads - 1) / threads;
  for (int t = 0; t < threads; ++t) {
    const int32_t lo = t * chunk, hi = std::min(total, lo + chunk);
    if (lo < hi) pool.emplace_back(work, lo, hi);
  }
  for (auto& th : pool) th.join();
}

}  // namespace fdx

// Model descriptors shared by the fused featurize+score kernel, the CSR scorer and the
// CPU path. All arrays live in the same memory space as the caller (device or host).
#pragma once
#include "common.h"

namespace fdx {

// CSR scratch layout of the fused featurizer: a document of L bytes has at most floor((L + 1) / 2)
// non-empty whitespace-separated tokens plus the empty one, i.e. <= floor(L / 2) + 2 distinct
// terms, so doc d starting at byte s gets the slot range [s / 2 + 2 d, s / 2 + 2 d + L / 2 + 2)
// (disjoint from its successor's: (s + L) / 2 - s / 2 >= L / 2). Capacity: bytes / 2 + 2 D + 1
// -- half of a slot per byte (4 B of indices + 4 B of values per text byte before).
FDX_HD int64_t csr_slot(int64_t s, int64_t d) { return (s >> 1) + 2 * d; }
FDX_HD int64_t csr_capacity(int64_t bytes, int64_t docs) { return (bytes >> 1) + 2 * docs + 1; }

// Flattened tree ensemble (DecisionTree / RandomForest / GBDT).
// node is a leaf iff feat[node] < 0; leaf payload = leaf[node * K + k].
struct TreeEnsemble {
  const int32_t* feat;
  const double* thr;
  const int32_t* left;
  const int32_t* right;
  const double* leaf;
  const int32_t* roots;
  const double* weights;
  int32_t num_trees;
  int32_t K;
};

template <class Lookup>
FDX_HD int32_t tree_find_leaf(const TreeEnsemble& te, int32_t node, bool cmp_less, const Lookup& lk) {
  // Depth is bounded by the tree size; a malformed (cyclic) model cannot hang a wave.
  for (int guard = 0; guard < 4096 && te.feat[node] >= 0; ++guard) {
    const double x = lk(te.feat[node]);
    const double t = te.thr[node];
    const bool go_left = cmp_less ? (x < t) : (x <= t);
    node = go_left ? te.left[node] : te.right[node];
  }
  return node;
}

// Binary search of `key` in sorted ascending u[0..n); returns position or -1.
template <class T>
FDX_HD int32_t sorted_find(const T* u, int32_t n, T key) {
  int32_t lo = 0, hi = n - 1;
  while (lo <= hi) {
    const int32_t mid = (lo + hi) >> 1;
    const T v = u[mid];
    if (v == key) return mid;
    if (v < key) lo = mid + 1; else hi = mid - 1;
  }
  return -1;
}

FDX_HD int32_t table_find(const StrTable& t, uint32_t h, const uint8_t* tok, int32_t len) {
  if (t.mask < 0) return -1;
  uint32_t i = h & (uint32_t)t.mask;
  for (int probe = 0; probe <= t.mask; ++probe) {
    const int32_t e = t.slots[i];
    if (e < 0) return -1;
    if (t.hashes[e] == h) {
      const int64_t o = t.offs[e];
      if (t.offs[e + 1] - o == len) {
        bool eq = true;
        for (int32_t k = 0; k < len; ++k) eq = eq && (t.bytes[o + k] == tok[k]);
        if (eq) return e;
      }
    }
    i = (i + 1) & (uint32_t)t.mask;
  }
  return -1;
}

struct FeatArgs {
  const uint8_t* text;       // padded by >= 4 bytes past the last document
  const int64_t* doc_off;    // [num_docs + 1]
  int32_t num_docs;
  int32_t flags;
  int32_t num_features;
  StrTable stop;
  StrTable vocab;
  double min_tf;
  const double* idf;         // [num_features] when kFlagIdf
  const double* lr_w;        // [num_features] when kFlagLR
  double lr_b;
  TreeEnsemble trees;
  // outputs
  int32_t* out_idx;          // CSR scratch: doc d's entries at csr_slot(doc_off[d], d) (csr_slot above)
  float* out_val;
  int32_t* out_nnz;          // [num_docs]
  int32_t* out_ntok;         // [num_docs] tokens after stop-word removal (may be null)
  double* out_raw;           // [num_docs * K] (K = trees.K, or 1 for LR)
  int32_t* out_status;       // [num_docs]
  // kFlagKeys: key of token i of doc d at out_keys[key_off[d] + i]; out_keys == nullptr -> count only
  const int64_t* key_off;
  uint64_t* out_keys;
  // long-dialogue launch: process only doc_list[0 .. n_list) (nullptr: every document)
  const int32_t* doc_list;
  int32_t n_list;
};

}  // namespace fdx

// Tree-engine argument structs shared by tree_kernels.hip (gfx950) and tree_cpu.cpp (host).
//
// Data layout (per data-parallel rank):
//   * quantized CSC: for each active feature fid, entries [colptr[fid], colptr[fid+1]) hold
//     (row int32, bin uint8) sorted by row; bins are ordered by value, bin zbin[fid] is the
//     implicit "value == 0" bin for rows absent from the column;
//   * rowstats[row] (8 B): the two statistics the histogram sums, each split into bf16 hi/lo
//     halves so one bf16 MFMA reproduces ~fp32 sums;
//       GBDT: (g, h);  classification: (w*[y==0], w*[y==1]);
//     gathered ONCE per tree into CSC entry order (est[e] = rowstats[csc_row[e]]), so every
//     level streams them sequentially instead of gathering 16 B per entry per level;
//   * slot8[row] (1 B): which of the <= 32 nodes built by the current histogram pass the row
//     belongs to (0xff: none) -- N bytes, L2-resident, the only per-level random access;
//   * histograms: hist[node][bin] = double2, bins of all features concatenated (boff[fid]).
#pragma once
#include <math.h>
#include <stdint.h>

#include "common.h"

namespace fdx {

struct RowStatsArgs {
  const float* g;             // GBDT gradients (mode 0)
  const float* h;
  const float* label;         // classification labels 0/1 (mode 1)
  const float* weight;        // optional instance weights
  uint64_t seed;              // Poisson(1) bootstrap when bootstrap != 0 (mode 1)
  int32_t tree;
  int32_t bootstrap;
  int32_t mode;               // 0 = gbdt, 1 = classification counts
  int64_t N;
  uint32_t* rowstats;         // [N * 2]
};

struct SlotArgs {
  const int32_t* row_node;    // [N] current node id of each row
  const int32_t* node_slot;   // [num_nodes] slot being built (absolute), -1 otherwise
  int32_t num_nodes;
  int32_t slot_base;          // this pass covers slots [slot_base, slot_base + nslots)
  int32_t nslots;
  int64_t N;
  uint8_t* slot8;             // [N] slot - slot_base, or 0xff
};

struct HistArgs {
  const int64_t* item_start;      // [I] entry range of each work item
  const int64_t* item_end;
  int32_t num_items;
  const int32_t* csc_row;
  const uint8_t* csc_bin;
  const uint8_t* slot8;           // [N] relative slot, 0xff = not built; nullptr = root pass (all slot 0)
  const uint32_t* est;            // [nnz * 2] packed statistics in entry order
  const uint32_t* rowstats;       // [N * 2] gather mode (est unused): statistics gathered per live entry
  float* slab;                   // [I][slots][bins][2]: 32-bin tiles [8*CT][32*BT], narrow [4*CT][16]
  const int32_t* wave_item;       // [num_slots] item of each wave slot (-1 idle); nullptr: slot = item
  int32_t num_slots;
};

struct HistReduceArgs {
  const float* slab;
  int32_t slab_slots;             // 8*CT
  int32_t slab_bins;              // 32*BT
  const int32_t* feat;            // [L] fid of each listed feature
  const int64_t* feat_item0;      // [L] first item of the feature in the item list
  const int32_t* feat_nitems;     // [L]
  int32_t L;
  const int64_t* boff;            // [Fa + 1]
  const int32_t* nbins;           // [Fa]
  const int32_t* slot_to_node;    // [8*CT] level-local node index or -1
  int32_t slot_base;
  int64_t total_bins;             // TB
  double* hist;                   // [nodes][TB][2]
};

struct SplitArgs {
  const double* hist;             // [nodes][TB][2]
  const double* totals;           // [nodes][2]
  int32_t num_nodes;
  int32_t Fa;
  const int64_t* boff;
  const int32_t* nbins;
  const int32_t* zbin;
  const int64_t* fid_orig;        // [Fa] original feature index (RF sampling key)
  const int32_t* node_ids;        // [nodes] tree-global node id (RF sampling key)
  int32_t mode;                   // 0 = xgboost newton gain, 1 = gini, 2 = entropy
  double lambda_;                 // L2 (gbdt)
  double min_child_weight;        // gbdt: min hessian per child; cls: min instances per child
  double feat_prob;               // RF per-node feature sampling probability (1 = all)
  uint64_t seed;
  int32_t tree;
  double* out_gain;               // [nodes][Fa]
  int32_t* out_bin;               // [nodes][Fa]
  double* out_left;               // [nodes][Fa][2]
};

struct PartitionArgs {
  int32_t* row_node;              // [N]
  const int32_t* default_child;   // [num_nodes] child for rows absent from the split column (-1: not split)
  int32_t num_nodes;
  int64_t N;
  // column pass
  const int64_t* item_start;      // [I] entry ranges (chunks of split columns)
  const int64_t* item_end;
  const int32_t* item_split;      // [I] index into the split arrays below
  int32_t num_items;
  const int32_t* split_default;   // [S] default child id
  const int32_t* split_other;     // [S] the other child id
  const int32_t* split_bin;       // [S] threshold bin: bin <= thr goes left
  const int32_t* split_left_is_default;  // [S]
  const int32_t* csc_row;
  const uint8_t* csc_bin;
};

// counter-based hash -> uniform in [0,1) (splitmix64 finaliser)
FDX_HD uint64_t mix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

FDX_HD double hash_uniform(uint64_t a, uint64_t b, uint64_t c) {
  const uint64_t x = mix64(a ^ mix64(b ^ mix64(c)));
  return (double)(x >> 11) * (1.0 / 9007199254740992.0);
}

// Poisson(1) draw by inversion of the CDF on a counter-based uniform.
FDX_HD int poisson1(double u) {
  double p = 0.36787944117144233, cdf = p;
  int k = 0;
  while (u > cdf && k < 32) { ++k; p /= k; cdf += p; }
  return k;
}

// round-to-nearest-even float -> bf16 bits, and back
FDX_HD uint32_t f2bf(float f) {
  union { float f; uint32_t u; } x; x.f = f;
  uint32_t u = x.u;
  u += 0x7FFFu + ((u >> 16) & 1u);
  return u >> 16;
}
FDX_HD float bf2f(uint32_t b) {
  union { float f; uint32_t u; } x; x.u = b << 16;
  return x.f;
}
// pack v as (hi | lo << 16) with v ~= hi + lo
FDX_HD uint32_t split_bf16(float v) {
  const uint32_t hi = f2bf(v);
  const uint32_t lo = f2bf(v - bf2f(hi));
  return hi | (lo << 16);
}

FDX_HD double gini(double c0, double c1) {
  const double n = c0 + c1;
  if (n <= 0) return 0.0;
  const double p0 = c0 / n, p1 = c1 / n;
  return 1.0 - p0 * p0 - p1 * p1;
}

// Spark Entropy.calculate: -sum p log2 p
FDX_HD double entropy2(double c0, double c1) {
  const double n = c0 + c1;
  if (n <= 0) return 0.0;
  double e = 0.0;
  if (c0 > 0) { const double p = c0 / n; e -= p * (log(p) / log(2.0)); }
  if (c1 > 0) { const double p = c1 / n; e -= p * (log(p) / log(2.0)); }
  return e;
}

FDX_HD double impurity(int mode, double c0, double c1) {
  return mode == 2 ? entropy2(c0, c1) : gini(c0, c1);
}

// Best split of one (node, feature) histogram: bins are scanned in value order, the zero bin
// is node_total - sum(stored bins). Returns the gain (or -inf) and writes bin/left stats.
// mode 0: XGBoost loss_chg = GL^2/(HL+l) + GR^2/(HR+l) - G^2/(H+l), children need H >= mcw.
// mode 1/2: Spark impurity gain, children need (c0+c1) >= min instances.
FDX_HD double best_split_scan(const double* hb, int nb, int zb, double T0, double T1, int mode,
                              double lambda_, double mcw, int* out_bin, double* out_l0, double* out_l1) {
  double s0 = 0.0, s1 = 0.0;
  for (int b = 0; b < nb; ++b)
    if (b != zb) { s0 += hb[2 * b]; s1 += hb[2 * b + 1]; }
  const double z0 = T0 - s0, z1 = T1 - s1;
  double best = -1.0 / 0.0;
  int best_b = -1;
  double bl0 = 0, bl1 = 0;
  double l0 = 0.0, l1 = 0.0;
  const double parent = (mode == 0) ? (T0 * T0) / (T1 + lambda_) : impurity(mode, T0, T1);
  for (int b = 0; b + 1 < nb; ++b) {
    l0 += (b == zb) ? z0 : hb[2 * b];
    l1 += (b == zb) ? z1 : hb[2 * b + 1];
    const double r0 = T0 - l0, r1 = T1 - l1;
    double gain;
    if (mode == 0) {
      if (l1 < mcw || r1 < mcw) continue;
      gain = (l0 * l0) / (l1 + lambda_) + (r0 * r0) / (r1 + lambda_) - parent;
    } else {
      const double nl = l0 + l1, nr = r0 + r1, n = nl + nr;
      if (nl < mcw || nr < mcw || n <= 0) continue;
      gain = parent - (nl / n) * impurity(mode, l0, l1) - (nr / n) * impurity(mode, r0, r1);
    }
    if (gain > best) { best = gain; best_b = b; bl0 = l0; bl1 = l1; }
  }
  *out_bin = best_b;
  *out_l0 = bl0;
  *out_l1 = bl1;
  return best;
}

}  // namespace fdx

// Tree-engine argument structs shared by tree_kernels.hip (gfx950) and tree_cpu.cpp (host).
//
// Exact integer histograms. Every per-row statistic v (GBDT g*w / h*w, or a class count) is
// quantised to q = rint(v * 2^k) with one exponent k per statistic and boosting round (chosen
// from the global max |v| so |q| <= 2^30), and q is stored as NP balanced base-256 digits
// d_i in [-128, 127] (q = sum_i d_i 256^i; NP = 4, or NP = 1 for small integer counts). The
// histogram kernel multiplies one-hot(bin) by digit planes on the i8 matrix cores
// (v_mfma_i32_16x16x64_i8: exact int32 sums), and the per-plane sums are recombined into int64
// histograms. Integer sums do not depend on the order of summation, so histograms, splits and
// trees are bitwise identical on host and device, for any work-item split and any number of
// data-parallel ranks (the int64 partial histograms are summed exactly by the collectives).
//
// Data layout (per data-parallel rank):
//   * quantized CSC: for each active feature fid, entries [colptr[fid], colptr[fid+1]) hold
//     (row int32, bin uint8) sorted by row (row partition, dense-block build);
//   * histogram CSC (models/quantize.py): the entries of the non-dense features re-laid out
//     row-super-block-major (one block's slot/digit slice stays in one XCD's L2), as (row, key)
//     with key = kbase[fid] + bin: work items that pack several small features into one 64-key
//     MFMA tile give each its own key range; single-feature items have kbase 0;
//   * rowdig[row] (2 x uint32): the digits of (q0, q1), plane i in byte i;
//   * slot8[row] (1 B): which of the nodes built by the current pass the row belongs to (0xff:
//     none) -- the only per-level random access besides the statistics;
//   * histograms: hist[node][gbin][stat] int64, bins of all features concatenated (boff[fid]).
#pragma once
#include <math.h>
#include <string.h>
#include <stdint.h>

#include "common.h"

namespace fdx {

// --------------------------------------------------------------------------------- quantisation
// Exponent k for a statistic whose max |v| is m: |rint(v * 2^k)| <= 2^30.
FDX_HD int32_t quant_exponent(double m) {
  if (!(m > 0.0)) return 0;
  int e = 0;
  (void)frexp(m, &e);            // m = f * 2^e, f in [0.5, 1)  ->  m <= 2^e
  return 30 - e;
}

FDX_HD int64_t quantize_value(double v, int32_t k) { return (int64_t)rint(ldexp(v, k)); }

// q (|q| < 2^31 - 2^23) -> 4 balanced base-256 digits, byte i = d_i (two's complement)
// GBDT leaf value of a node's exact sums (G, H scaled by 2^-k): eta * clip(-G / (H + lambda)),
// the fp64 operations of TreeTable.build in the same order (bitwise the host table's value)
FDX_HD double leaf_value(int64_t g, int64_t h, int32_t k0, int32_t k1, double eta, double lambda, double mds) {
  const double G = (double)g * ldexp(1.0, -k0);
  const double H = (double)h * ldexp(1.0, -k1);
  double w = -G / (H + lambda);
  if (mds > 0) w = w < -mds ? -mds : (w > mds ? mds : w);
  return eta * w;
}

FDX_HD uint32_t digits4(int64_t q) { return (uint32_t)(q + 0x80808080ll) ^ 0x80808080u; }
FDX_HD int64_t undigits4(uint32_t d) { return (int64_t)(d ^ 0x80808080u) - 0x80808080ll; }
// NP = 1: the value itself (|q| <= 127) in byte 0
FDX_HD uint32_t digits1(int64_t q) { return (uint32_t)(uint8_t)(int8_t)q; }
FDX_HD int64_t undigits1(uint32_t d) { return (int64_t)(int8_t)(uint8_t)(d & 0xffu); }

struct QuantArgs {
  const float* g;             // GBDT gradients (mode 0)
  const float* h;
  const float* label;         // classification labels 0/1 (mode 1)
  const float* weight;        // optional instance weights
  uint64_t seed;              // Poisson(1) bootstrap when bootstrap != 0 (mode 1)
  int32_t tree;
  int32_t bootstrap;
  int32_t mode;               // 0 = gbdt (g, h), 1 = classification counts (w[y==0], w[y==1])
  int32_t np;                 // digits per statistic: 4, or 1 for integer counts <= 127
  int32_t* kexp_out;          // [2] quantisation exponents used (written once)
  int64_t N;
  uint32_t* rowdig;           // [N * 2]
  int64_t* totals;            // [2] += sum of q over the rows (exact)
  uint8_t* digp;              // optional plane-major copy [2 * np][n_pad] (dense histogram path)
  int64_t n_pad;
  int64_t row0;               // global index of row 0 of this shard (bootstrap draws are per global row)
  // optional, one-launch forms (device level loop, models/grower.py): the last workgroup to finish
  // (ticket) reduces the per-workgroup partials itself instead of a second launch, and then
  // writes the root state of the tree: stats[0] = totals[0] row = the exact totals, open[0] = 0,
  // the exponents into the node-table arena; row_node[r] = 0 for every row on the way
  unsigned int* ticket;
  int64_t* root_stats;
  int64_t* root_totals;
  int32_t* root_open;
  int32_t* kexp_copy;
  int32_t* row_node;
  // ... or with no ticket (atomic_root): every workgroup adds its partial sums into one of
  // kRootSlots slots of root_parts (slot = workgroup % kRootSlots, a 128-byte line each; the
  // same-address form serialised at ~11 ns per atomic, bench/probes/atomic_contention.hip) and
  // workgroup 0 writes open[0], the exponents and zeroes root_parts_clear (the next tree's slots).
  // The level-0 split search and plan sum the slots themselves (SplitArgs / LevelPlanArgs
  // root_parts) -- no grid-wide completion test and no reduction launch.
  uint16_t* dig16;            // optional (np == 1): [N] the row's two count digits (byte 0: q0, byte 1: q1)
  int32_t atomic_root;
  int64_t* root_parts;        // [kRootSlots][kRootStride] (words 0, 1: the two sums)
  int64_t* root_parts_clear;
  // max |g|, |h| as kRootSlots slots of bit patterns (grad_max_kernel); nullptr: maxv
  const unsigned long long* max_parts;
  int64_t* zero;              // optional: [zero_n] int64 zeroed on the way (the root histogram)
  int64_t zero_n;
};
constexpr int kRootSlots = 32;
constexpr int kRootStride = 16;           // int64 words per slot (one 128-byte line)

// the root's exact sums from the kRootSlots slots (a wave: lanes 0..31 one slot each)
FDX_HD void root_sums(const int64_t* parts, int64_t* t0, int64_t* t1) {
  int64_t a = 0, b = 0;
  for (int k = 0; k < kRootSlots; ++k) {
    a += parts[kRootStride * k];
    b += parts[kRootStride * k + 1];
  }
  *t0 = a;
  *t1 = b;
}

// Tree-start work folded into the first launch of a GBDT round (grad_max_kernel): the node-table
// arena image copied in (init_n 8-byte words), the root histogram zeroed, and the other parity's
// max |g|, |h| slot cleared for the next round's atomics.
struct PrologueInit {
  const uint64_t* init_src;
  uint64_t* init_dst;
  int64_t init_n;
  int64_t* zero;
  int64_t zero_n;
  unsigned long long* max_clear;   // [kRootSlots][kRootStride]: the next round's max slots
};

struct SlotArgs {
  const int32_t* row_node;    // [N] current node id of each row
  const int32_t* node_slot;   // [num_nodes] slot being built (absolute), -1 otherwise
  int32_t num_nodes;
  int32_t slot_base;          // this pass covers slots [slot_base, slot_base + nslots)
  int32_t nslots;
  int64_t N;
  uint8_t* slot8;             // [N] slot - slot_base, or 0xff
  const uint32_t* rowdig;     // optional (single-slot passes): rowdig [N * 2] ->
  uint32_t* masked;           //   masked [N * 2] = the row's digit words in slot 0, else 0
  uint32_t* pack;             // optional (np = 1): pack [N] = slot | (rowdig[2r] & 0xff) << 8 | (rowdig[2r+1] & 0xff) << 16
};

// Work item meta (item_meta): stride_log2 | nfeat << 8 | koff << 16. The item covers keys
// [koff, koff + 16*BT); key ek belongs to feature f0 + (ek >> stride_log2), bin ek & (stride-1).
FDX_HD int32_t item_stride_log2(int32_t m) { return m & 0xff; }
FDX_HD int32_t item_nfeat(int32_t m) { return (m >> 8) & 0xff; }
FDX_HD int32_t item_koff(int32_t m) { return (m >> 16) & 0xff; }

struct HistArgs {
  const int64_t* item_start;      // [I] entry range of each work item
  const int64_t* item_end;
  const int32_t* item_f0;         // [I] first feature of the item
  const int32_t* item_meta;       // [I]
  int32_t num_items;
  const int32_t* wave_item;       // [num_slots] item of each wave slot (-1 idle); nullptr: slot = item
  int32_t num_slots;
  const int32_t* csc_row;
  const uint8_t* csc_key;
  const uint8_t* slot8;           // [N] relative slot, 0xff = not built; nullptr = root pass (all slot 0)
  const uint32_t* rowdig;         // [N * 2]
  const int64_t* boff;            // [Fa + 1]
  const int32_t* nbins;           // [Fa]
  const int32_t* slot_node;       // [nslots] histogram row of each slot of the pass (-1: none)
  int32_t nslots;
  int64_t hist_stride;            // bins per histogram row (TB, or TB + 1 when padded)
  int64_t* hist;                  // [rows][hist_stride][2], accumulated (+=)
  const uint8_t* feat_active;     // [Fa] optional: items without an active feature are skipped (RF)
  const uint32_t* rowpack;        // [N] optional, np = 1 passes: slot | digit0 << 8 | digit1 << 16 (slot8 unused)
  int32_t* active_list;           // optional: listed pass, the active items compacted per XCD ...
  int32_t* active_count;          //   ... [8]: their count per XCD (list x at x * list_cap)
  int32_t list_cap;               // wave slots per XCD (set by the launch)
  // optional (data-parallel batched levels): feature f's bins start at boff[f] + shard_of[f] *
  // shard_bins (its shard's chunk of the batch's send buffer), so the per-level offsets need no
  // separate add pass
  const int64_t* shard_of;
  int64_t shard_bins;
  int32_t listed_per_xcd;         // -1: the launch compacts the list and strides a fixed grid over
                                  // it; >= 0: the list was compacted beforehand (hist_select) and
                                  // its largest per-XCD count is known: one wave per active item
  int32_t lds;                    // np = 1 passes: LDS-atomic kernel (hist_lds_kernel) instead of MFMA
};

// waves of a listed histogram pass (they stride over the active items): 8 per SIMD of 256 CUs
constexpr int32_t kListedWaves = 8192;

FDX_HD int64_t hist_boff(const HistArgs& a, int32_t f) {
  return a.boff[f] + (a.shard_of ? a.shard_of[f] * a.shard_bins : 0);
}

// ------------------------------------------------------------------ row-group histogram engine
// Row-group CSR ("RG", models/quantize.py RowGroups): the active features are packed, densest
// first, into groups of at most kRgBins local bins (a feature's bins stay contiguous inside its
// group); for group g, row r's entries are ent[gbase[g] + ptr[g][r] .. gbase[g] + ptr[g][r + 1])
// as uint16 local bins. A level's built rows are listed by node slot (rg_list), and a workgroup
// of the histogram pass (row_kernels.hip) takes one group and a contiguous range of that list:
// each lane walks one row's run of entries with 16-byte loads (a row's entries are contiguous,
// so the per-entry row gathers of the CSC passes become one gather per (row, group)) and adds the
// row's two quantised statistics into int64 LDS histograms of the group's bins, flushed with
// integer atomics per node slot. Integer sums are order-free: the histograms are bitwise those of
// the CSC passes and the host.
constexpr int kRgBins = 8192;               // max local bins per group: 2 x 8192 x int64 = 128 KB of LDS
                                            // (4096-bin groups: two workgroups per CU)
constexpr int kRgWaves = 16;                // 1024 threads per workgroup (one workgroup per CU)
constexpr int kRgMaxSlots = 64;

struct RgBuildArgs {
  const int32_t* csc_row;         // feature-major CSC (quantized)
  const uint8_t* csc_bin;
  const int64_t* colptr;          // [Fa + 1]
  int32_t Fa;
  int64_t nnz;
  int64_t N;
  const int32_t* fgroup;          // [Fa] group of each feature (-1: not in the engine)
  const int32_t* flocal;          // [Fa] local bin of the feature's bin 0 inside its group
  int32_t entries_per_thread;
  uint32_t* ptr;                  // pass 0: [G][N + 1], entry counts added at [g][r + 1]
  uint32_t* cursor;               // pass 1: [G][N] next free position of each (group, row) (advanced)
  const int64_t* gbase;           // pass 1: [G + 1] first entry of each group
  uint16_t* ent;                  // pass 1 out
};

// Row-group CSR straight from the count-path CSR (rows of term counts, the bench corpus): a wave
// per row, groups counted / placed with ballots, so runs keep the CSR order and no atomics are
// needed (the CSC build: ~2 returning atomics per entry, ~0.1 s at 10M rows).
// Entry (row r, feature f, count c): fa = remap[f] (-1: inactive), bin = c <= 0 ? 0 :
// min(c, 255, max_bin) (the count path's binning), local = flocal[fa] + bin.
template <class V>
struct RgCsrBuildArgs {
  const int64_t* indptr;          // [N + 1]
  const int32_t* idx;             // [nnz] original feature ids
  const V* counts;                // [nnz]
  int64_t N;
  const int32_t* remap;           // [F] active index of each feature (-1: inactive)
  int32_t max_bin;                // max_bins - 1
  const int32_t* fgroup;          // [Fa]
  const int32_t* flocal;          // [Fa]
  const int32_t* fgl;             // (device) [F] group << 16 | local offset of each feature, -1:
                                  //   none (remap, fgroup and flocal folded into one lookup)
  int32_t G;
  uint32_t* ptr;                  // [G][N + 1] out: exclusive starts of every (group, row) run
  const int64_t* gbase;
  uint16_t* ent;                  // out
  uint32_t* wave_base;            // [G][stride] scratch: per-wave group totals, then bases (+ totals)
  uint32_t* erow;                 // optional out: erow[gbase[g] - ebase + k] = row of entry k of
  int32_t em_g0;                  //   group g >= em_g0 (the entry-major rows, RgHistArgs::erow)
  int64_t ebase;
};

// Built rows of a level grouped by slot. The slot of row r is node_slot[row_node[r]] when
// row_node is given (slots outside [0, nslots): not built), else slot8[r] (0xff: not built).
// rows per wave of the list kernels: 512 up to 4M rows (1M rows: ~2K waves; 2048-row chunks left
// ~500 waves and 19 us per pass), 2048 beyond (profiles/r4/gbdt_list_rows_ab.txt). Host only (the
// kernel takes RgListArgs::list_rows); tests lower the 4M threshold to run the large-shard paths
// (2048-row waves, no partition row counts, fewest-rows sibling choice) on small data.
inline int64_t g_rg_list_big_rows = 4ll << 20;
inline int32_t rg_list_rows(int64_t N) { return N <= g_rg_list_big_rows ? 512 : 2048; }
struct RgListArgs {
  const int32_t* row_node;        // [N] or nullptr
  const int32_t* node_slot;       // [num_nodes] slot of each node (-1: not built)
  int32_t num_nodes;
  const uint8_t* slot8;           // [N] (when row_node is nullptr)
  int64_t N;
  int32_t nslots;
  int32_t* slot_count;            // [nslots] totals (pass 2)
  int32_t list_rows;              // rg_list_rows(N) (set by launch_rg_list)
  int32_t* wave_count;            // [ceil(N / rg_list_rows(N))][nslots]: per-wave counts (pass 0), then
                                  //   per-wave offsets inside each slot (pass 2)
  int32_t* slot_start;            // [nslots + 1] out (pass 1)
  int32_t* list;                  // [N] out (pass 1): built rows grouped by slot, ascending inside each
                                  //   wave's chunk of rows
  const uint32_t* rowdig;         // optional [N * 2]: pass 1 also writes
  uint32_t* listdig;              //   listdig[2 pos + k] = rowdig[2 list[pos] + k] (coalesced in the pass)
  uint32_t* masked;               // optional [N * 2] (nslots == 1, with rowdig): pass 1 writes every
                                  //   row's digit words, zero outside slot 0 (the entry-major pass)
  int32_t counted;                // pass 0's per-wave counts already written (PartitionArgs count_work)
  // optional (row_node mode): the partition's rows per next-level node per 512-row wave
  // (PartitionArgs node_counts) and that level's first node id (*nc_base): the scan (pass 2) sums
  // a list wave's 512-row waves for its slot's node, and pass 0 is skipped
  const int32_t* node_counts;
  const int32_t* nc_base;
};
constexpr int32_t kPartWaveRows = 512;   // rows of one partition wave (64 lanes x 8 rows)

FDX_HD uint32_t rg_slot_of(const RgListArgs& a, int64_t r) {
  if (!a.row_node) return a.slot8[r];
  const int32_t n = a.row_node[r];
  const int32_t s = (n >= 0 && n < a.num_nodes) ? a.node_slot[n] : -1;
  return (s >= 0 && s < a.nslots) ? (uint32_t)s : 0xffu;
}

struct RgHistArgs {
  const uint32_t* ptr;            // [G][N + 1]
  const uint16_t* ent;            // entries (readable padding behind the end)
  const int64_t* gbase;           // [G + 1]
  const int32_t* gbin;            // [G][gbins] histogram column of each local bin (-1: unused)
  int32_t gbins;                  // local bins per group: 4096 or 8192
  int32_t G;
  int64_t N;
  const uint32_t* rowdig;         // [N * 2] digit words (by row; the list pass reads listdig)
  int32_t np;                     // 4: q = undigits4, 1: q = undigits1
  const int32_t* list;            // built rows grouped by slot (nullptr: rows 0..N-1, one slot)
  const uint32_t* listdig;        // [T * 2] digit words by list position (with list)
  const uint8_t* gmode;           // [G] 1: lane-balanced batches (dense groups), 0: a lane per row
  const int32_t* slot_start;      // [nslots + 1] (nullptr with list == nullptr)
  int32_t nslots;
  // work table: workgroup w takes chunk wg_p[w] of the wg_np[w] equal chunks of the list, for
  // group wg_g[w] (groups get chunks in proportion to their entries)
  const int32_t* wg_g;
  const int32_t* wg_p;
  const int32_t* wg_np;
  int32_t n_wg;
  // diagnostics (bench/probes/rg_probe.py): bit 1 replaces the LDS atomics by a register sum,
  // bit 2 skips the flushes (wrong sums)
  int32_t dbg;
  // output: hist[(slot_node[s] * hist_stride + off(column)) * 2 + stat] +=
  const int32_t* slot_node;
  int64_t hist_stride;
  int64_t* hist;
  int32_t nshards;                // 0: off(c) = c; else column c of shard s (shard_lo[s] <= c <
                                  //   shard_lo[s + 1]) -> s * shard_stride + c - shard_lo[s]
  const int64_t* shard_lo;
  int64_t shard_stride;
  // Entry-major pass of the sparse groups (gmode 0, entries from ebase on) at single-slot levels:
  // erow[e - ebase] = row of entry e. The all-rows pass always takes it (digits from rowdig); a
  // listed level takes it when it lists >= em_min_rows rows, with emdig = every row's digit words
  // zeroed outside slot 0 (RgListArgs::masked). nullptr erow: the row-list pass everywhere.
  const uint32_t* erow;
  int64_t ebase;
  const uint32_t* emdig;
  int64_t em_min_rows;
  // optional (data-parallel root level): workgroup 0 also writes the root's sums (the
  // quantisation's kRootSlots slots) into bin 0 of row nslots of every shard chunk (the totals
  // row the reduce-scatter sums across ranks)
  const int64_t* root_parts;
  // optional: workgroup w stores its whole LDS table to part[w][gbins][2] (plain stores) and
  // rg_reduce_kernel sums the workgroups of each group (work-table entries wg_first[g] ..
  // wg_first[g + 1]) into the level histogram, instead of every workgroup adding its table into
  // the same bins with integer atomics (~30 % of the root pass at 1M rows with ~200 workgroups on
  // the dense group; ~50 us of every listed level there, profiles/r5/NOTES.md). Several slots:
  // only a workgroup whose chunk lies inside one slot stores its table (rg_part_slot); the few
  // across a slot boundary flush with atomics
  int64_t* part;
  const int32_t* wg_first;
};

// After a level's partition: per sibling pair of the next level, build the child with FEWER ROWS
// (rows from PartitionArgs rows_out) instead of the plan's smaller hessian sum, rewriting the
// plan's build tables (node_slot, s2n, sub_dst, sub_sib, sub_of). The histograms are exact
// integer sums, so the trees do not depend on which sibling is built; the row lists get shorter
// (bench/probes/list_oracle.py: the hessian rule listed 6-24 % more rows than needed).
struct LevelChooseArgs {
  const int32_t* counts;          // the level's counts row ([2] = builds of the next level)
  const int32_t* rows_base;       // first node id of the next level
  int32_t* rows_out;              // [32][64] spread row counts (read and zeroed here)
  const int32_t* next_open;
  int32_t* node_slot;
  int32_t* s2n;
  int32_t* sub_dst;
  int32_t* sub_sib;
  int32_t* sub_of;                // optional
};

// Whether group g of a pass listing T rows takes the entry-major pass.
FDX_HD bool rg_use_em(const RgHistArgs& a, int g, int64_t T) {
  if (a.erow == nullptr || a.gmode[g] != 0 || a.gbase[g] < a.ebase || a.nslots != 1) return false;
  if (a.list == nullptr) return true;
  return a.emdig != nullptr && T >= a.em_min_rows;
}

// Partial tables of a listed pass over several slots: the slot whose list range holds workgroup
// w's whole chunk [T p / np, T (p + 1) / np) -- its table goes to part[w] -- else -1 (an empty
// chunk, or one across a slot boundary: that workgroup flushes with atomics). The same slot search
// as rg_hist_kernel's.
FDX_HD int rg_part_slot(const RgHistArgs& a, int w, int64_t T) {
  const int64_t p = a.wg_p[w], np = a.wg_np[w];
  const int64_t a0 = T * p / np, a1 = T * (p + 1) / np;
  if (a0 >= a1) return -1;
  int s = 0;
  while (s + 1 < a.nslots && a.slot_start[s + 1] <= a0) ++s;
  return a1 <= (int64_t)a.slot_start[s + 1] ? s : -1;
}

// Digit words of the entry-major pass, by row.
FDX_HD const uint32_t* rg_em_digits(const RgHistArgs& a) { return a.list ? a.emdig : a.rowdig; }

// erow of the groups from g0 on: erow[gbase[g] - gbase[g0] + e] = r for every entry e of row r.
struct RgErowArgs {
  const uint32_t* ptr;            // [G][N + 1]
  const int64_t* gbase;           // [G + 1] (host copy for the CPU twin, device for the kernel)
  int32_t G;
  int32_t g0;
  int64_t N;
  int64_t ebase;                  // gbase[g0]
  uint32_t* erow;
};

FDX_HD int64_t rg_col_offset(const RgHistArgs& a, int64_t b) {
  if (a.nshards <= 0) return b;
  int s = 0;
  while (s + 1 < a.nshards && b >= a.shard_lo[s + 1]) ++s;
  return (int64_t)s * a.shard_stride + b - a.shard_lo[s];
}

FDX_HD int64_t rg_q(uint32_t d, int np) { return np == 4 ? undigits4(d) : undigits1(d); }

// RF per-level feature sampling (rf_kernels.hip / tree_cpu.cpp): for each of `nnodes` nodes the
// k-th smallest feature_priority over feature indices 0..F-1 (exact, as a 53-bit integer u with
// priority = u * 2^-53), and the union mask over the active features fid_orig[0..Fa).
struct RfSampleArgs {
  uint64_t seed;
  int32_t tree;
  const int32_t* nodes;           // [nnodes]
  const int32_t* node_trees;      // [nnodes] optional per-node tree (RF batches); nullptr: `tree`
  int32_t nnodes;
  int64_t F;
  int64_t k;
  const int64_t* fid_orig;        // [Fa]
  int64_t Fa;
  double* thr;                    // [nnodes] out
  uint8_t* mask;                  // [Fa] out
  uint8_t* scratch;               // device: rf_scratch_bytes(nnodes) for the window fast path (or null)
  // optional (with scratch): one launch for window + threshold. [3 * fused_cap] uint32, zero at
  // the first use and left zero by every launch: per node its workgroup ticket, the count below
  // the window and the candidate count (the last window workgroup of a node ranks its candidates)
  uint32_t* fused_counts;
  int32_t fused_cap;
  const uint64_t* fmix;           // optional [F]: mix64(f) (feature_priority_u53_pre)
};

FDX_HD int32_t rf_tree_of(const RfSampleArgs& a, int64_t i) { return a.node_trees ? a.node_trees[i] : a.tree; }

// Compact data-parallel layout of one RF level (models/grower.py FeatureShards.compact): shard s
// owns the active features [fs[s], fs[s+1]); inside the shard, the features of the level's union
// sample mask get consecutive bin ranges (local[f] = exclusive prefix of the masked nbins) and
// every other feature points at the shard's trash range [sizes[s], sizes[s] + max nbins), which
// only the entries of unsampled features sharing a work item with a sampled one ever reach and
// nothing reads. A level's reduce-scatter then carries the sampled features' bins only (a node
// samples ceil(sqrt(F)) of F features: ~3% of the bins at 16 nodes, 0.2% at the root).
struct RfCompactArgs {
  const uint8_t* mask;            // [Fa] union sample mask of the level
  const int32_t* nbins;           // [Fa]
  const int64_t* fs;              // [S + 1] shard feature boundaries
  int32_t S;
  int64_t Fa;
  int64_t* local;                 // [Fa + 1] out: offset inside the feature's shard row (local[Fa] = 0)
  int64_t* sizes;                 // [S] out: masked bins per shard (= the trash range start)
  int64_t* chunk_sums;            // optional: [S][chunk_stride] scratch of the multi-workgroup layout
  int64_t chunk_stride;           //   (rf_compact_chunks(largest shard's feature count) per shard)
};

inline int64_t rf_scratch_bytes(int64_t nnodes) { return 8 * ((2 * nnodes * 4 + 7) / 8) + nnodes * 2048 * 8; }

// Dense path for high-density features: dense[d][row] = bin of hot feature d (zbin when absent),
// column-major with n_pad (multiple of 64) bytes per feature; the row statistics are streamed from
// the plane-major digit copy, the slots from slot8 (padded to n_pad with 0xff). A wave builds the
// histograms of FG features (gfid[grp * FG + j]: Fa index, -1 none; gdense: row of `dense`) over a
// range of range_rows rows; ranges are placed so that all groups of one range share an XCD.
struct DenseHistArgs {
  const uint8_t* dense;           // [Fh][n_pad]
  const uint8_t* digp;            // [2 * NP][n_pad]
  const uint32_t* rowdig;         // [N * 2] (host path)
  int64_t n_rows;
  const uint8_t* slot8;           // [n_pad] (nullptr: root pass)
  int64_t n_pad;
  int64_t range_rows;             // multiple of 64
  int32_t nranges;
  int32_t ngroups;
  const int32_t* gfid;            // [ngroups * FG]
  const int32_t* gdense;          // [ngroups * FG]
  const int64_t* boff;
  const int32_t* nbins;
  const int32_t* slot_node;
  int32_t nslots;
  int64_t hist_stride;
  int64_t* hist;
};

struct SplitArgs {
  const int64_t* hist;            // [nodes][hist_stride][2]
  const int64_t* totals;          // [nodes][2]
  int64_t hist_stride;            // bins per node row of hist (0: boff[Fa])
  int32_t num_nodes;
  int32_t Fa;
  const int64_t* boff;
  const int32_t* nbins;
  const int32_t* zbin;
  const int64_t* fid_orig;        // [Fa] original feature index (RF sampling key)
  const int32_t* node_ids;        // [nodes] tree-global node id (RF sampling key)
  const int32_t* kexp;            // [2] quantisation exponents of the two statistics
  int32_t mode;                   // 0 = xgboost newton gain, 1 = gini, 2 = entropy
  double lambda_;                 // L2 (gbdt)
  double min_child_weight;        // gbdt: min hessian per child; cls: min instances per child
  const double* feat_thr;         // RF: [nodes] sampling threshold (feature kept iff u <= thr); nullptr: all
  uint64_t seed;
  int32_t tree;
  const int32_t* node_tree;       // RF batches: [nodes] tree index of each node (nullptr: `tree`)
  const uint64_t* fmix;           // optional [F]: mix64(f) of the sampling priorities
  double* out_gain;               // [nodes][Fa]
  int32_t* out_bin;               // [nodes][Fa]
  int64_t* out_left;              // [nodes][Fa][2]
  // optional: the features with more than kSplitWide bins, searched a wave per (node, feature)
  // (the thread-per-feature kernel skips them)
  const int32_t* wide;
  int32_t n_wide;
  // optional: histogram row of node n (data-parallel levels: the reduce-scattered built rows and
  // the subtracted siblings stay where they were written, see LevelRowsArgs); nullptr: row n
  const int32_t* row_of;
  // optional (Fa >= 64): per wave of the narrow search, the best (gain, feature) of each of the
  // <= 2 nodes its features belong to ([2 * waves]; NaN gain: a NaN in the segment). The
  // best-split pass then reads ~Fa / 64 partials per node instead of Fa gains.
  double* part_gain;
  int32_t* part_f;
  // optional: the root's totals as QuantArgs root_parts slots (level 0 of the fused prologue)
  const int64_t* root_parts;
  // optional (single-process levels >= 1): the sibling subtraction inside the search. Open node n
  // with sub_of[n] = k >= 0 has no histogram yet: (n, f)'s bins are parent_hist row sub_par[k] -
  // hist row sub_sib[k], written to row n as they are searched (hist_subtract_kernel's result,
  // without its launch and its second pass over the rows)
  const int32_t* sub_of;
  const int32_t* sub_par;
  const int32_t* sub_sib;
  const int64_t* parent_hist;
};
constexpr int32_t kSplitWide = 16;

FDX_HD int64_t split_row(const SplitArgs& a, int n) { return a.row_of ? a.row_of[n] : n; }

// Data-parallel level rows (models/grower.py, DP levels of the device loop): the built nodes'
// reduce-scattered partials stay where the collective left them (row bld_base + slot k) and the
// larger sibling of slot k is written to row sub_base + k of the same buffer, so no histogram row
// is ever copied into open-node order. Per built slot k: row_of[open index] for the split search,
// and the subtraction triple as rows (dst, sib in this level's buffer; par in the previous
// level's, through its row_of; nullptr: the previous level's rows are its open indices).
struct LevelRowsArgs {
  const int32_t* s2n;             // [nb] open index of slot k (tree.h level_plan)
  const int32_t* sub_dst;         // [nb] open index of slot k's larger sibling (-1: none)
  const int32_t* sub_par;         // [nb] open index of the parent in the previous level
  const int32_t* prev_row_of;     // [previous n_open] or nullptr
  int32_t nb;
  int32_t bld_base, sub_base;
  int32_t* row_of;                // [n_open] out
  int32_t* dst_row;               // [nb] out (-1: no subtraction)
  int32_t* par_row;
  int32_t* sib_row;
};

FDX_HD void level_rows_slot(const LevelRowsArgs& a, int32_t k) {
  const int32_t bld = a.bld_base + k, d = a.sub_dst[k];
  a.row_of[a.s2n[k]] = bld;
  a.sib_row[k] = bld;
  if (d >= 0) {
    a.row_of[d] = a.sub_base + k;
    a.dst_row[k] = a.sub_base + k;
    a.par_row[k] = a.prev_row_of ? a.prev_row_of[a.sub_par[k]] : a.sub_par[k];
  } else {
    a.dst_row[k] = a.par_row[k] = -1;
  }
}

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
  const int32_t* csc_row;         // feature-major CSC (all features)
  const uint8_t* csc_bin;
  // splits on dense-block (hot) features are applied in the row pass from the column-major bins:
  // node_dense[4 n] = {dense row (-1: column pass), threshold bin, left child, right child}
  const int32_t* node_dense;
  const uint8_t* dense;           // [Fh][n_pad]
  int64_t n_pad;
  // optional (RF sampled levels): the next level's packed row state written with the partition
  // (csrc/tree.h SlotArgs pack: slot of the row's new node | class-count digits << 8), so that
  // level needs no row pass of its own: pack[r] from pack_slot[node] (the next level's node
  // slots, level_plan's node_slot; -1 = not built) and the digit words pack_dig [N][2]
  const int32_t* pack_slot;
  const uint32_t* pack_dig;
  uint32_t* pack;
  // ... or the digits as [N] uint16 (QuantArgs dig16: 2 bytes a row read instead of 8)
  const uint16_t* pack_dig16;
  // optional: the node table's parent array. Then the column pass runs FIRST (moving a split
  // node's rows present in its column to the other child: row_node == parent[default child]) and
  // the row pass second, so the row pass sees every row's final node -- it writes the packed
  // state of all rows and, with count_work, the next level's per-wave slot counts (RgListArgs
  // pass 0: count_work[2 ns + w ns + s] for the 512-row wave w, ns = *count_nslots slots of
  // count_slot[node]) -- one pass over the rows less per level
  const int32_t* node_parent;
  int32_t* count_work;
  const int32_t* count_slot;
  const int32_t* count_nslots;
  // optional (rows_base given): the rows of each next-level node, node id *rows_base + i for i < 64,
  // added into rows_out[(block % 32) * 64 + i] (32 spread copies; LevelChooseArgs; one grid pass
  // over the rows), and / or kept per 512-row chunk w in node_counts[i * ceil(N / 512) + w] (every
  // lane written; any grid), from which the next level's row lists take their per-wave slot counts
  // (RgListArgs node_counts) instead of a counting pass over row_node
  int32_t* rows_out;
  const int32_t* rows_base;
  int32_t* node_counts;
  int32_t count_ballot;           // the counts above and count_work's by wave ballots (<= 4 values)
  // optional: zero this int64 range on the way (the next level's histograms: no fill launch)
  int64_t* zero;
  int64_t zero_n;
};

FDX_HD uint32_t partition_pack_word(const PartitionArgs& a, int32_t node, int64_t r) {
  const int32_t s = (node >= 0 && node < a.num_nodes) ? a.pack_slot[node] : -1;
  const uint32_t sb = (s >= 0 && s < 255) ? (uint32_t)s : 0xffu;
  if (a.pack_dig16) return sb | ((uint32_t)a.pack_dig16[r] << 8);
  const uint32_t d0 = a.pack_dig[2 * r], d1 = a.pack_dig[2 * r + 1];
  return sb | ((d0 & 0xffu) << 8) | ((d1 & 0xffu) << 16);
}

// Child of row r of split node n in the row pass.
FDX_HD int32_t partition_row_child(const PartitionArgs& a, int32_t n, int64_t r) {
  const int32_t c = a.default_child[n];
  if (c < 0 || a.node_dense == nullptr) return c;
  const int32_t* nd = a.node_dense + 4 * (int64_t)n;
  if (nd[0] < 0) return c;
  return (int32_t)a.dense[(int64_t)nd[0] * a.n_pad + r] <= nd[1] ? nd[2] : nd[3];
}

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

// RF per-node feature priority (uniform in [0,1)): the node samples the features with the k
// smallest priorities (exactly k, without replacement).
FDX_HD double feature_priority(uint64_t seed, int32_t tree, int32_t node, int64_t fid) {
  return hash_uniform(seed ^ 0x5bd1e995ull, ((uint64_t)(uint32_t)tree << 32) | (uint32_t)node, (uint64_t)fid);
}

// The 53-bit integer behind feature_priority (priority == u * 2^-53 exactly).
FDX_HD uint64_t feature_priority_u53(uint64_t seed, int32_t tree, int32_t node, int64_t fid) {
  const uint64_t x = mix64((seed ^ 0x5bd1e995ull) ^
                           mix64((((uint64_t)(uint32_t)tree << 32) | (uint32_t)node) ^ mix64((uint64_t)fid)));
  return x >> 11;
}

// feature_priority_u53 with mix64(fid) looked up (RfSampleArgs / SplitArgs fmix: the table of
// mix64(f) over the F features, shared by every node and tree): one mix64 of three per priority
FDX_HD uint64_t feature_priority_u53_pre(uint64_t seed, int32_t tree, int32_t node, uint64_t mf) {
  return mix64((seed ^ 0x5bd1e995ull) ^ mix64((((uint64_t)(uint32_t)tree << 32) | (uint32_t)node) ^ mf)) >> 11;
}

// Work item `item` holds at least one active feature (always true without a mask).
// The active-item selects of one level's sampled item groups in one launch (grid row g = group
// g): hist_select_kernel's body per group; counts zeroed beforehand (LevelPlanArgs counts_tail).
constexpr int kSelGroups = 4;
struct SelectArgs {
  const int32_t* item_f0[kSelGroups];
  const int32_t* item_meta[kSelGroups];
  const int32_t* wave_item[kSelGroups];
  int32_t num_items[kSelGroups];
  int32_t num_slots[kSelGroups];
  int32_t list_cap[kSelGroups];
  int32_t* list[kSelGroups];
  int32_t* count[kSelGroups];       // [8] per-XCD counts of the group
  int32_t n;
  const uint8_t* feat_active;
};

FDX_HD bool item_active(const HistArgs& a, int64_t item) {
  if (!a.feat_active) return true;
  const int32_t f0 = a.item_f0[item];
  const int nf = (a.item_meta[item] >> 8) & 0xFF;
  for (int j = 0; j < nf; ++j)
    if (a.feat_active[f0 + j]) return true;
  return false;
}

// Poisson(1) draw by inversion of the CDF on a counter-based uniform (at most 32).
FDX_HD int poisson1(double u) {
  double p = 0.36787944117144233, cdf = p;
  int k = 0;
  while (u > cdf && k < 32) { ++k; p /= k; cdf += p; }
  return k;
}

// The two statistics of one row before quantisation.
FDX_HD void row_stats(const QuantArgs& a, int64_t r, double* v0, double* v1) {
  if (a.mode == 0) {
    const double w = a.weight ? (double)a.weight[r] : 1.0;
    *v0 = (double)a.g[r] * w;
    *v1 = (double)a.h[r] * w;
  } else {
    double w = a.weight ? (double)a.weight[r] : 1.0;
    if (a.bootstrap) w *= (double)poisson1(hash_uniform(a.seed, (uint64_t)a.tree, (uint64_t)(a.row0 + r)));
    const double y = (double)a.label[r];
    *v0 = w * (1.0 - y);
    *v1 = w * y;
  }
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

// Parent term of the split gain of a node with exact totals (T0, T1).
FDX_HD double split_parent(int mode, int64_t T0, int64_t T1, double s0, double s1, double lambda_) {
  const double G = (double)T0 * s0, H = (double)T1 * s1;
  return (mode == 0) ? (G * G) / (H + lambda_) : impurity(mode, G, H);
}

// Gain of sending the left sums (l0, l1) left; false when a child violates the minimum.
FDX_HD bool split_gain_at(int mode, int64_t l0, int64_t l1, int64_t T0, int64_t T1, double s0, double s1,
                          double parent, double lambda_, double mcw, double* gain) {
  const double L0 = (double)l0 * s0, L1 = (double)l1 * s1;
  const double R0 = (double)(T0 - l0) * s0, R1 = (double)(T1 - l1) * s1;
  if (mode == 0) {
    if (L1 < mcw || R1 < mcw) return false;
    *gain = (L0 * L0) / (L1 + lambda_) + (R0 * R0) / (R1 + lambda_) - parent;
  } else {
    const double nl = L0 + L1, nr = R0 + R1, n = nl + nr;
    if (nl < mcw || nr < mcw || n <= 0) return false;
    *gain = parent - (nl / n) * impurity(mode, L0, L1) - (nr / n) * impurity(mode, R0, R1);
  }
  return true;
}

// Best split of one (node, feature) histogram of exact integer sums: bins are scanned in value
// order, the zero bin is node_total - sum(stored bins). s0/s1 = 2^-k of the two statistics.
// Returns the gain (or -inf) and writes the bin and the left sums: the first bin of the largest
// gain (NaN gains never win). split_wide_kernel (tree_kernels.hip) computes the same per lane.
// mode 0: XGBoost loss_chg = GL^2/(HL+l) + GR^2/(HR+l) - G^2/(H+l), children need H >= mcw.
// mode 1/2: Spark impurity gain, children need (c0+c1) >= min instances.
FDX_HD double best_split_scan(const int64_t* hb, int nb, int zb, int64_t T0, int64_t T1, double s0, double s1,
                              int mode, double lambda_, double mcw, int* out_bin, int64_t* out_l0, int64_t* out_l1) {
  int64_t a0 = 0, a1 = 0;
  for (int b = 0; b < nb; ++b)
    if (b != zb) { a0 += hb[2 * b]; a1 += hb[2 * b + 1]; }
  const int64_t z0 = T0 - a0, z1 = T1 - a1;
  double best = -1.0 / 0.0;
  int best_b = -1;
  int64_t bl0 = 0, bl1 = 0;
  int64_t l0 = 0, l1 = 0;
  const double parent = split_parent(mode, T0, T1, s0, s1, lambda_);
  for (int b = 0; b + 1 < nb; ++b) {
    l0 += (b == zb) ? z0 : hb[2 * b];
    l1 += (b == zb) ? z1 : hb[2 * b + 1];
    double gain;
    if (!split_gain_at(mode, l0, l1, T0, T1, s0, s1, parent, lambda_, mcw, &gain)) continue;
    if (gain > best) { best = gain; best_b = b; bl0 = l0; bl1 = l1; }
  }
  *out_bin = best_b;
  *out_l0 = bl0;
  *out_l1 = bl1;
  return best;
}

// Device-resident level loop of a tree (models/grower.py grow_tree_device): after the split
// search of level d, ONE thread applies the best splits of the level's open nodes to the node
// table, writes this level's partition tables and plans level d + 1 (open list, smaller-sibling
// builds, subtraction triples), exactly as the host loop (grower.TreeTable.apply_splits and the
// build selection of grow_tree) does -- same node numbering, same tie rules -- so the host only
// reads two counts per level and the node table once per tree. Newton gain (GBDT) and Spark's
// gini / entropy (DT / RF, optionally building every open node for per-node feature sampling).
struct LevelPlanArgs {
  const int64_t* packed;          // [n_shards][L][5] best split per open node {gain bits, feature, bin, left0, left1}
  int32_t L;                      // open-list capacity of this level
  int32_t n_shards;               // data parallel: the all-gathered per-shard bests (<= 1: one table);
  int64_t shard_stride;           //   the best over shards per node, ties to the lowest shard
  int32_t depth, max_depth;
  int32_t mode;                   // 0 newton (gain > max(min_gain, 1e-6)), 1 gini / 2 entropy (gain > 0, >= min_gain)
  int32_t build_all;              // build every open node (RF: no sibling subtraction)
  const int32_t* kexp;            // [2] quantisation exponents (classification purity test)
  double min_gain;
  const int32_t* zbin;            // [Fa] zero bin of each feature (missing entries)
  const int32_t* hot_row;         // [Fa] row of the feature in the dense block (-1), nullptr: none
  int32_t max_nodes;
  // node table (in/out)
  int32_t* n_nodes;               // [1]
  int64_t* stats;                 // [max_nodes][2] exact integer sums
  int32_t* parent;
  int32_t* left;
  int32_t* right;
  int32_t* feat;                  // Fa index of the split feature (-1 leaf / not split)
  int32_t* bin;
  uint8_t* leaf;
  double* gain;
  // this level (in): open nodes, local index i = row i of the level's histogram
  const int32_t* open;            // [L] (-1 pad)
  const int32_t* n_open;          // [1]
  // this level's partition (out)
  int32_t* default_child;         // [max_nodes]
  int32_t* node_dense;            // [max_nodes][4] or nullptr
  int32_t* cs_feat;               // [L] column-pass splits
  int32_t* cs_default;
  int32_t* cs_other;
  int32_t* cs_bin;
  int32_t* cs_left_default;
  int32_t* counts;                // [4] out: n_cs, n_next_open, n_build, n_nodes
  int32_t* counts_host;           // optional host-mapped copy of the 4 counts (pinned; no D2H copy)
  int32_t counts_tail;            // counts[4 .. 4 + counts_tail) zeroed (the next level's select counts)
  const int64_t* root_parts;      // optional (depth 0): the root's totals as QuantArgs root_parts
                                  //   slots, summed here into stats[0]
  const int64_t* root_tot;        // optional (depth 0, data parallel): the root's reduced sums [2]
  // optional (data-parallel levels, device plan only): level d + 1's histogram rows as
  // level_rows_kernel writes them (LevelRowsArgs with bld_base 0, sub_base = level d + 1's builds,
  // prev_row_of = lr_prev: this level's rows, nullptr at depth 0), so they need no launch
  const int32_t* lr_prev;
  int32_t* lr_row_of;
  int32_t* lr_dst;
  int32_t* lr_par;
  int32_t* lr_sib;
  // level d + 1 (out; capacity 2L open, L built)
  int32_t* next_open;             // [2L] (-1 pad)
  int64_t* next_totals;           // [2L][2]
  int32_t* node_slot;             // [max_nodes] pass slot of the built nodes (-1)
  int32_t* s2n;                   // [L] histogram row of slot s (-1)
  int32_t* sub_dst;               // [L] subtraction: larger sibling (row in level d + 1) =
  int32_t* sub_par;               //     parent (row in level d) - smaller sibling (row in level d + 1)
  int32_t* sub_sib;
  int32_t* sub_of;                // optional [2L]: per level d + 1 open index, its subtraction slot (-1)
};

// The plan's table resets, split over nthreads workers (the device runs them on 64 lanes before
// the single-thread plan; the host on one).
FDX_HD void level_plan_reset(const LevelPlanArgs& a, int32_t t, int32_t nthreads) {
  for (int32_t n = t; n < a.max_nodes; n += nthreads) {
    a.default_child[n] = -1;
    a.node_slot[n] = -1;
    if (a.node_dense) for (int k = 0; k < 4; ++k) a.node_dense[4 * n + k] = -1;
  }
  for (int32_t i = t; i < 2 * a.L; i += nthreads) {
    a.next_open[i] = -1;
    if (a.sub_of) a.sub_of[i] = -1;
    a.next_totals[2 * i] = a.next_totals[2 * i + 1] = 0;
  }
  for (int32_t i = t; i < a.L; i += nthreads) a.s2n[i] = a.sub_dst[i] = a.sub_par[i] = a.sub_sib[i] = -1;
}

FDX_HD void level_plan(const LevelPlanArgs& a, bool reset = true) {
  if (reset) level_plan_reset(a, 0, 1);
  if (a.root_parts) root_sums(a.root_parts, &a.stats[0], &a.stats[1]);
  const double thr = a.min_gain > 1e-6 ? a.min_gain : 1e-6;
  const double s0 = ldexp(1.0, -a.kexp[0]), s1 = ldexp(1.0, -a.kexp[1]);
  int32_t nn = *a.n_nodes, n_cs = 0, n_next = 0;
  const int32_t no = *a.n_open;
  for (int32_t i = 0; i < no; ++i) {
    const int32_t n = a.open[i];
    const int64_t* p = a.packed + 5 * (int64_t)i;
    double g;
    memcpy(&g, &p[0], sizeof(double));
    for (int32_t sh = 1; sh < a.n_shards; ++sh) {     // shard order = feature order: ties keep the lowest
      const int64_t* q = a.packed + sh * a.shard_stride + 5 * (int64_t)i;
      double gq;
      memcpy(&gq, &q[0], sizeof(double));
      if (gq > g) { g = gq; p = q; }
    }
    const int32_t f = (int32_t)p[1], b = (int32_t)p[2];
    const bool ok = a.mode == 0 ? (b >= 0 && isfinite(g) && g > thr)
                                : (b >= 0 && isfinite(g) && g > 0.0 && g >= a.min_gain);
    if (!ok || nn + 2 > a.max_nodes) {
      a.leaf[n] = 1;
      continue;
    }
    const int32_t li = nn, ri = nn + 1;
    nn += 2;
    const int64_t l0 = p[3], l1 = p[4];
    a.stats[2 * li] = l0;
    a.stats[2 * li + 1] = l1;
    a.stats[2 * ri] = a.stats[2 * n] - l0;
    a.stats[2 * ri + 1] = a.stats[2 * n + 1] - l1;
    for (int32_t c = li; c <= ri; ++c) {
      bool leafy = a.depth + 1 >= a.max_depth;
      if (a.mode != 0)   // pure node (grower._impurity == 0)
        leafy = leafy || impurity(a.mode, (double)a.stats[2 * c] * s0, (double)a.stats[2 * c + 1] * s1) == 0.0;
      a.parent[c] = n;
      a.left[c] = a.right[c] = -1;
      a.feat[c] = -1;
      a.bin[c] = -1;
      a.gain[c] = -1.0;
      a.leaf[c] = leafy ? 1 : 0;
    }
    a.feat[n] = f;
    a.bin[n] = b;
    a.left[n] = li;
    a.right[n] = ri;
    a.gain[n] = g;
    const bool left_default = a.zbin[f] <= b;
    const int32_t dflt = left_default ? li : ri, other = left_default ? ri : li;
    a.default_child[n] = dflt;
    const int32_t hr = a.hot_row ? a.hot_row[f] : -1;
    if (a.node_dense && hr >= 0) {
      int32_t* nd = a.node_dense + 4 * (int64_t)n;
      nd[0] = hr; nd[1] = b; nd[2] = li; nd[3] = ri;
    } else {
      a.cs_feat[n_cs] = f;
      a.cs_default[n_cs] = dflt;
      a.cs_other[n_cs] = other;
      a.cs_bin[n_cs] = b;
      a.cs_left_default[n_cs] = left_default ? 1 : 0;
      ++n_cs;
    }
    for (int32_t c = li; c <= ri; ++c)
      if (!a.leaf[c]) {
        a.next_open[n_next] = c;
        a.next_totals[2 * n_next] = a.stats[2 * c];
        a.next_totals[2 * n_next + 1] = a.stats[2 * c + 1];
        ++n_next;
      }
  }
  // builds of level d + 1: per parent (in order of first appearance), the smaller open child
  // (hessian sum / instance count, ties to the left child), the larger one by subtraction; or
  // every open node (build_all)
  int32_t nb = 0;
  if (a.build_all) {
    for (int32_t j = 0; j < n_next; ++j) {
      a.node_slot[a.next_open[j]] = j;
      a.s2n[j] = j;
    }
    nb = n_next;
  }
  for (int32_t j = 0; j < n_next && !a.build_all; ++j) {
    const int32_t c = a.next_open[j], pnode = a.parent[c];
    if (j > 0 && a.parent[a.next_open[j - 1]] == pnode) continue;      // siblings are adjacent
    const int32_t lc = a.left[pnode], rc = a.right[pnode];
    const bool lo = !a.leaf[lc], ro = !a.leaf[rc];
    int32_t build, large = -1;
    if (lo && ro) {
      const int64_t wl = a.mode == 0 ? a.stats[2 * lc + 1] : a.stats[2 * lc] + a.stats[2 * lc + 1];
      const int64_t wr = a.mode == 0 ? a.stats[2 * rc + 1] : a.stats[2 * rc] + a.stats[2 * rc + 1];
      const bool lsmall = wl <= wr;
      build = lsmall ? lc : rc;
      large = lsmall ? rc : lc;
    } else {
      build = lo ? lc : rc;
    }
    int32_t jb = -1, jl = -1, ip = -1;
    for (int32_t k = 0; k < n_next; ++k) {
      if (a.next_open[k] == build) jb = k;
      if (a.next_open[k] == large) jl = k;
    }
    for (int32_t k = 0; k < no; ++k)
      if (a.open[k] == pnode) ip = k;
    a.node_slot[build] = nb;
    a.s2n[nb] = jb;
    if (large >= 0) {
      a.sub_dst[nb] = jl;
      if (a.sub_of) a.sub_of[jl] = nb;
      a.sub_par[nb] = ip;
      a.sub_sib[nb] = jb;
    }
    ++nb;
  }
  *a.n_nodes = nn;
  a.counts[0] = n_cs;
  a.counts[1] = n_next;
  a.counts[2] = nb;
  a.counts[3] = nn;
  if (a.counts_host)
    for (int k = 0; k < 4; ++k) a.counts_host[k] = a.counts[k];
}

// ------------------------------------------------------------------ lane-batched launches
// A forest's trees in flight grow in lockstep batches (bindings_level.cpp RfBatch): every stage
// of a level is ONE launch for all the batch's trees, tree (lane) l's arguments at args[l] in
// device memory (blockIdx.z = l), the grid the largest lane's; each kernel returns early from the
// blocks beyond its own lane's grid. The per-lane arguments are exactly those of the per-tree
// launches, so the trees are bitwise the same (tests/test_level_runner.py).
struct BestPartials {              // (split_best_node: the narrow search's per-wave partials)
  const double* part_gain;
  const int32_t* part_f;
  const int32_t* wide;
  int32_t n_wide;
};
struct QuantLane {
  QuantArgs a;
  const double* maxv;
  unsigned long long* part;
};
struct SplitBestLane {
  const double* gain;
  const int32_t* bin;
  const int64_t* left;
  int32_t nodes;
  int32_t Fa;
  int64_t f0;
  int64_t* out;
  BestPartials bp;
};
struct SplitBestPlanLane {
  SplitBestLane b;
  LevelPlanArgs p;
  unsigned int* ticket;
};
// (data-parallel batches) the lane's root sums (its quantisation's kRootSlots slots) into words
// tot_word, tot_word + 1 of every shard chunk of the batch's send buffer
struct RootSendLane {
  const int64_t* root_parts;
  int64_t* send;
  int32_t S;
  int64_t chunk_words;
  int64_t tot_word;
};
// a small copy per lane (node-table images, a level's count rows into host-mapped pinned rows)
struct CopyLane {
  void* dst;
  const void* src;
  int64_t bytes;
};
struct PartColsLane {
  PartitionArgs a;
  const int64_t* colptr;
  const int32_t* cs_feat;
  const int32_t* n_cs;
  int32_t max_splits;
  int32_t wps;
};

}  // namespace fdx

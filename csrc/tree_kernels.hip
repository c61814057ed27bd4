// Histogram tree engine for gfx950 (K-10..K-15 of SURVEY.md §2.5).
//
// Histogram build on the matrix cores: for one feature column chunk, the per-(bin, node, stat)
// sums are the product  C[bin][col] = sum_k A[bin][k] * B[k][col]  over the chunk's entries k,
// with A = one-hot(bin_k) (exact in bf16) and B[k][col] = (slot_k == node(col)) * stat(col)_k,
// stat split into bf16 hi/lo halves so the fp32-accumulating v_mfma_f32_32x32x16_bf16 yields
// ~fp32-accurate sums (class counts are small integers and exact). One wave per work item,
// 16 entries per MFMA K-step, no atomics, fixed summation order -> deterministic histograms.
// The rest of the level (reduce of chunk partials, sibling subtraction, split search, row
// partition) are small bandwidth-bound kernels.
#include "ops.h"
#include "tree.h"

#pragma clang fp contract(off)

namespace fdx {

namespace {
constexpr int kWave = 64;

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// 0x01 in every byte of x that is zero, 0x00 elsewhere (SWAR, no carries across bytes).
__device__ __forceinline__ uint32_t match_bytes(uint32_t x) {
  const uint32_t y = (x & 0x7f7f7f7fu) + 0x7f7f7f7fu;
  return ~(y | x | 0x7f7f7f7fu) >> 7;
}
// bytes b0,b1 (lo) / b2,b3 (hi) of z -> b | b' << 16: one flag per 16-bit MFMA operand element,
// then a 24-bit multiply turns each flag into the element value (0x3f80 = bf16 1.0, 0xffff mask).
__device__ __forceinline__ uint32_t spread_lo(uint32_t z) { return __builtin_amdgcn_perm(z, z, 0x0c010c00u); }
__device__ __forceinline__ uint32_t spread_hi(uint32_t z) { return __builtin_amdgcn_perm(z, z, 0x0c030c02u); }

__device__ __forceinline__ void lds_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

// ------------------------------------------------------------------ per-tree / per-pass row state
__global__ __launch_bounds__(256) void rowstats_kernel(RowStatsArgs a) {
  for (int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x; r < a.N; r += (int64_t)gridDim.x * 256) {
    uint2 st;
    if (a.mode == 0) {
      const float w = a.weight ? a.weight[r] : 1.0f;
      st.x = split_bf16(a.g[r] * w);
      st.y = split_bf16(a.h[r] * w);
    } else {
      float w = a.weight ? a.weight[r] : 1.0f;
      if (a.bootstrap) w *= (float)poisson1(hash_uniform(a.seed, (uint64_t)a.tree, (uint64_t)r));
      const float y = a.label[r];
      st.x = split_bf16(w * (1.0f - y));
      st.y = split_bf16(w * y);
    }
    reinterpret_cast<uint2*>(a.rowstats)[r] = st;
  }
}

// est[e] = rowstats[csc_row[e]]: the one random gather of the tree (4 entries per thread).
__global__ __launch_bounds__(256) void entry_stats_kernel(const int32_t* __restrict__ csc_row,
                                                          const uint2* __restrict__ rowstats, int64_t nnz,
                                                          uint2* __restrict__ est) {
  const int64_t n4 = nnz / 4;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    const int4 r = reinterpret_cast<const int4*>(csc_row)[i];
    const uint2 a = rowstats[r.x], b = rowstats[r.y], c = rowstats[r.z], d = rowstats[r.w];
    reinterpret_cast<uint4*>(est)[2 * i] = make_uint4(a.x, a.y, b.x, b.y);
    reinterpret_cast<uint4*>(est)[2 * i + 1] = make_uint4(c.x, c.y, d.x, d.y);
  }
  const int64_t t = 4 * n4 + (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t < nnz) est[t] = rowstats[csc_row[t]];
}

// Item-ordered variant (same wave -> item table as the histogram launches): each XCD gathers from
// the ~1 MB row-statistics slice of the row block it is working on, which stays in its L2.
__global__ __launch_bounds__(256) void entry_stats_items_kernel(const int64_t* __restrict__ item_start,
                                                                const int64_t* __restrict__ item_end,
                                                                const int32_t* __restrict__ wave_item, int32_t num_items,
                                                                const int32_t* __restrict__ csc_row,
                                                                const uint2* __restrict__ rowstats,
                                                                uint2* __restrict__ est) {
  const int wslot = blockIdx.x * 4 + threadIdx.x / kWave;
  const int lane = threadIdx.x & (kWave - 1);
  const int item = wave_item[wslot];
  if (item < 0 || item >= num_items) return;
  const int64_t e0 = item_start[item], e1 = item_end[item];
  const int64_t e_last = (e1 - 1) & ~(int64_t)3;   // csc_row is padded, so a clamped 4-group is readable
  // 4 consecutive entries per lane and U steps per round: U 16-B row loads, then 4U independent
  // gathers in flight, then the 16-B stores (masked at the item's ends).
  constexpr int U = 4;
  for (int64_t base = e0 & ~(int64_t)3; base < e1; base += U * 4 * kWave) {
    int4 r[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t e = base + (int64_t)u * 4 * kWave + 4 * lane;
      r[u] = *reinterpret_cast<const int4*>(csc_row + (e < e_last ? e : e_last));
    }
    uint2 g[U][4];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      g[u][0] = rowstats[r[u].x]; g[u][1] = rowstats[r[u].y];
      g[u][2] = rowstats[r[u].z]; g[u][3] = rowstats[r[u].w];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t e = base + (int64_t)u * 4 * kWave + 4 * lane;
      if (e >= e0 && e + 4 <= e1) {
        reinterpret_cast<uint4*>(est)[e / 2] = make_uint4(g[u][0].x, g[u][0].y, g[u][1].x, g[u][1].y);
        reinterpret_cast<uint4*>(est)[e / 2 + 1] = make_uint4(g[u][2].x, g[u][2].y, g[u][3].x, g[u][3].y);
      } else if (e < e1 && e + 4 > e0) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (e + j >= e0 && e + j < e1) est[e + j] = g[u][j];
      }
    }
  }
}

__global__ __launch_bounds__(256) void slot8_kernel(SlotArgs a) {
  for (int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x; r < a.N; r += (int64_t)gridDim.x * 256) {
    const int32_t node = a.row_node[r];
    const int32_t s = ((node >= 0 && node < a.num_nodes) ? a.node_slot[node] : -1) - a.slot_base;
    a.slot8[r] = (s >= 0 && s < a.nslots) ? (uint8_t)s : (uint8_t)0xff;
  }
}

// One lane's 4 consecutive entries of a histogram step: rows (root: 0 = valid, -1 = outside the
// item), bins (0xff outside) and the packed statistics (0 outside). Branch-free, so the compiler
// can keep the next step's loads in flight across the current step: lanes past the item's end
// re-read its last 4-group (clamped address), and the CSC arrays carry >= 4 readable entries of
// padding, so a 4-group never leaves the allocation.
struct StepData {
  int4 r4;
  uint32_t bins4;
  uint4 p, q;
};

template <bool ROOT>
__device__ __forceinline__ void load_step(const HistArgs& a, int64_t e, int64_t e0, int64_t e1, int64_t e_last,
                                          StepData& d) {
  const int64_t el = e < e_last ? e : e_last;
  const uint32_t bins = *reinterpret_cast<const uint32_t*>(a.csc_bin + el);
  int4 r = make_int4(0, 0, 0, 0);
  if constexpr (!ROOT) r = *reinterpret_cast<const int4*>(a.csc_row + el);
  uint4 p = reinterpret_cast<const uint4*>(a.est)[el / 2];
  uint4 q = reinterpret_cast<const uint4*>(a.est)[el / 2 + 1];
  const bool v0 = e >= e0 && e < e1, v1 = e + 1 >= e0 && e + 1 < e1;
  const bool v2 = e + 2 >= e0 && e + 2 < e1, v3 = e + 3 >= e0 && e + 3 < e1;
  const uint32_t keep = (v0 ? 0xffu : 0u) | (v1 ? 0xff00u : 0u) | (v2 ? 0xff0000u : 0u) | (v3 ? 0xff000000u : 0u);
  d.bins4 = (bins & keep) | ~keep;
  d.r4 = make_int4(v0 ? r.x : -1, v1 ? r.y : -1, v2 ? r.z : -1, v3 ? r.w : -1);
  d.p = make_uint4(v0 ? p.x : 0u, v0 ? p.y : 0u, v1 ? p.z : 0u, v1 ? p.w : 0u);
  d.q = make_uint4(v2 ? q.x : 0u, v2 ? q.y : 0u, v3 ? q.z : 0u, v3 ? q.w : 0u);
}

// Gather mode: only rows and bins stream (5 B per entry); the 1-byte slot and, for live entries
// only, the 8-byte row statistics are gathered from the current row block's slice (~1.1 MB,
// resident in the XCD's L2 under the XCD-ordered item placement). No per-tree entry-order copy
// of the statistics is made, and entries outside the nodes being built cost no statistics bytes.
struct RowStep {
  int4 r4;
  uint32_t bins4;
};

__device__ __forceinline__ void load_rows(const HistArgs& a, int64_t e, int64_t e0, int64_t e1, int64_t e_last,
                                          RowStep& d) {
  const int64_t el = e < e_last ? e : e_last;
  const uint32_t bins = *reinterpret_cast<const uint32_t*>(a.csc_bin + el);
  const int4 r = *reinterpret_cast<const int4*>(a.csc_row + el);
  const bool v0 = e >= e0 && e < e1, v1 = e + 1 >= e0 && e + 1 < e1;
  const bool v2 = e + 2 >= e0 && e + 2 < e1, v3 = e + 3 >= e0 && e + 3 < e1;
  const uint32_t keep = (v0 ? 0xffu : 0u) | (v1 ? 0xff00u : 0u) | (v2 ? 0xff0000u : 0u) | (v3 ? 0xff000000u : 0u);
  d.bins4 = (bins & keep) | ~keep;
  d.r4 = make_int4(v0 ? r.x : -1, v1 ? r.y : -1, v2 ? r.z : -1, v3 ? r.w : -1);
}

// slot byte of each of the 4 entries (0xff: outside the item or not in a node of this pass)
template <bool ROOT>
__device__ __forceinline__ uint32_t entry_slots(const HistArgs& a, int4 r4) {
  if constexpr (ROOT) {
    return (r4.x >= 0 ? 0u : 0xffu) | (r4.y >= 0 ? 0u : 0xff00u) | (r4.z >= 0 ? 0u : 0xff0000u) |
           (r4.w >= 0 ? 0u : 0xff000000u);
  } else {
    const uint32_t s0 = a.slot8[r4.x >= 0 ? r4.x : 0];
    const uint32_t s1 = a.slot8[r4.y >= 0 ? r4.y : 0];
    const uint32_t s2 = a.slot8[r4.z >= 0 ? r4.z : 0];
    const uint32_t s3 = a.slot8[r4.w >= 0 ? r4.w : 0];
    return (r4.x >= 0 ? s0 : 0xffu) | ((r4.y >= 0 ? s1 : 0xffu) << 8) | ((r4.z >= 0 ? s2 : 0xffu) << 16) |
           ((r4.w >= 0 ? s3 : 0xffu) << 24);
  }
}

// packed statistics of the live entries among the 4 (0 for dead ones: they are never staged)
__device__ __forceinline__ void gather_stats(const uint2* __restrict__ rs, int4 r4, uint32_t slots4, uint32_t w[8]) {
  const int32_t rr[4] = {r4.x, r4.y, r4.z, r4.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    uint2 v = make_uint2(0u, 0u);
    if (((slots4 >> (8 * j)) & 0xffu) != 0xffu) v = rs[rr[j]];
    w[2 * j] = v.x;
    w[2 * j + 1] = v.y;
  }
}

// ------------------------------------------------------------------ MFMA histogram
// One wave per work item (a chunk of one feature column); per step the wave takes 256 entries,
// 4 consecutive ones per lane so that rows (int4), bins (u32) and statistics (2 x uint4) are
// single vector loads; the next step's loads are in flight while this one is multiplied.
// ROOT: the pass builds only the root, so every entry is live in slot 0 and neither rows nor
// the slot table are read. Otherwise only live entries (row in a node of this pass) are
// compacted into LDS and MFMA K-steps run on ceil(live / KS) groups.
// Tiles: NARROW (features with <= 16 bins, ~90 % of entries on text data) uses
// v_mfma_f32_16x16x32_bf16: 16 bins x (4 slots x 4 stat halves), 32 entries per K-step; otherwise
// v_mfma_f32_32x32x16_bf16: 32 bins x (8 slots x 4 stat halves), 16 entries per K-step. Operand
// construction is VALU-issue bound, so the narrow tile halves the one-hot work per entry.
// GATHER selects where the statistics come from:
//   false  per-tree entry-order copy streamed with the rows and bins (load_step);
//   true   row gathers (see load_rows): rows/bins of step i+3, slots of step i+2 and statistics
//          of step i+1 are in flight while step i is staged and multiplied. (Measured at 10M
//          rows / 1B entries: 34 ms per depth-6 round against 38.5 ms streaming, which also
//          pays a per-tree entry-statistics pass; a 16-byte (slot, statistics) record per row
//          and level, gathered once per entry, was slower still at 45 ms: the gathers are bound
//          by L2 lines moved, not by instructions.)
template <int BT, int CT, bool ROOT, bool NARROW, bool GATHER>
__global__ __launch_bounds__(256) void hist_mfma_kernel(HistArgs a) {
  constexpr int G = 4 * kWave;                 // entries per wave step
  constexpr int KS = NARROW ? 32 : 16;         // entries per MFMA K-step
  constexpr int NSLOT = NARROW ? 4 : 8;        // node slots per column tile
  constexpr int NBIN = NARROW ? 16 : 32;       // bins per row tile
  constexpr int NREG = NARROW ? 4 : 16;        // accumulator registers per lane
  typedef float acc_t __attribute__((ext_vector_type(NREG)));
  __shared__ __attribute__((aligned(16))) uint8_t s_bin[4][G + KS];
  __shared__ __attribute__((aligned(16))) uint8_t s_slot[4][G + KS];
  __shared__ __attribute__((aligned(16))) uint16_t s_comp[4][4][G + KS];

  const int wid = threadIdx.x / kWave;
  const int lane = threadIdx.x & (kWave - 1);
  const int wslot = blockIdx.x * 4 + wid;
  const int item = a.wave_item ? a.wave_item[wslot] : wslot;
  if (item < 0 || item >= a.num_items) return;
  const int64_t e0 = a.item_start[item], e1 = a.item_end[item];

  const int col = NARROW ? (lane & 15) : (lane & 31);   // MFMA column / A-row index owned by this lane
  const int kgrp = NARROW ? (lane >> 4) : (lane >> 5);  // which 8 entries of a K-step the lane supplies
  const int comp = col & 3;                             // 0 stat0_hi, 1 stat0_lo, 2 stat1_hi, 3 stat1_lo
  const int slot_sub = col >> 2;

  acc_t acc[BT][CT];
#pragma unroll
  for (int bt = 0; bt < BT; ++bt)
#pragma unroll
    for (int ct = 0; ct < CT; ++ct)
#pragma unroll
      for (int i = 0; i < NREG; ++i) acc[bt][ct][i] = 0.0f;

  const int64_t first = e0 & ~(int64_t)3;
  const int64_t e_last = (e1 - 1) & ~(int64_t)3;   // last 4-group holding an entry of the item
  StepData cur, nxt;
  // gather-mode pipeline state: statistics/slots/bins of step i, slots of step i+1, rows of i+1, i+2
  const uint2* rs = reinterpret_cast<const uint2*>(a.rowstats);
  RowStep g1, g2;
  uint32_t g_sl0 = 0, g_sl1 = 0, g_bins0 = 0, g_w[8];
  if constexpr (GATHER) {
    RowStep g0;
    load_rows(a, first + 4 * lane, e0, e1, e_last, g0);
    load_rows(a, first + G + 4 * lane, e0, e1, e_last, g1);
    g_sl0 = entry_slots<ROOT>(a, g0.r4);
    g_bins0 = g0.bins4;
    g_sl1 = entry_slots<ROOT>(a, g1.r4);
    gather_stats(rs, g0.r4, g_sl0, g_w);
    load_rows(a, first + 2 * G + 4 * lane, e0, e1, e_last, g2);
  } else {
    load_step<ROOT>(a, first + 4 * lane, e0, e1, e_last, cur);
  }
  for (int64_t base = first; base < e1; base += G) {
    uint32_t slots4, bins4, w[8];
    if constexpr (GATHER) {
      slots4 = g_sl0;
      bins4 = g_bins0;
#pragma unroll
      for (int j = 0; j < 8; ++j) w[j] = g_w[j];
      // statistics of step i+1, slots of step i+2, rows of step i+3 (clamped, so unconditional)
      gather_stats(rs, g1.r4, g_sl1, g_w);
      const uint32_t sl2 = entry_slots<ROOT>(a, g2.r4);
      RowStep g3;
      load_rows(a, base + 3 * G + 4 * lane, e0, e1, e_last, g3);
      g_sl0 = g_sl1;
      g_bins0 = g1.bins4;
      g_sl1 = sl2;
      g1 = g2;
      g2 = g3;
    } else {
      // slot of each of the lane's 4 entries (the only random access: a 1-byte table, L2-resident)
      slots4 = entry_slots<ROOT>(a, cur.r4);
      // prefetch the next step (clamped, so unconditional) while this one is staged and multiplied
      load_step<ROOT>(a, base + G + 4 * lane, e0, e1, e_last, nxt);
      bins4 = cur.bins4;
      w[0] = cur.p.x; w[1] = cur.p.y; w[2] = cur.p.z; w[3] = cur.p.w;
      w[4] = cur.q.x; w[5] = cur.q.y; w[6] = cur.q.z; w[7] = cur.q.w;
    }
    const bool any = slots4 != 0xffffffffu;
    unsigned long long live = 0;
    int n_live = G;
    if constexpr (ROOT) {
      live = __ballot(any);
      *reinterpret_cast<uint32_t*>(&s_bin[wid][4 * lane]) = bins4;
      *reinterpret_cast<uint32_t*>(&s_slot[wid][4 * lane]) = slots4;
      // comp c of entry j = 16-bit half (c & 1) of word (c >> 1) of entry j
      *reinterpret_cast<uint2*>(&s_comp[wid][0][4 * lane]) =
          make_uint2((w[0] & 0xffffu) | (w[2] << 16), (w[4] & 0xffffu) | (w[6] << 16));
      *reinterpret_cast<uint2*>(&s_comp[wid][1][4 * lane]) =
          make_uint2((w[0] >> 16) | (w[2] & 0xffff0000u), (w[4] >> 16) | (w[6] & 0xffff0000u));
      *reinterpret_cast<uint2*>(&s_comp[wid][2][4 * lane]) =
          make_uint2((w[1] & 0xffffu) | (w[3] << 16), (w[5] & 0xffffu) | (w[7] << 16));
      *reinterpret_cast<uint2*>(&s_comp[wid][3][4 * lane]) =
          make_uint2((w[1] >> 16) | (w[3] & 0xffff0000u), (w[5] >> 16) | (w[7] & 0xffff0000u));
    } else {
      int nb = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t sj = (slots4 >> (8 * j)) & 0xffu;
        const unsigned long long bj = __ballot(sj != 0xffu);
        if (sj != 0xffu) {
          const int p = nb + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bj >> 32),
                                                            __builtin_amdgcn_mbcnt_lo((uint32_t)bj, 0u));
          s_bin[wid][p] = (uint8_t)(bins4 >> (8 * j));
          s_slot[wid][p] = (uint8_t)sj;
          s_comp[wid][0][p] = (uint16_t)w[2 * j];
          s_comp[wid][1][p] = (uint16_t)(w[2 * j] >> 16);
          s_comp[wid][2][p] = (uint16_t)w[2 * j + 1];
          s_comp[wid][3][p] = (uint16_t)(w[2 * j + 1] >> 16);
        }
        nb += __popcll(bj);
      }
      n_live = nb;
      // pad the last partial K-step: bin/slot 0xff match no row/column, so stale comps drop out
      if (lane < KS) {
        s_bin[wid][nb + lane] = 0xffu;
        s_slot[wid][nb + lane] = 0xffu;
      }
    }
    lds_sync();
#pragma unroll
    for (int ks = 0; ks < G / KS; ++ks) {
      if constexpr (ROOT) {
        constexpr unsigned long long kLaneMask = (1ull << (KS / 4)) - 1ull;   // lanes holding the K-step
        if (((live >> (ks * (KS / 4))) & kLaneMask) == 0ull) continue;
      } else {
        if (ks * KS >= n_live) break;
      }
      const int k0 = ks * KS + 8 * kgrp;
      const uint2 bins8 = *reinterpret_cast<const uint2*>(&s_bin[wid][k0]);
      const uint2 slots8 = *reinterpret_cast<const uint2*>(&s_slot[wid][k0]);
      const uint4 cv = *reinterpret_cast<const uint4*>(&s_comp[wid][comp][k0]);
      bf16x8 A[BT];
#pragma unroll
      for (int bt = 0; bt < BT; ++bt) {
        const uint32_t rep = (uint32_t)(col + NBIN * bt) * 0x01010101u;
        const uint32_t zl = match_bytes(bins8.x ^ rep), zh = match_bytes(bins8.y ^ rep);
        const u32x4 av = {spread_lo(zl) * 0x3f80u, spread_hi(zl) * 0x3f80u,    // bf16 1.0 where bin == row
                          spread_lo(zh) * 0x3f80u, spread_hi(zh) * 0x3f80u};
        A[bt] = __builtin_bit_cast(bf16x8, av);
      }
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) {
        bf16x8 B;
        if constexpr (ROOT) {
          // one node: no slot mask; columns of the other slots collect junk the reduce never reads
          B = __builtin_bit_cast(bf16x8, cv);
        } else {
          const uint32_t rep = (uint32_t)(ct * NSLOT + slot_sub) * 0x01010101u;
          const uint32_t zl = match_bytes(slots8.x ^ rep), zh = match_bytes(slots8.y ^ rep);
          const u32x4 bv = {cv.x & (spread_lo(zl) * 0xffffu), cv.y & (spread_hi(zl) * 0xffffu),
                            cv.z & (spread_lo(zh) * 0xffffu), cv.w & (spread_hi(zh) * 0xffffu)};
          B = __builtin_bit_cast(bf16x8, bv);
        }
#pragma unroll
        for (int bt = 0; bt < BT; ++bt) {
          if constexpr (NARROW)
            acc[bt][ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[bt], B, acc[bt][ct], 0, 0, 0);
          else
            acc[bt][ct] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[bt], B, acc[bt][ct], 0, 0, 0);
        }
      }
    }
    lds_sync();
    if constexpr (!GATHER) cur = nxt;
  }

  // C[row][col]: 32x32 tile row = (reg&3) + 8*(reg>>2) + 4*kgrp, 16x16 tile row = 4*kgrp + reg;
  // col = lane's column. Combine hi+lo halves (adjacent columns), store [item][slot][bin][stat].
  float* out = a.slab + (int64_t)item * (NSLOT * CT) * (NBIN * BT) * 2;
#pragma unroll
  for (int bt = 0; bt < BT; ++bt)
#pragma unroll
    for (int ct = 0; ct < CT; ++ct)
#pragma unroll
      for (int reg = 0; reg < NREG; ++reg) {
        const float v = acc[bt][ct][reg];
        const float w2 = __shfl_xor(v, 1, kWave);
        if ((col & 1) == 0) {
          const int row = (NARROW ? 4 * kgrp + reg : (reg & 3) + 8 * (reg >> 2) + 4 * kgrp) + NBIN * bt;
          const int slot = ct * NSLOT + slot_sub;
          const int stat = (col >> 1) & 1;
          out[((int64_t)slot * (NBIN * BT) + row) * 2 + stat] = v + w2;
        }
      }
}

// ------------------------------------------------------------------ reduce chunk partials
__global__ __launch_bounds__(256) void hist_reduce_kernel(HistReduceArgs a) {
  const int64_t tid = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t per_feat = (int64_t)a.slab_slots * a.slab_bins;
  if (tid >= (int64_t)a.L * per_feat) return;
  const int li = (int)(tid / per_feat);
  const int rem = (int)(tid % per_feat);
  const int s = rem / a.slab_bins, b = rem % a.slab_bins;
  const int fid = a.feat[li];
  if (b >= a.nbins[fid]) return;
  const int node = a.slot_to_node[s];
  if (node < 0) return;
  double g = 0.0, h = 0.0;
  const int64_t i0 = a.feat_item0[li];
  for (int i = 0; i < a.feat_nitems[li]; ++i) {
    const float* p = a.slab + ((i0 + i) * per_feat + (int64_t)s * a.slab_bins + b) * 2;
    g += (double)p[0];
    h += (double)p[1];
  }
  double* dst = a.hist + ((int64_t)node * a.total_bins + a.boff[fid] + b) * 2;
  dst[0] = g;
  dst[1] = h;
}

// ------------------------------------------------------------------ sibling subtraction
__global__ __launch_bounds__(256) void hist_subtract_kernel(const double* parent_hist, double* cur_hist,
                                                            const int32_t* dst, const int32_t* par,
                                                            const int32_t* sib, int32_t n_pairs, int64_t TB) {
  const int64_t per = TB * 2;
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < (int64_t)n_pairs * per;
       t += (int64_t)gridDim.x * 256) {
    const int p = (int)(t / per);
    const int64_t k = t % per;
    cur_hist[(int64_t)dst[p] * per + k] = parent_hist[(int64_t)par[p] * per + k] - cur_hist[(int64_t)sib[p] * per + k];
  }
}

// ------------------------------------------------------------------ split search
__global__ __launch_bounds__(256) void split_kernel(SplitArgs a) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= (int64_t)a.num_nodes * a.Fa) return;
  const int n = (int)(t / a.Fa), f = (int)(t % a.Fa);
  double gain = -1.0 / 0.0;
  int bin = -1;
  double l0 = 0, l1 = 0;
  bool use = true;
  if (a.feat_prob < 1.0)
    use = hash_uniform(a.seed ^ 0x5bd1e995ull, ((uint64_t)a.tree << 32) | (uint32_t)a.node_ids[n],
                       (uint64_t)a.fid_orig[f]) < a.feat_prob;
  if (use) {
    const double* hb = a.hist + ((int64_t)n * (a.boff[a.Fa]) + a.boff[f]) * 2;
    gain = best_split_scan(hb, a.nbins[f], a.zbin[f], a.totals[2 * n], a.totals[2 * n + 1], a.mode, a.lambda_,
                           a.min_child_weight, &bin, &l0, &l1);
  }
  a.out_gain[t] = gain;
  a.out_bin[t] = bin;
  a.out_left[2 * t] = l0;
  a.out_left[2 * t + 1] = l1;
}

// ------------------------------------------------------------------ partition
__global__ __launch_bounds__(256) void partition_default_kernel(PartitionArgs a) {
  for (int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x; r < a.N; r += (int64_t)gridDim.x * 256) {
    const int32_t n = a.row_node[r];
    if (n >= 0 && n < a.num_nodes) {
      const int32_t c = a.default_child[n];
      if (c >= 0) a.row_node[r] = c;
    }
  }
}

__global__ __launch_bounds__(256) void partition_column_kernel(PartitionArgs a) {
  const int item = blockIdx.x;
  if (item >= a.num_items) return;
  const int sp = a.item_split[item];
  const int32_t dflt = a.split_default[sp], other = a.split_other[sp];
  const int32_t thr = a.split_bin[sp];
  const bool left_default = a.split_left_is_default[sp] != 0;
  for (int64_t e = a.item_start[item] + threadIdx.x; e < a.item_end[item]; e += 256) {
    const int32_t row = a.csc_row[e];
    const bool left = (int32_t)a.csc_bin[e] <= thr;
    if (left != left_default && a.row_node[row] == dflt) a.row_node[row] = other;
  }
}

// ------------------------------------------------------------------ gbdt helpers
__global__ __launch_bounds__(256) void logistic_grad_kernel(const double* margin, const float* label,
                                                            const float* weight, float* g, float* h, int64_t N) {
  for (int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x; r < N; r += (int64_t)gridDim.x * 256) {
    const double p = 1.0 / (1.0 + exp(-margin[r]));
    const double w = weight ? (double)weight[r] : 1.0;
    g[r] = (float)((p - (double)label[r]) * w);
    h[r] = (float)(fmax(p * (1.0 - p), 1e-16) * w);
  }
}

__global__ __launch_bounds__(256) void leaf_update_kernel(double* margin, const int32_t* row_node,
                                                          const double* node_value, int64_t N) {
  for (int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x; r < N; r += (int64_t)gridDim.x * 256)
    margin[r] += node_value[row_node[r]];
}

inline unsigned grid_for(int64_t n, int64_t cap = 8192) {
  const int64_t b = (n + 255) / 256;
  return (unsigned)(b < 1 ? 1 : (b > cap ? cap : b));
}
}  // namespace

void launch_rowstats(const RowStatsArgs& a, hipStream_t s) {
  if (a.N > 0) hipLaunchKernelGGL(rowstats_kernel, dim3(grid_for(a.N)), dim3(256), 0, s, a);
}

void launch_entry_stats(const int32_t* csc_row, const uint32_t* rowstats, int64_t nnz, uint32_t* est, hipStream_t s) {
  if (nnz <= 0) return;
  hipLaunchKernelGGL(entry_stats_kernel, dim3(grid_for(nnz / 4 + 1, 16384)), dim3(256), 0, s, csc_row,
                     reinterpret_cast<const uint2*>(rowstats), nnz, reinterpret_cast<uint2*>(est));
}

void launch_entry_stats_items(const int64_t* item_start, const int64_t* item_end, const int32_t* wave_item,
                              int32_t num_slots, int32_t num_items, const int32_t* csc_row, const uint32_t* rowstats,
                              uint32_t* est, hipStream_t s) {
  if (num_slots <= 0) return;
  hipLaunchKernelGGL(entry_stats_items_kernel, dim3((unsigned)(num_slots / 4)), dim3(256), 0, s, item_start, item_end,
                     wave_item, num_items, csc_row, reinterpret_cast<const uint2*>(rowstats),
                     reinterpret_cast<uint2*>(est));
}

void launch_slot8(const SlotArgs& a, hipStream_t s) {
  if (a.N > 0) hipLaunchKernelGGL(slot8_kernel, dim3(grid_for(a.N)), dim3(256), 0, s, a);
}

void launch_hist_mfma(const HistArgs& a, int bt, int ct, hipStream_t s) {
  if (a.num_items <= 0) return;
  const int32_t slots = a.wave_item ? a.num_slots : a.num_items;
  const dim3 grid((slots + 3) / 4), block(256);
  const bool root = a.slot8 == nullptr;
  const bool gather = a.rowstats != nullptr;
  // bt 0: narrow 16-bin tile (ct = 1/2/4/8 groups of 4 slots); bt 1/2: 32-bin tiles (ct groups of 8)
#define FDX_HIST_SRC(B, C, N, S)                                                                         \
  if (gather == S) {                                                                                    \
    if (root) hipLaunchKernelGGL((hist_mfma_kernel<B, C, true, N, S>), grid, block, 0, s, a);           \
    else hipLaunchKernelGGL((hist_mfma_kernel<B, C, false, N, S>), grid, block, 0, s, a);               \
  }
#define FDX_HIST_CASE(B, C, N)                                                                           \
  if (bt == (N ? 0 : B) && ct == C) {                                                                   \
    FDX_HIST_SRC(B, C, N, false) FDX_HIST_SRC(B, C, N, true)                                            \
    return;                                                                                             \
  }
  FDX_HIST_CASE(1, 1, true) FDX_HIST_CASE(1, 2, true) FDX_HIST_CASE(1, 4, true) FDX_HIST_CASE(1, 8, true)
  FDX_HIST_CASE(1, 1, false) FDX_HIST_CASE(1, 2, false) FDX_HIST_CASE(1, 4, false)
  FDX_HIST_CASE(2, 1, false) FDX_HIST_CASE(2, 2, false) FDX_HIST_CASE(2, 4, false)
#undef FDX_HIST_CASE
#undef FDX_HIST_SRC
}

void launch_hist_reduce(const HistReduceArgs& a, hipStream_t s) {
  const int64_t n = (int64_t)a.L * a.slab_slots * a.slab_bins;
  if (n <= 0) return;
  hipLaunchKernelGGL(hist_reduce_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, a);
}

void launch_hist_subtract(const double* parent, double* cur, const int32_t* dst, const int32_t* par, const int32_t* sib,
                          int32_t n_pairs, int64_t TB, hipStream_t s) {
  if (n_pairs <= 0 || TB <= 0) return;
  hipLaunchKernelGGL(hist_subtract_kernel, dim3(grid_for((int64_t)n_pairs * TB * 2)), dim3(256), 0, s, parent, cur,
                     dst, par, sib, n_pairs, TB);
}

void launch_split(const SplitArgs& a, hipStream_t s) {
  const int64_t n = (int64_t)a.num_nodes * a.Fa;
  if (n <= 0) return;
  hipLaunchKernelGGL(split_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, a);
}

void launch_partition(const PartitionArgs& a, hipStream_t s) {
  if (a.N > 0) hipLaunchKernelGGL(partition_default_kernel, dim3(grid_for(a.N)), dim3(256), 0, s, a);
  if (a.num_items > 0) hipLaunchKernelGGL(partition_column_kernel, dim3(a.num_items), dim3(256), 0, s, a);
}

void launch_logistic_grad(const double* margin, const float* label, const float* weight, float* g, float* h,
                          int64_t N, hipStream_t s) {
  if (N > 0) hipLaunchKernelGGL(logistic_grad_kernel, dim3(grid_for(N)), dim3(256), 0, s, margin, label, weight, g, h, N);
}

void launch_leaf_update(double* margin, const int32_t* row_node, const double* node_value, int64_t N, hipStream_t s) {
  if (N > 0) hipLaunchKernelGGL(leaf_update_kernel, dim3(grid_for(N)), dim3(256), 0, s, margin, row_node, node_value, N);
}

}  // namespace fdx

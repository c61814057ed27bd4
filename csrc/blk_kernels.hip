// Row-blocked i8-MFMA histogram engine (gfx950): the blocked CSC build and the histogram pass of
// tree.h "row-blocked histogram engine". Replaces, at the levels that build at most four node
// slots, the gather-bound CSC passes of tree_kernels.hip: there every entry fetched its row's
// slot byte and 8-byte digit word from global memory -- one distinct cache line per entry, since
// a sparse feature's entries are ~700 rows apart -- which bound a level at ~3 ms on 10M rows
// (profiles/r2s3/NOTES.md). Here a workgroup stages each 4096-row chunk's row state in LDS with
// coalesced loads and its 16 waves look the rows up there (bench/probes/gather_probe.hip: the
// same ~0.39 B entries take 0.34-0.45 ms with LDS-staged row state against 1.6-3.4 ms with global
// gathers). Histogram sums stay exact integers, so every tree is bitwise the one the CSC passes
// (and the host) grow.
#include "hist_i8.h"
#include "ops.h"
#include "tree.h"

#pragma clang fp contract(off)

namespace fdx {

namespace {

// ------------------------------------------------------------------ blocked CSC build
// largest f with colptr[f] <= e (empty features share their successor's start: the search lands
// on the non-empty one)
__device__ __forceinline__ int32_t feature_of_entry(const int64_t* colptr, int32_t Fa, int64_t e) {
  int32_t lo = 0, hi = Fa;
  while (hi - lo > 1) {
    const int32_t mid = (lo + hi) >> 1;
    if (colptr[mid] <= e) lo = mid;
    else hi = mid;
  }
  return lo;
}

// Thread t walks entries [t * ept, (t + 1) * ept) of the feature-major CSC. Consecutive entries of
// one feature fall into the same (chunk, 16-bin tile) sub-segment for runs of several entries, so the
// segment counters take one atomic per run: pass 0 counts, pass 1 reserves the run's slots with
// one returning atomic and writes the (row offset, key) pairs. The order of runs inside a segment
// depends on the atomics; histogram sums are exact, so no result depends on it.
__global__ __launch_bounds__(256) void blk_build_kernel(BlkBuildArgs a, int pass) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t e0 = t * a.entries_per_thread;
  if (e0 >= a.nnz) return;
  const int64_t e1 = e0 + a.entries_per_thread < a.nnz ? e0 + a.entries_per_thread : a.nnz;
  int32_t f = feature_of_entry(a.colptr, a.Fa, e0);
  int64_t fend = a.colptr[f + 1];
  int64_t run_key = -1, run_start = e0;
  int32_t run_f = f, run_len = 0;
  auto flush = [&]() {
    if (run_len == 0) return;
    if (pass == 0) {
      atomicAdd(a.counts + run_key, run_len);
      return;
    }
    const int64_t base =
        (int64_t)atomicAdd(reinterpret_cast<unsigned long long*>(a.cursor + run_key), (unsigned long long)run_len);
    int32_t g = run_f;
    int64_t gend = a.colptr[g + 1];
    for (int32_t j = 0; j < run_len; ++j) {
      const int64_t e = run_start + j;
      while (e >= gend) gend = a.colptr[++g + 1];
      const int64_t gb = a.boff[g] + a.csc_bin[e];
      a.ent_row[base + j] = (uint16_t)(a.csc_row[e] % a.chunk_rows);
      a.ent_key[base + j] = (uint8_t)(gb & (kBlkKeys - 1));
    }
  };
  for (int64_t e = e0; e < e1; ++e) {
    while (e >= fend) fend = a.colptr[++f + 1];
    const int64_t gb = a.boff[f] + a.csc_bin[e];
    const int64_t key = (int64_t)(a.csc_row[e] / a.chunk_rows) * (kBlkTiles * a.NG) + gb / 16;
    if (key != run_key) {
      flush();
      run_key = key;
      run_start = e;
      run_f = f;
      run_len = 0;
    }
    ++run_len;
  }
  flush();
}

// ------------------------------------------------------------------ histogram pass
// Plane rows of the staged step are 288 B apart (256 + 32): the 16 lanes of one ds_read_b128
// group read planes q = 0..7 at K offsets 16 g, and at a 256-B stride all 8 planes hit the same
// banks (8-way conflicts, measured 70 % of the LDS cycles); at 288 B = 72 dwords the 16 reads of
// a lane group start at 8 q + 4 g (mod 64) dwords: 16 distinct 4-bank blocks.
constexpr int kBlkPlaneStride = 288;
// LDS: double-buffered chunk row state (digit words + slot bytes) shared by the workgroup, and per
// compute wave one 256-entry step staged plane-major (keys, 8 digit planes, slots) as MFMA operands.
// Segment descriptors of the workgroup's groups for kBlkDescBufs chunks (a ring the staging wave
// keeps kBlkDescBufs - 2 chunks ahead of the chunk being processed), so that a compute wave walks
// its (chunk, group, step) sequence -- and issues the entry loads of steps ahead -- without a
// dependent global load per segment.
constexpr int kBlkDescBufs = 8;
constexpr int kBlkSlots = kBlkCompute * kBlkGroupsMax;    // (wave, group) slots of a workgroup

template <bool ROOT>
struct BlkShared {
  uint2 dig[2][kBlkRows];
  uint8_t slot[2][ROOT ? 16 : kBlkRows];
  uint8_t key[kBlkCompute][256];
  uint8_t pl[kBlkCompute][8][kBlkPlaneStride];
  uint8_t sl[kBlkCompute][ROOT ? 16 : 256];
  int64_t d_e0[kBlkDescBufs][kBlkSlots];                 // segment start
  int32_t d_n[kBlkDescBufs][kBlkSlots];                  // segment length
  int32_t d_t[kBlkDescBufs][3][kBlkSlots];               // tile 1..3 starts relative to d_e0
};

// The staging wave: chunk c's row state -> LDS buffer buf (rows past N read as zero / no slot).
// All 36 KB of the chunk are requested at once (36 x 16 B per lane in registers: the staging wave
// holds no accumulators), so a chunk costs one memory latency, not one per 4 KB.
template <bool ROOT>
__device__ __forceinline__ void stage_chunk(const BlkHistArgs& a, BlkShared<ROOT>& sh, int buf, int32_t c, int lane) {
  const int64_t r0 = (int64_t)c * kBlkRows;
  const int64_t nrow = a.N - r0 < kBlkRows ? a.N - r0 : kBlkRows;
  if (nrow == kBlkRows) {
    constexpr int KD = kBlkRows / 2 / 64;                      // uint4 (2 rows) per lane: 32
    const uint4* src = reinterpret_cast<const uint4*>(a.rowdig + 2 * r0);
    uint4* dst = reinterpret_cast<uint4*>(&sh.dig[buf][0]);
    uint4 v[KD];
#pragma unroll
    for (int u = 0; u < KD; ++u) v[u] = src[u * 64 + lane];
    uint4 sv[4];
    if constexpr (!ROOT) {
      const uint4* ss = reinterpret_cast<const uint4*>(a.slot8 + r0);
#pragma unroll
      for (int u = 0; u < 4; ++u) sv[u] = ss[u * 64 + lane];
    }
#pragma unroll
    for (int u = 0; u < KD; ++u) dst[u * 64 + lane] = v[u];
    if constexpr (!ROOT) {
      uint4* sd = reinterpret_cast<uint4*>(&sh.slot[buf][0]);
#pragma unroll
      for (int u = 0; u < 4; ++u) sd[u * 64 + lane] = sv[u];
    }
  } else {
    for (int i = lane; i < kBlkRows; i += 64) {
      const bool in = i < nrow;
      sh.dig[buf][i] = in ? make_uint2(a.rowdig[2 * (r0 + i)], a.rowdig[2 * (r0 + i) + 1]) : make_uint2(0u, 0u);
      if constexpr (!ROOT) sh.slot[buf][i] = in ? a.slot8[r0 + i] : (uint8_t)0xff;
    }
  }
}

// One 256-entry step of a segment [e0, e1): 4 entries per lane, their row state looked up in the
// chunk's LDS image and staged plane-major (keys, 8 digit planes, slots) for the K-steps.
template <bool ROOT>
__device__ __forceinline__ void blk_stage_step(BlkShared<ROOT>& sh, int buf, int wid, int lane, int32_t base,
                                               int32_t e0, int32_t e1, uint2 rr, uint32_t keys4) {
  const int32_t e = base + 4 * lane;
  uint32_t w[8];
  uint32_t slots4 = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int row = (int)(((j < 2 ? rr.x : rr.y) >> (16 * (j & 1))) & 0xffffu);
    const bool live = e + j >= e0 && e + j < e1;
    const uint2 d = sh.dig[buf][row];
    w[2 * j] = live ? d.x : 0u;
    w[2 * j + 1] = live ? d.y : 0u;
    if (!live) keys4 |= 0xffu << (8 * j);
    if constexpr (!ROOT) slots4 |= (uint32_t)(live ? sh.slot[buf][row] : (uint8_t)0xff) << (8 * j);
  }
  *reinterpret_cast<uint32_t*>(&sh.key[wid][4 * lane]) = keys4;
#pragma unroll
  for (int st = 0; st < 2; ++st)
#pragma unroll
    for (int p = 0; p < 4; ++p)
      *reinterpret_cast<uint32_t*>(&sh.pl[wid][st * 4 + p][4 * lane]) =
          gather_byte(w[st], w[2 + st], w[4 + st], w[6 + st], (uint32_t)p);
  if constexpr (!ROOT) *reinterpret_cast<uint32_t*>(&sh.sl[wid][4 * lane]) = slots4;
}

// The K-steps of one staged step into one group's accumulators: A = one-hot(key) over the group's
// 4 row tiles, B = digit planes (masked to the column's slot on non-root passes).
// Entries of a segment are ordered by 16-bin tile (tile t = entries [t_t, t_{t+1}) relative to
// the segment start), so each 64-entry K-step multiplies only the 1-2 tiles it actually holds.
template <int CT, bool ROOT>
__device__ __forceinline__ void blk_ksteps(BlkShared<ROOT>& sh, int wid, int lane, int32_t base, int32_t n,
                                           int32_t t1, int32_t t2, int32_t t3, i32x4 (&acc)[4][CT]) {
  const int r = lane & 15, g = lane >> 4;
  const int slot_sub = r / 8, q = r % 8;                 // NP = 4: 8 columns per slot, 2 slots per tile
  const int32_t span = n - base < 256 ? n - base : 256;
  const int nks = (span + 63) >> 6;
  // rolled: unrolling it (nks <= 4) removed the accumulator copies around each step but raised the
  // register pressure until the entry-load ring lost its static registers (every load then waited
  // for vmcnt(0): 3.5x slower end to end, profiles/r3/NOTES.md)
#pragma unroll 1
  for (int ks = 0; ks < nks; ++ks) {
    const int32_t lo = base + 64 * ks > 0 ? base + 64 * ks : 0;          // first live entry (segment-relative)
    const int32_t hi = (base + 64 * ks + 64 < n ? base + 64 * ks + 64 : n) - 1;   // last live entry
    const int tlo = (lo >= t1) + (lo >= t2) + (lo >= t3), thi = (hi >= t1) + (hi >= t2) + (hi >= t3);
    const int k0 = ks * 64 + 16 * g;
    const uint4 kv = *reinterpret_cast<const uint4*>(&sh.key[wid][k0]);
    const uint4 dv = *reinterpret_cast<const uint4*>(&sh.pl[wid][q][k0]);
    const uint4 k7 = make_uint4(kv.x & 0x7f7f7f7fu, kv.y & 0x7f7f7f7fu, kv.z & 0x7f7f7f7fu, kv.w & 0x7f7f7f7fu);
    i32x4 B[CT];
    if constexpr (ROOT) {
      B[0] = i32x4{(int)dv.x, (int)dv.y, (int)dv.z, (int)dv.w};
    } else {
      const uint4 sv = *reinterpret_cast<const uint4*>(&sh.sl[wid][k0]);
      slot_masked_b<CT, 4>(dv, sv, slot_sub, B);
    }
#pragma unroll
    for (int bt = 0; bt < 4; ++bt) {
      if (bt < tlo || bt > thi) continue;                 // wave-uniform
      const uint32_t nk = ~((uint32_t)(r + 16 * bt) * 0x01010101u);
      const i32x4 A = {(int)onehot7(k7.x, nk), (int)onehot7(k7.y, nk), (int)onehot7(k7.z, nk), (int)onehot7(k7.w, nk)};
#pragma unroll
      for (int ct = 0; ct < CT; ++ct)
        acc[bt][ct] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A, B[ct], acc[bt][ct], 0, 0, 0);
    }
  }
}

// acc of one group -> int64 histogram (exact: -128 * plane sums recombined over the 4 planes),
// then zeroed. Lanes q % 4 == 0 hold a (slot, statistic) column's recombined sums.
template <int CT>
__device__ __forceinline__ void blk_flush(const BlkHistArgs& a, int grp, int lane, i32x4 (&acc)[4][CT]) {
  const int r = lane & 15, g = lane >> 4;
  const int slot_sub = r / 8, q = r % 8, stat = q / 4;
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) {
    const int slot = ct * 2 + slot_sub;
    const int node = slot < a.nslots ? a.slot_node[slot] : -1;
#pragma unroll
    for (int bt = 0; bt < 4; ++bt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int32_t s = -(acc[bt][ct][i] >> 7);
        const int32_t s1 = __shfl_down(s, 1, kWave), s2 = __shfl_down(s, 2, kWave), s3 = __shfl_down(s, 3, kWave);
        const int64_t v = (int64_t)s + (int64_t)s1 * 256 + (int64_t)s2 * 65536 + (int64_t)s3 * 16777216;
        const int64_t bin = (int64_t)grp * kBlkKeys + 16 * bt + 4 * g + i;
        if ((q & 3) == 0 && v != 0 && node >= 0 && bin < a.TB) {
          int64_t* dst = a.hist + ((int64_t)node * a.hist_stride + blk_bin_offset(a, bin)) * 2 + stat;
          atomicAdd(reinterpret_cast<unsigned long long*>(dst), (unsigned long long)v);
        }
        acc[bt][ct][i] = 0;
      }
  }
}

// The staging wave's segment descriptors of chunk cc for the workgroup's (wave, group) slots:
// lane s < 7 gw loads slot s's five segment bounds (one latency for the whole table).
struct BlkDescRegs {
  int64_t s[5];
};

__device__ __forceinline__ BlkDescRegs load_descs(const BlkHistArgs& a, int32_t cc, int my_g) {
  BlkDescRegs r{};
  if (my_g >= 0) {
    const int64_t* sg = a.seg + ((int64_t)cc * a.NG + my_g) * kBlkTiles;
#pragma unroll
    for (int i = 0; i < 5; ++i) r.s[i] = sg[i];
  }
  return r;
}

template <bool ROOT>
__device__ __forceinline__ void store_descs(BlkShared<ROOT>& sh, int32_t rel, int lane, int nslots, const BlkDescRegs& r) {
  if (lane >= nslots) return;
  const int b = rel & (kBlkDescBufs - 1);
  sh.d_e0[b][lane] = r.s[0];
  sh.d_n[b][lane] = (int32_t)(r.s[4] - r.s[0]);
#pragma unroll
  for (int i = 0; i < 3; ++i) sh.d_t[b][i][lane] = (int32_t)(r.s[i + 1] - r.s[0]);
}

// One 256-entry step of a compute wave: chunk c, the wave's group slot j, segment [e0, e0 + n),
// entries [e0 + base, e0 + base + 256) (e0 + base 4-aligned; base may be -1 .. -3). n == 0 marks
// a step without work: a bubble (the walk may not look further ahead yet) or, at c == c1, the end.
struct BlkStep {
  int32_t c, j, n, base, t1, t2, t3;
  int64_t e0;
};

// The wave's walk: the next step of its sequence, read from the descriptor ring in LDS. The walk
// may enter chunks <= limit only (their descriptors are staged); beyond, it yields bubbles.
struct BlkWalk {
  int32_t c, j;
  bool ready;
  BlkStep cur;
};

__device__ __forceinline__ int32_t uni(int32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ int64_t uni64(int64_t v) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v), hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return (int64_t)(((uint64_t)hi << 32) | lo);
}

template <bool ROOT>
__device__ __forceinline__ BlkStep blk_take(const BlkShared<ROOT>& sh, BlkWalk& w, int wid, int gw, int32_t c0,
                                            int32_t c1, int32_t limit) {
  while (!w.ready && w.c < c1 && w.c <= limit) {
    if (w.j >= gw) {
      ++w.c;
      w.j = 0;
      continue;
    }
    const int b = (w.c - c0) & (kBlkDescBufs - 1), s = wid * gw + w.j;
    const int32_t n = uni(sh.d_n[b][s]);
    if (n > 0) {
      w.cur.c = w.c;
      w.cur.j = w.j;
      w.cur.n = n;
      w.cur.e0 = uni64(sh.d_e0[b][s]);
      w.cur.base = -(int32_t)(w.cur.e0 & 3);
      w.cur.t1 = uni(sh.d_t[b][0][s]);
      w.cur.t2 = uni(sh.d_t[b][1][s]);
      w.cur.t3 = uni(sh.d_t[b][2][s]);
      w.ready = true;
    } else {
      ++w.j;
    }
  }
  if (w.ready) {
    const BlkStep s = w.cur;
    w.cur.base += 256;
    if (w.cur.base >= w.cur.n) {
      w.ready = false;
      ++w.j;
    }
    return s;
  }
  BlkStep s{};
  s.c = w.c < c1 ? w.c : c1;        // bubble at the chunk the walk waits in, or the end
  return s;
}

__device__ __forceinline__ void blk_load(const BlkHistArgs& a, const BlkStep& k, int lane, uint2& rr, uint32_t& keys4) {
  // always one load pair per step (a step without work reads entry 0): the wave's loads stay a
  // fixed-depth ring, so the wait for a step's entries is vmcnt(2 * (kBlkAhead - 1)), never 0
  int64_t el = 0;
  if (k.n > 0) {
    const int64_t abs_last4 = (k.e0 + k.n - 1) & ~(int64_t)3;       // last 4-group holding an entry
    const int64_t abs_e = k.e0 + k.base + 4 * lane;
    el = abs_e < abs_last4 ? abs_e : abs_last4;
  }
  rr = *reinterpret_cast<const uint2*>(a.ent_row + el);
  keys4 = *reinterpret_cast<const uint32_t*>(a.ent_key + el);
}

constexpr int kBlkAhead = 4;       // steps of entry loads in flight per compute wave

// GW groups per compute wave (GW * CT * 16 accumulator registers <= 128). The accumulators are
// flushed once, at the end: the planner keeps every workgroup's chunk range short enough that no
// int32 (key, column) sum can overflow (models/quantize.py BlockedCSC.plan; an in-loop flush made
// the compiler spill the accumulators).
//
// Chunk protocol (all 8 waves execute 1 + (c1 - c0) barriers): before the first barrier the
// staging wave writes chunk c0's row state and the descriptors of chunks c0 .. c0 + kBlkDescBufs
// - 2; between barriers c and c + 1 the compute waves process chunk c while it writes chunk c +
// 1's row state and chunk c + kBlkDescBufs - 1's descriptors into the buffers chunk c - 1 used.
// A compute wave passes barrier c when its walk reaches a step of a later chunk (a bubble
// included); its ring of kBlkAhead steps is indexed statically (the loop is unrolled kBlkAhead
// times), so no loaded register is ever moved -- a move would wait for the load.
template <int CT, bool ROOT, int GW>
__global__ __launch_bounds__(kBlkWaves * 64) void hist_blk_kernel(BlkHistArgs a) {
  __shared__ BlkShared<ROOT> sh;
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const bool stager = wid == kBlkCompute;
  const int w = blockIdx.x;
  if (w >= a.n_wg) return;
  const int band = a.wg_band[w];
  const int32_t c0 = a.wg_c0[w], c1 = a.wg_c1[w];
  const int gw = a.gw;
  if (stager) {
    const int nslots = kBlkCompute * gw;
    const int my_g = lane < nslots ? a.band_groups[(int64_t)band * nslots + lane] : -1;
    BlkDescRegs d[kBlkDescBufs - 1];
#pragma unroll
    for (int k = 0; k < kBlkDescBufs - 1; ++k) d[k] = c0 + k < c1 ? load_descs(a, c0 + k, my_g) : BlkDescRegs{};
    stage_chunk<ROOT>(a, sh, 0, c0, lane);
#pragma unroll
    for (int k = 0; k < kBlkDescBufs - 1; ++k) store_descs<ROOT>(sh, k, lane, nslots, d[k]);
    __syncthreads();
    for (int32_t c = c0; c < c1; ++c) {
      const int32_t cd = c + kBlkDescBufs - 1;
      const BlkDescRegs dn = cd < c1 ? load_descs(a, cd, my_g) : BlkDescRegs{};
      if (c + 1 < c1 && !(a.dbg & 4)) stage_chunk<ROOT>(a, sh, (c - c0 + 1) & 1, c + 1, lane);   // overlaps chunk c
      if (cd < c1) store_descs<ROOT>(sh, cd - c0, lane, nslots, dn);
      __syncthreads();
    }
    return;
  }
  i32x4 acc[GW][4][CT];
#pragma unroll
  for (int j = 0; j < GW; ++j)
#pragma unroll
    for (int bt = 0; bt < 4; ++bt)
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) acc[j][bt][ct] = i32x4{0, 0, 0, 0};
  __syncthreads();                                         // chunk c0 and the first descriptors staged
  int32_t cur = c0;
  BlkWalk walk{c0, 0, false, BlkStep{}};
  BlkStep ring[kBlkAhead];
  uint2 rq[kBlkAhead];
  uint32_t kq[kBlkAhead];
#pragma unroll
  for (int i = 0; i < kBlkAhead; ++i) {
    ring[i] = blk_take<ROOT>(sh, walk, wid, gw, c0, c1, cur + kBlkDescBufs - 2);
    // issue order fixed (slot 0 first): the loop header's wait for slot 0 is then vmcnt(6), not 0
    __builtin_amdgcn_sched_barrier(0);
    blk_load(a, ring[i], lane, rq[i], kq[i]);
    __builtin_amdgcn_sched_barrier(0);
  }
  // trips of kBlkAhead steps; the exit test sits at the trip end only, so every slot's loads are
  // issued on every path (a mid-trip exit let the compiler skip a slot's load on the path that
  // leaves, and the merged wait state then drained the whole ring at each step)
  bool more = true;
  while (more) {
#pragma unroll
    for (int u = 0; u < kBlkAhead; ++u) {
      const BlkStep now = ring[u];
      while (cur < now.c) {                                // chunk cur done
        __syncthreads();
        ++cur;
      }
      const bool work = now.n > 0 && cur < c1;
      // staged unconditionally (a step without work stages nothing live): every path consumes the
      // slot's loads before the slot is reloaded, so no path waits for younger loads
      if (!(a.dbg & 2)) blk_stage_step<ROOT>(sh, (cur - c0) & 1, wid, lane, now.base, 0, work ? now.n : 0, rq[u], kq[u]);
      ring[u] = blk_take<ROOT>(sh, walk, wid, gw, c0, c1, cur + kBlkDescBufs - 2);
      __builtin_amdgcn_sched_barrier(0);
      blk_load(a, ring[u], lane, rq[u], kq[u]);
      __builtin_amdgcn_sched_barrier(0);
      if (work && !(a.dbg & 1)) {
        lds_sync();
        switch (now.j) {
#define FDX_BLK_CASE(J) \
  case J:               \
    if constexpr (J < GW) blk_ksteps<CT, ROOT>(sh, wid, lane, now.base, now.n, now.t1, now.t2, now.t3, acc[J]); \
    break;
          FDX_BLK_CASE(0) FDX_BLK_CASE(1) FDX_BLK_CASE(2) FDX_BLK_CASE(3)
          FDX_BLK_CASE(4) FDX_BLK_CASE(5) FDX_BLK_CASE(6) FDX_BLK_CASE(7)
#undef FDX_BLK_CASE
          default: break;
        }
        lds_sync();
      }
    }
    more = cur < c1;
  }
  {
    const int nslots = kBlkCompute * gw;
#pragma unroll
    for (int j = 0; j < GW; ++j) {
      const int g = j < gw ? a.band_groups[(int64_t)band * nslots + wid * gw + j] : -1;
      if (g >= 0) blk_flush<CT>(a, g, lane, acc[j]);
    }
  }
}

}  // namespace

void launch_blk_build(const BlkBuildArgs& a, int pass, hipStream_t s) {
  if (a.nnz <= 0) return;
  const int64_t threads = (a.nnz + a.entries_per_thread - 1) / a.entries_per_thread;
  hipLaunchKernelGGL(blk_build_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, s, a, pass);
}

int blk_groups_per_wave(int ct) { return ct <= 1 ? kBlkGroupsMax : kBlkGroupsMax / 2; }

void launch_hist_blk(const BlkHistArgs& a, int ct, hipStream_t s) {
  if (a.n_wg <= 0) return;
  const bool root = a.slot8 == nullptr;
  const dim3 grid(a.n_wg), block(kBlkWaves * 64);
  if (root) hipLaunchKernelGGL((hist_blk_kernel<1, true, kBlkGroupsMax>), grid, block, 0, s, a);
  else if (ct == 1) hipLaunchKernelGGL((hist_blk_kernel<1, false, kBlkGroupsMax>), grid, block, 0, s, a);
  else if (ct == 2) hipLaunchKernelGGL((hist_blk_kernel<2, false, kBlkGroupsMax / 2>), grid, block, 0, s, a);
}

}  // namespace fdx

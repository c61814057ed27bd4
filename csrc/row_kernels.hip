// Row-group histogram engine (gfx950): the row-group CSR build, the per-level list of built rows
// grouped by node slot, and the histogram pass of tree.h "row-group histogram engine".
//
// Why rows: the CSC passes (tree_kernels.hip) walk every entry of every feature and gather the
// entry's row state (slot byte + 8-byte digit word) from global memory. A sparse feature's entries
// are ~700 rows apart, so each gather is a distinct cache line: ~386M lines per level at 10M rows,
// texture-address bound at ~3 ms per level whatever the tiling (profiles/r2s3/NOTES.md,
// profiles/r2s4/hist_REJECTED_*). Here the entries are laid out row-major inside each bin group,
// so a row's entries are contiguous: a lane loads its row's state ONCE and streams the row's run
// with 16-byte loads, and deep levels touch only the rows of the nodes they build (the list).
// Accumulation is into int64 LDS histograms (ds_add_u64: exact, order-free), one bin group of
// <= 8192 bins per workgroup, flushed to the level histogram with integer atomics per node slot.
#include "ops.h"
#include "tree.h"

#pragma clang fp contract(off)

namespace fdx {

namespace {

constexpr int kRgThreads = kRgWaves * 64;
constexpr int kRgBuildEpl = 32;        // build: entries per lane (a wave covers 64 x 32 consecutive entries)

// largest f with colptr[f] <= e (empty features share their successor's start)
__device__ __forceinline__ int32_t rg_feature_of(const int64_t* colptr, int32_t Fa, int64_t e) {
  int32_t lo = 0, hi = Fa;
  while (hi - lo > 1) {
    const int32_t mid = (lo + hi) >> 1;
    if (colptr[mid] <= e) lo = mid;
    else hi = mid;
  }
  return lo;
}

// A wave covers 64 * kRgBuildEpl consecutive CSC entries, lane l taking e = base + l + 64 k
// (coalesced loads; each lane tracks its feature forward). Pass 0 counts entries per (group, row),
// pass 1 reserves a position with a returning atomic and writes the local bin. The order inside a
// (group, row) run depends on the atomics; histogram sums are exact, so nothing depends on it.
__global__ __launch_bounds__(256) void rg_build_kernel(RgBuildArgs a, int pass) {
  const int64_t wave = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  const int64_t base = wave * (64 * kRgBuildEpl);
  if (base >= a.nnz) return;
  int64_t e = base + lane;
  if (e >= a.nnz) return;
  int32_t f = rg_feature_of(a.colptr, a.Fa, e);
  int64_t fend = a.colptr[f + 1];
  int32_t g = a.fgroup[f], loc = a.flocal[f];
  for (int k = 0; k < kRgBuildEpl; ++k, e += 64) {
    if (e >= a.nnz) break;
    while (e >= fend) {
      fend = a.colptr[++f + 1];
      g = a.fgroup[f];
      loc = a.flocal[f];
    }
    if (g < 0) continue;
    const int64_t r = a.csc_row[e];
    if (pass == 0) {
      atomicAdd(a.ptr + (int64_t)g * (a.N + 1) + r + 1, 1u);
    } else {
      const uint32_t pos = atomicAdd(a.cursor + (int64_t)g * a.N + r, 1u);
      a.ent[a.gbase[g] + pos] = (uint16_t)(loc + a.csc_bin[e]);
    }
  }
}

// One wave per kRgListRows consecutive rows, slots counted and placed with wave ballots (one
// ballot per distinct slot among each 64 rows, no atomics on the rows): pass 0 stores the wave's
// per-slot counts and adds them to the slot totals; pass 1 derives the slot starts (a wave scan of
// the totals), reserves the wave's share of every slot with one atomic per slot and writes its
// rows in ascending order.
__global__ __launch_bounds__(256) void rg_list_kernel(RgListArgs a, int pass) {
  const int64_t wave = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  const int64_t r0 = wave * kRgListRows;
  if (r0 >= a.N) return;
  const int64_t r1 = r0 + kRgListRows < a.N ? r0 + kRgListRows : a.N;
  const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  int32_t* wc = a.wave_count + wave * 64;
  if (pass == 0) {
    int32_t cnt = 0;                           // lane s: rows of slot s
    for (int64_t rb = r0; rb < r1; rb += 64) {
      const int64_t r = rb + lane;
      const uint32_t sl = r < r1 ? rg_slot_of(a, r) : 0xffu;
      uint64_t act = __ballot(sl < (uint32_t)a.nslots);
      while (act) {
        const uint32_t s = __shfl(sl, __ffsll((unsigned long long)act) - 1, 64);
        const uint64_t m = __ballot(sl == s);
        if ((uint32_t)lane == s) cnt += __popcll(m);
        act &= ~m;
      }
    }
    if (lane < a.nslots) {
      wc[lane] = cnt;
      if (cnt) atomicAdd(a.slot_count + lane, cnt);
    }
    return;
  }
  // slot starts: exclusive scan of the totals over lanes 0..nslots-1
  const int32_t tot = lane < a.nslots ? a.slot_count[lane] : 0;
  int32_t incl = tot;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int32_t o = __shfl_up(incl, d, 64);
    if (lane >= d) incl += o;
  }
  if (wave == 0) {
    if (lane < a.nslots) a.slot_start[lane] = incl - tot;
    if (lane == a.nslots - 1) a.slot_start[a.nslots] = incl;
  }
  const int32_t mine = lane < a.nslots ? wc[lane] : 0;
  int32_t base = lane < a.nslots ? incl - tot + (mine ? atomicAdd(a.slot_fill + lane, mine) : 0) : 0;
  for (int64_t rb = r0; rb < r1; rb += 64) {
    const int64_t r = rb + lane;
    const uint32_t sl = r < r1 ? rg_slot_of(a, r) : 0xffu;
    uint64_t act = __ballot(sl < (uint32_t)a.nslots);
    while (act) {
      const uint32_t s = __shfl(sl, __ffsll((unsigned long long)act) - 1, 64);
      const uint64_t m = __ballot(sl == s);
      const int32_t b = __shfl(base, (int)s, 64);
      if (sl == s) a.list[b + __popcll(m & lt)] = (int32_t)r;
      if ((uint32_t)lane == s) base += __popcll(m);
      act &= ~m;
    }
  }
}

template <int BINS>
struct RgShared {
  // separate statistic arrays (a lane's 8-byte atomic spans 2 of 64 banks); bins BINS + lane are
  // per-lane sinks for the lanes of a block outside their row's run (never flushed)
  int64_t hg[BINS + 64];
  int64_t hh[BINS + 64];
  // per wave: the 64 rows of the current batch (run start / end, statistics, first block index)
  uint32_t st[kRgWaves][64];
  uint32_t en[kRgWaves][64];
  int32_t q0[kRgWaves][64];
  int32_t q1[kRgWaves][64];
  uint32_t pb[kRgWaves][64];
};

template <int BINS>
__device__ __forceinline__ void rg_flush(const RgHistArgs& a, RgShared<BINS>& sh, int g, int s, int tid) {
  const int64_t hrow = a.slot_node[s];
  const int32_t* gbin = a.gbin + (int64_t)g * a.gbins;
  for (int i = tid; i < BINS; i += kRgThreads) {
    const int64_t v0 = sh.hg[i], v1 = sh.hh[i];
    if ((v0 | v1) != 0 && hrow >= 0) {
      const int32_t col = gbin[i];
      if (col >= 0) {
        int64_t* dst = a.hist + (hrow * a.hist_stride + rg_col_offset(a, col)) * 2;
        atomicAdd(reinterpret_cast<unsigned long long*>(dst), (unsigned long long)v0);
        atomicAdd(reinterpret_cast<unsigned long long*>(dst + 1), (unsigned long long)v1);
      }
    }
    sh.hg[i] = 0;
    sh.hh[i] = 0;
  }
}

__device__ __forceinline__ uint32_t rg_nblk(uint32_t st, uint32_t en) {
  return en > st ? ((en - 1) >> 3) - (st >> 3) + 1 : 0u;
}

// One batch of 64 rows of a wave, lane-balanced: the rows' 8-entry blocks are numbered
// consecutively (row by row) and lane l takes the contiguous block range [l K, (l + 1) K), K =
// ceil(blocks / 64), so every lane streams the same number of blocks whatever the row lengths
// (rows of the dense group vary ~2x: a lane per row left ~58% of the LDS atomic slots idle).
// Entries of a block outside its row's run go to the lane's sink bin: no divergent branches.
template <int BINS>
__device__ __forceinline__ void rg_batch(RgShared<BINS>& sh, const uint16_t* ent, int wv, int lane, uint32_t st,
                                         uint32_t en, int32_t q0, int32_t q1, int dbg, unsigned long long& sink) {
  const uint32_t nb = rg_nblk(st, en);
  uint32_t incl = nb;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t o = __shfl_up(incl, d, 64);
    if (lane >= d) incl += o;
  }
  const uint32_t total = __shfl(incl, 63, 64);
  if (total == 0) return;
  sh.st[wv][lane] = st;
  sh.en[wv][lane] = en;
  sh.q0[wv][lane] = q0;
  sh.q1[wv][lane] = q1;
  sh.pb[wv][lane] = incl - nb;
  __builtin_amdgcn_s_waitcnt(0xc07f);          // lgkmcnt(0): this wave's row table is in LDS
  __builtin_amdgcn_wave_barrier();
  const uint32_t K = (total + 63) >> 6;
  uint32_t t = (uint32_t)lane * K;
  const uint32_t t1 = t + K < total ? t + K : total;
  if (t < t1) {
    // row of block t: the largest r with pb[r] <= t (empty rows share their successor's pb)
    int r = 0;
#pragma unroll
    for (int step = 32; step >= 1; step >>= 1)
      if (r + step <= 63 && sh.pb[wv][r + step] <= t) r += step;
    uint32_t rst = sh.st[wv][r], ren = sh.en[wv][r];
    unsigned long long a0 = (unsigned long long)(int64_t)sh.q0[wv][r], a1 = (unsigned long long)(int64_t)sh.q1[wv][r];
    uint32_t rnb = rg_nblk(rst, ren);
    uint32_t j = t - sh.pb[wv][r];
    const uint32_t sinkb = BINS + lane;
    uint32_t blk = (rst & ~7u) + 8u * j;
    uint4 v = *reinterpret_cast<const uint4*>(ent + blk);
    for (;;) {
      // next block (same row, or the next non-empty row), loaded before this one is consumed
      const uint32_t cst = rst, cen = ren, cblk = blk;
      const unsigned long long c0 = a0, c1 = a1;
      ++t;
      const bool more = t < t1;
      uint4 vn = v;
      if (more) {
        if (++j == rnb) {
          do {                                   // the next row with blocks (t < total: one exists)
            ++r;
          } while (rg_nblk(sh.st[wv][r], sh.en[wv][r]) == 0);
          rst = sh.st[wv][r];
          ren = sh.en[wv][r];
          a0 = (unsigned long long)(int64_t)sh.q0[wv][r];
          a1 = (unsigned long long)(int64_t)sh.q1[wv][r];
          rnb = rg_nblk(rst, ren);
          j = 0;
        }
        blk = (rst & ~7u) + 8u * j;
        vn = *reinterpret_cast<const uint4*>(ent + blk);
      }
      const uint32_t wd[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const uint32_t i = cblk + k;
        const uint32_t bin = (wd[k >> 1] >> (16 * (k & 1))) & 0xffffu;
        const uint32_t b = (i >= cst && i < cen) ? bin : sinkb;
        if (dbg & 2) {
          sink += b;
        } else {
          atomicAdd(reinterpret_cast<unsigned long long*>(&sh.hg[b]), c0);
          atomicAdd(reinterpret_cast<unsigned long long*>(&sh.hh[b]), c1);
        }
      }
      if (!more) break;
      v = vn;
    }
  }
  __builtin_amdgcn_wave_barrier();               // the row table is rewritten by the next batch
}

// Workgroup w: chunk wg_p[w] (of wg_np[w]) of the built-row list, bin group wg_g[w]. Each wave
// takes batches of 64 listed rows and streams their runs inside the group in aligned 8-entry
// (16-byte) blocks, adding every entry's row statistics into the LDS histograms; at every slot
// boundary of the chunk the workgroup flushes its histograms to that slot's level histogram row.
// The pass is latency-bound (list -> (ptr, digits) -> entry blocks), so the next batch's row
// state and the next entry block are loaded before the current ones are consumed.
template <int BINS>
__global__ __launch_bounds__(kRgThreads) void rg_hist_kernel(RgHistArgs a) {
  __shared__ RgShared<BINS> sh;
  const int w = blockIdx.x;
  if (w >= a.n_wg) return;
  const int g = a.wg_g[w], p = a.wg_p[w], np_g = a.wg_np[w];
  const int64_t T = a.list ? (int64_t)a.slot_start[a.nslots] : a.N;
  const int64_t a0 = T * p / np_g, a1 = T * (p + 1) / np_g;
  if (a0 >= a1) return;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  for (int i = tid; i < BINS; i += kRgThreads) {
    sh.hg[i] = 0;
    sh.hh[i] = 0;
  }
  __syncthreads();
  int s = 0;
  if (a.list)
    while (s + 1 < a.nslots && a.slot_start[s + 1] <= a0) ++s;
  const uint32_t* ptr = a.ptr + (int64_t)g * (a.N + 1);
  const uint16_t* ent = a.ent + a.gbase[g];
  const int32_t* list = a.list;
  const int np = a.np, dbg = a.dbg;
  unsigned long long sink = 0;
  for (;;) {
    const int64_t ss0 = list ? (int64_t)a.slot_start[s] : 0;
    const int64_t ss1 = list ? (int64_t)a.slot_start[s + 1] : a.N;
    const int64_t lo = a0 > ss0 ? a0 : ss0, hi = a1 < ss1 ? a1 : ss1;
    // rows of batch k are pos = lo + wv * 64 + k * kRgThreads + lane; the list entry is read two
    // batches ahead, (ptr, digits) one batch ahead
    int64_t pos = lo + wv * 64 + lane;
    int64_t row_c = list ? (pos < hi ? (int64_t)list[pos] : -1) : (pos < hi ? pos : -1);
    int64_t row_n = -1;
    if (list && pos + kRgThreads < hi) row_n = list[pos + kRgThreads];
    uint32_t st = 0, en = 0;
    uint2 dg = make_uint2(0u, 0u);
    if (row_c >= 0) {
      st = ptr[row_c];
      en = ptr[row_c + 1];
      dg = *reinterpret_cast<const uint2*>(a.rowdig + 2 * row_c);
    }
    for (int64_t b0 = lo + wv * 64; b0 < hi; b0 += kRgThreads, pos += kRgThreads) {
      const int64_t pn = pos + kRgThreads;
      const int64_t rn = list ? row_n : (pn < hi ? pn : -1);
      if (list) row_n = pn + kRgThreads < hi ? (int64_t)list[pn + kRgThreads] : -1;
      uint32_t nst = 0, nen = 0;
      uint2 ndg = make_uint2(0u, 0u);
      if (rn >= 0) {
        nst = ptr[rn];
        nen = ptr[rn + 1];
        ndg = *reinterpret_cast<const uint2*>(a.rowdig + 2 * rn);
      }
      rg_batch<BINS>(sh, ent, wv, lane, st, en, (int32_t)rg_q(dg.x, np), (int32_t)rg_q(dg.y, np), dbg, sink);
      st = nst;
      en = nen;
      dg = ndg;
    }
    if (dbg & 2) atomicAdd(reinterpret_cast<unsigned long long*>(&sh.hg[lane]), sink);
    __syncthreads();
    rg_flush<BINS>(a, sh, g, s, tid);
    __syncthreads();
    if (!list || ss1 >= a1 || s + 1 >= a.nslots) break;
    ++s;
  }
}

}  // namespace

void launch_rg_build(const RgBuildArgs& a, int pass, hipStream_t s) {
  const int64_t waves = (a.nnz + 64 * kRgBuildEpl - 1) / (64 * kRgBuildEpl);
  const int64_t blocks = (waves + 3) / 4;
  if (blocks > 0) hipLaunchKernelGGL(rg_build_kernel, dim3((unsigned)blocks), dim3(256), 0, s, a, pass);
}

void launch_rg_list(const RgListArgs& a, int pass, hipStream_t s) {
  const int64_t waves = (a.N + kRgListRows - 1) / kRgListRows;
  const int64_t blocks = (waves + 3) / 4;
  if (blocks > 0) hipLaunchKernelGGL(rg_list_kernel, dim3((unsigned)blocks), dim3(256), 0, s, a, pass);
}

void launch_rg_hist(const RgHistArgs& a, hipStream_t s) {
  const int64_t blocks = a.n_wg;
  if (blocks <= 0) return;
  if (a.gbins == 4096)
    hipLaunchKernelGGL(rg_hist_kernel<4096>, dim3((unsigned)blocks), dim3(kRgThreads), 0, s, a);
  else
    hipLaunchKernelGGL(rg_hist_kernel<8192>, dim3((unsigned)blocks), dim3(kRgThreads), 0, s, a);
}

}  // namespace fdx

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

// Pass 0: per-slot row counts (LDS counters, one global atomic per (block, slot)).
// Pass 1: every block derives the slot starts from the counts, reserves its share of each slot
// with one atomic and places its rows. Rows of one block stay within one 4096-row window of the
// list; their order inside it depends on the LDS atomics (sums are exact: nothing depends on it).
__global__ __launch_bounds__(256) void rg_list_kernel(RgListArgs a, int pass) {
  __shared__ int32_t s_cnt[kRgMaxSlots];
  __shared__ int32_t s_base[kRgMaxSlots];
  const int tid = threadIdx.x;
  if (tid < kRgMaxSlots) s_cnt[tid] = 0;
  __syncthreads();
  const int64_t r0 = (int64_t)blockIdx.x * a.rows_per_block;
  const int64_t r1 = r0 + a.rows_per_block < a.N ? r0 + a.rows_per_block : a.N;
  for (int64_t r = r0 + tid; r < r1; r += 256) {
    const uint32_t s = a.slot8[r];
    if (s < (uint32_t)a.nslots) atomicAdd(&s_cnt[s], 1);
  }
  __syncthreads();
  if (pass == 0) {
    if (tid < a.nslots && s_cnt[tid] > 0) atomicAdd(a.slot_count + tid, s_cnt[tid]);
    return;
  }
  if (tid == 0) {
    int32_t acc = 0;
    for (int s = 0; s < a.nslots; ++s) {
      const int32_t c = a.slot_count[s];
      if (blockIdx.x == 0) a.slot_start[s] = acc;
      s_base[s] = acc;
      acc += c;
    }
    if (blockIdx.x == 0) a.slot_start[a.nslots] = acc;
  }
  __syncthreads();
  if (tid < a.nslots) {
    const int32_t c = s_cnt[tid];
    s_base[tid] += c > 0 ? atomicAdd(a.slot_fill + tid, c) : 0;
    s_cnt[tid] = 0;
  }
  __syncthreads();
  for (int64_t r = r0 + tid; r < r1; r += 256) {
    const uint32_t s = a.slot8[r];
    if (s < (uint32_t)a.nslots) a.list[s_base[s] + atomicAdd(&s_cnt[s], 1)] = (int32_t)r;
  }
}

template <int BINS>
struct RgShared {
  int64_t hg[BINS];               // separate statistic arrays: a lane's 8-byte atomic spans 2 of 64 banks
  int64_t hh[BINS];
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

// Workgroup w: chunk wg_p[w] (of wg_np[w]) of the built-row list, bin group wg_g[w]. Lane = row:
// the row's run inside the group is streamed in aligned 8-entry (16-byte) blocks and every entry
// adds the row's two statistics into the LDS histograms; at every slot boundary of the chunk the
// workgroup flushes its histograms to that slot's level histogram row. The pass is latency-bound
// (per batch of 64 rows: list -> (ptr, digits) -> entry blocks), so the next batch's row state and
// the next entry block are loaded before the current ones are consumed.
template <int BINS>
__device__ __forceinline__ void rg_row_run(RgShared<BINS>& sh, const uint16_t* ent, uint32_t st, uint32_t en,
                                           unsigned long long q0, unsigned long long q1, int dbg,
                                           unsigned long long& sink) {
  if (en <= st) return;
  uint32_t blk = st & ~7u;
  uint4 v = *reinterpret_cast<const uint4*>(ent + blk);
  for (;;) {
    const uint32_t nxt = blk + 8;
    uint4 vn = v;
    if (nxt < en) vn = *reinterpret_cast<const uint4*>(ent + nxt);
    const uint32_t wd[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const uint32_t i = blk + k;
      if (i >= st && i < en) {
        const uint32_t b = (wd[k >> 1] >> (16 * (k & 1))) & 0xffffu;
        if (dbg & 2) {
          sink += b;
        } else if (dbg & 4) {
          atomicAdd(reinterpret_cast<unsigned int*>(&sh.hg[b]), (unsigned int)q0);
          atomicAdd(reinterpret_cast<unsigned int*>(&sh.hh[b]), (unsigned int)q1);
        } else {
          atomicAdd(reinterpret_cast<unsigned long long*>(&sh.hg[b]), q0);
          atomicAdd(reinterpret_cast<unsigned long long*>(&sh.hh[b]), q1);
        }
      }
    }
    if (nxt >= en) break;
    blk = nxt;
    v = vn;
  }
}

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
      // prefetch: batch k + 1's row state, batch k + 2's list entry
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
      rg_row_run<BINS>(sh, ent, st, en, (unsigned long long)rg_q(dg.x, np), (unsigned long long)rg_q(dg.y, np), dbg,
                       sink);
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
  const int64_t blocks = (a.N + a.rows_per_block - 1) / a.rows_per_block;
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

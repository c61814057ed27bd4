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

struct RgShared {
  int64_t hg[kRgBins];            // separate statistic arrays: a lane's 8-byte atomic spans 2 of 64 banks
  int64_t hh[kRgBins];
};

__device__ __forceinline__ void rg_flush(const RgHistArgs& a, RgShared& sh, int g, int s, int tid) {
  const int64_t hrow = a.slot_node[s];
  const int32_t* gbin = a.gbin + (int64_t)g * kRgBins;
  for (int i = tid; i < kRgBins; i += kRgThreads) {
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

// Workgroup w: group g and list chunk p, w = ((p / 8) * G + g) * 8 + p % 8, so the G workgroups of
// one chunk share an XCD (workgroups are dealt round-robin over the 8 XCDs) and its L2 serves the
// chunk's row state G times. Lane = row: the row's (group) run is streamed in aligned 8-entry
// (16-byte) blocks; every entry adds the row's two statistics into the LDS histograms.
__global__ __launch_bounds__(kRgThreads) void rg_hist_kernel(RgHistArgs a) {
  __shared__ RgShared sh;
  const int w = blockIdx.x;
  const int x = w & 7, rest = w >> 3;
  const int g = rest % a.G;
  const int p = (rest / a.G) * 8 + x;
  if (p >= a.P) return;
  const int64_t T = a.list ? (int64_t)a.slot_start[a.nslots] : a.N;
  const int64_t a0 = T * p / a.P, a1 = T * (p + 1) / a.P;
  if (a0 >= a1) return;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  for (int i = tid; i < kRgBins; i += kRgThreads) {
    sh.hg[i] = 0;
    sh.hh[i] = 0;
  }
  __syncthreads();
  int s = 0;
  if (a.list)
    while (s + 1 < a.nslots && a.slot_start[s + 1] <= a0) ++s;
  const uint32_t* ptr = a.ptr + (int64_t)g * (a.N + 1);
  const uint16_t* ent = a.ent + a.gbase[g];
  const int np = a.np;
  for (;;) {
    const int64_t ss0 = a.list ? (int64_t)a.slot_start[s] : 0;
    const int64_t ss1 = a.list ? (int64_t)a.slot_start[s + 1] : a.N;
    const int64_t lo = a0 > ss0 ? a0 : ss0, hi = a1 < ss1 ? a1 : ss1;
    for (int64_t b0 = lo + wv * 64; b0 < hi; b0 += kRgThreads) {
      const int64_t pos = b0 + lane;
      uint32_t st = 0, en = 0;
      unsigned long long q0 = 0, q1 = 0;
      if (pos < hi) {
        const int64_t row = a.list ? (int64_t)a.list[pos] : pos;
        st = ptr[row];
        en = ptr[row + 1];
        if (en > st) {
          const uint2 d = *reinterpret_cast<const uint2*>(a.rowdig + 2 * row);
          q0 = (unsigned long long)rg_q(d.x, np);
          q1 = (unsigned long long)rg_q(d.y, np);
        }
      }
      for (uint32_t blk = st & ~7u; blk < en; blk += 8) {
        const uint4 v = *reinterpret_cast<const uint4*>(ent + blk);
        const uint32_t wd[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const uint32_t i = blk + k;
          if (i >= st && i < en) {
            const uint32_t b = (wd[k >> 1] >> (16 * (k & 1))) & 0xffffu;
            atomicAdd(reinterpret_cast<unsigned long long*>(&sh.hg[b]), q0);
            atomicAdd(reinterpret_cast<unsigned long long*>(&sh.hh[b]), q1);
          }
        }
      }
    }
    __syncthreads();
    rg_flush(a, sh, g, s, tid);
    __syncthreads();
    if (!a.list || ss1 >= a1 || s + 1 >= a.nslots) break;
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
  const int64_t blocks = (int64_t)a.G * a.P;
  if (blocks > 0) hipLaunchKernelGGL(rg_hist_kernel, dim3((unsigned)blocks), dim3(kRgThreads), 0, s, a);
}

}  // namespace fdx

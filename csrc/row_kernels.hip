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

template <class V>
__device__ __forceinline__ int32_t rg_count_bin(V c, int32_t max_bin) {
  if (!(c > (V)0)) return 0;
  const double d = (double)c;
  const int32_t b = d >= 255.0 ? 255 : (int32_t)d;
  return b < max_bin ? b : max_bin;
}

// A wave per 16 consecutive rows; their entries are consecutive in the CSR and are taken in chunks
// of up to 64 (a chunk never crosses a row), lanes over the chunk's entries (coalesced CSR reads).
// An entry's group and local offset come from one [F] lookup (fgl) of its feature id, so the chunks
// go through a 2-stage pipeline: the id / count loads of chunk k + 2 and the lookups of k + 1 are
// in flight while chunk k is placed. Every lane finds the lanes of its own group with one ballot
// per bit of the group id (4 for 11 groups; a ballot per distinct group was ~9 a chunk) and the
// groups' counts, then cursors, live in a per-wave LDS row. Runs keep the CSR order; no atomics.
// (A thread per row streamed ~97 entries serially at 2 blocks per CU: ~0.17 s at 10M rows; a wave
// per 64 rows, one row at a time: 34 ms.)
constexpr int kRgBuildRowsPerWave = 16;
// Pass 1 stages a wave's placed entries in LDS (local bin | row in the wave << 16), group by
// group, and writes each group's run of them with coalesced stores at the end: placing them
// straight into HBM was 2-byte stores scattered over the groups' regions, 22 ms of the 34 ms
// build at 10M rows. A wave with more entries than kRgStage places them directly.
constexpr int kRgStage = 2048;

__host__ __device__ __forceinline__ int64_t rg_build_waves(int64_t N) {
  return (N + kRgBuildRowsPerWave - 1) / kRgBuildRowsPerWave;
}
// per group in wave_base: the waves' totals, then the group total, padded to 16 bytes
__host__ __device__ __forceinline__ int64_t rg_build_stride(int64_t nwaves) { return (nwaves + 1 + 3) / 4 * 4; }

template <class V, int pass>
__device__ __forceinline__ void rg_build_csr_wave(const RgCsrBuildArgs<V>& a, uint32_t* stage, uint32_t* runs) {
  const int64_t wave = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  const int64_t wstride = rg_build_stride(rg_build_waves(a.N));   // wave_base [G][stride] (+ the totals)
  const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  const int64_t r0 = wave * kRgBuildRowsPerWave;
  if (r0 >= a.N) return;
  const int R = (int)(r0 + kRgBuildRowsPerWave < a.N ? kRgBuildRowsPerWave : a.N - r0);
  // lane j <= R: the start of row r0 + j (row j's entries: [start(j), start(j + 1)))
  const int64_t rb = lane <= R ? a.indptr[r0 + lane] : 0;
  auto start = [&](int j) -> int64_t {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)rb, j);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)rb >> 32), j);
    return (int64_t)(((uint64_t)hi << 32) | lo);
  };
  struct Chunk {
    int j;                         // row (R: past the wave's last chunk)
    int64_t e, end;                // entries [e, min(e + 64, end))
  };
  auto settle = [&](Chunk c) {     // skip past rows without (further) entries
    while (c.j < R && c.e >= c.end) {
      ++c.j;
      if (c.j < R) {
        c.e = start(c.j);
        c.end = start(c.j + 1);
      }
    }
    return c;
  };
  auto next = [&](Chunk c) {
    if (c.j >= R) return c;
    c.e += 64;
    return settle(c);
  };
  // stage 1: ids and counts; stage 2: group and local offset (-> local bin)
  auto load_ids = [&](const Chunk& c, int32_t& id, V& cnt) {
    const int64_t e = c.e + lane;
    const bool ok = c.j < R && e < c.end;
    id = ok ? a.idx[e] : -1;
    cnt = (ok && pass == 1) ? a.counts[e] : (V)0;
  };
  auto load_group = [&](int32_t id, V cnt, int32_t& g, int32_t& loc) {
    const int32_t v = id >= 0 ? a.fgl[id] : -1;
    g = v >= 0 ? (v >> 16) : -1;
    loc = (pass == 1 && g >= 0) ? (v & 0xffff) + rg_count_bin<V>(cnt, a.max_bin) : 0;
  };
  // runs[g] (the wave's LDS row): group g's running count over the wave's rows (pass 0), then its
  // next position (pass 1)
  const int ga = lane, gb = lane + 64;
  // pass 1: the wave's bases and counts per group; staged: run0 / run1 count from the group's
  // offset in the stage (sh0 / sh1 turn them back into group positions)
  uint32_t wb0 = 0, wb1 = 0, c0n = 0, c1n = 0;
  if (pass == 1) {
    if (ga < a.G) {
      wb0 = a.wave_base[ga * wstride + wave];
      c0n = a.wave_base[ga * wstride + wave + 1] - wb0;
    }
    if (gb < a.G) {
      wb1 = a.wave_base[gb * wstride + wave];
      c1n = a.wave_base[gb * wstride + wave + 1] - wb1;
    }
  }
  uint32_t o0 = c0n, o1 = c1n;               // inclusive, then exclusive offsets in the stage
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t x0 = __shfl_up(o0, d, 64), x1 = __shfl_up(o1, d, 64);
    if (lane >= d) {
      o0 += x0;
      o1 += x1;
    }
  }
  const uint32_t tot0 = __shfl(o0, 63, 64);
  o0 -= c0n;
  o1 += tot0 - c1n;
  const bool staged = pass == 1 && tot0 + __shfl(o1 + c1n, 63, 64) - tot0 <= (uint32_t)kRgStage;
  runs[ga] = pass == 1 ? (staged ? o0 : wb0) : 0u;
  runs[gb] = pass == 1 ? (staged ? o1 : wb1) : 0u;
  const uint32_t sh0 = staged ? wb0 - o0 : 0u, sh1 = staged ? wb1 - o1 : 0u;
  // bits of a group id: one ballot per bit gives every lane the lanes of its own group
  const int nbits = a.G > 1 ? 32 - __clz((unsigned)(a.G - 1)) : 0;
  int pj = 0;                      // (pass 1) rows whose run starts are not written yet: pj..
  auto write_starts = [&](int upto) {   // rows pj .. upto - 1 start at the current counts
    for (; pj < upto; ++pj) {
      if (ga < a.G) a.ptr[(int64_t)ga * (a.N + 1) + r0 + pj] = runs[ga] + sh0;
      if (gb < a.G) a.ptr[(int64_t)gb * (a.N + 1) + r0 + pj] = runs[gb] + sh1;
    }
  };
  Chunk c0 = settle(Chunk{0, start(0), start(1)});
  Chunk c1 = next(c0);
  int32_t id0, id1, g0, loc0;
  V n0, n1;
  load_ids(c0, id0, n0);
  load_ids(c1, id1, n1);
  load_group(id0, n0, g0, loc0);
  while (c0.j < R) {
    const Chunk c2 = next(c1);
    int32_t id2;
    V n2;
    load_ids(c2, id2, n2);                     // chunk k + 2
    int32_t g1, loc1;
    load_group(id1, n1, g1, loc1);             // chunk k + 1
    // chunk k: place (pass 1) / count its entries
    if (pass == 1) write_starts(c0.j + 1);
    const int64_t r = r0 + c0.j;
    const bool act = g0 >= 0;
    uint64_t same = __ballot(act);             // -> the lanes whose group is this lane's
    for (int b = 0; b < nbits; ++b) {
      const bool bit = (g0 >> b) & 1;
      const uint64_t mb = __ballot(act && bit);
      same &= bit ? mb : ~mb;
    }
    if (act) {
      const uint32_t rank = __popcll(same & lt);
      const uint32_t base = runs[g0];          // (every lane reads before the leaders write)
      if (pass == 1) {
        if (staged) {
          stage[base + rank] = (uint32_t)loc0 | ((uint32_t)c0.j << 16);
        } else {
          const int64_t pos = a.gbase[g0] + base + rank;
          a.ent[pos] = (uint16_t)loc0;
          if (a.erow != nullptr && g0 >= a.em_g0) a.erow[pos - a.ebase] = (uint32_t)r;
        }
      }
      if (rank == 0) runs[g0] = base + __popcll(same);
    }
    c0 = c1;
    g0 = g1;
    loc0 = loc1;
    c1 = c2;
    id1 = id2;
    n1 = n2;
  }
  if (pass == 0) {
    if (ga < a.G) a.wave_base[ga * wstride + wave] = runs[ga];            // the wave's totals
    if (gb < a.G) a.wave_base[gb * wstride + wave] = runs[gb];
  } else {
    write_starts(R);                                                      // (trailing empty rows)
    if (staged) {                  // each group's staged run to its place, coalesced
      __builtin_amdgcn_s_waitcnt(0xc07f);                                 // lgkmcnt(0)
      __builtin_amdgcn_wave_barrier();
      for (int g = 0; g < a.G; ++g) {
        const int src = g & 63;
        const uint32_t cnt = (uint32_t)__builtin_amdgcn_readlane((int)(g < 64 ? c0n : c1n), src);
        if (cnt == 0) continue;
        const uint32_t off = (uint32_t)__builtin_amdgcn_readlane((int)(g < 64 ? o0 : o1), src);
        const uint32_t wb = (uint32_t)__builtin_amdgcn_readlane((int)(g < 64 ? wb0 : wb1), src);
        const int64_t dst = a.gbase[g] + wb;
        const bool rows = a.erow != nullptr && g >= a.em_g0;
        for (uint32_t i = lane; i < cnt; i += 64) {
          const uint32_t v = stage[off + i];
          a.ent[dst + i] = (uint16_t)(v & 0xffffu);
          if (rows) a.erow[dst + i - a.ebase] = (uint32_t)(r0 + (v >> 16));
        }
      }
    }
    if (r0 + R == a.N) {                                                  // the groups' ends
      if (ga < a.G) a.ptr[(int64_t)ga * (a.N + 1) + a.N] = runs[ga] + sh0;
      if (gb < a.G) a.ptr[(int64_t)gb * (a.N + 1) + a.N] = runs[gb] + sh1;
    }
  }
}

template <class V>
__global__ __launch_bounds__(256) void rg_build_csr_count_kernel(RgCsrBuildArgs<V> a) {
  __shared__ uint32_t runs[4][128];
  rg_build_csr_wave<V, 0>(a, nullptr, runs[threadIdx.x >> 6]);
}

template <class V>
__global__ __launch_bounds__(256) void rg_build_csr_place_kernel(RgCsrBuildArgs<V> a) {
  __shared__ uint32_t stage[4][kRgStage];
  __shared__ uint32_t runs[4][128];
  rg_build_csr_wave<V, 1>(a, stage[threadIdx.x >> 6], runs[threadIdx.x >> 6]);
}

// Block g: group g's per-wave totals -> exclusive per-wave bases (in place), the group's total
// behind them. Tiles of 4096 consecutive waves, 4 per thread as one 16-byte load (the row stride
// is a multiple of 4): coalesced, one block scan per tile (a thread per contiguous 1/1024 of the
// waves read 4-byte words 2.4 KB apart: 1.6 ms at 10M rows).
__global__ __launch_bounds__(1024) void rg_build_scan_kernel(uint32_t* wave_base, int64_t nwaves, int32_t G) {
  __shared__ uint32_t s_sum[1024];
  const int g = blockIdx.x, t = threadIdx.x;
  uint32_t* wbg = wave_base + (int64_t)g * rg_build_stride(nwaves);   // group g's waves, then its total
  uint32_t carry = 0;
  for (int64_t base = 0; base < nwaves; base += 4096) {
    const int64_t w = base + 4 * (int64_t)t;
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (w + 3 < nwaves) {
      v = *reinterpret_cast<const uint4*>(wbg + w);
    } else {
      if (w < nwaves) v.x = wbg[w];
      if (w + 1 < nwaves) v.y = wbg[w + 1];
      if (w + 2 < nwaves) v.z = wbg[w + 2];
    }
    const uint32_t sum = v.x + v.y + v.z + v.w;
    s_sum[t] = sum;
    __syncthreads();
    for (int d = 1; d < 1024; d <<= 1) {
      const uint32_t o = t >= d ? s_sum[t - d] : 0u;
      __syncthreads();
      s_sum[t] += o;
      __syncthreads();
    }
    const uint32_t ex = carry + s_sum[t] - sum;
    const uint4 out = make_uint4(ex, ex + v.x, ex + v.x + v.y, ex + v.x + v.y + v.z);
    if (w + 3 < nwaves) {
      *reinterpret_cast<uint4*>(wbg + w) = out;
    } else {
      if (w < nwaves) wbg[w] = out.x;
      if (w + 1 < nwaves) wbg[w + 1] = out.y;
      if (w + 2 < nwaves) wbg[w + 2] = out.z;
    }
    carry += s_sum[1023];
    __syncthreads();                             // (s_sum is rewritten by the next tile)
  }
  if (t == 0) wbg[nwaves] = carry;
}

// One wave per rg_list_rows(N) consecutive rows (its row_node / slot loads issued 8 steps at a time), slots
// counted and placed with wave ballots (one ballot per distinct slot among each 64 rows). Pass 0
// stores the wave's per-slot counts; pass 2 (one block per slot) turns them into per-wave offsets
// inside the slot plus the slot totals; pass 1 derives the slot starts (a wave scan of the totals)
// and writes the wave's rows (and their digit words) in ascending order. No atomics: the list is
// sorted by (slot, row), and no counter is contended (one global counter per slot, added to by
// every wave, serialised ~39K atomics per level at 10M rows: ~1.4 ms).


__global__ __launch_bounds__(256) void rg_list_kernel(RgListArgs a, int pass) {
  const int64_t wave = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  const int32_t list_rows = a.list_rows, list_steps = list_rows / 64;
  const int64_t r0 = wave * list_rows;
  if (r0 >= a.N) return;
  const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  int32_t* wc = a.wave_count + wave * a.nslots;
  constexpr int KB = 8;                        // steps whose slot loads are in flight together
  uint32_t sl[KB];
  if (pass == 0) {
    int32_t cnt = 0;                           // lane s: rows of slot s
    for (int k0 = 0; k0 < list_steps; k0 += KB) {
#pragma unroll
      for (int k = 0; k < KB; ++k) {
        const int64_t r = r0 + 64 * (k0 + k) + lane;
        sl[k] = r < a.N ? rg_slot_of(a, r) : 0xffu;
      }
#pragma unroll
      for (int k = 0; k < KB; ++k) {
        uint64_t act = __ballot(sl[k] < (uint32_t)a.nslots);
        while (act) {
          const uint32_t s = __shfl(sl[k], __ffsll((unsigned long long)act) - 1, 64);
          const uint64_t m = __ballot(sl[k] == s);
          if ((uint32_t)lane == s) cnt += __popcll(m);
          act &= ~m;
        }
      }
    }
    if (lane < a.nslots) wc[lane] = cnt;
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
  // the wave's running position in each slot (lane s writes slot s's), read by every lane of the
  // slot: one ballot per slot-id bit finds a lane's slot mates (a ballot per distinct slot took up
  // to ~16 rounds per step at the deep levels)
  __shared__ int32_t s_base[4][64];
  int32_t* base = s_base[threadIdx.x >> 6];
  if (lane < a.nslots) base[lane] = incl - tot + wc[lane];
  __builtin_amdgcn_s_waitcnt(0xc07f);
  __builtin_amdgcn_wave_barrier();
  const int nbits = a.nslots > 1 ? 32 - __clz((unsigned)(a.nslots - 1)) : 0;
  for (int k0 = 0; k0 < list_steps; k0 += KB) {
    uint2 d[KB];
#pragma unroll
    for (int k = 0; k < KB; ++k) {
      const int64_t r = r0 + 64 * (k0 + k) + lane;
      sl[k] = r < a.N ? rg_slot_of(a, r) : 0xffu;
    }
#pragma unroll
    for (int k = 0; k < KB; ++k) {
      const int64_t r = r0 + 64 * (k0 + k) + lane;
      d[k] = (a.listdig && sl[k] < (uint32_t)a.nslots) ? *reinterpret_cast<const uint2*>(a.rowdig + 2 * r)
                                                         : make_uint2(0u, 0u);
    }
    if (a.masked) {                              // (nslots == 1: the listed rows are slot 0's)
#pragma unroll
      for (int k = 0; k < KB; ++k) {
        const int64_t r = r0 + 64 * (k0 + k) + lane;
        if (r < a.N) *reinterpret_cast<uint2*>(a.masked + 2 * r) = sl[k] == 0u ? d[k] : make_uint2(0u, 0u);
      }
    }
#pragma unroll
    for (int k = 0; k < KB; ++k) {
      const int64_t r = r0 + 64 * (k0 + k) + lane;
      const bool act = sl[k] < (uint32_t)a.nslots;
      uint64_t same = __ballot(act);
      for (int b = 0; b < nbits; ++b) {
        const bool bit = (sl[k] >> b) & 1u;
        const uint64_t mb = __ballot(act && bit);
        same &= bit ? mb : ~mb;
      }
      if (act) {
        const uint32_t rank = __popcll(same & lt);
        const int32_t b0 = base[sl[k]];          // (every lane reads before the leaders write)
        const int64_t pos = b0 + rank;
        a.list[pos] = (int32_t)r;
        if (a.listdig) *reinterpret_cast<uint2*>(a.listdig + 2 * pos) = d[k];
        if (rank == 0) base[sl[k]] = b0 + __popcll(same);
      }
      __builtin_amdgcn_s_waitcnt(0xc07f);
      __builtin_amdgcn_wave_barrier();
    }
  }
}

// Pass 2: block s scans slot s's per-wave counts into per-wave offsets (in place) and its total.
// With node_counts, a wave's count is the sum of its 512-row partition waves' counts of the node
// whose slot is s (that level's nodes *nc_base + i, i < 64).
__device__ __forceinline__ int32_t rg_node_wave_count(const RgListArgs& a, int node_i, int64_t w) {
  if (node_i < 0) return 0;
  const int64_t per = a.list_rows / kPartWaveRows, pw_end = (a.N + kPartWaveRows - 1) / kPartWaveRows;
  int32_t c = 0;
  const int32_t* nc = a.node_counts + (int64_t)node_i * pw_end;
  for (int64_t pw = w * per; pw < (w + 1) * per && pw < pw_end; ++pw) c += nc[pw];
  return c;
}

__global__ __launch_bounds__(1024) void rg_list_scan_kernel(RgListArgs a, int64_t nwaves) {
  __shared__ int32_t s_wsum[16];
  __shared__ int32_t s_node;
  const int s = blockIdx.x, t = threadIdx.x, lane = t & 63, wid = t >> 6;
  if (a.node_counts != nullptr) {
    if (t == 0) s_node = -1;
    __syncthreads();
    if (t < 64) {
      const int32_t node = *a.nc_base + t;
      if (node >= 0 && node < a.num_nodes && a.node_slot[node] == s) s_node = t;
    }
    __syncthreads();
  }
  const int node_i = a.node_counts != nullptr ? s_node : -1;
  auto count_of = [&](int64_t w) {
    return a.node_counts != nullptr ? rg_node_wave_count(a, node_i, w) : a.wave_count[w * a.nslots + s];
  };
  // thread t: waves [w0, w1), their counts kept in registers (up to 8 a thread: 16M rows at
  // 2048-row waves; beyond, read again)
  constexpr int kKeep = 8;
  const int64_t per = (nwaves + 1023) / 1024;
  const int64_t w0 = t * per, w1 = w0 + per < nwaves ? w0 + per : nwaves;
  int32_t keep[kKeep];
  int32_t sum = 0;
#pragma unroll
  for (int i = 0; i < kKeep; ++i) {
    keep[i] = w0 + i < w1 ? count_of(w0 + i) : 0;
    sum += keep[i];
  }
  for (int64_t w = w0 + kKeep; w < w1; ++w) sum += count_of(w);
  // block exclusive scan of the thread sums: wave scans, then a scan of the 16 wave totals
  int32_t incl = sum;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int32_t o = __shfl_up(incl, d, 64);
    if (lane >= d) incl += o;
  }
  if (lane == 63) s_wsum[wid] = incl;
  __syncthreads();
  if (wid == 0) {
    int32_t x = lane < 16 ? s_wsum[lane] : 0;
#pragma unroll
    for (int d = 1; d < 16; d <<= 1) {
      const int32_t o = __shfl_up(x, d, 64);
      if (lane >= d) x += o;
    }
    if (lane < 16) s_wsum[lane] = x;
  }
  __syncthreads();
  int32_t acc = incl - sum + (wid > 0 ? s_wsum[wid - 1] : 0);
#pragma unroll
  for (int i = 0; i < kKeep; ++i) {
    if (w0 + i < w1) {
      a.wave_count[(w0 + i) * a.nslots + s] = acc;
      acc += keep[i];
    }
  }
  for (int64_t w = w0 + kKeep; w < w1; ++w) {
    const int32_t c = count_of(w);
    a.wave_count[w * a.nslots + s] = acc;
    acc += c;
  }
  if (t == 0) a.slot_count[s] = s_wsum[15];
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

// (part) workgroup w's table of a single-slot pass, every bin, zeros included
template <int BINS>
__device__ __forceinline__ void rg_store_part(const RgHistArgs& a, RgShared<BINS>& sh, int tid, bool zero) {
  longlong2* dst = reinterpret_cast<longlong2*>(a.part) + (int64_t)blockIdx.x * BINS;
  for (int i = tid; i < BINS; i += kRgThreads) {
    dst[i] = zero ? make_longlong2(0, 0) : make_longlong2(sh.hg[i], sh.hh[i]);
    if (!zero) {
      sh.hg[i] = 0;
      sh.hh[i] = 0;
    }
  }
}

// whole: the workgroup's chunk lies inside slot s (its table may go to the partials)
template <int BINS>
__device__ __forceinline__ void rg_flush(const RgHistArgs& a, RgShared<BINS>& sh, int g, int s, int tid,
                                         bool whole = true) {
  if (a.part != nullptr && (a.nslots == 1 || whole)) {
    rg_store_part<BINS>(a, sh, tid, false);
    return;
  }
  const int64_t hrow = (a.dbg & 4) ? -1 : a.slot_node[s];          // dbg bit 2: no flush (timing)
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

// Dense groups: batches of 64 listed rows, block-balanced (rg_batch); the list entry is read two
// batches ahead, (ptr, digits) one batch ahead.
template <int BINS>
__device__ __forceinline__ void rg_range_dense(RgShared<BINS>& sh, const RgHistArgs& a, const uint32_t* ptr,
                                             const uint16_t* ent, const uint32_t* pdig, int64_t lo, int64_t hi,
                                             int wv, int lane, int np, int dbg, unsigned long long& sink) {
  const int32_t* list = a.list;
  int64_t pos = lo + wv * 64 + lane;
  int64_t row_c = list ? (pos < hi ? (int64_t)list[pos] : -1) : (pos < hi ? pos : -1);
  int64_t row_n = -1;
  if (list && pos + kRgThreads < hi) row_n = list[pos + kRgThreads];
  uint32_t st = 0, en = 0;
  uint2 dg = make_uint2(0u, 0u);
  if (row_c >= 0) {
    st = ptr[row_c];
    en = ptr[row_c + 1];
    dg = *reinterpret_cast<const uint2*>(pdig + 2 * pos);
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
      ndg = *reinterpret_cast<const uint2*>(pdig + 2 * pn);
    }
    rg_batch<BINS>(sh, ent, wv, lane, st, en, (int32_t)rg_q(dg.x, np), (int32_t)rg_q(dg.y, np), dbg, sink);
    st = nst;
    en = nen;
    dg = ndg;
  }
}

// Sparse groups (~2 entries per row): the per-batch work (~16 atomics per lane) is far shorter
// than a memory round trip, and a lane per row, a lane-balanced batch and an entry-granular batch
// all ran at ~1.1 ms for the 205M sparse entries of the root pass (bench/probes/rg_probe.py,
// profiles/r3s2): each batch waited ~one HBM latency. So a wave walks its rows in super-batches
// of kRgSB batches (a lane per row) through a 3-stage pipeline -- list entries of super-batch
// j + 3, (ptr, digits) of j + 2, the rows' first 8-entry blocks of j + 1 -- while the atomics of
// super-batch j run: every load has a whole super-batch of work to arrive in.
// (3 spilled 48 B per lane of rg_hist_kernel<8192> and fit 10M rows in 0.5098 s against 0.5015 s
// with 2, same trees: profiles/r6/gbdt_late/NOTES.md §14)
constexpr int kRgSB = 2;

template <int BINS>
__device__ __forceinline__ void rg_run_block(RgShared<BINS>& sh, uint4 v, uint32_t blk, uint32_t st, uint32_t en,
                                             unsigned long long c0, unsigned long long c1, uint32_t sinkb, int dbg,
                                             unsigned long long& sink) {
  const uint32_t wd[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const uint32_t i = blk + k;
    const uint32_t bin = (wd[k >> 1] >> (16 * (k & 1))) & 0xffffu;
    const uint32_t b = (i >= st && i < en) ? bin : sinkb;
    if (dbg & 2) {
      sink += b;
    } else {
      atomicAdd(reinterpret_cast<unsigned long long*>(&sh.hg[b]), c0);
      atomicAdd(reinterpret_cast<unsigned long long*>(&sh.hh[b]), c1);
    }
  }
}

template <int BINS>
__device__ __forceinline__ void rg_range_sparse(RgShared<BINS>& sh, const RgHistArgs& a, const uint32_t* ptr,
                                                const uint16_t* ent, const uint32_t* pdig, int64_t lo, int64_t hi,
                                                int wv, int lane, int np, int dbg, unsigned long long& sink) {
  const int32_t* list = a.list;
  const int64_t p0 = lo + wv * 64 + lane;
  constexpr int64_t kSBStride = (int64_t)kRgSB * kRgThreads;      // positions per super-batch
  const uint32_t sinkb = BINS + lane;
  auto pos_of = [&](int64_t j, int i) -> int64_t { return p0 + j * kSBStride + (int64_t)i * kRgThreads; };
  auto rows_of = [&](int64_t j, int32_t* r) {
#pragma unroll
    for (int i = 0; i < kRgSB; ++i) {
      const int64_t p = pos_of(j, i);
      r[i] = p < hi ? (list ? list[p] : (int32_t)p) : -1;
    }
  };
  auto info_of = [&](int64_t j, const int32_t* r, uint32_t* st, uint32_t* en, uint2* dg) {
#pragma unroll
    for (int i = 0; i < kRgSB; ++i) {
      st[i] = en[i] = 0u;
      dg[i] = make_uint2(0u, 0u);
      if (r[i] >= 0) {
        st[i] = ptr[r[i]];
        en[i] = ptr[r[i] + 1];
        dg[i] = *reinterpret_cast<const uint2*>(pdig + 2 * pos_of(j, i));
      }
    }
  };
  auto blocks_of = [&](const uint32_t* st, const uint32_t* en, uint4* v) {
#pragma unroll
    for (int i = 0; i < kRgSB; ++i)
      v[i] = en[i] > st[i] ? *reinterpret_cast<const uint4*>(ent + (st[i] & ~7u)) : make_uint4(0u, 0u, 0u, 0u);
  };
  if (p0 - lane >= hi) return;
  // prologue: super-batch 0 through stage 3, 1 through stage 2, 2 through stage 1
  int32_t r0[kRgSB], r1[kRgSB], r2[kRgSB];
  uint32_t st0[kRgSB], en0[kRgSB], st1[kRgSB], en1[kRgSB];
  uint2 dg0[kRgSB], dg1[kRgSB];
  uint4 v0[kRgSB];
  rows_of(0, r0);
  rows_of(1, r1);
  rows_of(2, r2);
  info_of(0, r0, st0, en0, dg0);
  info_of(1, r1, st1, en1, dg1);
  blocks_of(st0, en0, v0);
  for (int64_t j = 0; pos_of(j, 0) - lane < hi; ++j) {
    int32_t r3[kRgSB];
    uint32_t st2[kRgSB], en2[kRgSB];
    uint2 dg2[kRgSB];
    uint4 v1[kRgSB];
    rows_of(j + 3, r3);
    info_of(j + 2, r2, st2, en2, dg2);
    blocks_of(st1, en1, v1);
#pragma unroll
    for (int i = 0; i < kRgSB; ++i) {
      if (en0[i] > st0[i]) {
        const unsigned long long c0 = (unsigned long long)rg_q(dg0[i].x, np);
        const unsigned long long c1 = (unsigned long long)rg_q(dg0[i].y, np);
        uint32_t blk = st0[i] & ~7u;
        rg_run_block<BINS>(sh, v0[i], blk, st0[i], en0[i], c0, c1, sinkb, dbg, sink);
        for (blk += 8; blk < en0[i]; blk += 8)        // rows longer than one block (rare here)
          rg_run_block<BINS>(sh, *reinterpret_cast<const uint4*>(ent + blk), blk, st0[i], en0[i], c0, c1, sinkb,
                             dbg, sink);
      }
    }
#pragma unroll
    for (int i = 0; i < kRgSB; ++i) {
      st0[i] = st1[i];
      en0[i] = en1[i];
      dg0[i] = dg1[i];
      v0[i] = v1[i];
      st1[i] = st2[i];
      en1[i] = en2[i];
      dg1[i] = dg2[i];
      r2[i] = r3[i];
    }
  }
}

// Entry-major pass of a sparse group at a single-slot level (tree.h rg_use_em). The row-list pass
// spends a lane per row on ~2 entries: its 16 LDS atomics per 64 rows (times the longest row's
// blocks) were ~55M of the root pass's 88M LDS instructions for 21% of its entries, and the pass
// is LDS-issue bound (~14 CU-cycles per random ds_add_u64, bench/probes/lds_atomic_probe.hip).
// Here a lane takes one entry: (local bin, row) from ent / erow, the row's digit word (rows of
// consecutive entries are consecutive: coalesced), two atomics -- 2 LDS instructions per 64
// entries. A wave streams kRgEmU entries per lane per step through a 3-stage pipeline: (bin, row)
// of step j + 2 and the digit words of step j + 1 are in flight while step j's atomics run.
constexpr int kRgEmU = 8;
constexpr uint32_t kRgNoRow = 0xffffffffu;

template <int BINS>
__device__ __forceinline__ void rg_range_em(RgShared<BINS>& sh, const RgHistArgs& a, const uint16_t* ent,
                                            const uint32_t* erow, int64_t lo, int64_t hi, int wv, int lane, int np,
                                            int dbg, unsigned long long& sink) {
  constexpr int64_t kStride = (int64_t)kRgThreads * kRgEmU;
  auto load_entries = [&](int64_t base, uint32_t* r, uint32_t* b) {
#pragma unroll
    for (int u = 0; u < kRgEmU; ++u) {
      const int64_t e = base + u * 64 + lane;
      r[u] = e < hi ? erow[e] : kRgNoRow;
      b[u] = e < hi ? (uint32_t)ent[e] : 0u;
    }
  };
  const uint32_t* dig = rg_em_digits(a);          // (a listed level: zero outside slot 0)
  auto load_digits = [&](uint32_t* r, uint2* d) {
#pragma unroll
    for (int u = 0; u < kRgEmU; ++u)
      d[u] = r[u] != kRgNoRow ? *reinterpret_cast<const uint2*>(dig + 2 * (int64_t)r[u]) : make_uint2(0u, 0u);
  };
  int64_t base = lo + (int64_t)wv * 64 * kRgEmU;
  if (base >= hi) return;
  uint32_t r0[kRgEmU], b0[kRgEmU], r1[kRgEmU], b1[kRgEmU];
  uint2 d0[kRgEmU];
  load_entries(base, r0, b0);
  load_entries(base + kStride, r1, b1);
  load_digits(r0, d0);
  for (; base < hi; base += kStride) {
    uint32_t r2[kRgEmU], b2[kRgEmU];
    uint2 d1[kRgEmU];
    load_entries(base + 2 * kStride, r2, b2);
    load_digits(r1, d1);
#pragma unroll
    for (int u = 0; u < kRgEmU; ++u) {
      if (r0[u] == kRgNoRow || (d0[u].x | d0[u].y) == 0u) continue;
      if (dbg & 2) {
        sink += b0[u];
      } else {
        atomicAdd(reinterpret_cast<unsigned long long*>(&sh.hg[b0[u]]), (unsigned long long)rg_q(d0[u].x, np));
        atomicAdd(reinterpret_cast<unsigned long long*>(&sh.hh[b0[u]]), (unsigned long long)rg_q(d0[u].y, np));
      }
    }
#pragma unroll
    for (int u = 0; u < kRgEmU; ++u) {
      r0[u] = r1[u];
      b0[u] = b1[u];
      d0[u] = d1[u];
      r1[u] = r2[u];
      b1[u] = b2[u];
    }
  }
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
  if (a.root_parts != nullptr && w == 0 && (int)threadIdx.x < a.nshards) {   // (the DP root's totals row)
    int64_t t0, t1;
    root_sums(a.root_parts, &t0, &t1);
    int64_t* dst = a.hist + ((int64_t)threadIdx.x * a.shard_stride + (int64_t)a.nslots * a.hist_stride) * 2;
    dst[0] = t0;
    dst[1] = t1;
  }
  const int g = a.wg_g[w], p = a.wg_p[w], np_g = a.wg_np[w];
  const int64_t T = a.list ? (int64_t)a.slot_start[a.nslots] : a.N;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  if (T > 0 && rg_use_em(a, g, T)) {            // chunk p of the group's entries instead
    const int64_t E = a.ptr[(int64_t)g * (a.N + 1) + a.N];
    const int64_t e0 = E * p / np_g, e1 = E * (p + 1) / np_g;
    if (e0 >= e1) {
      if (a.part != nullptr) rg_store_part<BINS>(a, sh, tid, true);
      return;
    }
    for (int i = tid; i < BINS; i += kRgThreads) {
      sh.hg[i] = 0;
      sh.hh[i] = 0;
    }
    __syncthreads();
    unsigned long long sink = 0;
    rg_range_em<BINS>(sh, a, a.ent + a.gbase[g], a.erow + (a.gbase[g] - a.ebase), e0, e1, wv, lane, a.np, a.dbg,
                      sink);
    if (a.dbg & 2) atomicAdd(reinterpret_cast<unsigned long long*>(&sh.hg[lane]), sink);
    __syncthreads();
    rg_flush<BINS>(a, sh, g, 0, tid);
    return;
  }
  const int64_t a0 = T * p / np_g, a1 = T * (p + 1) / np_g;
  if (a0 >= a1) {                    // (several slots: the reduction skips an empty chunk itself)
    if (a.part != nullptr && a.nslots == 1) rg_store_part<BINS>(a, sh, tid, true);
    return;
  }
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
  // digit words by list position (coalesced): listdig with a list, rowdig at the all-rows pass
  const uint32_t* pdig = list ? a.listdig : a.rowdig;
  const bool bal = a.gmode[g] != 0;
  const int np = a.np, dbg = a.dbg;
  unsigned long long sink = 0;
  for (;;) {
    const int64_t ss0 = list ? (int64_t)a.slot_start[s] : 0;
    const int64_t ss1 = list ? (int64_t)a.slot_start[s + 1] : a.N;
    const int64_t lo = a0 > ss0 ? a0 : ss0, hi = a1 < ss1 ? a1 : ss1;
    if (bal)
      rg_range_dense<BINS>(sh, a, ptr, ent, pdig, lo, hi, wv, lane, np, dbg, sink);
    else
      rg_range_sparse<BINS>(sh, a, ptr, ent, pdig, lo, hi, wv, lane, np, dbg, sink);
    if (dbg & 2) atomicAdd(reinterpret_cast<unsigned long long*>(&sh.hg[lane]), sink);
    __syncthreads();
    rg_flush<BINS>(a, sh, g, s, tid, a0 >= ss0 && a1 <= ss1);
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

template <class V>
void launch_rg_build_csr(const RgCsrBuildArgs<V>& a, hipStream_t s) {
  const int64_t waves = rg_build_waves(a.N);
  const int64_t blocks = (waves + 3) / 4;
  if (blocks <= 0) return;
  hipLaunchKernelGGL(rg_build_csr_count_kernel<V>, dim3((unsigned)blocks), dim3(256), 0, s, a);
  hipLaunchKernelGGL(rg_build_scan_kernel, dim3((unsigned)a.G), dim3(1024), 0, s, a.wave_base, waves, a.G);
  hipLaunchKernelGGL(rg_build_csr_place_kernel<V>, dim3((unsigned)blocks), dim3(256), 0, s, a);
}
int64_t rg_build_csr_waves(int64_t N) { return rg_build_stride(rg_build_waves(N)); }   // (per group)
template void launch_rg_build_csr<float>(const RgCsrBuildArgs<float>&, hipStream_t);
template void launch_rg_build_csr<double>(const RgCsrBuildArgs<double>&, hipStream_t);
template void launch_rg_build_csr<int32_t>(const RgCsrBuildArgs<int32_t>&, hipStream_t);

void launch_rg_list(const RgListArgs& a0, hipStream_t s) {
  RgListArgs a = a0;
  a.list_rows = rg_list_rows(a.N);
  const int64_t waves = (a.N + a.list_rows - 1) / a.list_rows;   // 4 per block
  const int64_t blocks = (waves + 3) / 4;
  if (blocks <= 0) return;
  if (a.node_counts != nullptr && (a.row_node == nullptr || a.list_rows % kPartWaveRows != 0)) a.node_counts = nullptr;
  if (!a.counted && a.node_counts == nullptr) hipLaunchKernelGGL(rg_list_kernel, dim3((unsigned)blocks), dim3(256), 0, s, a, 0);
  hipLaunchKernelGGL(rg_list_scan_kernel, dim3((unsigned)a.nslots), dim3(1024), 0, s, a, waves);
  hipLaunchKernelGGL(rg_list_kernel, dim3((unsigned)blocks), dim3(256), 0, s, a, 1);
}

namespace {
// Thread per (row, group from g0 on): writes the row's index over its run of the group.
__global__ __launch_bounds__(256) void rg_erow_kernel(RgErowArgs a) {
  const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (r >= a.N) return;
  const int g = a.g0 + (int)blockIdx.y;
  const uint32_t* ptr = a.ptr + (int64_t)g * (a.N + 1);
  uint32_t* out = a.erow + (a.gbase[g] - a.ebase);
  for (uint32_t e = ptr[r]; e < ptr[r + 1]; ++e) out[e] = (uint32_t)r;
}
}  // namespace

void launch_rg_erow(const RgErowArgs& a, hipStream_t s) {
  if (a.N <= 0 || a.g0 >= a.G) return;
  hipLaunchKernelGGL(rg_erow_kernel, dim3((unsigned)((a.N + 255) / 256), (unsigned)(a.G - a.g0)), dim3(256), 0, s, a);
}

namespace {
// The single-slot pass's partial tables summed per group into the level histogram: a thread per
// (group, local bin, run of kRedRun workgroups), the run's tables read kRedU at a time (coalesced
// over the bins; one thread walking the dense group's ~200 tables serially took ~32 us).
// Several slots: the run's workgroups that stored a table (rg_part_slot >= 0) are summed per slot
// (a group's chunks follow the list order, so a slot's tables are consecutive) and each slot's sum
// is added to its node's row.
constexpr int kRedRun = 32, kRedU = 8;
__device__ __forceinline__ void rg_reduce_add(const RgHistArgs& a, int slot, int32_t col, int64_t s0, int64_t s1) {
  const int64_t hrow = slot >= 0 ? a.slot_node[slot] : -1;
  if ((s0 | s1) == 0 || hrow < 0) return;
  int64_t* dst = a.hist + (hrow * a.hist_stride + rg_col_offset(a, col)) * 2;
  atomicAdd(reinterpret_cast<unsigned long long*>(dst), (unsigned long long)s0);
  atomicAdd(reinterpret_cast<unsigned long long*>(dst + 1), (unsigned long long)s1);
}

__global__ __launch_bounds__(256) void rg_reduce_kernel(RgHistArgs a) {
  __shared__ int32_t wslot[kRedRun];
  const int g = blockIdx.y;
  const int i = blockIdx.x * 256 + threadIdx.x;
  const int w0 = a.wg_first[g] + (int)blockIdx.z * kRedRun, w1 = min(w0 + kRedRun, a.wg_first[g + 1]);
  if (w0 >= w1) return;                                   // (uniform over the block)
  if (threadIdx.x < w1 - w0) {
    const int64_t T = a.list ? (int64_t)a.slot_start[a.nslots] : a.N;
    wslot[threadIdx.x] = a.nslots == 1 ? 0 : rg_part_slot(a, w0 + (int)threadIdx.x, T);
  }
  __syncthreads();
  if (i >= a.gbins) return;
  const int32_t col = a.gbin[(int64_t)g * a.gbins + i];
  if (col < 0) return;
  const longlong2* part = reinterpret_cast<const longlong2*>(a.part);
  int64_t s0 = 0, s1 = 0;
  int cur = -1;
  for (int w = w0; w < w1; w += kRedU) {
    longlong2 v[kRedU];
#pragma unroll
    for (int u = 0; u < kRedU; ++u)
      v[u] = (w + u < w1 && wslot[w + u - w0] >= 0) ? part[(int64_t)(w + u) * a.gbins + i] : make_longlong2(0, 0);
#pragma unroll
    for (int u = 0; u < kRedU; ++u) {
      const int ws = w + u < w1 ? wslot[w + u - w0] : -1;
      if (ws < 0) continue;
      if (ws != cur) {
        rg_reduce_add(a, cur, col, s0, s1);
        cur = ws;
        s0 = s1 = 0;
      }
      s0 += v[u].x;
      s1 += v[u].y;
    }
  }
  rg_reduce_add(a, cur, col, s0, s1);
}

}  // namespace

void launch_rg_hist(const RgHistArgs& a, hipStream_t s) {
  const int64_t blocks = a.n_wg;
  if (blocks <= 0) return;
  if (a.gbins == 4096)
    hipLaunchKernelGGL(rg_hist_kernel<4096>, dim3((unsigned)blocks), dim3(kRgThreads), 0, s, a);
  else
    hipLaunchKernelGGL(rg_hist_kernel<8192>, dim3((unsigned)blocks), dim3(kRgThreads), 0, s, a);
  if (a.part != nullptr && !(a.dbg & 4))
    hipLaunchKernelGGL(rg_reduce_kernel, dim3((unsigned)((a.gbins + 255) / 256), (unsigned)a.G,
                                              (unsigned)((a.n_wg + kRedRun - 1) / kRedRun)), dim3(256), 0, s, a);
}

}  // namespace fdx

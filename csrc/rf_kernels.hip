// Random-forest per-level feature sampling on the device (X-10, K-14).
//
// Spark samples exactly k = ceil(sqrt(F)) feature indices per node without replacement
// (/root/reference/fraud_detection_spark.py:67-74). Node n keeps the k indices with the smallest
// counter-based priority u53(seed, tree, n, fid) (csrc/tree.h), so its sample is defined by the
// k-th smallest priority. rf_threshold_kernel finds it exactly with one workgroup per node: radix
// passes of 12 bits build LDS histograms of the priorities that still match the selected prefix
// (priorities are recomputed, never stored), until the k-th element's bucket holds <= CAP
// candidates; those are gathered into LDS and ranked exactly. With F = 2^18 one pass leaves ~64
// candidates. rf_mask_kernel then marks the active features any node of the level samples (the
// histogram work items of unsampled features are skipped). One launch pair per tree level
// replaces ~40 small torch launches per node.
#include "ops.h"
#include "tree.h"

namespace fdx {

namespace {
constexpr int kThreads = 256;
constexpr int kRadixBits = 12;
constexpr int kBuckets = 1 << kRadixBits;
constexpr int kCap = 2048;

constexpr int kSlices = 64;       // workgroups per node of the window scan

__device__ __forceinline__ uint64_t rf_priority(const RfSampleArgs& a, int32_t tree, int32_t node, int64_t f) {
  return a.fmix ? feature_priority_u53_pre(a.seed, tree, node, a.fmix[f]) : feature_priority_u53(a.seed, tree, node, f);
}

// Fast path, pass 1: every priority below the window [ulo, uhi] is counted, those inside are
// appended to the node's candidate list. The window holds the k-th smallest with probability
// 1 - 1e-15 (+-8 sigma of the binomial count around k); rf_select_kernel checks it and falls back
// to the exact radix search otherwise.
__global__ __launch_bounds__(kThreads) void rf_window_kernel(RfSampleArgs a, uint64_t ulo, uint64_t uhi,
                                                             unsigned int* below, unsigned int* ncand,
                                                             uint64_t* cand) {
  __shared__ unsigned int s_below;
  const int i = blockIdx.y;
  const int node = a.nodes[i];
  if (node < 0) return;                           // padding of a capacity-sized open list
  if (threadIdx.x == 0) s_below = 0;
  __syncthreads();
  unsigned int mine = 0;
  for (int64_t f = (int64_t)blockIdx.x * kThreads + threadIdx.x; f < a.F; f += (int64_t)gridDim.x * kThreads) {
    const uint64_t u = rf_priority(a, rf_tree_of(a, i), node, f);
    if (u < ulo) {
      ++mine;
    } else if (u <= uhi) {
      const unsigned int j = atomicAdd(&ncand[i], 1u);
      if (j < (unsigned int)kCap) cand[(int64_t)i * kCap + j] = u;
    }
  }
  atomicAdd(&s_below, mine);
  __syncthreads();
  if (threadIdx.x == 0 && s_below) atomicAdd(&below[i], s_below);
}

// Node bi's threshold (its k-th smallest priority), by the calling workgroup: from the window
// pass's candidates when the window holds the k-th (below / ncand / cand non-null), else by the
// exact radix search. Workgroup-uniform control flow (barriers inside).
__device__ void rf_threshold_node(const RfSampleArgs& a, int bi, const unsigned int* below,
                                  const unsigned int* ncand, const uint64_t* cand) {
  __shared__ uint32_t s_hist[kBuckets];
  __shared__ uint64_t s_cand[kCap];
  __shared__ uint32_t s_ncand;
  __shared__ uint64_t s_prefix;
  __shared__ int s_known;
  __shared__ int64_t s_k;
  __shared__ int64_t s_count;

  const int node = a.nodes[bi];
  const int tid = threadIdx.x;
  if (node < 0) {                                 // padding: samples nothing
    if (tid == 0) a.thr[bi] = -1.0;
    return;
  }
  if (below != nullptr) {
    const int64_t r = a.k - (int64_t)below[bi];     // rank of the k-th inside the window
    const int n = (int)ncand[bi];
    if (r >= 1 && r <= n && n <= kCap) {
      // the window's candidates sorted in LDS (bitonic, padded to a power of two with the largest
      // value): the r-th smallest is then s_cand[r - 1] -- ~45 barrier steps for ~400 candidates
      // instead of an all-pairs rank (n^2 LDS reads per node, the larger part of this kernel)
      int m = 1;
      while (m < n) m <<= 1;
      for (int j = tid; j < m; j += kThreads) s_cand[j] = j < n ? cand[(int64_t)bi * kCap + j] : ~0ull;
      __syncthreads();
      for (int size = 2; size <= m; size <<= 1)
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
          for (int i = tid; i < (m >> 1); i += kThreads) {
            const int lo = 2 * i - (i & (stride - 1)), hi = lo + stride;
            const uint64_t x = s_cand[lo], y = s_cand[hi];
            if ((x > y) == ((lo & size) == 0)) {
              s_cand[lo] = y;
              s_cand[hi] = x;
            }
          }
          __syncthreads();
        }
      if (tid == 0) a.thr[bi] = (double)s_cand[r - 1] * (1.0 / 9007199254740992.0);
      return;                  // uniform per workgroup: every thread took this branch
    }
  }
  if (tid == 0) {
    s_prefix = 0;
    s_known = 0;
    s_k = a.k;                // 1-based rank of the wanted priority among those matching the prefix
    s_count = a.F;
  }
  __syncthreads();
  // radix passes until the wanted bucket is small enough to rank in LDS
  while (s_count > kCap && s_known < 53) {
    const int known = s_known;
    const uint64_t prefix = s_prefix;
    const int nbits = min(kRadixBits, 53 - known);
    const int shift = 53 - known - nbits;
    for (int i = tid; i < kBuckets; i += kThreads) s_hist[i] = 0;
    __syncthreads();
    for (int64_t f = tid; f < a.F; f += kThreads) {
      const uint64_t u = rf_priority(a, rf_tree_of(a, bi), node, f);
      if (known == 0 || (u >> (53 - known)) == prefix)
        atomicAdd(&s_hist[(u >> shift) & ((1u << nbits) - 1)], 1u);
    }
    __syncthreads();
    if (tid == 0) {
      int64_t k = s_k, cum = 0;
      int b = 0;
      for (; b < (1 << nbits); ++b) {
        if (cum + (int64_t)s_hist[b] >= k) break;
        cum += s_hist[b];
      }
      s_k = k - cum;
      s_count = s_hist[b];
      s_prefix = (prefix << nbits) | (uint64_t)b;
      s_known = known + nbits;
    }
    __syncthreads();
  }
  // gather the candidates of the selected prefix and rank them exactly
  if (tid == 0) s_ncand = 0;
  __syncthreads();
  const int known = s_known;
  const uint64_t prefix = s_prefix;
  for (int64_t f = tid; f < a.F; f += kThreads) {
    const uint64_t u = rf_priority(a, rf_tree_of(a, bi), node, f);
    if (known == 0 || (u >> (53 - known)) == prefix) {
      const uint32_t i = atomicAdd(&s_ncand, 1u);
      if (i < (uint32_t)kCap) s_cand[i] = u;
    }
  }
  __syncthreads();
  const int n = (int)min(s_ncand, (uint32_t)kCap);
  const int64_t k = s_k;
  for (int i = tid; i < n; i += kThreads) {
    const uint64_t ui = s_cand[i];
    int64_t less = 0, eq = 0;
    for (int j = 0; j < n; ++j) {
      less += s_cand[j] < ui;
      eq += s_cand[j] == ui;
    }
    if (less < k && k <= less + eq)    // ties: every holder of the k-th value writes the same result
      a.thr[bi] = (double)ui * (1.0 / 9007199254740992.0);
  }
}

__global__ __launch_bounds__(kThreads) void rf_threshold_kernel(RfSampleArgs a, const unsigned int* below,
                                                                const unsigned int* ncand, const uint64_t* cand) {
  rf_threshold_node(a, blockIdx.x, below, ncand, cand);
}

// Window pass + threshold in one launch (RfSampleArgs fused_counts): the window kernel's body,
// then per node a ticket; the node's last workgroup (one device-scope release per workgroup, see
// tree_kernels.hip last_workgroup) ranks the candidates and zeroes the node's counters for the
// next launch -- no memset and no second launch per level.
__device__ __forceinline__ void rf_window_threshold_kernel_body(RfSampleArgs a, uint64_t ulo, uint64_t uhi,
                                                                       uint64_t* cand) {
  __shared__ unsigned int s_below;
  __shared__ int s_last;
  const int i = blockIdx.y;
  const int node = a.nodes[i];
  unsigned int* ticket = a.fused_counts;
  unsigned int* below = a.fused_counts + a.fused_cap;
  unsigned int* ncand = a.fused_counts + 2 * a.fused_cap;
  if (node < 0) {                                 // padding: samples nothing (uniform per node)
    if (blockIdx.x == 0 && threadIdx.x == 0) a.thr[i] = -1.0;
    return;
  }
  if (threadIdx.x == 0) s_below = 0;
  __syncthreads();
  unsigned int mine = 0;
  for (int64_t f = (int64_t)blockIdx.x * kThreads + threadIdx.x; f < a.F; f += (int64_t)gridDim.x * kThreads) {
    const uint64_t u = rf_priority(a, rf_tree_of(a, i), node, f);
    if (u < ulo) {
      ++mine;
    } else if (u <= uhi) {
      const unsigned int j = atomicAdd(&ncand[i], 1u);
      if (j < (unsigned int)kCap) cand[(int64_t)i * kCap + j] = u;
    }
  }
  atomicAdd(&s_below, mine);
  __syncthreads();
  if (threadIdx.x == 0) {
    if (s_below) atomicAdd(&below[i], s_below);
    __threadfence();
    const unsigned int t = atomicAdd(&ticket[i], 1u);
    s_last = t == gridDim.x - 1 ? 1 : 0;
  }
  __syncthreads();
  if (!s_last) return;
  __threadfence();
  rf_threshold_node(a, i, below, ncand, cand);
  __syncthreads();
  if (threadIdx.x == 0) {
    below[i] = 0;
    ncand[i] = 0;
    ticket[i] = 0;
  }
}
__global__ __launch_bounds__(kThreads) void rf_window_threshold_kernel(RfSampleArgs a, uint64_t ulo, uint64_t uhi,
                                                                       uint64_t* cand) { rf_window_threshold_kernel_body(a, ulo, uhi, cand); }

__device__ __forceinline__ void rf_mask_kernel_body(RfSampleArgs a) {
  const int64_t f = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (f >= a.Fa) return;
  const int64_t fid = a.fid_orig[f];
  uint8_t m = 0;
  for (int i = 0; i < a.nnodes && !m; ++i) {
    if (a.nodes[i] < 0) continue;
    const uint64_t u = rf_priority(a, rf_tree_of(a, i), a.nodes[i], fid);
    m = ((double)u * (1.0 / 9007199254740992.0) <= a.thr[i]) ? 1 : 0;
  }
  a.mask[f] = m;
}
__global__ __launch_bounds__(kThreads) void rf_mask_kernel(RfSampleArgs a) { rf_mask_kernel_body(a); }

// lane-batched forms (tree.h "lane-batched launches"): lane l = blockIdx.z
__global__ __launch_bounds__(kThreads) void rf_window_threshold_lanes_kernel(const RfSampleArgs* __restrict__ args,
                                                                             uint64_t ulo, uint64_t uhi) {
  const RfSampleArgs a = args[blockIdx.z];
  if ((int)blockIdx.y >= a.nnodes) return;
  uint64_t* cand = reinterpret_cast<uint64_t*>(a.scratch + 8 * ((2 * a.nnodes * 4 + 7) / 8));
  rf_window_threshold_kernel_body(a, ulo, uhi, cand);
}

__global__ __launch_bounds__(kThreads) void rf_mask_lanes_kernel(const RfSampleArgs* __restrict__ args) {
  rf_mask_kernel_body(args[blockIdx.z]);
}
}  // namespace

namespace {
// One workgroup, shards one after another: each thread sums a contiguous slice of the shard's
// masked nbins, a block scan of the 1024 partials gives every slice its start, a second pass
// writes the offsets (unsampled features: the shard's trash start, known after the scan).
constexpr int kCompactThreads = 1024;
__global__ __launch_bounds__(kCompactThreads) void rf_compact_kernel(RfCompactArgs a) {
  __shared__ int64_t part[kCompactThreads];
  const int t = threadIdx.x;
  for (int32_t sh = 0; sh < a.S; ++sh) {
    const int64_t f0 = a.fs[sh], n = a.fs[sh + 1] - f0;
    const int64_t per = (n + kCompactThreads - 1) / kCompactThreads;
    const int64_t lo = f0 + per * t, hi = lo + per < f0 + n ? lo + per : f0 + n;
    int64_t sum = 0;
    for (int64_t f = lo; f < hi; ++f) sum += a.mask[f] ? a.nbins[f] : 0;
    part[t] = sum;
    __syncthreads();
    for (int d = 1; d < kCompactThreads; d <<= 1) {          // inclusive Hillis-Steele scan
      const int64_t o = t >= d ? part[t - d] : 0;
      __syncthreads();
      part[t] += o;
      __syncthreads();
    }
    const int64_t total = part[kCompactThreads - 1];
    int64_t acc = part[t] - sum;
    for (int64_t f = lo; f < hi; ++f) {
      if (a.mask[f]) { a.local[f] = acc; acc += a.nbins[f]; }
      else a.local[f] = total;
    }
    if (t == 0) a.sizes[sh] = total;
    __syncthreads();
  }
  if (t == 0) a.local[a.Fa] = 0;
}

// Multi-workgroup layout (chunk_sums given): shard s's features in chunks of kChunkFeat, workgroup
// (c, s) on chunk c. Pass 0 sums the chunk's masked nbins; pass 1 takes its start from the sums of
// the shard's earlier chunks, scans the chunk (8 consecutive features per thread, a wave scan and
// the 4 wave totals) and writes the offsets, the shard's total as the trash start of unsampled
// features. The single-workgroup kernel above walked ~90K features in one block: ~42 us a level,
// on every tree-level of a data-parallel forest (profiles/r5/NOTES.md).
constexpr int kChunkThreads = 256, kChunkPer = 8, kChunkFeat = kChunkThreads * kChunkPer;

__device__ __forceinline__ int64_t chunk_wave_incl(int64_t v, int lane) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int64_t o = __shfl_up(v, d, 64);
    if (lane >= d) v += o;
  }
  return v;
}

__device__ __forceinline__ void rf_compact_chunks_kernel_body(RfCompactArgs a, int pass) {
  const int sh = blockIdx.y, c = blockIdx.x, t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int64_t f0 = a.fs[sh], f1 = a.fs[sh + 1];
  const int64_t lo = f0 + (int64_t)c * kChunkFeat;
  const int64_t nchunks = (f1 - f0 + kChunkFeat - 1) / kChunkFeat;
  if (lo >= f1 && !(pass == 1 && c == 0)) return;
  const int64_t base = lo + (int64_t)t * kChunkPer;
  int64_t v[kChunkPer];
  int64_t sum = 0;
#pragma unroll
  for (int j = 0; j < kChunkPer; ++j) {
    const int64_t f = base + j;
    v[j] = (f < f1 && a.mask[f]) ? (int64_t)a.nbins[f] : 0;
    sum += v[j];
  }
  __shared__ int64_t s_w[4];
  __shared__ int64_t s_start, s_total;
  const int64_t incl = chunk_wave_incl(sum, lane);
  if (lane == 63) s_w[w] = incl;
  if (pass == 1 && t == 0) {
    int64_t before = 0, total = 0;
    for (int64_t k = 0; k < nchunks; ++k) {
      const int64_t cs = a.chunk_sums[(int64_t)sh * a.chunk_stride + k];
      if (k < c) before += cs;
      total += cs;
    }
    s_start = before;
    s_total = total;
  }
  __syncthreads();
  if (pass == 0) {
    if (t == 0) a.chunk_sums[(int64_t)sh * a.chunk_stride + c] = s_w[0] + s_w[1] + s_w[2] + s_w[3];
    return;
  }
  int64_t acc = s_start + incl - sum;
  for (int k = 0; k < w; ++k) acc += s_w[k];
  const int64_t total = s_total;
#pragma unroll
  for (int j = 0; j < kChunkPer; ++j) {
    const int64_t f = base + j;
    if (f < f1) {
      a.local[f] = a.mask[f] ? acc : total;
      acc += v[j];
    }
  }
  if (c == 0 && t == 0) {
    a.sizes[sh] = total;
    if (sh == 0) a.local[a.Fa] = 0;
  }
}
__global__ __launch_bounds__(kChunkThreads) void rf_compact_chunks_kernel(RfCompactArgs a, int pass) { rf_compact_chunks_kernel_body(a, pass); }
__global__ __launch_bounds__(kChunkThreads) void rf_compact_chunks_lanes_kernel(const RfCompactArgs* __restrict__ args,
                                                                               int pass) {
  rf_compact_chunks_kernel_body(args[blockIdx.z], pass);
}
}  // namespace

int64_t rf_compact_chunks(int64_t max_shard_features) { return (max_shard_features + kChunkFeat - 1) / kChunkFeat; }

void launch_rf_compact(const RfCompactArgs& a, hipStream_t s) {
  if (a.chunk_sums == nullptr) {
    hipLaunchKernelGGL(rf_compact_kernel, dim3(1), dim3(kCompactThreads), 0, s, a);
    return;
  }
  const dim3 grid((unsigned)(a.chunk_stride > 0 ? a.chunk_stride : 1), (unsigned)a.S);
  hipLaunchKernelGGL(rf_compact_chunks_kernel, grid, dim3(kChunkThreads), 0, s, a, 0);
  hipLaunchKernelGGL(rf_compact_chunks_kernel, grid, dim3(kChunkThreads), 0, s, a, 1);
}

void launch_rf_sample(const RfSampleArgs& a, hipStream_t s) {
  // k >= F (every feature) is handled by the caller: thresholds 1.0, mask all ones
  if (a.nnodes <= 0 || a.k >= a.F) return;
  if (a.scratch != nullptr) {
    // window [lo, hi] of expected counts k -+ (8 sqrt(k) + 8), as 53-bit priorities
    const double sd = 8.0 * sqrt((double)a.k) + 8.0;
    const double lo = fmax(0.0, (double)a.k - sd) / (double)a.F, hi = fmin((double)a.F, (double)a.k + sd) / (double)a.F;
    const uint64_t ulo = (uint64_t)(lo * 9007199254740992.0);
    const uint64_t uhi = hi >= 1.0 ? (1ull << 53) : (uint64_t)(hi * 9007199254740992.0);
    unsigned int* below = reinterpret_cast<unsigned int*>(a.scratch);
    unsigned int* ncand = below + a.nnodes;
    uint64_t* cand = reinterpret_cast<uint64_t*>(a.scratch + 8 * ((2 * a.nnodes * 4 + 7) / 8));
    if (a.fused_counts != nullptr && a.nnodes <= a.fused_cap) {
      hipLaunchKernelGGL(rf_window_threshold_kernel, dim3(kSlices, a.nnodes), dim3(kThreads), 0, s, a, ulo, uhi, cand);
      if (a.Fa > 0)
        hipLaunchKernelGGL(rf_mask_kernel, dim3((unsigned)((a.Fa + kThreads - 1) / kThreads)), dim3(kThreads), 0, s, a);
      return;
    }
    hipMemsetAsync(below, 0, sizeof(unsigned int) * 2 * (size_t)a.nnodes, s);
    hipLaunchKernelGGL(rf_window_kernel, dim3(kSlices, a.nnodes), dim3(kThreads), 0, s, a, ulo, uhi, below, ncand,
                       cand);
    hipLaunchKernelGGL(rf_threshold_kernel, dim3(a.nnodes), dim3(kThreads), 0, s, a, below, ncand, cand);
  } else {
    hipLaunchKernelGGL(rf_threshold_kernel, dim3(a.nnodes), dim3(kThreads), 0, s, a, nullptr, nullptr, nullptr);
  }
  if (a.Fa > 0)
    hipLaunchKernelGGL(rf_mask_kernel, dim3((unsigned)((a.Fa + kThreads - 1) / kThreads)), dim3(kThreads), 0, s, a);
}

// window bounds of the fused sample (launch_rf_sample)
static void rf_window(const RfSampleArgs& a, uint64_t* ulo, uint64_t* uhi) {
  const double sd = 8.0 * sqrt((double)a.k) + 8.0;
  const double lo = fmax(0.0, (double)a.k - sd) / (double)a.F, hi = fmin((double)a.F, (double)a.k + sd) / (double)a.F;
  *ulo = (uint64_t)(lo * 9007199254740992.0);
  *uhi = hi >= 1.0 ? (1ull << 53) : (uint64_t)(hi * 9007199254740992.0);
}

void launch_rf_sample_lanes(const RfSampleArgs* h, const RfSampleArgs* d, int L, hipStream_t s) {
  if (L <= 0 || h[0].k >= h[0].F) return;
  int32_t ny = 0;
  for (int l = 0; l < L; ++l) {
    FDX_LANES_CHECK(h[l].k == h[0].k && h[l].F == h[0].F && h[l].Fa == h[0].Fa && h[l].scratch != nullptr &&
                    h[l].fused_counts != nullptr && h[l].nnodes <= h[l].fused_cap);
    ny = h[l].nnodes > ny ? h[l].nnodes : ny;
  }
  if (ny <= 0) return;
  uint64_t ulo, uhi;
  rf_window(h[0], &ulo, &uhi);
  hipLaunchKernelGGL(rf_window_threshold_lanes_kernel, dim3(kSlices, ny, L), dim3(kThreads), 0, s, d, ulo, uhi);
  if (h[0].Fa > 0)
    hipLaunchKernelGGL(rf_mask_lanes_kernel, dim3((unsigned)((h[0].Fa + kThreads - 1) / kThreads), 1, L), dim3(kThreads),
                       0, s, d);
}

void launch_rf_compact_lanes(const RfCompactArgs* h, const RfCompactArgs* d, int L, hipStream_t s) {
  if (L <= 0) return;
  for (int l = 0; l < L; ++l)
    FDX_LANES_CHECK(h[l].chunk_sums != nullptr && h[l].chunk_stride == h[0].chunk_stride && h[l].S == h[0].S);
  const dim3 grid((unsigned)(h[0].chunk_stride > 0 ? h[0].chunk_stride : 1), (unsigned)h[0].S, L);
  hipLaunchKernelGGL(rf_compact_chunks_lanes_kernel, grid, dim3(kChunkThreads), 0, s, d, 0);
  hipLaunchKernelGGL(rf_compact_chunks_lanes_kernel, grid, dim3(kChunkThreads), 0, s, d, 1);
}

}  // namespace fdx

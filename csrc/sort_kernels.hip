// Feature-major ordering of a CSR matrix for gfx950 (K-06 docFreq, K-09 binning, CSC build).
//
// A count-valued CSR (rows = documents, sorted unique feature ids per row) is turned into its CSC
// without atomics:
//   1. pack:   one wave per row writes key = feature id and payload = min(count, 255) << 32 | row
//              for every entry (coalesced, the row's entries are contiguous);
//   2. sort:   rocPRIM radix sort of (key, payload) pairs over only ceil(log2 F) key bits
//              (stable, so each column keeps its rows in increasing order);
//   3. unpack: csc_row / csc_bin streams (no random gathers: the payload carried everything);
//   4. per feature: max count by a wave-segmented max over the sorted keys (one atomic per key
//      run per wave) and docFreq = column length - zero-count entries.
// The previous torch formulation spent most of its time in contended scatter-max / bincount
// atomics on the hottest features; here every per-feature quantity is a segmented reduction.
#include <hipcub/hipcub.hpp>

#include "ops.h"

namespace fdx {

namespace {
constexpr int kWave = 64;

template <class V>
__global__ __launch_bounds__(256) void pack_entries_kernel(const int64_t* __restrict__ indptr,
                                                           const int32_t* __restrict__ idx,
                                                           const V* __restrict__ counts, int64_t rows,
                                                           int32_t* __restrict__ keys, uint64_t* __restrict__ payload) {
  const int64_t r = (int64_t)blockIdx.x * 4 + threadIdx.x / kWave;
  const int lane = threadIdx.x & (kWave - 1);
  if (r >= rows) return;
  const int64_t e1 = indptr[r + 1];
  for (int64_t e = indptr[r] + lane; e < e1; e += kWave) {
    const double c = (double)counts[e];
    const uint64_t b = c <= 0.0 ? 0u : (c >= 255.0 ? 255u : (uint64_t)c);
    keys[e] = idx[e];
    payload[e] = (b << 32) | (uint64_t)(uint32_t)r;
  }
}

__global__ __launch_bounds__(256) void unpack_entries_kernel(const uint64_t* __restrict__ payload, int64_t n,
                                                             int32_t* __restrict__ csc_row, uint8_t* __restrict__ csc_cnt) {
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n; e += (int64_t)gridDim.x * 256) {
    const uint64_t p = payload[e];
    csc_row[e] = (int32_t)(uint32_t)p;
    csc_cnt[e] = (uint8_t)(p >> 32);
  }
}

// colptr from the sorted keys: every boundary between key k0 and k1 > k0 fills colptr[k0+1..k1]
__global__ __launch_bounds__(256) void colptr_kernel(const int32_t* __restrict__ sorted_keys, int64_t n, int32_t F,
                                                     int64_t* __restrict__ colptr) {
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e <= n; e += (int64_t)gridDim.x * 256) {
    const int32_t prev = e == 0 ? -1 : sorted_keys[e - 1];
    const int32_t cur = e == n ? F : sorted_keys[e];
    for (int32_t k = prev + 1; k <= cur; ++k) colptr[k] = e;
  }
}

// Per-feature max count and count of zero-count entries over the key-sorted entries: a wave
// covers 64 consecutive entries, a segmented max over runs of equal keys (sorted, so runs are
// contiguous) leaves the run maximum in the run's first lane, which issues the only atomic. Hot
// features (millions of entries) thus cost one atomic per wave instead of a serial walk.
__global__ __launch_bounds__(256) void feature_stats_kernel(const int32_t* __restrict__ sorted_keys,
                                                            const uint8_t* __restrict__ csc_cnt, int64_t n,
                                                            int32_t* __restrict__ maxc, int64_t* __restrict__ zeros) {
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t base = (int64_t)blockIdx.x * 256 + (threadIdx.x & ~(kWave - 1)); base < n; base += stride) {
    const int64_t e = base + lane;
    const int32_t k = e < n ? sorted_keys[e] : -1;
    const int32_t c = e < n ? (int32_t)csc_cnt[e] : 0;
    if (e < n && c == 0) atomicAdd(reinterpret_cast<unsigned long long*>(&zeros[k]), 1ull);
    int32_t m = c;
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
      const int32_t km = __shfl_down(k, o, kWave);
      const int32_t mm = __shfl_down(m, o, kWave);
      if (lane + o < kWave && km == k) m = mm > m ? mm : m;
    }
    const int32_t kp = __shfl_up(k, 1, kWave);
    if (k >= 0 && (lane == 0 || kp != k) && m > 0) atomicMax(&maxc[k], m);
  }
}

// in place: `zeros` and `df` are the same buffer
__global__ __launch_bounds__(256) void df_kernel(const int64_t* __restrict__ colptr, const int64_t* zeros, int32_t F,
                                                 int64_t* df) {
  const int32_t f = (int32_t)((int64_t)blockIdx.x * 256 + threadIdx.x);
  if (f < F) df[f] = colptr[f + 1] - colptr[f] - zeros[f];
}

// bounds[i][b] = first entry of column cols[i] whose row >= b * row_block (b = 0..nblk), i.e. the
// row-block segments of a column whose rows are sorted (XCD-aware work items, quantize.py).
__global__ __launch_bounds__(256) void block_bounds_kernel(const int32_t* __restrict__ csc_row,
                                                           const int64_t* __restrict__ colptr,
                                                           const int32_t* __restrict__ cols, int32_t ncols,
                                                           int32_t nblk, int64_t row_block, int64_t* __restrict__ bounds) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= (int64_t)ncols * (nblk + 1)) return;
  const int32_t i = (int32_t)(t / (nblk + 1)), b = (int32_t)(t % (nblk + 1));
  const int32_t c = cols[i];
  int64_t lo = colptr[c], hi = colptr[c + 1];
  const int64_t target = (int64_t)b * row_block;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if ((int64_t)csc_row[mid] < target) lo = mid + 1;
    else hi = mid;
  }
  bounds[t] = lo;
}

// dst[seg_dst[i] + k] = src[seg_src[i] + k] for k < seg_len[i], rows (int32) and keys (uint8):
// one workgroup per segment (the super-block-major copy of the histogram CSC).
__global__ __launch_bounds__(256) void copy_segments_kernel(const int32_t* __restrict__ src_row,
                                                            const uint8_t* __restrict__ src_key,
                                                            const int64_t* __restrict__ seg_src,
                                                            const int64_t* __restrict__ seg_dst,
                                                            const int64_t* __restrict__ seg_len, int64_t nseg,
                                                            const uint8_t* __restrict__ seg_add,
                                                            int32_t* __restrict__ dst_row, uint8_t* __restrict__ dst_key) {
  for (int64_t i = blockIdx.x; i < nseg; i += gridDim.x) {
    const int64_t a = seg_src[i], d = seg_dst[i], n = seg_len[i];
    const uint8_t add = seg_add ? seg_add[i] : (uint8_t)0;
    for (int64_t k = threadIdx.x; k < n; k += 256) {
      dst_row[d + k] = src_row[a + k];
      dst_key[d + k] = (uint8_t)(src_key[a + k] + add);
    }
  }
}

// The dense block of the hot features (models/quantize.py _build_dense): segment i (= hot feature
// i's CSC range) scatters its entries' bins into row i of dense [nseg, n_pad] (pre-filled with the
// features' zero bins). Workgroups (x, i): a grid-stride over segment i's entries.
__global__ __launch_bounds__(256) void dense_scatter_kernel(const int32_t* __restrict__ row, const uint8_t* __restrict__ bin,
                                                            const int64_t* __restrict__ seg_src,
                                                            const int64_t* __restrict__ seg_len, int64_t n_pad,
                                                            uint8_t* __restrict__ dense) {
  const int64_t i = blockIdx.y;
  const int64_t a = seg_src[i], n = seg_len[i];
  uint8_t* out = dense + i * n_pad;
  for (int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x; k < n; k += (int64_t)gridDim.x * 256)
    out[row[a + k]] = bin[a + k];
}

__global__ __launch_bounds__(256) void clamp_u8_kernel(const uint8_t* __restrict__ in, int64_t n, uint8_t maxv,
                                                       uint8_t* __restrict__ out) {
  const int64_t n16 = n / 16;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (int64_t)gridDim.x * 256) {
    uint4 v = reinterpret_cast<const uint4*>(in)[i];
    uint32_t* w = reinterpret_cast<uint32_t*>(&v);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      uint32_t x = w[k], y = 0;
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const uint32_t c = (x >> (8 * b)) & 0xffu;
        y |= (c > maxv ? (uint32_t)maxv : c) << (8 * b);
      }
      w[k] = y;
    }
    reinterpret_cast<uint4*>(out)[i] = v;
  }
  const int64_t t = 16 * n16 + (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t < n && blockIdx.x * 256 + threadIdx.x < 16) out[t] = in[t] > maxv ? maxv : in[t];
}

inline unsigned grid_for(int64_t n, int64_t cap = 16384) {
  const int64_t b = (n + 255) / 256;
  return (unsigned)(b < 1 ? 1 : (b > cap ? cap : b));
}

inline int key_bits(int32_t F) {
  int b = 1;
  while (b < 31 && (1ll << b) < (int64_t)F) ++b;
  return b;
}
}  // namespace

size_t feature_order_temp_bytes(int64_t nnz, int32_t F) {
  size_t bytes = 0;
  hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, (const int32_t*)nullptr, (int32_t*)nullptr,
                                     (const uint64_t*)nullptr, (uint64_t*)nullptr, (size_t)nnz, 0, key_bits(F));
  return bytes;
}

template <class V>
void launch_feature_order(const FeatureOrderArgs<V>& a, hipStream_t s) {
  if (a.nnz > 0) {
    hipLaunchKernelGGL((pack_entries_kernel<V>), dim3((unsigned)((a.rows + 3) / 4)), dim3(256), 0, s, a.indptr, a.idx,
                       a.counts, a.rows, a.keys_tmp, a.payload_tmp);
    size_t bytes = a.temp_bytes;
    hipcub::DeviceRadixSort::SortPairs(a.temp, bytes, a.keys_tmp, a.keys_sorted, a.payload_tmp, a.payload_sorted,
                                       (size_t)a.nnz, 0, key_bits(a.F), s);
    hipLaunchKernelGGL(unpack_entries_kernel, dim3(grid_for(a.nnz)), dim3(256), 0, s, a.payload_sorted, a.nnz, a.csc_row,
                       a.csc_cnt);
  }
  hipLaunchKernelGGL(colptr_kernel, dim3(grid_for(a.nnz + 1)), dim3(256), 0, s, a.keys_sorted, a.nnz, a.F, a.colptr);
  hipMemsetAsync(a.maxc, 0, sizeof(int32_t) * (size_t)a.F, s);
  hipMemsetAsync(a.df, 0, sizeof(int64_t) * (size_t)a.F, s);          // zero-count entries first
  if (a.nnz > 0)
    hipLaunchKernelGGL(feature_stats_kernel, dim3(grid_for(a.nnz)), dim3(256), 0, s, a.keys_sorted, a.csc_cnt, a.nnz,
                       a.maxc, a.df);
  hipLaunchKernelGGL(df_kernel, dim3((unsigned)((a.F + 255) / 256)), dim3(256), 0, s, a.colptr, a.df, a.F, a.df);
}

void launch_block_bounds(const int32_t* csc_row, const int64_t* colptr, const int32_t* cols, int32_t ncols, int32_t nblk,
                         int64_t row_block, int64_t* bounds, hipStream_t s) {
  const int64_t n = (int64_t)ncols * (nblk + 1);
  if (n > 0)
    hipLaunchKernelGGL(block_bounds_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, csc_row, colptr, cols, ncols,
                       nblk, row_block, bounds);
}

void launch_dense_scatter(const int32_t* row, const uint8_t* bin, const int64_t* seg_src, const int64_t* seg_len,
                          int64_t nseg, int64_t max_len, int64_t n_pad, uint8_t* dense, hipStream_t s) {
  if (nseg <= 0 || max_len <= 0) return;
  const int64_t bx = (max_len + 255) / 256;
  hipLaunchKernelGGL(dense_scatter_kernel, dim3((unsigned)(bx < 256 ? bx : 256), (unsigned)nseg), dim3(256), 0, s, row, bin,
                     seg_src, seg_len, n_pad, dense);
}

void launch_copy_segments(const int32_t* src_row, const uint8_t* src_key, const int64_t* seg_src, const int64_t* seg_dst,
                          const int64_t* seg_len, int64_t nseg, const uint8_t* seg_add, int32_t* dst_row, uint8_t* dst_key,
                          hipStream_t s) {
  if (nseg <= 0) return;
  const unsigned grid = (unsigned)(nseg < 65536 ? nseg : 65536);
  hipLaunchKernelGGL(copy_segments_kernel, dim3(grid), dim3(256), 0, s, src_row, src_key, seg_src, seg_dst, seg_len, nseg,
                     seg_add, dst_row, dst_key);
}

void launch_clamp_u8(const uint8_t* in, int64_t n, uint8_t maxv, uint8_t* out, hipStream_t s) {
  if (n > 0) hipLaunchKernelGGL(clamp_u8_kernel, dim3(grid_for(n / 16 + 1)), dim3(256), 0, s, in, n, maxv, out);
}

template void launch_feature_order<float>(const FeatureOrderArgs<float>&, hipStream_t);
template void launch_feature_order<double>(const FeatureOrderArgs<double>&, hipStream_t);
template void launch_feature_order<int32_t>(const FeatureOrderArgs<int32_t>&, hipStream_t);

}  // namespace fdx

// Sparse-matrix kernels for gfx950: CSR scoring (LR margin / tree ensembles, K-07/K-16 over an
// existing feature column), SpMV and transposed SpMV for logistic-regression training (K-08),
// and the IDF document-frequency count (K-06).
//
// Row-wise kernels assign one 64-lane wavefront per row (rows of TF-IDF vectors are ~100 nnz,
// so a wave reads a row in one or two coalesced passes). Reductions use the same lane-strided
// partial + xor-butterfly order as the fused featurizer, so the two paths agree bit-for-bit.
#include "scoring.h"
#include "ops.h"

#pragma clang fp contract(off)

namespace fdx {

namespace {
constexpr int kWave = 64;
constexpr int kBlock = 256;

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = kWave / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

template <class V>
__device__ __forceinline__ double row_lookup(const int32_t* idx, const V* val, int64_t a, int64_t b, int32_t f) {
  int64_t lo = a, hi = b - 1;
  while (lo <= hi) {
    const int64_t mid = (lo + hi) >> 1;
    const int32_t k = idx[mid];
    if (k == f) return (double)val[mid];
    if (k < f) lo = mid + 1; else hi = mid - 1;
  }
  return 0.0;
}

template <class V>
__global__ __launch_bounds__(kBlock) void score_csr_kernel(CsrArgs<V> a) {
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t r = (int64_t)blockIdx.x * (kBlock / kWave) + threadIdx.x / kWave;
  if (r >= a.rows) return;
  const int64_t s = a.indptr[r], e = a.indptr[r + 1];
  if (a.lr_w) {
    double part = 0.0;
    for (int64_t j = s + lane; j < e; j += kWave) part += (double)a.val[j] * a.lr_w[a.idx[j]];
    part = wave_sum(part);
    if (lane == 0) a.out[r] = part + a.lr_b;
    return;
  }
  const TreeEnsemble& te = a.trees;
  auto lookup = [&](int32_t f) { return row_lookup(a.idx, a.val, s, e, f); };
  double acc0 = 0.0, acc1 = 0.0;
  for (int t = lane; t < te.num_trees; t += kWave) {
    const int32_t leaf = tree_find_leaf(te, te.roots[t], a.cmp_less, lookup);
    acc0 += te.weights[t] * te.leaf[(int64_t)leaf * te.K];
    if (te.K > 1) acc1 += te.weights[t] * te.leaf[(int64_t)leaf * te.K + 1];
  }
  acc0 = wave_sum(acc0);
  acc1 = wave_sum(acc1);
  if (lane == 0) {
    a.out[r * te.K] = acc0;
    if (te.K > 1) a.out[r * te.K + 1] = acc1;
  }
}

// y[r] = sum_j val[j] * x[idx[j]]  (+ optional per-row scale applied by the caller)
template <class V>
__global__ __launch_bounds__(kBlock) void spmv_kernel(const int64_t* indptr, const int32_t* idx, const V* val,
                                                     const double* x, double* y, int64_t rows) {
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t r = (int64_t)blockIdx.x * (kBlock / kWave) + threadIdx.x / kWave;
  if (r >= rows) return;
  double part = 0.0;
  for (int64_t j = indptr[r] + lane; j < indptr[r + 1]; j += kWave) part += (double)val[j] * x[idx[j]];
  part = wave_sum(part);
  if (lane == 0) y[r] = part;
}

// g[idx[j]] += val[j] * r[row(j)]  — wave per row, fp64 atomics into the (L2-resident) gradient.
template <class V>
__global__ __launch_bounds__(kBlock) void spmv_t_kernel(const int64_t* indptr, const int32_t* idx, const V* val,
                                                       const double* rvec, double* g, int64_t rows) {
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t r = (int64_t)blockIdx.x * (kBlock / kWave) + threadIdx.x / kWave;
  if (r >= rows) return;
  const double rr = rvec[r];
  if (rr == 0.0) return;
  for (int64_t j = indptr[r] + lane; j < indptr[r + 1]; j += kWave)
    atomicAdd(&g[idx[j]], (double)val[j] * rr);
}

// docFreq[f] += 1 for every stored non-zero (IDF fit, X-06).
template <class V>
__global__ __launch_bounds__(kBlock) void doc_freq_kernel(const int32_t* idx, const V* val, int64_t nnz, int64_t* df) {
  for (int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x; j < nnz; j += (int64_t)gridDim.x * kBlock)
    if (val[j] != (V)0) atomicAdd(reinterpret_cast<unsigned long long*>(&df[idx[j]]), 1ull);
}

inline dim3 row_grid(int64_t rows) { return dim3((unsigned)((rows + (kBlock / kWave) - 1) / (kBlock / kWave))); }
}  // namespace

template <class V>
void launch_score_csr(const CsrArgs<V>& a, hipStream_t stream) {
  if (a.rows <= 0) return;
  hipLaunchKernelGGL(score_csr_kernel<V>, row_grid(a.rows), dim3(kBlock), 0, stream, a);
}
template void launch_score_csr<float>(const CsrArgs<float>&, hipStream_t);
template void launch_score_csr<double>(const CsrArgs<double>&, hipStream_t);

template <class V>
void launch_spmv(const int64_t* indptr, const int32_t* idx, const V* val, const double* x, double* y, int64_t rows,
                 hipStream_t stream) {
  if (rows <= 0) return;
  hipLaunchKernelGGL(spmv_kernel<V>, row_grid(rows), dim3(kBlock), 0, stream, indptr, idx, val, x, y, rows);
}
template void launch_spmv<float>(const int64_t*, const int32_t*, const float*, const double*, double*, int64_t, hipStream_t);
template void launch_spmv<double>(const int64_t*, const int32_t*, const double*, const double*, double*, int64_t, hipStream_t);

template <class V>
void launch_spmv_t(const int64_t* indptr, const int32_t* idx, const V* val, const double* r, double* g, int64_t rows,
                   hipStream_t stream) {
  if (rows <= 0) return;
  hipLaunchKernelGGL(spmv_t_kernel<V>, row_grid(rows), dim3(kBlock), 0, stream, indptr, idx, val, r, g, rows);
}
template void launch_spmv_t<float>(const int64_t*, const int32_t*, const float*, const double*, double*, int64_t, hipStream_t);
template void launch_spmv_t<double>(const int64_t*, const int32_t*, const double*, const double*, double*, int64_t, hipStream_t);

template <class V>
void launch_doc_freq(const int32_t* idx, const V* val, int64_t nnz, int64_t* df, hipStream_t stream) {
  if (nnz <= 0) return;
  const int64_t want = (nnz + kBlock - 1) / kBlock;
  const unsigned grid = (unsigned)(want < 8192 ? want : 8192);
  hipLaunchKernelGGL(doc_freq_kernel<V>, dim3(grid), dim3(kBlock), 0, stream, idx, val, nnz, df);
}
template void launch_doc_freq<float>(const int32_t*, const float*, int64_t, int64_t*, hipStream_t);
template void launch_doc_freq<double>(const int32_t*, const double*, int64_t, int64_t*, hipStream_t);

}  // namespace fdx

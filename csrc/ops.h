// Host-callable entry points of the native core (HIP launchers + CPU implementations).
#pragma once
#include <hip/hip_runtime.h>

#include "scoring.h"

namespace fdx {

// text_kernels.hip
void launch_featurize_score(const FeatArgs& a, hipStream_t stream);
// text_cpu.cpp
void featurize_score_cpu(const FeatArgs& a, const int32_t* only_docs, int32_t n_only, int threads);

// ---------------------------------------------------------------- sparse (sparse_kernels.hip / sparse_cpu.cpp)
template <class V>
struct CsrArgs {
  const int64_t* indptr;
  const int32_t* idx;
  const V* val;
  int64_t rows;
  const double* lr_w;   // LR scorer when non-null
  double lr_b;
  TreeEnsemble trees;   // tree scorer otherwise
  bool cmp_less;
  double* out;          // [rows * K]
};

template <class V> void launch_score_csr(const CsrArgs<V>& a, hipStream_t stream);
template <class V> void launch_spmv(const int64_t* indptr, const int32_t* idx, const V* val, const double* x,
                                   double* y, int64_t rows, hipStream_t stream);
template <class V> void launch_spmv_t(const int64_t* indptr, const int32_t* idx, const V* val, const double* r,
                                     double* g, int64_t rows, hipStream_t stream);
template <class V> void launch_doc_freq(const int32_t* idx, const V* val, int64_t nnz, int64_t* df,
                                       hipStream_t stream);

template <class V> void score_csr_cpu(const CsrArgs<V>& a, int threads);
template <class V> void spmv_cpu(const int64_t* indptr, const int32_t* idx, const V* val, const double* x, double* y,
                                 int64_t rows, int threads);
template <class V> void spmv_t_cpu(const int64_t* indptr, const int32_t* idx, const V* val, const double* r,
                                   double* g, int64_t rows, int64_t cols, int threads);

}  // namespace fdx

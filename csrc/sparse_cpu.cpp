// Host implementations of the sparse kernels (same contracts and summation order as
// sparse_kernels.hip: lane-strided partials over 64 "lanes" + xor butterfly).
#include <cstring>
#include <vector>

#include "ops.h"
#include "parallel_for.h"

namespace fdx {

namespace {
inline double butterfly(double* p) {
  for (int o = 32; o > 0; o >>= 1)
    for (int l = 0; l < 64; ++l)
      if (l < (l ^ o)) { const double t = p[l] + p[l ^ o]; p[l] = t; p[l ^ o] = t; }
  return p[0];
}
}  // namespace

template <class V>
void score_csr_cpu(const CsrArgs<V>& a, int threads) {
  parallel_for(a.rows, threads, 256, [&](int64_t lo, int64_t hi) {
    for (int64_t r = lo; r < hi; ++r) {
      const int64_t s = a.indptr[r], e = a.indptr[r + 1];
      if (a.lr_w) {
        double p[64] = {0};
        for (int64_t j = s; j < e; ++j) p[(j - s) & 63] += (double)a.val[j] * a.lr_w[a.idx[j]];
        a.out[r] = butterfly(p) + a.lr_b;
        continue;
      }
      const TreeEnsemble& te = a.trees;
      auto lookup = [&](int32_t f) -> double {
        int64_t l = s, h = e - 1;
        while (l <= h) {
          const int64_t m = (l + h) >> 1;
          if (a.idx[m] == f) return (double)a.val[m];
          if (a.idx[m] < f) l = m + 1; else h = m - 1;
        }
        return 0.0;
      };
      double p0[64] = {0}, p1[64] = {0};
      for (int t = 0; t < te.num_trees; ++t) {
        const int32_t leaf = tree_find_leaf(te, te.roots[t], a.cmp_less, lookup);
        p0[t & 63] += te.weights[t] * te.leaf[(int64_t)leaf * te.K];
        if (te.K > 1) p1[t & 63] += te.weights[t] * te.leaf[(int64_t)leaf * te.K + 1];
      }
      a.out[r * te.K] = butterfly(p0);
      if (te.K > 1) a.out[r * te.K + 1] = butterfly(p1);
    }
  });
}
template void score_csr_cpu<float>(const CsrArgs<float>&, int);
template void score_csr_cpu<double>(const CsrArgs<double>&, int);

template <class V>
void spmv_cpu(const int64_t* indptr, const int32_t* idx, const V* val, const double* x, double* y, int64_t rows,
              int threads) {
  parallel_for(rows, threads, 1024, [&](int64_t lo, int64_t hi) {
    for (int64_t r = lo; r < hi; ++r) {
      double p[64] = {0};
      for (int64_t j = indptr[r]; j < indptr[r + 1]; ++j) p[(j - indptr[r]) & 63] += (double)val[j] * x[idx[j]];
      y[r] = butterfly(p);
    }
  });
}
template void spmv_cpu<float>(const int64_t*, const int32_t*, const float*, const double*, double*, int64_t, int);
template void spmv_cpu<double>(const int64_t*, const int32_t*, const double*, const double*, double*, int64_t, int);

template <class V>
void spmv_t_cpu(const int64_t* indptr, const int32_t* idx, const V* val, const double* r, double* g, int64_t rows,
                int64_t cols, int threads) {
  // per-thread private gradients, reduced in fixed thread order (deterministic for a fixed pool)
  const int T = std::max(1, std::min<int>(threads <= 0 ? 8 : threads, (int)std::max<int64_t>(1, rows / 4096)));
  std::vector<std::vector<double>> priv(T, std::vector<double>(cols, 0.0));
  const int64_t chunk = (rows + T - 1) / T;
  parallel_for(T, T, 1, [&](int64_t lo, int64_t hi) {
    for (int64_t t = lo; t < hi; ++t) {
      double* gp = priv[t].data();
      const int64_t r0 = t * chunk, r1 = std::min(rows, r0 + chunk);
      for (int64_t row = r0; row < r1; ++row) {
        const double rr = r[row];
        if (rr == 0.0) continue;
        for (int64_t j = indptr[row]; j < indptr[row + 1]; ++j) gp[idx[j]] += (double)val[j] * rr;
      }
    }
  });
  for (int t = 0; t < T; ++t)
    for (int64_t c = 0; c < cols; ++c) g[c] += priv[t][c];
}
template void spmv_t_cpu<float>(const int64_t*, const int32_t*, const float*, const double*, double*, int64_t, int64_t, int);
template void spmv_t_cpu<double>(const int64_t*, const int32_t*, const double*, const double*, double*, int64_t, int64_t, int);

}  // namespace fdx

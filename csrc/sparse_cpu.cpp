// Host implementations of the sparse kernels (same contracts and summation order as
// sparse_kernels.hip: lane-strided partials over 64 "lanes" + xor butterfly).
#include <algorithm>
#include <climits>
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

// Stable counting sort by feature (host twin of launch_feature_order).
template <class V>
void feature_order_cpu(const FeatureOrderArgs<V>& a) {
  for (int32_t f = 0; f <= a.F; ++f) a.colptr[f] = 0;
  for (int64_t e = 0; e < a.nnz; ++e) a.colptr[a.idx[e] + 1]++;
  for (int32_t f = 0; f < a.F; ++f) a.colptr[f + 1] += a.colptr[f];
  std::vector<int64_t> cur(a.colptr, a.colptr + a.F);
  for (int64_t r = 0; r < a.rows; ++r)
    for (int64_t e = a.indptr[r]; e < a.indptr[r + 1]; ++e) {
      const int64_t p = cur[a.idx[e]]++;
      const double c = (double)a.counts[e];
      a.csc_row[p] = (int32_t)r;
      a.csc_cnt[p] = (uint8_t)(c <= 0.0 ? 0 : (c >= 255.0 ? 255 : (int)c));
    }
  parallel_for(a.F, 0, 1024, [&](int64_t lo, int64_t hi) {
    for (int64_t f = lo; f < hi; ++f) {
      int64_t nz = 0;
      int32_t mx = 0;
      for (int64_t e = a.colptr[f]; e < a.colptr[f + 1]; ++e) {
        nz += a.csc_cnt[e] > 0;
        mx = a.csc_cnt[e] > mx ? a.csc_cnt[e] : mx;
      }
      a.df[f] = nz;
      a.maxc[f] = mx;
    }
  });
}

void block_bounds_cpu(const int32_t* csc_row, const int64_t* colptr, const int32_t* cols, int32_t ncols, int32_t nblk,
                      int64_t row_block, int64_t* bounds) {
  parallel_for((int64_t)ncols * (nblk + 1), 0, 4096, [&](int64_t lo_t, int64_t hi_t) {
    for (int64_t t = lo_t; t < hi_t; ++t) {
      const int32_t c = cols[t / (nblk + 1)];
      const int64_t target = (t % (nblk + 1)) * row_block;
      const int32_t* b = csc_row + colptr[c];
      const int32_t* e = csc_row + colptr[c + 1];
      bounds[t] = colptr[c] + (std::lower_bound(b, e, (int32_t)std::min<int64_t>(target, INT32_MAX)) - b);
    }
  });
}

void copy_segments_cpu(const int32_t* src_row, const uint8_t* src_key, const int64_t* seg_src, const int64_t* seg_dst,
                       const int64_t* seg_len, int64_t nseg, const uint8_t* seg_add, int32_t* dst_row, uint8_t* dst_key) {
  parallel_for(nseg, 0, 64, [&](int64_t lo, int64_t hi) {
    for (int64_t i = lo; i < hi; ++i) {
      std::copy(src_row + seg_src[i], src_row + seg_src[i] + seg_len[i], dst_row + seg_dst[i]);
      const uint8_t add = seg_add ? seg_add[i] : (uint8_t)0;
      for (int64_t k = 0; k < seg_len[i]; ++k) dst_key[seg_dst[i] + k] = (uint8_t)(src_key[seg_src[i] + k] + add);
    }
  });
}

void dense_scatter_cpu(const int32_t* row, const uint8_t* bin, const int64_t* seg_src, const int64_t* seg_len,
                       int64_t nseg, int64_t n_pad, uint8_t* dense) {
  parallel_for(nseg, 0, 1, [&](int64_t lo, int64_t hi) {
    for (int64_t i = lo; i < hi; ++i)
      for (int64_t k = 0; k < seg_len[i]; ++k) dense[i * n_pad + row[seg_src[i] + k]] = bin[seg_src[i] + k];
  });
}

template void feature_order_cpu<float>(const FeatureOrderArgs<float>&);
template void feature_order_cpu<double>(const FeatureOrderArgs<double>&);
template void feature_order_cpu<int32_t>(const FeatureOrderArgs<int32_t>&);

}  // namespace fdx

// Host implementation of the tree engine (same contracts as tree_kernels.hip). The histogram is
// accumulated in fp64 straight from the bf16 hi/lo statistics, so it agrees with the MFMA path
// to ~1e-7 relative (the device accumulates each chunk in fp32); split decisions match except
// for exact gain ties within that tolerance.
#include <cmath>
#include <vector>

#include "ops.h"
#include "parallel_for.h"
#include "tree.h"

namespace fdx {

void rowstats_cpu(const RowStatsArgs& a) {
  parallel_for(a.N, 0, 1 << 16, [&](int64_t lo, int64_t hi) {
    for (int64_t r = lo; r < hi; ++r) {
      uint32_t* st = a.rowstats + 2 * r;
      if (a.mode == 0) {
        const float w = a.weight ? a.weight[r] : 1.0f;
        st[0] = split_bf16(a.g[r] * w);
        st[1] = split_bf16(a.h[r] * w);
      } else {
        float w = a.weight ? a.weight[r] : 1.0f;
        if (a.bootstrap) w *= (float)poisson1(hash_uniform(a.seed, (uint64_t)a.tree, (uint64_t)r));
        const float y = a.label[r];
        st[0] = split_bf16(w * (1.0f - y));
        st[1] = split_bf16(w * y);
      }
    }
  });
}

void entry_stats_cpu(const int32_t* csc_row, const uint32_t* rowstats, int64_t nnz, uint32_t* est) {
  parallel_for(nnz, 0, 1 << 16, [&](int64_t lo, int64_t hi) {
    for (int64_t e = lo; e < hi; ++e) {
      est[2 * e] = rowstats[2 * (int64_t)csc_row[e]];
      est[2 * e + 1] = rowstats[2 * (int64_t)csc_row[e] + 1];
    }
  });
}

void entry_stats_items_cpu(const int64_t* item_start, const int64_t* item_end, int32_t num_items,
                           const int32_t* csc_row, const uint32_t* rowstats, uint32_t* est) {
  parallel_for(num_items, 0, 16, [&](int64_t lo, int64_t hi) {
    for (int64_t it = lo; it < hi; ++it)
      for (int64_t e = item_start[it]; e < item_end[it]; ++e) {
        est[2 * e] = rowstats[2 * (int64_t)csc_row[e]];
        est[2 * e + 1] = rowstats[2 * (int64_t)csc_row[e] + 1];
      }
  });
}

void slot8_cpu(const SlotArgs& a) {
  parallel_for(a.N, 0, 1 << 16, [&](int64_t lo, int64_t hi) {
    for (int64_t r = lo; r < hi; ++r) {
      const int32_t node = a.row_node[r];
      const int32_t s = ((node >= 0 && node < a.num_nodes) ? a.node_slot[node] : -1) - a.slot_base;
      a.slot8[r] = (s >= 0 && s < a.nslots) ? (uint8_t)s : (uint8_t)0xff;
    }
  });
}

static inline double unpack(uint32_t v) { return (double)bf2f(v & 0xffffu) + (double)bf2f(v >> 16); }

void hist_cpu(const HistArgs& h, const HistReduceArgs& r, int slots) {
  parallel_for(r.L, 0, 16, [&](int64_t lo, int64_t hi) {
    std::vector<double> acc;
    for (int64_t li = lo; li < hi; ++li) {
      const int fid = r.feat[li];
      const int nb = r.nbins[fid];
      acc.assign((size_t)slots * nb * 2, 0.0);
      for (int i = 0; i < r.feat_nitems[li]; ++i) {
        const int64_t it = r.feat_item0[li] + i;
        for (int64_t e = h.item_start[it]; e < h.item_end[it]; ++e) {
          const int64_t row = h.csc_row[e];
          const int s = h.slot8 ? (int)h.slot8[row] : 0;
          if (s >= slots) continue;
          const int b = h.csc_bin[e];
          if (b >= nb) continue;
          const uint32_t* st = h.rowstats ? h.rowstats + 2 * row : h.est + 2 * e;
          acc[((size_t)s * nb + b) * 2] += unpack(st[0]);
          acc[((size_t)s * nb + b) * 2 + 1] += unpack(st[1]);
        }
      }
      for (int s = 0; s < slots; ++s) {
        const int node = r.slot_to_node[s];
        if (node < 0) continue;
        double* dst = r.hist + ((int64_t)node * r.total_bins + r.boff[fid]) * 2;
        for (int b = 0; b < nb; ++b) {
          dst[2 * b] = acc[((size_t)s * nb + b) * 2];
          dst[2 * b + 1] = acc[((size_t)s * nb + b) * 2 + 1];
        }
      }
    }
  });
}

void hist_subtract_cpu(const double* parent, double* cur, const int32_t* dst, const int32_t* par, const int32_t* sib,
                       int32_t n_pairs, int64_t TB) {
  const int64_t per = TB * 2;
  for (int p = 0; p < n_pairs; ++p)
    for (int64_t k = 0; k < per; ++k)
      cur[(int64_t)dst[p] * per + k] = parent[(int64_t)par[p] * per + k] - cur[(int64_t)sib[p] * per + k];
}

void split_cpu(const SplitArgs& a) {
  parallel_for((int64_t)a.num_nodes * a.Fa, 0, 4096, [&](int64_t lo, int64_t hi) {
    for (int64_t t = lo; t < hi; ++t) {
      const int n = (int)(t / a.Fa), f = (int)(t % a.Fa);
      double gain = -INFINITY, l0 = 0, l1 = 0;
      int bin = -1;
      bool use = true;
      if (a.feat_prob < 1.0)
        use = hash_uniform(a.seed ^ 0x5bd1e995ull, ((uint64_t)a.tree << 32) | (uint32_t)a.node_ids[n],
                           (uint64_t)a.fid_orig[f]) < a.feat_prob;
      if (use) {
        const double* hb = a.hist + ((int64_t)n * a.boff[a.Fa] + a.boff[f]) * 2;
        gain = best_split_scan(hb, a.nbins[f], a.zbin[f], a.totals[2 * n], a.totals[2 * n + 1], a.mode, a.lambda_,
                               a.min_child_weight, &bin, &l0, &l1);
      }
      a.out_gain[t] = gain;
      a.out_bin[t] = bin;
      a.out_left[2 * t] = l0;
      a.out_left[2 * t + 1] = l1;
    }
  });
}

void partition_cpu(const PartitionArgs& a) {
  for (int64_t r = 0; r < a.N; ++r) {
    const int32_t n = a.row_node[r];
    if (n >= 0 && n < a.num_nodes && a.default_child[n] >= 0) a.row_node[r] = a.default_child[n];
  }
  for (int it = 0; it < a.num_items; ++it) {
    const int sp = a.item_split[it];
    const bool left_default = a.split_left_is_default[sp] != 0;
    for (int64_t e = a.item_start[it]; e < a.item_end[it]; ++e) {
      const int32_t row = a.csc_row[e];
      const bool left = (int32_t)a.csc_bin[e] <= a.split_bin[sp];
      if (left != left_default && a.row_node[row] == a.split_default[sp]) a.row_node[row] = a.split_other[sp];
    }
  }
}

void logistic_grad_cpu(const double* margin, const float* label, const float* weight, float* g, float* h, int64_t N) {
  for (int64_t r = 0; r < N; ++r) {
    const double p = 1.0 / (1.0 + std::exp(-margin[r]));
    const double w = weight ? (double)weight[r] : 1.0;
    g[r] = (float)((p - (double)label[r]) * w);
    h[r] = (float)(std::fmax(p * (1.0 - p), 1e-16) * w);
  }
}

void leaf_update_cpu(double* margin, const int32_t* row_node, const double* node_value, int64_t N) {
  for (int64_t r = 0; r < N; ++r) margin[r] += node_value[row_node[r]];
}

}  // namespace fdx

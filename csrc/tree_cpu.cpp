// Host implementation of the tree engine (same contracts as tree_kernels.hip). Histograms are the
// same exact int64 sums of quantised statistics as on the device, so host and device trees are
// bitwise identical.
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstring>
#include <mutex>
#include <vector>

#include "ops.h"
#include "parallel_for.h"
#include "tree.h"

namespace fdx {

void quant_max_cpu(const QuantArgs& a, double* out) {
  std::mutex mu;
  out[0] = out[1] = 0.0;
  parallel_for(a.N, 0, 1 << 16, [&](int64_t lo, int64_t hi) {
    double x0 = 0.0, x1 = 0.0;
    for (int64_t r = lo; r < hi; ++r) {
      double v0, v1;
      row_stats(a, r, &v0, &v1);
      x0 = std::fmax(x0, std::fabs(v0));
      x1 = std::fmax(x1, std::fabs(v1));
    }
    std::lock_guard<std::mutex> lk(mu);   // max is order-independent
    out[0] = std::fmax(out[0], x0);
    out[1] = std::fmax(out[1], x1);
  });
}

void quant_cpu(const QuantArgs& a, const double* maxv) {
  const int32_t k0 = maxv ? quant_exponent(maxv[0]) : 0, k1 = maxv ? quant_exponent(maxv[1]) : 0;
  a.kexp_out[0] = k0;
  a.kexp_out[1] = k1;
  std::atomic<int64_t> t0{0}, t1{0};
  parallel_for(a.N, 0, 1 << 16, [&](int64_t lo, int64_t hi) {
    int64_t s0 = 0, s1 = 0;
    for (int64_t r = lo; r < hi; ++r) {
      double v0, v1;
      row_stats(a, r, &v0, &v1);
      const int64_t q0 = quantize_value(v0, k0), q1 = quantize_value(v1, k1);
      s0 += q0;
      s1 += q1;
      a.rowdig[2 * r] = a.np == 1 ? digits1(q0) : digits4(q0);
      a.rowdig[2 * r + 1] = a.np == 1 ? digits1(q1) : digits4(q1);
      if (a.digp)
        for (int p = 0; p < a.np; ++p) {
          a.digp[(int64_t)p * a.n_pad + r] = (uint8_t)(a.rowdig[2 * r] >> (8 * p));
          a.digp[(int64_t)(a.np + p) * a.n_pad + r] = (uint8_t)(a.rowdig[2 * r + 1] >> (8 * p));
        }
    }
    t0 += s0;
    t1 += s1;
  });
  a.totals[0] = t0.load();
  a.totals[1] = t1.load();
}

void slot8_cpu(const SlotArgs& a) {
  parallel_for(a.N, 0, 1 << 16, [&](int64_t lo, int64_t hi) {
    for (int64_t r = lo; r < hi; ++r) {
      const int32_t node = a.row_node[r];
      const int32_t s = ((node >= 0 && node < a.num_nodes) ? a.node_slot[node] : -1) - a.slot_base;
      const uint32_t sb = (s >= 0 && s < a.nslots) ? (uint32_t)s : 0xffu;
      if (a.slot8) a.slot8[r] = (uint8_t)sb;
      if (a.pack) a.pack[r] = sb | ((a.rowdig[2 * r] & 0xffu) << 8) | ((a.rowdig[2 * r + 1] & 0xffu) << 16);
      if (a.masked) {
        a.masked[2 * r] = s == 0 ? a.rowdig[2 * r] : 0u;
        a.masked[2 * r + 1] = s == 0 ? a.rowdig[2 * r + 1] : 0u;
      }
    }
  });
}

void rf_compact_cpu(const RfCompactArgs& a) {
  for (int32_t sh = 0; sh < a.S; ++sh) {
    int64_t acc = 0;
    for (int64_t f = a.fs[sh]; f < a.fs[sh + 1]; ++f)
      if (a.mask[f]) { a.local[f] = acc; acc += a.nbins[f]; }
    for (int64_t f = a.fs[sh]; f < a.fs[sh + 1]; ++f)
      if (!a.mask[f]) a.local[f] = acc;
    a.sizes[sh] = acc;
  }
  a.local[a.Fa] = 0;
}

void rf_sample_cpu(const RfSampleArgs& a) {
  if (a.nnodes <= 0 || a.k >= a.F) return;
  parallel_for(a.nnodes, 0, 1, [&](int64_t lo, int64_t hi) {
    std::vector<uint64_t> u((size_t)a.F);
    for (int64_t i = lo; i < hi; ++i) {
      if (a.nodes[i] < 0) { a.thr[i] = -1.0; continue; }   // padding of a capacity-sized open list
      for (int64_t f = 0; f < a.F; ++f) u[(size_t)f] = feature_priority_u53(a.seed, rf_tree_of(a, i), a.nodes[i], f);
      std::nth_element(u.begin(), u.begin() + (a.k - 1), u.end());
      a.thr[i] = (double)u[(size_t)(a.k - 1)] * (1.0 / 9007199254740992.0);
    }
  });
  parallel_for(a.Fa, 0, 4096, [&](int64_t lo, int64_t hi) {
    for (int64_t f = lo; f < hi; ++f) {
      uint8_t m = 0;
      for (int i = 0; i < a.nnodes && !m; ++i)
        m = a.nodes[i] >= 0 &&
            ((double)feature_priority_u53(a.seed, rf_tree_of(a, i), a.nodes[i], a.fid_orig[f]) * (1.0 / 9007199254740992.0) <=
             a.thr[i]) ? 1 : 0;
      a.mask[f] = m;
    }
  });
}

void hist_cpu(const HistArgs& h, int bt, int np) {
  parallel_for(h.num_items, 0, 4, [&](int64_t lo, int64_t hi) {
    for (int64_t it = lo; it < hi; ++it) {
      if (!item_active(h, it)) continue;
      const int32_t meta = h.item_meta[it];
      const int sl2 = item_stride_log2(meta), nfeat = item_nfeat(meta), koff = item_koff(meta);
      const int32_t f0 = h.item_f0[it];
      for (int64_t e = h.item_start[it]; e < h.item_end[it]; ++e) {
        const int64_t row = h.csc_row[e];
        const int s = h.rowpack ? (int)(h.rowpack[row] & 0xffu) : h.slot8 ? (int)h.slot8[row] : 0;
        if (s >= h.nslots) continue;
        const int node = h.slot_node[s];
        const int key = h.csc_key[e];
        if (node < 0 || key < koff || key >= koff + 16 * bt) continue;
        const int fl = key >> sl2, b = key & ((1 << sl2) - 1);
        if (fl >= nfeat) continue;
        const int f = f0 + fl;
        if (b >= h.nbins[f]) continue;
        const uint32_t* d = h.rowdig + 2 * row;
        int64_t q0 = np == 1 ? undigits1(d[0]) : undigits4(d[0]);
        int64_t q1 = np == 1 ? undigits1(d[1]) : undigits4(d[1]);
        if (h.rowpack) {
          q0 = undigits1((h.rowpack[row] >> 8) & 0xffu);
          q1 = undigits1((h.rowpack[row] >> 16) & 0xffu);
        }
        int64_t* dst = h.hist + ((int64_t)node * h.hist_stride + hist_boff(h, f) + b) * 2;
        __atomic_fetch_add(dst, q0, __ATOMIC_RELAXED);
        __atomic_fetch_add(dst + 1, q1, __ATOMIC_RELAXED);
      }
    }
  });
}

// Row-group CSR build (host twin of rg_build_kernel): sequential, so each (group, row) run keeps
// the CSC order (any order gives the same exact sums).
void rg_build_cpu(const RgBuildArgs& a, int pass) {
  int32_t f = 0;
  for (int64_t e = 0; e < a.nnz; ++e) {
    while (e >= a.colptr[f + 1]) ++f;
    const int32_t g = a.fgroup[f];
    if (g < 0) continue;
    const int64_t r = a.csc_row[e];
    if (pass == 0) {
      a.ptr[(int64_t)g * (a.N + 1) + r + 1] += 1;
    } else {
      const uint32_t pos = a.cursor[(int64_t)g * a.N + r]++;
      a.ent[a.gbase[g] + pos] = (uint16_t)(a.flocal[f] + a.csc_bin[e]);
    }
  }
}

// Host twin of rg_build_csr_kernel: counts per (group, row), exclusive scan per group, placement
// in CSR order (every (group, row) run is written by its row only).
template <class V>
void rg_build_csr_cpu(const RgCsrBuildArgs<V>& a) {
  auto bin_of = [&](V v) {
    int32_t b = 0;
    if (v > (V)0) {
      const double d = (double)v;
      b = d >= 255.0 ? 255 : (int32_t)d;
      b = b < a.max_bin ? b : a.max_bin;
    }
    return b;
  };
  for (int g = 0; g < a.G; ++g) a.ptr[(int64_t)g * (a.N + 1)] = 0;
  parallel_for(a.N, 0, 4096, [&](int64_t lo, int64_t hi) {
    std::vector<uint32_t> c((size_t)a.G);
    for (int64_t r = lo; r < hi; ++r) {
      std::fill(c.begin(), c.end(), 0u);
      for (int64_t e = a.indptr[r]; e < a.indptr[r + 1]; ++e) {
        const int32_t fa = a.remap[a.idx[e]];
        if (fa >= 0 && a.fgroup[fa] >= 0) ++c[(size_t)a.fgroup[fa]];
      }
      for (int g = 0; g < a.G; ++g) a.ptr[(int64_t)g * (a.N + 1) + r + 1] = c[(size_t)g];
    }
  });
  for (int g = 0; g < a.G; ++g) {
    uint32_t* p = a.ptr + (int64_t)g * (a.N + 1);
    for (int64_t r = 0; r < a.N; ++r) p[r + 1] += p[r];
  }
  parallel_for(a.N, 0, 4096, [&](int64_t lo, int64_t hi) {
    std::vector<uint32_t> c((size_t)a.G);
    for (int64_t r = lo; r < hi; ++r) {
      for (int g = 0; g < a.G; ++g) c[(size_t)g] = a.ptr[(int64_t)g * (a.N + 1) + r];
      for (int64_t e = a.indptr[r]; e < a.indptr[r + 1]; ++e) {
        const int32_t fa = a.remap[a.idx[e]];
        if (fa < 0) continue;
        const int32_t g = a.fgroup[fa];
        if (g < 0) continue;
        const int64_t pos = a.gbase[g] + c[(size_t)g]++;
        a.ent[pos] = (uint16_t)(a.flocal[fa] + bin_of(a.counts[e]));
        if (a.erow != nullptr && g >= a.em_g0) a.erow[pos - a.ebase] = (uint32_t)r;
      }
    }
  });
}
template void rg_build_csr_cpu<float>(const RgCsrBuildArgs<float>&);
template void rg_build_csr_cpu<double>(const RgCsrBuildArgs<double>&);
template void rg_build_csr_cpu<int32_t>(const RgCsrBuildArgs<int32_t>&);

// Built rows grouped by slot, ascending inside each slot (the device order inside a 4096-row
// window may differ; the histogram sums do not depend on it).
void rg_list_cpu(const RgListArgs& a) {
  std::vector<int64_t> cnt(a.nslots + 1, 0);
  for (int64_t r = 0; r < a.N; ++r) {
    const uint32_t s = rg_slot_of(a, r);
    if (s < (uint32_t)a.nslots) ++cnt[s + 1];
  }
  for (int s = 0; s < a.nslots; ++s) cnt[s + 1] += cnt[s];
  for (int s = 0; s <= a.nslots; ++s) a.slot_start[s] = (int32_t)cnt[s];
  for (int s = 0; s < a.nslots; ++s) a.slot_count[s] = (int32_t)(cnt[s + 1] - cnt[s]);
  for (int64_t r = 0; r < a.N; ++r) {
    const uint32_t s = rg_slot_of(a, r);
    if (a.masked) {
      a.masked[2 * r] = s == 0u ? a.rowdig[2 * r] : 0u;
      a.masked[2 * r + 1] = s == 0u ? a.rowdig[2 * r + 1] : 0u;
    }
    if (s >= (uint32_t)a.nslots) continue;
    const int64_t pos = cnt[s]++;
    a.list[pos] = (int32_t)r;
    if (a.listdig) {
      a.listdig[2 * pos] = a.rowdig[2 * r];
      a.listdig[2 * pos + 1] = a.rowdig[2 * r + 1];
    }
  }
}

void rg_erow_cpu(const RgErowArgs& a) {
  for (int g = a.g0; g < a.G; ++g) {
    const uint32_t* ptr = a.ptr + (int64_t)g * (a.N + 1);
    uint32_t* out = a.erow + (a.gbase[g] - a.ebase);
    parallel_for(a.N, 0, 65536, [&](int64_t lo, int64_t hi) {
      for (int64_t r = lo; r < hi; ++r)
        for (uint32_t e = ptr[r]; e < ptr[r + 1]; ++e) out[e] = (uint32_t)r;
    });
  }
}

// Host twin of rg_hist_kernel, following the same (group, list chunk, slot) work split, so a host
// test checks that the plan covers every built row of every group exactly once.
void rg_hist_cpu(const RgHistArgs& a) {
  const int64_t T = a.list ? (int64_t)a.slot_start[a.nslots] : a.N;
  parallel_for((int64_t)a.n_wg, 0, 1, [&](int64_t lo_w, int64_t hi_w) {
    for (int64_t w = lo_w; w < hi_w; ++w) {
      const int g = a.wg_g[w], p = a.wg_p[w], np_g = a.wg_np[w];
      const uint32_t* ptr = a.ptr + (int64_t)g * (a.N + 1);
      const uint16_t* ent = a.ent + a.gbase[g];
      if (T > 0 && rg_use_em(a, g, T)) {         // entry-major: chunk p of the group's entries
        const int64_t E = ptr[a.N], e0 = E * p / np_g, e1 = E * (p + 1) / np_g;
        const uint32_t* erow = a.erow + (a.gbase[g] - a.ebase);
        const int64_t hrow = a.slot_node[0];
        for (int64_t e = e0; e < e1 && hrow >= 0; ++e) {
          const int64_t row = erow[e];
          const uint32_t* dig = rg_em_digits(a) + 2 * row;     // (zero outside slot 0 when listed)
          const int32_t col = a.gbin[(int64_t)g * a.gbins + ent[e]];
          if (col < 0) continue;
          const int64_t q0 = rg_q(dig[0], a.np), q1 = rg_q(dig[1], a.np);
          int64_t* dst = a.hist + (hrow * a.hist_stride + rg_col_offset(a, col)) * 2;
          __atomic_fetch_add(dst, q0, __ATOMIC_RELAXED);
          __atomic_fetch_add(dst + 1, q1, __ATOMIC_RELAXED);
        }
        continue;
      }
      const int64_t a0 = T * p / np_g, a1 = T * (p + 1) / np_g;
      int s = 0;
      if (a.list)
        while (s + 1 < a.nslots && a.slot_start[s + 1] <= a0) ++s;
      for (int64_t pos = a0; pos < a1; ++pos) {
        if (a.list)
          while (a.slot_start[s + 1] <= pos) ++s;
        const int64_t hrow = a.slot_node[s];
        if (hrow < 0) continue;
        const int64_t row = a.list ? (int64_t)a.list[pos] : pos;
        const uint32_t* dg = a.list ? a.listdig + 2 * pos : a.rowdig + 2 * row;
        const int64_t q0 = rg_q(dg[0], a.np), q1 = rg_q(dg[1], a.np);
        for (uint32_t i = ptr[row]; i < ptr[row + 1]; ++i) {
          const int32_t col = a.gbin[(int64_t)g * a.gbins + ent[i]];
          if (col < 0) continue;
          int64_t* dst = a.hist + (hrow * a.hist_stride + rg_col_offset(a, col)) * 2;
          __atomic_fetch_add(dst, q0, __ATOMIC_RELAXED);
          __atomic_fetch_add(dst + 1, q1, __ATOMIC_RELAXED);
        }
      }
    }
  });
}

void hist_dense_cpu(const DenseHistArgs& a, int fg, int np) {
  parallel_for((int64_t)a.ngroups * fg, 0, 1, [&](int64_t lo, int64_t hi) {
    for (int64_t t = lo; t < hi; ++t) {
      const int f = a.gfid[t];
      if (f < 0) continue;
      const uint8_t* col = a.dense + (int64_t)a.gdense[t] * a.n_pad;
      for (int64_t row = 0; row < a.n_rows; ++row) {
        const int s = a.slot8 ? (int)a.slot8[row] : 0;
        if (s >= a.nslots) continue;
        const int node = a.slot_node[s];
        const int b = col[row];
        if (node < 0 || b >= a.nbins[f]) continue;
        const uint32_t* d = a.rowdig + 2 * row;
        int64_t* dst = a.hist + ((int64_t)node * a.hist_stride + a.boff[f] + b) * 2;
        __atomic_fetch_add(dst, np == 1 ? undigits1(d[0]) : undigits4(d[0]), __ATOMIC_RELAXED);
        __atomic_fetch_add(dst + 1, np == 1 ? undigits1(d[1]) : undigits4(d[1]), __ATOMIC_RELAXED);
      }
    }
  });
}

void hist_subtract_cpu(const int64_t* parent, int64_t* cur, const int32_t* dst, const int32_t* par, const int32_t* sib,
                       int32_t n_pairs, int64_t TB) {
  const int64_t per = TB * 2;
  for (int p = 0; p < n_pairs; ++p)
    if (dst[p] >= 0)
      for (int64_t k = 0; k < per; ++k)
      cur[(int64_t)dst[p] * per + k] = parent[(int64_t)par[p] * per + k] - cur[(int64_t)sib[p] * per + k];
}

void split_cpu(const SplitArgs& a) {
  const double s0 = std::ldexp(1.0, -a.kexp[0]), s1 = std::ldexp(1.0, -a.kexp[1]);
  parallel_for((int64_t)a.num_nodes * a.Fa, 0, 4096, [&](int64_t lo, int64_t hi) {
    for (int64_t t = lo; t < hi; ++t) {
      const int n = (int)(t / a.Fa), f = (int)(t % a.Fa);
      double gain = -INFINITY;
      int64_t l0 = 0, l1 = 0;
      int bin = -1;
      bool use = a.node_ids[n] >= 0;
      if (use && a.feat_thr)
        use = feature_priority(a.seed, a.node_tree ? a.node_tree[n] : a.tree, a.node_ids[n], a.fid_orig[f]) <=
              a.feat_thr[n];
      if (use) {
        const int64_t* hb = a.hist + (split_row(a, n) * (a.hist_stride ? a.hist_stride : a.boff[a.Fa]) + a.boff[f]) * 2;
        gain = best_split_scan(hb, a.nbins[f], a.zbin[f], a.totals[2 * n], a.totals[2 * n + 1], s0, s1, a.mode,
                               a.lambda_, a.min_child_weight, &bin, &l0, &l1);
      }
      a.out_gain[t] = gain;
      a.out_bin[t] = bin;
      a.out_left[2 * t] = l0;
      a.out_left[2 * t + 1] = l1;
    }
  });
}

void split_best_cpu(const double* gain, const int32_t* bin, const int64_t* left, int32_t nodes, int32_t Fa, int64_t f0,
                    int64_t* out) {
  for (int n = 0; n < nodes; ++n) {
    const double* g = gain + (int64_t)n * Fa;
    double best = -INFINITY;
    int bf = Fa;
    bool nan = false;
    for (int f = 0; f < Fa; ++f) {
      if (std::isnan(g[f])) nan = true;
      else if (g[f] > best) { best = g[f]; bf = f; }
    }
    if (nan) { best = std::nan(""); bf = 0; }
    if (bf >= Fa) bf = 0;
    const int64_t t = (int64_t)n * Fa + bf;
    int64_t* o = out + 5 * (int64_t)n;
    std::memcpy(&o[0], &best, sizeof(double));
    o[1] = bf + f0;
    o[2] = bin[t];
    o[3] = left[2 * t];
    o[4] = left[2 * t + 1];
  }
}

void level_plan_cpu(const LevelPlanArgs& a) { level_plan(a); }
void level_rows_cpu(const LevelRowsArgs& a) {
  for (int32_t k = 0; k < a.nb; ++k) level_rows_slot(a, k);
}

void partition_cols_cpu(const PartitionArgs& a, const int64_t* colptr, const int32_t* cs_feat, const int32_t* n_cs) {
  PartitionArgs d = a;
  d.num_items = 0;
  partition_cpu(d);                                  // default pass
  for (int32_t sp = 0; sp < *n_cs; ++sp) {
    const int32_t dflt = a.split_default[sp], other = a.split_other[sp], thr = a.split_bin[sp];
    const bool left_default = a.split_left_is_default[sp] != 0;
    const int32_t f = cs_feat[sp];
    for (int64_t e = colptr[f]; e < colptr[f + 1]; ++e) {
      const int32_t row = a.csc_row[e];
      const bool left = (int32_t)a.csc_bin[e] <= thr;
      if (left != left_default && a.row_node[row] == dflt) {
        a.row_node[row] = other;
        if (a.pack) a.pack[row] = partition_pack_word(a, other, row);
      }
    }
  }
}

void partition_cpu(const PartitionArgs& a) {
  parallel_for(a.N, 0, 1 << 16, [&](int64_t lo, int64_t hi) {
    for (int64_t r = lo; r < hi; ++r) {
      int32_t n = a.row_node[r];
      if (n >= 0 && n < a.num_nodes) {
        const int32_t c = partition_row_child(a, n, r);
        if (c >= 0) a.row_node[r] = n = c;
      }
      if (a.pack) a.pack[r] = partition_pack_word(a, n, r);
    }
  });
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

void leaf_values_cpu(const int64_t* stats, const int32_t* kexp, int64_t M, double eta, double lambda, double mds,
                     double* out) {
  for (int64_t n = 0; n < M; ++n) out[n] = leaf_value(stats[2 * n], stats[2 * n + 1], kexp[0], kexp[1], eta, lambda, mds);
}

void leaf_update_cpu(double* margin, const int32_t* row_node, const double* node_value, int64_t N) {
  for (int64_t r = 0; r < N; ++r) margin[r] += node_value[row_node[r]];
}

}  // namespace fdx

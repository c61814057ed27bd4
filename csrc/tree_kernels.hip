// Histogram tree engine for gfx950 (K-10..K-15 of SURVEY.md §2.5).
//
// Histogram build on the matrix cores: for one feature column chunk, the per-(bin, node, stat)
// sums are the product  C[bin][col] = sum_k A[bin][k] * B[k][col]  over the chunk's entries k,
// with A = one-hot(bin_k) (exact in bf16) and B[k][col] = (slot_k == node(col)) * stat(col)_k,
// stat split into bf16 hi/lo halves so the fp32-accumulating v_mfma_f32_32x32x16_bf16 yields
// ~fp32-accurate sums (class counts are small integers and exact). One wave per work item,
// 16 entries per MFMA K-step, no atomics, fixed summation order -> deterministic histograms.
// The rest of the level (reduce of chunk partials, sibling subtraction, split search, row
// partition) are small bandwidth-bound kernels.
#include "ops.h"
#include "tree.h"

#pragma clang fp contract(off)

namespace fdx {

namespace {
constexpr int kWave = 64;

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ void lds_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

// ------------------------------------------------------------------ rowstate
__global__ __launch_bounds__(256) void rowstate_kernel(RowStateArgs a) {
  for (int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x; r < a.N; r += (int64_t)gridDim.x * 256) {
    const int32_t node = a.row_node[r];
    const int32_t slot = (node >= 0 && node < a.num_nodes) ? a.node_slot[node] : -1;
    uint4 st;
    st.x = (uint32_t)slot;
    st.w = 0;
    if (slot < 0) {
      st.y = st.z = 0;
    } else if (a.mode == 0) {
      const float w = a.weight ? a.weight[r] : 1.0f;
      st.y = split_bf16(a.g[r] * w);
      st.z = split_bf16(a.h[r] * w);
    } else {
      float w = a.weight ? a.weight[r] : 1.0f;
      if (a.bootstrap) w *= (float)poisson1(hash_uniform(a.seed, (uint64_t)a.tree, (uint64_t)r));
      const float y = a.label[r];
      st.y = split_bf16(w * (1.0f - y));
      st.z = split_bf16(w * y);
    }
    reinterpret_cast<uint4*>(a.rowstate)[r] = st;
  }
}

// ------------------------------------------------------------------ MFMA histogram
template <int BT, int CT>
__global__ __launch_bounds__(256) void hist_mfma_kernel(HistArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t s_bin[4][kWave];
  __shared__ __attribute__((aligned(16))) int8_t s_slot[4][kWave];
  __shared__ __attribute__((aligned(16))) uint16_t s_comp[4][4][kWave];

  const int wid = threadIdx.x / kWave;
  const int lane = threadIdx.x & (kWave - 1);
  const int item = blockIdx.x * 4 + wid;
  if (item >= a.num_items) return;
  const int64_t e0 = a.item_start[item], e1 = a.item_end[item];

  const int col = lane & 31;        // MFMA column / A-row index owned by this lane
  const int half = lane >> 5;       // k half (entries 8*half .. 8*half+7 of each 16-step)
  const int comp = col & 3;         // 0 g_hi, 1 g_lo, 2 h_hi, 3 h_lo
  const int slot_sub = col >> 2;

  f32x16 acc[BT][CT];
#pragma unroll
  for (int bt = 0; bt < BT; ++bt)
#pragma unroll
    for (int ct = 0; ct < CT; ++ct)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[bt][ct][i] = 0.0f;

  for (int64_t base = e0; base < e1; base += kWave) {
    const int64_t e = base + lane;
    uint8_t bin = 0xff;
    int8_t slot = -1;
    uint32_t y = 0, z = 0;
    if (e < e1) {
      const int32_t row = a.csc_row[e];
      bin = a.csc_bin[e];
      const uint4 st = reinterpret_cast<const uint4*>(a.rowstate)[row];
      const int s = (int)st.x - a.slot_base;
      if (s >= 0 && s < 8 * CT) { slot = (int8_t)s; y = st.y; z = st.z; }
    }
    s_bin[wid][lane] = bin;
    s_slot[wid][lane] = slot;
    s_comp[wid][0][lane] = (uint16_t)(y & 0xffffu);
    s_comp[wid][1][lane] = (uint16_t)(y >> 16);
    s_comp[wid][2][lane] = (uint16_t)(z & 0xffffu);
    s_comp[wid][3][lane] = (uint16_t)(z >> 16);
    lds_sync();
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int k0 = ks * 16 + 8 * half;
      const uint64_t bins8 = *reinterpret_cast<const uint64_t*>(&s_bin[wid][k0]);
      const uint64_t slots8 = *reinterpret_cast<const uint64_t*>(&s_slot[wid][k0]);
      const s16x8 cv = *reinterpret_cast<const s16x8*>(&s_comp[wid][comp][k0]);
      bf16x8 A[BT];
#pragma unroll
      for (int bt = 0; bt < BT; ++bt) {
        s16x8 av;
#pragma unroll
        for (int j = 0; j < 8; ++j)
          av[j] = (((bins8 >> (8 * j)) & 0xffu) == (uint64_t)(col + 32 * bt)) ? (short)0x3f80 : (short)0;
        A[bt] = __builtin_bit_cast(bf16x8, av);
      }
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) {
        s16x8 bv;
        const uint64_t want = (uint64_t)(ct * 8 + slot_sub);
#pragma unroll
        for (int j = 0; j < 8; ++j) bv[j] = (((slots8 >> (8 * j)) & 0xffu) == want) ? cv[j] : (short)0;
        const bf16x8 B = __builtin_bit_cast(bf16x8, bv);
#pragma unroll
        for (int bt = 0; bt < BT; ++bt)
          acc[bt][ct] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[bt], B, acc[bt][ct], 0, 0, 0);
      }
    }
    lds_sync();
  }

  // C[row][col]: row = (reg&3) + 8*(reg>>2) + 4*half (+32*bt), col = lane&31.
  // Combine hi+lo halves (adjacent columns) and store [item][slot][bin][stat].
  float* out = a.slab + (int64_t)item * (8 * CT) * (32 * BT) * 2;
#pragma unroll
  for (int bt = 0; bt < BT; ++bt)
#pragma unroll
    for (int ct = 0; ct < CT; ++ct)
#pragma unroll
      for (int reg = 0; reg < 16; ++reg) {
        const float v = acc[bt][ct][reg];
        const float w = __shfl_xor(v, 1, kWave);
        if ((col & 1) == 0) {
          const int row = (reg & 3) + 8 * (reg >> 2) + 4 * half + 32 * bt;
          const int slot = ct * 8 + slot_sub;
          const int stat = (col >> 1) & 1;
          out[((int64_t)slot * (32 * BT) + row) * 2 + stat] = v + w;
        }
      }
}

// v2: U groups of 64 entries are loaded per step (U dependent-gather chains in flight per wave
// instead of one), and MFMA K-steps whose 16 entries belong to no built node are skipped
// (wave-uniform ballot test), which at deep levels removes most of the VALU/MFMA work.
template <int BT, int CT, int U>
__global__ __launch_bounds__(256) void hist_mfma_v2_kernel(HistArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t s_bin[4][U * kWave];
  __shared__ __attribute__((aligned(16))) int8_t s_slot[4][U * kWave];
  __shared__ __attribute__((aligned(16))) uint16_t s_comp[4][4][U * kWave];

  const int wid = threadIdx.x / kWave;
  const int lane = threadIdx.x & (kWave - 1);
  const int item = blockIdx.x * 4 + wid;
  if (item >= a.num_items) return;
  const int64_t e0 = a.item_start[item], e1 = a.item_end[item];

  const int col = lane & 31;
  const int half = lane >> 5;
  const int comp = col & 3;
  const int slot_sub = col >> 2;

  f32x16 acc[BT][CT];
#pragma unroll
  for (int bt = 0; bt < BT; ++bt)
#pragma unroll
    for (int ct = 0; ct < CT; ++ct)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[bt][ct][i] = 0.0f;

  for (int64_t base = e0; base < e1; base += U * kWave) {
    int32_t row[U];
    uint8_t bin[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t e = base + u * kWave + lane;
      row[u] = (e < e1) ? a.csc_row[e] : -1;
      bin[u] = (e < e1) ? a.csc_bin[e] : (uint8_t)0xff;
    }
    uint4 st[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      st[u] = make_uint4(0xffffffffu, 0, 0, 0);
      if (row[u] >= 0) st[u] = reinterpret_cast<const uint4*>(a.rowstate)[row[u]];
    }
    unsigned long long live[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int s = (int)st[u].x - a.slot_base;
      const bool ok = s >= 0 && s < 8 * CT;
      live[u] = __ballot(ok);
      const int k = u * kWave + lane;
      s_bin[wid][k] = bin[u];
      s_slot[wid][k] = ok ? (int8_t)s : (int8_t)-1;
      s_comp[wid][0][k] = ok ? (uint16_t)(st[u].y & 0xffffu) : (uint16_t)0;
      s_comp[wid][1][k] = ok ? (uint16_t)(st[u].y >> 16) : (uint16_t)0;
      s_comp[wid][2][k] = ok ? (uint16_t)(st[u].z & 0xffffu) : (uint16_t)0;
      s_comp[wid][3][k] = ok ? (uint16_t)(st[u].z >> 16) : (uint16_t)0;
    }
    lds_sync();
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (live[u] == 0ull) continue;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        if (((live[u] >> (16 * ks)) & 0xffffull) == 0ull) continue;
        const int k0 = u * kWave + ks * 16 + 8 * half;
        const uint64_t bins8 = *reinterpret_cast<const uint64_t*>(&s_bin[wid][k0]);
        const uint64_t slots8 = *reinterpret_cast<const uint64_t*>(&s_slot[wid][k0]);
        const s16x8 cv = *reinterpret_cast<const s16x8*>(&s_comp[wid][comp][k0]);
        bf16x8 A[BT];
#pragma unroll
        for (int bt = 0; bt < BT; ++bt) {
          s16x8 av;
#pragma unroll
          for (int j = 0; j < 8; ++j)
            av[j] = (((bins8 >> (8 * j)) & 0xffu) == (uint64_t)(col + 32 * bt)) ? (short)0x3f80 : (short)0;
          A[bt] = __builtin_bit_cast(bf16x8, av);
        }
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) {
          s16x8 bv;
          const uint64_t want = (uint64_t)(ct * 8 + slot_sub);
#pragma unroll
          for (int j = 0; j < 8; ++j) bv[j] = (((slots8 >> (8 * j)) & 0xffu) == want) ? cv[j] : (short)0;
          const bf16x8 B = __builtin_bit_cast(bf16x8, bv);
#pragma unroll
          for (int bt = 0; bt < BT; ++bt)
            acc[bt][ct] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[bt], B, acc[bt][ct], 0, 0, 0);
        }
      }
    }
    lds_sync();
  }

  float* out = a.slab + (int64_t)item * (8 * CT) * (32 * BT) * 2;
#pragma unroll
  for (int bt = 0; bt < BT; ++bt)
#pragma unroll
    for (int ct = 0; ct < CT; ++ct)
#pragma unroll
      for (int reg = 0; reg < 16; ++reg) {
        const float v = acc[bt][ct][reg];
        const float w = __shfl_xor(v, 1, kWave);
        if ((col & 1) == 0) {
          const int r = (reg & 3) + 8 * (reg >> 2) + 4 * half + 32 * bt;
          const int slot = ct * 8 + slot_sub;
          const int stat = (col >> 1) & 1;
          out[((int64_t)slot * (32 * BT) + r) * 2 + stat] = v + w;
        }
      }
}

// ------------------------------------------------------------------ reduce chunk partials
__global__ __launch_bounds__(256) void hist_reduce_kernel(HistReduceArgs a) {
  const int64_t tid = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t per_feat = (int64_t)a.slab_slots * a.slab_bins;
  if (tid >= (int64_t)a.L * per_feat) return;
  const int li = (int)(tid / per_feat);
  const int rem = (int)(tid % per_feat);
  const int s = rem / a.slab_bins, b = rem % a.slab_bins;
  const int fid = a.feat[li];
  if (b >= a.nbins[fid]) return;
  const int node = a.slot_to_node[s];
  if (node < 0) return;
  double g = 0.0, h = 0.0;
  const int64_t i0 = a.feat_item0[li];
  for (int i = 0; i < a.feat_nitems[li]; ++i) {
    const float* p = a.slab + ((i0 + i) * per_feat + (int64_t)s * a.slab_bins + b) * 2;
    g += (double)p[0];
    h += (double)p[1];
  }
  double* dst = a.hist + ((int64_t)node * a.total_bins + a.boff[fid] + b) * 2;
  dst[0] = g;
  dst[1] = h;
}

// ------------------------------------------------------------------ sibling subtraction
__global__ __launch_bounds__(256) void hist_subtract_kernel(const double* parent_hist, double* cur_hist,
                                                            const int32_t* dst, const int32_t* par,
                                                            const int32_t* sib, int32_t n_pairs, int64_t TB) {
  const int64_t per = TB * 2;
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < (int64_t)n_pairs * per;
       t += (int64_t)gridDim.x * 256) {
    const int p = (int)(t / per);
    const int64_t k = t % per;
    cur_hist[(int64_t)dst[p] * per + k] = parent_hist[(int64_t)par[p] * per + k] - cur_hist[(int64_t)sib[p] * per + k];
  }
}

// ------------------------------------------------------------------ split search
__global__ __launch_bounds__(256) void split_kernel(SplitArgs a) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= (int64_t)a.num_nodes * a.Fa) return;
  const int n = (int)(t / a.Fa), f = (int)(t % a.Fa);
  double gain = -1.0 / 0.0;
  int bin = -1;
  double l0 = 0, l1 = 0;
  bool use = true;
  if (a.feat_prob < 1.0)
    use = hash_uniform(a.seed ^ 0x5bd1e995ull, ((uint64_t)a.tree << 32) | (uint32_t)a.node_ids[n],
                       (uint64_t)a.fid_orig[f]) < a.feat_prob;
  if (use) {
    const double* hb = a.hist + ((int64_t)n * (a.boff[a.Fa]) + a.boff[f]) * 2;
    gain = best_split_scan(hb, a.nbins[f], a.zbin[f], a.totals[2 * n], a.totals[2 * n + 1], a.mode, a.lambda_,
                           a.min_child_weight, &bin, &l0, &l1);
  }
  a.out_gain[t] = gain;
  a.out_bin[t] = bin;
  a.out_left[2 * t] = l0;
  a.out_left[2 * t + 1] = l1;
}

// ------------------------------------------------------------------ partition
__global__ __launch_bounds__(256) void partition_default_kernel(PartitionArgs a) {
  for (int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x; r < a.N; r += (int64_t)gridDim.x * 256) {
    const int32_t n = a.row_node[r];
    if (n >= 0 && n < a.num_nodes) {
      const int32_t c = a.default_child[n];
      if (c >= 0) a.row_node[r] = c;
    }
  }
}

__global__ __launch_bounds__(256) void partition_column_kernel(PartitionArgs a) {
  const int item = blockIdx.x;
  if (item >= a.num_items) return;
  const int sp = a.item_split[item];
  const int32_t dflt = a.split_default[sp], other = a.split_other[sp];
  const int32_t thr = a.split_bin[sp];
  const bool left_default = a.split_left_is_default[sp] != 0;
  for (int64_t e = a.item_start[item] + threadIdx.x; e < a.item_end[item]; e += 256) {
    const int32_t row = a.csc_row[e];
    const bool left = (int32_t)a.csc_bin[e] <= thr;
    if (left != left_default && a.row_node[row] == dflt) a.row_node[row] = other;
  }
}

// ------------------------------------------------------------------ gbdt helpers
__global__ __launch_bounds__(256) void logistic_grad_kernel(const double* margin, const float* label,
                                                            const float* weight, float* g, float* h, int64_t N) {
  for (int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x; r < N; r += (int64_t)gridDim.x * 256) {
    const double p = 1.0 / (1.0 + exp(-margin[r]));
    const double w = weight ? (double)weight[r] : 1.0;
    g[r] = (float)((p - (double)label[r]) * w);
    h[r] = (float)(fmax(p * (1.0 - p), 1e-16) * w);
  }
}

__global__ __launch_bounds__(256) void leaf_update_kernel(double* margin, const int32_t* row_node,
                                                          const double* node_value, int64_t N) {
  for (int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x; r < N; r += (int64_t)gridDim.x * 256)
    margin[r] += node_value[row_node[r]];
}

inline unsigned grid_for(int64_t n, int64_t cap = 8192) {
  const int64_t b = (n + 255) / 256;
  return (unsigned)(b < 1 ? 1 : (b > cap ? cap : b));
}
}  // namespace

void launch_rowstate(const RowStateArgs& a, hipStream_t s) {
  if (a.N <= 0) return;
  hipLaunchKernelGGL(rowstate_kernel, dim3(grid_for(a.N)), dim3(256), 0, s, a);
}

int hist_kernel_version() {
  static int v = [] {
    const char* e = getenv("FDX_HIST_KERNEL");
    return e ? atoi(e) : 2;
  }();
  return v;
}

void launch_hist_mfma(const HistArgs& a, int bt, int ct, hipStream_t s) {
  if (a.num_items <= 0) return;
  const dim3 grid((a.num_items + 3) / 4), block(256);
  if (hist_kernel_version() == 1) {
#define FDX_HIST_CASE(B, C) \
  if (bt == B && ct == C) { hipLaunchKernelGGL((hist_mfma_kernel<B, C>), grid, block, 0, s, a); return; }
    FDX_HIST_CASE(1, 1) FDX_HIST_CASE(1, 2) FDX_HIST_CASE(1, 4)
    FDX_HIST_CASE(2, 1) FDX_HIST_CASE(2, 2) FDX_HIST_CASE(2, 4)
#undef FDX_HIST_CASE
    return;
  }
#define FDX_HIST2_CASE(B, C) \
  if (bt == B && ct == C) { hipLaunchKernelGGL((hist_mfma_v2_kernel<B, C, 4>), grid, block, 0, s, a); return; }
  FDX_HIST2_CASE(1, 1) FDX_HIST2_CASE(1, 2) FDX_HIST2_CASE(1, 4)
  FDX_HIST2_CASE(2, 1) FDX_HIST2_CASE(2, 2) FDX_HIST2_CASE(2, 4)
#undef FDX_HIST2_CASE
}

void launch_hist_reduce(const HistReduceArgs& a, hipStream_t s) {
  const int64_t n = (int64_t)a.L * a.slab_slots * a.slab_bins;
  if (n <= 0) return;
  hipLaunchKernelGGL(hist_reduce_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, a);
}

void launch_hist_subtract(const double* parent, double* cur, const int32_t* dst, const int32_t* par, const int32_t* sib,
                          int32_t n_pairs, int64_t TB, hipStream_t s) {
  if (n_pairs <= 0 || TB <= 0) return;
  hipLaunchKernelGGL(hist_subtract_kernel, dim3(grid_for((int64_t)n_pairs * TB * 2)), dim3(256), 0, s, parent, cur,
                     dst, par, sib, n_pairs, TB);
}

void launch_split(const SplitArgs& a, hipStream_t s) {
  const int64_t n = (int64_t)a.num_nodes * a.Fa;
  if (n <= 0) return;
  hipLaunchKernelGGL(split_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, a);
}

void launch_partition(const PartitionArgs& a, hipStream_t s) {
  if (a.N > 0) hipLaunchKernelGGL(partition_default_kernel, dim3(grid_for(a.N)), dim3(256), 0, s, a);
  if (a.num_items > 0) hipLaunchKernelGGL(partition_column_kernel, dim3(a.num_items), dim3(256), 0, s, a);
}

void launch_logistic_grad(const double* margin, const float* label, const float* weight, float* g, float* h,
                          int64_t N, hipStream_t s) {
  if (N > 0) hipLaunchKernelGGL(logistic_grad_kernel, dim3(grid_for(N)), dim3(256), 0, s, margin, label, weight, g, h, N);
}

void launch_leaf_update(double* margin, const int32_t* row_node, const double* node_value, int64_t N, hipStream_t s) {
  if (N > 0) hipLaunchKernelGGL(leaf_update_kernel, dim3(grid_for(N)), dim3(256), 0, s, margin, row_node, node_value, N);
}

}  // namespace fdx

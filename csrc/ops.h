// Host-callable entry points of the native core (HIP launchers + CPU implementations).
#pragma once
#include <hip/hip_runtime.h>

#include <stdexcept>

#include "scoring.h"

// host-side argument checks of the launchers (pybind turns the exception into a RuntimeError)
#define FDX_LANES_CHECK(c)                                                     \
  do {                                                                         \
    if (!(c)) throw std::runtime_error("fdx lane-batched launch: " #c);        \
  } while (0)

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

// ---------------------------------------------------------------- feature-major order (sort_kernels.hip)
template <class V>
struct FeatureOrderArgs {
  const int64_t* indptr;      // [rows + 1] CSR
  const int32_t* idx;         // [nnz] feature ids (sorted unique within a row)
  const V* counts;            // [nnz] term counts
  int64_t rows, nnz;
  int32_t F;
  // device scratch (nullptr on the host path)
  int32_t* keys_tmp;
  uint64_t* payload_tmp;
  int32_t* keys_sorted;
  uint64_t* payload_sorted;
  void* temp;
  size_t temp_bytes;
  // outputs
  int32_t* csc_row;           // [nnz] rows, column-major, increasing within a column
  uint8_t* csc_cnt;           // [nnz] min(count, 255) (0 for count <= 0)
  int64_t* colptr;            // [F + 1]
  int64_t* df;                // [F] entries with count > 0 (document frequency)
  int32_t* maxc;              // [F] max min(count, 255)
};
size_t feature_order_temp_bytes(int64_t nnz, int32_t F);
template <class V> void launch_feature_order(const FeatureOrderArgs<V>& a, hipStream_t s);
template <class V> void feature_order_cpu(const FeatureOrderArgs<V>& a);
void launch_clamp_u8(const uint8_t* in, int64_t n, uint8_t maxv, uint8_t* out, hipStream_t s);
void launch_block_bounds(const int32_t* csc_row, const int64_t* colptr, const int32_t* cols, int32_t ncols, int32_t nblk,
                         int64_t row_block, int64_t* bounds, hipStream_t s);
// dense[i * n_pad + row[seg_src[i] + k]] = bin[seg_src[i] + k] for k < seg_len[i] (the hot features'
// dense block; max_len: the longest segment)
void launch_dense_scatter(const int32_t* row, const uint8_t* bin, const int64_t* seg_src, const int64_t* seg_len,
                          int64_t nseg, int64_t max_len, int64_t n_pad, uint8_t* dense, hipStream_t s);
void dense_scatter_cpu(const int32_t* row, const uint8_t* bin, const int64_t* seg_src, const int64_t* seg_len,
                       int64_t nseg, int64_t n_pad, uint8_t* dense);
void launch_copy_segments(const int32_t* src_row, const uint8_t* src_key, const int64_t* seg_src, const int64_t* seg_dst,
                          const int64_t* seg_len, int64_t nseg, const uint8_t* seg_add, int32_t* dst_row, uint8_t* dst_key,
                          hipStream_t s);
void copy_segments_cpu(const int32_t* src_row, const uint8_t* src_key, const int64_t* seg_src, const int64_t* seg_dst,
                       const int64_t* seg_len, int64_t nseg, const uint8_t* seg_add, int32_t* dst_row, uint8_t* dst_key);
void block_bounds_cpu(const int32_t* csc_row, const int64_t* colptr, const int32_t* cols, int32_t ncols, int32_t nblk,
                      int64_t row_block, int64_t* bounds);

// ---------------------------------------------------------------- tree engine (tree_kernels.hip / tree_cpu.cpp)
struct LevelChooseArgs;
struct QuantArgs;
struct SlotArgs;
struct HistArgs;
struct DenseHistArgs;
struct SplitArgs;
struct PartitionArgs;
struct LevelPlanArgs;
struct LevelRowsArgs;
struct RfSampleArgs;
void launch_rf_sample(const RfSampleArgs& a, hipStream_t s);
void rf_sample_cpu(const RfSampleArgs& a);
struct RfCompactArgs;
void launch_rf_compact(const RfCompactArgs& a, hipStream_t s);
// partials: the SplitArgs of the split search whose per-workgroup partials (part_gain) replace
// the full per-feature scan (nullptr / no part_gain: the full scan)
void launch_split_best_plan(const double* gain, const int32_t* bin, const int64_t* left, int32_t nodes, int32_t Fa,
                            int64_t f0, int64_t* out, const LevelPlanArgs& p, unsigned int* ticket, hipStream_t s,
                            const SplitArgs* partials = nullptr);
// entries of SplitArgs part_gain / part_f for a search of nodes x Fa (0: Fa < 64, no partials)
int64_t split_partials(int32_t nodes, int32_t Fa);
struct PrologueInit;
void launch_grad_max(const double* margin, const float* label, float* g, float* h, int64_t N, double* maxv,
                     const PrologueInit& pi, hipStream_t s);
void launch_leaf_update_stats(double* margin, const int32_t* row_node, const int64_t* stats, const int32_t* kexp,
                              double eta, double lambda, double mds, int64_t N, hipStream_t s);
int64_t rf_compact_chunks(int64_t max_shard_features);
void rf_compact_cpu(const RfCompactArgs& a);
// partials: device scratch of 2 x quant_blocks(N) x 8 bytes (per-workgroup results, reduced by a
// second one-block kernel that writes out / totals)
int quant_blocks(int64_t n);
void launch_quant_max(const QuantArgs& a, double* out, void* partials, hipStream_t s);
void launch_quant(const QuantArgs& a, const double* maxv, void* partials, hipStream_t s);
void launch_slot8(const SlotArgs& a, hipStream_t s);
void launch_level_plan(const LevelPlanArgs& a, hipStream_t s);
void launch_level_rows(const LevelRowsArgs& a, hipStream_t s);
void launch_partition_cols(const PartitionArgs& a, const int64_t* colptr, const int32_t* cs_feat, const int32_t* n_cs,
                           int32_t max_splits, int32_t wps, hipStream_t s);
struct SelectArgs;
// lane-batched launches (tree.h "lane-batched launches"): h on the host, d the same array on the device
struct QuantLane;
struct SplitBestLane;
struct SplitBestPlanLane;
struct PartColsLane;
struct RootSendLane;
struct CopyLane;
// 16-byte words (bytes % 16 == 0, both 16-byte aligned) from src (may be a pinned host page's
// device mapping) to dst, on the stream
void launch_stage_copy(void* dst, const void* src, int64_t bytes, hipStream_t s);
void launch_copy_lanes(const CopyLane* h, const CopyLane* d, int L, hipStream_t s);
void launch_root_send_lanes(const RootSendLane* d, int L, hipStream_t s);
void launch_quant_lanes(const QuantLane* h, const QuantLane* d, int L, hipStream_t s);
void launch_hist_lanes(const HistArgs* h, const HistArgs* d, int L, int bt, hipStream_t s);
void launch_split_lanes(const SplitArgs* h, const SplitArgs* d, int L, hipStream_t s);
void launch_split_best_lanes(const SplitBestLane* h, const SplitBestLane* d, int L, hipStream_t s);
void launch_split_best_plan_lanes(const SplitBestPlanLane* h, const SplitBestPlanLane* d, int L, hipStream_t s);
void launch_level_plan_lanes(const LevelPlanArgs* d, int L, hipStream_t s);
void launch_select_groups_lanes(const SelectArgs* h, const SelectArgs* d, int L, hipStream_t s);
void launch_partition_lanes(const PartColsLane* h, const PartColsLane* d, const PartitionArgs* dp, int L,
                            hipStream_t s);
void launch_rf_sample_lanes(const RfSampleArgs* h, const RfSampleArgs* d, int L, hipStream_t s);
void launch_rf_compact_lanes(const RfCompactArgs* h, const RfCompactArgs* d, int L, hipStream_t s);
// the partition's row pass may write the next level's row-list counts (PartitionArgs count_work):
// 512-row list waves and one grid pass over the rows
bool partition_counts_ok(int64_t N);
void launch_level_choose_builds(const LevelChooseArgs& a, hipStream_t s);
void launch_hist_select_groups(const SelectArgs& a, hipStream_t s);
void launch_split_best(const double* gain, const int32_t* bin, const int64_t* left, int32_t nodes, int32_t Fa,
                       int64_t f0, int64_t* out, hipStream_t s, const SplitArgs* partials = nullptr);
void launch_hist(const HistArgs& a, int bt, int ct, int np, hipStream_t s);
void launch_hist_select(const HistArgs& a, hipStream_t s);
struct RgBuildArgs;
struct RgListArgs;
struct RgHistArgs;
void launch_rg_build(const RgBuildArgs& a, int pass, hipStream_t s);
template <class V> struct RgCsrBuildArgs;
template <class V> void launch_rg_build_csr(const RgCsrBuildArgs<V>& a, hipStream_t s);
template <class V> void rg_build_csr_cpu(const RgCsrBuildArgs<V>& a);
int64_t rg_build_csr_waves(int64_t N);
void launch_rg_list(const RgListArgs& a, hipStream_t s);
void launch_rg_hist(const RgHistArgs& a, hipStream_t s);
struct RgErowArgs;
void launch_rg_erow(const RgErowArgs& a, hipStream_t s);
void rg_erow_cpu(const RgErowArgs& a);
void rg_build_cpu(const RgBuildArgs& a, int pass);
void rg_list_cpu(const RgListArgs& a);
void rg_hist_cpu(const RgHistArgs& a);
void launch_hist_dense(const DenseHistArgs& a, int bt, int ct, int np, hipStream_t s);
int dense_features_per_wave(int bt, int ct);
int dense_waves_per_group();
void launch_hist_subtract(const int64_t* parent, int64_t* cur, const int32_t* dst, const int32_t* par,
                          const int32_t* sib, int32_t n_pairs, int64_t TB, hipStream_t s);
void launch_split(const SplitArgs& a, hipStream_t s);
void launch_partition(const PartitionArgs& a, hipStream_t s);
void launch_logistic_grad(const double* margin, const float* label, const float* weight, float* g, float* h,
                          int64_t N, hipStream_t s);
void launch_leaf_values(const int64_t* stats, const int32_t* kexp, int64_t M, double eta, double lambda, double mds,
                        double* out, hipStream_t s);
void leaf_values_cpu(const int64_t* stats, const int32_t* kexp, int64_t M, double eta, double lambda, double mds,
                     double* out);
void launch_leaf_update(double* margin, const int32_t* row_node, const double* node_value, int64_t N, hipStream_t s);
void quant_max_cpu(const QuantArgs& a, double* out);
void quant_cpu(const QuantArgs& a, const double* maxv);
void slot8_cpu(const SlotArgs& a);
void level_plan_cpu(const LevelPlanArgs& a);
void level_rows_cpu(const LevelRowsArgs& a);
void partition_cols_cpu(const PartitionArgs& a, const int64_t* colptr, const int32_t* cs_feat, const int32_t* n_cs);
void split_best_cpu(const double* gain, const int32_t* bin, const int64_t* left, int32_t nodes, int32_t Fa, int64_t f0,
                    int64_t* out);
void hist_cpu(const HistArgs& h, int bt, int np);
void hist_dense_cpu(const DenseHistArgs& a, int fg, int np);
void hist_subtract_cpu(const int64_t* parent, int64_t* cur, const int32_t* dst, const int32_t* par, const int32_t* sib,
                       int32_t n_pairs, int64_t TB);
void split_cpu(const SplitArgs& a);
void partition_cpu(const PartitionArgs& a);
void logistic_grad_cpu(const double* margin, const float* label, const float* weight, float* g, float* h, int64_t N);
void leaf_update_cpu(double* margin, const int32_t* row_node, const double* node_value, int64_t N);

// json_text.cpp
int64_t extract_json_field(const uint8_t* in, const int64_t* in_off, int64_t n, const uint8_t* field, int64_t flen,
                           uint8_t* out, int64_t out_cap, int64_t* out_off, int32_t* status, int threads);
int64_t extract_json_field_ptrs(const uint8_t* const* begin, const int64_t* len, int64_t n, const uint8_t* field,
                                int64_t flen, uint8_t* out, int64_t out_cap, int64_t* out_off, int32_t* status,
                                int threads);

int64_t encode_records(const double* pred, const double* conf, const uint8_t* text, const int64_t* off,
                       const int32_t* skip, int64_t n, uint8_t* out, int64_t cap, int64_t* out_off, int32_t* status,
                       int threads);

template <class V> void score_csr_cpu(const CsrArgs<V>& a, int threads);
template <class V> void spmv_cpu(const int64_t* indptr, const int32_t* idx, const V* val, const double* x, double* y,
                                 int64_t rows, int threads);
template <class V> void spmv_t_cpu(const int64_t* indptr, const int32_t* idx, const V* val, const double* r,
                                   double* g, int64_t rows, int64_t cols, int threads);

}  // namespace fdx

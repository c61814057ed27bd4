// Native per-level driver of the device level loop (models/grower.py device_tree_steps) for the
// RandomForest / DecisionTree class-count trees (np = 1, sampled passes).
//
// A forest level is a handful of small launches (histogram passes per item group, split search,
// best split, level plan, next level's feature sample + data-parallel layout, count copy,
// partition). Driven from Python, each costs a pybind call that converts 10-30 tensor arguments
// plus the interpreter glue between them: ~220 us of host time per tree-level, against a GPU that
// finishes the level's kernels of a 1.25M-row shard (BASELINE config 3 at DP=8) much sooner -- the
// forest was host bound (bench/probes/rf_host_probe.py --forced: ~5 % of the wall blocked on the
// device). An RfLevels object is built once per lane workspace with every buffer that stays put
// (item groups, CSC, node table, level tables, scratch), and a level is three calls -- hist, split,
// tail -- whose arguments are the few per-level tensors. The kernels and their arguments are
// exactly those of the single-purpose bindings (bindings_tree.cpp), so the trees are bitwise the
// same (tests: the device loop with and without the runner, and every DP world size).
#include <torch/extension.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <map>
#include <thread>
#include <unordered_map>
#include <string>
#include <vector>

#include <c10/hip/HIPGuard.h>
#include <c10/hip/HIPStream.h>
#include <dlfcn.h>
#include <rccl/rccl.h>

#include "ops.h"
#include "tree.h"

namespace {

namespace py = pybind11;
using at::Tensor;
using c10::optional;

#define FDX_CHECK(cond, ...) TORCH_CHECK(cond, "fdx.level: ", __VA_ARGS__)

hipStream_t cur_stream(const at::Device& d) { return c10::hip::getCurrentHIPStream(d.index()).stream(); }

Tensor get(const py::dict& c, const char* k) { return c[k].cast<Tensor>(); }

optional<Tensor> get_opt(const py::dict& c, const char* k) {
  if (!c.contains(k) || c[k].is_none()) return c10::nullopt;
  return c[k].cast<Tensor>();
}

template <class T>
T* p(const Tensor& t) { return t.data_ptr<T>(); }

// the split search's per-wave partials for the best-split pass (tree_kernels.hip best_partials)
fdx::BestPartials best_partials(const fdx::SplitArgs& sa) {
  fdx::BestPartials bp{};
  if (sa.part_gain) bp = fdx::BestPartials{sa.part_gain, sa.part_f, sa.wide, sa.wide ? sa.n_wide : 0};
  return bp;
}

// Host wait for a level's event, called with the GIL released: spins on hipEventQuery while the
// wait is short (a level's counts usually arrive within 3-40 us), then yields, then sleeps; raises
// after FDX_LEVEL_TIMEOUT_S (default 600 s) so a hung device never spins forever.
void wait_event(hipEvent_t ev) {
  static const double timeout_s = [] {
    const char* e = std::getenv("FDX_LEVEL_TIMEOUT_S");
    return e ? std::atof(e) : 600.0;
  }();
  using clk = std::chrono::steady_clock;
  const auto t0 = clk::now();
  for (;;) {
    const hipError_t e = hipEventQuery(ev);
    if (e == hipSuccess) return;
    FDX_CHECK(e == hipErrorNotReady, "level event: ", hipGetErrorString(e));
    const double el = std::chrono::duration<double>(clk::now() - t0).count();
    FDX_CHECK(el < timeout_s, "level event still pending after ", timeout_s, " s (FDX_LEVEL_TIMEOUT_S)");
    if (el > 2e-3) std::this_thread::sleep_for(std::chrono::microseconds(50));
    else if (el > 2e-4) std::this_thread::yield();
  }
}

template <class T>
T* p(const optional<Tensor>& t) { return (t && t->defined()) ? t->data_ptr<T>() : nullptr; }

// RCCL called from the runner on the level's stream. The communicator is the process group's own
// (ProcessGroupNCCL._comm_ptr) and the entry points come from the librccl.so instance torch already
// loaded (dlopen RTLD_NOLOAD), so no second RCCL and no second communicator is created; every
// rank issues its collectives from one host thread in the same order as the Python path did.
struct Rccl {
  using RsFn = ncclResult_t (*)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t);
  using AgFn = ncclResult_t (*)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t);
  using ErrFn = const char* (*)(ncclResult_t);
  RsFn rs = nullptr, ar = nullptr;
  AgFn ag = nullptr;
  ErrFn err = nullptr;
  ncclComm_t comm = nullptr;

  bool load(const std::string& lib, int64_t comm_ptr) {
    void* h = dlopen(lib.c_str(), RTLD_NOW | RTLD_NOLOAD);
    if (h == nullptr || comm_ptr == 0) return false;
    rs = reinterpret_cast<RsFn>(dlsym(h, "ncclReduceScatter"));
    ar = reinterpret_cast<RsFn>(dlsym(h, "ncclAllReduce"));
    ag = reinterpret_cast<AgFn>(dlsym(h, "ncclAllGather"));
    err = reinterpret_cast<ErrFn>(dlsym(h, "ncclGetErrorString"));
    comm = reinterpret_cast<ncclComm_t>(comm_ptr);
    return rs && ar && ag && err;
  }
  void check(ncclResult_t r, const char* what) const {
    FDX_CHECK(r == ncclSuccess, what, ": ", err ? err(r) : "rccl error");
  }
};

struct ItemGroup {
  Tensor start, end, f0, meta, wave;
  int bt = 1;
};

// What one lane (tree in flight) of an RfBatch queued during a stage: the launches its per-tree
// calls would have made, kept as argument structs (tree.h "lane-batched launches") and issued by
// RfBatch::flush as ONE launch per position for all the batch's lanes.
enum RecKind : int { kRecQuant, kRecHist, kRecSplit, kRecSplitBest, kRecSplitBestPlan, kRecLevelPlan, kRecRfSample,
                     kRecRfCompact, kRecSelectGroups, kRecPartition, kRecCopy, kRecRootSend };
struct RecCopy {
  void* dst;
  const void* src;
  size_t bytes;
  bool to_host;                  // dst is pinned host memory (written through its device mapping)
};
struct RecEntry {
  int kind;
  int aux;                       // (kRecHist: the group's bt)
  std::vector<uint8_t> bytes;
};
struct LaneRec {
  std::vector<RecEntry> entries;
  template <class T>
  void add(int kind, const T& v, int aux = 0) {
    RecEntry e{kind, aux, std::vector<uint8_t>(sizeof(T))};
    std::memcpy(e.bytes.data(), &v, sizeof(T));
    entries.push_back(std::move(e));
  }
};

class RfLevels {
 public:
  LaneRec* rec_ = nullptr;       // set by RfBatch while it drives this lane: launches are recorded
  const int64_t* plan_root_tot_ = nullptr;   // (RfBatch, DP root level) LevelPlanArgs root_tot
  fdx::LevelPlanArgs plan_base_{};           // plan_args' fixed fields (built on first use)
  bool plan_base_ready_ = false;
  int32_t* counts_ptr_ = nullptr;
  int64_t counts_w_ = 0;
  friend class RfBatch;

  explicit RfLevels(const py::dict& c) {
    for (auto g : c["groups"].cast<py::list>()) {
      auto t = g.cast<py::tuple>();
      ItemGroup ig;
      ig.start = t[0].cast<Tensor>();
      ig.end = t[1].cast<Tensor>();
      ig.f0 = t[2].cast<Tensor>();
      ig.meta = t[3].cast<Tensor>();
      ig.wave = t[4].cast<Tensor>();
      ig.bt = t[5].cast<int>();
      groups_.push_back(ig);
    }
    h_row_ = get_opt(c, "h_row");
    h_key_ = get_opt(c, "h_key");
    csc_row_ = get(c, "csc_row");
    csc_bin_ = get(c, "csc_bin");
    colptr_ = get(c, "colptr");
    nbins_ = get(c, "nbins");
    zbin_ = get(c, "zbin");
    fid_orig_ = get(c, "fid_orig");
    dense_ = get_opt(c, "dense");
    hot_row_ = get_opt(c, "hot_row");
    rowdig_ = get(c, "rowdig");
    rowpack_ = get_opt(c, "rowpack");
    dig16_ = get_opt(c, "dig16");
    if (dig16_) FDX_CHECK(dig16_->scalar_type() == at::kShort && dig16_->numel() >= row_node_.numel() &&
                              reinterpret_cast<uintptr_t>(dig16_->data_ptr()) % 16 == 0, "dig16 [N] int16, 16-byte aligned");
    build_all_ = c["build_all"].cast<bool>();
    for (const char* k : {"arena_stats", "open0", "totals0", "kexp_slot"}) st_[k] = get(c, k);
    row_node_ = get(c, "row_node");
    kexp_ = get(c, "kexp");
    for (const char* k : {"stats", "parent", "left", "right", "feat", "bin", "leaf", "gain", "n_nodes", "counts",
                          "counts_host", "default_child", "cs_feat", "cs_default", "cs_other", "cs_bin",
                          "cs_left_default", "node_slot", "s2n", "sub_dst", "sub_par", "sub_sib"})
      st_[k] = get(c, k);
    node_dense_ = get_opt(c, "node_dense");
    sub_of_ = get_opt(c, "sub_of");
    arena_ = get_opt(c, "arena");
    {
      // the counts' pinned host rows as the device sees them: the plan writes the 4 counts there
      // itself (no D2H copy launch per level); none when the pointer is not mappable
      void* dp = nullptr;
      if (hipHostGetDevicePointer(&dp, st_["counts_host"].data_ptr(), 0) == hipSuccess) counts_host_dev_ = (int32_t*)dp;
      else (void)hipGetLastError();
    }
    wide_ = get_opt(c, "wide");
    fmix_ = get_opt(c, "fmix");
    if (fmix_) FDX_CHECK(fmix_->scalar_type() == at::kLong && fmix_->numel() == c["F"].cast<int64_t>(), "fmix [F] int64");
    mode_ = c["mode"].cast<int>();
    max_depth_ = c["max_depth"].cast<int>();
    min_gain_ = c["min_gain"].cast<double>();
    lambda_ = c["lambda_"].cast<double>();
    mcw_ = c["mcw"].cast<double>();
    seed_ = c["seed"].cast<int64_t>();
    F_ = c["F"].cast<int64_t>();
    k_ = c["k"].cast<int64_t>();
    lds_ = c["lds"].cast<bool>();
    wps_ = c["wps"].cast<int>();
    dev_ = row_node_.device();
    FDX_CHECK(dev_.is_cuda(), "the level runner drives device levels only");
    const int64_t cap = st_["s2n"].numel();
    scratch_ = at::empty({fdx::rf_scratch_bytes(2 * cap)}, row_node_.options().dtype(at::kByte));
    sample_counts_ = at::zeros({3 * 2 * cap}, row_node_.options());     // (left zero by every sample launch)
    ticket_ = at::zeros({4}, row_node_.options());
    // per parity: kRootSlots slots of the max |g|, |h| bit patterns / of the root's sums
    maxv_ = at::zeros({2 * fdx::kRootSlots * fdx::kRootStride}, row_node_.options().dtype(at::kLong));
    root_parts_ = at::zeros({2 * fdx::kRootSlots * fdx::kRootStride}, row_node_.options().dtype(at::kLong));
    parts_ = at::empty({2 * (int64_t)fdx::quant_blocks(row_node_.numel())}, row_node_.options().dtype(at::kLong));
  }

  // Tree prologue, one launch each: quantisation of the row statistics (GBDT: the fused logistic
  // gradient + max |g|, |h| launch first, when margin is given) whose last workgroup reduces the
  // totals and writes the root state (stats[0], the level-0 totals, open[0], the arena's
  // exponents) and row_node = 0 -- what quant_max + 2 reductions + 4 fills / copies did.
  // No grid-wide completion test anywhere (QuantArgs atomic_root): the max |g|, |h| are 64-bit
  // atomic maxima into this round's parity slot of maxv_ (the previous round cleared it), the
  // totals atomic adds into stats[0]. With margin, the first launch also copies the arena image
  // in (arena_init, device) and zeroes the root histogram (zero); without, quant zeroes it and
  // the caller has copied the arena image.
  void prologue(const optional<Tensor>& margin, const optional<Tensor>& g, const optional<Tensor>& h,
                const optional<Tensor>& label, const optional<Tensor>& weight, int64_t tree, bool bootstrap,
                int64_t np, const optional<Tensor>& maxabs, const Tensor& totals, const optional<Tensor>& digp,
                int64_t row0, const optional<Tensor>& zero, const optional<Tensor>& arena_init) {
    c10::hip::HIPGuard guard(dev_.index());
    const hipStream_t s = cur_stream(dev_);
    const int64_t N = row_node_.numel();
    if (zero)
      FDX_CHECK(zero->scalar_type() == at::kLong && zero->is_contiguous() &&
                    reinterpret_cast<uintptr_t>(zero->data_ptr()) % 16 == 0, "zero: contiguous int64, 16-byte aligned");
    const double* maxv = maxabs ? p<double>(*maxabs) : nullptr;
    const unsigned long long* max_parts = nullptr;
    if (margin) {
      FDX_CHECK(g && h && label && !weight && mode_ == 0, "the fused gradient prologue: unweighted GBDT");
      FDX_CHECK(arena_init && arena_ && arena_init->numel() == arena_->numel() && arena_->numel() % 8 == 0,
                "arena image [arena bytes], a multiple of 8");
      fdx::PrologueInit pi{};
      pi.init_src = reinterpret_cast<const uint64_t*>(arena_init->data_ptr());
      pi.init_dst = reinterpret_cast<uint64_t*>(arena_->data_ptr());
      pi.init_n = arena_->numel() / 8;
      if (zero) {
        pi.zero = p<int64_t>(*zero);
        pi.zero_n = zero->numel();
      }
      constexpr int64_t kSet = fdx::kRootSlots * fdx::kRootStride;
      unsigned long long* mv = reinterpret_cast<unsigned long long*>(p<int64_t>(maxv_));
      pi.max_clear = mv + kSet * (1 - parity_);
      fdx::launch_grad_max(p<double>(*margin), p<float>(*label), p<float>(*g), p<float>(*h), N,
                           reinterpret_cast<double*>(mv + kSet * parity_), pi, s);
      max_parts = mv + kSet * parity_;
      // data parallel: the max |g|, |h| slots all-reduced (MAX of the bit patterns of non-negative
      // doubles) before the quantisation reads them, so every rank quantises with one exponent
      if (dp_) dp_all_reduce_max(maxv_.narrow(0, kSet * parity_, kSet), s);
      maxv = nullptr;
      parity_ ^= 1;
    }
    fdx::QuantArgs a{};
    a.g = p<float>(g);
    a.h = p<float>(h);
    a.label = p<float>(label);
    a.weight = p<float>(weight);
    a.seed = (uint64_t)seed_;
    a.tree = (int32_t)tree;
    a.bootstrap = bootstrap ? 1 : 0;
    a.mode = mode_ == 0 ? 0 : 1;
    a.np = (int32_t)np;
    a.N = N;
    a.row0 = row0;
    a.kexp_out = p<int32_t>(kexp_);
    a.rowdig = reinterpret_cast<uint32_t*>(p<int32_t>(rowdig_));
    if (dig16_ && np == 1) a.dig16 = reinterpret_cast<uint16_t*>(dig16_->data_ptr());
    a.totals = p<int64_t>(totals);
    if (digp) {
      a.digp = p<uint8_t>(*digp);
      a.n_pad = digp->size(1);
    }
    constexpr int64_t kSet = fdx::kRootSlots * fdx::kRootStride;
    a.atomic_root = 1;
    a.root_parts = p<int64_t>(root_parts_) + kSet * tparity_;
    a.root_parts_clear = p<int64_t>(root_parts_) + kSet * (1 - tparity_);
    a.max_parts = max_parts;
    root_pending_ = a.root_parts;          // (level 0's split search and plan sum the slots)
    tparity_ ^= 1;
    a.root_open = p<int32_t>(st_["open0"]);
    a.kexp_copy = p<int32_t>(st_["kexp_slot"]);
    a.row_node = p<int32_t>(row_node_);
    if (zero && !margin) {
      a.zero = p<int64_t>(*zero);
      a.zero_n = zero->numel();
    }
    if (rec_) {
      FDX_CHECK(a.atomic_root && maxv == nullptr, "a batched prologue: counts (np 1), atomic root");
      rec_->add(kRecQuant, fdx::QuantLane{a, maxv, reinterpret_cast<unsigned long long*>(p<int64_t>(parts_))});
      return;
    }
    fdx::launch_quant(a, maxv, p<int64_t>(parts_), s);
    C10_HIP_KERNEL_LAUNCH_CHECK();
  }

  ~RfLevels() {
    if (g_ev_) (void)hipEventDestroy(g_ev_);
    for (auto& e : dp_timing_) {
      (void)hipEventDestroy(e.first);
      (void)hipEventDestroy(e.second);
    }
  }
  RfLevels(const RfLevels&) = delete;
  RfLevels& operator=(const RfLevels&) = delete;

  // ---- GBDT trees of one process on the row-group engine: the whole level loop in here --------
  // grower.device_tree_steps' generic loop spends ~33 us of interpreter time per level between the
  // plan's counts and the next level's first launch (profiles/r5/gbdt_host_profile_*.txt), which
  // the GPU sees as idle time at 1M rows. gbdt_root queues level 0 after the prologue; gbdt_levels
  // runs levels 1.. -- wait for the previous plan's event, read its counts from the pinned row the
  // plan wrote, queue row lists + row-group pass + split/plan (sibling subtraction inside) +
  // partition -- with the same kernels and arguments as the Python loop (trees bitwise equal:
  // tests/test_level_runner.py). Buffers are fixed: the level histograms alternate between two
  // tensors (each sized for its parity's widest level), the partition zeroing the next one.
  void gbdt_setup(const py::dict& c) {
    rg_setup(c);
    for (int k = 0; k < 2; ++k) {
      g_hist_[k] = get(c, k ? "hist_b" : "hist_a");
      int64_t need = 1;                     // (level d opens at most 2^d nodes)
      for (int64_t d = k; d < max_depth_; d += 2) need = int64_t{1} << d;
      FDX_CHECK(g_hist_[k].scalar_type() == at::kLong && g_hist_[k].dim() == 3 && g_hist_[k].size(2) == 2 &&
                    g_hist_[k].is_contiguous() && g_hist_[k].size(0) >= need &&
                    reinterpret_cast<uintptr_t>(g_hist_[k].data_ptr()) % 16 == 0,
                "gbdt_setup: hist_a / hist_b [rows >= widest level of the parity, TB, 2] int64");
    }
    gh_.hist_stride = g_hist_[0].size(1);
    FDX_CHECK(g_hist_[1].size(1) == gh_.hist_stride, "gbdt_setup: hist strides");
    g_packed_ = get(c, "packed");
    FDX_CHECK(g_packed_.scalar_type() == at::kLong && g_packed_.dim() == 2 && g_packed_.size(1) == 5 &&
                  g_packed_.is_contiguous() && g_packed_.size(0) >= (int64_t{1} << (max_depth_ - 1)),
              "gbdt_setup: packed [widest level, 5] int64");
    // fewest-rows builds (LevelChooseArgs) where the row lists are counted by their own pass; the
    // partition counts the rows in one grid pass (8 rows a thread, <= 8192 blocks)
    const int64_t N = row_node_.numel();
    g_choose_ = c["choose_rows"].cast<bool>() && (N + 7) / 8 <= 8192ll * 256;
    if (g_choose_ && !g_rows_.defined()) g_rows_ = at::zeros({32 * 64}, row_node_.options());
  }

  // The row-group tables and fixed level buffers shared by the single-process (gbdt_setup) and
  // the data-parallel (gbdt_dp_setup) GBDT level loops.
  void rg_setup(const py::dict& c) {
    const Tensor ptr = get(c, "rg_ptr"), ent = get(c, "rg_ent"), gbase = get(c, "rg_gbase"),
                 gbin = get(c, "rg_gbin"), gmode = get(c, "rg_gmode"), wg = get(c, "rg_wg");
    const int64_t G = ptr.size(0), N = ptr.size(1) - 1;
    FDX_CHECK(N == row_node_.numel() && gbin.dim() == 2 && gbin.size(0) == G && gbase.numel() == G + 1 &&
                  gmode.numel() == G && wg.dim() == 2 && wg.size(0) == 3 && ent.scalar_type() == at::kShort &&
                  reinterpret_cast<uintptr_t>(ent.data_ptr()) % 16 == 0 && !build_all_ && mode_ == 0,
              "gbdt_setup: row groups of this runner's rows, GBDT");
    g_keep_ = {ptr, ent, gbase, gbin, gmode, wg};
    fdx::RgHistArgs& a = gh_;
    a = fdx::RgHistArgs{};
    a.ptr = reinterpret_cast<const uint32_t*>(p<int32_t>(ptr));
    a.ent = reinterpret_cast<const uint16_t*>(ent.data_ptr());
    a.gbase = p<int64_t>(gbase);
    a.gbin = p<int32_t>(gbin);
    a.gbins = (int32_t)gbin.size(1);
    a.G = (int32_t)G;
    a.N = N;
    a.rowdig = reinterpret_cast<const uint32_t*>(p<int32_t>(rowdig_));
    a.np = 4;
    a.gmode = p<uint8_t>(gmode);
    a.wg_g = p<int32_t>(wg);
    a.wg_p = a.wg_g + wg.size(1);
    a.wg_np = a.wg_p + wg.size(1);
    a.n_wg = (int32_t)wg.size(1);
    a.dbg = c["dbg"].cast<int32_t>();
    g_erow_ = get_opt(c, "rg_erow");
    if (g_erow_) {
      a.erow = reinterpret_cast<const uint32_t*>(p<int32_t>(*g_erow_));
      a.ebase = c["rg_ebase"].cast<int64_t>();
    }
    g_emdig_ = get_opt(c, "emdig");
    g_em_min_rows_ = c["em_min_rows"].cast<int64_t>();
    g_part_ = get_opt(c, "rg_part");
    g_wg_first_ = get_opt(c, "rg_wg_first");
    FDX_CHECK(!g_part_ || (g_wg_first_ && g_part_->numel() >= 2 * a.n_wg * (int64_t)a.gbins &&
                           g_wg_first_->numel() == G + 1), "gbdt_setup: part [n_wg, gbins, 2], wg_first [G + 1]");
    // optional: the listed levels' own work table (fewer rows than the root's all-rows pass)
    const optional<Tensor> wl = get_opt(c, "rg_wg_list");
    g_wl_ = {a.wg_g, a.wg_p, a.wg_np, a.n_wg};
    g_wg_first_list_ = g_wg_first_;
    if (wl) {
      FDX_CHECK(wl->dim() == 2 && wl->size(0) == 3 && wl->scalar_type() == at::kInt, "rg_wg_list [3, n_wg] int32");
      g_keep_.push_back(*wl);
      g_wl_.g = p<int32_t>(*wl);
      g_wl_.p = g_wl_.g + wl->size(1);
      g_wl_.np = g_wl_.p + wl->size(1);
      g_wl_.n = (int32_t)wl->size(1);
      g_wg_first_list_ = get_opt(c, "rg_wg_first_list");
      FDX_CHECK(!g_part_ || (g_wg_first_list_ && g_wg_first_list_->numel() == G + 1 &&
                             g_part_->numel() >= 2 * g_wl_.n * (int64_t)a.gbins), "rg_wg_first_list / part size");
    }
    g_list_work_ = get(c, "list_work");
    g_rg_start_ = get(c, "rg_start");
    g_rg_list_ = get(c, "rg_list");
    g_rg_listdig_ = get(c, "rg_listdig");
    const int64_t nwaves = (N + fdx::rg_list_rows(N) - 1) / fdx::rg_list_rows(N);
    FDX_CHECK(g_list_work_.numel() >= fdx::kRgMaxSlots * (2 + nwaves) && g_rg_list_.numel() >= N &&
                  g_rg_start_.numel() >= fdx::kRgMaxSlots + 1 && g_rg_listdig_.numel() >= 2 * N,
              "gbdt_setup: row-list buffers");
    fdx::RgListArgs& l = gl_;
    l = fdx::RgListArgs{};
    l.row_node = p<int32_t>(row_node_);
    l.node_slot = p<int32_t>(st_["node_slot"]);
    l.num_nodes = (int32_t)st_["node_slot"].numel();
    l.N = N;
    l.slot_count = p<int32_t>(g_list_work_);
    l.slot_start = p<int32_t>(g_rg_start_);
    l.list = p<int32_t>(g_rg_list_);
    l.rowdig = reinterpret_cast<const uint32_t*>(p<int32_t>(rowdig_));
    l.listdig = reinterpret_cast<uint32_t*>(p<int32_t>(g_rg_listdig_));
    g_one_ = get(c, "one");
    g_zero1_ = get(c, "zero1");
    g_open_[0] = st_["open0"];
    g_open_[1] = get(c, "open1");
    g_totals_[0] = st_["totals0"];
    g_totals_[1] = get(c, "totals1");
    g_boff_ = get(c, "boff");
    g_wide_ = get_opt(c, "wide");
    g_counted_ok_ = c["counted"].cast<bool>() && fdx::partition_counts_ok(N);
    // where the partition does not write the row lists' per-slot counts (above 4M rows: 2048-row
    // list waves), it keeps its rows per next-level node per 512-row chunk (PartitionArgs
    // node_counts) and the lists skip their counting pass over row_node
    const bool nc = !g_counted_ok_ && (c.contains("node_counts") ? c["node_counts"].cast<bool>() : true) &&
                    fdx::rg_list_rows(N) % fdx::kPartWaveRows == 0;
    g_node_counts_ = nc ? at::empty({64 * ((N + fdx::kPartWaveRows - 1) / fdx::kPartWaveRows)}, row_node_.options())
                        : Tensor();
    nc_base_ = nullptr;
    g_part_multi_ = c["part_multi"].cast<bool>();
    FDX_CHECK(sub_of_.has_value() && counts_host_dev_ != nullptr, "gbdt_setup: sub_of and mapped counts");
    if (!g_ev_) FDX_CHECK(hipEventCreateWithFlags(&g_ev_, hipEventDisableTiming) == hipSuccess, "event");
  }

  // Level 0 of a tree whose prologue just ran (its root histogram: hist_a row 0, zeroed there).
  void gbdt_root(int64_t tree) {
    FDX_CHECK(g_ev_ != nullptr, "gbdt_root before gbdt_setup");
    c10::hip::HIPGuard guard(dev_.index());
    const hipStream_t s = cur_stream(dev_);
    gbdt_level(0, 1, 1, tree, s);
  }

  // Levels 1 .. max_depth - 1; returns (n_open, n_build) of every level run, the root's first.
  std::vector<int64_t> gbdt_levels(int64_t tree) {
    c10::hip::HIPGuard guard(dev_.index());
    const hipStream_t s = cur_stream(dev_);
    std::vector<int64_t> shape{1, 1};
    const Tensor& ch = st_["counts_host"];
    const int64_t cw = ch.size(1);
    for (int64_t d = 1; d < max_depth_; ++d) {
      wait_event(g_ev_);
      const volatile int32_t* row = p<int32_t>(ch) + (d - 1) * cw;     // (written by the plan itself)
      const int32_t n_open = row[1], n_build = row[2];
      if (n_open == 0) break;
      FDX_CHECK(n_open <= g_hist_[d & 1].size(0) && n_build >= 1 && n_build <= fdx::kRgMaxSlots && n_build <= n_open,
                "level counts");
      gbdt_level(d, n_open, n_build, tree, s);
      shape.push_back(n_open);
      shape.push_back(n_build);
    }
    return shape;
  }

  // ---- GBDT trees under data parallelism: the same level loop around the level's collectives ----
  // A DP level (grower.device_tree_steps' shards branch, launch for launch): the row-group pass
  // writes the built nodes' partial histograms straight into the shard-major send buffer, ONE
  // reduce-scatter (callback rs) leaves this rank's feature shard of them in out[cur], the split
  // search runs over the shard (the larger siblings subtracted inside it, rows from level_rows),
  // ONE all-gather (callback ag) of the best-split tuples feeds the level plan (best over shards),
  // then the partition zeroes the next level's send region on the way. The root totals ride in the
  // root's reduce-scatter (dp_root phase 0 / 1) and the quantisation max is one all-reduce (callback
  // mx, inside prologue()): 13 collectives per depth-6 tree. The callbacks are Python (the process
  // group's collectives on the current stream); every other launch and the host waits are here.
  // Sibling choice by rows is off: rows are rank-local, and every rank must build the same nodes.
  void gbdt_dp_setup(const py::dict& c) {
    rg_setup(c);
    dp_ = true;
    dp_rs_cb_ = c["rs"];
    dp_ag_cb_ = c["ag"];
    dp_max_cb_ = c["mx"];
    dp_S_ = c["S"].cast<int64_t>();
    dp_Bs_ = c["Bs"].cast<int64_t>();
    dp_bin_lo_ = get(c, "bin_lo");
    dp_send_ = get(c, "send");
    for (int k = 0; k < 2; ++k) {
      dp_out_[k] = get(c, k ? "out_b" : "out_a");
      dp_row_of_[k] = get(c, k ? "row_of1" : "row_of0");
    }
    dp_ag_in_ = get(c, "ag_in");
    dp_boff_ = get(c, "sboff");
    dp_nbins_ = get(c, "snbins");
    dp_zbin_ = get(c, "szbin");
    dp_fid_ = get(c, "sfid");
    dp_f0_ = c["f0"].cast<int64_t>();
    dp_wide_ = get_opt(c, "swide");
    dp_dst_row_ = get(c, "dst_row");
    dp_par_row_ = get(c, "par_row");
    dp_sib_row_ = get(c, "sib_row");
    dp_iota_ = get(c, "iota");
    dp_direct_ = c.contains("comm") && !c["comm"].is_none() &&
                 rccl_.load(c["rccl_lib"].cast<std::string>(), c["comm"].cast<int64_t>());
    const int64_t widest = int64_t{1} << std::max<int64_t>(max_depth_ - 1, 1);
    FDX_CHECK(dp_S_ >= 1 && dp_Bs_ >= 1 && dp_bin_lo_.numel() == dp_S_ + 1 && dp_bin_lo_.scalar_type() == at::kLong,
              "gbdt_dp_setup: S, Bs, bin_lo [S + 1]");
    FDX_CHECK(dp_send_.scalar_type() == at::kLong && dp_send_.is_contiguous() &&
                  dp_send_.numel() >= dp_S_ * std::max<int64_t>(widest, 2) * dp_Bs_ * 2 &&
                  reinterpret_cast<uintptr_t>(dp_send_.data_ptr()) % 16 == 0,
              "gbdt_dp_setup: send [S * max(2, widest level) * Bs * 2] int64");
    for (int k = 0; k < 2; ++k)
      FDX_CHECK(dp_out_[k].scalar_type() == at::kLong && dp_out_[k].dim() == 3 && dp_out_[k].size(1) == dp_Bs_ &&
                    dp_out_[k].size(2) == 2 && dp_out_[k].is_contiguous() && dp_out_[k].size(0) >= std::max<int64_t>(widest, 2) &&
                    dp_row_of_[k].numel() >= widest,
                "gbdt_dp_setup: out [max(2, widest level), Bs, 2], row_of");
    FDX_CHECK(dp_ag_in_.scalar_type() == at::kLong && dp_ag_in_.dim() == 2 && dp_ag_in_.size(1) == 5 &&
                  dp_ag_in_.size(0) >= widest && dp_iota_.numel() >= fdx::kRgMaxSlots &&
                  dp_boff_.numel() == dp_nbins_.numel() + 1,
              "gbdt_dp_setup: ag_in [widest, 5], iota, shard tables");
    if (dp_direct_) dp_allt_buf_ = at::empty({dp_S_ * widest * 5}, dp_ag_in_.options());
  }

  // The direct-RCCL collectives issued so far (reduce-scatter, all-gather, all-reduce) and the
  // milliseconds of the timed ones (every 8th, scaled; events resolved here: call after a sync
  // point, e.g. once per fit); the counters restart.
  std::vector<double> dp_coll_stats() {
    double ms = 0.0;
    for (auto& e : dp_timing_) {
      float t = 0.f;
      if (hipEventSynchronize(e.second) == hipSuccess && hipEventElapsedTime(&t, e.first, e.second) == hipSuccess)
        ms += 8.0 * t;
      (void)hipEventDestroy(e.first);
      (void)hipEventDestroy(e.second);
    }
    dp_timing_.clear();
    std::vector<double> out{(double)dp_calls_[0], (double)dp_calls_[1], (double)dp_calls_[2], ms};
    dp_calls_[0] = dp_calls_[1] = dp_calls_[2] = 0;
    return out;
  }

  bool dp_direct() const { return dp_direct_; }

  // Prologue (with its max all-reduce) done by the caller; level 0 of a DP tree.
  void gbdt_dp_root(int64_t tree) {
    FDX_CHECK(dp_ && g_ev_ != nullptr, "gbdt_dp_root before gbdt_dp_setup");
    c10::hip::HIPGuard guard(dev_.index());
    gbdt_dp_level(0, 1, 1, tree, cur_stream(dev_));
  }

  // Levels 1 .. max_depth - 1 of a DP tree (host waits with the GIL released; the collective
  // callbacks take it back); returns (n_open, n_build) of every level, the root's first.
  std::vector<int64_t> gbdt_dp_levels(int64_t tree) {
    c10::hip::HIPGuard guard(dev_.index());
    const hipStream_t s = cur_stream(dev_);
    std::vector<int64_t> shape{1, 1};
    const Tensor& ch = st_["counts_host"];
    const int64_t cw = ch.size(1);
    for (int64_t d = 1; d < max_depth_; ++d) {
      {
        py::gil_scoped_release nogil;
        wait_event(g_ev_);
      }
      const volatile int32_t* row = p<int32_t>(ch) + (d - 1) * cw;
      const int32_t n_open = row[1], n_build = row[2];
      if (n_open == 0) break;
      FDX_CHECK(n_open <= dp_ag_in_.size(0) && n_build >= 1 && n_build <= fdx::kRgMaxSlots && n_build <= n_open,
                "dp level counts");
      gbdt_dp_level(d, n_open, n_build, tree, s);
      shape.push_back(n_open);
      shape.push_back(n_build);
    }
    dp_allt_ = Tensor();
    return shape;
  }

  // GBDT leaf update from the node table (leaf_values + leaf_update in one launch)
  void leaf_update(const Tensor& margin, double eta, double lambda, double mds) {
    c10::hip::HIPGuard guard(dev_.index());
    fdx::launch_leaf_update_stats(p<double>(margin), p<int32_t>(row_node_), p<int64_t>(st_["stats"]), p<int32_t>(kexp_),
                                  eta, lambda, mds, row_node_.numel(), cur_stream(dev_));
    C10_HIP_KERNEL_LAUNCH_CHECK();
  }

  // Histogram passes of level d over every item group (tree_hist_sampled per group): hist [*, stride, 2]
  // accumulated at node rows s2n[slot]; pack: the packed row state (None at the root); lists[j] /
  // counts[j] / npx[j]: group j's listed pass (None: a wave per item slot; npx -1: compacted here).
  void hist(int64_t n_build, const Tensor& hist, const Tensor& boff, const Tensor& feat_mask, const Tensor& s2n,
            const optional<Tensor>& pack, const std::vector<optional<Tensor>>& lists,
            const std::vector<optional<Tensor>>& counts, const std::vector<int64_t>& npx,
            const optional<Tensor>& shard_of, int64_t shard_bins) {
    FDX_CHECK(lists.size() == groups_.size() && counts.size() == groups_.size() && npx.size() == groups_.size(),
              "one list / count / npx per item group");
    FDX_CHECK(hist.dim() == 3 && hist.size(2) == 2 && hist.scalar_type() == at::kLong, "hist [rows, stride, 2] int64");
    FDX_CHECK(boff.numel() == nbins_.numel() + 1 && feat_mask.numel() == nbins_.numel(), "boff [Fa + 1], mask [Fa]");
    FDX_CHECK(n_build >= 1 && n_build <= 8 * 8 && s2n.numel() >= n_build, "slots");
    FDX_CHECK(h_row_.has_value() && h_key_.has_value(), "the CSC passes need the histogram CSC");
    const int ct = pass_ct(n_build);
    c10::hip::HIPGuard guard(dev_.index());
    const hipStream_t s = cur_stream(dev_);
    for (size_t j = 0; j < groups_.size(); ++j) {
      const ItemGroup& g = groups_[j];
      const int64_t I = g.start.numel();
      if (I == 0) continue;
      fdx::HistArgs a{};
      a.listed_per_xcd = -1;
      a.item_start = p<int64_t>(g.start);
      a.item_end = p<int64_t>(g.end);
      a.item_f0 = p<int32_t>(g.f0);
      a.item_meta = p<int32_t>(g.meta);
      a.num_items = (int32_t)I;
      a.csc_row = p<int32_t>(*h_row_);
      a.csc_key = p<uint8_t>(*h_key_);
      a.rowdig = reinterpret_cast<const uint32_t*>(p<int32_t>(rowdig_));
      a.boff = p<int64_t>(boff);
      a.nbins = p<int32_t>(nbins_);
      a.slot_node = p<int32_t>(s2n);
      a.nslots = (int32_t)n_build;
      a.hist_stride = hist.size(1);
      a.hist = p<int64_t>(hist);
      a.wave_item = p<int32_t>(g.wave);
      a.num_slots = (int32_t)g.wave.numel();
      a.feat_active = p<uint8_t>(feat_mask);
      if (shard_of) {
        FDX_CHECK(shard_of->numel() == boff.numel(), "shard_of [Fa + 1]");
        a.shard_of = p<int64_t>(*shard_of);
        a.shard_bins = shard_bins;
      }
      if (pack) a.rowpack = reinterpret_cast<const uint32_t*>(p<int32_t>(*pack));
      if (lists[j]) {
        FDX_CHECK(counts[j].has_value(), "a listed pass needs its count");
        const int64_t cap = ((a.num_slots + 3) / 4 + 7) / 8 * 4;
        FDX_CHECK(lists[j]->numel() >= 8 * cap && counts[j]->numel() >= 8 && npx[j] <= cap, "list / count sizes");
        a.active_list = p<int32_t>(*lists[j]);
        a.active_count = p<int32_t>(*counts[j]);
        a.list_cap = (int32_t)cap;
        a.listed_per_xcd = (int32_t)npx[j];
      }
      a.lds = (lds_ && 4 * 16 * g.bt * n_build * 8 <= 65536) ? 1 : 0;
      if (rec_) {
        FDX_CHECK(a.lds, "batched histogram passes: the LDS-atomic kernel");
        rec_->add(kRecHist, a, g.bt);
        continue;
      }
      fdx::launch_hist(a, g.bt, ct, 1, s);
    }
    C10_HIP_KERNEL_LAUNCH_CHECK();
  }

  // Split search of the open nodes (split_find + split_best): hist rows [nodes, stride, 2] (row_of:
  // a node's row; None: node i = row i), best tuples into out [nodes, 5] with features + f0.
  void split(const Tensor& hist, const Tensor& totals, const Tensor& boff, const Tensor& nbins, const Tensor& zbin,
             const Tensor& fid_orig, const Tensor& node_ids, const optional<Tensor>& feat_thr, int64_t tree, int64_t f0,
             const Tensor& out, const optional<Tensor>& row_of, const optional<Tensor>& wide) {
    c10::hip::HIPGuard guard(dev_.index());
    const hipStream_t s = cur_stream(dev_);
    const int32_t nodes = (int32_t)node_ids.numel(), Fa = (int32_t)nbins.numel();
    if (!find(hist, totals, boff, nbins, zbin, fid_orig, node_ids, feat_thr, tree, out, row_of, wide, s)) return;
    if (rec_) {
      rec_->add(kRecSplitBest, fdx::SplitBestLane{p<double>(gain_), p<int32_t>(sbin_), p<int64_t>(sleft_), nodes, Fa, f0,
                                                  p<int64_t>(out), best_partials(last_split_)});
      return;
    }
    fdx::launch_split_best(p<double>(gain_), p<int32_t>(sbin_), p<int64_t>(sleft_), nodes, Fa, f0, p<int64_t>(out), s,
                           &last_split_);
    C10_HIP_KERNEL_LAUNCH_CHECK();
  }

  // split_find into the runner's scratch (gain_, sbin_, sleft_); false when there is nothing to
  // search (out then holds "no candidate" tuples for every node)
  bool find(const Tensor& hist, const Tensor& totals, const Tensor& boff, const Tensor& nbins, const Tensor& zbin,
            const Tensor& fid_orig, const Tensor& node_ids, const optional<Tensor>& feat_thr, int64_t tree,
            const Tensor& out, const optional<Tensor>& row_of, const optional<Tensor>& wide, hipStream_t s) {
    const int32_t nodes = (int32_t)node_ids.numel(), Fa = (int32_t)nbins.numel();
    FDX_CHECK(out.numel() == 5ll * nodes && out.is_contiguous() && boff.numel() == Fa + 1, "out [nodes, 5], boff");
    FDX_CHECK(hist.dim() == 3 && hist.size(2) == 2 && (row_of || hist.size(0) >= nodes), "hist rows");
    if (nodes == 0) return false;
    if (Fa == 0) {                         // a shard without features: no candidate anywhere
      const double ninf = -1.0 / 0.0;
      int64_t bits;
      std::memcpy(&bits, &ninf, sizeof(double));
      Tensor o = out.view({nodes, 5});
      o.zero_();
      o.select(1, 0).fill_(bits);
      o.narrow(1, 1, 2).fill_(-1);
      return false;
    }
    const int64_t need = (int64_t)nodes * Fa;
    if (!gain_.defined() || gain_.numel() < need) {
      gain_ = at::empty({need}, out.options().dtype(at::kDouble));
      sbin_ = at::empty({need}, out.options().dtype(at::kInt));
      sleft_ = at::empty({2 * need}, out.options().dtype(at::kLong));
    }
    // (the row stride always comes from hist: a compact DP level's boff[Fa] is the next shard's
    // offset, not this shard's bin total, so the kernels' boff[Fa] fallback must never be taken)
    FDX_CHECK(hist.size(1) > 0, "hist rows of at least one bin");
    fdx::SplitArgs a{};
    a.hist = p<int64_t>(hist);
    a.totals = p<int64_t>(totals);
    a.hist_stride = hist.size(1);
    a.num_nodes = nodes;
    a.Fa = Fa;
    a.boff = p<int64_t>(boff);
    a.nbins = p<int32_t>(nbins);
    a.zbin = p<int32_t>(zbin);
    a.fid_orig = p<int64_t>(fid_orig);
    a.node_ids = p<int32_t>(node_ids);
    a.kexp = p<int32_t>(kexp_);
    a.mode = mode_;
    a.lambda_ = lambda_;
    a.min_child_weight = mcw_;
    a.feat_thr = p<double>(feat_thr);
    a.seed = (uint64_t)seed_;
    a.tree = (int32_t)tree;
    if (fmix_ && feat_thr) a.fmix = reinterpret_cast<const uint64_t*>(p<int64_t>(*fmix_));
    a.out_gain = p<double>(gain_);
    a.out_bin = p<int32_t>(sbin_);
    a.out_left = p<int64_t>(sleft_);
    if (wide && wide->numel() > 0) {
      a.wide = p<int32_t>(*wide);
      a.n_wide = (int32_t)wide->numel();
    }
    a.row_of = p<int32_t>(row_of);
    a.root_parts = find_root_;
    if (find_prev_) {
      a.parent_hist = find_prev_;
      a.sub_of = p<int32_t>(*sub_of_);
      // (data-parallel levels: the subtraction triples as rows, LevelRowsArgs par_row / sib_row)
      a.sub_par = find_sub_par_ ? find_sub_par_ : p<int32_t>(st_["sub_par"]);
      a.sub_sib = find_sub_sib_ ? find_sub_sib_ : p<int32_t>(st_["sub_sib"]);
    }
    const int64_t np_ = fdx::split_partials(nodes, Fa);
    if (np_ > 0) {
      if (!part_gain_.defined() || part_gain_.numel() < np_) {
        part_gain_ = at::empty({np_}, out.options().dtype(at::kDouble));
        part_f_ = at::empty({np_}, out.options().dtype(at::kInt));
      }
      a.part_gain = p<double>(part_gain_);
      a.part_f = p<int32_t>(part_f_);
    }
    if (rec_) rec_->add(kRecSplit, a);
    else fdx::launch_split(a, s);
    last_split_ = a;
    return true;
  }

  fdx::LevelPlanArgs plan_args(int64_t d, int64_t n_open, const Tensor& packed, const Tensor& open,
                               const Tensor& n_open_ptr, const Tensor& next_open, const Tensor& next_totals) {
    if (!plan_base_ready_) {               // (the node table and level tables never move: once)
      fdx::LevelPlanArgs& a = plan_base_;
      a = fdx::LevelPlanArgs{};
      a.max_depth = max_depth_;
      a.mode = mode_;
      a.build_all = build_all_ ? 1 : 0;
      a.kexp = p<int32_t>(kexp_);
      a.min_gain = min_gain_;
      a.zbin = p<int32_t>(zbin_);
      a.hot_row = p<int32_t>(hot_row_);
      a.max_nodes = (int32_t)st_["parent"].numel();
      a.n_nodes = p<int32_t>(st_["n_nodes"]);
      a.stats = p<int64_t>(st_["stats"]);
      a.parent = p<int32_t>(st_["parent"]);
      a.left = p<int32_t>(st_["left"]);
      a.right = p<int32_t>(st_["right"]);
      a.feat = p<int32_t>(st_["feat"]);
      a.bin = p<int32_t>(st_["bin"]);
      a.leaf = p<uint8_t>(st_["leaf"]);
      a.gain = p<double>(st_["gain"]);
      a.default_child = p<int32_t>(st_["default_child"]);
      a.node_dense = p<int32_t>(node_dense_);
      a.cs_feat = p<int32_t>(st_["cs_feat"]);
      a.cs_default = p<int32_t>(st_["cs_default"]);
      a.cs_other = p<int32_t>(st_["cs_other"]);
      a.cs_bin = p<int32_t>(st_["cs_bin"]);
      a.cs_left_default = p<int32_t>(st_["cs_left_default"]);
      a.node_slot = p<int32_t>(st_["node_slot"]);
      a.s2n = p<int32_t>(st_["s2n"]);
      a.sub_dst = p<int32_t>(st_["sub_dst"]);
      a.sub_par = p<int32_t>(st_["sub_par"]);
      a.sub_sib = p<int32_t>(st_["sub_sib"]);
      a.sub_of = p<int32_t>(sub_of_);
      counts_ptr_ = p<int32_t>(st_["counts"]);
      counts_w_ = st_["counts"].size(1);
      plan_base_ready_ = true;
    }
    fdx::LevelPlanArgs a = plan_base_;
    a.packed = p<int64_t>(packed);
    a.L = (int32_t)n_open;
    a.n_shards = packed.dim() == 3 ? (int32_t)packed.size(0) : 1;
    a.shard_stride = packed.dim() == 3 ? packed.stride(0) : packed.size(-2) * 5;
    FDX_CHECK(packed.size(-1) == 5 && packed.stride(-1) == 1 && packed.stride(-2) == 5 && packed.size(-2) >= n_open,
              "packed rows of 5");
    a.depth = (int32_t)d;
    a.open = p<int32_t>(open);
    a.n_open = p<int32_t>(n_open_ptr);
    a.counts = counts_ptr_ + d * counts_w_;
    a.next_open = p<int32_t>(next_open);
    a.next_totals = p<int64_t>(next_totals);
    a.root_tot = plan_root_tot_;
    return a;
  }

  // Level plan of level d (tree.h level_plan) from the best tuples packed [L, 5] / [S, L, 5]; then
  // the after-plan work of after_plan().
  void plan(int64_t d, int64_t n_open, const Tensor& packed, const Tensor& open, const Tensor& n_open_ptr,
            const Tensor& next_open, const Tensor& next_totals, int64_t tree, bool sample_next,
            const optional<Tensor>& thr, const optional<Tensor>& mask, const optional<Tensor>& fs,
            const optional<Tensor>& nbins_all, const optional<Tensor>& local, const optional<Tensor>& sizes,
            const optional<Tensor>& sizes_host, int64_t max_shard_features,
            const std::vector<optional<Tensor>>& sel_lists) {
    c10::hip::HIPGuard guard(dev_.index());
    const hipStream_t s = cur_stream(dev_);
    fdx::LevelPlanArgs a = plan_args(d, n_open, packed, open, n_open_ptr, next_open, next_totals);
    const bool zc = counts_zero_copy(a, d, sample_next, sel_lists);
    if (rec_) rec_->add(kRecLevelPlan, a);
    else fdx::launch_level_plan(a, s);
    after_plan(d, n_open, next_open, tree, sample_next, thr, mask, fs, nbins_all, local, sizes, sizes_host,
               max_shard_features, sel_lists, s, zc);
  }

  // The plan writes the level's counts into the host-mapped row itself unless the per-XCD
  // item counts of a preselected next level follow it (then one D2H copy of the whole row).
  bool counts_zero_copy(fdx::LevelPlanArgs& a, int64_t d, bool sample_next,
                        const std::vector<optional<Tensor>>& sel_lists) const {
    bool sel = false;
    for (const auto& l : sel_lists) sel = sel || l.has_value();
    if (sample_next && sel) {               // the select's per-XCD counts, zeroed by the plan
      int64_t n_sel = 0;
      for (const auto& l : sel_lists) n_sel += l ? 1 : 0;
      a.counts_tail = (int32_t)(8 * n_sel);
    }
    if (counts_host_dev_ == nullptr || (sample_next && sel)) return false;
    a.counts_host = counts_host_dev_ + d * st_.at("counts").size(1);
    return true;
  }

  // Split search + best split + level plan with no collective between them (split_all_kernel, then
  // split_best_plan_kernel: the last node's workgroup plans the level), then after_plan().
  void split_plan(int64_t d, int64_t n_open, const Tensor& hist, const Tensor& totals, const Tensor& boff,
                  const optional<Tensor>& feat_thr, int64_t tree, const Tensor& out, const optional<Tensor>& wide,
                  const Tensor& open, const Tensor& n_open_ptr, const Tensor& next_open, const Tensor& next_totals,
                  bool sample_next, const optional<Tensor>& thr, const optional<Tensor>& mask,
                  const std::vector<optional<Tensor>>& sel_lists, const optional<Tensor>& prev_hist) {
    c10::hip::HIPGuard guard(dev_.index());
    const hipStream_t s = cur_stream(dev_);
    const int32_t Fa = (int32_t)nbins_.numel();
    if (prev_hist) {          // this level's sibling subtraction inside the search (SplitArgs sub_of)
      FDX_CHECK(sub_of_.has_value() && d > 0 && prev_hist->scalar_type() == at::kLong && prev_hist->dim() == 3 &&
                    prev_hist->size(1) == hist.size(1), "prev_hist [rows, stride, 2] int64 with sub_of");
      find_prev_ = p<int64_t>(*prev_hist);
    }
    FDX_CHECK(open.numel() == n_open, "open [n_open]");
    const int64_t* root = d == 0 ? root_pending_ : nullptr;
    root_pending_ = nullptr;
    find_root_ = root;
    const bool any = find(hist, totals, boff, nbins_, zbin_, fid_orig_, open, feat_thr, tree, out, c10::nullopt, wide, s);
    find_root_ = nullptr;
    find_prev_ = nullptr;
    fdx::LevelPlanArgs a = plan_args(d, n_open, out, open, n_open_ptr, next_open, next_totals);
    a.root_parts = root;
    const bool zc = counts_zero_copy(a, d, sample_next, sel_lists);
    if (rec_ && any)
      rec_->add(kRecSplitBestPlan,
                fdx::SplitBestPlanLane{fdx::SplitBestLane{p<double>(gain_), p<int32_t>(sbin_), p<int64_t>(sleft_),
                                                          (int32_t)n_open, Fa, 0, p<int64_t>(out),
                                                          best_partials(last_split_)},
                                       a, reinterpret_cast<unsigned int*>(p<int32_t>(ticket_)) + 2});
    else if (rec_)
      rec_->add(kRecLevelPlan, a);
    else if (any)
      fdx::launch_split_best_plan(p<double>(gain_), p<int32_t>(sbin_), p<int64_t>(sleft_), (int32_t)n_open, Fa, 0,
                                  p<int64_t>(out), a, reinterpret_cast<unsigned int*>(p<int32_t>(ticket_)) + 2, s,
                                  &last_split_);
    else                                   // (no features: out holds "no candidate" tuples)
      fdx::launch_level_plan(a, s);
    after_plan(d, n_open, next_open, tree, sample_next, thr, mask, c10::nullopt, c10::nullopt, c10::nullopt,
               c10::nullopt, c10::nullopt, 0, sel_lists, s, zc);
  }

  // The k-of-F feature sample of the (-1 padded) nodes [nnodes] into thr / mask, then the compact
  // DP layout (local / sizes, sizes copied to sizes_host) when given.
  void sample_level(const Tensor& nodes, int64_t nnodes, int64_t tree, const optional<Tensor>& thr,
                    const optional<Tensor>& mask, const optional<Tensor>& fs, const optional<Tensor>& nbins_all,
                    const optional<Tensor>& local, const optional<Tensor>& sizes, const optional<Tensor>& sizes_host,
                    int64_t max_shard_features, hipStream_t s) {
    FDX_CHECK(thr && mask, "a next-level sample needs thr and mask");
    fdx::RfSampleArgs r{};
    r.seed = (uint64_t)seed_;
    r.tree = (int32_t)tree;
    r.nodes = p<int32_t>(nodes);
    r.nnodes = (int32_t)nnodes;
    r.F = F_;
    r.k = k_;
    r.fid_orig = p<int64_t>(fid_orig_);
    r.Fa = fid_orig_.numel();
    r.thr = p<double>(*thr);
    r.mask = p<uint8_t>(*mask);
    FDX_CHECK(nodes.numel() >= nnodes && thr->numel() >= nnodes && mask->numel() == r.Fa &&
                  scratch_.numel() >= fdx::rf_scratch_bytes(r.nnodes), "next-level sample sizes");
    r.scratch = p<uint8_t>(scratch_);
    r.fused_counts = reinterpret_cast<uint32_t*>(p<int32_t>(sample_counts_));
    r.fused_cap = (int32_t)(sample_counts_.numel() / 3);
    if (fmix_) r.fmix = reinterpret_cast<const uint64_t*>(p<int64_t>(*fmix_));
    if (rec_) rec_->add(kRecRfSample, r);
    else fdx::launch_rf_sample(r, s);
    if (local) {
      fdx::RfCompactArgs cp{};
      cp.mask = p<uint8_t>(*mask);
      cp.nbins = p<int32_t>(*nbins_all);
      cp.fs = p<int64_t>(*fs);
      cp.S = (int32_t)(fs->numel() - 1);
      cp.Fa = mask->numel();
      cp.local = p<int64_t>(*local);
      cp.sizes = p<int64_t>(*sizes);
      if (max_shard_features > 0) {
        cp.chunk_stride = fdx::rf_compact_chunks(max_shard_features);
        if (!chunk_sums_.defined() || chunk_sums_.numel() < cp.S * cp.chunk_stride)
          chunk_sums_ = at::empty({cp.S * cp.chunk_stride}, local->options());
        cp.chunk_sums = p<int64_t>(chunk_sums_);
      }
      if (rec_) {
        rec_->add(kRecRfCompact, cp);
        rec_->add(kRecCopy, RecCopy{sizes_host->data_ptr(), sizes->data_ptr(), (size_t)sizes->nbytes(), true});
      } else {
        fdx::launch_rf_compact(cp, s);
        FDX_CHECK(hipMemcpyAsync(sizes_host->data_ptr(), sizes->data_ptr(), sizes->nbytes(), hipMemcpyDeviceToHost,
                                 s) == hipSuccess, "sizes copy");
      }
    }
  }

  // For a next level: its feature sample over the (-1 padded) next open list into thr / mask, the
  // compact DP layout (local / sizes, sizes copied to sizes_host) when given, and the per-group
  // active-item lists (sel_lists / counts[d, 4:]); then the level's counts to counts_host[d].
  void after_plan(int64_t d, int64_t n_open, const Tensor& next_open, int64_t tree, bool sample_next,
                  const optional<Tensor>& thr, const optional<Tensor>& mask, const optional<Tensor>& fs,
                  const optional<Tensor>& nbins_all, const optional<Tensor>& local, const optional<Tensor>& sizes,
                  const optional<Tensor>& sizes_host, int64_t max_shard_features,
                  const std::vector<optional<Tensor>>& sel_lists, hipStream_t s, bool counts_written) {
    const Tensor& counts = st_["counts"];
    const int64_t cw = counts.size(1);
    int32_t* counts_d = p<int32_t>(counts) + d * cw;
    if (sample_next) {
      FDX_CHECK(next_open.numel() >= 2 * n_open, "next-level sample: the open list");
      sample_level(next_open, 2 * n_open, tree, thr, mask, fs, nbins_all, local, sizes, sizes_host, max_shard_features, s);
      if (!sel_lists.empty()) {
        // per-XCD counts of the selected groups (the non-None lists, in group order) at counts[d, 4 + 8 js]
        int64_t n_sel = 0;
        for (const auto& l : sel_lists) n_sel += l ? 1 : 0;
        FDX_CHECK(sel_lists.size() == groups_.size() && cw >= 4 + 8 * n_sel && n_sel <= fdx::kSelGroups,
                  "select lists");
        // (counts[d, 4:] zeroed by the plan: LevelPlanArgs counts_tail)
        fdx::SelectArgs sa{};
        sa.feat_active = p<uint8_t>(*mask);
        for (size_t j = 0; j < groups_.size(); ++j) {
          if (!sel_lists[j]) continue;
          const ItemGroup& g = groups_[j];
          const int k = sa.n++;
          sa.item_f0[k] = p<int32_t>(g.f0);
          sa.item_meta[k] = p<int32_t>(g.meta);
          sa.wave_item[k] = p<int32_t>(g.wave);
          sa.num_items[k] = (int32_t)g.start.numel();
          sa.num_slots[k] = (int32_t)g.wave.numel();
          sa.list_cap[k] = (int32_t)(((sa.num_slots[k] + 3) / 4 + 7) / 8 * 4);
          sa.list[k] = p<int32_t>(*sel_lists[j]);
          sa.count[k] = counts_d + 4 + 8 * k;
        }
        if (rec_) rec_->add(kRecSelectGroups, sa);
        else fdx::launch_hist_select_groups(sa, s);
      }
    }
    if (counts_written) {
      C10_HIP_KERNEL_LAUNCH_CHECK();
      return;
    }
    const Tensor& ch = st_["counts_host"];
    if (rec_) {
      rec_->add(kRecCopy, RecCopy{p<int32_t>(ch) + d * cw, counts_d, cw * sizeof(int32_t), true});
      return;
    }
    FDX_CHECK(hipMemcpyAsync(p<int32_t>(ch) + d * cw, counts_d, cw * sizeof(int32_t), hipMemcpyDeviceToHost, s) ==
                  hipSuccess, "counts copy");
    C10_HIP_KERNEL_LAUNCH_CHECK();
  }

  // Partition of level d (tree_partition_cols), writing the next level's packed row state when fuse
  // (its count digits from dig16 when this tree's prologue ran here and wrote them: dig16).
  void partition(int64_t d, int64_t n_open, bool fuse, const optional<Tensor>& zero, bool dig16,
                 const optional<Tensor>& count_work) {
    c10::hip::HIPGuard guard(dev_.index());
    const hipStream_t s = cur_stream(dev_);
    fdx::PartitionArgs a{};
    a.row_node = p<int32_t>(row_node_);
    a.default_child = p<int32_t>(st_["default_child"]);
    a.num_nodes = (int32_t)st_["default_child"].numel();
    a.N = row_node_.numel();
    a.split_default = p<int32_t>(st_["cs_default"]);
    a.split_other = p<int32_t>(st_["cs_other"]);
    a.split_bin = p<int32_t>(st_["cs_bin"]);
    a.split_left_is_default = p<int32_t>(st_["cs_left_default"]);
    a.csc_row = p<int32_t>(csc_row_);
    a.csc_bin = p<uint8_t>(csc_bin_);
    if (node_dense_) {
      a.node_dense = p<int32_t>(node_dense_);
      a.dense = p<uint8_t>(dense_);
      a.n_pad = dense_->size(1);
    }
    if (fuse) {
      FDX_CHECK(rowpack_.has_value(), "a fused partition writes the packed row state");
      a.pack_slot = p<int32_t>(st_["node_slot"]);
      a.pack_dig = reinterpret_cast<const uint32_t*>(p<int32_t>(rowdig_));
      if (dig16_ && dig16) a.pack_dig16 = reinterpret_cast<const uint16_t*>(dig16_->data_ptr());
      a.pack = reinterpret_cast<uint32_t*>(p<int32_t>(*rowpack_));
    }
    if (zero) {
      FDX_CHECK(zero->scalar_type() == at::kLong && zero->is_contiguous() && zero->numel() % 2 == 0 &&
                    reinterpret_cast<uintptr_t>(zero->data_ptr()) % 16 == 0, "zero: contiguous int64, 16-byte aligned");
      a.zero = p<int64_t>(*zero);
      a.zero_n = zero->numel();
    }
    const Tensor& counts = st_["counts"];
    a.node_parent = p<int32_t>(st_["parent"]);    // (column pass first: the row pass sees final nodes)
    a.count_ballot = 2 * n_open <= 4 ? 1 : 0;        // (next-level nodes: at most 2 n_open)
    if (rows_base_) {                                // (GBDT levels: rows per next-level node)
      a.rows_base = rows_base_;
      if (rows_choose_) a.rows_out = p<int32_t>(g_rows_);
      if (g_node_counts_.defined()) a.node_counts = p<int32_t>(g_node_counts_);
    }
    if (count_work) {                                // the next level's row-list counts (RgListArgs pass 0)
      FDX_CHECK(fdx::partition_counts_ok(a.N) && count_work->scalar_type() == at::kInt, "row-list counts: N / work");
      a.count_work = p<int32_t>(*count_work);
      a.count_slot = p<int32_t>(st_["node_slot"]);
      a.count_nslots = p<int32_t>(counts) + d * counts.size(1) + 2;
    }
    if (rec_) {
      rec_->add(kRecPartition, fdx::PartColsLane{a, p<int64_t>(colptr_), p<int32_t>(st_["cs_feat"]),
                                                 p<int32_t>(counts) + d * counts.size(1), (int32_t)n_open, (int32_t)wps_});
      return;
    }
    fdx::launch_partition_cols(a, p<int64_t>(colptr_), p<int32_t>(st_["cs_feat"]), p<int32_t>(counts) + d * counts.size(1),
                               (int32_t)n_open, (int32_t)wps_, s);
    C10_HIP_KERNEL_LAUNCH_CHECK();
  }

 private:
  static int pass_ct(int64_t n) {
    int ct = 1;
    while (ct * 8 < n) ct *= 2;          // 8 slots per 16-column tile at np = 1 (grower.pass_ct)
    return ct;
  }

  // One GBDT level (the generic loop's rg branch + split_plan + partition, launch for launch).
  void gbdt_level(int64_t d, int32_t n_open, int32_t n_build, int64_t tree, hipStream_t s) {
    const int cur = (int)(d & 1), nxt = cur ^ 1;
    const bool more = d + 1 < max_depth_;
    const Tensor& hist = g_hist_[cur];
    fdx::RgHistArgs a = gh_;
    a.hist = p<int64_t>(hist);
    a.nslots = n_build;
    if (d == 0) {
      a.slot_node = p<int32_t>(g_zero1_);
    } else {
      // the built rows grouped by slot (pass 0's per-wave counts from the last partition when
      // counted); a single built node also gets every row's digit words zeroed outside it
      const bool em = n_build == 1 && g_emdig_.has_value();
      fdx::RgListArgs l = gl_;
      l.nslots = n_build;
      l.wave_count = l.slot_count + 2 * n_build;
      l.counted = g_counted_ ? 1 : 0;
      l.masked = em ? reinterpret_cast<uint32_t*>(p<int32_t>(*g_emdig_)) : nullptr;
      if (nc_base_ != nullptr) {                  // (the last partition's counts per node)
        l.node_counts = p<int32_t>(g_node_counts_);
        l.nc_base = nc_base_;
      }
      fdx::launch_rg_list(l, s);
      a.list = l.list;
      a.slot_start = l.slot_start;
      a.listdig = l.listdig;
      a.slot_node = p<int32_t>(st_["s2n"]);
      a.wg_g = g_wl_.g;
      a.wg_p = g_wl_.p;
      a.wg_np = g_wl_.np;
      a.n_wg = g_wl_.n;
      if (a.erow && em) {
        a.emdig = l.masked;
        a.em_min_rows = g_em_min_rows_;
      }
    }
    if (g_part_ && (n_build == 1 || g_part_multi_)) {
      a.part = p<int64_t>(*g_part_);
      a.wg_first = p<int32_t>(d == 0 ? *g_wg_first_ : *g_wg_first_list_);
    }
    fdx::launch_rg_hist(a, s);
    C10_HIP_KERNEL_LAUNCH_CHECK();
    const Tensor n_open_ptr = d == 0 ? g_one_ : st_["counts"].select(0, d - 1).narrow(0, 1, 1);
    const optional<Tensor> prev = d == 0 ? optional<Tensor>() : optional<Tensor>(g_hist_[nxt]);
    split_plan(d, n_open, hist.narrow(0, 0, n_open),
               d == 0 ? st_["stats"].narrow(0, 0, 1) : g_totals_[cur].narrow(0, 0, n_open), g_boff_, c10::nullopt,
               tree, g_packed_.narrow(0, 0, n_open), g_wide_, g_open_[cur].narrow(0, 0, n_open), n_open_ptr,
               g_open_[nxt], g_totals_[nxt], false, c10::nullopt, c10::nullopt, {}, prev);
    FDX_CHECK(hipEventRecord(g_ev_, s) == hipSuccess, "level event record");
    optional<Tensor> zero;
    if (more) {
      FDX_CHECK(2 * (int64_t)n_open <= g_hist_[nxt].size(0), "next level rows");
      zero = g_hist_[nxt].narrow(0, 0, 2 * (int64_t)n_open);
    }
    g_counted_ = more && g_counted_ok_;
    const bool choose = more && g_choose_ && !g_counted_;
    const Tensor& counts = st_["counts"];
    const int32_t* base = d == 0 ? p<int32_t>(g_one_) : p<int32_t>(counts) + (d - 1) * counts.size(1) + 3;
    // (per-node counts cover the next level's first 64 nodes: 2 n_open of them)
    const bool nc = more && !g_counted_ && g_node_counts_.defined() && 2 * (int64_t)n_open <= 64;
    rows_base_ = choose || nc ? base : nullptr;   // (read by partition())
    rows_choose_ = choose;
    partition(d, n_open, false, zero, false, g_counted_ ? optional<Tensor>(g_list_work_) : c10::nullopt);
    rows_base_ = nullptr;
    rows_choose_ = false;
    nc_base_ = nc ? base : nullptr;
    if (choose) {
      fdx::LevelChooseArgs ca{};
      ca.counts = p<int32_t>(counts) + d * counts.size(1);
      ca.rows_base = base;
      ca.rows_out = p<int32_t>(g_rows_);
      ca.next_open = p<int32_t>(g_open_[nxt]);
      ca.node_slot = p<int32_t>(st_["node_slot"]);
      ca.s2n = p<int32_t>(st_["s2n"]);
      ca.sub_dst = p<int32_t>(st_["sub_dst"]);
      ca.sub_sib = p<int32_t>(st_["sub_sib"]);
      ca.sub_of = p<int32_t>(sub_of_);
      fdx::launch_level_choose_builds(ca, s);
      C10_HIP_KERNEL_LAUNCH_CHECK();
    }
  }

  void gbdt_dp_level(int64_t d, int32_t n_open, int32_t n_build, int64_t tree, hipStream_t s) {
    const int cur = (int)(d & 1), nxt = cur ^ 1;
    const bool more = d + 1 < max_depth_;
    const int64_t S = dp_S_, Bs = dp_Bs_;
    const int64_t R = n_build + (d == 0 ? 1 : 0), subs = d == 0 ? 0 : n_build;   // (root: + the totals row)
    const int64_t chunk = R * Bs;
    FDX_CHECK(R + subs <= dp_out_[cur].size(0) && S * chunk * 2 <= dp_send_.numel(), "dp level rows");
    Tensor send = dp_send_.narrow(0, 0, S * chunk * 2).view({S, R, Bs, 2});
    const Tensor& out = dp_out_[cur];
    // the built nodes' partial histograms, shard-major (slot k -> row k of every shard chunk)
    fdx::RgHistArgs a = gh_;
    a.hist = p<int64_t>(send);
    a.hist_stride = Bs;
    a.nslots = n_build;
    a.nshards = (int32_t)S;
    a.shard_lo = p<int64_t>(dp_bin_lo_);
    a.shard_stride = chunk;
    if (d == 0) {
      a.slot_node = p<int32_t>(g_zero1_);
    } else {
      const bool em = n_build == 1 && g_emdig_.has_value();
      fdx::RgListArgs l = gl_;
      l.nslots = n_build;
      l.wave_count = l.slot_count + 2 * n_build;
      l.counted = g_counted_ ? 1 : 0;
      l.masked = em ? reinterpret_cast<uint32_t*>(p<int32_t>(*g_emdig_)) : nullptr;
      if (nc_base_ != nullptr) {                  // (the last partition's counts per node)
        l.node_counts = p<int32_t>(g_node_counts_);
        l.nc_base = nc_base_;
      }
      fdx::launch_rg_list(l, s);
      a.list = l.list;
      a.slot_start = l.slot_start;
      a.listdig = l.listdig;
      a.slot_node = p<int32_t>(dp_iota_);
      a.wg_g = g_wl_.g;
      a.wg_p = g_wl_.p;
      a.wg_np = g_wl_.np;
      a.n_wg = g_wl_.n;
      if (a.erow && em) {
        a.emdig = l.masked;
        a.em_min_rows = g_em_min_rows_;
      }
    }
    if (g_part_ && (n_build == 1 || g_part_multi_)) {
      a.part = p<int64_t>(*g_part_);
      a.wg_first = p<int32_t>(d == 0 ? *g_wg_first_ : *g_wg_first_list_);
    }
    if (d == 0) {                 // (+ the local root sums into the totals row of every shard chunk)
      FDX_CHECK(root_pending_ != nullptr, "dp root level without its prologue");
      a.root_parts = root_pending_;
      root_pending_ = nullptr;
    }
    fdx::launch_rg_hist(a, s);
    C10_HIP_KERNEL_LAUNCH_CHECK();
    dp_reduce_scatter(send, out.narrow(0, 0, R), s);
    if (d > 0) {
      // the built rows stay where the collective wrote them, the larger siblings behind them (rows
      // written by the previous level's plan: LevelPlanArgs lr_*), subtracted inside the search
      find_prev_ = p<int64_t>(dp_out_[nxt]);
      find_sub_par_ = p<int32_t>(dp_par_row_);
      find_sub_sib_ = p<int32_t>(dp_sib_row_);
    }
    // split search over this rank's features (+ the fused subtraction), best tuples into ag_in
    Tensor ag_in = dp_ag_in_.narrow(0, 0, n_open);
    const Tensor open = g_open_[cur].narrow(0, 0, n_open);
    // (the root's totals: the reduced totals row)
    const Tensor totals = d == 0 ? out.select(0, R - 1).narrow(0, 0, 1) : g_totals_[cur].narrow(0, 0, n_open);
    const bool any = find(out, totals, dp_boff_, dp_nbins_, dp_zbin_, dp_fid_, open, c10::nullopt, tree, ag_in,
                          d > 0 ? optional<Tensor>(dp_row_of_[cur]) : c10::nullopt, dp_wide_, s);
    find_prev_ = nullptr;
    find_sub_par_ = find_sub_sib_ = nullptr;
    if (any)
      fdx::launch_split_best(p<double>(gain_), p<int32_t>(sbin_), p<int64_t>(sleft_), n_open,
                             (int32_t)dp_nbins_.numel(), dp_f0_, p<int64_t>(ag_in), s, &last_split_);
    C10_HIP_KERNEL_LAUNCH_CHECK();
    dp_allt_ = dp_all_gather(ag_in, s);                  // [S, n_open, 5]
    FDX_CHECK(dp_allt_.dim() == 3 && dp_allt_.size(0) == S && dp_allt_.size(1) == n_open && dp_allt_.is_contiguous(),
              "all-gathered best splits [S, n_open, 5]");
    const Tensor n_open_ptr = d == 0 ? g_one_ : st_["counts"].select(0, d - 1).narrow(0, 1, 1);
    fdx::LevelPlanArgs pa = plan_args(d, n_open, dp_allt_, open, n_open_ptr, g_open_[nxt], g_totals_[nxt]);
    if (d == 0) pa.root_tot = p<int64_t>(totals);
    if (more) {                   // the next level's histogram rows
      pa.lr_prev = d > 0 ? p<int32_t>(dp_row_of_[cur]) : nullptr;
      pa.lr_row_of = p<int32_t>(dp_row_of_[nxt]);
      pa.lr_dst = p<int32_t>(dp_dst_row_);
      pa.lr_par = p<int32_t>(dp_par_row_);
      pa.lr_sib = p<int32_t>(dp_sib_row_);
    }
    const bool zc = counts_zero_copy(pa, d, false, {});
    fdx::launch_level_plan(pa, s);
    after_plan(d, n_open, g_open_[nxt], tree, false, c10::nullopt, c10::nullopt, c10::nullopt, c10::nullopt,
               c10::nullopt, c10::nullopt, c10::nullopt, 0, {}, s, zc);
    FDX_CHECK(hipEventRecord(g_ev_, s) == hipSuccess, "level event record");
    // the partition zeroes the next level's send region (its builds <= this level's open nodes)
    optional<Tensor> zero;
    if (more) zero = dp_send_.narrow(0, 0, S * n_open * Bs * 2);
    g_counted_ = more && g_counted_ok_;
    const bool nc = more && !g_counted_ && g_node_counts_.defined() && 2 * (int64_t)n_open <= 64;
    const int32_t* base = d == 0 ? p<int32_t>(g_one_) : p<int32_t>(st_["counts"]) + (d - 1) * st_["counts"].size(1) + 3;
    rows_base_ = nc ? base : nullptr;
    partition(d, n_open, false, zero, false, g_counted_ ? optional<Tensor>(g_list_work_) : c10::nullopt);
    rows_base_ = nullptr;
    nc_base_ = nc ? base : nullptr;
  }

  // timing events around every 8th direct collective (dp_coll_stats)
  struct CollTimer {
    RfLevels* r;
    hipStream_t s;
    hipEvent_t b = nullptr;
    CollTimer(RfLevels* r_, hipStream_t s_, int kind) : r(r_), s(s_) {
      ++r->dp_calls_[kind];
      if ((r->dp_timed_++ & 7) == 0 && hipEventCreate(&b) == hipSuccess) (void)hipEventRecord(b, s);
    }
    ~CollTimer() {
      hipEvent_t e = nullptr;
      if (b && hipEventCreate(&e) == hipSuccess && hipEventRecord(e, s) == hipSuccess) r->dp_timing_.emplace_back(b, e);
    }
  };

  void dp_reduce_scatter(const Tensor& send, const Tensor& out, hipStream_t s) {
    if (!dp_direct_) {
      dp_rs_cb_(send, out);
      return;
    }
    CollTimer t(this, s, 0);
    rccl_.check(rccl_.rs(send.data_ptr(), out.data_ptr(), (size_t)out.numel(), ncclInt64, ncclSum, rccl_.comm, s),
                "ncclReduceScatter");
  }

  Tensor dp_all_gather(const Tensor& in, hipStream_t s) {
    if (!dp_direct_) return dp_ag_cb_(in).cast<Tensor>();
    CollTimer t(this, s, 1);
    Tensor out = dp_allt_buf_.narrow(0, 0, dp_S_ * in.numel()).view({dp_S_, in.size(0), in.size(1)});
    rccl_.check(rccl_.ag(in.data_ptr(), out.data_ptr(), (size_t)in.numel(), ncclInt64, rccl_.comm, s), "ncclAllGather");
    return out;
  }

  void dp_all_reduce_max(const Tensor& buf, hipStream_t s) {
    if (!dp_direct_) {
      dp_max_cb_(buf);
      return;
    }
    CollTimer t(this, s, 2);
    rccl_.check(rccl_.ar(buf.data_ptr(), buf.data_ptr(), (size_t)buf.numel(), ncclInt64, ncclMax, rccl_.comm, s),
                "ncclAllReduce");
  }

  std::vector<ItemGroup> groups_;
  Tensor csc_row_, csc_bin_, colptr_, nbins_, zbin_, fid_orig_, rowdig_, row_node_, kexp_;
  optional<Tensor> h_row_, h_key_, rowpack_, dense_, hot_row_, node_dense_, wide_, dig16_, fmix_;
  std::map<std::string, Tensor> st_;
  Tensor scratch_, gain_, sbin_, sleft_, chunk_sums_, ticket_, parts_, maxv_, part_gain_, part_f_;
  fdx::SplitArgs last_split_{};           // the last search (its partials feed the best-split pass)
  optional<Tensor> arena_;
  int32_t* counts_host_dev_ = nullptr;
  int parity_ = 0, tparity_ = 0;
  Tensor root_parts_, sample_counts_;
  const int64_t* root_pending_ = nullptr;   // the last prologue's root slots, until level 0's split
  const int64_t* find_root_ = nullptr;
  const int64_t* find_prev_ = nullptr;
  const int32_t* find_sub_par_ = nullptr;
  const int32_t* find_sub_sib_ = nullptr;
  optional<Tensor> sub_of_;
  // data-parallel GBDT level loop (gbdt_dp_setup)
  bool dp_ = false;
  py::object dp_rs_cb_, dp_ag_cb_, dp_max_cb_;
  int64_t dp_S_ = 1, dp_Bs_ = 1, dp_f0_ = 0;
  Tensor dp_bin_lo_, dp_send_, dp_out_[2], dp_row_of_[2], dp_ag_in_, dp_boff_, dp_nbins_, dp_zbin_, dp_fid_,
      dp_dst_row_, dp_par_row_, dp_sib_row_, dp_iota_, dp_allt_;
  optional<Tensor> dp_wide_;
  bool dp_direct_ = false;
  Rccl rccl_;
  Tensor dp_allt_buf_;
  int64_t dp_calls_[3] = {0, 0, 0}, dp_timed_ = 0;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> dp_timing_;
  bool build_all_ = true;
  int mode_ = 1, max_depth_ = 5, wps_ = 256;
  double min_gain_ = 0.0, lambda_ = 1.0, mcw_ = 1.0;
  int64_t seed_ = 0, F_ = 1, k_ = 1;
  bool lds_ = true;
  at::Device dev_{at::kCPU};
  // GBDT level loop (gbdt_setup)
  fdx::RgHistArgs gh_{};
  fdx::RgListArgs gl_{};
  std::vector<Tensor> g_keep_;
  Tensor g_hist_[2], g_open_[2], g_totals_[2], g_packed_, g_one_, g_zero1_, g_boff_, g_list_work_, g_rg_start_,
      g_rg_list_, g_rg_listdig_;
  optional<Tensor> g_erow_, g_emdig_, g_part_, g_wg_first_, g_wg_first_list_, g_wide_;
  struct {
    const int32_t *g, *p, *np;
    int32_t n;
  } g_wl_{};                               // the listed levels' work table
  int64_t g_em_min_rows_ = 0;
  bool g_counted_ok_ = false, g_counted_ = false, g_part_multi_ = false, g_choose_ = false;
  Tensor g_rows_;
  const int32_t* rows_base_ = nullptr;
  bool rows_choose_ = false;                     // (partition(): rows_out for LevelChooseArgs)
  const int32_t* nc_base_ = nullptr;             // first node id of the level whose partition wrote
  Tensor g_node_counts_;                         //   g_node_counts_ (PartitionArgs node_counts)
  hipEvent_t g_ev_ = nullptr;
};

// ---- RandomForest trees in flight as lockstep batches (PAR-05) -------------------------------
// Spark grows the nodes of many trees per pass over the data (SURVEY PAR-05; reference
// /root/reference/fraud_detection_spark.py:67-74). Here up to `lanes` trees grow level by level in
// lockstep: every stage of a level -- histogram passes per item group, split search, best split +
// plan (+ the next level's feature sample, DP layout and item selects), partition -- is recorded
// per lane by the lane's own runner (RfLevels with rec_ set: the exact argument structs of its
// per-tree launches) and issued as ONE lane-batched launch (tree.h "lane-batched launches"), so a
// forest level costs ~12 launches for all its trees instead of ~18 per tree, and the host does no
// per-tree interpreter work at all. Under data parallelism a level's histograms of all the lanes
// go out in ONE reduce-scatter and their best splits in ONE all-gather (RCCL called here on the
// process group's communicator, or Python callbacks on gloo). Every lane's arguments are the ones
// its per-tree level loop (grower._rf_runner_levels) passes, so the forest is bitwise the same.
class RfBatch {
 public:
  explicit RfBatch(const py::dict& c) {
    for (auto item : c["lanes"].cast<py::list>()) {
      const py::dict d = item.cast<py::dict>();
      Lane ln;
      ln.obj = d["runner"];
      ln.r = ln.obj.cast<RfLevels*>();
      for (int k = 0; k < 2; ++k) {
        ln.open[k] = get(d, k ? "open1" : "open0");
        ln.totals[k] = get(d, k ? "totals1" : "totals0");
        ln.thr[k] = get(d, k ? "thr1" : "thr0");
        ln.mask[k] = get(d, k ? "mask1" : "mask0");
      }
      ln.arena = get(d, "arena");
      ln.arena_init = get(d, "arena_init");
      ln.arena_host[0] = get(d, "arena_host0");
      ln.arena_host[1] = get(d, "arena_host1");
      ln.tot_scratch = get(d, "tot_scratch");
      ln.hist = get_opt(d, "hist");
      ln.packed = get_opt(d, "packed");
      ln.rowpack = get(d, "rowpack");
      for (auto t : d["sel"].cast<py::list>()) ln.sel.push_back(t.is_none() ? optional<Tensor>() : t.cast<Tensor>());
      for (auto t : d["listed"].cast<py::list>()) {
        auto pr = t.cast<py::tuple>();
        ln.listed.push_back(pr[0].is_none() ? optional<Tensor>() : pr[0].cast<Tensor>());
        ln.listed_cnt.push_back(pr[1].is_none() ? optional<Tensor>() : pr[1].cast<Tensor>());
      }
      if (d.contains("sh_local0")) {
        for (int k = 0; k < 2; ++k) {
          ln.sh_local[k] = get(d, k ? "sh_local1" : "sh_local0");
          ln.sh_sizes[k] = get(d, k ? "sh_sizes1" : "sh_sizes0");
          ln.sh_sizes_host[k] = get(d, k ? "sh_sizes_host1" : "sh_sizes_host0");
        }
      }
      FDX_CHECK(ln.r->groups_.size() == ln.sel.size() && ln.sel.size() == ln.listed.size(), "lane group lists");
      lanes_.push_back(std::move(ln));
    }
    FDX_CHECK(!lanes_.empty(), "RfBatch: at least one lane");
    D_ = c["max_depth"].cast<int64_t>();
    boff_ = get(c, "boff");
    wide_ = get_opt(c, "wide");
    listed_max_ = c["listed_max_nodes"].cast<int64_t>();
    presel_ = c["presel"].cast<bool>();
    one_ = get(c, "one");
    zero1_ = get(c, "zero1");
    iota_ = get(c, "iota");
    dp_ = c["dp"].cast<bool>();
    if (dp_) {
      S_ = c["S"].cast<int64_t>();
      Bs_full_ = c["Bs"].cast<int64_t>();
      max_nb_ = c["max_nb"].cast<int64_t>();
      compact_ = c["compact"].cast<bool>();
      shard_of_ = get(c, "shard_of");
      sh_local_full_ = get(c, "sh_local");
      sh_boff_ = get(c, "sh_boff");
      sh_nbins_ = get(c, "sh_nbins");
      sh_zbin_ = get(c, "sh_zbin");
      sh_fid_ = get(c, "sh_fid");
      sh_fs_ = get(c, "sh_fs");
      nbins_all_ = get(c, "nbins_all");
      f0_ = c["f0"].cast<int64_t>();
      Fa_s_ = c["Fa_s"].cast<int64_t>();
      max_shard_features_ = c["max_shard_features"].cast<int64_t>();
      rs_cb_ = c["rs"];
      ag_cb_ = c["ag"];
      direct_ = c.contains("comm") && !c["comm"].is_none() &&
                rccl_.load(c["rccl_lib"].cast<std::string>(), c["comm"].cast<int64_t>());
    }
    const auto dev = lanes_[0].r->dev_;
    host_ = at::empty({kRegions * kRegion}, at::TensorOptions().dtype(at::kByte).pinned_memory(true));
    dev_args_ = at::empty({kRegions * kRegion}, at::TensorOptions().dtype(at::kByte).device(dev));
    i64_ = at::TensorOptions().dtype(at::kLong).device(dev);
    FDX_CHECK(hipEventCreateWithFlags(&ev_, hipEventDisableTiming) == hipSuccess, "event");
    for (auto& e : half_ev_) FDX_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming) == hipSuccess, "event");
    FDX_CHECK(hipEventCreateWithFlags(&done_, hipEventDisableTiming) == hipSuccess, "event");
  }
  ~RfBatch() {
    for (hipEvent_t e : half_ev_)
      if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : {ev_, done_})
      if (e) (void)hipEventDestroy(e);
    for (auto& e : timing_) {
      (void)hipEventDestroy(e.first);
      (void)hipEventDestroy(e.second);
    }
    for (auto& ln : lanes_) ln.r->rec_ = nullptr;
  }
  RfBatch(const RfBatch&) = delete;
  RfBatch& operator=(const RfBatch&) = delete;

  // A batch of trees in three calls, so that a driver can interleave two batches on one stream
  // (the host prepares one batch's level while the GPU runs the other's):
  //   start(trees)  lane l grows trees[l] (l < number of trees <= lanes): node-table images in, the
  //                 prologue (bootstrap counts, digits, row_node = 0, root) and the root's sample
  //                 queued; level 0 too unless it needs the root's compact layout sizes first;
  //   step()        waits (GIL released) for the last queued level's counts and queues the next
  //                 level of the lanes whose trees go on; false when every tree is finished;
  //   finish(p)     queues the node tables into the lanes' arena_host[p] and records the batch's
  //                 event (wait()); returns the level counters since start: levels, built nodes,
  //                 listed passes, listed active items, listed grid waves, reduce-scatters,
  //                 all-gathers.
  void start(const std::vector<int64_t>& trees, const Tensor& label, const optional<Tensor>& weight, bool bootstrap,
             int64_t row0) {
    const int64_t L = (int64_t)trees.size();
    FDX_CHECK(L >= 1 && L <= (int64_t)lanes_.size(), "RfBatch.start: 1 .. lanes trees");
    c10::hip::HIPGuard guard(lanes_[0].r->dev_.index());
    const hipStream_t s = cur_stream(lanes_[0].r->dev_);
    stat_.assign(7, 0);
    n_trees_ = L;
    live_.clear();
    for (int64_t l = 0; l < L; ++l) {
      Lane& ln = lanes_[l];
      ln.tree = trees[l];
      ln.n_open = ln.n_build = 1;
      live_.push_back((int)l);
    }
    begin_region();
    for (int l : live_) {
      Lane& ln = lanes_[l];
      // (the node-table image first: one batched copy kernel, recorded like the count rows)
      ln.rec.add(kRecCopy, RecCopy{ln.arena.data_ptr(), ln.arena_init.data_ptr(), (size_t)ln.arena.nbytes(), false});
      ln.r->rec_ = &ln.rec;
      ln.r->prologue(c10::nullopt, c10::nullopt, c10::nullopt, label, weight, ln.tree, bootstrap, 1, c10::nullopt,
                     ln.tot_scratch, c10::nullopt, row0, dp_ ? optional<Tensor>() : optional<Tensor>(ln.hist->narrow(0, 0, 1)),
                     c10::nullopt);
      ln.r->sample_level(ln.open[0], 1, ln.tree, ln.thr[0], ln.mask[0], sh_fs(), nbins_all(), sh_local(ln, 0),
                         sh_sizes(ln, 0), sh_sizes_host(ln, 0), max_shard_features_, s);
    }
    flush(s);
    d_ = 0;
    if (dp_ && compact_) {
      FDX_CHECK(hipEventRecord(ev_, s) == hipSuccess, "event");        // (level 0 needs the root's sizes)
    } else {
      run_level(s);
    }
  }

  bool step() {
    if (d_ >= D_ || live_.empty()) return false;
    c10::hip::HIPGuard guard(lanes_[0].r->dev_.index());
    const hipStream_t s = cur_stream(lanes_[0].r->dev_);
    {
      const auto t0 = std::chrono::steady_clock::now();
      py::gil_scoped_release nogil;
      wait_event(ev_);
      host_s_[2] += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    }
    if (d_ > 0) {                // the counts of the previous plan, the lanes whose trees go on
      std::vector<int> still;
      for (int l : live_) {
        Lane& ln = lanes_[l];
        const Tensor& ch = ln.r->st_["counts_host"];
        const int32_t* row = p<int32_t>(ch) + (d_ - 1) * ch.size(1);
        ln.n_open = row[1];
        ln.n_build = row[2];
        if (ln.n_open > 0) still.push_back(l);
      }
      live_ = still;
      if (live_.empty()) return false;
    }
    run_level(s);
    return true;
  }

  std::vector<int64_t> finish(int64_t parity) {
    c10::hip::HIPGuard guard(lanes_[0].r->dev_.index());
    const hipStream_t s = cur_stream(lanes_[0].r->dev_);
    begin_region();
    live_.clear();
    for (int64_t l = 0; l < n_trees_; ++l) {
      Lane& ln = lanes_[l];
      ln.r->rec_ = nullptr;
      ln.rec.add(kRecCopy,
                 RecCopy{ln.arena_host[parity & 1].data_ptr(), ln.arena.data_ptr(), (size_t)ln.arena.nbytes(), true});
      live_.push_back((int)l);
    }
    flush(s);
    live_.clear();
    FDX_CHECK(hipEventRecord(done_, s) == hipSuccess, "event");
    stat_[5] = rs_calls_;
    stat_[6] = ag_calls_;
    rs_calls_ = ag_calls_ = 0;
    return stat_;
  }

  // start + every step + finish (one batch alone); on_wait (if not None) is called once, before
  // the first host wait (the caller builds the previous batch's trees meanwhile)
  std::vector<int64_t> grow(const std::vector<int64_t>& trees, const Tensor& label, const optional<Tensor>& weight,
                            bool bootstrap, int64_t row0, int64_t parity, const py::object& on_wait) {
    start(trees, label, weight, bootstrap, row0);
    if (!on_wait.is_none()) on_wait();
    while (step()) {
    }
    return finish(parity);
  }

  bool direct() const { return direct_; }

  // host seconds since the last call: queuing the levels (recording + flushes), of which the
  // flushes (argument packing, copies, launches), and the waits for level counts
  std::vector<double> host_times() {
    std::vector<double> out{host_s_[0], host_s_[1], host_s_[2]};
    host_s_[0] = host_s_[1] = host_s_[2] = 0.0;
    return out;
  }

  // Milliseconds of the direct collectives since the last call (every 8th timed, scaled; waits for
  // their events)
  double coll_ms() {
    double ms = 0.0;
    for (auto& e : timing_) {
      float t = 0.f;
      if (hipEventSynchronize(e.second) == hipSuccess && hipEventElapsedTime(&t, e.first, e.second) == hipSuccess)
        ms += 8.0 * t;
      (void)hipEventDestroy(e.first);
      (void)hipEventDestroy(e.second);
    }
    timing_.clear();
    return ms;
  }

  // The last grow's node tables are in the lanes' arena_host (GIL released while waiting).
  void wait() {
    py::gil_scoped_release nogil;
    wait_event(done_);
  }

 private:
  // argument staging: a ring of kRegions regions, one per level (and prologue) in turn; a region is
  // reused kRegions levels later, after its copy (event) completed -- long since, as every level
  // waits for the previous one's counts
  static constexpr int kRegions = 4;
  static constexpr int64_t kRegion = 1 << 19;

  struct Lane {
    py::object obj;
    RfLevels* r = nullptr;
    Tensor open[2], totals[2], thr[2], mask[2], arena, arena_init, arena_host[2], tot_scratch, rowpack;
    optional<Tensor> hist, packed;
    std::vector<optional<Tensor>> sel, listed, listed_cnt;
    Tensor sh_local[2], sh_sizes[2], sh_sizes_host[2];
    LaneRec rec;
    // views of the lane's fixed buffers, made once (an ATen view costs ~1-2 us of host time and a
    // level asked for ~15 per lane)
    std::unordered_map<uint64_t, Tensor> views;
    template <class F>
    const Tensor& view(uint64_t tag, int64_t a, int64_t b, F make) {
      const uint64_t key = (tag << 56) | ((uint64_t)(a & 0xffffff) << 28) | (uint64_t)(b & 0xfffffff);
      auto it = views.find(key);
      if (it != views.end()) return it->second;
      return views.emplace(key, make()).first->second;
    }
    int64_t tree = 0;
    int32_t n_open = 0, n_build = 0;
    std::vector<int32_t> npx;
    std::vector<int> sel_j;
    int64_t row0 = 0, l0 = 0, tb = -1, Bs = 0;
  };

  optional<Tensor> sh_fs() const { return dp_ && compact_ ? optional<Tensor>(sh_fs_) : c10::nullopt; }
  optional<Tensor> nbins_all() const { return dp_ && compact_ ? optional<Tensor>(nbins_all_) : c10::nullopt; }
  optional<Tensor> sh_local(const Lane& ln, int k) const {
    return dp_ && compact_ ? optional<Tensor>(ln.sh_local[k]) : c10::nullopt;
  }
  optional<Tensor> sh_sizes(const Lane& ln, int k) const {
    return dp_ && compact_ ? optional<Tensor>(ln.sh_sizes[k]) : c10::nullopt;
  }
  optional<Tensor> sh_sizes_host(const Lane& ln, int k) const {
    return dp_ && compact_ ? optional<Tensor>(ln.sh_sizes_host[k]) : c10::nullopt;
  }

  void begin_region() {
    half_ = (half_ + 1) % kRegions;
    off_ = 0;
    if (half_used_[half_]) (void)hipEventSynchronize(half_ev_[half_]);
  }

  // Queues level d_ of the live lanes (their n_open / n_build read) and advances d_.
  void run_level(hipStream_t s) {
    const int64_t d = d_;
    begin_region();
    for (int l : live_) {
      Lane& ln = lanes_[l];
      stat_[0] += 1;
      stat_[1] += ln.n_build;
      ln.npx.assign(ln.r->groups_.size(), -1);
      ln.sel_j.assign(ln.r->groups_.size(), -1);
      if (presel_ && d > 0) {
        const Tensor& ch = ln.r->st_["counts_host"];
        const int32_t* row = p<int32_t>(ch) + (d - 1) * ch.size(1);
        int j = 0;
        for (size_t gi = 0; gi < ln.r->groups_.size(); ++gi) {
          if (!ln.sel[gi]) continue;
          int32_t m = 0, sum = 0;
          for (int x = 0; x < 8; ++x) {
            m = std::max(m, row[4 + 8 * j + x]);
            sum += row[4 + 8 * j + x];
          }
          ln.npx[gi] = m;
          ln.sel_j[gi] = j;
          if (m) {
            stat_[2] += 1;
            stat_[3] += sum;
            stat_[4] += (m + 3) / 4 * 8 * 4;
          }
          ++j;
        }
      }
    }
    const auto t0 = std::chrono::steady_clock::now();
    level(d, (int)(d & 1), (int)(d & 1) ^ 1, d + 1 < D_, s, stat_);
    host_s_[0] += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    ++d_;
  }

  void level(int64_t d, int cur, int nxt, bool more, hipStream_t s, std::vector<int64_t>& stat) {
    // Every stage of the level is recorded first (the arguments depend only on host-known sizes and
    // buffers fixed for the level), packed in one copy and then issued segment by segment with the
    // collectives in between: the GPU runs the level's stages back to back instead of idling while
    // the host records the next one (profiles/r6/rf_dp_busy_*.txt: the idle sat before each flush).
    // ---- histogram passes (DP: into the batch's shard-major send buffer)
    Tensor send, out, ag_in, allt;
    int64_t R = 0, Bs = 0, nrows = 0, nopen = 0;
    if (dp_) {
      for (int l : live_) {
        Lane& ln = lanes_[l];
        ln.Bs = Bs_full_;
        if (compact_) {
          const int64_t* sz = p<int64_t>(ln.sh_sizes_host[cur]);
          int64_t m = 0;
          for (int64_t k = 0; k < S_; ++k) m = std::max(m, sz[k]);
          ln.Bs = m + max_nb_;
        }
        Bs = std::max(Bs, ln.Bs);
        ln.row0 = nrows;
        ln.l0 = nopen;
        nrows += ln.n_build;
        nopen += ln.n_open;
      }
      Bs = std::max<int64_t>(Bs, 1);
      const int64_t ntot = d == 0 ? (int64_t)live_.size() : 0;
      R = nrows + (ntot + Bs - 1) / Bs;
      int64_t t = 0;
      for (int l : live_) lanes_[l].tb = d == 0 ? nrows * Bs + t++ : -1;
      send = buffer(send_, S_ * R * Bs * 2).view({S_, R, Bs, 2});
      out = buffer(out_, R * Bs * 2).view({R, Bs, 2});
      ag_in = buffer(ag_in_, nopen * 5).view({nopen, 5});
      allt = buffer(allt_, S_ * nopen * 5).view({S_, nopen, 5});
      FDX_CHECK(hipMemsetAsync(send.data_ptr(), 0, send.nbytes(), s) == hipSuccess, "send zero");
    }
    for (int l : live_) {
      Lane& ln = lanes_[l];
      std::vector<optional<Tensor>> lists, cnts;
      std::vector<int64_t> npxs;
      for (size_t gi = 0; gi < ln.r->groups_.size(); ++gi) {
        const bool items = ln.r->groups_[gi].start.numel() > 0;
        if (items && presel_ && d > 0 && ln.sel[gi]) {
          lists.push_back(ln.sel[gi]);
          cnts.push_back(ln.view(1, d, ln.sel_j[gi], [&] {
            return ln.r->st_["counts"].select(0, d - 1).narrow(0, 4 + 8 * ln.sel_j[gi], 8);
          }));
          npxs.push_back(ln.npx[gi]);
        } else if (items && ln.n_open <= listed_max_) {
          lists.push_back(ln.listed[gi]);
          cnts.push_back(ln.listed_cnt[gi]);
          npxs.push_back(-1);
        } else {
          lists.push_back(c10::nullopt);
          cnts.push_back(c10::nullopt);
          npxs.push_back(-1);
        }
      }
      const optional<Tensor> pack = d > 0 ? optional<Tensor>(ln.rowpack) : c10::nullopt;
      const Tensor& mask = ln.mask[cur];
      if (!dp_) {
        const Tensor& s2n =
            d == 0 ? zero1_ : ln.view(2, ln.n_build, 0, [&] { return ln.r->st_["s2n"].narrow(0, 0, ln.n_build); });
        ln.r->hist(ln.n_build, ln.view(3, ln.n_open, 0, [&] { return ln.hist->narrow(0, 0, ln.n_open); }), boff_, mask,
                   s2n, pack, lists, cnts, npxs, c10::nullopt, 0);
      } else {
        const Tensor tgt = send.view({-1, Bs, 2}).narrow(0, ln.row0, S_ * R - ln.row0);
        const Tensor& hb = compact_ ? ln.sh_local[cur] : sh_local_full_;
        ln.r->hist(ln.n_build, tgt, hb, mask, ln.view(4, ln.n_build, 0, [&] { return iota_.narrow(0, 0, ln.n_build); }),
                   pack, lists, cnts, npxs, shard_of_, R * Bs);
        if (d == 0)
          ln.rec.add(kRecRootSend, fdx::RootSendLane{ln.r->root_pending_, p<int64_t>(send), (int32_t)S_, R * Bs * 2,
                                                     ln.tb * 2});
      }
    }
    const int64_t m_hist = mark();
    // ---- split search (+ best split + plan in one launch without a collective between them)
    if (dp_) {
      for (int l : live_) {
        Lane& ln = lanes_[l];
        const Tensor& open = ln.view(5, cur, ln.n_open, [&] { return ln.open[cur].narrow(0, 0, ln.n_open); });
        const Tensor totals = d == 0 ? out.view({-1, 2}).narrow(0, ln.tb, 1)
                                     : ln.view(6, cur, ln.n_open, [&] { return ln.totals[cur].narrow(0, 0, ln.n_open); });
        const Tensor& split_boff =
            compact_ ? ln.view(7, cur, 0, [&] { return ln.sh_local[cur].narrow(0, f0_, Fa_s_ + 1); }) : sh_boff_;
        ln.r->split(out.narrow(0, ln.row0, ln.n_build), totals, split_boff, sh_nbins_, sh_zbin_, sh_fid_, open,
                    ln.view(8, cur, ln.n_open, [&] { return ln.thr[cur].narrow(0, 0, ln.n_open); }), ln.tree, f0_,
                    ag_in.narrow(0, ln.l0, ln.n_open), c10::nullopt, wide_);
      }
    }
    const int64_t m_split = mark();
    for (int l : live_) {
      Lane& ln = lanes_[l];
      const Tensor& open = ln.view(5, cur, ln.n_open, [&] { return ln.open[cur].narrow(0, 0, ln.n_open); });
      const Tensor& n_open_ptr =
          d == 0 ? one_ : ln.view(9, d, 0, [&] { return ln.r->st_["counts"].select(0, d - 1).narrow(0, 1, 1); });
      std::vector<optional<Tensor>> sel;
      if (presel_ && more) sel = ln.sel;
      const optional<Tensor> thr_n = more ? optional<Tensor>(ln.thr[nxt]) : c10::nullopt;
      const optional<Tensor> mask_n = more ? optional<Tensor>(ln.mask[nxt]) : c10::nullopt;
      if (!dp_) {
        const Tensor& totals = d == 0 ? ln.view(10, 0, 0, [&] { return ln.r->st_["stats"].narrow(0, 0, 1); })
                                      : ln.view(6, cur, ln.n_open, [&] { return ln.totals[cur].narrow(0, 0, ln.n_open); });
        ln.r->split_plan(d, ln.n_open, ln.view(3, ln.n_open, 0, [&] { return ln.hist->narrow(0, 0, ln.n_open); }), totals,
                         boff_, ln.view(8, cur, ln.n_open, [&] { return ln.thr[cur].narrow(0, 0, ln.n_open); }), ln.tree,
                         ln.view(11, ln.n_open, 0, [&] { return ln.packed->narrow(0, 0, ln.n_open); }), wide_, open,
                         n_open_ptr, ln.open[nxt], ln.totals[nxt], more, thr_n, mask_n, sel, c10::nullopt);
      } else {
        ln.r->root_pending_ = nullptr;
        if (d == 0) ln.r->plan_root_tot_ = p<int64_t>(out) + ln.tb * 2;
        ln.r->plan(d, ln.n_open, allt.narrow(1, ln.l0, ln.n_open), open, n_open_ptr, ln.open[nxt], ln.totals[nxt], ln.tree,
                   more, thr_n, mask_n, more ? sh_fs() : c10::nullopt, more ? nbins_all() : c10::nullopt,
                   more ? sh_local(ln, nxt) : c10::nullopt, more ? sh_sizes(ln, nxt) : c10::nullopt,
                   more ? sh_sizes_host(ln, nxt) : c10::nullopt, max_shard_features_, sel);
        ln.r->plan_root_tot_ = nullptr;
      }
    }
    const int64_t m_plan = mark();
    // ---- partition (writes the next level's packed row state; single process: zeroes its histograms)
    for (int l : live_) {
      Lane& ln = lanes_[l];
      const optional<Tensor> zero =
          (!dp_ && more) ? optional<Tensor>(ln.view(3, 2 * (int64_t)ln.n_open, 0,
                                                    [&] { return ln.hist->narrow(0, 0, 2 * (int64_t)ln.n_open); }))
                         : c10::nullopt;
      ln.r->partition(d, ln.n_open, more, zero, true, c10::nullopt);
    }
    const int64_t m_end = mark();
    if (live_.empty()) return;
    pack(s);
    launch(0, m_hist, s);
    if (dp_) {
      reduce_scatter(send, out, s);
      launch(m_hist, m_split, s);
      all_gather(ag_in, allt, s);
    }
    launch(m_split, m_plan, s);
    FDX_CHECK(hipEventRecord(ev_, s) == hipSuccess, "level event");
    launch(m_plan, m_end, s);
    done();
    (void)stat;
  }

  // the device's view of a pinned host pointer (memoised per pointer)
  void* mapped(void* host) {
    auto it = mapped_.find(host);
    if (it != mapped_.end()) return it->second;
    void* d = nullptr;
    FDX_CHECK(hipHostGetDevicePointer(&d, host, 0) == hipSuccess && d != nullptr, "pinned host rows must be mapped");
    mapped_[host] = d;
    return d;
  }

  Tensor buffer(Tensor& b, int64_t n) {
    if (!b.defined() || b.numel() < n) b = at::empty({std::max<int64_t>(n, 1)}, i64_);
    return b.narrow(0, 0, n);
  }

  // timing events around every 8th direct collective (coll_ms)
  struct Timed {
    RfBatch* b;
    hipStream_t s;
    hipEvent_t e0 = nullptr;
    Timed(RfBatch* b_, hipStream_t s_) : b(b_), s(s_) {
      if ((b->timed_++ & 7) == 0 && hipEventCreate(&e0) == hipSuccess) (void)hipEventRecord(e0, s);
    }
    ~Timed() {
      hipEvent_t e1 = nullptr;
      if (e0 && hipEventCreate(&e1) == hipSuccess && hipEventRecord(e1, s) == hipSuccess) b->timing_.emplace_back(e0, e1);
    }
  };

  void reduce_scatter(const Tensor& send, const Tensor& out, hipStream_t s) {
    ++rs_calls_;
    if (!direct_) {
      rs_cb_(send, out);
      return;
    }
    Timed t(this, s);
    rccl_.check(rccl_.rs(send.data_ptr(), out.data_ptr(), (size_t)out.numel(), ncclInt64, ncclSum, rccl_.comm, s),
                "ncclReduceScatter");
  }

  // in [n, 5] from every rank into out [S, n, 5] (the callback's result is copied there on the stream)
  void all_gather(const Tensor& in, const Tensor& out, hipStream_t s) {
    ++ag_calls_;
    if (!direct_) {
      const Tensor r = ag_cb_(in).cast<Tensor>();
      FDX_CHECK(r.numel() == out.numel(), "all-gather callback result size");
      out.copy_(r.view_as(out));
      return;
    }
    Timed t(this, s);
    rccl_.check(rccl_.ag(in.data_ptr(), out.data_ptr(), (size_t)in.numel(), ncclInt64, rccl_.comm, s), "ncclAllGather");
  }

  // Issues what the live lanes recorded: position i of every lane's record is one lane-batched
  // launch (the lanes recorded the same sequence). The argument arrays go to the device in one copy.
  void flush(hipStream_t s) {
    if (live_.empty()) return;
    pack(s);
    launch(0, (int64_t)pk_offs_.size(), s);
    done();
  }

  // the number of launches the live lanes recorded so far (a segment boundary for launch())
  int64_t mark() const { return live_.empty() ? 0 : (int64_t)lanes_[live_[0]].rec.entries.size(); }

  struct Acc {
    double& a;
    std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
    ~Acc() { a += std::chrono::duration<double>(std::chrono::steady_clock::now() - t).count(); }
  };

  // Packs every recorded launch's lane arguments into the staging region and copies them to the
  // device in one H2D copy; launch(i0, i1) then issues positions [i0, i1), done() clears the records.
  void pack(hipStream_t s) {
    Acc acc{host_s_[1]};
    const int L = (int)live_.size();
    const auto& E0 = lanes_[live_[0]].rec.entries;
    for (int l : live_) {
      const auto& E = lanes_[l].rec.entries;
      FDX_CHECK(E.size() == E0.size(), "lanes recorded different stages");
      for (size_t i = 0; i < E.size(); ++i)
        FDX_CHECK(E[i].kind == E0[i].kind && E[i].aux == E0[i].aux && E[i].bytes.size() == E0[i].bytes.size(),
                  "lanes recorded different launches");
    }
    uint8_t* host = p<uint8_t>(host_) + half_ * kRegion;
    uint8_t* dev = p<uint8_t>(dev_args_) + half_ * kRegion;
    off_ = (off_ + 15) & ~int64_t{15};
    const int64_t start = off_;
    std::vector<int64_t>& offs = pk_offs_;
    std::vector<int64_t>& offs2 = pk_offs2_;
    offs.assign(E0.size(), -1);
    offs2.assign(E0.size(), -1);
    for (size_t i = 0; i < E0.size(); ++i) {
      if (E0[i].kind == kRecCopy) {            // D2H rows: one kernel writing the host-mapped rows
        off_ = (off_ + 15) & ~int64_t{15};
        FDX_CHECK(off_ + L * (int64_t)sizeof(fdx::CopyLane) <= kRegion, "argument staging overflow");
        offs[i] = off_;
        for (int k = 0; k < L; ++k) {
          RecCopy c;
          std::memcpy(&c, lanes_[live_[k]].rec.entries[i].bytes.data(), sizeof(c));
          const fdx::CopyLane cl{c.to_host ? mapped(c.dst) : c.dst, c.src, (int64_t)c.bytes};
          std::memcpy(host + off_ + k * sizeof(fdx::CopyLane), &cl, sizeof(cl));
        }
        off_ += L * (int64_t)sizeof(fdx::CopyLane);
        continue;
      }
      const int64_t sz = (int64_t)E0[i].bytes.size();
      off_ = (off_ + 15) & ~int64_t{15};
      FDX_CHECK(off_ + L * sz + L * (int64_t)sizeof(fdx::PartitionArgs) + 16 <= kRegion, "argument staging overflow");
      offs[i] = off_;
      for (int k = 0; k < L; ++k) std::memcpy(host + off_ + k * sz, lanes_[live_[k]].rec.entries[i].bytes.data(), sz);
      off_ += L * sz;
      if (E0[i].kind == kRecPartition) {       // (the row pass takes the PartitionArgs alone)
        off_ = (off_ + 15) & ~int64_t{15};
        offs2[i] = off_;
        for (int k = 0; k < L; ++k) {
          fdx::PartColsLane q;
          std::memcpy(&q, lanes_[live_[k]].rec.entries[i].bytes.data(), sizeof(q));
          std::memcpy(host + off_ + k * sizeof(fdx::PartitionArgs), &q.a, sizeof(fdx::PartitionArgs));
        }
        off_ += L * (int64_t)sizeof(fdx::PartitionArgs);
      }
    }
    off_ = (off_ + 15) & ~int64_t{15};
    if (off_ > start) {
      FDX_CHECK(off_ <= kRegion, "argument staging overflow");
      // (read by a kernel through the pinned region's device mapping: no runtime H2D path)
      uint8_t* src = static_cast<uint8_t*>(mapped(p<uint8_t>(host_))) + half_ * kRegion;
      fdx::launch_stage_copy(dev + start, src + start, off_ - start, s);
      FDX_CHECK(hipEventRecord(half_ev_[half_], s) == hipSuccess, "event");
      half_used_[half_] = true;
    }
    pk_host_ = host;
    pk_dev_ = dev;
    pk_L_ = L;
  }

  void launch(int64_t i0, int64_t i1, hipStream_t s) {
    Acc acc{host_s_[1]};
    const int L = pk_L_;
    const auto& E0 = lanes_[live_[0]].rec.entries;
    FDX_CHECK(i0 >= 0 && i0 <= i1 && i1 <= (int64_t)pk_offs_.size() && pk_offs_.size() == E0.size(),
              "launch range of the packed records");
    uint8_t* host = pk_host_;
    uint8_t* dev = pk_dev_;
    const std::vector<int64_t>& offs2 = pk_offs2_;
    for (int64_t i = i0; i < i1; ++i) {
      const int64_t o = pk_offs_[i];
      switch (E0[i].kind) {
        case kRecQuant:
          fdx::launch_quant_lanes((const fdx::QuantLane*)(host + o), (const fdx::QuantLane*)(dev + o), L, s);
          break;
        case kRecHist:
          fdx::launch_hist_lanes((const fdx::HistArgs*)(host + o), (const fdx::HistArgs*)(dev + o), L, E0[i].aux, s);
          break;
        case kRecSplit:
          fdx::launch_split_lanes((const fdx::SplitArgs*)(host + o), (const fdx::SplitArgs*)(dev + o), L, s);
          break;
        case kRecSplitBest:
          fdx::launch_split_best_lanes((const fdx::SplitBestLane*)(host + o), (const fdx::SplitBestLane*)(dev + o), L, s);
          break;
        case kRecSplitBestPlan:
          fdx::launch_split_best_plan_lanes((const fdx::SplitBestPlanLane*)(host + o),
                                            (const fdx::SplitBestPlanLane*)(dev + o), L, s);
          break;
        case kRecLevelPlan:
          fdx::launch_level_plan_lanes((const fdx::LevelPlanArgs*)(dev + o), L, s);
          break;
        case kRecRfSample:
          fdx::launch_rf_sample_lanes((const fdx::RfSampleArgs*)(host + o), (const fdx::RfSampleArgs*)(dev + o), L, s);
          break;
        case kRecRfCompact:
          fdx::launch_rf_compact_lanes((const fdx::RfCompactArgs*)(host + o), (const fdx::RfCompactArgs*)(dev + o), L, s);
          break;
        case kRecSelectGroups:
          fdx::launch_select_groups_lanes((const fdx::SelectArgs*)(host + o), (const fdx::SelectArgs*)(dev + o), L, s);
          break;
        case kRecPartition:
          fdx::launch_partition_lanes((const fdx::PartColsLane*)(host + o), (const fdx::PartColsLane*)(dev + o),
                                      (const fdx::PartitionArgs*)(dev + offs2[i]), L, s);
          break;
        case kRecRootSend:
          fdx::launch_root_send_lanes((const fdx::RootSendLane*)(dev + o), L, s);
          break;
        case kRecCopy:
          fdx::launch_copy_lanes((const fdx::CopyLane*)(host + o), (const fdx::CopyLane*)(dev + o), L, s);
          break;
        default:
          FDX_CHECK(false, "unknown recorded launch");
      }
    }
    C10_HIP_KERNEL_LAUNCH_CHECK();
  }

  void done() {
    for (int l : live_) lanes_[l].rec.entries.clear();
    pk_offs_.clear();
    pk_offs2_.clear();
  }

  std::vector<Lane> lanes_;
  std::vector<int> live_;
  int64_t D_ = 5, listed_max_ = 2, d_ = 0, n_trees_ = 0;
  double host_s_[3] = {0.0, 0.0, 0.0};
  std::vector<int64_t> stat_;
  bool presel_ = true, dp_ = false, compact_ = false, direct_ = false;
  Tensor boff_, one_, zero1_, iota_;
  optional<Tensor> wide_;
  // data parallel
  int64_t S_ = 1, Bs_full_ = 1, max_nb_ = 1, f0_ = 0, Fa_s_ = 0, max_shard_features_ = 0;
  Tensor shard_of_, sh_local_full_, sh_boff_, sh_nbins_, sh_zbin_, sh_fid_, sh_fs_, nbins_all_;
  py::object rs_cb_, ag_cb_;
  Rccl rccl_;
  Tensor send_, out_, ag_in_, allt_;
  int64_t rs_calls_ = 0, ag_calls_ = 0, timed_ = 0;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> timing_;
  // argument staging (pinned host + device, two halves by level parity)
  Tensor host_, dev_args_;
  int half_ = -1;
  int64_t off_ = 0;
  // the packed records (pack -> launch -> done)
  std::vector<int64_t> pk_offs_, pk_offs2_;
  uint8_t* pk_host_ = nullptr;
  uint8_t* pk_dev_ = nullptr;
  int pk_L_ = 0;
  bool half_used_[kRegions] = {};
  hipEvent_t ev_ = nullptr, half_ev_[kRegions] = {}, done_ = nullptr;
  at::TensorOptions i64_;
  std::map<void*, void*> mapped_;
};

}  // namespace

void register_level_ops(pybind11::module& m) {
  py::class_<RfLevels>(m, "RfLevels")
      .def(py::init<const py::dict&>())
      .def("hist", &RfLevels::hist)
      .def("split", &RfLevels::split)
      .def("plan", &RfLevels::plan)
      .def("partition", &RfLevels::partition)
      .def("split_plan", &RfLevels::split_plan)
      .def("prologue", &RfLevels::prologue)
      .def("leaf_update", &RfLevels::leaf_update)
      .def("gbdt_setup", &RfLevels::gbdt_setup)
      .def("gbdt_root", &RfLevels::gbdt_root)
      .def("gbdt_dp_setup", &RfLevels::gbdt_dp_setup)
      .def("gbdt_dp_root", &RfLevels::gbdt_dp_root)
      .def("gbdt_dp_levels", &RfLevels::gbdt_dp_levels)
      .def("dp_coll_stats", &RfLevels::dp_coll_stats)
      .def("dp_direct", &RfLevels::dp_direct)
      // (no Python objects inside: the GIL is released for the level loop and its host waits, so a
      // concurrent forest thread keeps running)
      .def("gbdt_levels", &RfLevels::gbdt_levels, py::call_guard<py::gil_scoped_release>());
  py::class_<RfBatch>(m, "RfBatch")
      .def(py::init<const py::dict&>())
      .def("grow", &RfBatch::grow)
      .def("start", &RfBatch::start)
      .def("step", &RfBatch::step)
      .def("finish", &RfBatch::finish)
      .def("wait", &RfBatch::wait)
      .def("direct", &RfBatch::direct)
      .def("coll_ms", &RfBatch::coll_ms)
      .def("host_times", &RfBatch::host_times);
}

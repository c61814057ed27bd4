// pybind11 bindings of the tree engine (registered from bindings.cpp via register_tree_ops).
#include <torch/extension.h>
#include <c10/hip/HIPGuard.h>
#include <c10/hip/HIPStream.h>

#include "ops.h"
#include "tree.h"

namespace {

using at::Tensor;
using c10::optional;

#define FDX_CHECK(cond, msg) TORCH_CHECK(cond, "fdx.tree: ", msg)

void chk(const Tensor& t, const at::Device& dev, at::ScalarType st, const char* name) {
  FDX_CHECK(t.device() == dev, std::string(name) + " on wrong device");
  FDX_CHECK(t.is_contiguous(), std::string(name) + " must be contiguous");
  FDX_CHECK(t.scalar_type() == st, std::string(name) + " has wrong dtype");
}

// t's storage extends at least `extra` elements past the end of t (views into padded buffers)
bool readable_tail(const Tensor& t, int64_t extra) {
  const int64_t have = (int64_t)t.storage().nbytes() / (int64_t)t.element_size();
  return t.storage_offset() + t.numel() + extra <= have;
}

template <class T>
const T* opt(const optional<Tensor>& t) { return (t && t->defined()) ? t->data_ptr<T>() : nullptr; }

hipStream_t stream(const at::Device& d) { return c10::hip::getCurrentHIPStream(d.index()).stream(); }

void rowstats(const optional<Tensor>& g, const optional<Tensor>& h, const optional<Tensor>& label,
              const optional<Tensor>& weight, int64_t seed, int64_t tree, bool bootstrap, int64_t mode,
              const Tensor& out) {
  const auto dev = out.device();
  chk(out, dev, at::kInt, "rowstats");
  FDX_CHECK(out.dim() == 2 && out.size(1) == 2, "rowstats must be [N,2] int32");
  const int64_t N = out.size(0);
  if (mode == 0) {
    FDX_CHECK(g && h, "gbdt mode needs g,h");
    chk(*g, dev, at::kFloat, "g");
    chk(*h, dev, at::kFloat, "h");
    FDX_CHECK(g->numel() == N && h->numel() == N, "g/h size");
  } else {
    FDX_CHECK(label.has_value(), "classification mode needs labels");
    chk(*label, dev, at::kFloat, "label");
    FDX_CHECK(label->numel() == N, "label size");
  }
  if (weight) { chk(*weight, dev, at::kFloat, "weight"); FDX_CHECK(weight->numel() == N, "weight size"); }
  fdx::RowStatsArgs a{};
  a.g = opt<float>(g);
  a.h = opt<float>(h);
  a.label = opt<float>(label);
  a.weight = opt<float>(weight);
  a.seed = (uint64_t)seed;
  a.tree = (int32_t)tree;
  a.bootstrap = bootstrap ? 1 : 0;
  a.mode = (int32_t)mode;
  a.N = N;
  a.rowstats = reinterpret_cast<uint32_t*>(out.data_ptr<int32_t>());
  if (dev.is_cuda()) {
    c10::hip::HIPGuard guard(dev.index());
    fdx::launch_rowstats(a, stream(dev));
    C10_HIP_KERNEL_LAUNCH_CHECK();
  } else {
    fdx::rowstats_cpu(a);
  }
}

// est[e] = rowstats[csc_row[e]] (once per tree)
void entry_stats(const Tensor& csc_row, const Tensor& rowstats, const Tensor& est) {
  const auto dev = csc_row.device();
  chk(csc_row, dev, at::kInt, "csc_row");
  chk(rowstats, dev, at::kInt, "rowstats");
  chk(est, dev, at::kInt, "est");
  const int64_t nnz = csc_row.numel();
  FDX_CHECK(est.numel() >= 2 * nnz, "est must hold [nnz,2] int32");
  FDX_CHECK(rowstats.dim() == 2 && rowstats.size(1) == 2, "rowstats must be [N,2]");
  FDX_CHECK(reinterpret_cast<uintptr_t>(csc_row.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(est.data_ptr()) % 16 == 0,
            "csc_row/est must be 16-byte aligned");
  const auto* rs = reinterpret_cast<const uint32_t*>(rowstats.data_ptr<int32_t>());
  auto* out = reinterpret_cast<uint32_t*>(est.data_ptr<int32_t>());
  if (dev.is_cuda()) {
    c10::hip::HIPGuard guard(dev.index());
    fdx::launch_entry_stats(csc_row.data_ptr<int32_t>(), rs, nnz, out, stream(dev));
    C10_HIP_KERNEL_LAUNCH_CHECK();
  } else {
    fdx::entry_stats_cpu(csc_row.data_ptr<int32_t>(), rs, nnz, out);
  }
}

// est[e] = rowstats[csc_row[e]] for the entries of the listed work items, in wave order
void entry_stats_items(const Tensor& item_start, const Tensor& item_end, const Tensor& wave_item,
                       const Tensor& csc_row, const Tensor& rowstats, const Tensor& est) {
  const auto dev = csc_row.device();
  chk(item_start, dev, at::kLong, "item_start");
  chk(item_end, dev, at::kLong, "item_end");
  chk(wave_item, dev, at::kInt, "wave_item");
  chk(csc_row, dev, at::kInt, "csc_row");
  chk(rowstats, dev, at::kInt, "rowstats");
  chk(est, dev, at::kInt, "est");
  FDX_CHECK(est.numel() >= 2 * csc_row.numel(), "est must hold [nnz,2] int32");
  FDX_CHECK(wave_item.numel() % 4 == 0, "wave_item: 4 slots per workgroup");
  FDX_CHECK(readable_tail(csc_row, 4), "csc_row needs 4 readable padding entries (quantize.CSC_PAD)");
  const auto* rs = reinterpret_cast<const uint32_t*>(rowstats.data_ptr<int32_t>());
  auto* out = reinterpret_cast<uint32_t*>(est.data_ptr<int32_t>());
  const int32_t ni = (int32_t)item_start.numel();
  if (dev.is_cuda()) {
    c10::hip::HIPGuard guard(dev.index());
    fdx::launch_entry_stats_items(item_start.data_ptr<int64_t>(), item_end.data_ptr<int64_t>(),
                                  wave_item.data_ptr<int32_t>(), (int32_t)wave_item.numel(), ni,
                                  csc_row.data_ptr<int32_t>(), rs, out, stream(dev));
    C10_HIP_KERNEL_LAUNCH_CHECK();
  } else {
    fdx::entry_stats_items_cpu(item_start.data_ptr<int64_t>(), item_end.data_ptr<int64_t>(), ni,
                               csc_row.data_ptr<int32_t>(), rs, out);
  }
}

// slot8[r] = node_slot[row_node[r]] - slot_base if in [0, nslots), else 0xff
void slot8(const Tensor& row_node, const Tensor& node_slot, int64_t slot_base, int64_t nslots, const Tensor& out) {
  const auto dev = row_node.device();
  chk(row_node, dev, at::kInt, "row_node");
  chk(node_slot, dev, at::kInt, "node_slot");
  chk(out, dev, at::kByte, "slot8");
  FDX_CHECK(out.numel() == row_node.numel(), "slot8 must be [N] uint8");
  FDX_CHECK(nslots >= 0 && nslots <= 255, "at most 255 slots per pass");
  fdx::SlotArgs a{};
  a.row_node = row_node.data_ptr<int32_t>();
  a.node_slot = node_slot.data_ptr<int32_t>();
  a.num_nodes = (int32_t)node_slot.numel();
  a.slot_base = (int32_t)slot_base;
  a.nslots = (int32_t)nslots;
  a.N = row_node.numel();
  a.slot8 = out.data_ptr<uint8_t>();
  if (dev.is_cuda()) {
    c10::hip::HIPGuard guard(dev.index());
    fdx::launch_slot8(a, stream(dev));
    C10_HIP_KERNEL_LAUNCH_CHECK();
  } else {
    fdx::slot8_cpu(a);
  }
}

// Build histograms of the listed features for the 8*ct slots of one pass. slot8 = None: root pass
// (every entry in slot 0).
void hist_build(const Tensor& item_start, const Tensor& item_end, const Tensor& csc_row, const Tensor& csc_bin,
                const optional<Tensor>& slot8_t, const Tensor& est, int64_t bt, int64_t ct, const Tensor& slab,
                const Tensor& feat, const Tensor& feat_item0, const Tensor& feat_nitems, const Tensor& boff,
                const Tensor& nbins, const Tensor& slot_to_node, const Tensor& hist, int64_t TB,
                const optional<Tensor>& wave_item, const optional<Tensor>& rowstats) {
  const auto dev = csc_row.device();
  chk(item_start, dev, at::kLong, "item_start");
  chk(item_end, dev, at::kLong, "item_end");
  chk(csc_row, dev, at::kInt, "csc_row");
  chk(csc_bin, dev, at::kByte, "csc_bin");
  if (slot8_t) chk(*slot8_t, dev, at::kByte, "slot8");
  chk(est, dev, at::kInt, "est");
  chk(feat, dev, at::kInt, "feat");
  chk(feat_item0, dev, at::kLong, "feat_item0");
  chk(feat_nitems, dev, at::kInt, "feat_nitems");
  chk(boff, dev, at::kLong, "boff");
  chk(nbins, dev, at::kInt, "nbins");
  chk(slot_to_node, dev, at::kInt, "slot_to_node");
  chk(hist, dev, at::kDouble, "hist");
  FDX_CHECK(item_start.numel() == item_end.numel(), "item arrays");
  // bt 0: narrow 16-bin tile, 4*ct slots (ct 1/2/4/8); bt 1/2: 32*bt bins, 8*ct slots (ct 1/2/4)
  FDX_CHECK((bt == 0 && (ct == 1 || ct == 2 || ct == 4 || ct == 8)) ||
                (bt >= 1 && bt <= 2 && (ct == 1 || ct == 2 || ct == 4)), "unsupported (bt, ct)");
  const int64_t tile_slots = bt == 0 ? 4 * ct : 8 * ct, tile_bins = bt == 0 ? 16 : 32 * bt;
  FDX_CHECK(slot_to_node.numel() == tile_slots, "slot_to_node must have one entry per tile slot");
  FDX_CHECK(csc_row.numel() == csc_bin.numel(), "csc arrays");
  const bool gather = rowstats.has_value() && rowstats->defined();
  if (gather) {
    // gather mode: statistics per row, est is not read
    chk(*rowstats, dev, at::kInt, "rowstats");
    FDX_CHECK(rowstats->dim() == 2 && rowstats->size(1) == 2, "rowstats must be [N,2] int32");
    FDX_CHECK(reinterpret_cast<uintptr_t>(rowstats->data_ptr()) % 8 == 0, "rowstats must be 8-byte aligned");
    FDX_CHECK(!slot8_t || slot8_t->numel() == rowstats->size(0), "slot8 and rowstats row counts differ");
  } else {
    FDX_CHECK(est.numel() >= 2 * csc_row.numel(), "est must hold [nnz,2]");
    FDX_CHECK(reinterpret_cast<uintptr_t>(est.data_ptr()) % 16 == 0 && readable_tail(est, 8),
              "est must be 16-byte aligned with 4 readable padding entries (see quantize.CSC_PAD)");
  }
  FDX_CHECK(TB >= 0 && boff.numel() == nbins.numel() + 1, "boff must be [Fa+1]");
  FDX_CHECK(hist.numel() % (2 * std::max<int64_t>(TB, 1)) == 0, "hist must be [nodes, TB, 2]");
  FDX_CHECK(reinterpret_cast<uintptr_t>(csc_row.data_ptr()) % 16 == 0 &&
                reinterpret_cast<uintptr_t>(csc_bin.data_ptr()) % 4 == 0,
            "csc_row must be 16-byte and csc_bin 4-byte aligned");
  FDX_CHECK(readable_tail(csc_row, 4) && readable_tail(csc_bin, 4),
            "csc_row/csc_bin need 4 readable padding entries behind their end (see quantize.CSC_PAD)");
  fdx::HistArgs h{};
  h.item_start = item_start.data_ptr<int64_t>();
  h.item_end = item_end.data_ptr<int64_t>();
  h.num_items = (int32_t)item_start.numel();
  h.csc_row = csc_row.data_ptr<int32_t>();
  h.csc_bin = csc_bin.data_ptr<uint8_t>();
  h.slot8 = slot8_t ? slot8_t->data_ptr<uint8_t>() : nullptr;
  h.est = gather ? nullptr : reinterpret_cast<const uint32_t*>(est.data_ptr<int32_t>());
  h.rowstats = gather ? reinterpret_cast<const uint32_t*>(rowstats->data_ptr<int32_t>()) : nullptr;
  if (wave_item) {
    chk(*wave_item, dev, at::kInt, "wave_item");
    FDX_CHECK(wave_item->numel() % 4 == 0, "wave_item: 4 slots per workgroup");
    h.wave_item = wave_item->data_ptr<int32_t>();
    h.num_slots = (int32_t)wave_item->numel();
  }
  fdx::HistReduceArgs r{};
  r.slab_slots = (int32_t)tile_slots;
  r.slab_bins = (int32_t)tile_bins;
  r.feat = feat.data_ptr<int32_t>();
  r.feat_item0 = feat_item0.data_ptr<int64_t>();
  r.feat_nitems = feat_nitems.data_ptr<int32_t>();
  r.L = (int32_t)feat.numel();
  r.boff = boff.data_ptr<int64_t>();
  r.nbins = nbins.data_ptr<int32_t>();
  r.slot_to_node = slot_to_node.data_ptr<int32_t>();
  r.slot_base = 0;
  r.total_bins = TB;
  r.hist = hist.data_ptr<double>();
  if (dev.is_cuda()) {
    chk(slab, dev, at::kFloat, "slab");
    FDX_CHECK(slab.numel() >= (int64_t)h.num_items * tile_slots * tile_bins * 2, "slab too small");
    h.slab = slab.data_ptr<float>();
    r.slab = h.slab;
    c10::hip::HIPGuard guard(dev.index());
    fdx::launch_hist_mfma(h, (int)bt, (int)ct, stream(dev));
    C10_HIP_KERNEL_LAUNCH_CHECK();
    fdx::launch_hist_reduce(r, stream(dev));
    C10_HIP_KERNEL_LAUNCH_CHECK();
  } else {
    fdx::hist_cpu(h, r, (int)tile_slots);
  }
}

void hist_subtract(const Tensor& parent, const Tensor& cur, const Tensor& dst, const Tensor& par, const Tensor& sib,
                   int64_t TB) {
  const auto dev = cur.device();
  chk(parent, dev, at::kDouble, "parent");
  chk(cur, dev, at::kDouble, "cur");
  chk(dst, dev, at::kInt, "dst");
  chk(par, dev, at::kInt, "par");
  chk(sib, dev, at::kInt, "sib");
  const int32_t n = (int32_t)dst.numel();
  if (dev.is_cuda()) {
    c10::hip::HIPGuard guard(dev.index());
    fdx::launch_hist_subtract(parent.data_ptr<double>(), cur.data_ptr<double>(), dst.data_ptr<int32_t>(),
                              par.data_ptr<int32_t>(), sib.data_ptr<int32_t>(), n, TB, stream(dev));
    C10_HIP_KERNEL_LAUNCH_CHECK();
  } else {
    fdx::hist_subtract_cpu(parent.data_ptr<double>(), cur.data_ptr<double>(), dst.data_ptr<int32_t>(),
                           par.data_ptr<int32_t>(), sib.data_ptr<int32_t>(), n, TB);
  }
}

void split_find(const Tensor& hist, const Tensor& totals, const Tensor& boff, const Tensor& nbins, const Tensor& zbin,
                const Tensor& fid_orig, const Tensor& node_ids, int64_t mode, double lambda_, double mcw,
                double feat_prob, int64_t seed, int64_t tree, const Tensor& out_gain, const Tensor& out_bin,
                const Tensor& out_left) {
  const auto dev = hist.device();
  chk(hist, dev, at::kDouble, "hist");
  chk(totals, dev, at::kDouble, "totals");
  chk(boff, dev, at::kLong, "boff");
  chk(nbins, dev, at::kInt, "nbins");
  chk(zbin, dev, at::kInt, "zbin");
  chk(fid_orig, dev, at::kLong, "fid_orig");
  chk(node_ids, dev, at::kInt, "node_ids");
  chk(out_gain, dev, at::kDouble, "out_gain");
  chk(out_bin, dev, at::kInt, "out_bin");
  chk(out_left, dev, at::kDouble, "out_left");
  const int32_t nodes = (int32_t)node_ids.numel();
  const int32_t Fa = (int32_t)nbins.numel();
  FDX_CHECK(out_gain.numel() >= (int64_t)nodes * Fa && out_left.numel() >= 2ll * nodes * Fa, "outputs too small");
  FDX_CHECK(totals.numel() >= 2 * nodes, "totals size");
  fdx::SplitArgs a{};
  a.hist = hist.data_ptr<double>();
  a.totals = totals.data_ptr<double>();
  a.num_nodes = nodes;
  a.Fa = Fa;
  a.boff = boff.data_ptr<int64_t>();
  a.nbins = nbins.data_ptr<int32_t>();
  a.zbin = zbin.data_ptr<int32_t>();
  a.fid_orig = fid_orig.data_ptr<int64_t>();
  a.node_ids = node_ids.data_ptr<int32_t>();
  a.mode = (int32_t)mode;
  a.lambda_ = lambda_;
  a.min_child_weight = mcw;
  a.feat_prob = feat_prob;
  a.seed = (uint64_t)seed;
  a.tree = (int32_t)tree;
  a.out_gain = out_gain.data_ptr<double>();
  a.out_bin = out_bin.data_ptr<int32_t>();
  a.out_left = out_left.data_ptr<double>();
  if (dev.is_cuda()) {
    c10::hip::HIPGuard guard(dev.index());
    fdx::launch_split(a, stream(dev));
    C10_HIP_KERNEL_LAUNCH_CHECK();
  } else {
    fdx::split_cpu(a);
  }
}

void partition(const Tensor& row_node, const Tensor& default_child, const Tensor& item_start, const Tensor& item_end,
               const Tensor& item_split, const Tensor& split_default, const Tensor& split_other,
               const Tensor& split_bin, const Tensor& split_left_is_default, const Tensor& csc_row,
               const Tensor& csc_bin) {
  const auto dev = row_node.device();
  chk(row_node, dev, at::kInt, "row_node");
  chk(default_child, dev, at::kInt, "default_child");
  chk(item_start, dev, at::kLong, "item_start");
  chk(item_end, dev, at::kLong, "item_end");
  chk(item_split, dev, at::kInt, "item_split");
  chk(split_default, dev, at::kInt, "split_default");
  chk(split_other, dev, at::kInt, "split_other");
  chk(split_bin, dev, at::kInt, "split_bin");
  chk(split_left_is_default, dev, at::kInt, "split_left_is_default");
  chk(csc_row, dev, at::kInt, "csc_row");
  chk(csc_bin, dev, at::kByte, "csc_bin");
  fdx::PartitionArgs a{};
  a.row_node = row_node.data_ptr<int32_t>();
  a.default_child = default_child.data_ptr<int32_t>();
  a.num_nodes = (int32_t)default_child.numel();
  a.N = row_node.numel();
  a.item_start = item_start.data_ptr<int64_t>();
  a.item_end = item_end.data_ptr<int64_t>();
  a.item_split = item_split.data_ptr<int32_t>();
  a.num_items = (int32_t)item_start.numel();
  a.split_default = split_default.data_ptr<int32_t>();
  a.split_other = split_other.data_ptr<int32_t>();
  a.split_bin = split_bin.data_ptr<int32_t>();
  a.split_left_is_default = split_left_is_default.data_ptr<int32_t>();
  a.csc_row = csc_row.data_ptr<int32_t>();
  a.csc_bin = csc_bin.data_ptr<uint8_t>();
  if (dev.is_cuda()) {
    c10::hip::HIPGuard guard(dev.index());
    fdx::launch_partition(a, stream(dev));
    C10_HIP_KERNEL_LAUNCH_CHECK();
  } else {
    fdx::partition_cpu(a);
  }
}

void logistic_grad(const Tensor& margin, const Tensor& label, const optional<Tensor>& weight, const Tensor& g,
                   const Tensor& h) {
  const auto dev = margin.device();
  chk(margin, dev, at::kDouble, "margin");
  chk(label, dev, at::kFloat, "label");
  chk(g, dev, at::kFloat, "g");
  chk(h, dev, at::kFloat, "h");
  if (weight) chk(*weight, dev, at::kFloat, "weight");
  const int64_t N = margin.numel();
  FDX_CHECK(label.numel() == N && g.numel() == N && h.numel() == N, "sizes");
  if (dev.is_cuda()) {
    c10::hip::HIPGuard guard(dev.index());
    fdx::launch_logistic_grad(margin.data_ptr<double>(), label.data_ptr<float>(), opt<float>(weight),
                              g.data_ptr<float>(), h.data_ptr<float>(), N, stream(dev));
    C10_HIP_KERNEL_LAUNCH_CHECK();
  } else {
    fdx::logistic_grad_cpu(margin.data_ptr<double>(), label.data_ptr<float>(), opt<float>(weight),
                           g.data_ptr<float>(), h.data_ptr<float>(), N);
  }
}

void leaf_update(const Tensor& margin, const Tensor& row_node, const Tensor& node_value) {
  const auto dev = margin.device();
  chk(margin, dev, at::kDouble, "margin");
  chk(row_node, dev, at::kInt, "row_node");
  chk(node_value, dev, at::kDouble, "node_value");
  FDX_CHECK(row_node.numel() == margin.numel(), "sizes");
  if (dev.is_cuda()) {
    c10::hip::HIPGuard guard(dev.index());
    fdx::launch_leaf_update(margin.data_ptr<double>(), row_node.data_ptr<int32_t>(), node_value.data_ptr<double>(),
                            margin.numel(), stream(dev));
    C10_HIP_KERNEL_LAUNCH_CHECK();
  } else {
    fdx::leaf_update_cpu(margin.data_ptr<double>(), row_node.data_ptr<int32_t>(), node_value.data_ptr<double>(),
                         margin.numel());
  }
}

}  // namespace

void register_tree_ops(pybind11::module& m) {
  m.def("tree_rowstats", &rowstats);
  m.def("tree_entry_stats", &entry_stats);
  m.def("tree_slot8", &slot8);
  m.def("tree_entry_stats_items", &entry_stats_items);
  m.def("tree_hist_build", &hist_build);
  m.def("tree_hist_subtract", &hist_subtract);
  m.def("tree_split_find", &split_find);
  m.def("tree_partition", &partition);
  m.def("tree_logistic_grad", &logistic_grad);
  m.def("tree_leaf_update", &leaf_update);
}

// pybind11 bindings of the tree engine (registered from bindings.cpp via register_tree_ops).
#include <torch/extension.h>

#include <cstdlib>
#include <c10/hip/HIPGuard.h>
#include <c10/hip/HIPStream.h>

#include "ops.h"
#include "tree.h"

namespace {

using at::Tensor;
using c10::optional;
using c10::nullopt;

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

fdx::QuantArgs quant_args(const optional<Tensor>& g, const optional<Tensor>& h, const optional<Tensor>& label,
                           const optional<Tensor>& weight, int64_t seed, int64_t tree, bool bootstrap, int64_t mode,
                           const at::Device& dev, int64_t N) {
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
  fdx::QuantArgs a{};
  a.g = opt<float>(g);
  a.h = opt<float>(h);
  a.label = opt<float>(label);
  a.weight = opt<float>(weight);
  a.seed = (uint64_t)seed;
  a.tree = (int32_t)tree;
  a.bootstrap = bootstrap ? 1 : 0;
  a.mode = (int32_t)mode;
  a.N = N;
  return a;
}

// out_max[2] (float64) = max |statistic| over the rows (exponent choice; all-reduce MAX under DP)
void quant_max(const optional<Tensor>& g, const optional<Tensor>& h, const optional<Tensor>& label,
               const optional<Tensor>& weight, int64_t seed, int64_t tree, bool bootstrap, int64_t mode, int64_t N,
               const Tensor& out_max, int64_t row0) {
  const auto dev = out_max.device();
  chk(out_max, dev, at::kDouble, "out_max");
  FDX_CHECK(out_max.numel() == 2, "out_max must have 2 entries");
  fdx::QuantArgs a = quant_args(g, h, label, weight, seed, tree, bootstrap, mode, dev, N);
  a.row0 = row0;
  if (dev.is_cuda()) {
    c10::hip::HIPGuard guard(dev.index());
    const Tensor part = at::empty({2 * (int64_t)std::max(1, fdx::quant_blocks(N))}, out_max.options().dtype(at::kLong));
    fdx::launch_quant_max(a, out_max.data_ptr<double>(), part.data_ptr<int64_t>(), stream(dev));
    C10_HIP_KERNEL_LAUNCH_CHECK();
  } else {
    fdx::quant_max_cpu(a, out_max.data_ptr<double>());
  }
}

// rowdig [N,2] int32 = digits of the quantised statistics; kexp [2] int32 = exponents used
// (from max_abs, or 0 when max_abs is None: integer counts); totals [2] int64 = exact sums.
void quant(const optional<Tensor>& g, const optional<Tensor>& h, const optional<Tensor>& label,
           const optional<Tensor>& weight, int64_t seed, int64_t tree, bool bootstrap, int64_t mode, int64_t np,
           const optional<Tensor>& max_abs, const Tensor& rowdig, const Tensor& kexp, const Tensor& totals,
           const optional<Tensor>& digp, int64_t row0) {
  const auto dev = rowdig.device();
  chk(rowdig, dev, at::kInt, "rowdig");
  chk(kexp, dev, at::kInt, "kexp");
  chk(totals, dev, at::kLong, "totals");
  FDX_CHECK(rowdig.dim() == 2 && rowdig.size(1) == 2, "rowdig must be [N,2] int32");
  FDX_CHECK(kexp.numel() == 2 && totals.numel() == 2, "kexp/totals must have 2 entries");
  FDX_CHECK(np == 1 || np == 4, "np must be 1 or 4");
  if (max_abs) { chk(*max_abs, dev, at::kDouble, "max_abs"); FDX_CHECK(max_abs->numel() == 2, "max_abs size"); }
  FDX_CHECK(np == 4 || !max_abs, "np == 1 is for integer counts (exponent 0, no max_abs)");
  fdx::QuantArgs a = quant_args(g, h, label, weight, seed, tree, bootstrap, mode, dev, rowdig.size(0));
  a.np = (int32_t)np;
  a.row0 = row0;
  a.kexp_out = kexp.data_ptr<int32_t>();
  a.rowdig = reinterpret_cast<uint32_t*>(rowdig.data_ptr<int32_t>());
  a.totals = totals.data_ptr<int64_t>();
  if (digp) {
    chk(*digp, dev, at::kByte, "digp");
    FDX_CHECK(digp->dim() == 2 && digp->size(0) >= 2 * np && digp->size(1) >= rowdig.size(0),
              "digp must be [>= 2*np, >= N] uint8");
    a.digp = digp->data_ptr<uint8_t>();
    a.n_pad = digp->size(1);
  }
  const double* mx = max_abs ? max_abs->data_ptr<double>() : nullptr;
  if (dev.is_cuda()) {
    c10::hip::HIPGuard guard(dev.index());
    const Tensor part = at::empty({2 * (int64_t)std::max(1, fdx::quant_blocks(rowdig.size(0)))},
                                  totals.options());
    fdx::launch_quant(a, mx, part.data_ptr<int64_t>(), stream(dev));
    C10_HIP_KERNEL_LAUNCH_CHECK();
  } else {
    fdx::quant_cpu(a, mx);
  }
}

// slot8[r] = node_slot[row_node[r]] - slot_base if in [0, nslots), else 0xff
void slot8(const Tensor& row_node, const Tensor& node_slot, int64_t slot_base, int64_t nslots, const Tensor& out,
           const optional<Tensor>& rowdig, const optional<Tensor>& masked) {
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
  if (masked) {   // single-slot pass: digit words of the slot's rows, zero elsewhere (root-style pass)
    FDX_CHECK(rowdig.has_value() && nslots == 1, "masked digits: single-slot passes with rowdig");
    chk(*rowdig, dev, at::kInt, "rowdig");
    chk(*masked, dev, at::kInt, "masked");
    FDX_CHECK(rowdig->numel() == 2 * a.N && masked->numel() == 2 * a.N, "rowdig / masked must be [N, 2] int32");
    a.rowdig = reinterpret_cast<const uint32_t*>(rowdig->data_ptr<int32_t>());
    a.masked = reinterpret_cast<uint32_t*>(masked->data_ptr<int32_t>());
  }
  if (dev.is_cuda()) {
    c10::hip::HIPGuard guard(dev.index());
    fdx::launch_slot8(a, stream(dev));
    C10_HIP_KERNEL_LAUNCH_CHECK();
  } else {
    fdx::slot8_cpu(a);
  }
}

// hist[slot_node[s]][boff[f] + b][stat] += exact sums of the quantised statistics of the entries of
// the listed work items whose row is in slot s of this pass (slot8 = None: root pass, slot 0).
// RF per-level sampling: thr [n] f64 (k-th smallest priority of each node over 0..F-1) and the
// union mask [Fa] u8 over the active features fid_orig.
// mix64(f) for f in [0, F) (the priorities' per-feature hash, RfSampleArgs / SplitArgs fmix), on
// the device of `like`
Tensor feature_mix(int64_t F, const Tensor& like) {
  FDX_CHECK(F >= 1, "F >= 1");
  Tensor h = at::empty({F}, at::TensorOptions().dtype(at::kLong));
  uint64_t* p = reinterpret_cast<uint64_t*>(h.data_ptr<int64_t>());
  for (int64_t f = 0; f < F; ++f) p[f] = fdx::mix64((uint64_t)f);
  return h.to(like.device());
}

void rf_sample(int64_t seed, int64_t tree, const Tensor& nodes, int64_t F, int64_t k, const Tensor& fid_orig,
               const Tensor& thr, const Tensor& mask, const optional<Tensor>& node_trees) {
  const auto dev = fid_orig.device();
  chk(nodes, dev, at::kInt, "nodes");
  chk(fid_orig, dev, at::kLong, "fid_orig");
  chk(thr, dev, at::kDouble, "thr");
  chk(mask, dev, at::kByte, "mask");
  FDX_CHECK(thr.numel() == nodes.numel() && mask.numel() == fid_orig.numel(), "thr [n], mask [Fa]");
  FDX_CHECK(k >= 1 && F >= 1, "k, F >= 1");
  if (k >= F) {
    thr.fill_(1.0);
    mask.fill_(1);
    return;
  }
  fdx::RfSampleArgs a{};
  a.seed = (uint64_t)seed;
  a.tree = (int32_t)tree;
  a.nodes = nodes.data_ptr<int32_t>();
  a.nnodes = (int32_t)nodes.numel();
  if (node_trees) {
    chk(*node_trees, dev, at::kInt, "node_trees");
    FDX_CHECK(node_trees->numel() == nodes.numel(), "node_trees [n]");
    a.node_trees = node_trees->data_ptr<int32_t>();
  }
  a.F = F;
  a.k = k;
  a.fid_orig = fid_orig.data_ptr<int64_t>();
  a.Fa = fid_orig.numel();
  a.thr = thr.data_ptr<double>();
  a.mask = mask.data_ptr<uint8_t>();
  if (dev.is_cuda()) {
    c10::hip::HIPGuard guard(dev.index());
    Tensor scratch = at::empty({fdx::rf_scratch_bytes(a.nnodes)}, fid_orig.options().dtype(at::kByte));
    a.scratch = scratch.data_ptr<uint8_t>();
    fdx::launch_rf_sample(a, stream(dev));
    C10_HIP_KERNEL_LAUNCH_CHECK();
  } else {
    fdx::rf_sample_cpu(a);
  }
}

// Compact DP layout of an RF level (tree.h RfCompactArgs): local [Fa + 1] int64, sizes [S] int64.
void rf_compact(const Tensor& mask, const Tensor& nbins, const Tensor& fs, const Tensor& local, const Tensor& sizes,
                int64_t max_shard_features) {
  const auto dev = mask.device();
  chk(mask, dev, at::kByte, "mask");
  chk(nbins, dev, at::kInt, "nbins");
  chk(fs, dev, at::kLong, "fs");
  chk(local, dev, at::kLong, "local");
  chk(sizes, dev, at::kLong, "sizes");
  const int64_t Fa = mask.numel();
  FDX_CHECK(nbins.numel() == Fa && local.numel() == Fa + 1 && fs.numel() >= 2 && sizes.numel() == fs.numel() - 1,
            "mask/nbins [Fa], local [Fa + 1], fs [S + 1], sizes [S]");
  fdx::RfCompactArgs a{};
  a.mask = mask.data_ptr<uint8_t>();
  a.nbins = nbins.data_ptr<int32_t>();
  a.fs = fs.data_ptr<int64_t>();
  a.S = (int32_t)(fs.numel() - 1);
  a.Fa = Fa;
  a.local = local.data_ptr<int64_t>();
  a.sizes = sizes.data_ptr<int64_t>();
  if (dev.is_cuda()) {
    c10::hip::HIPGuard guard(dev.index());
    Tensor chunk_sums;
    if (max_shard_features > 0) {      // the multi-workgroup layout (max_shard_features: the largest shard's)
      a.chunk_stride = fdx::rf_compact_chunks(max_shard_features);
      chunk_sums = at::empty({a.S * a.chunk_stride}, local.options());
      a.chunk_sums = chunk_sums.data_ptr<int64_t>();
    }
    fdx::launch_rf_compact(a, stream(dev));
    C10_HIP_KERNEL_LAUNCH_CHECK();
  } else {
    fdx::rf_compact_cpu(a);
  }
}

void hist_build_impl(const Tensor& item_start, const Tensor& item_end, const Tensor& item_f0, const Tensor& item_meta,
                     const optional<Tensor>& wave_item, const Tensor& csc_row, const Tensor& csc_key,
                     const optional<Tensor>& slot8_t, const Tensor& rowdig, const Tensor& boff, const Tensor& nbins,
                     const Tensor& slot_node, const Tensor& hist, int64_t TB, int64_t bt, int64_t ct, int64_t np,
                     const optional<Tensor>& feat_active, const optional<Tensor>& rowpack,
                     const optional<Tensor>& list, const optional<Tensor>& count, bool lds = false,
                     int64_t listed_per_xcd = -1) {
  const auto dev = csc_row.device();
  chk(item_start, dev, at::kLong, "item_start");
  chk(item_end, dev, at::kLong, "item_end");
  chk(item_f0, dev, at::kInt, "item_f0");
  chk(item_meta, dev, at::kInt, "item_meta");
  chk(csc_row, dev, at::kInt, "csc_row");
  chk(csc_key, dev, at::kByte, "csc_key");
  if (slot8_t) chk(*slot8_t, dev, at::kByte, "slot8");
  chk(rowdig, dev, at::kInt, "rowdig");
  chk(boff, dev, at::kLong, "boff");
  chk(nbins, dev, at::kInt, "nbins");
  chk(slot_node, dev, at::kInt, "slot_node");
  chk(hist, dev, at::kLong, "hist");
  const int64_t I = item_start.numel();
  FDX_CHECK(item_end.numel() == I && item_f0.numel() == I && item_meta.numel() == I, "item arrays");
  FDX_CHECK((bt == 1 || bt == 2 || bt == 4) && (ct == 1 || ct == 2 || ct == 4 || ct == 8), "unsupported (bt, ct)");
  FDX_CHECK(np == 1 || np == 4, "np must be 1 or 4");
  const int64_t spt = 16 / (2 * np);
  const int64_t nslots = slot_node.numel();
  FDX_CHECK(nslots >= 1 && nslots <= spt * ct, "slot_node must have 1 .. 16*ct/(2*np) entries");
  FDX_CHECK(slot8_t || rowpack || nslots == 1, "the root pass builds one slot");
  FDX_CHECK(!rowpack || np == 1, "packed row state: np = 1 passes");
  FDX_CHECK(csc_row.numel() == csc_key.numel(), "csc arrays");
  FDX_CHECK(rowdig.dim() == 2 && rowdig.size(1) == 2, "rowdig must be [N,2] int32");
  FDX_CHECK(reinterpret_cast<uintptr_t>(rowdig.data_ptr()) % 8 == 0, "rowdig must be 8-byte aligned");
  FDX_CHECK(!slot8_t || slot8_t->numel() == rowdig.size(0), "slot8 and rowdig row counts differ");
  FDX_CHECK(boff.numel() == nbins.numel() + 1, "boff must be [Fa+1]");
  FDX_CHECK(hist.dim() == 3 && hist.size(2) == 2, "hist must be [rows, stride, 2] int64");
  FDX_CHECK(boff.numel() - 1 == nbins.numel() && hist.size(1) >= TB, "hist stride smaller than the total bin count");
  FDX_CHECK(reinterpret_cast<uintptr_t>(csc_row.data_ptr()) % 16 == 0 &&
                reinterpret_cast<uintptr_t>(csc_key.data_ptr()) % 4 == 0,
            "csc_row must be 16-byte and csc_key 4-byte aligned");
  FDX_CHECK(readable_tail(csc_row, 4) && readable_tail(csc_key, 4),
            "csc_row/csc_key need 4 readable padding entries behind their end (see quantize.CSC_PAD)");
  fdx::HistArgs a{};
  a.listed_per_xcd = -1;
  a.item_start = item_start.data_ptr<int64_t>();
  a.item_end = item_end.data_ptr<int64_t>();
  a.item_f0 = item_f0.data_ptr<int32_t>();
  a.item_meta = item_meta.data_ptr<int32_t>();
  a.num_items = (int32_t)I;
  a.csc_row = csc_row.data_ptr<int32_t>();
  a.csc_key = csc_key.data_ptr<uint8_t>();
  a.slot8 = slot8_t ? slot8_t->data_ptr<uint8_t>() : nullptr;
  a.rowdig = reinterpret_cast<const uint32_t*>(rowdig.data_ptr<int32_t>());
  a.boff = boff.data_ptr<int64_t>();
  a.nbins = nbins.data_ptr<int32_t>();
  a.slot_node = slot_node.data_ptr<int32_t>();
  a.nslots = (int32_t)nslots;
  a.hist_stride = hist.size(1);
  a.hist = hist.data_ptr<int64_t>();
  if (wave_item) {
    chk(*wave_item, dev, at::kInt, "wave_item");
    FDX_CHECK(wave_item->numel() % 4 == 0, "wave_item: 4 slots per workgroup");
    a.wave_item = wave_item->data_ptr<int32_t>();
    a.num_slots = (int32_t)wave_item->numel();
  }
  if (feat_active) {
    chk(*feat_active, dev, at::kByte, "feat_active");
    FDX_CHECK(feat_active->numel() == nbins.numel(), "feat_active must be [Fa] uint8");
    a.feat_active = feat_active->data_ptr<uint8_t>();
  }
  if (rowpack) {
    chk(*rowpack, dev, at::kInt, "rowpack");
    FDX_CHECK(rowpack->numel() == rowdig.size(0), "rowpack must be [N] int32");
    a.rowpack = reinterpret_cast<const uint32_t*>(rowpack->data_ptr<int32_t>());
  }
  if (list) {
    FDX_CHECK(count.has_value() && feat_active.has_value(), "a listed pass needs count and feat_active");
    chk(*list, dev, at::kInt, "list");
    chk(*count, dev, at::kInt, "count");
    // per-XCD lists: XCD x holds the items of its wave slots (workgroups b = x mod 8, 4 slots each)
    const int64_t slots = wave_item ? wave_item->numel() : I;
    const int64_t cap = ((slots + 3) / 4 + 7) / 8 * 4;
    FDX_CHECK(list->numel() >= 8 * cap && count->numel() >= 8,
              "list must hold 8 x ceil(slots / 32) x 4 items, count 8 int32 (one per XCD)");
    a.active_list = list->data_ptr<int32_t>();
    a.active_count = count->data_ptr<int32_t>();
    a.list_cap = (int32_t)cap;
    FDX_CHECK(listed_per_xcd <= cap, "listed_per_xcd exceeds the per-XCD list capacity");
    a.listed_per_xcd = (int32_t)listed_per_xcd;
  }
  // LDS-atomic count kernel: 4 waves x 16 bt keys x nslots int64 cells must fit 64 KB
  a.lds = (lds && np == 1 && !slot8_t && 4 * 16 * bt * nslots * 8 <= 65536) ? 1 : 0;
  if (dev.is_cuda()) {
    c10::hip::HIPGuard guard(dev.index());
    fdx::launch_hist(a, (int)bt, (int)ct, (int)np, stream(dev));
    C10_HIP_KERNEL_LAUNCH_CHECK();
  } else {
    fdx::hist_cpu(a, (int)bt, (int)np);
  }
}

void hist_build(const Tensor& item_start, const Tensor& item_end, const Tensor& item_f0, const Tensor& item_meta,
                const optional<Tensor>& wave_item, const Tensor& csc_row, const Tensor& csc_key,
                const optional<Tensor>& slot8_t, const Tensor& rowdig, const Tensor& boff, const Tensor& nbins,
                const Tensor& slot_node, const Tensor& hist, int64_t TB, int64_t bt, int64_t ct, int64_t np,
                const optional<Tensor>& feat_active) {
  hist_build_impl(item_start, item_end, item_f0, item_meta, wave_item, csc_row, csc_key, slot8_t, rowdig, boff, nbins,
                  slot_node, hist, TB, bt, ct, np, feat_active, nullopt, nullopt, nullopt);
}

// RF count pass (np = 1) over the sampled features' work items: rowpack [N] int32 (tree_slot_pack;
// None at the root: rowdig only), feat_active [Fa] u8, list [>= wave slots] / count [1] int32
// scratch of the listed pass (the active items are compacted on the device, no host round trip;
// None: one wave per wave slot).
void hist_sampled(const Tensor& item_start, const Tensor& item_end, const Tensor& item_f0, const Tensor& item_meta,
                  const optional<Tensor>& wave_item, const Tensor& csc_row, const Tensor& csc_key,
                  const optional<Tensor>& rowpack, const Tensor& rowdig, const Tensor& boff, const Tensor& nbins,
                  const Tensor& slot_node, const Tensor& hist, int64_t TB, int64_t bt, int64_t ct,
                  const Tensor& feat_active, const optional<Tensor>& list, const optional<Tensor>& count,
                  bool lds, int64_t listed_per_xcd) {
  hist_build_impl(item_start, item_end, item_f0, item_meta, wave_item, csc_row, csc_key, nullopt, rowdig, boff, nbins,
                  slot_node, hist, TB, bt, ct, 1, feat_active, rowpack, list, count, lds, listed_per_xcd);
}

// hist_select over several item groups in one call: counts [G, 8] is zeroed here, then group j's
// active items go to lists[j] / counts[j] (the RF level loop queues this with the previous level's
// plan: one host call per level instead of a fill and a launch per group).
void hist_select(const Tensor& item_start, const Tensor& item_f0, const Tensor& item_meta,
                 const optional<Tensor>& wave_item, const Tensor& nbins, const Tensor& feat_active, const Tensor& list,
                 const Tensor& count);

void hist_select_groups(const std::vector<std::vector<Tensor>>& groups, const Tensor& nbins, const Tensor& feat_active,
                        const std::vector<Tensor>& lists, const Tensor& counts) {
  const auto dev = counts.device();
  chk(counts, dev, at::kInt, "counts");
  FDX_CHECK(groups.size() == lists.size() && counts.dim() == 2 && counts.size(0) == (int64_t)groups.size() &&
                counts.size(1) == 8, "groups / lists / counts [G, 8]");
  FDX_CHECK(dev.is_cuda(), "hist_select_groups: device lists only");
  {
    c10::hip::HIPGuard guard(dev.index());
    FDX_CHECK(hipMemsetAsync(counts.data_ptr<int32_t>(), 0, counts.numel() * sizeof(int32_t), stream(dev)) == hipSuccess,
              "hipMemsetAsync failed");
  }
  for (size_t j = 0; j < groups.size(); ++j) {
    const auto& g = groups[j];
    FDX_CHECK(g.size() == 4, "a group is (item_start, item_f0, item_meta, wave_item)");
    hist_select(g[0], g[1], g[2], g[3], nbins, feat_active, lists[j], counts[(int64_t)j]);
  }
}

// Compact the active work items of an item group (feature in feat_active) into per-XCD lists
// ahead of the listed pass that reads them (count [8] int32 zeroed by the caller, atomically
// advanced here): the RF level loop queues this with the previous level's plan so the counts
// reach the host with the level's counts and the pass launches one wave per active item.
void hist_select(const Tensor& item_start, const Tensor& item_f0, const Tensor& item_meta,
                 const optional<Tensor>& wave_item, const Tensor& nbins, const Tensor& feat_active, const Tensor& list,
                 const Tensor& count) {
  const auto dev = item_start.device();
  chk(item_start, dev, at::kLong, "item_start");
  chk(item_f0, dev, at::kInt, "item_f0");
  chk(item_meta, dev, at::kInt, "item_meta");
  chk(nbins, dev, at::kInt, "nbins");
  chk(feat_active, dev, at::kByte, "feat_active");
  chk(list, dev, at::kInt, "list");
  chk(count, dev, at::kInt, "count");
  const int64_t I = item_start.numel();
  FDX_CHECK(item_f0.numel() == I && item_meta.numel() == I && feat_active.numel() == nbins.numel(), "item arrays");
  const int64_t slots = wave_item ? wave_item->numel() : I;
  const int64_t cap = ((slots + 3) / 4 + 7) / 8 * 4;
  FDX_CHECK(list.numel() >= 8 * cap && count.numel() >= 8, "list must hold 8 x ceil(slots / 32) x 4 items, count 8");
  fdx::HistArgs a{};
  a.listed_per_xcd = -1;
  a.item_start = item_start.data_ptr<int64_t>();
  a.item_f0 = item_f0.data_ptr<int32_t>();
  a.item_meta = item_meta.data_ptr<int32_t>();
  a.num_items = (int32_t)I;
  a.nbins = nbins.data_ptr<int32_t>();
  a.feat_active = feat_active.data_ptr<uint8_t>();
  if (wave_item) {
    chk(*wave_item, dev, at::kInt, "wave_item");
    a.wave_item = wave_item->data_ptr<int32_t>();
    a.num_slots = (int32_t)wave_item->numel();
  }
  a.active_list = list.data_ptr<int32_t>();
  a.active_count = count.data_ptr<int32_t>();
  a.list_cap = (int32_t)cap;
  FDX_CHECK(dev.is_cuda(), "hist_select: device lists only (the host pass scans every item)");
  c10::hip::HIPGuard guard(dev.index());
  fdx::launch_hist_select(a, stream(dev));
  C10_HIP_KERNEL_LAUNCH_CHECK();
}

// pack [N] int32 = slot (0xff: not built in this pass) | class-count digits << 8 (np = 1 passes)
void slot_pack(const Tensor& row_node, const Tensor& node_slot, int64_t nslots, const Tensor& rowdig,
               const Tensor& pack) {
  const auto dev = row_node.device();
  chk(row_node, dev, at::kInt, "row_node");
  chk(node_slot, dev, at::kInt, "node_slot");
  chk(rowdig, dev, at::kInt, "rowdig");
  chk(pack, dev, at::kInt, "pack");
  FDX_CHECK(nslots >= 0 && nslots <= 255, "at most 255 slots per pass");
  FDX_CHECK(rowdig.numel() == 2 * row_node.numel() && pack.numel() == row_node.numel(),
            "rowdig [N, 2], pack [N] int32");
  fdx::SlotArgs a{};
  a.row_node = row_node.data_ptr<int32_t>();
  a.node_slot = node_slot.data_ptr<int32_t>();
  a.num_nodes = (int32_t)node_slot.numel();
  a.nslots = (int32_t)nslots;
  a.N = row_node.numel();
  a.rowdig = reinterpret_cast<const uint32_t*>(rowdig.data_ptr<int32_t>());
  a.pack = reinterpret_cast<uint32_t*>(pack.data_ptr<int32_t>());
  if (dev.is_cuda()) {
    c10::hip::HIPGuard guard(dev.index());
    fdx::launch_slot8(a, stream(dev));
    C10_HIP_KERNEL_LAUNCH_CHECK();
  } else {
    fdx::slot8_cpu(a);
  }
}


// Row-group CSR build from the quantized CSC. pass 0: ptr [G, N + 1] int32 (zeroed) += entry
// counts at [g][r + 1]; pass 1: cursor [G, N] (the exclusive starts) advanced, ent (uint16 bits in
// int16) written at gbase[g] + position.
void rg_build(const Tensor& csc_row, const Tensor& csc_bin, const Tensor& colptr, const Tensor& fgroup,
              const Tensor& flocal, int64_t N, int64_t pass, const optional<Tensor>& ptr,
              const optional<Tensor>& cursor, const optional<Tensor>& gbase, const optional<Tensor>& ent) {
  const auto dev = csc_row.device();
  chk(csc_row, dev, at::kInt, "csc_row");
  chk(csc_bin, dev, at::kByte, "csc_bin");
  chk(colptr, dev, at::kLong, "colptr");
  chk(fgroup, dev, at::kInt, "fgroup");
  chk(flocal, dev, at::kInt, "flocal");
  FDX_CHECK(fgroup.numel() + 1 == colptr.numel() && flocal.numel() == fgroup.numel(), "fgroup/flocal must be [Fa]");
  FDX_CHECK(csc_row.numel() == csc_bin.numel(), "csc_row / csc_bin sizes");
  fdx::RgBuildArgs a{};
  a.csc_row = csc_row.data_ptr<int32_t>();
  a.csc_bin = csc_bin.data_ptr<uint8_t>();
  a.colptr = colptr.data_ptr<int64_t>();
  a.Fa = (int32_t)fgroup.numel();
  a.nnz = csc_row.numel();
  a.N = N;
  a.fgroup = fgroup.data_ptr<int32_t>();
  a.flocal = flocal.data_ptr<int32_t>();
  if (pass == 0) {
    FDX_CHECK(ptr.has_value(), "pass 0 needs ptr");
    chk(*ptr, dev, at::kInt, "ptr");
    FDX_CHECK(ptr->dim() == 2 && ptr->size(1) == N + 1, "ptr must be [G, N + 1]");
    a.ptr = reinterpret_cast<uint32_t*>(ptr->data_ptr<int32_t>());
  } else {
    FDX_CHECK(cursor && gbase && ent, "pass 1 needs cursor, gbase, ent");
    chk(*cursor, dev, at::kInt, "cursor");
    chk(*gbase, dev, at::kLong, "gbase");
    FDX_CHECK(cursor->dim() == 2 && cursor->size(1) == N && gbase->numel() == cursor->size(0) + 1,
              "cursor must be [G, N], gbase [G + 1]");
    FDX_CHECK(ent->device() == dev && ent->scalar_type() == at::kShort && ent->is_contiguous(), "ent must be int16");
    a.cursor = reinterpret_cast<uint32_t*>(cursor->data_ptr<int32_t>());
    a.gbase = gbase->data_ptr<int64_t>();
    a.ent = reinterpret_cast<uint16_t*>(ent->data_ptr<int16_t>());
  }
  if (dev.is_cuda()) {
    c10::hip::HIPGuard guard(dev.index());
    fdx::launch_rg_build(a, (int)pass, stream(dev));
    C10_HIP_KERNEL_LAUNCH_CHECK();
  } else {
    fdx::rg_build_cpu(a, (int)pass);
  }
}

// Row-group CSR build from a count-path CSR (indptr, idx, counts float32 / float64 / int32):
// ptr [G, N + 1] int32 gets the exclusive starts of every (group, row) run, ent (int16) the local
// bins at gbase[g] + start + k, in CSR order. work: int32 scratch of >= G * ceil(N / 64).
template <class V>
void rg_build_csr_t(const Tensor& indptr, const Tensor& idx, const Tensor& counts, const Tensor& remap,
                    int64_t max_bin, const Tensor& fgroup, const Tensor& flocal, const Tensor& ptr,
                    const Tensor& gbase, const Tensor& ent, const Tensor& work, const optional<Tensor>& erow,
                    int64_t em_g0, int64_t ebase) {
  const auto dev = indptr.device();
  fdx::RgCsrBuildArgs<V> a{};
  a.indptr = indptr.data_ptr<int64_t>();
  a.idx = idx.data_ptr<int32_t>();
  a.counts = counts.data_ptr<V>();
  a.N = indptr.numel() - 1;
  a.remap = remap.data_ptr<int32_t>();
  a.max_bin = (int32_t)max_bin;
  a.fgroup = fgroup.data_ptr<int32_t>();
  a.flocal = flocal.data_ptr<int32_t>();
  a.G = (int32_t)ptr.size(0);
  a.ptr = reinterpret_cast<uint32_t*>(ptr.data_ptr<int32_t>());
  a.gbase = gbase.data_ptr<int64_t>();
  a.ent = reinterpret_cast<uint16_t*>(ent.data_ptr<int16_t>());
  a.wave_base = reinterpret_cast<uint32_t*>(work.data_ptr<int32_t>());
  if (erow && erow->defined()) {
    a.erow = reinterpret_cast<uint32_t*>(erow->data_ptr<int32_t>());
    a.em_g0 = (int32_t)em_g0;
    a.ebase = ebase;
  }
  if (dev.is_cuda()) {
    c10::hip::HIPGuard guard(dev.index());
    // one [F] lookup instead of the remap -> fgroup / flocal chain (freed in stream order)
    Tensor fgl = at::full({remap.numel()}, -1, remap.options());
    if (fgroup.numel() > 0) {
      const Tensor fa = remap.clamp_min(0).to(at::kLong);
      const Tensor g = fgroup.index_select(0, fa), l = flocal.index_select(0, fa);
      fgl = at::where((remap >= 0) & (g >= 0), g.__lshift__(16).bitwise_or(l), fgl).contiguous();
    }
    a.fgl = fgl.data_ptr<int32_t>();
    fdx::launch_rg_build_csr<V>(a, stream(dev));
    C10_HIP_KERNEL_LAUNCH_CHECK();
  } else {
    fdx::rg_build_csr_cpu<V>(a);
  }
}

void rg_build_csr(const Tensor& indptr, const Tensor& idx, const Tensor& counts, const Tensor& remap,
                  int64_t max_bin, const Tensor& fgroup, const Tensor& flocal, const Tensor& ptr,
                  const Tensor& gbase, const Tensor& ent, const Tensor& work, const optional<Tensor>& erow,
                  int64_t em_g0, int64_t ebase) {
  const auto dev = indptr.device();
  chk(indptr, dev, at::kLong, "indptr");
  if (erow && erow->defined()) {
    chk(*erow, dev, at::kInt, "erow");
    FDX_CHECK(em_g0 >= 0 && em_g0 <= ptr.size(0) && ebase >= 0 && ebase <= ent.numel() &&
                  erow->numel() >= ent.numel() - ebase, "erow must cover the entries from ebase on");
  }
  chk(idx, dev, at::kInt, "idx");
  chk(remap, dev, at::kInt, "remap");
  chk(fgroup, dev, at::kInt, "fgroup");
  chk(flocal, dev, at::kInt, "flocal");
  chk(ptr, dev, at::kInt, "ptr");
  chk(gbase, dev, at::kLong, "gbase");
  chk(work, dev, at::kInt, "work");
  FDX_CHECK(ent.device() == dev && ent.scalar_type() == at::kShort && ent.is_contiguous(), "ent must be int16");
  FDX_CHECK(counts.device() == dev && counts.is_contiguous() && counts.numel() >= idx.numel(), "counts");
  FDX_CHECK(ptr.dim() == 2 && ptr.size(1) == indptr.numel() && ptr.size(0) <= 128,
            "ptr must be [G <= 128, N + 1]");
  FDX_CHECK(gbase.numel() == ptr.size(0) + 1, "gbase must be [G + 1]");
  FDX_CHECK(fgroup.numel() == flocal.numel(), "fgroup / flocal");
  FDX_CHECK(work.numel() >= ptr.size(0) * fdx::rg_build_csr_waves(indptr.numel() - 1), "work too small");
  switch (counts.scalar_type()) {
    case at::kFloat: rg_build_csr_t<float>(indptr, idx, counts, remap, max_bin, fgroup, flocal, ptr, gbase, ent, work, erow,
                                               em_g0, ebase); break;
    case at::kDouble: rg_build_csr_t<double>(indptr, idx, counts, remap, max_bin, fgroup, flocal, ptr, gbase, ent, work, erow,
                                               em_g0, ebase); break;
    case at::kInt: rg_build_csr_t<int32_t>(indptr, idx, counts, remap, max_bin, fgroup, flocal, ptr, gbase, ent, work, erow,
                                               em_g0, ebase); break;
    default: FDX_CHECK(false, "counts must be float32, float64 or int32");
  }
}

// Built rows of a level grouped by slot: list [N] int32, slot_start [nslots + 1] int32 (device).
// The slot of a row is node_slot[row_node[r]] (row_node given) or slot8[r]. work: int32 scratch of
// at least nslots * (2 + ceil(N / rg_list_rows(N))). With rowdig, listdig [N, 2] receives the digit
// words of the listed rows by list position.
void rg_list(const optional<Tensor>& row_node, const optional<Tensor>& node_slot, const optional<Tensor>& slot8,
             int64_t N, int64_t nslots, const Tensor& work, const Tensor& slot_start, const Tensor& list,
             const optional<Tensor>& rowdig, const optional<Tensor>& listdig, const optional<Tensor>& masked,
             bool counted) {
  const auto dev = list.device();
  chk(work, dev, at::kInt, "work");
  chk(slot_start, dev, at::kInt, "slot_start");
  chk(list, dev, at::kInt, "list");
  FDX_CHECK(nslots >= 1 && nslots <= fdx::kRgMaxSlots, "nslots out of range");
  FDX_CHECK(list.numel() >= N && slot_start.numel() >= nslots + 1, "list / slot_start sizes");
  const int64_t nwaves = (N + fdx::rg_list_rows(N) - 1) / fdx::rg_list_rows(N);
  FDX_CHECK(work.numel() >= 2 * nslots + nslots * nwaves, "work too small");
  fdx::RgListArgs a{};
  if (row_node) {
    FDX_CHECK(node_slot.has_value(), "row_node needs node_slot");
    chk(*row_node, dev, at::kInt, "row_node");
    chk(*node_slot, dev, at::kInt, "node_slot");
    FDX_CHECK(row_node->numel() >= N, "row_node must cover the rows");
    a.row_node = row_node->data_ptr<int32_t>();
    a.node_slot = node_slot->data_ptr<int32_t>();
    a.num_nodes = (int32_t)node_slot->numel();
  } else {
    FDX_CHECK(slot8.has_value(), "slot8 or row_node required");
    chk(*slot8, dev, at::kByte, "slot8");
    FDX_CHECK(slot8->numel() >= N, "slot8 must cover the rows");
    a.slot8 = slot8->data_ptr<uint8_t>();
  }
  a.N = N;
  a.nslots = (int32_t)nslots;
  a.counted = counted ? 1 : 0;        // (the partition's row pass wrote pass 0's counts)
  a.slot_count = work.data_ptr<int32_t>();
  a.wave_count = a.slot_count + 2 * nslots;
  a.slot_start = slot_start.data_ptr<int32_t>();
  a.list = list.data_ptr<int32_t>();
  FDX_CHECK(rowdig.has_value() == listdig.has_value(), "rowdig and listdig go together");
  if (rowdig) {
    chk(*rowdig, dev, at::kInt, "rowdig");
    chk(*listdig, dev, at::kInt, "listdig");
    FDX_CHECK(rowdig->numel() >= 2 * N && listdig->numel() >= 2 * N, "rowdig / listdig must be [N, 2]");
    a.rowdig = reinterpret_cast<const uint32_t*>(rowdig->data_ptr<int32_t>());
    a.listdig = reinterpret_cast<uint32_t*>(listdig->data_ptr<int32_t>());
  }
  if (masked && masked->defined()) {
    FDX_CHECK(rowdig.has_value() && nslots == 1, "masked digit words need rowdig and one slot");
    chk(*masked, dev, at::kInt, "masked");
    FDX_CHECK(masked->numel() >= 2 * N, "masked must be [N, 2]");
    a.masked = reinterpret_cast<uint32_t*>(masked->data_ptr<int32_t>());
  }
  if (dev.is_cuda()) {
    c10::hip::HIPGuard guard(dev.index());
    fdx::launch_rg_list(a, stream(dev));
    C10_HIP_KERNEL_LAUNCH_CHECK();
  } else {
    fdx::rg_list_cpu(a);
  }
}

// Row-group histogram pass: hist[(slot_node[s] * stride + off(gbin[g][b])) * 2 + stat] += exact
// sums over the built rows (list = None: every row, one slot). wg [3, n_wg]: the work table.
void rg_hist(const Tensor& ptr, const Tensor& ent, const Tensor& gbase, const Tensor& gbin, const Tensor& rowdig,
             int64_t np, const optional<Tensor>& list, const optional<Tensor>& slot_start,
             const optional<Tensor>& listdig, int64_t nslots, const Tensor& gmode, const Tensor& wg,
             const Tensor& slot_node, const Tensor& hist, int64_t stride, const optional<Tensor>& shard_lo,
             int64_t shard_stride, int64_t dbg, const optional<Tensor>& erow, int64_t ebase,
             const optional<Tensor>& emdig, int64_t em_min_rows, const optional<Tensor>& part,
             const optional<Tensor>& wg_first) {
  const auto dev = ptr.device();
  chk(ptr, dev, at::kInt, "ptr");
  chk(gbase, dev, at::kLong, "gbase");
  chk(gbin, dev, at::kInt, "gbin");
  chk(rowdig, dev, at::kInt, "rowdig");
  chk(slot_node, dev, at::kInt, "slot_node");
  chk(hist, dev, at::kLong, "hist");
  FDX_CHECK(ent.device() == dev && ent.scalar_type() == at::kShort && ent.is_contiguous(), "ent must be int16");
  FDX_CHECK(ptr.dim() == 2, "ptr must be [G, N + 1]");
  const int64_t G = ptr.size(0), N = ptr.size(1) - 1;
  FDX_CHECK(gbin.dim() == 2 && gbin.size(0) == G && (gbin.size(1) == 4096 || gbin.size(1) == 8192) &&
                gbase.numel() == G + 1, "gbase [G + 1] / gbin [G, 4096 or 8192]");
  FDX_CHECK(rowdig.dim() == 2 && rowdig.size(0) == N && rowdig.size(1) == 2, "rowdig must be [N, 2]");
  FDX_CHECK(reinterpret_cast<uintptr_t>(ent.data_ptr()) % 16 == 0 && readable_tail(ent, 8),
            "ent must be 16-byte aligned with 8 readable padding entries");
  FDX_CHECK(np == 1 || np == 4, "np must be 1 or 4");
  chk(wg, dev, at::kInt, "wg");
  FDX_CHECK(wg.dim() == 2 && wg.size(0) == 3, "wg must be [3, n_wg] (group, chunk, chunks)");
  FDX_CHECK(list.has_value() == slot_start.has_value(), "list and slot_start go together");
  chk(gmode, dev, at::kByte, "gmode");
  FDX_CHECK(gmode.numel() == G, "gmode must be [G]");
  if (list) {
    chk(*list, dev, at::kInt, "list");
    chk(*slot_start, dev, at::kInt, "slot_start");
    FDX_CHECK(listdig.has_value(), "a list pass needs listdig");
    chk(*listdig, dev, at::kInt, "listdig");
    FDX_CHECK(list->numel() >= N && slot_start->numel() >= nslots + 1 && listdig->numel() >= 2 * N,
              "list / slot_start / listdig sizes");
    FDX_CHECK(nslots >= 1 && nslots <= fdx::kRgMaxSlots, "nslots out of range");
  } else {
    FDX_CHECK(nslots == 1, "the all-rows pass has one slot");
  }
  FDX_CHECK(slot_node.numel() >= nslots, "slot_node must cover the slots");
  FDX_CHECK(hist.dim() == 3 && hist.size(2) == 2 && hist.size(1) == stride, "hist must be [rows, stride, 2] int64");
  fdx::RgHistArgs a{};
  a.ptr = reinterpret_cast<const uint32_t*>(ptr.data_ptr<int32_t>());
  a.ent = reinterpret_cast<const uint16_t*>(ent.data_ptr<int16_t>());
  a.gbase = gbase.data_ptr<int64_t>();
  a.gbin = gbin.data_ptr<int32_t>();
  a.gbins = (int32_t)gbin.size(1);
  a.G = (int32_t)G;
  a.N = N;
  a.rowdig = reinterpret_cast<const uint32_t*>(rowdig.data_ptr<int32_t>());
  a.np = (int32_t)np;
  a.list = opt<int32_t>(list);
  a.slot_start = opt<int32_t>(slot_start);
  a.listdig = list ? reinterpret_cast<const uint32_t*>(listdig->data_ptr<int32_t>()) : nullptr;
  a.gmode = gmode.data_ptr<uint8_t>();
  a.nslots = (int32_t)nslots;
  a.wg_g = wg.data_ptr<int32_t>();
  a.wg_p = a.wg_g + wg.size(1);
  a.wg_np = a.wg_p + wg.size(1);
  a.n_wg = (int32_t)wg.size(1);
  a.dbg = (int32_t)dbg;
  a.slot_node = slot_node.data_ptr<int32_t>();
  a.hist_stride = stride;
  a.hist = hist.data_ptr<int64_t>();
  if (shard_lo && shard_lo->defined()) {
    chk(*shard_lo, dev, at::kLong, "shard_lo");
    a.nshards = (int32_t)(shard_lo->numel() - 1);
    a.shard_lo = shard_lo->data_ptr<int64_t>();
    a.shard_stride = shard_stride;
  }
  if (erow && erow->defined()) {
    chk(*erow, dev, at::kInt, "erow");
    // (ent holds exactly gbase[G] entries: no device read here)
    FDX_CHECK(ebase >= 0 && ebase <= ent.numel() && erow->numel() >= ent.numel() - ebase,
              "erow must cover the entries from ebase on");
    a.erow = reinterpret_cast<const uint32_t*>(erow->data_ptr<int32_t>());
    a.ebase = ebase;
    a.em_min_rows = em_min_rows;
    if (list && emdig && emdig->defined()) {     // (without emdig a listed level keeps the row lists)
      chk(*emdig, dev, at::kInt, "emdig");
      FDX_CHECK(emdig->numel() >= 2 * N, "emdig must be [N, 2]");
      a.emdig = reinterpret_cast<const uint32_t*>(emdig->data_ptr<int32_t>());
    }
  }
  if (part && part->defined() && dev.is_cuda()) {     // (the host twin adds straight into hist)
    FDX_CHECK(wg_first.has_value() && (nslots == 1 || list), "partial tables: wg_first (several slots: a list pass)");
    chk(*part, dev, at::kLong, "part");
    chk(*wg_first, dev, at::kInt, "wg_first");
    FDX_CHECK(part->numel() >= 2 * a.n_wg * (int64_t)a.gbins && wg_first->numel() == G + 1 &&
                  reinterpret_cast<uintptr_t>(part->data_ptr()) % 16 == 0, "part [n_wg, gbins, 2], wg_first [G + 1]");
    a.part = part->data_ptr<int64_t>();
    a.wg_first = wg_first->data_ptr<int32_t>();
  }
  if (dev.is_cuda()) {
    c10::hip::HIPGuard guard(dev.index());
    fdx::launch_rg_hist(a, stream(dev));
    C10_HIP_KERNEL_LAUNCH_CHECK();
  } else {
    fdx::rg_hist_cpu(a);
  }
}

// Row of every entry of the groups from g0 on (entry-major sparse pass): erow[gbase[g] - gbase[g0] + e].
void rg_erow(const Tensor& ptr, const Tensor& gbase, int64_t g0, const Tensor& erow) {
  const auto dev = ptr.device();
  chk(ptr, dev, at::kInt, "ptr");
  chk(gbase, dev, at::kLong, "gbase");
  chk(erow, dev, at::kInt, "erow");
  FDX_CHECK(ptr.dim() == 2 && gbase.numel() == ptr.size(0) + 1, "ptr [G, N + 1] / gbase [G + 1]");
  const int64_t G = ptr.size(0), N = ptr.size(1) - 1;
  FDX_CHECK(g0 >= 0 && g0 <= G, "g0 out of range");
  const Tensor gb = gbase.cpu();
  const int64_t* gh = gb.data_ptr<int64_t>();
  FDX_CHECK(erow.numel() >= gh[G] - gh[g0], "erow must cover the entries from gbase[g0] on");
  fdx::RgErowArgs a{};
  a.ptr = reinterpret_cast<const uint32_t*>(ptr.data_ptr<int32_t>());
  a.gbase = gbase.data_ptr<int64_t>();
  a.G = (int32_t)G;
  a.g0 = (int32_t)g0;
  a.N = N;
  a.ebase = gh[g0];
  a.erow = reinterpret_cast<uint32_t*>(erow.data_ptr<int32_t>());
  if (dev.is_cuda()) {
    c10::hip::HIPGuard guard(dev.index());
    fdx::launch_rg_erow(a, stream(dev));
    C10_HIP_KERNEL_LAUNCH_CHECK();
  } else {
    fdx::rg_erow_cpu(a);
  }
}

// Dense hot-feature histograms (see DenseHistArgs): gfid/gdense [ngroups * fg] with fg =
// tree_dense_fg(bt, ct); rows are processed in ranges of range_rows (multiple of 64).
void hist_dense(const Tensor& dense, const Tensor& digp, const Tensor& rowdig, const optional<Tensor>& slot8_t,
                const Tensor& gfid, const Tensor& gdense, const Tensor& boff, const Tensor& nbins,
                const Tensor& slot_node, const Tensor& hist, int64_t TB, int64_t n_rows, int64_t range_rows,
                int64_t bt, int64_t ct, int64_t np) {
  const auto dev = dense.device();
  chk(dense, dev, at::kByte, "dense");
  chk(digp, dev, at::kByte, "digp");
  chk(rowdig, dev, at::kInt, "rowdig");
  if (slot8_t) chk(*slot8_t, dev, at::kByte, "slot8");
  chk(gfid, dev, at::kInt, "gfid");
  chk(gdense, dev, at::kInt, "gdense");
  chk(boff, dev, at::kLong, "boff");
  chk(nbins, dev, at::kInt, "nbins");
  chk(slot_node, dev, at::kInt, "slot_node");
  chk(hist, dev, at::kLong, "hist");
  FDX_CHECK((bt == 1 || bt == 2 || bt == 4) && (ct == 1 || ct == 2 || ct == 4 || ct == 8), "unsupported (bt, ct)");
  FDX_CHECK(np == 1 || np == 4, "np must be 1 or 4");
  const int64_t fg = fdx::dense_features_per_wave((int)bt, slot8_t ? (int)ct : 1);
  FDX_CHECK(gfid.numel() == gdense.numel() && gfid.numel() % (fg * fdx::dense_waves_per_group()) == 0,
            "gfid/gdense must be [ngroups * fg], ngroups a multiple of tree_dense_waves()");
  const int64_t n_pad = dense.size(1);
  FDX_CHECK(dense.dim() == 2 && n_pad % 64 == 0 && n_pad >= n_rows, "dense must be [Fh, n_pad], n_pad % 64 == 0");
  FDX_CHECK(digp.dim() == 2 && digp.size(0) >= 2 * np && digp.size(1) == n_pad, "digp must be [2*np, n_pad]");
  FDX_CHECK(rowdig.dim() == 2 && rowdig.size(0) == n_rows, "rowdig rows");
  FDX_CHECK(!slot8_t || slot8_t->numel() >= n_pad, "slot8 must be padded to n_pad (0xff)");
  FDX_CHECK(range_rows > 0 && range_rows % 64 == 0, "range_rows must be a positive multiple of 64");
  const int64_t nslots = slot_node.numel();
  FDX_CHECK(nslots >= 1 && nslots <= (16 / (2 * np)) * ct, "slot_node size");
  FDX_CHECK(slot8_t || nslots == 1, "the root pass builds one slot");
  FDX_CHECK(hist.dim() == 3 && hist.size(2) == 2 && hist.size(1) >= TB, "hist must be [rows, >= TB, 2] int64");
  FDX_CHECK(boff.numel() == nbins.numel() + 1, "boff must be [Fa+1]");
  fdx::DenseHistArgs a{};
  a.dense = dense.data_ptr<uint8_t>();
  a.digp = digp.data_ptr<uint8_t>();
  a.rowdig = reinterpret_cast<const uint32_t*>(rowdig.data_ptr<int32_t>());
  a.n_rows = n_rows;
  a.slot8 = slot8_t ? slot8_t->data_ptr<uint8_t>() : nullptr;
  a.n_pad = n_pad;
  a.range_rows = range_rows;
  a.nranges = (int32_t)((n_pad + range_rows - 1) / range_rows);
  a.ngroups = (int32_t)(gfid.numel() / fg);
  a.gfid = gfid.data_ptr<int32_t>();
  a.gdense = gdense.data_ptr<int32_t>();
  a.boff = boff.data_ptr<int64_t>();
  a.nbins = nbins.data_ptr<int32_t>();
  a.slot_node = slot_node.data_ptr<int32_t>();
  a.nslots = (int32_t)nslots;
  a.hist_stride = hist.size(1);
  a.hist = hist.data_ptr<int64_t>();
  if (a.ngroups == 0) return;
  if (dev.is_cuda()) {
    c10::hip::HIPGuard guard(dev.index());
    fdx::launch_hist_dense(a, (int)bt, (int)ct, (int)np, stream(dev));
    C10_HIP_KERNEL_LAUNCH_CHECK();
  } else {
    fdx::hist_dense_cpu(a, (int)fg, (int)np);
  }
}

int64_t dense_fg(int64_t bt, int64_t ct) { return fdx::dense_features_per_wave((int)bt, (int)ct); }
int64_t dense_waves() { return fdx::dense_waves_per_group(); }

void hist_subtract(const Tensor& parent, const Tensor& cur, const Tensor& dst, const Tensor& par, const Tensor& sib,
                   int64_t TB) {
  const auto dev = cur.device();
  chk(parent, dev, at::kLong, "parent");
  chk(cur, dev, at::kLong, "cur");
  chk(dst, dev, at::kInt, "dst");
  chk(par, dev, at::kInt, "par");
  chk(sib, dev, at::kInt, "sib");
  const int32_t n = (int32_t)dst.numel();
  if (dev.is_cuda()) {
    c10::hip::HIPGuard guard(dev.index());
    fdx::launch_hist_subtract(parent.data_ptr<int64_t>(), cur.data_ptr<int64_t>(), dst.data_ptr<int32_t>(),
                              par.data_ptr<int32_t>(), sib.data_ptr<int32_t>(), n, TB, stream(dev));
    C10_HIP_KERNEL_LAUNCH_CHECK();
  } else {
    fdx::hist_subtract_cpu(parent.data_ptr<int64_t>(), cur.data_ptr<int64_t>(), dst.data_ptr<int32_t>(),
                           par.data_ptr<int32_t>(), sib.data_ptr<int32_t>(), n, TB);
  }
}

// best split per node: packed [nodes, 5] int64 {gain bits, feature + f0, bin, left0, left1}
void split_best(const Tensor& gain, const Tensor& bin, const Tensor& left, int64_t f0, const Tensor& out) {
  const auto dev = gain.device();
  chk(gain, dev, at::kDouble, "gain");
  chk(bin, dev, at::kInt, "bin");
  chk(left, dev, at::kLong, "left");
  chk(out, dev, at::kLong, "out");
  FDX_CHECK(gain.dim() == 2 && bin.sizes() == gain.sizes() && left.numel() == 2 * gain.numel(), "gain/bin [n, Fa], left [n, Fa, 2]");
  const int32_t nodes = (int32_t)gain.size(0), Fa = (int32_t)gain.size(1);
  FDX_CHECK(out.numel() == 5ll * nodes, "out must be [nodes, 5]");
  if (dev.is_cuda()) {
    c10::hip::HIPGuard guard(dev.index());
    fdx::launch_split_best(gain.data_ptr<double>(), bin.data_ptr<int32_t>(), left.data_ptr<int64_t>(), nodes, Fa, f0,
                           out.data_ptr<int64_t>(), stream(dev));
    C10_HIP_KERNEL_LAUNCH_CHECK();
  } else {
    fdx::split_best_cpu(gain.data_ptr<double>(), bin.data_ptr<int32_t>(), left.data_ptr<int64_t>(), nodes, Fa, f0,
                        out.data_ptr<int64_t>());
  }
}

void split_find(const Tensor& hist, const Tensor& totals, const Tensor& boff, const Tensor& nbins, const Tensor& zbin,
                const Tensor& fid_orig, const Tensor& node_ids, const Tensor& kexp, int64_t mode, double lambda_,
                double mcw, const optional<Tensor>& feat_thr, int64_t seed, int64_t tree, const Tensor& out_gain,
                const Tensor& out_bin, const Tensor& out_left, const optional<Tensor>& node_tree,
                const optional<Tensor>& wide, const optional<Tensor>& row_of) {
  const auto dev = hist.device();
  chk(hist, dev, at::kLong, "hist");
  chk(totals, dev, at::kLong, "totals");
  chk(boff, dev, at::kLong, "boff");
  chk(nbins, dev, at::kInt, "nbins");
  chk(zbin, dev, at::kInt, "zbin");
  chk(fid_orig, dev, at::kLong, "fid_orig");
  chk(node_ids, dev, at::kInt, "node_ids");
  chk(kexp, dev, at::kInt, "kexp");
  chk(out_gain, dev, at::kDouble, "out_gain");
  chk(out_bin, dev, at::kInt, "out_bin");
  chk(out_left, dev, at::kLong, "out_left");
  const int32_t nodes = (int32_t)node_ids.numel();
  const int32_t Fa = (int32_t)nbins.numel();
  FDX_CHECK(out_gain.numel() >= (int64_t)nodes * Fa && out_left.numel() >= 2ll * nodes * Fa, "outputs too small");
  FDX_CHECK(totals.numel() >= 2 * nodes, "totals size");
  FDX_CHECK(kexp.numel() == 2, "kexp size");
  if (feat_thr) { chk(*feat_thr, dev, at::kDouble, "feat_thr"); FDX_CHECK(feat_thr->numel() >= nodes, "feat_thr size"); }
  fdx::SplitArgs a{};
  a.hist = hist.data_ptr<int64_t>();
  a.totals = totals.data_ptr<int64_t>();
  // the node row stride is the tensor's own ([nodes, stride, 2]): a data-parallel level searches
  // the reduce-scattered [n, Bs, 2] rows in place (Bs >= this shard's bins)
  FDX_CHECK(hist.dim() == 3 && hist.size(2) == 2, "hist must be [rows, stride, 2]");
  if (row_of && row_of->defined()) {
    // (the rows are level_rows' own: every one lies in this buffer, no device read here)
    chk(*row_of, dev, at::kInt, "row_of");
    FDX_CHECK(row_of->numel() >= nodes, "row_of must cover the nodes");
    a.row_of = row_of->data_ptr<int32_t>();
  } else {
    FDX_CHECK(hist.size(0) >= nodes, "hist must have a row per node");
  }
  // (the row stride comes from hist, never the kernels' boff[Fa] fallback: a compact DP level's
  // boff[Fa] is the next shard's offset, not this shard's bin total)
  FDX_CHECK(hist.size(1) > 0, "hist rows of at least one bin");
  a.hist_stride = hist.size(1);
  a.num_nodes = nodes;
  a.Fa = Fa;
  a.boff = boff.data_ptr<int64_t>();
  a.nbins = nbins.data_ptr<int32_t>();
  a.zbin = zbin.data_ptr<int32_t>();
  a.fid_orig = fid_orig.data_ptr<int64_t>();
  a.node_ids = node_ids.data_ptr<int32_t>();
  a.kexp = kexp.data_ptr<int32_t>();
  a.mode = (int32_t)mode;
  a.lambda_ = lambda_;
  a.min_child_weight = mcw;
  a.feat_thr = opt<double>(feat_thr);
  a.seed = (uint64_t)seed;
  a.tree = (int32_t)tree;
  if (node_tree) {
    chk(*node_tree, dev, at::kInt, "node_tree");
    FDX_CHECK(node_tree->numel() >= nodes, "node_tree size");
    a.node_tree = node_tree->data_ptr<int32_t>();
  }
  a.out_gain = out_gain.data_ptr<double>();
  a.out_bin = out_bin.data_ptr<int32_t>();
  a.out_left = out_left.data_ptr<int64_t>();
  if (wide && wide->defined() && wide->numel() > 0) {      // (features with > kSplitWide bins)
    chk(*wide, dev, at::kInt, "wide");
    a.wide = wide->data_ptr<int32_t>();
    a.n_wide = (int32_t)wide->numel();
  }
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
               const Tensor& csc_bin, const optional<Tensor>& node_dense, const optional<Tensor>& dense) {
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
  FDX_CHECK(reinterpret_cast<uintptr_t>(row_node.data_ptr()) % 16 == 0, "row_node must be 16-byte aligned");
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
  if (node_dense) {
    FDX_CHECK(dense.has_value(), "node_dense needs the dense bin block");
    chk(*node_dense, dev, at::kInt, "node_dense");
    chk(*dense, dev, at::kByte, "dense");
    FDX_CHECK(node_dense->numel() == 4ll * a.num_nodes, "node_dense must be [num_nodes, 4]");
    FDX_CHECK(dense->dim() == 2 && dense->size(1) >= a.N, "dense must be [Fh, n_pad >= N]");
    a.node_dense = node_dense->data_ptr<int32_t>();
    a.dense = dense->data_ptr<uint8_t>();
    a.n_pad = dense->size(1);
  }
  if (dev.is_cuda()) {
    c10::hip::HIPGuard guard(dev.index());
    fdx::launch_partition(a, stream(dev));
    C10_HIP_KERNEL_LAUNCH_CHECK();
  } else {
    fdx::partition_cpu(a);
  }
}

// Data-parallel level rows (tree.h LevelRowsArgs): nb slots, row_of [>= n_open], triples [nb].
void level_rows(const Tensor& s2n, const Tensor& sub_dst, const Tensor& sub_par, const optional<Tensor>& prev_row_of,
                int64_t nb, int64_t bld_base, int64_t sub_base, const Tensor& row_of, const Tensor& dst_row,
                const Tensor& par_row, const Tensor& sib_row) {
  const auto dev = s2n.device();
  for (const Tensor* t : {&s2n, &sub_dst, &sub_par, &row_of, &dst_row, &par_row, &sib_row})
    chk(*t, dev, at::kInt, "level_rows int32 array");
  FDX_CHECK(nb >= 0 && s2n.numel() >= nb && sub_dst.numel() >= nb && sub_par.numel() >= nb && dst_row.numel() >= nb &&
                par_row.numel() >= nb && sib_row.numel() >= nb, "level_rows: [nb] arrays");
  FDX_CHECK(bld_base >= 0 && sub_base >= 0 && sub_base + nb <= INT32_MAX, "level_rows: bases");
  fdx::LevelRowsArgs a{};
  a.s2n = s2n.data_ptr<int32_t>();
  a.sub_dst = sub_dst.data_ptr<int32_t>();
  a.sub_par = sub_par.data_ptr<int32_t>();
  if (prev_row_of && prev_row_of->defined()) {
    chk(*prev_row_of, dev, at::kInt, "prev_row_of");
    a.prev_row_of = prev_row_of->data_ptr<int32_t>();
  }
  a.nb = (int32_t)nb;
  a.bld_base = (int32_t)bld_base;
  a.sub_base = (int32_t)sub_base;
  a.row_of = row_of.data_ptr<int32_t>();
  a.dst_row = dst_row.data_ptr<int32_t>();
  a.par_row = par_row.data_ptr<int32_t>();
  a.sib_row = sib_row.data_ptr<int32_t>();
  if (dev.is_cuda()) {
    c10::hip::HIPGuard guard(dev.index());
    fdx::launch_level_rows(a, stream(dev));
    C10_HIP_KERNEL_LAUNCH_CHECK();
  } else {
    fdx::level_rows_cpu(a);
  }
}

// Device level loop (tree.h level_plan): applies the level's best splits and plans the next level.
void level_plan(const Tensor& packed, int64_t L, int64_t depth, int64_t max_depth, int64_t mode, bool build_all,
                const Tensor& kexp, double min_gain, const Tensor& zbin,
                const optional<Tensor>& hot_row, const Tensor& n_nodes, const Tensor& stats, const Tensor& parent,
                const Tensor& left, const Tensor& right, const Tensor& feat, const Tensor& bin, const Tensor& leaf,
                const Tensor& gain, const Tensor& open, const Tensor& n_open, const Tensor& default_child,
                const optional<Tensor>& node_dense, const Tensor& cs_feat, const Tensor& cs_default,
                const Tensor& cs_other, const Tensor& cs_bin, const Tensor& cs_left_default, const Tensor& counts,
                const Tensor& next_open, const Tensor& next_totals, const Tensor& node_slot, const Tensor& s2n,
                const Tensor& sub_dst, const Tensor& sub_par, const Tensor& sub_sib) {
  const auto dev = packed.device();
  FDX_CHECK(packed.device() == dev && packed.scalar_type() == at::kLong, "packed must be int64");
  chk(stats, dev, at::kLong, "stats");
  chk(next_totals, dev, at::kLong, "next_totals");
  chk(gain, dev, at::kDouble, "gain");
  chk(leaf, dev, at::kByte, "leaf");
  for (const Tensor* t : {&zbin, &n_nodes, &parent, &left, &right, &feat, &bin, &open, &n_open, &default_child, &cs_feat,
                          &cs_default, &cs_other, &cs_bin, &cs_left_default, &counts, &next_open, &node_slot, &s2n,
                          &sub_dst, &sub_par, &sub_sib})
    chk(*t, dev, at::kInt, "level_plan int32 array");
  const int64_t M = parent.numel();
  // packed: [L, 5] or the all-gathered [S, L, 5] of a data-parallel level (best over shards here);
  // the shard stride is the tensor's own, so a tree's [S, L, 5] slice of a batched all-gather
  // ([S, sum L, 5] over the trees in flight) is read in place
  const int64_t S = packed.dim() == 3 ? packed.size(0) : 1;
  FDX_CHECK((packed.dim() == 2 || packed.dim() == 3) && packed.size(-1) == 5 && packed.stride(-1) == 1 &&
                packed.stride(-2) == 5 && packed.size(-2) >= L, "packed must be [L, 5] or [S, L, 5] with rows of 5");
  FDX_CHECK(L >= 1 && open.numel() >= L, "open [L]");
  FDX_CHECK(stats.numel() == 2 * M && left.numel() == M && right.numel() == M && feat.numel() == M &&
                bin.numel() == M && leaf.numel() == M && gain.numel() == M && default_child.numel() == M &&
                node_slot.numel() == M, "node tables must be [max_nodes]");
  FDX_CHECK(next_open.numel() >= 2 * L && next_totals.numel() >= 4 * L && s2n.numel() >= L && sub_dst.numel() >= L &&
                sub_par.numel() >= L && sub_sib.numel() >= L && cs_feat.numel() >= L && cs_default.numel() >= L &&
                cs_other.numel() >= L && cs_bin.numel() >= L && cs_left_default.numel() >= L && counts.numel() >= 4,
            "level_plan output capacities");
  fdx::LevelPlanArgs a{};
  a.packed = packed.data_ptr<int64_t>();
  a.L = (int32_t)L;
  a.n_shards = (int32_t)S;
  a.shard_stride = packed.dim() == 3 ? packed.stride(0) : packed.size(-2) * 5;
  a.depth = (int32_t)depth;
  a.max_depth = (int32_t)max_depth;
  a.mode = (int32_t)mode;
  a.build_all = build_all ? 1 : 0;
  chk(kexp, dev, at::kInt, "kexp");
  FDX_CHECK(kexp.numel() == 2, "kexp [2]");
  a.kexp = kexp.data_ptr<int32_t>();
  a.min_gain = min_gain;
  a.zbin = zbin.data_ptr<int32_t>();
  if (hot_row) {
    chk(*hot_row, dev, at::kInt, "hot_row");
    FDX_CHECK(hot_row->numel() == zbin.numel(), "hot_row must be [Fa]");
    a.hot_row = hot_row->data_ptr<int32_t>();
  }
  a.max_nodes = (int32_t)M;
  a.n_nodes = n_nodes.data_ptr<int32_t>();
  a.stats = stats.data_ptr<int64_t>();
  a.parent = parent.data_ptr<int32_t>();
  a.left = left.data_ptr<int32_t>();
  a.right = right.data_ptr<int32_t>();
  a.feat = feat.data_ptr<int32_t>();
  a.bin = bin.data_ptr<int32_t>();
  a.leaf = leaf.data_ptr<uint8_t>();
  a.gain = gain.data_ptr<double>();
  a.open = open.data_ptr<int32_t>();
  a.n_open = n_open.data_ptr<int32_t>();
  a.default_child = default_child.data_ptr<int32_t>();
  if (node_dense) {
    chk(*node_dense, dev, at::kInt, "node_dense");
    FDX_CHECK(node_dense->numel() == 4 * M, "node_dense must be [max_nodes, 4]");
    a.node_dense = node_dense->data_ptr<int32_t>();
  }
  a.cs_feat = cs_feat.data_ptr<int32_t>();
  a.cs_default = cs_default.data_ptr<int32_t>();
  a.cs_other = cs_other.data_ptr<int32_t>();
  a.cs_bin = cs_bin.data_ptr<int32_t>();
  a.cs_left_default = cs_left_default.data_ptr<int32_t>();
  a.counts = counts.data_ptr<int32_t>();
  a.next_open = next_open.data_ptr<int32_t>();
  a.next_totals = next_totals.data_ptr<int64_t>();
  a.node_slot = node_slot.data_ptr<int32_t>();
  a.s2n = s2n.data_ptr<int32_t>();
  a.sub_dst = sub_dst.data_ptr<int32_t>();
  a.sub_par = sub_par.data_ptr<int32_t>();
  a.sub_sib = sub_sib.data_ptr<int32_t>();
  if (dev.is_cuda()) {
    c10::hip::HIPGuard guard(dev.index());
    fdx::launch_level_plan(a, stream(dev));
    C10_HIP_KERNEL_LAUNCH_CHECK();
  } else {
    fdx::level_plan_cpu(a);
  }
}

// Partition of the device level loop: default pass over the rows, then the column pass of the
// (device-counted, counts[0]) column splits, wps blocks per split.
void partition_cols(const Tensor& row_node, const Tensor& default_child, const Tensor& cs_feat,
                    const Tensor& cs_default, const Tensor& cs_other, const Tensor& cs_bin,
                    const Tensor& cs_left_default, const Tensor& counts, const Tensor& colptr, const Tensor& csc_row,
                    const Tensor& csc_bin, const optional<Tensor>& node_dense, const optional<Tensor>& dense,
                    int64_t max_splits, int64_t wps, const optional<Tensor>& pack_slot,
                    const optional<Tensor>& pack_dig, const optional<Tensor>& pack) {
  const auto dev = row_node.device();
  chk(row_node, dev, at::kInt, "row_node");
  chk(default_child, dev, at::kInt, "default_child");
  for (const Tensor* t : {&cs_feat, &cs_default, &cs_other, &cs_bin, &cs_left_default, &counts})
    chk(*t, dev, at::kInt, "column split arrays");
  chk(colptr, dev, at::kLong, "colptr");
  chk(csc_row, dev, at::kInt, "csc_row");
  chk(csc_bin, dev, at::kByte, "csc_bin");
  FDX_CHECK(cs_feat.numel() >= max_splits && wps >= 1, "cs arrays hold max_splits entries");
  FDX_CHECK(reinterpret_cast<uintptr_t>(row_node.data_ptr()) % 16 == 0, "row_node must be 16-byte aligned");
  fdx::PartitionArgs a{};
  a.row_node = row_node.data_ptr<int32_t>();
  a.default_child = default_child.data_ptr<int32_t>();
  a.num_nodes = (int32_t)default_child.numel();
  a.N = row_node.numel();
  a.split_default = cs_default.data_ptr<int32_t>();
  a.split_other = cs_other.data_ptr<int32_t>();
  a.split_bin = cs_bin.data_ptr<int32_t>();
  a.split_left_is_default = cs_left_default.data_ptr<int32_t>();
  a.csc_row = csc_row.data_ptr<int32_t>();
  a.csc_bin = csc_bin.data_ptr<uint8_t>();
  if (node_dense) {
    FDX_CHECK(dense.has_value(), "node_dense needs the dense bin block");
    chk(*node_dense, dev, at::kInt, "node_dense");
    chk(*dense, dev, at::kByte, "dense");
    FDX_CHECK(node_dense->numel() == 4ll * a.num_nodes, "node_dense must be [num_nodes, 4]");
    FDX_CHECK(dense->dim() == 2 && dense->size(1) >= a.N, "dense must be [Fh, n_pad >= N]");
    a.node_dense = node_dense->data_ptr<int32_t>();
    a.dense = dense->data_ptr<uint8_t>();
    a.n_pad = dense->size(1);
  }
  FDX_CHECK(pack_slot.has_value() == pack.has_value() && pack_dig.has_value() == pack.has_value(),
            "pack_slot, pack_dig and pack go together");
  if (pack) {
    chk(*pack_slot, dev, at::kInt, "pack_slot");
    chk(*pack_dig, dev, at::kInt, "pack_dig");
    chk(*pack, dev, at::kInt, "pack");
    FDX_CHECK(pack_slot->numel() == a.num_nodes && pack_dig->numel() == 2 * a.N && pack->numel() == a.N,
              "pack_slot [num_nodes], pack_dig [N, 2], pack [N]");
    FDX_CHECK(reinterpret_cast<uintptr_t>(pack_dig->data_ptr()) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(pack->data_ptr()) % 16 == 0, "pack_dig / pack must be 16-byte aligned");
    a.pack_slot = pack_slot->data_ptr<int32_t>();
    a.pack_dig = reinterpret_cast<const uint32_t*>(pack_dig->data_ptr<int32_t>());
    a.pack = reinterpret_cast<uint32_t*>(pack->data_ptr<int32_t>());
  }
  if (dev.is_cuda()) {
    c10::hip::HIPGuard guard(dev.index());
    fdx::launch_partition_cols(a, colptr.data_ptr<int64_t>(), cs_feat.data_ptr<int32_t>(), counts.data_ptr<int32_t>(),
                               (int32_t)max_splits, (int32_t)wps, stream(dev));
    C10_HIP_KERNEL_LAUNCH_CHECK();
  } else {
    fdx::partition_cols_cpu(a, colptr.data_ptr<int64_t>(), cs_feat.data_ptr<int32_t>(), counts.data_ptr<int32_t>());
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

// GBDT leaf values of every row of the device node table's sums (one launch per tree)
void leaf_values(const Tensor& stats, const Tensor& kexp, double eta, double lambda, double mds, const Tensor& out) {
  const auto dev = stats.device();
  chk(stats, dev, at::kLong, "stats");
  chk(kexp, dev, at::kInt, "kexp");
  chk(out, dev, at::kDouble, "out");
  FDX_CHECK(stats.dim() == 2 && stats.size(1) == 2 && kexp.numel() >= 2 && out.numel() == stats.size(0), "sizes");
  if (dev.is_cuda()) {
    c10::hip::HIPGuard guard(dev.index());
    fdx::launch_leaf_values(stats.data_ptr<int64_t>(), kexp.data_ptr<int32_t>(), stats.size(0), eta, lambda, mds,
                            out.data_ptr<double>(), stream(dev));
    C10_HIP_KERNEL_LAUNCH_CHECK();
  } else {
    fdx::leaf_values_cpu(stats.data_ptr<int64_t>(), kexp.data_ptr<int32_t>(), stats.size(0), eta, lambda, mds,
                         out.data_ptr<double>());
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
  namespace py = pybind11;
  m.def("tree_quant_max", &quant_max);
  m.def("tree_quant", &quant);
  m.def("tree_slot8", &slot8);
  m.def("tree_level_plan", &level_plan);
  m.def("tree_level_rows", &level_rows);
  m.def("tree_partition_cols", &partition_cols);
  m.def("tree_split_best", &split_best);
  m.def("tree_hist_build", &hist_build);
  m.def("tree_hist_sampled", &hist_sampled, py::arg("item_start"), py::arg("item_end"), py::arg("item_f0"),
        py::arg("item_meta"), py::arg("wave_item"), py::arg("csc_row"), py::arg("csc_key"), py::arg("rowpack"),
        py::arg("rowdig"), py::arg("boff"), py::arg("nbins"), py::arg("slot_node"), py::arg("hist"), py::arg("TB"),
        py::arg("bt"), py::arg("ct"), py::arg("feat_active"), py::arg("list"), py::arg("count"),
        py::arg("lds") = false, py::arg("listed_per_xcd") = -1);
  m.def("tree_hist_select", &hist_select);
  m.def("tree_hist_select_groups", &hist_select_groups);
  m.def("tree_slot_pack", &slot_pack);
  m.def("tree_rg_build", &rg_build);
  m.def("tree_rg_list", &rg_list, py::arg("row_node"), py::arg("node_slot"), py::arg("slot8"), py::arg("N"),
        py::arg("nslots"), py::arg("work"), py::arg("slot_start"), py::arg("list"), py::arg("rowdig"),
        py::arg("listdig"), py::arg("masked") = py::none(), py::arg("counted") = false);
  m.def("tree_rg_build_csr", &rg_build_csr, py::arg("indptr"), py::arg("idx"), py::arg("counts"), py::arg("remap"),
        py::arg("max_bin"), py::arg("fgroup"), py::arg("flocal"), py::arg("ptr"), py::arg("gbase"), py::arg("ent"),
        py::arg("work"), py::arg("erow") = py::none(), py::arg("em_g0") = 0, py::arg("ebase") = 0);
  m.def("tree_rg_hist", &rg_hist, py::arg("ptr"), py::arg("ent"), py::arg("gbase"), py::arg("gbin"),
        py::arg("rowdig"), py::arg("np"), py::arg("list"), py::arg("slot_start"), py::arg("listdig"),
        py::arg("nslots"), py::arg("gmode"), py::arg("wg"), py::arg("slot_node"), py::arg("hist"), py::arg("stride"),
        py::arg("shard_lo"), py::arg("shard_stride"), py::arg("dbg"), py::arg("erow") = py::none(),
        py::arg("ebase") = 0, py::arg("emdig") = py::none(), py::arg("em_min_rows") = 0,
        py::arg("part") = py::none(), py::arg("wg_first") = py::none());
  m.def("tree_rg_erow", &rg_erow);
  m.def("tree_rg_list_rows", [](int64_t N) { return (int64_t)fdx::rg_list_rows(N); });
  m.def("tree_rg_build_csr_waves", &fdx::rg_build_csr_waves);
  // (tests) rows above which the list kernels take 2048-row waves; returns the previous value
  m.def("tree_set_list_big_rows", [](int64_t n) {
    const int64_t old = fdx::g_rg_list_big_rows;
    fdx::g_rg_list_big_rows = n;
    return old;
  });
  m.def("tree_partition_counts_ok", &fdx::partition_counts_ok);
  m.def("tree_rf_sample", &rf_sample);
  m.def("tree_feature_mix", &feature_mix);
  m.def("tree_rf_compact", &rf_compact, py::arg("mask"), py::arg("nbins"), py::arg("fs"), py::arg("local"),
        py::arg("sizes"), py::arg("max_shard_features") = 0);
  m.def("tree_hist_dense", &hist_dense);
  m.def("tree_dense_fg", &dense_fg);
  m.def("tree_dense_waves", &dense_waves);
  m.def("tree_hist_subtract", &hist_subtract);
  m.def("tree_split_find", &split_find, py::arg("hist"), py::arg("totals"), py::arg("boff"), py::arg("nbins"),
        py::arg("zbin"), py::arg("fid_orig"), py::arg("node_ids"), py::arg("kexp"), py::arg("mode"),
        py::arg("lambda_"), py::arg("mcw"), py::arg("feat_thr"), py::arg("seed"), py::arg("tree"),
        py::arg("out_gain"), py::arg("out_bin"), py::arg("out_left"), py::arg("node_tree"),
        py::arg("wide") = py::none(), py::arg("row_of") = py::none());
  m.def("tree_partition", &partition);
  m.def("tree_logistic_grad", &logistic_grad);
  m.def("tree_leaf_update", &leaf_update);
  m.def("tree_leaf_values", &leaf_values);
}

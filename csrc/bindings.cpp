// pybind11 bindings of the native core. Every op dispatches on the device of its tensors:
// HIP tensors launch the gfx950 kernels on the current PyTorch HIP stream, CPU tensors run
// the host C++ implementation. Shapes are validated here, before any kernel launch.
#include <torch/extension.h>
#include <c10/hip/HIPGuard.h>
#include <c10/hip/HIPStream.h>

#include "scoring.h"
#include "ops.h"

namespace {

using at::Tensor;
using c10::optional;

#define FDX_CHECK(cond, msg) TORCH_CHECK(cond, "fdx: ", msg)

template <class T>
const T* cptr(const optional<Tensor>& t) {
  return (t && t->defined()) ? t->data_ptr<T>() : nullptr;
}
template <class T>
T* mptr(const optional<Tensor>& t) {
  return (t && t->defined()) ? t->data_ptr<T>() : nullptr;
}

void check_dev(const Tensor& t, const at::Device& dev, const char* name) {
  FDX_CHECK(t.device() == dev, std::string(name) + " must live on " + dev.str());
  FDX_CHECK(t.is_contiguous(), std::string(name) + " must be contiguous");
}

// Output buffer for a device kernel: either on the device, or page-locked host memory that the
// kernel writes through PCIe directly (zero-copy results, no D2H copy on the SDMA queue).
template <class T>
T* out_ptr(const Tensor& t, const at::Device& dev, const char* name) {
  FDX_CHECK(t.is_contiguous(), std::string(name) + " must be contiguous");
  if (t.device() == dev) return t.data_ptr<T>();
  FDX_CHECK(dev.is_cuda() && t.device().is_cpu() && t.is_pinned(),
            std::string(name) + " must be on " + dev.str() + " or pinned host memory");
  void* dptr = nullptr;
  FDX_CHECK(hipHostGetDevicePointer(&dptr, t.data_ptr(), 0) == hipSuccess, "hipHostGetDevicePointer failed");
  return static_cast<T*>(dptr);
}

fdx::StrTable make_table(const optional<std::vector<Tensor>>& tab, const at::Device& dev) {
  fdx::StrTable t{nullptr, nullptr, nullptr, nullptr, -1};
  if (!tab || tab->empty()) return t;
  FDX_CHECK(tab->size() == 4, "string table = (slots, hashes, offs, bytes)");
  const auto& v = *tab;
  for (const auto& x : v) check_dev(x, dev, "string table");
  FDX_CHECK(v[0].scalar_type() == at::kInt && v[1].scalar_type() == at::kInt &&
                v[2].scalar_type() == at::kLong && v[3].scalar_type() == at::kByte,
            "string table dtypes (int32, int32, int64, uint8)");
  const int64_t size = v[0].numel();
  FDX_CHECK(size > 0 && (size & (size - 1)) == 0, "table size must be a power of two");
  FDX_CHECK(v[2].numel() == v[1].numel() + 1, "offs must have n+1 entries");
  t.slots = v[0].data_ptr<int32_t>();
  t.hashes = reinterpret_cast<const uint32_t*>(v[1].data_ptr<int32_t>());
  t.offs = v[2].data_ptr<int64_t>();
  t.bytes = v[3].data_ptr<uint8_t>();
  t.mask = (int32_t)(size - 1);
  return t;
}

fdx::TreeEnsemble make_trees(const optional<std::vector<Tensor>>& tr, int64_t K, const at::Device& dev) {
  fdx::TreeEnsemble te{};
  if (!tr || tr->empty()) return te;
  FDX_CHECK(tr->size() == 7, "trees = (feat, thr, left, right, leaf, roots, weights)");
  const auto& v = *tr;
  for (const auto& x : v) check_dev(x, dev, "tree arrays");
  const int64_t nodes = v[0].numel();
  FDX_CHECK(v[1].numel() == nodes && v[2].numel() == nodes && v[3].numel() == nodes, "node arrays size");
  FDX_CHECK(v[4].numel() == nodes * K, "leaf array must be nodes*K");
  FDX_CHECK(v[5].numel() == v[6].numel(), "roots/weights size");
  FDX_CHECK(v[0].scalar_type() == at::kInt && v[1].scalar_type() == at::kDouble &&
                v[2].scalar_type() == at::kInt && v[3].scalar_type() == at::kInt &&
                v[4].scalar_type() == at::kDouble && v[5].scalar_type() == at::kInt &&
                v[6].scalar_type() == at::kDouble,
            "tree dtypes");
  te.feat = v[0].data_ptr<int32_t>();
  te.thr = v[1].data_ptr<double>();
  te.left = v[2].data_ptr<int32_t>();
  te.right = v[3].data_ptr<int32_t>();
  te.leaf = v[4].data_ptr<double>();
  te.roots = v[5].data_ptr<int32_t>();
  te.weights = v[6].data_ptr<double>();
  te.num_trees = (int32_t)v[5].numel();
  te.K = (int32_t)K;
  return te;
}

// CountVectorizer fit (K-05): per kept token a 64-bit key (murmur3 seed 42 << 32 | murmur3 seed 2)
// after clean / tokenize / stop-word removal. Without key_off/out_keys only the per-document token
// counts are written (pass 1); with them the keys land at key_off[d] + i (pass 2).
void token_keys(const Tensor& text, const Tensor& doc_off, int64_t flags, const optional<std::vector<Tensor>>& stop,
                const Tensor& out_ntok, const Tensor& out_status, const optional<Tensor>& key_off,
                const optional<Tensor>& out_keys, const optional<Tensor>& only_docs, int64_t threads) {
  const auto dev = text.device();
  check_dev(text, dev, "text");
  check_dev(doc_off, dev, "doc_off");
  check_dev(out_ntok, dev, "out_ntok");
  check_dev(out_status, dev, "out_status");
  FDX_CHECK(text.scalar_type() == at::kByte && doc_off.scalar_type() == at::kLong, "text u8 / doc_off i64");
  const int64_t D = doc_off.numel() - 1;
  FDX_CHECK(out_ntok.scalar_type() == at::kInt && out_status.scalar_type() == at::kInt && out_ntok.numel() >= D &&
                out_status.numel() >= D, "out_ntok/out_status int32 [D]");
  FDX_CHECK(key_off.has_value() == out_keys.has_value(), "key_off and out_keys go together");
  if (out_keys) {
    check_dev(*key_off, dev, "key_off");
    check_dev(*out_keys, dev, "out_keys");
    FDX_CHECK(key_off->scalar_type() == at::kLong && key_off->numel() >= D + 1, "key_off int64 [D+1]");
    FDX_CHECK(out_keys->scalar_type() == at::kLong, "out_keys int64");
  }
  fdx::FeatArgs a{};
  a.text = text.data_ptr<uint8_t>();
  a.doc_off = doc_off.data_ptr<int64_t>();
  a.num_docs = (int32_t)D;
  a.flags = (int32_t)((flags & (fdx::kFlagClean | fdx::kFlagPreLowered | fdx::kFlagStopwords)) | fdx::kFlagKeys);
  a.num_features = 1;
  a.stop = make_table(stop, dev);
  a.out_ntok = out_ntok.data_ptr<int32_t>();
  a.out_status = out_status.data_ptr<int32_t>();
  a.key_off = out_keys ? key_off->data_ptr<int64_t>() : nullptr;
  a.out_keys = out_keys ? reinterpret_cast<uint64_t*>(out_keys->data_ptr<int64_t>()) : nullptr;
  if (dev.is_cuda()) {
    FDX_CHECK(!only_docs, "only_docs is a host-path option");
    c10::hip::HIPGuard guard(dev.index());
    fdx::launch_featurize_score(a, c10::hip::getCurrentHIPStream(dev.index()).stream());
    C10_HIP_KERNEL_LAUNCH_CHECK();
  } else {
    const int32_t* only = nullptr;
    int32_t n_only = 0;
    if (only_docs) {
      FDX_CHECK(only_docs->scalar_type() == at::kInt && only_docs->is_contiguous(), "only_docs int32");
      only = only_docs->data_ptr<int32_t>();
      n_only = (int32_t)only_docs->numel();
    }
    fdx::featurize_score_cpu(a, only, n_only, (int)threads);
  }
}

void featurize_score(const Tensor& text, const Tensor& doc_off, int64_t flags, int64_t num_features,
                     const optional<std::vector<Tensor>>& stop, const optional<std::vector<Tensor>>& vocab,
                     double min_tf, const optional<Tensor>& idf, const optional<Tensor>& lr_w, double lr_b,
                     const optional<std::vector<Tensor>>& trees, int64_t K, const Tensor& out_idx,
                     const Tensor& out_val, const Tensor& out_nnz, const optional<Tensor>& out_ntok,
                     const Tensor& out_raw, const Tensor& out_status, const optional<Tensor>& only_docs,
                     int64_t threads, const optional<Tensor>& long_docs) {
  const auto dev = text.device();
  check_dev(text, dev, "text");
  check_dev(doc_off, dev, "doc_off");
  FDX_CHECK(text.scalar_type() == at::kByte && doc_off.scalar_type() == at::kLong, "text u8 / doc_off i64");
  const int64_t D = doc_off.numel() - 1;
  FDX_CHECK(D >= 0, "doc_off needs at least one entry");
  for (const Tensor* t : {&out_idx, &out_val, &out_nnz}) check_dev(*t, dev, "outputs");
  FDX_CHECK(out_nnz.numel() >= D && out_status.numel() >= D, "per-doc outputs too small");
  FDX_CHECK(out_idx.numel() >= fdx::csr_capacity(text.numel(), D) || !(flags & fdx::kFlagWriteCsr),
            "CSR scratch too small");
  FDX_CHECK(out_idx.numel() == out_val.numel(), "CSR idx/val size mismatch");
  FDX_CHECK(num_features > 0 || (flags & fdx::kFlagVocab), "num_features must be positive");
  if (flags & fdx::kFlagIdf) FDX_CHECK(idf && idf->numel() >= num_features && idf->scalar_type() == at::kDouble, "idf");
  if (flags & fdx::kFlagLR) FDX_CHECK(lr_w && lr_w->numel() >= num_features && lr_w->scalar_type() == at::kDouble, "lr_w");
  if (flags & fdx::kFlagTrees) FDX_CHECK(trees && K >= 1 && K <= 2, "trees");
  FDX_CHECK(out_raw.numel() >= D * ((flags & fdx::kFlagTrees) ? K : 1), "out_raw too small");
  if (idf) check_dev(*idf, dev, "idf");
  if (lr_w) check_dev(*lr_w, dev, "lr_w");
  if (out_ntok) check_dev(*out_ntok, dev, "out_ntok");

  fdx::FeatArgs a{};
  a.text = text.data_ptr<uint8_t>();
  a.doc_off = doc_off.data_ptr<int64_t>();
  a.num_docs = (int32_t)D;
  a.flags = (int32_t)flags;
  a.num_features = (int32_t)num_features;
  a.stop = make_table(stop, dev);
  a.vocab = make_table(vocab, dev);
  a.min_tf = min_tf;
  a.idf = cptr<double>(idf);
  a.lr_w = cptr<double>(lr_w);
  a.lr_b = lr_b;
  a.trees = make_trees(trees, K, dev);
  a.out_idx = out_idx.data_ptr<int32_t>();
  a.out_val = out_val.data_ptr<float>();
  a.out_nnz = out_nnz.data_ptr<int32_t>();
  a.out_ntok = mptr<int32_t>(out_ntok);
  FDX_CHECK(out_raw.scalar_type() == at::kDouble && out_status.scalar_type() == at::kInt, "out_raw f64 / status i32");
  a.out_raw = out_ptr<double>(out_raw, dev, "out_raw");
  a.out_status = out_ptr<int32_t>(out_status, dev, "out_status");
  if (dev.is_cuda()) {
    FDX_CHECK(!only_docs, "only_docs is a host-path option");
    if (long_docs) {      // second launch: the long-dialogue kernel on the listed documents only
      check_dev(*long_docs, dev, "long_docs");
      FDX_CHECK(long_docs->scalar_type() == at::kInt && long_docs->is_contiguous(), "long_docs int32");
      a.doc_list = long_docs->data_ptr<int32_t>();
      a.n_list = (int32_t)long_docs->numel();
    }
    c10::hip::HIPGuard guard(dev.index());
    fdx::launch_featurize_score(a, c10::hip::getCurrentHIPStream(dev.index()).stream());
    C10_HIP_KERNEL_LAUNCH_CHECK();
  } else {
    const int32_t* only = nullptr;
    int32_t n_only = 0;
    if (only_docs) {
      FDX_CHECK(only_docs->scalar_type() == at::kInt && only_docs->is_contiguous(), "only_docs int32");
      only = only_docs->data_ptr<int32_t>();
      n_only = (int32_t)only_docs->numel();
    }
    fdx::featurize_score_cpu(a, only, n_only, (int)threads);
  }
}

hipStream_t stream_of(const at::Device& dev) {
  return c10::hip::getCurrentHIPStream(dev.index()).stream();
}

void check_csr(const Tensor& indptr, const Tensor& idx, const Tensor& val, const at::Device& dev) {
  check_dev(indptr, dev, "indptr");
  check_dev(idx, dev, "indices");
  check_dev(val, dev, "values");
  FDX_CHECK(indptr.scalar_type() == at::kLong && idx.scalar_type() == at::kInt, "indptr i64 / indices i32");
  FDX_CHECK(val.scalar_type() == at::kFloat || val.scalar_type() == at::kDouble, "values f32|f64");
  FDX_CHECK(idx.numel() == val.numel(), "indices/values size mismatch");
  FDX_CHECK(indptr.numel() >= 1, "indptr needs rows+1 entries");
}

template <class V>
void score_csr_t(const Tensor& indptr, const Tensor& idx, const Tensor& val, const optional<Tensor>& lr_w, double lr_b,
                 const optional<std::vector<Tensor>>& trees, int64_t K, bool cmp_less, const Tensor& out,
                 int64_t threads) {
  const auto dev = indptr.device();
  fdx::CsrArgs<V> a{};
  a.indptr = indptr.data_ptr<int64_t>();
  a.idx = idx.data_ptr<int32_t>();
  a.val = val.data_ptr<V>();
  a.rows = indptr.numel() - 1;
  a.lr_w = cptr<double>(lr_w);
  a.lr_b = lr_b;
  a.trees = make_trees(trees, K, dev);
  a.cmp_less = cmp_less;
  a.out = out.data_ptr<double>();
  if (dev.is_cuda()) {
    c10::hip::HIPGuard guard(dev.index());
    fdx::launch_score_csr<V>(a, stream_of(dev));
    C10_HIP_KERNEL_LAUNCH_CHECK();
  } else {
    fdx::score_csr_cpu<V>(a, (int)threads);
  }
}

void score_csr(const Tensor& indptr, const Tensor& idx, const Tensor& val, const optional<Tensor>& lr_w, double lr_b,
               const optional<std::vector<Tensor>>& trees, int64_t K, bool cmp_less, const Tensor& out,
               int64_t threads) {
  const auto dev = indptr.device();
  check_csr(indptr, idx, val, dev);
  check_dev(out, dev, "out");
  FDX_CHECK(out.scalar_type() == at::kDouble, "out must be float64");
  const int64_t rows = indptr.numel() - 1;
  FDX_CHECK(lr_w.has_value() != (trees.has_value() && !trees->empty()), "exactly one scorer (lr_w or trees)");
  if (lr_w) {
    check_dev(*lr_w, dev, "lr_w");
    FDX_CHECK(lr_w->scalar_type() == at::kDouble, "lr_w must be float64");
    FDX_CHECK(out.numel() >= rows, "out too small");
  } else {
    FDX_CHECK(K >= 1 && K <= 2 && out.numel() >= rows * K, "out too small for K");
  }
  if (val.scalar_type() == at::kFloat)
    score_csr_t<float>(indptr, idx, val, lr_w, lr_b, trees, K, cmp_less, out, threads);
  else
    score_csr_t<double>(indptr, idx, val, lr_w, lr_b, trees, K, cmp_less, out, threads);
}

void spmv(const Tensor& indptr, const Tensor& idx, const Tensor& val, const Tensor& x, const Tensor& y,
          int64_t threads) {
  const auto dev = indptr.device();
  check_csr(indptr, idx, val, dev);
  check_dev(x, dev, "x");
  check_dev(y, dev, "y");
  FDX_CHECK(x.scalar_type() == at::kDouble && y.scalar_type() == at::kDouble, "x/y float64");
  const int64_t rows = indptr.numel() - 1;
  FDX_CHECK(y.numel() >= rows, "y too small");
  auto run = [&](auto* vp) {
    using V = std::remove_const_t<std::remove_pointer_t<decltype(vp)>>;
    if (dev.is_cuda()) {
      c10::hip::HIPGuard guard(dev.index());
      fdx::launch_spmv<V>(indptr.data_ptr<int64_t>(), idx.data_ptr<int32_t>(), val.data_ptr<V>(),
                          x.data_ptr<double>(), y.data_ptr<double>(), rows, stream_of(dev));
      C10_HIP_KERNEL_LAUNCH_CHECK();
    } else {
      fdx::spmv_cpu<V>(indptr.data_ptr<int64_t>(), idx.data_ptr<int32_t>(), val.data_ptr<V>(),
                       x.data_ptr<double>(), y.data_ptr<double>(), rows, (int)threads);
    }
  };
  if (val.scalar_type() == at::kFloat) run((float*)nullptr); else run((double*)nullptr);
}

void spmv_t(const Tensor& indptr, const Tensor& idx, const Tensor& val, const Tensor& r, const Tensor& g,
            int64_t threads) {
  const auto dev = indptr.device();
  check_csr(indptr, idx, val, dev);
  check_dev(r, dev, "r");
  check_dev(g, dev, "g");
  FDX_CHECK(r.scalar_type() == at::kDouble && g.scalar_type() == at::kDouble, "r/g float64");
  const int64_t rows = indptr.numel() - 1;
  FDX_CHECK(r.numel() >= rows, "r too small");
  auto run = [&](auto* vp) {
    using V = std::remove_const_t<std::remove_pointer_t<decltype(vp)>>;
    if (dev.is_cuda()) {
      c10::hip::HIPGuard guard(dev.index());
      fdx::launch_spmv_t<V>(indptr.data_ptr<int64_t>(), idx.data_ptr<int32_t>(), val.data_ptr<V>(),
                            r.data_ptr<double>(), g.data_ptr<double>(), rows, stream_of(dev));
      C10_HIP_KERNEL_LAUNCH_CHECK();
    } else {
      fdx::spmv_t_cpu<V>(indptr.data_ptr<int64_t>(), idx.data_ptr<int32_t>(), val.data_ptr<V>(),
                         r.data_ptr<double>(), g.data_ptr<double>(), rows, g.numel(), (int)threads);
    }
  };
  if (val.scalar_type() == at::kFloat) run((float*)nullptr); else run((double*)nullptr);
}

void doc_freq(const Tensor& idx, const Tensor& val, const Tensor& df) {
  const auto dev = idx.device();
  check_dev(idx, dev, "indices");
  check_dev(val, dev, "values");
  check_dev(df, dev, "df");
  FDX_CHECK(dev.is_cuda(), "doc_freq is a device kernel (host path uses torch.bincount)");
  FDX_CHECK(idx.scalar_type() == at::kInt && df.scalar_type() == at::kLong, "indices i32 / df i64");
  c10::hip::HIPGuard guard(dev.index());
  if (val.scalar_type() == at::kFloat)
    fdx::launch_doc_freq<float>(idx.data_ptr<int32_t>(), val.data_ptr<float>(), idx.numel(), df.data_ptr<int64_t>(), stream_of(dev));
  else
    fdx::launch_doc_freq<double>(idx.data_ptr<int32_t>(), val.data_ptr<double>(), idx.numel(), df.data_ptr<int64_t>(), stream_of(dev));
  C10_HIP_KERNEL_LAUNCH_CHECK();
}

// Feature-major order of a count CSR (see sort_kernels.hip). csc_row/csc_cnt may be views into
// larger (padded) buffers; they must hold nnz entries.
template <class V>
void feature_order_t(const Tensor& indptr, const Tensor& idx, const Tensor& counts, int64_t F, const Tensor& csc_row,
                     const Tensor& csc_cnt, const Tensor& colptr, const Tensor& df, const Tensor& maxc) {
  const auto dev = idx.device();
  for (const Tensor* t : {&indptr, &counts, &csc_row, &csc_cnt, &colptr, &df, &maxc}) check_dev(*t, dev, "feature_order");
  FDX_CHECK(indptr.scalar_type() == at::kLong && idx.scalar_type() == at::kInt, "indptr i64 / idx i32");
  FDX_CHECK(csc_row.scalar_type() == at::kInt && csc_cnt.scalar_type() == at::kByte, "csc_row i32 / csc_cnt u8");
  FDX_CHECK(colptr.scalar_type() == at::kLong && df.scalar_type() == at::kLong && maxc.scalar_type() == at::kInt,
            "colptr/df i64, maxc i32");
  const int64_t nnz = idx.numel();
  FDX_CHECK(counts.numel() == nnz && csc_row.numel() >= nnz && csc_cnt.numel() >= nnz, "entry arrays");
  FDX_CHECK(colptr.numel() == F + 1 && df.numel() == F && maxc.numel() == F && F > 0 && F < (1ll << 31), "F");
  fdx::FeatureOrderArgs<V> a{};
  a.indptr = indptr.data_ptr<int64_t>();
  a.idx = idx.data_ptr<int32_t>();
  a.counts = counts.data_ptr<V>();
  a.rows = indptr.numel() - 1;
  a.nnz = nnz;
  a.F = (int32_t)F;
  a.csc_row = csc_row.data_ptr<int32_t>();
  a.csc_cnt = csc_cnt.data_ptr<uint8_t>();
  a.colptr = colptr.data_ptr<int64_t>();
  a.df = df.data_ptr<int64_t>();
  a.maxc = maxc.data_ptr<int32_t>();
  if (dev.is_cuda()) {
    c10::hip::HIPGuard guard(dev.index());
    const auto o32 = idx.options();
    const auto o64 = indptr.options();
    Tensor keys_tmp = at::empty({std::max<int64_t>(nnz, 1)}, o32), keys_sorted = at::empty({std::max<int64_t>(nnz, 1)}, o32);
    Tensor pay_tmp = at::empty({std::max<int64_t>(nnz, 1)}, o64), pay_sorted = at::empty({std::max<int64_t>(nnz, 1)}, o64);
    const size_t tb = fdx::feature_order_temp_bytes(nnz, (int32_t)F);
    Tensor temp = at::empty({(int64_t)std::max<size_t>(tb, 1)}, idx.options().dtype(at::kByte));
    a.keys_tmp = keys_tmp.data_ptr<int32_t>();
    a.keys_sorted = keys_sorted.data_ptr<int32_t>();
    a.payload_tmp = reinterpret_cast<uint64_t*>(pay_tmp.data_ptr<int64_t>());
    a.payload_sorted = reinterpret_cast<uint64_t*>(pay_sorted.data_ptr<int64_t>());
    a.temp = temp.data_ptr();
    a.temp_bytes = tb;
    fdx::launch_feature_order<V>(a, c10::hip::getCurrentHIPStream(dev.index()).stream());
    C10_HIP_KERNEL_LAUNCH_CHECK();
  } else {
    fdx::feature_order_cpu<V>(a);
  }
}

void feature_order(const Tensor& indptr, const Tensor& idx, const Tensor& counts, int64_t F, const Tensor& csc_row,
                   const Tensor& csc_cnt, const Tensor& colptr, const Tensor& df, const Tensor& maxc) {
  FDX_CHECK(indptr.is_contiguous() && idx.is_contiguous() && counts.is_contiguous(), "contiguous inputs");
  if (counts.scalar_type() == at::kFloat) feature_order_t<float>(indptr, idx, counts, F, csc_row, csc_cnt, colptr, df, maxc);
  else if (counts.scalar_type() == at::kDouble) feature_order_t<double>(indptr, idx, counts, F, csc_row, csc_cnt, colptr, df, maxc);
  else if (counts.scalar_type() == at::kInt) feature_order_t<int32_t>(indptr, idx, counts, F, csc_row, csc_cnt, colptr, df, maxc);
  else FDX_CHECK(false, "counts must be int32, float32 or float64");
}

// out = min(in, maxv) over uint8 (bin clamp of the count path); in/out 16-byte aligned on the device
void clamp_u8(const Tensor& in, int64_t maxv, const Tensor& out) {
  const auto dev = in.device();
  check_dev(out, dev, "clamp_u8");
  FDX_CHECK(in.scalar_type() == at::kByte && out.scalar_type() == at::kByte && out.numel() >= in.numel() &&
                in.is_contiguous() && out.is_contiguous() && maxv >= 0 && maxv <= 255, "clamp_u8 args");
  if (dev.is_cuda()) {
    FDX_CHECK(reinterpret_cast<uintptr_t>(in.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(out.data_ptr()) % 16 == 0,
              "clamp_u8: 16-byte aligned buffers");
    c10::hip::HIPGuard guard(dev.index());
    fdx::launch_clamp_u8(in.data_ptr<uint8_t>(), in.numel(), (uint8_t)maxv, out.data_ptr<uint8_t>(),
                         c10::hip::getCurrentHIPStream(dev.index()).stream());
    C10_HIP_KERNEL_LAUNCH_CHECK();
  } else {
    const uint8_t* a = in.data_ptr<uint8_t>();
    uint8_t* b = out.data_ptr<uint8_t>();
    for (int64_t i = 0; i < in.numel(); ++i) b[i] = a[i] > maxv ? (uint8_t)maxv : a[i];
  }
}

// Row-block segment bounds of sorted-row columns (XCD-aware histogram items).
// dst[seg_dst[i] + k] = src[seg_src[i] + k] for k < seg_len[i]; keys get + seg_add[i] (uint8, optional)
void copy_segments(const Tensor& src_row, const Tensor& src_key, const Tensor& seg_src, const Tensor& seg_dst,
                   const Tensor& seg_len, const Tensor& dst_row, const Tensor& dst_key, const optional<Tensor>& seg_add) {
  const auto dev = src_row.device();
  for (const Tensor* t : {&src_key, &seg_src, &seg_dst, &seg_len, &dst_row, &dst_key}) check_dev(*t, dev, "copy_segments");
  TORCH_CHECK(src_row.scalar_type() == at::kInt && dst_row.scalar_type() == at::kInt && src_key.scalar_type() == at::kByte &&
                  dst_key.scalar_type() == at::kByte && seg_src.scalar_type() == at::kLong &&
                  seg_dst.scalar_type() == at::kLong && seg_len.scalar_type() == at::kLong,
              "copy_segments dtypes");
  TORCH_CHECK(src_row.numel() == src_key.numel() && dst_row.numel() == dst_key.numel() &&
                  seg_src.numel() == seg_dst.numel() && seg_src.numel() == seg_len.numel(),
              "copy_segments sizes");
  const int64_t n = seg_src.numel();
  const uint8_t* add = nullptr;
  if (seg_add) {
    check_dev(*seg_add, dev, "copy_segments");
    TORCH_CHECK(seg_add->scalar_type() == at::kByte && seg_add->numel() == n && seg_add->is_contiguous(),
                "seg_add must be [nseg] uint8");
    add = seg_add->data_ptr<uint8_t>();
  }
  if (dev.is_cuda()) {
    c10::hip::HIPGuard guard(dev.index());
    fdx::launch_copy_segments(src_row.data_ptr<int32_t>(), src_key.data_ptr<uint8_t>(), seg_src.data_ptr<int64_t>(),
                              seg_dst.data_ptr<int64_t>(), seg_len.data_ptr<int64_t>(), n, add, dst_row.data_ptr<int32_t>(),
                              dst_key.data_ptr<uint8_t>(), c10::hip::getCurrentHIPStream(dev.index()).stream());
    C10_HIP_KERNEL_LAUNCH_CHECK();
  } else {
    fdx::copy_segments_cpu(src_row.data_ptr<int32_t>(), src_key.data_ptr<uint8_t>(), seg_src.data_ptr<int64_t>(),
                           seg_dst.data_ptr<int64_t>(), seg_len.data_ptr<int64_t>(), n, add, dst_row.data_ptr<int32_t>(),
                           dst_key.data_ptr<uint8_t>());
  }
}

// The hot features' dense block: dense [nseg, n_pad] uint8 (pre-filled with the zero bins) gets
// row seg_src[i].. of the CSC (row, bin) of segment i scattered into its row i.
void dense_scatter(const Tensor& csc_row, const Tensor& csc_bin, const Tensor& seg_src, const Tensor& seg_len,
                   const Tensor& dense, int64_t max_len) {
  const auto dev = csc_row.device();
  for (const Tensor* t : {&csc_bin, &seg_src, &seg_len, &dense}) check_dev(*t, dev, "dense_scatter");
  TORCH_CHECK(csc_row.scalar_type() == at::kInt && csc_bin.scalar_type() == at::kByte && seg_src.scalar_type() == at::kLong &&
                  seg_len.scalar_type() == at::kLong && dense.scalar_type() == at::kByte && dense.dim() == 2 &&
                  dense.is_contiguous() && seg_src.numel() == dense.size(0) && seg_len.numel() == dense.size(0),
              "dense_scatter: int32 rows, uint8 bins, int64 [nseg] segments, uint8 dense [nseg, n_pad]");
  const int64_t nseg = dense.size(0), n_pad = dense.size(1);
  if (dev.is_cuda()) {
    c10::hip::HIPGuard guard(dev.index());
    fdx::launch_dense_scatter(csc_row.data_ptr<int32_t>(), csc_bin.data_ptr<uint8_t>(), seg_src.data_ptr<int64_t>(),
                              seg_len.data_ptr<int64_t>(), nseg, max_len, n_pad, dense.data_ptr<uint8_t>(),
                              c10::hip::getCurrentHIPStream(dev.index()).stream());
    C10_HIP_KERNEL_LAUNCH_CHECK();
  } else {
    fdx::dense_scatter_cpu(csc_row.data_ptr<int32_t>(), csc_bin.data_ptr<uint8_t>(), seg_src.data_ptr<int64_t>(),
                           seg_len.data_ptr<int64_t>(), nseg, n_pad, dense.data_ptr<uint8_t>());
  }
}

// Greedy packing of histogram work items (models/quantize.py _finish_items): runs of consecutive
// packable features, each run at most `pack_keys` keys at the run's largest stride and at most
// `max_entries` entries. Returns [runs, 3] int64 (first, end, log2 stride). Host-only.
Tensor pack_runs(const Tensor& packable, const Tensor& stride, const Tensor& ncol, int64_t pack_keys,
                 int64_t max_entries) {
  TORCH_CHECK(!packable.is_cuda() && packable.scalar_type() == at::kByte && stride.scalar_type() == at::kLong &&
                  ncol.scalar_type() == at::kLong && packable.numel() == stride.numel() &&
                  stride.numel() == ncol.numel(),
              "pack_runs: host uint8 packable, int64 stride/ncol of equal length");
  const auto pk = packable.contiguous();
  const auto st = stride.contiguous();
  const auto nc = ncol.contiguous();
  const uint8_t* p = pk.data_ptr<uint8_t>();
  const int64_t* s = st.data_ptr<int64_t>();
  const int64_t* c = nc.data_ptr<int64_t>();
  const int64_t S = pk.numel();
  std::vector<int64_t> out;
  int64_t i = 0;
  while (i < S) {
    if (!p[i]) { ++i; continue; }
    const int64_t i0 = i;
    int64_t st_max = s[i], ent = 0, k = 0;
    while (i < S && p[i]) {
      const int64_t s2 = std::max(st_max, s[i]);
      if ((k + 1) * s2 > pack_keys || ent + c[i] > max_entries) break;
      st_max = s2;
      ent += c[i];
      ++k;
      ++i;
    }
    if (k == 0) { ++i; continue; }   // a single feature over the limits: not packed (caller treats it as single)
    int64_t l2 = 0;
    while ((int64_t(1) << l2) < st_max) ++l2;
    out.insert(out.end(), {i0, i0 + k, l2});
  }
  auto res = torch::empty({(int64_t)out.size() / 3, 3}, torch::kLong);
  std::copy(out.begin(), out.end(), res.data_ptr<int64_t>());
  return res;
}

void block_bounds(const Tensor& csc_row, const Tensor& colptr, const Tensor& cols, int64_t nblk, int64_t row_block,
                  const Tensor& bounds) {
  const auto dev = csc_row.device();
  for (const Tensor* t : {&colptr, &cols, &bounds}) check_dev(*t, dev, "block_bounds");
  FDX_CHECK(csc_row.scalar_type() == at::kInt && colptr.scalar_type() == at::kLong && cols.scalar_type() == at::kInt &&
                bounds.scalar_type() == at::kLong, "dtypes");
  FDX_CHECK(bounds.numel() == cols.numel() * (nblk + 1) && row_block > 0, "bounds [ncols, nblk+1]");
  if (dev.is_cuda()) {
    c10::hip::HIPGuard guard(dev.index());
    fdx::launch_block_bounds(csc_row.data_ptr<int32_t>(), colptr.data_ptr<int64_t>(), cols.data_ptr<int32_t>(),
                             (int32_t)cols.numel(), (int32_t)nblk, row_block, bounds.data_ptr<int64_t>(),
                             c10::hip::getCurrentHIPStream(dev.index()).stream());
    C10_HIP_KERNEL_LAUNCH_CHECK();
  } else {
    fdx::block_bounds_cpu(csc_row.data_ptr<int32_t>(), colptr.data_ptr<int64_t>(), cols.data_ptr<int32_t>(),
                          (int32_t)cols.numel(), (int32_t)nblk, row_block, bounds.data_ptr<int64_t>());
  }
}

// Python-json.dumps-identical output records of the streaming classifier (see json_encode.cpp).
// Returns the total size, or -(needed size) when `out` is too small.
int64_t encode_records(const Tensor& pred, const Tensor& conf, const Tensor& text, const Tensor& off,
                       const optional<Tensor>& skip, const Tensor& out, const Tensor& out_off, const Tensor& status,
                       int64_t threads) {
  for (const Tensor* t : {&pred, &conf, &text, &off, &out, &out_off, &status})
    FDX_CHECK(t->device().is_cpu() && t->is_contiguous(), "encode_records: contiguous host tensors");
  const int64_t n = pred.numel();
  FDX_CHECK(pred.scalar_type() == at::kDouble && conf.scalar_type() == at::kDouble && conf.numel() == n, "pred/conf f64 [n]");
  FDX_CHECK(text.scalar_type() == at::kByte && off.scalar_type() == at::kLong && off.numel() >= n + 1, "text u8 / off i64 [n+1]");
  FDX_CHECK(out.scalar_type() == at::kByte && out_off.scalar_type() == at::kLong && out_off.numel() >= n + 1, "out u8 / out_off i64");
  FDX_CHECK(status.scalar_type() == at::kInt && status.numel() >= n, "status i32 [n]");
  if (skip) FDX_CHECK(skip->scalar_type() == at::kInt && skip->numel() >= n && skip->is_contiguous(), "skip i32 [n]");
  pybind11::gil_scoped_release nogil;   // partition reader / output threads run this concurrently
  return fdx::encode_records(pred.data_ptr<double>(), conf.data_ptr<double>(), text.data_ptr<uint8_t>(),
                             off.data_ptr<int64_t>(), skip ? skip->data_ptr<int32_t>() : nullptr, n,
                             out.data_ptr<uint8_t>(), out.numel(), out_off.data_ptr<int64_t>(),
                             status.data_ptr<int32_t>(), (int)threads);
}

int64_t extract_json_field(const Tensor& in, const Tensor& in_off, const std::string& field, const Tensor& out,
                           const Tensor& out_off, const Tensor& status, int64_t threads) {
  for (const Tensor* t : {&in, &in_off, &out, &out_off, &status})
    FDX_CHECK(!t->is_cuda() && t->is_contiguous(), "json extraction runs on host tensors");
  FDX_CHECK(in.scalar_type() == at::kByte && out.scalar_type() == at::kByte && in_off.scalar_type() == at::kLong &&
                out_off.scalar_type() == at::kLong && status.scalar_type() == at::kInt,
            "dtypes u8/i64/u8/i64/i32");
  const int64_t n = in_off.numel() - 1;
  FDX_CHECK(n >= 0 && out_off.numel() >= n + 1 && status.numel() >= n, "offset/status sizes");
  pybind11::gil_scoped_release nogil;
  return fdx::extract_json_field(in.data_ptr<uint8_t>(), in_off.data_ptr<int64_t>(), n,
                                 reinterpret_cast<const uint8_t*>(field.data()), (int64_t)field.size(),
                                 out.data_ptr<uint8_t>(), out.numel(), out_off.data_ptr<int64_t>(),
                                 status.data_ptr<int32_t>(), (int)threads);
}

// extract_json_field over a list of separate values (bytes / None) without packing
// them into one buffer first: the buffers are located with the GIL held, read without it.
int64_t extract_json_field_refs(pybind11::list values, int64_t count, const std::string& field, const Tensor& out,
                                const Tensor& out_off, const Tensor& status, int64_t threads) {
  for (const Tensor* t : {&out, &out_off, &status})
    FDX_CHECK(!t->is_cuda() && t->is_contiguous(), "json extraction runs on host tensors");
  FDX_CHECK(out.scalar_type() == at::kByte && out_off.scalar_type() == at::kLong && status.scalar_type() == at::kInt,
            "dtypes u8/i64/i32");
  const int64_t n = count;
  FDX_CHECK(n >= 0 && n <= (int64_t)PyList_GET_SIZE(values.ptr()), "count exceeds the list");
  FDX_CHECK(out_off.numel() >= n + 1 && status.numel() >= n, "offset/status sizes");
  std::vector<const uint8_t*> begin((size_t)n, nullptr);
  std::vector<int64_t> len((size_t)n, 0);
  for (int64_t i = 0; i < n; ++i) {
    PyObject* v = PyList_GET_ITEM(values.ptr(), i);
    if (PyBytes_Check(v)) {
      begin[i] = reinterpret_cast<const uint8_t*>(PyBytes_AS_STRING(v));
      len[i] = PyBytes_GET_SIZE(v);
    } else if (v != Py_None) {   // (immutable bytes only: read with the GIL released)
      throw pybind11::type_error("values must be bytes or None");
    }
  }
  // the list (held by the caller) keeps every buffer alive while the GIL is released
  pybind11::gil_scoped_release nogil;
  return fdx::extract_json_field_ptrs(begin.data(), len.data(), n, reinterpret_cast<const uint8_t*>(field.data()),
                                      (int64_t)field.size(), out.data_ptr<uint8_t>(), out.numel(),
                                      out_off.data_ptr<int64_t>(), status.data_ptr<int32_t>(), (int)threads);
}

// Page-lock an existing host buffer (a shared-memory segment mapped by several processes) so the
// GPU process DMAs micro-batches straight out of it; a CPU tensor over it then reports is_pinned.
void host_register(const Tensor& t) {
  FDX_CHECK(t.device().is_cpu() && t.is_contiguous(), "host_register needs a contiguous CPU tensor");
  const size_t n = (size_t)t.numel() * t.element_size();
  FDX_CHECK(hipHostRegister(t.data_ptr(), n, hipHostRegisterMapped | hipHostRegisterPortable) == hipSuccess,
            "hipHostRegister failed");
}

void host_unregister(const Tensor& t) {
  FDX_CHECK(hipHostUnregister(t.data_ptr()) == hipSuccess, "hipHostUnregister failed");
}

}  // namespace

void register_tree_ops(pybind11::module& m);
void register_kafka_ops(pybind11::module& m);
void register_level_ops(pybind11::module& m);

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "MI355X-native core of fraud_detection_spark_kafka_llm_amd";
  register_tree_ops(m);
  register_kafka_ops(m);
  register_level_ops(m);
  m.def("token_keys", &token_keys, "CountVectorizer fit: 64-bit token keys (count pass / key pass)");
  m.def("featurize_score", &featurize_score, "Fused clean/tokenize/stopword/hash/idf/score");
  m.def("score_csr", &score_csr, "LR / tree-ensemble scoring of a CSR feature matrix");
  m.def("spmv", &spmv, "y = X x (CSR, fp64 accumulate)");
  m.def("spmv_t", &spmv_t, "g += X^T r (CSR, fp64)");
  m.def("doc_freq", &doc_freq, "IDF document frequencies (device)");
  m.def("clamp_u8", &clamp_u8, "uint8 clamp (bins)");
  m.def("copy_segments", &copy_segments, "segment copy of (row, key) arrays (+ per-segment key offset)");
  m.def("dense_scatter", &dense_scatter, "the hot features' dense bin block from their CSC segments");
  m.def("pack_runs", &pack_runs, "greedy packing runs of histogram work items (host)");
  m.def("block_bounds", &block_bounds, "row-block segment bounds of sorted-row columns");
  m.def("feature_order", &feature_order, "CSR -> CSC by feature (radix sort), docFreq and max count per feature");
  m.def("encode_records", &encode_records, "json.dumps-identical classification records (batch)");
  m.def("extract_json_field", &extract_json_field, "Bulk JSON string-field extraction into a packed buffer");
  m.def("extract_json_field_refs", &extract_json_field_refs,
        "extract_json_field over the first count values of a list of bytes (no packing copy)");
  m.def("host_register", &host_register, "hipHostRegister a CPU tensor's buffer (mapped, portable)");
  m.def("host_unregister", &host_unregister, "hipHostUnregister a buffer registered by host_register");
  m.attr("gfx_arch") = "gfx950";
}

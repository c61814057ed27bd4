// Host-path self-test for sanitizer builds: exercises the multi-threaded CPU
// implementations (featurizer incl. token keys, JSON extraction, tree engine) on edge cases and
// checks them against simple scalar references. Built with -fsanitize=address,undefined by
// fraud_detection_spark_kafka_llm_amd/_build.py:build_host_selftest(); exits non-zero on failure.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "ops.h"
#include "tree.h"

using namespace fdx;

static int g_fail = 0;
#define EXPECT(c)                                                       \
  do {                                                                  \
    if (!(c)) { std::fprintf(stderr, "FAIL %s:%d %s\n", __FILE__, __LINE__, #c); ++g_fail; } \
  } while (0)

struct OwnedTable {
  std::vector<int32_t> slots;
  std::vector<uint32_t> hashes;
  std::vector<int64_t> offs;
  std::vector<uint8_t> bytes;
  StrTable view() const { return StrTable{slots.data(), hashes.data(), offs.data(), bytes.data(), (int32_t)slots.size() - 1}; }
};

static OwnedTable make_table(const std::vector<std::string>& words) {
  OwnedTable t;
  size_t size = 16;
  while (size < 2 * words.size()) size <<= 1;
  t.slots.assign(size, -1);
  t.offs.push_back(0);
  for (size_t i = 0; i < words.size(); ++i) {
    const auto* p = reinterpret_cast<const uint8_t*>(words[i].data());
    const uint32_t h = murmur3_bytes(p, (uint32_t)words[i].size(), 42u);
    t.hashes.push_back(h);
    size_t j = h & (size - 1);
    while (t.slots[j] >= 0) j = (j + 1) & (size - 1);
    t.slots[j] = (int32_t)i;
    t.bytes.insert(t.bytes.end(), p, p + words[i].size());
    t.offs.push_back((int64_t)t.bytes.size());
  }
  t.bytes.push_back(0);
  return t;
}

// scalar reference: lower + keep [a-z ], split on ' ' (Java semantics), drop stop words
static std::vector<std::string> ref_tokens(const std::string& s, const std::vector<std::string>& stop) {
  std::string c;
  for (unsigned char ch : s) {
    const unsigned char l = (ch >= 'A' && ch <= 'Z') ? ch + 32 : ch;
    if ((l >= 'a' && l <= 'z') || l == ' ') c.push_back((char)l);
  }
  std::vector<std::string> parts;
  size_t q = c.find_last_not_of(' ');
  if (q == std::string::npos) {
    if (c.empty()) parts.push_back("");
  } else {
    std::string cur;
    for (size_t i = 0; i <= q; ++i) {
      if (c[i] == ' ') { parts.push_back(cur); cur.clear(); } else { cur.push_back(c[i]); }
    }
    parts.push_back(cur);
  }
  std::vector<std::string> out;
  for (auto& p : parts) {
    bool sw = false;
    for (auto& w : stop) sw = sw || (w == p);
    if (!sw) out.push_back(p);
  }
  return out;
}

static void test_featurizer() {
  const std::vector<std::string> stop = {"the", "a", "is"};
  OwnedTable st = make_table(stop);
  std::vector<std::string> docs = {"Hello World, the END is near!", "", "   ", "a  b  c ", "ABC d\xc3\xa9" "f 123",
                                   "the the the", std::string(9000, 'x') + " tail words here"};
  for (int i = 0; i < 200; ++i) docs.push_back("doc " + std::to_string(i) + " scam bank verify account please");
  std::vector<uint8_t> text;
  std::vector<int64_t> off = {0};
  for (auto& d : docs) { text.insert(text.end(), d.begin(), d.end()); off.push_back((int64_t)text.size()); }
  text.resize(text.size() + 16, 0);
  const int64_t D = (int64_t)docs.size();
  const int F = 1 << 10;

  // 1. CSR counts (HashingTF) on 4 threads
  std::vector<int32_t> idx(text.size() + D), nnz(D), ntok(D), status(D, -1);
  std::vector<float> val(text.size() + D);
  std::vector<double> raw(D);
  FeatArgs a{};
  a.text = text.data();
  a.doc_off = off.data();
  a.num_docs = (int32_t)D;
  a.flags = kFlagClean | kFlagStopwords | kFlagWriteCsr;
  a.num_features = F;
  a.stop = st.view();
  a.vocab.mask = -1;
  a.min_tf = 1.0;
  a.out_idx = idx.data();
  a.out_val = val.data();
  a.out_nnz = nnz.data();
  a.out_ntok = ntok.data();
  a.out_raw = raw.data();
  a.out_status = status.data();
  featurize_score_cpu(a, nullptr, 0, 4);
  for (int64_t d = 0; d < D; ++d) {
    EXPECT(status[d] == kStatusOk);
    const auto toks = ref_tokens(docs[d], stop);
    EXPECT(ntok[d] == (int32_t)toks.size());
    std::map<int, double> ref;
    for (auto& t : toks)
      ref[non_negative_mod(murmur3_bytes(reinterpret_cast<const uint8_t*>(t.data()), (uint32_t)t.size(), 42u), F)] += 1;
    EXPECT(nnz[d] == (int32_t)ref.size());
    const int64_t base = csr_slot(off[d], d);
    for (int32_t j = 0; j < nnz[d] && j < (int32_t)ref.size(); ++j) EXPECT(ref.count(idx[base + j]) && ref[idx[base + j]] == val[base + j]);
  }

  // 2. token keys: count pass, then key pass at the scanned offsets
  std::vector<int32_t> kt(D), ks(D, -1);
  FeatArgs k = a;
  k.flags = kFlagClean | kFlagStopwords | kFlagKeys;
  k.out_ntok = kt.data();
  k.out_status = ks.data();
  featurize_score_cpu(k, nullptr, 0, 3);
  std::vector<int64_t> koff(D + 1, 0);
  for (int64_t d = 0; d < D; ++d) koff[d + 1] = koff[d] + kt[d];
  std::vector<uint64_t> keys(koff[D]);
  k.key_off = koff.data();
  k.out_keys = keys.data();
  featurize_score_cpu(k, nullptr, 0, 3);
  for (int64_t d = 0; d < D; ++d) {
    const auto toks = ref_tokens(docs[d], stop);
    EXPECT(kt[d] == (int32_t)toks.size());
    for (size_t i = 0; i < toks.size() && (int64_t)i < kt[d]; ++i) {
      const auto* p = reinterpret_cast<const uint8_t*>(toks[i].data());
      const uint64_t want = ((uint64_t)murmur3_bytes(p, (uint32_t)toks[i].size(), 42u) << 32) |
                            murmur3_bytes(p, (uint32_t)toks[i].size(), kKeySeed2);
      EXPECT(keys[koff[d] + i] == want);
    }
  }
}

static void test_json() {
  const std::vector<std::string> msgs = {R"({"text": "hi \"there\" é\n"})", R"({"other": 1, "text":"x"})",
                                         R"({"no": "field"})", "not json", R"({"text": 5})", ""};
  std::vector<uint8_t> in;
  std::vector<int64_t> off = {0};
  for (auto& m : msgs) { in.insert(in.end(), m.begin(), m.end()); off.push_back((int64_t)in.size()); }
  in.resize(in.size() + 16, 0);
  std::vector<uint8_t> out(in.size() * 2 + 64);
  std::vector<int64_t> out_off(msgs.size() + 1);
  std::vector<int32_t> st(msgs.size());
  const char* field = "text";
  extract_json_field(in.data(), off.data(), (int64_t)msgs.size(), reinterpret_cast<const uint8_t*>(field), 4,
                     out.data(), (int64_t)out.size(), out_off.data(), st.data(), 2);
  EXPECT(st[0] == 0 && std::string(out.begin() + out_off[0], out.begin() + out_off[1]) == "hi \"there\" \xc3\xa9\n");
  EXPECT(st[1] == 0 && std::string(out.begin() + out_off[1], out.begin() + out_off[2]) == "x");
  EXPECT(st[2] != 0 && st[3] != 0 && st[4] != 0 && st[5] != 0);
}

static void test_tree() {
  // 6 rows x 3 features, CSC with bins; statistics g = row - 2.5, h = 1 (exact in the quantised grid)
  const int64_t N = 6;
  const std::vector<int64_t> colptr = {0, 3, 5, 8};
  std::vector<int32_t> rows = {0, 2, 5, 1, 2, 0, 3, 4};
  std::vector<uint8_t> bins = {1, 2, 1, 1, 3, 2, 2, 1};
  rows.resize(rows.size() + 16, 0);
  bins.resize(bins.size() + 16, 0xff);
  std::vector<float> g(N), h(N, 1.0f);
  for (int i = 0; i < N; ++i) g[i] = (float)i - 2.5f;
  std::vector<uint32_t> rd(2 * N);
  std::vector<int32_t> kexp(2);
  std::vector<int64_t> totals(2);
  QuantArgs qa{};
  qa.g = g.data();
  qa.h = h.data();
  qa.N = N;
  qa.np = 4;
  qa.rowdig = rd.data();
  qa.kexp_out = kexp.data();
  qa.totals = totals.data();
  double mx[2];
  quant_max_cpu(qa, mx);
  EXPECT(mx[0] == 2.5 && mx[1] == 1.0);
  quant_cpu(qa, mx);
  EXPECT(kexp[0] == 28 && kexp[1] == 29);
  for (int i = 0; i < N; ++i) EXPECT(undigits4(rd[2 * i]) == (int64_t)std::ldexp((double)g[i], 28));
  EXPECT(totals[0] == 0 && totals[1] == 6 * (int64_t(1) << 29));
  std::vector<int32_t> row_node = {0, 1, 0, 1, 0, 1}, node_slot = {0, 1};
  std::vector<uint8_t> slot8(N);
  SlotArgs sa{row_node.data(), node_slot.data(), 2, 0, 2, N, slot8.data()};
  slot8_cpu(sa);
  // one single-feature item per column (key = bin, stride 256)
  const std::vector<int64_t> item_start = {0, 3, 5}, item_end = {3, 5, 8}, boff = {0, 4, 8, 12};
  const std::vector<int32_t> f0 = {0, 1, 2}, meta = {8 | (1 << 8), 8 | (1 << 8), 8 | (1 << 8)};
  const std::vector<int32_t> nbins = {4, 4, 4}, s2n = {0, 1};
  std::vector<int64_t> hist(2 * 12 * 2, 0);
  HistArgs ha{};
  ha.item_start = item_start.data();
  ha.item_end = item_end.data();
  ha.item_f0 = f0.data();
  ha.item_meta = meta.data();
  ha.num_items = 3;
  ha.csc_row = rows.data();
  ha.csc_key = bins.data();
  ha.slot8 = slot8.data();
  ha.rowdig = rd.data();
  ha.boff = boff.data();
  ha.nbins = nbins.data();
  ha.slot_node = s2n.data();
  ha.nslots = 2;
  ha.hist_stride = 12;
  ha.hist = hist.data();
  hist_cpu(ha, 1, 4);
  int64_t ref[2][12] = {};
  for (int f = 0; f < 3; ++f)
    for (int64_t e = colptr[f]; e < colptr[f + 1]; ++e)
      ref[row_node[rows[e]]][boff[f] + bins[e]] += (int64_t)std::ldexp((double)g[rows[e]], 28);
  for (int n = 0; n < 2; ++n)
    for (int b = 0; b < 12; ++b) EXPECT(hist[((size_t)n * 12 + b) * 2] == ref[n][b]);
}

// Row-group engine on the host: CSR layout build (with the entry-major rows of the sparse group),
// row lists with masked digit words, and the histogram pass at the root and at a listed
// single-node level (entry-major for the sparse group) against scalar sums.
static void test_rowgroups() {
  const int64_t N = 7;
  // rows x features (counts; 0 = absent): features 0, 1 -> group 0 (balanced), 2, 3 -> group 1
  const int cnt[7][4] = {{1, 2, 0, 1}, {3, 0, 1, 0}, {1, 1, 0, 0}, {0, 2, 2, 1}, {2, 0, 0, 3}, {1, 1, 1, 1}, {0, 0, 0, 0}};
  std::vector<int64_t> indptr = {0};
  std::vector<int32_t> idx, counts;
  for (int r = 0; r < N; ++r) {
    for (int f = 0; f < 4; ++f)
      if (cnt[r][f]) { idx.push_back(f); counts.push_back(cnt[r][f]); }
    indptr.push_back((int64_t)idx.size());
  }
  const std::vector<int32_t> remap = {0, 1, 2, 3}, fgroup = {0, 0, 1, 1}, flocal = {0, 8, 0, 8};
  int64_t e0 = 0, e1 = 0;
  for (int r = 0; r < N; ++r)
    for (int f = 0; f < 4; ++f) if (cnt[r][f]) (f < 2 ? e0 : e1) += 1;
  const std::vector<int64_t> gbase = {0, (e0 + 7) / 8 * 8, (e0 + 7) / 8 * 8 + (e1 + 7) / 8 * 8};
  std::vector<uint32_t> ptr(2 * (N + 1));
  std::vector<uint16_t> ent((size_t)gbase[2] + 16, 0);
  std::vector<uint32_t> wave_base(64), erow((size_t)(gbase[2] - gbase[1]) + 8, 0xffffffffu);
  RgCsrBuildArgs<int32_t> ba{};
  ba.indptr = indptr.data(); ba.idx = idx.data(); ba.counts = counts.data(); ba.N = N; ba.remap = remap.data();
  ba.max_bin = 7; ba.fgroup = fgroup.data(); ba.flocal = flocal.data(); ba.G = 2; ba.ptr = ptr.data();
  ba.gbase = gbase.data(); ba.ent = ent.data(); ba.wave_base = wave_base.data();
  ba.erow = erow.data(); ba.em_g0 = 1; ba.ebase = gbase[1];
  rg_build_csr_cpu<int32_t>(ba);
  for (int64_t i = 0; i < e1; ++i) {           // the entry-major rows of group 1: its row runs, in order
    int64_t r = 0;
    while (!(ptr[N + 1 + r] <= (uint32_t)i && (uint32_t)i < ptr[N + 1 + r + 1])) ++r;
    EXPECT(erow[i] == (uint32_t)r);
  }
  // statistics q0 = 3 r - 7, q1 = r + 1 (digit words)
  std::vector<uint32_t> rd(2 * N);
  for (int r = 0; r < N; ++r) { rd[2 * r] = digits4(3 * r - 7); rd[2 * r + 1] = digits4(r + 1); }
  const std::vector<int32_t> gbin = [] {
    std::vector<int32_t> v(2 * 8192, -1);
    for (int b = 0; b < 16; ++b) { v[b] = b; v[8192 + b] = 16 + b; }      // global column = 8 f + count bin
    return v;
  }();
  const std::vector<uint8_t> gmode = {1, 0};
  const std::vector<int32_t> wg_g = {0, 0, 1, 1}, wg_p = {0, 1, 0, 1}, wg_np = {2, 2, 2, 2}, slot_node = {0};
  auto run = [&](const int32_t* list, const int32_t* slot_start, const uint32_t* listdig, const uint32_t* emdig,
                 std::vector<int64_t>& hist) {
    RgHistArgs ha{};
    ha.ptr = ptr.data(); ha.ent = ent.data(); ha.gbase = gbase.data(); ha.gbin = gbin.data(); ha.gbins = 8192;
    ha.G = 2; ha.N = N; ha.rowdig = rd.data(); ha.np = 4; ha.list = list; ha.listdig = listdig; ha.gmode = gmode.data();
    ha.slot_start = slot_start; ha.nslots = 1; ha.wg_g = wg_g.data(); ha.wg_p = wg_p.data(); ha.wg_np = wg_np.data();
    ha.n_wg = 4; ha.slot_node = slot_node.data(); ha.hist_stride = 32; ha.hist = hist.data();
    ha.erow = erow.data(); ha.ebase = gbase[1]; ha.emdig = emdig; ha.em_min_rows = 1;
    rg_hist_cpu(ha);
  };
  auto ref_of = [&](const std::vector<int>& built) {
    std::vector<int64_t> ref(64, 0);
    for (int r : built)
      for (int f = 0; f < 4; ++f)
        if (cnt[r][f]) {
          const int col = 8 * f + std::min(cnt[r][f], 7);
          ref[2 * col] += 3 * r - 7;
          ref[2 * col + 1] += r + 1;
        }
    return ref;
  };
  std::vector<int64_t> hist(64, 0);
  run(nullptr, nullptr, nullptr, nullptr, hist);               // root: every row, group 1 entry-major
  EXPECT(hist == ref_of({0, 1, 2, 3, 4, 5, 6}));
  // a listed level with one built node (rows 1, 3, 4, 5)
  const std::vector<int32_t> row_node = {2, 1, 2, 1, 1, 1, -1}, node_slot = {-1, 0, -1};
  std::vector<int32_t> list(N, -7), slot_start(2), work(2 + 2 * (int)((N + rg_list_rows(N) - 1) / rg_list_rows(N)));
  std::vector<uint32_t> listdig(2 * N), masked(2 * N, 99u);
  RgListArgs la{};
  la.row_node = row_node.data(); la.node_slot = node_slot.data(); la.num_nodes = 3; la.N = N; la.nslots = 1;
  la.slot_count = work.data(); la.wave_count = work.data() + 2; la.slot_start = slot_start.data(); la.list = list.data();
  la.rowdig = rd.data(); la.listdig = listdig.data(); la.masked = masked.data();
  rg_list_cpu(la);
  EXPECT(slot_start[0] == 0 && slot_start[1] == 4);
  for (int r = 0; r < N; ++r) {
    const bool b = row_node[r] == 1;
    EXPECT(masked[2 * r] == (b ? rd[2 * r] : 0u) && masked[2 * r + 1] == (b ? rd[2 * r + 1] : 0u));
  }
  std::fill(hist.begin(), hist.end(), 0);
  run(list.data(), slot_start.data(), listdig.data(), masked.data(), hist);
  EXPECT(hist == ref_of({1, 3, 4, 5}));
  std::fill(hist.begin(), hist.end(), 0);
  run(list.data(), slot_start.data(), listdig.data(), nullptr, hist);   // (row lists for both groups)
  EXPECT(hist == ref_of({1, 3, 4, 5}));
}

int main() {
  test_featurizer();
  test_json();
  test_tree();
  test_rowgroups();
  if (g_fail) {
    std::fprintf(stderr, "%d failures\n", g_fail);
    return 1;
  }
  std::printf("host selftest OK\n");
  return 0;
}

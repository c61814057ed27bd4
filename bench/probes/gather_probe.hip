// Cost of the per-entry row-state access of the cold CSC histogram pass, isolated (gfx950).
//
// Synthetic CSC shaped like the 10M-row GBDT training matrix's cold features (28,493 features,
// ~386M entries, entries of one feature ~700 rows apart, sorted by row inside a row block).
// Every wave walks one work item (a chunk of consecutive entries: int32 rows + uint8 keys, 4 per
// lane per step, like hist_i8_kernel) and folds what it reads into an xor so nothing is dead code.
//   stream    : rows + keys only (the floor of any CSC pass)
//   g8        : + one 8-byte gather of the row's digit word per entry (global, L2/MALL)
//   g8s1      : + one 1-byte gather of the row's slot too (the current non-root pass)
//   lds       : row blocks of R rows; a workgroup stages the block's digit words in LDS with
//               coalesced loads, then its waves walk the block's items and read the words from LDS
// Layout A: 262,144-row super-blocks (the current quantizer); layout B: R-row blocks.
// Usage: gather_probe [reps]    prints one JSON line per variant.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1); } } while (0)

constexpr int64_t N = 10000000;
constexpr int F = 28493;
constexpr double P = 386.0e6 / (10.0e6 * F);      // entry density of a cold feature

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16; return x;
}

// segment s = (block b, feature f): m entries at stratified random rows of the block, ascending
__global__ void gen_kernel(int32_t* rows, uint8_t* keys, int64_t nseg, int m, int64_t blk_rows, int nblk) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t total = nseg * m;
  for (int64_t e = t; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t s = e / m;
    const int j = (int)(e % m);
    const int64_t b = s / F;
    const int64_t r0 = b * blk_rows;
    const int64_t r1 = (r0 + blk_rows < N) ? r0 + blk_rows : N;
    const int64_t span = r1 - r0;
    const int64_t stride = span / m;
    int64_t r = r0 + j * stride + (int64_t)(hash32((uint32_t)e * 2654435761u) % (uint32_t)(stride > 0 ? stride : 1));
    if (r >= r1) r = r1 - 1;
    rows[e] = (int32_t)r;
    keys[e] = (uint8_t)(hash32((uint32_t)e) & 15);
  }
}

struct Items {
  const int64_t* start;
  const int64_t* end;
  const int32_t* blk;
  const int32_t* wave_item;   // optional: wave slot -> item (XCD-aware order)
  int n;
  int nslots;
};

template <int MODE>   // 0 stream, 1 g8, 2 g8s1, 3 g16 (one 16-byte record: digits + slot)
__global__ __launch_bounds__(256) void walk_kernel(Items it, const int32_t* __restrict__ rows, const uint8_t* __restrict__ keys,
                                                   const uint2* __restrict__ dig, const uint8_t* __restrict__ slot,
                                                   uint32_t* out) {
  const int lane = threadIdx.x & 63;
  const int ws = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int item = it.wave_item ? (ws < it.nslots ? it.wave_item[ws] : -1) : ws;
  if (item < 0 || item >= it.n) return;
  const int64_t e0 = it.start[item], e1 = it.end[item];
  uint32_t acc = 0;
  const int64_t first = e0 & ~(int64_t)3;
  const int64_t last4 = (e1 - 1) & ~(int64_t)3;
  int4 nr;
  uint32_t nk;
  {
    const int64_t e = first + 4 * lane < last4 ? first + 4 * lane : last4;
    nr = *reinterpret_cast<const int4*>(rows + e);
    nk = *reinterpret_cast<const uint32_t*>(keys + e);
  }
  for (int64_t base = first; base < e1; base += 256) {
    const int4 r4 = nr;
    const uint32_t k4 = nk;
    {
      const int64_t e = base + 256 + 4 * lane < last4 ? base + 256 + 4 * lane : last4;
      nr = *reinterpret_cast<const int4*>(rows + e);
      nk = *reinterpret_cast<const uint32_t*>(keys + e);
    }
    acc ^= k4 ^ (uint32_t)r4.x ^ (uint32_t)r4.w;
    if constexpr (MODE == 3) {
      const uint4* rec = reinterpret_cast<const uint4*>(slot);
      const uint4 a = rec[r4.x], b = rec[r4.y], c = rec[r4.z], d = rec[r4.w];
      acc += a.x ^ b.y ^ c.z ^ d.w;
    } else if constexpr (MODE >= 1) {
      const uint2 a = dig[r4.x], b = dig[r4.y], c = dig[r4.z], d = dig[r4.w];
      acc += a.x ^ b.y ^ c.x ^ d.y;
    }
    if constexpr (MODE == 2) {
      acc += (uint32_t)slot[r4.x] + slot[r4.y] + slot[r4.z] + slot[r4.w];
    }
  }
  if (acc == 0x12345678u) out[item] = acc;   // practically never: keeps the loads live
}

// one workgroup per row block (R rows): stage digits in LDS, then the block's items
template <int R>
__global__ __launch_bounds__(1024) void lds_kernel(const int64_t* blk_item0, Items it, const int32_t* __restrict__ rows,
                                                   const uint8_t* __restrict__ keys, const uint2* __restrict__ dig,
                                                   uint32_t* out, int nblk, int64_t blk_rows) {
  extern __shared__ uint2 s_dig[];
  const int b = blockIdx.x;
  if (b >= nblk) return;
  const int64_t r0 = (int64_t)b * blk_rows;
  const int nrows = (int)((r0 + blk_rows < N ? r0 + blk_rows : N) - r0);
  for (int i = threadIdx.x * 2; i < nrows; i += 2 * blockDim.x) {
    const uint4 v = *reinterpret_cast<const uint4*>(dig + r0 + i);
    s_dig[i] = make_uint2(v.x, v.y);
    if (i + 1 < nrows) s_dig[i + 1] = make_uint2(v.z, v.w);
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  uint32_t acc = 0;
  for (int64_t item = blk_item0[b] + w; item < blk_item0[b + 1]; item += nw) {
    const int64_t e0 = it.start[item], e1 = it.end[item];
    const int64_t first = e0 & ~(int64_t)3;
    const int64_t last4 = (e1 - 1) & ~(int64_t)3;
    for (int64_t base = first; base < e1; base += 256) {
      const int64_t e = base + 4 * lane < last4 ? base + 4 * lane : last4;
      const int4 r4 = *reinterpret_cast<const int4*>(rows + e);
      const uint32_t k4 = *reinterpret_cast<const uint32_t*>(keys + e);
      const int lim = nrows - 1;
      const int ix = min(max((int)(r4.x - r0), 0), lim), iy = min(max((int)(r4.y - r0), 0), lim);
      const int iz = min(max((int)(r4.z - r0), 0), lim), iw = min(max((int)(r4.w - r0), 0), lim);
      const uint2 a = s_dig[ix], bb = s_dig[iy], c = s_dig[iz], d = s_dig[iw];
      acc ^= k4 + (a.x ^ bb.y ^ c.x ^ d.y);
    }
  }
  if (acc == 0x12345678u) out[b] = acc;
}

struct Layout {
  int64_t blk_rows;
  int nblk, m;
  int64_t nent;
  int32_t* rows;
  uint8_t* keys;
  Items it;
  int64_t* blk_item0;
  int64_t* d_start;
  int64_t* d_end;
  int32_t* d_blk;
  int64_t* d_bi0;
  int32_t* d_wi;
};

static Layout make_layout(int64_t blk_rows, int feats_per_item) {
  Layout L{};
  L.blk_rows = blk_rows;
  L.nblk = (int)((N + blk_rows - 1) / blk_rows);
  L.m = (int)(blk_rows * P + 0.5);
  if (L.m < 1) L.m = 1;
  const int64_t nseg = (int64_t)L.nblk * F;
  L.nent = nseg * L.m;
  CK(hipMalloc(&L.rows, (L.nent + 64) * 4));
  CK(hipMalloc(&L.keys, L.nent + 64));
  CK(hipMemset(L.rows, 0, (L.nent + 64) * 4));
  CK(hipMemset(L.keys, 0, L.nent + 64));
  gen_kernel<<<8192, 256>>>(L.rows, L.keys, nseg, L.m, blk_rows, L.nblk);
  CK(hipGetLastError());
  std::vector<int64_t> st, en, bi0;
  std::vector<int32_t> bl;
  for (int b = 0; b < L.nblk; ++b) {
    bi0.push_back((int64_t)st.size());
    for (int f = 0; f < F; f += feats_per_item) {
      const int f1 = f + feats_per_item < F ? f + feats_per_item : F;
      st.push_back(((int64_t)b * F + f) * L.m);
      en.push_back(((int64_t)b * F + f1) * L.m);
      bl.push_back(b);
    }
  }
  bi0.push_back((int64_t)st.size());
  L.it.n = (int)st.size();
  // XCD-aware wave order: blocks b and b+8 share an XCD; XCD x takes the row blocks x, x+8, ...
  std::vector<std::vector<int32_t>> per(8);
  for (int i = 0; i < L.it.n; ++i) per[bl[i] % 8].push_back(i);
  size_t mx = 0;
  for (auto& p : per) mx = p.size() > mx ? p.size() : mx;
  const size_t nblocks = (mx + 3) / 4 * 8;
  std::vector<int32_t> wi(nblocks * 4, -1);
  for (int x = 0; x < 8; ++x)
    for (size_t k = 0; k < per[x].size(); ++k) wi[((k / 4) * 8 + x) * 4 + k % 4] = per[x][k];
  L.it.nslots = (int)wi.size();
  CK(hipMalloc(&L.d_wi, wi.size() * 4));
  CK(hipMemcpy(L.d_wi, wi.data(), wi.size() * 4, hipMemcpyHostToDevice));
  CK(hipMalloc(&L.d_start, st.size() * 8));
  CK(hipMalloc(&L.d_end, en.size() * 8));
  CK(hipMalloc(&L.d_blk, bl.size() * 4));
  CK(hipMalloc(&L.d_bi0, bi0.size() * 8));
  CK(hipMemcpy(L.d_start, st.data(), st.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(L.d_end, en.data(), en.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(L.d_blk, bl.data(), bl.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(L.d_bi0, bi0.data(), bi0.size() * 8, hipMemcpyHostToDevice));
  L.it.start = L.d_start;
  L.it.end = L.d_end;
  L.it.blk = L.d_blk;
  L.blk_item0 = L.d_bi0;
  CK(hipDeviceSynchronize());
  return L;
}

static void free_layout(Layout& L) {
  hipFree(L.rows); hipFree(L.keys); hipFree(L.d_start); hipFree(L.d_end); hipFree(L.d_blk); hipFree(L.d_bi0); hipFree(L.d_wi);
}

template <typename Fn>
static float time_ms(Fn fn, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  fn();
  CK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int i = 0; i < reps; ++i) {
    CK(hipEventRecord(a));
    fn();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    best = ms < best ? ms : best;
  }
  return best;
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 5;
  uint2* dig;
  uint8_t* slot;
  uint32_t* out;
  CK(hipMalloc(&dig, (N + 64) * 8));
  CK(hipMalloc(&slot, (N + 64) * 16));
  CK(hipMalloc(&out, 1 << 24));
  CK(hipMemset(dig, 0x5a, (N + 64) * 8));
  CK(hipMemset(slot, 3, (N + 64) * 16));
  struct Cfg { int64_t blk; int fpi; };
  const Cfg cfgs[] = {{262144, 4}, {16384, 64}, {8192, 128}};
  for (const Cfg& c : cfgs) {
    Layout L = make_layout(c.blk, c.fpi);
    const int grid = (L.it.n + 3) / 4;
    const double ent = (double)L.nent;
    auto report = [&](const char* name, float ms) {
      printf("{\"variant\": \"%s\", \"blk_rows\": %lld, \"items\": %d, \"entries\": %.0f, \"ms\": %.3f, \"G_entries_per_s\": %.1f}\n",
             name, (long long)c.blk, L.it.n, ent, ms, ent / ms / 1e6);
      fflush(stdout);
    };
    report("stream", time_ms([&] { walk_kernel<0><<<grid, 256>>>(L.it, L.rows, L.keys, dig, slot, out); }, reps));
    report("g8", time_ms([&] { walk_kernel<1><<<grid, 256>>>(L.it, L.rows, L.keys, dig, slot, out); }, reps));
    report("g8s1", time_ms([&] { walk_kernel<2><<<grid, 256>>>(L.it, L.rows, L.keys, dig, slot, out); }, reps));
    Items ix = L.it;
    ix.wave_item = L.d_wi;
    const int gx = (ix.nslots + 3) / 4;
    report("stream_xcd", time_ms([&] { walk_kernel<0><<<gx, 256>>>(ix, L.rows, L.keys, dig, slot, out); }, reps));
    report("g8_xcd", time_ms([&] { walk_kernel<1><<<gx, 256>>>(ix, L.rows, L.keys, dig, slot, out); }, reps));
    report("g8s1_xcd", time_ms([&] { walk_kernel<2><<<gx, 256>>>(ix, L.rows, L.keys, dig, slot, out); }, reps));
    report("g16_xcd", time_ms([&] { walk_kernel<3><<<gx, 256>>>(ix, L.rows, L.keys, dig, slot, out); }, reps));
    if (c.blk <= 16384) {
      const size_t lds = (size_t)c.blk * 8;
      CK(hipFuncSetAttribute((const void*)lds_kernel<0>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
      auto fn1024 = [&] { lds_kernel<0><<<L.nblk, 1024, lds>>>(L.blk_item0, L.it, L.rows, L.keys, dig, out, L.nblk, c.blk); };
      auto fn512 = [&] { lds_kernel<0><<<L.nblk, 512, lds>>>(L.blk_item0, L.it, L.rows, L.keys, dig, out, L.nblk, c.blk); };
      report("lds_1024t", time_ms(fn1024, reps));
      report("lds_512t", time_ms(fn512, reps));
    }
    free_layout(L);
  }
  return 0;
}

// Histogram tree engine for gfx950 (K-10..K-15 of SURVEY.md §2.5), exact integer arithmetic.
//
// Histogram build on the i8 matrix cores: for one work item (a chunk of one feature column, or
// several small whole columns packed into one 64-key tile), the per-(key, node slot, statistic)
// sums are the product  C[key][col] = sum_k A[key][k] * B[k][col]  over the item's entries k,
// with A = one-hot(key_k) (0x80 = -128 in the matching byte) and B[k][col] = the entry's digit
// of (statistic, plane) of col, masked to the entries in col's node slot. v_mfma_i32_16x16x64_i8
// accumulates exactly in int32; the epilogue divides by -128, recombines the NP digit planes into
// int64 and adds them to the int64 histogram with integer atomics (order-independent, so the
// result is bitwise deterministic). One wave per work item, 64 entries per MFMA K-step.
// The rest of the level (sibling subtraction, split search, row partition) are small
// bandwidth-bound kernels on the same int64 histograms.
#include "hist_i8.h"
#include <cstdlib>

#include "ops.h"
#include "tree.h"

#pragma clang fp contract(off)

namespace fdx {

namespace {
// ------------------------------------------------------------------ quantised row statistics
// max |v| of the two statistics over the rows (doubles are >= 0, so their bit patterns order
// like unsigned integers: exact, order-independent atomic max).
__global__ __launch_bounds__(256) void quant_max_kernel(QuantArgs a, unsigned long long* out) {
  double m0 = 0.0, m1 = 0.0;
  for (int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x; r < a.N; r += (int64_t)gridDim.x * 256) {
    double v0, v1;
    row_stats(a, r, &v0, &v1);
    m0 = fmax(m0, fabs(v0));
    m1 = fmax(m1, fabs(v1));
  }
  for (int o = 32; o > 0; o >>= 1) {
    m0 = fmax(m0, __shfl_xor(m0, o, kWave));
    m1 = fmax(m1, __shfl_xor(m1, o, kWave));
  }
  // one partial per block, reduced by quant_reduce_kernel: atomics of every block on the same two
  // addresses serialised in L2 (2048 blocks: ~40 us of a ~60 us kernel at 1M rows)
  __shared__ double s_m[2][4];
  const int w = threadIdx.x / kWave;
  if ((threadIdx.x & (kWave - 1)) == 0) { s_m[0][w] = m0; s_m[1][w] = m1; }
  __syncthreads();
  if (threadIdx.x == 0) {
    m0 = fmax(fmax(s_m[0][0], s_m[0][1]), fmax(s_m[0][2], s_m[0][3]));
    m1 = fmax(fmax(s_m[1][0], s_m[1][1]), fmax(s_m[1][2], s_m[1][3]));
    out[2 * blockIdx.x] = (unsigned long long)__double_as_longlong(m0);
    out[2 * blockIdx.x + 1] = (unsigned long long)__double_as_longlong(m1);
  }
}

// One block: the per-block partials (pairs) -> out: MAX of the (non-negative double) bit patterns
// (MAX = 1) or the int64 SUM (MAX = 0). Exact and order-independent either way.
template <bool MAX>
__global__ __launch_bounds__(256) void quant_reduce_kernel(const unsigned long long* part, int nparts,
                                                           unsigned long long* out) {
  unsigned long long v0 = 0, v1 = 0;
  for (int i = threadIdx.x; i < nparts; i += 256) {
    const unsigned long long a0 = part[2 * i], a1 = part[2 * i + 1];
    if (MAX) { v0 = a0 > v0 ? a0 : v0; v1 = a1 > v1 ? a1 : v1; }
    else { v0 += a0; v1 += a1; }
  }
  __shared__ unsigned long long s[2][256];
  s[0][threadIdx.x] = v0;
  s[1][threadIdx.x] = v1;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) {
      const unsigned long long b0 = s[0][threadIdx.x + o], b1 = s[1][threadIdx.x + o];
      if (MAX) {
        s[0][threadIdx.x] = b0 > s[0][threadIdx.x] ? b0 : s[0][threadIdx.x];
        s[1][threadIdx.x] = b1 > s[1][threadIdx.x] ? b1 : s[1][threadIdx.x];
      } else {
        s[0][threadIdx.x] += b0;
        s[1][threadIdx.x] += b1;
      }
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) { out[0] = s[0][0]; out[1] = s[1][0]; }
}

// The last workgroup of a partials pass (ticket: a zeroed counter, reset here for the next
// launch): true for one workgroup, after every other workgroup's partial is visible.
// One device-scope release per workgroup, from the ticket thread only, after the barrier has
// drained every wave's stores: an agent-scope fence writes the XCD's L2 back, and one per wave
// of a 2048-workgroup grid cost ~140 us per pass (profiles/r5/NOTES.md); the acquire side runs
// in the last workgroup alone.
__device__ __forceinline__ bool last_workgroup(unsigned int* ticket, unsigned total = 0) {
  __shared__ int s_last;
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    const unsigned int t = atomicAdd(ticket, 1u);
    s_last = (t == (total ? total : gridDim.x) - 1) ? 1 : 0;
    if (s_last) atomicExch(ticket, 0u);
  }
  __syncthreads();
  if (!s_last) return false;
  __threadfence();
  return true;
}

// quant_reduce_kernel's body for the calling 256-thread workgroup
template <bool MAX>
__device__ void reduce_parts_block(const unsigned long long* part, int nparts, unsigned long long* out) {
  unsigned long long v0 = 0, v1 = 0;
  for (int i = threadIdx.x; i < nparts; i += 256) {
    const unsigned long long a0 = part[2 * i], a1 = part[2 * i + 1];
    if (MAX) { v0 = a0 > v0 ? a0 : v0; v1 = a1 > v1 ? a1 : v1; }
    else { v0 += a0; v1 += a1; }
  }
  __shared__ unsigned long long s[2][256];
  s[0][threadIdx.x] = v0;
  s[1][threadIdx.x] = v1;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) {
      const unsigned long long b0 = s[0][threadIdx.x + o], b1 = s[1][threadIdx.x + o];
      if (MAX) {
        s[0][threadIdx.x] = b0 > s[0][threadIdx.x] ? b0 : s[0][threadIdx.x];
        s[1][threadIdx.x] = b1 > s[1][threadIdx.x] ? b1 : s[1][threadIdx.x];
      } else {
        s[0][threadIdx.x] += b0;
        s[1][threadIdx.x] += b1;
      }
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) { out[0] = s[0][0]; out[1] = s[1][0]; }
}

constexpr int kPrologueU = 4;           // rows per thread per step of the prologue passes

// zero [n] int64 (16-byte stores where aligned) and copy [m] 8-byte words, grid-stride
__device__ __forceinline__ void prologue_fill(int64_t* zero, int64_t n, const uint64_t* src, uint64_t* dst, int64_t m) {
  const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, step = (int64_t)gridDim.x * blockDim.x;
  if (zero) {
    const int64_t n2 = n >> 1;
    for (int64_t i = t0; i < n2; i += step) reinterpret_cast<int4*>(zero)[i] = make_int4(0, 0, 0, 0);
    if ((n & 1) && t0 == 0) zero[n - 1] = 0;
  }
  for (int64_t i = t0; i < m; i += step) dst[i] = src[i];
}

// GBDT round prologue in one launch: g = p - y, h = max(p (1 - p), 1e-16) from the margins
// (logistic_grad_kernel's arithmetic) and max |g|, |h| into maxv with one 64-bit atomic max per
// workgroup and statistic (non-negative doubles order as their bit patterns; maxv zero at entry:
// the previous round cleared this parity's slot), plus the tree-start work of PrologueInit.
__global__ __launch_bounds__(256) void grad_max_kernel(const double* margin, const float* label, float* g, float* h,
                                                       int64_t N, unsigned long long* maxv, PrologueInit pi) {
  // kPrologueU rows per thread per step, every load issued before the first store: the grid is
  // kept small (one 64-bit atomic per workgroup and statistic), so each wave needs several loads
  // in flight (a row at a time left the pass at ~19 us for 1M rows, latency bound)
  double m0 = 0.0, m1 = 0.0;
  const int64_t step = (int64_t)gridDim.x * 256 * kPrologueU;
  for (int64_t r0 = (int64_t)blockIdx.x * 256 * kPrologueU + threadIdx.x; r0 < N; r0 += step) {
    double mg[kPrologueU];
    float lb[kPrologueU];
#pragma unroll
    for (int u = 0; u < kPrologueU; ++u) {
      const int64_t r = r0 + 256 * u;
      mg[u] = r < N ? margin[r] : 0.0;
      lb[u] = r < N ? label[r] : 0.0f;
    }
#pragma unroll
    for (int u = 0; u < kPrologueU; ++u) {
      const int64_t r = r0 + 256 * u;
      if (r >= N) break;
      const double p = 1.0 / (1.0 + exp(-mg[u]));
      const float gv = (float)(p - (double)lb[u]);
      const float hv = (float)fmax(p * (1.0 - p), 1e-16);
      g[r] = gv;
      h[r] = hv;
      m0 = fmax(m0, fabs((double)gv));
      m1 = fmax(m1, fabs((double)hv));
    }
  }
  prologue_fill(pi.zero, pi.zero_n, pi.init_src, pi.init_dst, pi.init_n);
  if (blockIdx.x == 0 && threadIdx.x < kRootSlots && pi.max_clear) {
    pi.max_clear[kRootStride * threadIdx.x] = 0ull;
    pi.max_clear[kRootStride * threadIdx.x + 1] = 0ull;
  }
  for (int o = 32; o > 0; o >>= 1) {
    m0 = fmax(m0, __shfl_xor(m0, o, kWave));
    m1 = fmax(m1, __shfl_xor(m1, o, kWave));
  }
  __shared__ double s_m[2][4];
  const int w = threadIdx.x / kWave;
  if ((threadIdx.x & (kWave - 1)) == 0) { s_m[0][w] = m0; s_m[1][w] = m1; }
  __syncthreads();
  if (threadIdx.x == 0) {
    m0 = fmax(fmax(s_m[0][0], s_m[0][1]), fmax(s_m[0][2], s_m[0][3]));
    m1 = fmax(fmax(s_m[1][0], s_m[1][1]), fmax(s_m[1][2], s_m[1][3]));
    unsigned long long* slot = maxv + kRootStride * (blockIdx.x % kRootSlots);
    atomicMax(slot, (unsigned long long)__double_as_longlong(m0));
    atomicMax(slot + 1, (unsigned long long)__double_as_longlong(m1));
  }
}

// rowdig[r] = digits of (q0, q1); totals += (sum q0, sum q1) (int64 atomics, exact)
__device__ __forceinline__ void quant_kernel_body(QuantArgs a, const double* maxv, unsigned long long* part) {
  int32_t k0 = maxv ? quant_exponent(maxv[0]) : 0, k1 = maxv ? quant_exponent(maxv[1]) : 0;
  if (a.max_parts) {                       // the max over grad_max_kernel's slots (every wave)
    const int lane = threadIdx.x & 63;
    unsigned long long b0 = lane < kRootSlots ? a.max_parts[kRootStride * lane] : 0ull;
    unsigned long long b1 = lane < kRootSlots ? a.max_parts[kRootStride * lane + 1] : 0ull;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const unsigned long long c0 = __shfl_xor(b0, o, kWave), c1 = __shfl_xor(b1, o, kWave);
      b0 = c0 > b0 ? c0 : b0;
      b1 = c1 > b1 ? c1 : b1;
    }
    k0 = quant_exponent(__longlong_as_double((long long)b0));
    k1 = quant_exponent(__longlong_as_double((long long)b1));
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) { a.kexp_out[0] = k0; a.kexp_out[1] = k1; }
  int64_t t0 = 0, t1 = 0;
  // kPrologueU rows per thread per step, the row statistics loaded before any store (see
  // grad_max_kernel)
  const int64_t step = (int64_t)gridDim.x * 256 * kPrologueU;
  for (int64_t r0 = (int64_t)blockIdx.x * 256 * kPrologueU + threadIdx.x; r0 < a.N; r0 += step) {
    double sv0[kPrologueU], sv1[kPrologueU];
#pragma unroll
    for (int u = 0; u < kPrologueU; ++u) {
      sv0[u] = sv1[u] = 0.0;
      if (r0 + 256 * u < a.N) row_stats(a, r0 + 256 * u, &sv0[u], &sv1[u]);
    }
#pragma unroll
    for (int u = 0; u < kPrologueU; ++u) {
      const int64_t r = r0 + 256 * u;
      if (r >= a.N) break;
      const double v0 = sv0[u], v1 = sv1[u];
      const int64_t q0 = quantize_value(v0, k0), q1 = quantize_value(v1, k1);
      t0 += q0;
      t1 += q1;
      uint2 d;
      d.x = a.np == 1 ? digits1(q0) : digits4(q0);
      d.y = a.np == 1 ? digits1(q1) : digits4(q1);
      reinterpret_cast<uint2*>(a.rowdig)[r] = d;
      if (a.dig16) a.dig16[r] = (uint16_t)((d.x & 0xffu) | ((d.y & 0xffu) << 8));
      if (a.row_node) a.row_node[r] = 0;
      if (a.digp) {
        for (int p = 0; p < a.np; ++p) {
          a.digp[(int64_t)p * a.n_pad + r] = (uint8_t)(d.x >> (8 * p));
          a.digp[(int64_t)(a.np + p) * a.n_pad + r] = (uint8_t)(d.y >> (8 * p));
        }
      }
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    t0 += __shfl_xor(t0, o, kWave);
    t1 += __shfl_xor(t1, o, kWave);
  }
  __shared__ int64_t s_t[2][4];                 // one partial per block (quant_reduce_kernel sums)
  const int w = threadIdx.x / kWave;
  if ((threadIdx.x & (kWave - 1)) == 0) { s_t[0][w] = t0; s_t[1][w] = t1; }
  __syncthreads();
  if (a.zero) prologue_fill(a.zero, a.zero_n, nullptr, nullptr, 0);
  if (threadIdx.x == 0) {
    t0 = s_t[0][0] + s_t[0][1] + s_t[0][2] + s_t[0][3];
    t1 = s_t[1][0] + s_t[1][1] + s_t[1][2] + s_t[1][3];
    if (a.atomic_root) {
      unsigned long long* slot = reinterpret_cast<unsigned long long*>(a.root_parts) + kRootStride * (blockIdx.x % kRootSlots);
      atomicAdd(slot, (unsigned long long)t0);
      atomicAdd(slot + 1, (unsigned long long)t1);
      if (blockIdx.x == 0) {
        if (a.root_open) a.root_open[0] = 0;
        if (a.kexp_copy) { a.kexp_copy[0] = k0; a.kexp_copy[1] = k1; }
      }
    } else {
      part[2 * blockIdx.x] = (unsigned long long)t0;
      part[2 * blockIdx.x + 1] = (unsigned long long)t1;
    }
  }
  if (a.atomic_root && blockIdx.x == 0 && threadIdx.x < kRootSlots) {
    a.root_parts_clear[kRootStride * threadIdx.x] = 0;
    a.root_parts_clear[kRootStride * threadIdx.x + 1] = 0;
  }
  if (a.atomic_root || a.ticket == nullptr || !last_workgroup(a.ticket)) return;
  // the last workgroup: the exact totals, then the tree's root state
  reduce_parts_block<false>(part, (int)gridDim.x, reinterpret_cast<unsigned long long*>(a.totals));
  if (threadIdx.x == 0) {
    const int64_t T0 = a.totals[0], T1 = a.totals[1];
    if (a.root_stats) { a.root_stats[0] = T0; a.root_stats[1] = T1; }
    if (a.root_totals) { a.root_totals[0] = T0; a.root_totals[1] = T1; }
    if (a.root_open) a.root_open[0] = 0;
    if (a.kexp_copy) { a.kexp_copy[0] = k0; a.kexp_copy[1] = k1; }
  }
}
__global__ __launch_bounds__(256) void quant_kernel(QuantArgs a, const double* maxv, unsigned long long* part) { quant_kernel_body(a, maxv, part); }

__global__ __launch_bounds__(256) void slot8_kernel(SlotArgs a) {
  for (int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x; r < a.N; r += (int64_t)gridDim.x * 256) {
    const int32_t node = a.row_node[r];
    const int32_t s = ((node >= 0 && node < a.num_nodes) ? a.node_slot[node] : -1) - a.slot_base;
    const uint32_t sb = (s >= 0 && s < a.nslots) ? (uint32_t)s : 0xffu;
    if (a.slot8) a.slot8[r] = (uint8_t)sb;
    if (a.masked)
      reinterpret_cast<uint2*>(a.masked)[r] = s == 0 ? reinterpret_cast<const uint2*>(a.rowdig)[r] : make_uint2(0u, 0u);
    if (a.pack) {
      const uint2 d = reinterpret_cast<const uint2*>(a.rowdig)[r];
      a.pack[r] = sb | ((d.x & 0xffu) << 8) | ((d.y & 0xffu) << 16);
    }
  }
}

// One lane's 4 consecutive entries of a histogram step: rows (-1 outside the item) and keys.
// Branch-free, so the next steps' loads stay in flight: lanes past the item's end re-read its
// last 4-group (clamped address), and the CSC arrays carry >= 4 readable entries of padding.
// The loaded rows stay raw in the pipeline: invalid entries are set to -1 only where the step is
// consumed (rows()), so no arithmetic on a load sits next to it and forces an early vmcnt wait.
struct RowStep {
  int4 raw;
  uint32_t keys4;
  uint32_t inval;            // bit j: entry j lies outside the item
  __device__ __forceinline__ int4 rows() const {
    return make_int4(raw.x | -(int)(inval & 1u), raw.y | -(int)((inval >> 1) & 1u), raw.z | -(int)((inval >> 2) & 1u),
                     raw.w | -(int)(inval >> 3));
  }
};

__device__ __forceinline__ void load_rows(const HistArgs& a, int64_t e, int64_t e0, int64_t e1, int64_t e_last,
                                          RowStep& d) {
  const int64_t el = e < e_last ? e : e_last;
  d.keys4 = *reinterpret_cast<const uint32_t*>(a.csc_key + el);
  d.raw = *reinterpret_cast<const int4*>(__builtin_assume_aligned(a.csc_row + el, 16));
  const bool v0 = e >= e0 && e < e1, v1 = e + 1 >= e0 && e + 1 < e1;
  const bool v2 = e + 2 >= e0 && e + 2 < e1, v3 = e + 3 >= e0 && e + 3 < e1;
  d.inval = (v0 ? 0u : 1u) | (v1 ? 0u : 2u) | (v2 ? 0u : 4u) | (v3 ? 0u : 8u);
}

// slot byte of each of the 4 entries (0xff: outside the item or not in a node of this pass)
template <bool ROOT, bool PACK = false>
__device__ __forceinline__ uint32_t entry_slots(const HistArgs& a, int4 r4) {
  if constexpr (PACK) {
    // packed row state (np = 1 passes): the slot is byte 0 of the row's word
    const uint32_t s0 = a.rowpack[r4.x >= 0 ? r4.x : 0] & 0xffu;
    const uint32_t s1 = a.rowpack[r4.y >= 0 ? r4.y : 0] & 0xffu;
    const uint32_t s2 = a.rowpack[r4.z >= 0 ? r4.z : 0] & 0xffu;
    const uint32_t s3 = a.rowpack[r4.w >= 0 ? r4.w : 0] & 0xffu;
    const uint32_t dead = (r4.x < 0 ? 0xffu : 0u) | (r4.y < 0 ? 0xff00u : 0u) | (r4.z < 0 ? 0xff0000u : 0u) |
                          (r4.w < 0 ? 0xff000000u : 0u);
    return (s0 | (s1 << 8) | (s2 << 16) | (s3 << 24)) | dead;
  } else if constexpr (ROOT) {
    return (r4.x >= 0 ? 0u : 0xffu) | (r4.y >= 0 ? 0u : 0xff00u) | (r4.z >= 0 ? 0u : 0xff0000u) |
           (r4.w >= 0 ? 0u : 0xff000000u);
  } else {
    const uint32_t s0 = a.slot8[r4.x >= 0 ? r4.x : 0];
    const uint32_t s1 = a.slot8[r4.y >= 0 ? r4.y : 0];
    const uint32_t s2 = a.slot8[r4.z >= 0 ? r4.z : 0];
    const uint32_t s3 = a.slot8[r4.w >= 0 ? r4.w : 0];
    const uint32_t dead = (r4.x < 0 ? 0xffu : 0u) | (r4.y < 0 ? 0xff00u : 0u) | (r4.z < 0 ? 0xff0000u : 0u) |
                          (r4.w < 0 ? 0xff000000u : 0u);
    return (s0 | (s1 << 8) | (s2 << 16) | (s3 << 24)) | dead;
  }
}

// digit words of the live entries among the 4 (0 for dead ones: they never contribute). The loads
// are unconditional (dead entries read row 0, one shared line) so that the compiler can count them
// in vmcnt: a conditional load makes it drain every outstanding load (vmcnt(0)) before the next use,
// which serialised the software pipeline.
__device__ __forceinline__ void gather_digits(const uint2* __restrict__ rd, int4 r4, uint32_t slots4, uint32_t w[8]) {
  const int32_t rr[4] = {r4.x, r4.y, r4.z, r4.w};
  uint2 v[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const bool live = ((slots4 >> (8 * j)) & 0xffu) != 0xffu;
    v[j] = rd[live ? rr[j] : 0];
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint32_t m = ((slots4 >> (8 * j)) & 0xffu) != 0xffu ? 0xffffffffu : 0u;
    w[2 * j] = v[j].x & m;
    w[2 * j + 1] = v[j].y & m;
  }
}

// np = 1 passes over the packed row state (rowpack[r] = slot | digit0 << 8 | digit1 << 16): the
// digits come from the word the slot was read from, one line per entry instead of two (slot byte
// + 8-byte digit words); the second read of the word hits the cache.
template <bool PACK>
__device__ __forceinline__ void gather_entry_digits(const HistArgs& a, const uint2* __restrict__ rd, int4 r4,
                                                    uint32_t slots4, uint32_t w[8]) {
  if constexpr (PACK) {
    const int32_t rr[4] = {r4.x, r4.y, r4.z, r4.w};
    uint32_t v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const bool live = ((slots4 >> (8 * j)) & 0xffu) != 0xffu;
      v[j] = a.rowpack[live ? rr[j] : 0];
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t m = ((slots4 >> (8 * j)) & 0xffu) != 0xffu ? 0xffu : 0u;
      w[2 * j] = (v[j] >> 8) & m;
      w[2 * j + 1] = (v[j] >> 16) & m;
    }
  } else {
    gather_digits(rd, r4, slots4, w);
  }
}

// ------------------------------------------------------------------ i8 MFMA histogram
// One wave per work item; per step the wave takes 256 entries, 4 consecutive ones per lane (rows
// int4, keys u32: single vector loads), with rows/keys of step i+3, slots of step i+2 and digits
// of step i+1 in flight while step i is staged in LDS and multiplied. Every load is unconditional
// (clamped addresses, dead entries read row 0), so the compiler keeps them counted in vmcnt and the
// steps overlap; a conditional load made it drain the queue (vmcnt(0)) every step.
// Tile: v_mfma_i32_16x16x64_i8, lane l: r = l & 15 (A row = key r + 16 bt + koff, B column r),
// g = l >> 4 (entries 16g .. 16g+15 of the K-step); C[key 4g + i][col r] in register i.
// Columns: slot_sub = r / (2 NP) within the tile, q = r % (2 NP) = statistic * NP + plane.
// ROOT: every entry of the item is live in slot 0 (no slot table, no compaction: the lane's 4
// digit words are transposed into plane-major LDS rows in registers). Otherwise the live entries
// (row in a node of this pass) are compacted, and K-steps run on ceil(live / 64) groups.
// Measured and kept out: dword staging of all entries with slot-masked B (0-20 % slower), and
// waves streaming lists of consecutive items through one pipeline (no faster for the ~1K-entry
// text-feature items, slower for the rest).
// (Forcing 4 waves per SIMD on the CT = 8 pass -- 128 registers, 15 spilled -- measured no
// faster than its 3 waves: profiles/r2s4/hist_REJECTED_w4_ab.txt)
template <int BT, int CT, int NP, bool ROOT, bool PACK = false>
__global__ __launch_bounds__(256) void hist_i8_kernel(HistArgs a) {
  constexpr int G = 4 * kWave;                 // entries per wave step
  constexpr int KS = 64;                       // entries per MFMA K-step
  constexpr int CPS = 2 * NP;                  // columns per node slot
  constexpr int SPT = 16 / CPS;                // node slots per 16-column tile
  constexpr int NQ = 2 * NP;                   // staged digit planes
  __shared__ __attribute__((aligned(16))) uint8_t s_key[4][G + KS];
  __shared__ __attribute__((aligned(16))) uint8_t s_slot[4][G + KS];
  __shared__ __attribute__((aligned(16))) uint8_t s_dig[4][NQ][G + KS];

  const int wid = threadIdx.x / kWave;
  const int lane = threadIdx.x & (kWave - 1);
  const int wslot = blockIdx.x * 4 + wid;
  // listed pass (RF): the waves of a fixed grid (a multiple of 8 workgroups) stride over their
  // XCD's compacted list of active items (hist_select_kernel); otherwise one wave per wave slot
  const bool listed = a.active_list != nullptr;
  const int xcd = blockIdx.x & 7;
  const int n_listed = listed ? a.active_count[xcd] : 0;
  const int32_t* xlist = listed ? a.active_list + (int64_t)xcd * a.list_cap : nullptr;
  // (claiming items through an atomic cursor instead: 8192 contended atomics cost ~0.2 ms a pass)
  const int stride = listed ? (int)(gridDim.x >> 3) * 4 : (int)gridDim.x * 4;
  int li = listed ? (int)(blockIdx.x >> 3) * 4 + wid : wslot;
  for (bool once = true;; once = false, li += stride) {
  int item;
  if (listed) {
    if (li >= n_listed) break;
    item = xlist[li];
  } else {
    if (!once) break;
    item = a.wave_item ? a.wave_item[wslot] : wslot;
    if (item < 0 || item >= a.num_items) break;
    if (!item_active(a, item)) break;          // RF: no feature of the item is sampled at this level
  }
  const int64_t e0 = a.item_start[item], e1 = a.item_end[item];
  const int32_t meta = a.item_meta[item];
  const int32_t f0 = a.item_f0[item];
  const uint32_t koff = (uint32_t)item_koff(meta);
  // every key of the item's entries is < 128 (packed items: < 64; single features: < nbins)
  const bool fast7 = item_nfeat(meta) > 1 || a.nbins[f0] <= 128;

  const int r = lane & 15, g = lane >> 4;
  const int slot_sub = r / CPS, q = r % CPS;
  i32x4 acc[BT][CT];
#pragma unroll
  for (int bt = 0; bt < BT; ++bt)
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) acc[bt][ct] = i32x4{0, 0, 0, 0};

  const int64_t first = e0 & ~(int64_t)3;
  const int64_t e_last = (e1 - 1) & ~(int64_t)3;   // last 4-group holding an entry of the item
  const uint2* rd = reinterpret_cast<const uint2*>(a.rowdig);
  RowStep g1, g2;
  uint32_t sl0, sl1, keys0, w0[8];
  {
    RowStep g0;
    load_rows(a, first + 4 * lane, e0, e1, e_last, g0);
    load_rows(a, first + G + 4 * lane, e0, e1, e_last, g1);
    sl0 = entry_slots<ROOT, PACK>(a, g0.rows());
    keys0 = g0.keys4;
    sl1 = entry_slots<ROOT, PACK>(a, g1.rows());
    gather_entry_digits<PACK>(a, rd, g0.rows(), sl0, w0);
    load_rows(a, first + 2 * G + 4 * lane, e0, e1, e_last, g2);
  }
  for (int64_t base = first; base < e1; base += G) {
    const uint32_t slots4 = sl0, keys4 = keys0;
    uint32_t w[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) w[j] = w0[j];
    // digits of step i+1, slots of step i+2, rows of step i+3 (clamped, so unconditional)
    gather_entry_digits<PACK>(a, rd, g1.rows(), sl1, w0);
    const uint32_t sl2 = entry_slots<ROOT, PACK>(a, g2.rows());
    RowStep g3;
    load_rows(a, base + 3 * G + 4 * lane, e0, e1, e_last, g3);
    sl0 = sl1;
    keys0 = g1.keys4;
    sl1 = sl2;
    g1 = g2;
    g2 = g3;

    int n_live = G;
    if constexpr (ROOT) {
      // plane-major rows: s_dig[stat * NP + p][4 lane + j] = digit p of statistic stat of entry j
      *reinterpret_cast<uint32_t*>(&s_key[wid][4 * lane]) = keys4;
#pragma unroll
      for (int st = 0; st < 2; ++st)
#pragma unroll
        for (int p = 0; p < NP; ++p)
          *reinterpret_cast<uint32_t*>(&s_dig[wid][st * NP + p][4 * lane]) =
              gather_byte(w[st], w[2 + st], w[4 + st], w[6 + st], (uint32_t)p);
    } else {
      int nb = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t sj = (slots4 >> (8 * j)) & 0xffu;
        const unsigned long long bj = __ballot(sj != 0xffu);
        if (sj != 0xffu) {
          const int pos = nb + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bj >> 32),
                                                              __builtin_amdgcn_mbcnt_lo((uint32_t)bj, 0u));
          s_key[wid][pos] = (uint8_t)(keys4 >> (8 * j));
          s_slot[wid][pos] = (uint8_t)sj;
#pragma unroll
          for (int st = 0; st < 2; ++st)
#pragma unroll
            for (int p = 0; p < NP; ++p) s_dig[wid][st * NP + p][pos] = (uint8_t)(w[2 * j + st] >> (8 * p));
        }
        nb += __popcll(bj);
      }
      n_live = nb;
      // pad the last partial K-step: slot 0xff matches no column, so stale digits drop out
      s_slot[wid][nb + lane] = 0xffu;
    }
    lds_sync();
    // K-steps over the live entries only. CT >= 4: a rolled loop (one exit), because breaking
    // out of the unrolled one made the compiler copy all CT * 4 accumulators between AGPRs and
    // VGPRs at each exit (32 extra VGPRs at CT = 8: 2 instead of 3 waves per SIMD)
    const int nks = (n_live + KS - 1) / KS;
    constexpr int KUNROLL = CT >= 4 ? 1 : G / KS;
#pragma unroll KUNROLL
    for (int ks = 0; ks < nks; ++ks) {
      const int k0 = ks * KS + 16 * g;
      const uint4 kv = *reinterpret_cast<const uint4*>(&s_key[wid][k0]);
      const uint4 dv = *reinterpret_cast<const uint4*>(&s_dig[wid][q][k0]);
      i32x4 A[BT];
      onehot_a<BT>(kv, (uint32_t)r + koff, fast7, A);
      if constexpr (ROOT) {
        const i32x4 B = {(int)dv.x, (int)dv.y, (int)dv.z, (int)dv.w};
#pragma unroll
        for (int bt = 0; bt < BT; ++bt) acc[bt][0] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[bt], B, acc[bt][0], 0, 0, 0);
      } else {
        const uint4 sv = *reinterpret_cast<const uint4*>(&s_slot[wid][k0]);
        if constexpr (NP == 4) {
          // B of one column tile at a time (the parity-masked digits and the tile selectors stay
          // live, not CT built operands: CT = 8 needed 32 more VGPRs and ran at 2 waves per SIMD)
          const uint32_t pat = (0x80u | (uint32_t)(slot_sub ^ 1)) * 0x01010101u;
          const uint4 dm = make_uint4(dv.x & live_parity_mask(sv.x, pat), dv.y & live_parity_mask(sv.y, pat),
                                      dv.z & live_parity_mask(sv.z, pat), dv.w & live_parity_mask(sv.w, pat));
          const uint4 sel = make_uint4((sv.x >> 1) & 0x07070707u, (sv.y >> 1) & 0x07070707u,
                                       (sv.z >> 1) & 0x07070707u, (sv.w >> 1) & 0x07070707u);
#pragma unroll
          for (int ct = 0; ct < CT; ++ct) {
            const i32x4 B = {(int)(dm.x & ct_select(sel.x, ct)), (int)(dm.y & ct_select(sel.y, ct)),
                             (int)(dm.z & ct_select(sel.z, ct)), (int)(dm.w & ct_select(sel.w, ct))};
#pragma unroll
            for (int bt = 0; bt < BT; ++bt)
              acc[bt][ct] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[bt], B, acc[bt][ct], 0, 0, 0);
          }
        } else {
          i32x4 B[CT];
          slot_masked_b<CT, NP>(dv, sv, slot_sub, B);
#pragma unroll
          for (int ct = 0; ct < CT; ++ct)
#pragma unroll
            for (int bt = 0; bt < BT; ++bt)
              acc[bt][ct] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[bt], B[ct], acc[bt][ct], 0, 0, 0);
        }
      }
    }
    lds_sync();
  }

  // Epilogue: C = -128 * (plane sum); lanes r .. r+NP-1 hold the NP planes of one (slot, stat)
  // column: the plane-0 lane recombines them into int64 and adds the nonzero sums to the
  // histogram. The bin offset of each of the lane's key rows is loaded first, all at once (clamped
  // indices), so no atomic waits on a dependent load. (A padded bin layout with one offset per item
  // would depend on each rank's local packing and break the data-parallel histogram shapes.)
  // histogram row of each column tile's slot (-1: none), loaded here rather than kept live
  // through the main loop (8 registers at CT = 8)
  int node_of[CT];
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) {
    const int slot = ct * SPT + slot_sub;
    const int n = a.slot_node[slot < a.nslots ? slot : a.nslots - 1];
    node_of[ct] = slot < a.nslots ? n : -1;
  }
  const int sl2 = item_stride_log2(meta), nfeat = item_nfeat(meta);
  int64_t bin_of[BT][4];
#pragma unroll
  for (int bt = 0; bt < BT; ++bt)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int ek = 16 * bt + 4 * g + i + (int)koff;
      const int fl = ek >> sl2, b = ek & ((1 << sl2) - 1);
      const int f = f0 + (fl < nfeat ? fl : 0);
      const int nb = a.nbins[f];
      const int64_t bo = hist_boff(a, f);
      bin_of[bt][i] = (fl < nfeat && b < nb) ? bo + b : -1;
    }
  const int stat = q / NP;
#pragma unroll
  for (int bt = 0; bt < BT; ++bt)
#pragma unroll
    for (int ct = 0; ct < CT; ++ct)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int32_t s = -(acc[bt][ct][i] >> 7);
        int64_t v = s;
        if constexpr (NP == 4) {
          const int32_t s1 = __shfl_down(s, 1, kWave), s2 = __shfl_down(s, 2, kWave), s3 = __shfl_down(s, 3, kWave);
          v = (int64_t)s + (int64_t)s1 * 256 + (int64_t)s2 * 65536 + (int64_t)s3 * 16777216;
        }
        if ((q % NP) == 0 && v != 0 && node_of[ct] >= 0 && bin_of[bt][i] >= 0) {
          int64_t* dst = a.hist + ((int64_t)node_of[ct] * a.hist_stride + bin_of[bt][i]) * 2 + stat;
          atomicAdd(reinterpret_cast<unsigned long long*>(dst), (unsigned long long)v);
        }
      }
  }  // items of the wave
}

// ------------------------------------------------------------------ LDS-atomic count histogram
// np = 1 passes (DT / RF class counts, |digit| <= 127): the i8 MFMA kernel's one-hot tiles and
// live-entry compaction cost ~100 instructions per 64 entries for one (slot, key) update each,
// ~25 G entries/s over a 500-tree forest. Here a wave per item keeps an LDS table of packed
// counts [16 BT keys][nslots] (q0 + q1 * 2^32 in one int64: the exact sums stay below 2^31 in
// magnitude -- an item has <= 2^15 entries -- so both halves decode exactly) and every live entry
// is ONE ds_add_u64. The entry pipeline (rows / keys 4 per lane, slots and count words one and
// two steps ahead) is the MFMA kernel's; the table is flushed per item with integer atomics.
template <int BT, bool PACK>
__device__ __forceinline__ void hist_lds_kernel_body(HistArgs a) {
  constexpr int G = 4 * kWave;
  constexpr int KEYS = 16 * BT;
  extern __shared__ unsigned long long s_tab[];          // [4 waves][KEYS * nslots]
  const int wid = threadIdx.x / kWave;
  const int lane = threadIdx.x & (kWave - 1);
  const int wslot = blockIdx.x * 4 + wid;
  const int ns = a.nslots;
  const int cells = KEYS * ns;
  unsigned long long* tab = s_tab + (int64_t)wid * cells;
  const bool listed = a.active_list != nullptr;
  const int xcd = blockIdx.x & 7;
  const int n_listed = listed ? a.active_count[xcd] : 0;
  const int32_t* xlist = listed ? a.active_list + (int64_t)xcd * a.list_cap : nullptr;
  const int stride = listed ? (int)(gridDim.x >> 3) * 4 : (int)gridDim.x * 4;
  const uint2* rd = reinterpret_cast<const uint2*>(a.rowdig);
  int li = listed ? (int)(blockIdx.x >> 3) * 4 + wid : wslot;
  for (bool once = true;; once = false, li += stride) {
    int item;
    if (listed) {
      if (li >= n_listed) break;
      item = xlist[li];
    } else {
      if (!once) break;
      item = a.wave_item ? a.wave_item[wslot] : wslot;
      if (item < 0 || item >= a.num_items) break;
      if (!item_active(a, item)) break;
    }
    const int64_t e0 = a.item_start[item], e1 = a.item_end[item];
    const int32_t meta = a.item_meta[item];
    const int32_t f0 = a.item_f0[item];
    const uint32_t koff = (uint32_t)item_koff(meta);
    // keys of the item's sampled features (lane k tests key koff + k): a packed item is active
    // when ANY of its features is, and its other features' entries (typically most of them at
    // k = sqrt(F)) are skipped instead of counted and flushed into bins nobody reads
    uint64_t amask = ~0ull;
    if (a.feat_active != nullptr && item_nfeat(meta) > 1) {
      const int fl = ((int)koff + lane) >> item_stride_log2(meta);
      amask = __ballot(lane < KEYS && fl < item_nfeat(meta) && a.feat_active[f0 + fl] != 0);
    }
    for (int i = lane; i < cells; i += kWave) tab[i] = 0ull;
    __builtin_amdgcn_wave_barrier();
    const int64_t first = e0 & ~(int64_t)3;
    const int64_t e_last = (e1 - 1) & ~(int64_t)3;
    RowStep g1, g2;
    uint32_t sl0, sl1, keys0, w0[8];
    {
      RowStep g0;
      load_rows(a, first + 4 * lane, e0, e1, e_last, g0);
      load_rows(a, first + G + 4 * lane, e0, e1, e_last, g1);
      sl0 = entry_slots<!PACK, PACK>(a, g0.rows());
      keys0 = g0.keys4;
      sl1 = entry_slots<!PACK, PACK>(a, g1.rows());
      gather_entry_digits<PACK>(a, rd, g0.rows(), sl0, w0);
      load_rows(a, first + 2 * G + 4 * lane, e0, e1, e_last, g2);
    }
    for (int64_t base = first; base < e1; base += G) {
      const uint32_t slots4 = sl0, keys4 = keys0;
      uint32_t w[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) w[j] = w0[j];
      gather_entry_digits<PACK>(a, rd, g1.rows(), sl1, w0);
      const uint32_t sl2 = entry_slots<!PACK, PACK>(a, g2.rows());
      RowStep g3;
      load_rows(a, base + 3 * G + 4 * lane, e0, e1, e_last, g3);
      sl0 = sl1;
      keys0 = g1.keys4;
      sl1 = sl2;
      g1 = g2;
      g2 = g3;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t s = (slots4 >> (8 * j)) & 0xffu;
        const uint32_t kk = ((keys4 >> (8 * j)) & 0xffu) - koff;     // (unsigned: keys below koff wrap)
        const int64_t q0 = (int64_t)(int8_t)(uint8_t)(w[2 * j] & 0xffu);
        const int64_t q1 = (int64_t)(int8_t)(uint8_t)(w[2 * j + 1] & 0xffu);
        if (s < (uint32_t)ns && kk < (uint32_t)KEYS && (q0 | q1) != 0 && ((amask >> kk) & 1ull))
          atomicAdd(&tab[kk * ns + s], (unsigned long long)(q0 + q1 * 4294967296ll));
      }
    }
    __builtin_amdgcn_wave_barrier();
    // flush: (key, slot) cells with counts -> the level histogram (decode the two halves)
    const int sl2 = item_stride_log2(meta), nfeat = item_nfeat(meta);
    for (int i = lane; i < cells; i += kWave) {
      const int64_t v = (int64_t)tab[i];
      if (v == 0) continue;
      const int kk = i / ns, s = i - kk * ns;
      const int key = (int)koff + kk;
      const int fl = key >> sl2, b = key & ((1 << sl2) - 1);
      if (fl >= nfeat) continue;
      const int f = f0 + fl;
      const int node = a.slot_node[s];
      if (b >= a.nbins[f] || node < 0) continue;
      const int64_t lo = (int64_t)(int32_t)(uint32_t)(uint64_t)v;
      const int64_t hi = (v - lo) >> 32;
      unsigned long long* dst = reinterpret_cast<unsigned long long*>(a.hist + ((int64_t)node * a.hist_stride + hist_boff(a, f) + b) * 2);
      if (lo) atomicAdd(dst, (unsigned long long)lo);
      if (hi) atomicAdd(dst + 1, (unsigned long long)hi);
    }
    __builtin_amdgcn_wave_barrier();               // the table is zeroed for the next item
  }
}
template <int BT, bool PACK>
__global__ __launch_bounds__(256) void hist_lds_kernel(HistArgs a) { hist_lds_kernel_body<BT, PACK>(a); }

// Compacted per-XCD lists of the active work items of a listed pass. A workgroup takes
// kSelPerThread x 256 consecutive wave slots (coalesced reads), places its active items in LDS
// order per XCD (LDS atomics), then reserves its runs of the 8 global lists with ONE global atomic
// per XCD: a wave-level global atomic per XCD (the earlier version) put ~40K atomics on the same 8
// counters per pass, ~40 us a launch. The order inside a list is free (integer histograms).
constexpr int kSelPerThread = 16;

__device__ __forceinline__ void hist_select_kernel_body(HistArgs a, int32_t* list, int32_t* count) {
  __shared__ int32_t s_cnt[8], s_base[8];
  const int t = threadIdx.x;
  if (t < 8) s_cnt[t] = 0;
  __syncthreads();
  const int64_t w0 = (int64_t)blockIdx.x * 256 * kSelPerThread;
  int32_t item[kSelPerThread], loc[kSelPerThread];
#pragma unroll
  for (int j = 0; j < kSelPerThread; ++j) {
    const int64_t w = w0 + (int64_t)j * 256 + t;
    int it = -1;
    if (w < a.num_slots) it = a.wave_item ? a.wave_item[w] : (int)w;
    const bool act = it >= 0 && it < a.num_items && item_active(a, it);
    item[j] = it;
    // the XCD the item's wave slot was placed on (wave_order: workgroup b = slot / 4 on XCD b % 8):
    // each XCD's waves of the listed pass take that XCD's items, so a row block's slot and count
    // words stay in the L2 they were placed for
    loc[j] = act ? atomicAdd(&s_cnt[(w >> 2) & 7], 1) : -1;
  }
  __syncthreads();
  if (t < 8) s_base[t] = s_cnt[t] ? atomicAdd(count + t, s_cnt[t]) : 0;
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kSelPerThread; ++j)
    if (loc[j] >= 0) {
      const int x = (int)(((w0 + (int64_t)j * 256 + t) >> 2) & 7);
      list[(int64_t)x * a.list_cap + s_base[x] + loc[j]] = item[j];
    }
}
__global__ __launch_bounds__(256) void hist_select_kernel(HistArgs a, int32_t* list, int32_t* count) { hist_select_kernel_body(a, list, count); }

// ------------------------------------------------------------------ dense i8 MFMA histogram
// Same tile as hist_i8_kernel; the K dimension runs over 64 consecutive rows, so the row state
// (digit planes, slot bytes) is streamed once per K-step and shared by the FG features of the
// wave. The FG x 64 bin bytes of a K-step arrive by ONE coalesced 16-byte load per lane (lane l:
// feature l / 4, rows 16 (l & 3) ..), are staged in a per-wave double-buffered LDS tile and read
// back as MFMA A fragments (16 lanes of a k-group share one 16-byte row: LDS broadcast). No
// compaction: dead rows (slot 0xff) are masked out of B. Loads run two K-steps ahead.
template <int BT, int CT, int NP, bool ROOT, int FG>
__global__ __launch_bounds__(256) void hist_dense_kernel(DenseHistArgs a) {
  constexpr int CPS = 2 * NP, SPT = 16 / CPS;
  static_assert(FG <= 16, "one 16-byte load per lane covers at most 16 features x 64 rows");
  __shared__ __attribute__((aligned(16))) uint8_t s_bins[4][2][FG][64];
  const int wid = threadIdx.x / kWave;
  const int lane = threadIdx.x & (kWave - 1);
  // XCD-aware placement: workgroups b and b + 8 share an L2 (observed round-robin dispatch,
  // speed only): XCD label x = b % 8 walks ranges x, x + 8, ... and all groups of a range.
  const int x = blockIdx.x & 7;
  const int k = (int)(blockIdx.x >> 3) * 4 + wid;
  const int grp = k % a.ngroups;
  const int range = x + 8 * (k / a.ngroups);
  if (range >= a.nranges) return;
  const int64_t r0 = (int64_t)range * a.range_rows;
  const int64_t r1 = r0 + a.range_rows < a.n_pad ? r0 + a.range_rows : a.n_pad;
  const int r = lane & 15, g = lane >> 4;
  const int slot_sub = r / CPS, q = r % CPS;
  int fid[FG];
#pragma unroll
  for (int j = 0; j < FG; ++j) fid[j] = a.gfid[grp * FG + j];
  // loader lane: feature lj = lane / 4 (if < FG), rows 16 * (lane & 3) .. + 15 of the K-step
  const int lj = lane >> 2;
  const bool loader = lj < FG && a.gfid[grp * FG + (lj < FG ? lj : 0)] >= 0;
  const uint8_t* lcol = a.dense + (int64_t)(loader ? a.gdense[grp * FG + lj] : 0) * a.n_pad + 16 * (lane & 3);
  const uint8_t* dig = a.digp + (int64_t)q * a.n_pad + 16 * g;
  const uint8_t* slt = a.slot8 + 16 * g;

  i32x4 acc[FG][BT][CT];
#pragma unroll
  for (int j = 0; j < FG; ++j)
#pragma unroll
    for (int bt = 0; bt < BT; ++bt)
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) acc[j][bt][ct] = i32x4{0, 0, 0, 0};

  // two K-steps of loads in flight: (bins, digits, slots) of steps i+1 and i+2. Unconditional
  // loads from clamped addresses (steps past the range re-read its last step, non-loader lanes read
  // column 0), so the compiler counts them in vmcnt instead of draining the queue every step.
  uint4 lb1 = make_uint4(0, 0, 0, 0), lb2 = lb1, d1 = lb1, d2 = lb1, s1 = lb1, s2 = lb1;
  const int64_t last = r1 - 64;
  auto load = [&](int64_t base, uint4& lb, uint4& d, uint4& sv) {
    const int64_t bc = base < last ? base : last;
    lb = *reinterpret_cast<const uint4*>(lcol + bc);
    d = *reinterpret_cast<const uint4*>(dig + bc);
    if constexpr (!ROOT) sv = *reinterpret_cast<const uint4*>(slt + bc);
  };
  uint4 lb0 = lb1, d0 = lb1, s0 = lb1;
  load(r0, lb0, d0, s0);
  load(r0 + 64, lb1, d1, s1);
  if (lj < FG) *reinterpret_cast<uint4*>(&s_bins[wid][0][lj][16 * (lane & 3)]) = lb0;
  int buf = 0;
  for (int64_t base = r0; base < r1; base += 64) {
    load(base + 128, lb2, d2, s2);
    lds_sync();                                             // bins of this step staged
    i32x4 B[CT];
    if constexpr (ROOT) B[0] = i32x4{(int)d0.x, (int)d0.y, (int)d0.z, (int)d0.w};
    else slot_masked_b<CT, NP>(d0, s0, slot_sub, B);
#pragma unroll
    for (int j = 0; j < FG; ++j) {
      if (fid[j] < 0) continue;
      // hot features have <= 64 bins, so every bin byte is < 64: the 2-VALU one-hot, unmasked
      const uint4 kv = *reinterpret_cast<const uint4*>(&s_bins[wid][buf][j][16 * g]);
#pragma unroll
      for (int bt = 0; bt < BT; ++bt) {
        const uint32_t nk = ~((uint32_t)(r + 16 * bt) * 0x01010101u);
        const i32x4 A = {(int)onehot7(kv.x, nk), (int)onehot7(kv.y, nk), (int)onehot7(kv.z, nk), (int)onehot7(kv.w, nk)};
#pragma unroll
        for (int ct = 0; ct < CT; ++ct)
          acc[j][bt][ct] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A, B[ct], acc[j][bt][ct], 0, 0, 0);
      }
    }
    // stage the next step's bins into the other buffer (read two steps from now)
    if (lj < FG) *reinterpret_cast<uint4*>(&s_bins[wid][buf ^ 1][lj][16 * (lane & 3)]) = lb1;
    buf ^= 1;
    lb1 = lb2;
    d0 = d1;
    d1 = d2;
    s0 = s1;
    s1 = s2;
  }

  // destinations first (independent loads), then the atomics
  const int stat = q / NP;
  int node_of[CT];
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) {
    const int slot = ct * SPT + slot_sub;
    const int n = a.slot_node[slot < a.nslots ? slot : a.nslots - 1];
    node_of[ct] = slot < a.nslots ? n : -1;
  }
  int nb_of[FG];
  int64_t bo_of[FG];
#pragma unroll
  for (int j = 0; j < FG; ++j) {
    const int f = fid[j] >= 0 ? fid[j] : 0;
    nb_of[j] = fid[j] >= 0 ? a.nbins[f] : 0;
    bo_of[j] = a.boff[f];
  }
#pragma unroll
  for (int j = 0; j < FG; ++j)
#pragma unroll
    for (int bt = 0; bt < BT; ++bt)
#pragma unroll
      for (int ct = 0; ct < CT; ++ct)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int32_t s = -(acc[j][bt][ct][i] >> 7);
          int64_t v = s;
          if constexpr (NP == 4) {
            const int32_t t1 = __shfl_down(s, 1, kWave), t2 = __shfl_down(s, 2, kWave), t3 = __shfl_down(s, 3, kWave);
            v = (int64_t)s + (int64_t)t1 * 256 + (int64_t)t2 * 65536 + (int64_t)t3 * 16777216;
          }
          const int b = 16 * bt + 4 * g + i;
          if ((q % NP) != 0 || v == 0 || node_of[ct] < 0 || b >= nb_of[j]) continue;
          int64_t* dst = a.hist + ((int64_t)node_of[ct] * a.hist_stride + bo_of[j] + b) * 2 + stat;
          atomicAdd(reinterpret_cast<unsigned long long*>(dst), (unsigned long long)v);
        }
}

// ------------------------------------------------------------------ sibling subtraction
// grid.y = pair (node triple), grid.x strides the pair's 2 TB int64 sums with 16-byte accesses:
// no per-element 64-bit div/mod. A padded triple (dst < 0, device level loop) exits at once.
__global__ __launch_bounds__(256) void hist_subtract_kernel(const int64_t* parent_hist, int64_t* cur_hist,
                                                            const int32_t* dst, const int32_t* par,
                                                            const int32_t* sib, int32_t n_pairs, int64_t TB) {
  const int p = blockIdx.y;
  const int32_t d = dst[p];
  if (d < 0) return;
  const int64_t per = TB;                     // (g, h) pairs = 16 B each
  const longlong2* src = reinterpret_cast<const longlong2*>(parent_hist) + (int64_t)par[p] * per;
  const longlong2* sb = reinterpret_cast<const longlong2*>(cur_hist) + (int64_t)sib[p] * per;
  longlong2* out = reinterpret_cast<longlong2*>(cur_hist) + (int64_t)d * per;
  for (int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x; k < per; k += (int64_t)gridDim.x * 256) {
    const longlong2 a = src[k], b = sb[k];
    out[k] = make_longlong2(a.x - b.x, a.y - b.y);
  }
}

// ------------------------------------------------------------------ split search
// node n's exact sums (level 0 of the fused prologue: from the quantisation's slots)
// feature_priority of (node n, feature f) as a double (fmix: mix64 of the original feature id looked up)
__device__ __forceinline__ double split_priority(const SplitArgs& a, int n, int f) {
  const int32_t tree = a.node_tree ? a.node_tree[n] : a.tree;
  if (a.fmix == nullptr) return feature_priority(a.seed, tree, a.node_ids[n], a.fid_orig[f]);
  return (double)feature_priority_u53_pre(a.seed, tree, a.node_ids[n], a.fmix[a.fid_orig[f]]) * (1.0 / 9007199254740992.0);
}

__device__ __forceinline__ void split_totals(const SplitArgs& a, int n, int64_t* t0, int64_t* t1) {
  if (a.root_parts) {
    root_sums(a.root_parts, t0, t1);
  } else {
    *t0 = a.totals[2 * n];
    *t1 = a.totals[2 * n + 1];
  }
}

// Returns the feature's gain; -inf with *fo = INT32_MAX when t holds no narrow feature.
__device__ __forceinline__ double split_narrow_at(const SplitArgs& a, int64_t t, int* fo) {
  *fo = INT32_MAX;
  if (t >= (int64_t)a.num_nodes * a.Fa) return -1.0 / 0.0;
  const int n = (int)(t / a.Fa), f = (int)(t % a.Fa);
  if (a.wide != nullptr && a.nbins[f] > kSplitWide) return -1.0 / 0.0;     // split_wide_kernel's
  double gain = -1.0 / 0.0;
  int bin = -1;
  int64_t l0 = 0, l1 = 0;
  bool use = a.node_ids[n] >= 0;              // -1: padded row of a device level loop
  if (use && a.feat_thr)
    use = split_priority(a, n, f) <= a.feat_thr[n];
  if (use) {
    const int64_t stride = a.hist_stride ? a.hist_stride : a.boff[a.Fa];
    const int64_t* hb = a.hist + (split_row(a, n) * stride + a.boff[f]) * 2;
    const int32_t k = a.sub_of ? a.sub_of[n] : -1;
    if (k >= 0) {            // the sibling subtraction of (n, f), written to row n (then read back)
      const int64_t* pb = a.parent_hist + ((int64_t)a.sub_par[k] * stride + a.boff[f]) * 2;
      const int64_t* sb = a.hist + ((int64_t)a.sub_sib[k] * stride + a.boff[f]) * 2;
      int64_t* ob = const_cast<int64_t*>(hb);
      for (int b = 0; b < 2 * a.nbins[f]; ++b) ob[b] = pb[b] - sb[b];
    }
    int64_t T0, T1;
    split_totals(a, n, &T0, &T1);
    gain = best_split_scan(hb, a.nbins[f], a.zbin[f], T0, T1, ldexp(1.0, -a.kexp[0]),
                           ldexp(1.0, -a.kexp[1]), a.mode, a.lambda_, a.min_child_weight, &bin, &l0, &l1);
  }
  a.out_gain[t] = gain;
  a.out_bin[t] = bin;
  a.out_left[2 * t] = l0;
  a.out_left[2 * t + 1] = l1;
  *fo = f;
  return gain;
}

// (gain, feature) order of the best split: the larger gain, ties to the lower feature; a NaN
// anywhere is sticky (split_best_node makes the node's gain NaN)
__device__ __forceinline__ void best_merge(double& g, int& f, double og, int of) {
  if (g != g || og != og) { g = __longlong_as_double(0x7ff8000000000000ll); return; }
  if (og > g || (og == g && of < f)) { g = og; f = of; }
}

// This wave's partials (SplitArgs part_gain / part_f, indexed by global wave t / 64): segment 0
// = the node of its first lane, segment 1 = a later node (Fa >= 64: at most one). Shuffles only:
// no barrier, so a wave whose scans end early leaves at once.
__device__ __forceinline__ void split_wave_partial(const SplitArgs& a, int64_t t, double gain, int f) {
  const int64_t tw = t & ~(int64_t)(kWave - 1);
  const int nf = (int)(tw / a.Fa);
  const bool in = t < (int64_t)a.num_nodes * a.Fa;
  const int seg = in && (int)(t / a.Fa) != nf ? 1 : 0;
  double g0 = -1.0 / 0.0, g1 = -1.0 / 0.0;
  int f0 = INT32_MAX, f1 = INT32_MAX;
  if (in && seg == 0) { g0 = gain; f0 = f; }
  if (in && seg == 1) { g1 = gain; f1 = f; }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    best_merge(g0, f0, __shfl_xor(g0, o, kWave), __shfl_xor(f0, o, kWave));
    best_merge(g1, f1, __shfl_xor(g1, o, kWave), __shfl_xor(f1, o, kWave));
  }
  const int lane = (int)(t & (kWave - 1));
  const int64_t w = tw / kWave;
  if (lane == 0) { a.part_gain[2 * w] = g0; a.part_f[2 * w] = f0; }
  if (lane == 1) { a.part_gain[2 * w + 1] = g1; a.part_f[2 * w + 1] = f1; }
}

__global__ __launch_bounds__(256) void split_kernel(SplitArgs a) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  int f;
  const double g = split_narrow_at(a, t, &f);
  if (a.part_gain) split_wave_partial(a, t, g, f);
}

// Wide features (> kSplitWide bins: the hot words' count bins): a wave per (node, feature), lane
// b on bin b (64-bin chunks with a carry), the stored-bin total and the left prefix sums by wave
// reductions / scans of the exact int64 sums, the gain of every candidate bin at once, and the
// best = the largest gain at the lowest bin (NaN never wins): best_split_scan's result, without
// the one thread walking ~56 bins twice while its wave's other lanes idle (~30 us at the root of
// 10M rows for 145 hot features).
__device__ __forceinline__ int64_t wave_sum_i64(int64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ int64_t wave_incl_scan_i64(int64_t v, int lane) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int64_t o = __shfl_up(v, d, 64);
    if (lane >= d) v += o;
  }
  return v;
}

__device__ __forceinline__ void split_wide_at(const SplitArgs& a, int64_t w, int lane) {
  if (w >= (int64_t)a.num_nodes * a.n_wide) return;                 // (wave-uniform)
  const int n = (int)(w / a.n_wide), f = a.wide[w % a.n_wide];
  const int64_t t = (int64_t)n * a.Fa + f;
  bool use = a.node_ids[n] >= 0;
  if (use && a.feat_thr)
    use = split_priority(a, n, f) <= a.feat_thr[n];
  double best = -1.0 / 0.0;
  int best_b = -1;
  int64_t bl0 = 0, bl1 = 0;
  if (use) {
    const int64_t stride = a.hist_stride ? a.hist_stride : a.boff[a.Fa];
    const int64_t* hb = a.hist + (split_row(a, n) * stride + a.boff[f]) * 2;
    const int nb = a.nbins[f], zb = a.zbin[f];
    const int32_t ks = a.sub_of ? a.sub_of[n] : -1;
    if (ks >= 0) {           // the sibling subtraction of (n, f): lane b writes bins b, b + 64, ...
      const int64_t* pb = a.parent_hist + ((int64_t)a.sub_par[ks] * stride + a.boff[f]) * 2;
      const int64_t* sb = a.hist + ((int64_t)a.sub_sib[ks] * stride + a.boff[f]) * 2;
      int64_t* ob = const_cast<int64_t*>(hb);
      for (int b = lane; b < nb; b += 64) {
        ob[2 * b] = pb[2 * b] - sb[2 * b];
        ob[2 * b + 1] = pb[2 * b + 1] - sb[2 * b + 1];
      }
      __threadfence_block();
      __builtin_amdgcn_wave_barrier();
    }
    int64_t T0, T1;
    split_totals(a, n, &T0, &T1);
    const double s0 = ldexp(1.0, -a.kexp[0]), s1 = ldexp(1.0, -a.kexp[1]);
    int64_t a0 = 0, a1 = 0;
    for (int b0 = 0; b0 < nb; b0 += 64) {
      const int b = b0 + lane;
      if (b < nb && b != zb) { a0 += hb[2 * b]; a1 += hb[2 * b + 1]; }
    }
    a0 = wave_sum_i64(a0);
    a1 = wave_sum_i64(a1);
    const int64_t z0 = T0 - a0, z1 = T1 - a1;
    const double parent = split_parent(a.mode, T0, T1, s0, s1, a.lambda_);
    int64_t c0 = 0, c1 = 0;                                          // carry of the earlier chunks
    for (int b0 = 0; b0 + 1 < nb; b0 += 64) {
      const int b = b0 + lane;
      int64_t v0 = 0, v1 = 0;
      if (b < nb) {
        v0 = (b == zb) ? z0 : hb[2 * b];
        v1 = (b == zb) ? z1 : hb[2 * b + 1];
      }
      const int64_t l0 = c0 + wave_incl_scan_i64(v0, lane), l1 = c1 + wave_incl_scan_i64(v1, lane);
      double gain;
      if (b + 1 < nb && split_gain_at(a.mode, l0, l1, T0, T1, s0, s1, parent, a.lambda_, a.min_child_weight, &gain) &&
          gain > best) {                                             // (within a lane: b increases)
        best = gain; best_b = b; bl0 = l0; bl1 = l1;
      }
      c0 = __shfl(l0, 63, 64);
      c1 = __shfl(l1, 63, 64);
    }
    // the largest gain, ties to the lowest bin (lanes without a candidate hold -inf, bin -1)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const double og = __shfl_xor(best, o, 64);
      const int ob = __shfl_xor(best_b, o, 64);
      const int64_t o0 = __shfl_xor(bl0, o, 64), o1 = __shfl_xor(bl1, o, 64);
      if (ob >= 0 && (best_b < 0 || og > best || (og == best && ob < best_b))) {
        best = og; best_b = ob; bl0 = o0; bl1 = o1;
      }
    }
  }
  if (lane == 0) {
    a.out_gain[t] = best;
    a.out_bin[t] = best_b;
    a.out_left[2 * t] = bl0;
    a.out_left[2 * t + 1] = bl1;
  }
}

__global__ __launch_bounds__(256) void split_wide_kernel(SplitArgs a) {
  split_wide_at(a, ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6, threadIdx.x & 63);
}

// split_kernel and split_wide_kernel in one launch: workgroups [0, nb_narrow) search the narrow
// features (a thread per (node, feature)), the rest the wide ones (a wave per (node, feature))
__device__ __forceinline__ void split_all_kernel_body(SplitArgs a, unsigned nb_narrow) {
  if (blockIdx.x < nb_narrow) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    int f;
    const double g = split_narrow_at(a, t, &f);
    if (a.part_gain) split_wave_partial(a, t, g, f);
  } else {
    split_wide_at(a, ((int64_t)(blockIdx.x - nb_narrow) * 256 + threadIdx.x) >> 6, threadIdx.x & 63);
  }
}
__global__ __launch_bounds__(256) void split_all_kernel(SplitArgs a, unsigned nb_narrow) { split_all_kernel_body(a, nb_narrow); }

// Best split per node over the per-feature results of split_kernel, as one int64 row
// {gain bits, feature + f0, bin, left0, left1}: the largest gain, ties to the lowest feature; a
// NaN gain anywhere makes the node's gain NaN (feature 0), like the torch max/where it replaces.
// One 1024-thread block per node, 4 independent loads in flight per thread (the 256-thread
// version was a latency-bound ~40 us per level at ~10^5 features).
constexpr int kBestThreads = 1024;
// With the narrow search's per-wave partials (bp.part_gain): their ~Fa / 64 values per node
// and the wide features' gains instead of all Fa gains -- the same maximum and tie rule, one
// round of loads per thread (the full scan was ~17 us per level whatever the node count).

__device__ __forceinline__ void split_best_node(const double* gain, const int32_t* bin, const int64_t* left,
                                                int32_t Fa, int64_t f0, int64_t* out, int n,
                                                const BestPartials& bp) {
  const double* g = gain + (int64_t)n * Fa;
  double best = -1.0 / 0.0;
  int bf = Fa;
  bool nan = false;
  if (bp.part_gain) {
    const int64_t t0 = (int64_t)n * Fa;
    const int64_t b0 = t0 / kWave, b1 = (t0 + Fa - 1) / kWave;
    for (int64_t b = b0 + threadIdx.x; b <= b1; b += kBestThreads) {
      const int k = (b * kWave) / Fa == n ? 0 : 1;
      const double v = bp.part_gain[2 * b + k];
      const int fu = bp.part_f[2 * b + k];
      if (v != v) nan = true;
      else if (fu < Fa && (v > best || (v == best && fu < bf))) { best = v; bf = fu; }
    }
    for (int j = threadIdx.x; j < bp.n_wide; j += kBestThreads) {
      const int fu = bp.wide[j];
      const double v = g[fu];
      if (v != v) nan = true;
      else if (v > best || (v == best && fu < bf)) { best = v; bf = fu; }
    }
  }
  for (int f = threadIdx.x; f < Fa && !bp.part_gain; f += 4 * kBestThreads) {
    double v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int fu = f + u * kBestThreads;
      v[u] = fu < Fa ? g[fu] : -1.0 / 0.0;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {           // increasing feature order per thread: ties keep the lower
      const int fu = f + u * kBestThreads;
      if (v[u] != v[u]) nan = true;
      else if (v[u] > best || (v[u] == best && fu < bf)) { best = v[u]; bf = fu; }
    }
  }
  __shared__ double s_g[kBestThreads];
  __shared__ int s_f[kBestThreads];
  __shared__ int s_nan;
  if (threadIdx.x == 0) s_nan = 0;
  __syncthreads();
  if (nan) s_nan = 1;
  s_g[threadIdx.x] = best;
  s_f[threadIdx.x] = bf;
  __syncthreads();
  for (int o = kBestThreads / 2; o > 0; o >>= 1) {
    if (threadIdx.x < o) {
      const double v = s_g[threadIdx.x + o];
      const int f = s_f[threadIdx.x + o];
      if (v > s_g[threadIdx.x] || (v == s_g[threadIdx.x] && f < s_f[threadIdx.x])) {
        s_g[threadIdx.x] = v;
        s_f[threadIdx.x] = f;
      }
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    double bg = s_g[0];
    int f = s_f[0];
    if (s_nan) { bg = __longlong_as_double(0x7ff8000000000000ll); f = 0; }
    if (f >= Fa) f = 0;                      // every gain -inf: feature 0 (its bin is -1)
    const int64_t t = (int64_t)n * Fa + f;
    int64_t* o = out + 5 * (int64_t)n;
    o[0] = __double_as_longlong(bg);
    o[1] = f + f0;
    o[2] = bin[t];
    o[3] = left[2 * t];
    o[4] = left[2 * t + 1];
  }
}

__global__ __launch_bounds__(kBestThreads) void split_best_kernel(const double* gain, const int32_t* bin,
                                                                  const int64_t* left, int32_t Fa, int64_t f0,
                                                                  int64_t* out, BestPartials bp) {
  split_best_node(gain, bin, left, Fa, f0, out, blockIdx.x, bp);
}

// ------------------------------------------------------------------ partition
// kPartRows consecutive rows per thread: the row -> node -> (default child, hot split) -> bin byte
// chain of dependent loads is paid once per 8 rows (16-byte row_node loads and stores) instead
// of once per row and grid-stride step (10M rows: 0.315 -> 0.232 ms per tree over 6 levels,
// profiles/r4/gbdt_10M_round_timeline_partition8.txt).
constexpr int kPartRows = 8;
static_assert(64 * kPartRows == kPartWaveRows, "partition wave rows");

// Lane i of the wave gets the number of (lane, k) with v[k] == i (v[k] < 64; 0xff: none): LDS
// atomics into the wave's own row, or with few distinct values a ballot per value. (Ballots alone
// took up to 64 rounds per k at the deep levels; atomics alone serialise on 2-4 addresses at the
// first levels. 10M rows, per level: 36 / 41 / 54 / 67 / 79 us with ballots, 45 / 45 / 52 / 59 /
// 63 with atomics: profiles/r6/gbdt_late/NOTES.md.)
__device__ __forceinline__ int32_t wave_count64(int32_t* row, const uint32_t (&v)[kPartRows], int lane, bool ballot) {
  if (ballot) {                      // (few distinct values: a ballot each beats same-address atomics)
    int32_t cnt = 0;
#pragma unroll
    for (int k = 0; k < kPartRows; ++k) {
      uint64_t act = __ballot(v[k] < 64u);
      while (act) {
        const uint32_t sv = __shfl(v[k], __ffsll((unsigned long long)act) - 1, 64);
        const uint64_t m = __ballot(v[k] == sv);
        if ((uint32_t)lane == sv) cnt += __popcll(m);
        act &= ~m;
      }
    }
    return cnt;
  }
  row[lane] = 0;
  __builtin_amdgcn_s_waitcnt(0xc07f);
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int k = 0; k < kPartRows; ++k)
    if (v[k] < 64u) atomicAdd(&row[v[k]], 1);
  __builtin_amdgcn_s_waitcnt(0xc07f);
  __builtin_amdgcn_wave_barrier();
  const int32_t c = row[lane];
  __builtin_amdgcn_s_waitcnt(0xc07f);
  __builtin_amdgcn_wave_barrier();
  return c;
}

// kCount: 0 no next-level row counts (the RF lanes, plain partitions: 49 VGPRs); 1 count_work, one
// grid pass, counted after the loop; 2 node_counts alone, counted per 512-row chunk inside the
// loop (any grid); 3 rows_out (+ node_counts), one grid pass, after the loop. Each variant holds
// only its own registers (one kernel for all of them took 81 VGPRs and 5 waves per SIMD: ~7 %
// slower at 10M rows).
template <int kCount>
__device__ __forceinline__ void partition_default_kernel_body(PartitionArgs a) {
  if (a.zero != nullptr) {           // the next level's histograms, zeroed on the way (16-byte stores)
    int4* z = reinterpret_cast<int4*>(a.zero);
    const int64_t nz = a.zero_n / 2;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nz; i += (int64_t)gridDim.x * 256)
      z[i] = make_int4(0, 0, 0, 0);
  }
  const int64_t stride = (int64_t)gridDim.x * 256 * kPartRows;
  uint32_t csl[kPartRows];                 // (count_work) the rows' next-level slots, 0xff: none
  uint32_t rix[kPartRows];                 // (rows_base) the rows' next-level node index, 0xff: none
#pragma unroll
  for (int k = 0; k < kPartRows; ++k) csl[k] = rix[k] = 0xffu;
  const int32_t rbase = (kCount == 2 || kCount == 3) && a.rows_base != nullptr ? *a.rows_base : 0;
  const int32_t cns = kCount == 1 && a.count_work != nullptr ? *a.count_nslots : 0;
  const int lane = threadIdx.x & 63;
  __shared__ int32_t s_wcnt[4][64];                 // (wave_count64: a row per wave of the block)
  // node_counts without rows_out: counted per 512-row chunk inside the loop (any grid); with
  // rows_out (one grid pass) after it
  const bool nc_loop = kCount == 2 && a.node_counts != nullptr;
  const int64_t npw = (a.N + kPartWaveRows - 1) / kPartWaveRows;
  // the loop is wave-uniform: lane l takes rows wb + 8 l .. of the wave's 512-row chunk wb
  for (int64_t wb = ((int64_t)blockIdx.x * 256 + (threadIdx.x & ~63)) * kPartRows; wb < a.N; wb += stride) {
    const int64_t r0 = wb + (int64_t)lane * kPartRows;
    if (nc_loop) {
#pragma unroll
      for (int k = 0; k < kPartRows; ++k) rix[k] = 0xffu;
    }
    if (r0 >= a.N) {
    } else if (r0 + kPartRows <= a.N) {
      int4* p = reinterpret_cast<int4*>(a.row_node + r0);      // (row_node: 16-byte aligned, r0 % 8 == 0)
      const int4 x0 = p[0], x1 = p[1];
      int32_t n[kPartRows] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
      int32_t c[kPartRows];
#pragma unroll
      for (int k = 0; k < kPartRows; ++k)
        c[k] = (n[k] >= 0 && n[k] < a.num_nodes) ? a.default_child[n[k]] : -1;
      if (a.node_dense != nullptr) {
#pragma unroll
        for (int k = 0; k < kPartRows; ++k) {
          if (c[k] < 0) continue;
          const int32_t* nd = a.node_dense + 4 * (int64_t)n[k];
          const int32_t hr = nd[0];
          if (hr >= 0) c[k] = (int32_t)a.dense[(int64_t)hr * a.n_pad + r0 + k] <= nd[1] ? nd[2] : nd[3];
        }
      }
#pragma unroll
      for (int k = 0; k < kPartRows; ++k) n[k] = c[k] >= 0 ? c[k] : n[k];
      if ((kCount == 2 || kCount == 3) && a.rows_base != nullptr) {
#pragma unroll
        for (int k = 0; k < kPartRows; ++k) {
          const int32_t i = n[k] - rbase;
          rix[k] = (i >= 0 && i < 64) ? (uint32_t)i : 0xffu;
        }
      }
      p[0] = make_int4(n[0], n[1], n[2], n[3]);
      p[1] = make_int4(n[4], n[5], n[6], n[7]);
      if (kCount == 1 && a.count_work != nullptr) {
#pragma unroll
        for (int k = 0; k < kPartRows; ++k) {
          const int32_t sk = (n[k] >= 0 && n[k] < a.num_nodes) ? a.count_slot[n[k]] : -1;
          csl[k] = (sk >= 0 && sk < cns) ? (uint32_t)sk : 0xffu;
        }
      }
      if (a.pack != nullptr && a.pack_dig16 != nullptr) {
        // the next level's packed row state (8 rows: 16 B of count digits in, 32 B out)
        const int4 dg = *reinterpret_cast<const int4*>(a.pack_dig16 + r0);
        const uint32_t dw[4] = {(uint32_t)dg.x, (uint32_t)dg.y, (uint32_t)dg.z, (uint32_t)dg.w};
        uint32_t w[kPartRows];
#pragma unroll
        for (int k = 0; k < kPartRows; ++k) {
          const int32_t sk = (n[k] >= 0 && n[k] < a.num_nodes) ? a.pack_slot[n[k]] : -1;
          w[k] = ((sk >= 0 && sk < 255) ? (uint32_t)sk : 0xffu) | (((dw[k >> 1] >> (16 * (k & 1))) & 0xffffu) << 8);
        }
        int4* q = reinterpret_cast<int4*>(a.pack + r0);
        q[0] = make_int4((int)w[0], (int)w[1], (int)w[2], (int)w[3]);
        q[1] = make_int4((int)w[4], (int)w[5], (int)w[6], (int)w[7]);
      } else if (a.pack != nullptr) {
        // the next level's packed row state (8 rows: 64 B of digit words in, 32 B out)
        const int4* dg = reinterpret_cast<const int4*>(a.pack_dig + 2 * r0);
        uint32_t w[kPartRows];
#pragma unroll
        for (int k = 0; k < kPartRows / 2; ++k) {
          const int4 d = dg[k];
          const int32_t s0 = (n[2 * k] >= 0 && n[2 * k] < a.num_nodes) ? a.pack_slot[n[2 * k]] : -1;
          const int32_t s1 = (n[2 * k + 1] >= 0 && n[2 * k + 1] < a.num_nodes) ? a.pack_slot[n[2 * k + 1]] : -1;
          w[2 * k] = ((s0 >= 0 && s0 < 255) ? (uint32_t)s0 : 0xffu) | (((uint32_t)d.x & 0xffu) << 8) |
                     (((uint32_t)d.y & 0xffu) << 16);
          w[2 * k + 1] = ((s1 >= 0 && s1 < 255) ? (uint32_t)s1 : 0xffu) | (((uint32_t)d.z & 0xffu) << 8) |
                         (((uint32_t)d.w & 0xffu) << 16);
        }
        int4* q = reinterpret_cast<int4*>(a.pack + r0);
        q[0] = make_int4((int)w[0], (int)w[1], (int)w[2], (int)w[3]);
        q[1] = make_int4((int)w[4], (int)w[5], (int)w[6], (int)w[7]);
      }
    } else {
      for (int64_t r = r0; r < a.N; ++r) {
        int32_t n = a.row_node[r];
        if (n >= 0 && n < a.num_nodes) {
          const int32_t c = partition_row_child(a, n, r);
          if (c >= 0) a.row_node[r] = n = c;
        }
        if (a.pack != nullptr) a.pack[r] = partition_pack_word(a, n, r);
        if (kCount == 1 && a.count_work != nullptr) {
          const int32_t sk = (n >= 0 && n < a.num_nodes) ? a.count_slot[n] : -1;
          csl[r - r0] = (sk >= 0 && sk < cns) ? (uint32_t)sk : 0xffu;
        }
        if ((kCount == 2 || kCount == 3) && a.rows_base != nullptr) {
          const int32_t i = n - rbase;
          rix[r - r0] = (i >= 0 && i < 64) ? (uint32_t)i : 0xffu;
        }
      }
    }
    if (nc_loop) {
      const int32_t cnt = wave_count64(s_wcnt[threadIdx.x >> 6], rix, lane, a.count_ballot != 0);
      a.node_counts[(int64_t)lane * npw + wb / kPartWaveRows] = cnt;
    }
  }
  const int64_t w = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
  if (kCount == 1 && a.count_work != nullptr && w * 64 * kPartRows < a.N) {       // (wave-uniform)
    // the wave's 512 rows (64 lanes x 8, one grid pass: host-checked) = RgListArgs pass 0's wave
    // w: lane s holds slot s's count
    const int32_t cnt = wave_count64(s_wcnt[threadIdx.x >> 6], csl, lane, a.count_ballot != 0);
    if (lane < cns) a.count_work[2 * cns + w * cns + lane] = cnt;
  }
  if (kCount == 3 && a.rows_out != nullptr) {   // (block-uniform; one grid pass: host-checked)
    // rows per next-level node: the wave's counts -> the block's LDS counts -> 64 spread atomics
    __shared__ int32_t s_rows[64];
    if (threadIdx.x < 64) s_rows[threadIdx.x] = 0;
    __syncthreads();
    const int32_t cnt = wave_count64(s_wcnt[threadIdx.x >> 6], rix, lane, a.count_ballot != 0);
    if (a.node_counts != nullptr && w * kPartWaveRows < a.N) a.node_counts[(int64_t)lane * npw + w] = cnt;
    if (cnt) atomicAdd(&s_rows[lane], cnt);
    __syncthreads();
    if (threadIdx.x < 64 && s_rows[threadIdx.x])
      atomicAdd(&a.rows_out[(blockIdx.x & 31) * 64 + threadIdx.x], s_rows[threadIdx.x]);
  }
}
template <int kCount>
__global__ __launch_bounds__(256) void partition_default_kernel(PartitionArgs a) { partition_default_kernel_body<kCount>(a); }


// LevelChooseArgs: one wave; lane i sums node i's 32 spread row counts (and zeroes them), then
// lane b < builds takes build b's sibling pair.
__global__ __launch_bounds__(64) void level_choose_builds_kernel(LevelChooseArgs a) {
  __shared__ int32_t rows[64];
  const int t = threadIdx.x;
  int32_t sum = 0;
  for (int c = 0; c < 32; ++c) {
    sum += a.rows_out[c * 64 + t];
    a.rows_out[c * 64 + t] = 0;
  }
  rows[t] = sum;
  __syncthreads();
  const int32_t nb = a.counts[2], base = *a.rows_base;
  for (int32_t b = t; b < nb; b += 64) {
    const int32_t jl = a.sub_dst[b];
    if (jl < 0) continue;                            // a lone open child: built anyway
    const int32_t jb = a.s2n[b];
    const int32_t nbuilt = a.next_open[jb], nlarge = a.next_open[jl];
    const int32_t ib = nbuilt - base, il = nlarge - base;
    if (ib < 0 || ib >= 64 || il < 0 || il >= 64 || rows[il] >= rows[ib]) continue;
    a.node_slot[nbuilt] = -1;
    a.node_slot[nlarge] = b;
    a.s2n[b] = jl;
    a.sub_dst[b] = jb;
    a.sub_sib[b] = jl;
    if (a.sub_of != nullptr) {
      a.sub_of[jl] = -1;
      a.sub_of[jb] = b;
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

// Column pass of the device level loop: block b handles split b / wps, entries
// part = b % wps of its column, grid-strided (the splits and their count live on the device).
__device__ __forceinline__ void partition_cols_kernel_body(PartitionArgs a, const int64_t* colptr, const int32_t* cs_feat,
                                                             const int32_t* n_cs, int32_t wps) {
  const int sp = blockIdx.x / wps, part = blockIdx.x % wps;
  if (sp >= *n_cs) return;
  const int32_t dflt = a.split_default[sp], other = a.split_other[sp];
  const int32_t thr = a.split_bin[sp];
  const bool left_default = a.split_left_is_default[sp] != 0;
  const int32_t f = cs_feat[sp];
  const int64_t e1 = colptr[f + 1];
  // (column pass first: the rows are still at the split node; else at its default child)
  const int32_t from = a.node_parent != nullptr ? a.node_parent[dflt] : dflt;
  for (int64_t e = colptr[f] + (int64_t)part * 256 + threadIdx.x; e < e1; e += (int64_t)wps * 256) {
    const int32_t row = a.csc_row[e];
    const bool left = (int32_t)a.csc_bin[e] <= thr;
    if (left != left_default && a.row_node[row] == from) {
      a.row_node[row] = other;
      if (a.pack != nullptr && a.node_parent == nullptr) a.pack[row] = partition_pack_word(a, other, row);
    }
  }
}
__global__ __launch_bounds__(256) void partition_cols_kernel(PartitionArgs a, const int64_t* colptr, const int32_t* cs_feat,
                                                             const int32_t* n_cs, int32_t wps) { partition_cols_kernel_body(a, colptr, cs_feat, n_cs, wps); }

// exclusive prefix count of the lanes below this one whose predicate holds, and the wave total
__device__ __forceinline__ int32_t lp_rank(bool pred, int32_t* total) {
  const unsigned long long m = __ballot(pred);
  *total = __popcll(m);
  return __popcll(m & ((1ull << (threadIdx.x & 63)) - 1ull));
}

// tree.h level_plan on one wave: lane i plans open node i (chunks of 64 with carried counters).
// The sequential plan's only cross-node dependencies are running counters -- child ids (nn),
// column splits (n_cs), next-level open slots (n_next), builds (nb) -- which are exclusive
// prefix sums over per-node predicates here, so the node table, partition and next-level
// tables are exactly the host twin's (tests: device level loop == host loop, bit for bit).
// A node that could split but would overflow max_nodes becomes a leaf, as in the sequential
// plan (child ids only grow, so once one split no longer fits no later one does).
__device__ void level_plan_wave(const LevelPlanArgs& a) {
  const int32_t lane = (int32_t)(threadIdx.x & 63);
  const double thr = a.min_gain > 1e-6 ? a.min_gain : 1e-6;
  const double s0 = ldexp(1.0, -a.kexp[0]), s1 = ldexp(1.0, -a.kexp[1]);
  int32_t nn = *a.n_nodes, n_cs = 0, n_next = 0, nb = 0;
  const int32_t no = *a.n_open;
  int64_t R0 = 0, R1 = 0;                  // (depth 0 of the fused prologue) the root's sums
  if (a.root_parts) {
    R0 = lane < kRootSlots ? a.root_parts[kRootStride * lane] : 0;
    R1 = lane < kRootSlots ? a.root_parts[kRootStride * lane + 1] : 0;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      R0 += __shfl_xor(R0, o, 64);
      R1 += __shfl_xor(R1, o, 64);
    }
    if (lane == 0) { a.stats[0] = R0; a.stats[1] = R1; }
  } else if (a.root_tot) {
    R0 = a.root_tot[0];
    R1 = a.root_tot[1];
    if (lane == 0) { a.stats[0] = R0; a.stats[1] = R1; }
  }
  for (int32_t base = 0; base < no; base += 64) {
    const int32_t i = base + lane;
    const bool live = i < no;
    const int32_t n = live ? a.open[i] : -1;
    double g = -1.0 / 0.0;
    const int64_t* p = a.packed + 5 * (int64_t)(live ? i : 0);
    int32_t f = -1, b = -1;
    if (live) {
      memcpy(&g, &p[0], sizeof(double));
      for (int32_t sh = 1; sh < a.n_shards; ++sh) {
        const int64_t* q = a.packed + sh * a.shard_stride + 5 * (int64_t)i;
        double gq;
        memcpy(&gq, &q[0], sizeof(double));
        if (gq > g) { g = gq; p = q; }
      }
      f = (int32_t)p[1];
      b = (int32_t)p[2];
    }
    const bool ok = live && (a.mode == 0 ? (b >= 0 && isfinite(g) && g > thr)
                                         : (b >= 0 && isfinite(g) && g > 0.0 && g >= a.min_gain));
    int32_t n_ok;
    const int32_t r_ok = lp_rank(ok, &n_ok);
    const bool split = ok && nn + 2 * (r_ok + 1) <= a.max_nodes;
    int32_t n_split;
    const int32_t r_split = lp_rank(split, &n_split);
    if (live && !split) a.leaf[n] = 1;
    const int32_t li = nn + 2 * r_split, ri = li + 1;
    bool cleaf[2] = {true, true};
    bool dense = false;
    if (split) {
      const int64_t l0 = p[3], l1 = p[4];
      const bool root = (a.root_parts || a.root_tot) && n == 0;
      const int64_t t0 = root ? R0 : a.stats[2 * n], t1 = root ? R1 : a.stats[2 * n + 1];
      const int64_t cs[2][2] = {{l0, l1}, {t0 - l0, t1 - l1}};
      for (int k = 0; k < 2; ++k) {
        const int32_t c = li + k;
        a.stats[2 * c] = cs[k][0];
        a.stats[2 * c + 1] = cs[k][1];
        bool leafy = a.depth + 1 >= a.max_depth;
        if (a.mode != 0) leafy = leafy || impurity(a.mode, (double)cs[k][0] * s0, (double)cs[k][1] * s1) == 0.0;
        a.parent[c] = n;
        a.left[c] = a.right[c] = -1;
        a.feat[c] = -1;
        a.bin[c] = -1;
        a.gain[c] = -1.0;
        a.leaf[c] = leafy ? 1 : 0;
        cleaf[k] = leafy;
      }
      a.feat[n] = f;
      a.bin[n] = b;
      a.left[n] = li;
      a.right[n] = ri;
      a.gain[n] = g;
      const int32_t hr = a.hot_row ? a.hot_row[f] : -1;
      dense = a.node_dense && hr >= 0;
      const bool left_default = a.zbin[f] <= b;
      const int32_t dflt = left_default ? li : ri;
      a.default_child[n] = dflt;
      if (dense) {
        int32_t* nd = a.node_dense + 4 * (int64_t)n;
        nd[0] = hr; nd[1] = b; nd[2] = li; nd[3] = ri;
      }
    }
    int32_t n_col;
    const int32_t r_col = lp_rank(split && !dense, &n_col);
    if (split && !dense) {
      const bool left_default = a.zbin[f] <= b;
      const int32_t k = n_cs + r_col;
      a.cs_feat[k] = f;
      a.cs_default[k] = left_default ? li : ri;
      a.cs_other[k] = left_default ? ri : li;
      a.cs_bin[k] = b;
      a.cs_left_default[k] = left_default ? 1 : 0;
    }
    // next-level open slots: the node's non-leaf children in order (left, right)
    const int32_t c_open = split ? (int32_t)!cleaf[0] + (int32_t)!cleaf[1] : 0;
    int32_t incl = c_open;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int32_t o = __shfl_up(incl, d, 64);
      if (lane >= d) incl += o;
    }
    const int32_t tot_open = __shfl(incl, 63, 64);
    const int32_t pos = n_next + incl - c_open;
    if (c_open) {
      int32_t j = pos;
      for (int k = 0; k < 2; ++k)
        if (!cleaf[k]) {
          const int32_t c = li + k;
          a.next_open[j] = c;
          a.next_totals[2 * j] = a.stats[2 * c];
          a.next_totals[2 * j + 1] = a.stats[2 * c + 1];
          ++j;
        }
    }
    // builds of level d + 1 (non-build_all): one per split node with an open child, in order
    int32_t n_bld;
    const int32_t r_bld = lp_rank(!a.build_all && c_open > 0, &n_bld);
    if (!a.build_all && c_open > 0) {
      const int32_t k = nb + r_bld;
      int32_t build, jb, large = -1, jl = -1;
      if (c_open == 2) {
        const int64_t wl = a.mode == 0 ? a.stats[2 * li + 1] : a.stats[2 * li] + a.stats[2 * li + 1];
        const int64_t wr = a.mode == 0 ? a.stats[2 * ri + 1] : a.stats[2 * ri] + a.stats[2 * ri + 1];
        const bool lsmall = wl <= wr;
        build = lsmall ? li : ri;
        large = lsmall ? ri : li;
        jb = lsmall ? pos : pos + 1;
        jl = lsmall ? pos + 1 : pos;
      } else {
        build = cleaf[0] ? ri : li;
        jb = pos;
      }
      a.node_slot[build] = k;
      a.s2n[k] = jb;
      if (large >= 0) {
        a.sub_dst[k] = jl;
        if (a.sub_of) a.sub_of[jl] = k;
        a.sub_par[k] = i;
        a.sub_sib[k] = jb;
      }
    }
    nn += 2 * n_split;
    n_cs += n_col;
    n_next += tot_open;
    nb += n_bld;
  }
  if (a.build_all) {
    for (int32_t j = lane; j < n_next; j += 64) {
      a.node_slot[a.next_open[j]] = j;
      a.s2n[j] = j;
    }
    nb = n_next;
  }
  if (lane == 0) {
    *a.n_nodes = nn;
    a.counts[0] = n_cs;
    a.counts[1] = n_next;
    a.counts[2] = nb;
    a.counts[3] = nn;
    for (int k = 0; k < a.counts_tail; ++k) a.counts[4 + k] = 0;
    if (a.counts_host) {         // host-mapped pinned row: visible to the host at the kernel's end
      a.counts_host[0] = n_cs;
      a.counts_host[1] = n_next;
      a.counts_host[2] = nb;
      a.counts_host[3] = nn;
    }
  }
  if (a.lr_row_of) {             // (the build tables written above by other lanes of this wave)
    __threadfence_block();
    __builtin_amdgcn_wave_barrier();
    LevelRowsArgs r{};
    r.s2n = a.s2n;
    r.sub_dst = a.sub_dst;
    r.sub_par = a.sub_par;
    r.prev_row_of = a.lr_prev;
    r.nb = nb;
    r.bld_base = 0;
    r.sub_base = nb;
    r.row_of = a.lr_row_of;
    r.dst_row = a.lr_dst;
    r.par_row = a.lr_par;
    r.sib_row = a.lr_sib;
    for (int32_t k = lane; k < nb; k += 64) level_rows_slot(r, k);
  }
}

__global__ __launch_bounds__(64) void level_rows_kernel(LevelRowsArgs a) {
  const int32_t k = (int32_t)(blockIdx.x * 64 + threadIdx.x);
  if (k < a.nb) level_rows_slot(a, k);
}

__device__ __forceinline__ void level_plan_kernel_body(LevelPlanArgs a) {
  if (blockIdx.x != 0) return;
  level_plan_reset(a, (int32_t)threadIdx.x, (int32_t)blockDim.x);
  __syncthreads();
  if (threadIdx.x < 64) level_plan_wave(a);
}
__global__ void level_plan_kernel(LevelPlanArgs a) { level_plan_kernel_body(a); }

// split_best_kernel + level_plan_kernel in one launch (levels without a collective between the
// split search and the plan): a workgroup per node writes its best split tuple, and the last
// workgroup to finish (ticket) plans the level from all of them -- the same two bodies, so the
// same node table bit for bit, one launch and one kernel boundary less per level.
__device__ __forceinline__ void split_best_plan_kernel_body(const double* gain, const int32_t* bin,
                                                                       const int64_t* left, int32_t Fa, int64_t f0,
                                                                       int64_t* out, LevelPlanArgs p,
                                                                       unsigned int* ticket, BestPartials bp,
                                                                       unsigned nblocks = 0) {
  split_best_node(gain, bin, left, Fa, f0, out, blockIdx.x, bp);
  if (!last_workgroup(ticket, nblocks)) return;
  level_plan_reset(p, (int32_t)threadIdx.x, (int32_t)blockDim.x);
  __syncthreads();
  if (threadIdx.x < 64) level_plan_wave(p);
}
__global__ __launch_bounds__(kBestThreads) void split_best_plan_kernel(const double* gain, const int32_t* bin,
                                                                       const int64_t* left, int32_t Fa, int64_t f0,
                                                                       int64_t* out, LevelPlanArgs p,
                                                                       unsigned int* ticket, BestPartials bp) { split_best_plan_kernel_body(gain, bin, left, Fa, f0, out, p, ticket, bp); }

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

// margin[r] += the leaf value of the row's node, computed from the node table (leaf_value: the
// same fp64 operations as leaf_values_kernel, so bitwise leaf_values + leaf_update in one launch)
__global__ __launch_bounds__(256) void leaf_update_stats_kernel(double* margin, const int32_t* row_node,
                                                               const int64_t* stats, const int32_t* kexp, double eta,
                                                               double lambda, double mds, int64_t N) {
  const int32_t k0 = kexp[0], k1 = kexp[1];
  for (int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x; r < N; r += (int64_t)gridDim.x * 256) {
    const int32_t n = row_node[r];
    margin[r] += leaf_value(stats[2 * n], stats[2 * n + 1], k0, k1, eta, lambda, mds);
  }
}

__global__ __launch_bounds__(256) void leaf_values_kernel(const int64_t* stats, const int32_t* kexp, int64_t M,
                                                          double eta, double lambda, double mds, double* out) {
  const int64_t n = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (n < M) out[n] = leaf_value(stats[2 * n], stats[2 * n + 1], kexp[0], kexp[1], eta, lambda, mds);
}

// ------------------------------------------------------------------ lane-batched kernels
// (tree.h "lane-batched launches": lane l = blockIdx.z, its arguments copied out of args[l])
__global__ __launch_bounds__(256) void quant_lanes_kernel(const QuantLane* __restrict__ args) {
  const QuantLane q = args[blockIdx.z];
  quant_kernel_body(q.a, q.maxv, q.part);
}

template <int BT, bool PACK>
__global__ __launch_bounds__(256) void hist_lds_lanes_kernel(const HistArgs* __restrict__ args) {
  const HistArgs a = args[blockIdx.z];
  if (a.active_list == nullptr && (int)blockIdx.x * 4 >= (a.wave_item ? a.num_slots : a.num_items)) return;
  hist_lds_kernel_body<BT, PACK>(a);
}

__global__ __launch_bounds__(64) void hist_count_zero_lanes_kernel(const HistArgs* __restrict__ args) {
  if (threadIdx.x < 8) args[blockIdx.z].active_count[threadIdx.x] = 0;
}

__global__ __launch_bounds__(256) void hist_select_lanes_kernel(const HistArgs* __restrict__ args) {
  HistArgs a = args[blockIdx.z];
  a.num_slots = a.wave_item ? a.num_slots : a.num_items;
  if ((int64_t)blockIdx.x * 256 * kSelPerThread >= a.num_slots) return;
  hist_select_kernel_body(a, a.active_list, a.active_count);
}

__global__ __launch_bounds__(256) void split_all_lanes_kernel(const SplitArgs* __restrict__ args) {
  const SplitArgs a = args[blockIdx.z];
  const int64_t n = (int64_t)a.num_nodes * a.Fa;
  const unsigned nb = (unsigned)((n + 255) / 256);
  const int64_t waves = (a.wide != nullptr && a.n_wide > 0) ? (int64_t)a.num_nodes * a.n_wide : 0;
  if (n <= 0 || blockIdx.x >= nb + (unsigned)((waves + 3) / 4)) return;
  split_all_kernel_body(a, nb);
}

__global__ __launch_bounds__(kBestThreads) void split_best_lanes_kernel(const SplitBestLane* __restrict__ args) {
  const SplitBestLane b = args[blockIdx.z];
  if ((int)blockIdx.x >= b.nodes || b.Fa <= 0) return;
  split_best_node(b.gain, b.bin, b.left, b.Fa, b.f0, b.out, blockIdx.x, b.bp);
}

__global__ __launch_bounds__(kBestThreads) void split_best_plan_lanes_kernel(const SplitBestPlanLane* __restrict__ args) {
  const SplitBestPlanLane q = args[blockIdx.z];
  if ((int)blockIdx.x >= q.b.nodes) return;
  split_best_plan_kernel_body(q.b.gain, q.b.bin, q.b.left, q.b.Fa, q.b.f0, q.b.out, q.p, q.ticket, q.b.bp,
                              (unsigned)q.b.nodes);
}

__global__ void level_plan_lanes_kernel(const LevelPlanArgs* __restrict__ args) { level_plan_kernel_body(args[blockIdx.z]); }

__global__ __launch_bounds__(256) void partition_cols_lanes_kernel(const PartColsLane* __restrict__ args) {
  const PartColsLane q = args[blockIdx.z];
  if ((int)blockIdx.x >= q.max_splits * q.wps) return;
  partition_cols_kernel_body(q.a, q.colptr, q.cs_feat, q.n_cs, q.wps);
}

__global__ __launch_bounds__(64) void root_send_lanes_kernel(const RootSendLane* __restrict__ args) {
  const RootSendLane a = args[blockIdx.z];
  int64_t t0, t1;
  root_sums(a.root_parts, &t0, &t1);
  for (int32_t sh = (int32_t)threadIdx.x; sh < a.S; sh += 64) {
    a.send[sh * a.chunk_words + a.tot_word] = t0;
    a.send[sh * a.chunk_words + a.tot_word + 1] = t1;
  }
}

__global__ __launch_bounds__(256) void copy_lanes_kernel(const CopyLane* __restrict__ args) {
  const CopyLane c = args[blockIdx.z];
  const bool words = ((reinterpret_cast<uintptr_t>(c.dst) | reinterpret_cast<uintptr_t>(c.src) | (uintptr_t)c.bytes) & 7) == 0;
  const int64_t n = words ? c.bytes / 8 : c.bytes;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    if (words) reinterpret_cast<uint64_t*>(c.dst)[i] = reinterpret_cast<const uint64_t*>(c.src)[i];
    else reinterpret_cast<uint8_t*>(c.dst)[i] = reinterpret_cast<const uint8_t*>(c.src)[i];
  }
}

// The lane-argument staging copy: 16-byte words from pinned host memory (read through its device
// mapping) into device memory. A kernel on the stream instead of hipMemcpyAsync: the runtime's H2D
// path put ~40 us (SDMA) to ~0.5 ms (a blit at a batch start) between a level's stages
// (profiles/r6/rf_dp_busy_gaps_*.txt).
__global__ __launch_bounds__(256) void stage_copy_kernel(uint4* __restrict__ dst, const uint4* __restrict__ src,
                                                         int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) dst[i] = src[i];
}

template <int kCount>
__global__ __launch_bounds__(256) void partition_default_lanes_kernel(const PartitionArgs* __restrict__ args) {
  partition_default_kernel_body<kCount>(args[blockIdx.z]);
}

constexpr int kQuantBlocks = 2048;      // workgroup cap of the quantisation passes (partials)
constexpr int kTicketBlocks = 512;      // ... of the single-launch (last-workgroup) passes
constexpr int kSlotBlocks = 2048;       // ... of the spread-slot passes (64 atomics per slot at most)

inline unsigned grid_for(int64_t n, int64_t cap = 8192) {
  const int64_t b = (n + 255) / 256;
  return (unsigned)(b < 1 ? 1 : (b > cap ? cap : b));
}

// the partition's row pass, with the counting variant where any count is asked for
void launch_partition_default(const PartitionArgs& a, hipStream_t s) {
  if (a.N <= 0) return;
  const dim3 grid(grid_for((a.N + kPartRows - 1) / kPartRows));
  FDX_LANES_CHECK(a.count_work == nullptr || a.rows_base == nullptr);   // (one counting mode at a time)
  if (a.count_work != nullptr)
    hipLaunchKernelGGL(partition_default_kernel<1>, grid, dim3(256), 0, s, a);
  else if (a.rows_out != nullptr && a.count_work == nullptr)
    hipLaunchKernelGGL(partition_default_kernel<3>, grid, dim3(256), 0, s, a);
  else if (a.rows_base != nullptr && a.node_counts != nullptr)
    hipLaunchKernelGGL(partition_default_kernel<2>, grid, dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL(partition_default_kernel<0>, grid, dim3(256), 0, s, a);
}
}  // namespace

int quant_blocks(int64_t n) { return (int)grid_for(n, kQuantBlocks); }

void launch_quant_max(const QuantArgs& a, double* out, void* partials, hipStream_t s) {
  auto* part = reinterpret_cast<unsigned long long*>(partials);
  const int nb = a.N > 0 ? quant_blocks(a.N) : 0;
  if (nb > 0) hipLaunchKernelGGL(quant_max_kernel, dim3(nb), dim3(256), 0, s, a, part);
  hipLaunchKernelGGL(quant_reduce_kernel<true>, dim3(1), dim3(256), 0, s, part, nb,
                     reinterpret_cast<unsigned long long*>(out));
}

void launch_grad_max(const double* margin, const float* label, float* g, float* h, int64_t N, double* maxv,
                     const PrologueInit& pi, hipStream_t s) {
  const int nb = (int)grid_for((N > 0 ? N : 1) / kPrologueU + 1, kSlotBlocks);
  hipLaunchKernelGGL(grad_max_kernel, dim3(nb), dim3(256), 0, s, margin, label, g, h, N,
                     reinterpret_cast<unsigned long long*>(maxv), pi);
}

void launch_quant(const QuantArgs& a, const double* maxv, void* partials, hipStream_t s) {
  auto* part = reinterpret_cast<unsigned long long*>(partials);
  const int nb = a.N > 0 ? quant_blocks(a.N) : 0;
  if (a.ticket != nullptr || a.atomic_root) {     // one launch (quant_kernel)
    const int nt = a.N > 0 ? (int)grid_for(a.N / kPrologueU + 1, a.atomic_root ? kSlotBlocks : kTicketBlocks) : 1;
    hipLaunchKernelGGL(quant_kernel, dim3(nt), dim3(256), 0, s, a, maxv, part);
    return;
  }
  if (nb > 0) hipLaunchKernelGGL(quant_kernel, dim3(nb), dim3(256), 0, s, a, maxv, part);
  else hipLaunchKernelGGL(quant_kernel, dim3(1), dim3(256), 0, s, a, maxv, part);     // (writes kexp)
  hipLaunchKernelGGL(quant_reduce_kernel<false>, dim3(1), dim3(256), 0, s, part, nb > 0 ? nb : 1,
                     reinterpret_cast<unsigned long long*>(a.totals));
}

void launch_slot8(const SlotArgs& a, hipStream_t s) {
  if (a.N > 0) hipLaunchKernelGGL(slot8_kernel, dim3(grid_for(a.N)), dim3(256), 0, s, a);
}

__device__ __forceinline__ void hist_select_groups_kernel_body(const SelectArgs& a) {
  const int g = blockIdx.y;
  const int64_t w0 = (int64_t)blockIdx.x * 256 * kSelPerThread;
  if (w0 >= a.num_slots[g]) return;                 // (workgroup-uniform)
  __shared__ int32_t s_cnt[8], s_base[8];
  const int t = threadIdx.x;
  if (t < 8) s_cnt[t] = 0;
  __syncthreads();
  const int32_t* wave_item = a.wave_item[g];
  const int32_t* item_f0 = a.item_f0[g];
  const int32_t* item_meta = a.item_meta[g];
  int32_t item[kSelPerThread], loc[kSelPerThread];
#pragma unroll
  for (int j = 0; j < kSelPerThread; ++j) {
    const int64_t w = w0 + (int64_t)j * 256 + t;
    int it = -1;
    if (w < a.num_slots[g]) it = wave_item ? wave_item[w] : (int)w;
    bool act = false;
    if (it >= 0 && it < a.num_items[g]) {
      const int32_t f0 = item_f0[it];
      const int nf = (item_meta[it] >> 8) & 0xFF;
      for (int k = 0; k < nf && !act; ++k) act = a.feat_active[f0 + k] != 0;
    }
    item[j] = it;
    loc[j] = act ? atomicAdd(&s_cnt[(w >> 2) & 7], 1) : -1;      // (hist_select_kernel: XCD of the slot)
  }
  __syncthreads();
  if (t < 8) s_base[t] = s_cnt[t] ? atomicAdd(a.count[g] + t, s_cnt[t]) : 0;
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kSelPerThread; ++j)
    if (loc[j] >= 0) {
      const int x = (int)(((w0 + (int64_t)j * 256 + t) >> 2) & 7);
      a.list[g][(int64_t)x * a.list_cap[g] + s_base[x] + loc[j]] = item[j];
    }
}
__global__ __launch_bounds__(256) void hist_select_groups_kernel(SelectArgs a) { hist_select_groups_kernel_body(a); }
__global__ __launch_bounds__(256) void hist_select_groups_lanes_kernel(const SelectArgs* __restrict__ args) {
  hist_select_groups_kernel_body(args[blockIdx.z]);
}

void launch_hist_select_groups(const SelectArgs& a, hipStream_t s) {
  int32_t most = 0;
  for (int g = 0; g < a.n; ++g) most = a.num_slots[g] > most ? a.num_slots[g] : most;
  if (a.n <= 0 || most <= 0) return;
  hipLaunchKernelGGL(hist_select_groups_kernel, dim3((most + 256 * kSelPerThread - 1) / (256 * kSelPerThread), a.n),
                     dim3(256), 0, s, a);
}

void launch_hist_select(const HistArgs& a, hipStream_t s) {
  const int32_t slots = a.wave_item ? a.num_slots : a.num_items;
  if (slots <= 0) return;
  HistArgs sel = a;
  sel.num_slots = slots;
  hipLaunchKernelGGL(hist_select_kernel, dim3((slots + 256 * kSelPerThread - 1) / (256 * kSelPerThread)), dim3(256), 0, s, sel,
                     const_cast<int32_t*>(a.active_list), const_cast<int32_t*>(a.active_count));
}

void launch_hist(const HistArgs& a, int bt, int ct, int np, hipStream_t s) {
  if (a.num_items <= 0) return;
  const int32_t slots = a.wave_item ? a.num_slots : a.num_items;
  dim3 grid((slots + 3) / 4);
  const dim3 block(256);
  const bool root = a.slot8 == nullptr && a.rowpack == nullptr;
  if (a.active_list != nullptr && a.listed_per_xcd >= 0) {
    // preselected list (launch_hist_select, queued with the previous level's plan; the per-XCD
    // counts reached the host with the level's counts): a wave per active item, none idle
    if (a.listed_per_xcd == 0) return;
    grid = dim3((unsigned)((a.listed_per_xcd + 3) / 4 * 8));
  } else if (a.active_list != nullptr) {
    // listed pass: compact the active items, then a grid of at most kListedWaves waves strides
    // over them (the full grid was ~300K wave slots, most of them exiting at once: ~100 us a pass)
    HistArgs sel = a;
    sel.num_slots = slots;
    (void)hipMemsetAsync(const_cast<int32_t*>(a.active_count), 0, 8 * sizeof(int32_t), s);   // per-XCD counts
    hipLaunchKernelGGL(hist_select_kernel, dim3((slots + 256 * kSelPerThread - 1) / (256 * kSelPerThread)), dim3(256), 0, s, sel,
                       const_cast<int32_t*>(a.active_list), const_cast<int32_t*>(a.active_count));
    static const int32_t listed_waves = [] {
      const char* e = getenv("FDX_LISTED_WAVES");                  // (experiments: the grid of a listed pass)
      return e ? atoi(e) : kListedWaves;
    }();
    const int32_t waves = slots < listed_waves ? slots : listed_waves;
    grid = dim3((unsigned)(((waves + 3) / 4 + 7) / 8 * 8));       // whole XCD rounds of workgroups
  }
  if (a.lds && np == 1) {
    // (host-checked: 4 waves x 16 bt keys x nslots x 8 B <= 64 KB)
    const size_t lds = (size_t)4 * 16 * bt * a.nslots * sizeof(unsigned long long);
    const bool pack = a.rowpack != nullptr;
    if (bt == 1) { if (pack) hipLaunchKernelGGL((hist_lds_kernel<1, true>), grid, block, lds, s, a); else hipLaunchKernelGGL((hist_lds_kernel<1, false>), grid, block, lds, s, a); }
    else if (bt == 2) { if (pack) hipLaunchKernelGGL((hist_lds_kernel<2, true>), grid, block, lds, s, a); else hipLaunchKernelGGL((hist_lds_kernel<2, false>), grid, block, lds, s, a); }
    else { if (pack) hipLaunchKernelGGL((hist_lds_kernel<4, true>), grid, block, lds, s, a); else hipLaunchKernelGGL((hist_lds_kernel<4, false>), grid, block, lds, s, a); }
    return;
  }
#define FDX_HIST_NP(B, C, P)                                                                             \
  if (np == P) {                                                                                        \
    if (root) hipLaunchKernelGGL((hist_i8_kernel<B, 1, P, true>), grid, block, 0, s, a);                \
    else if (P == 1 && a.rowpack) hipLaunchKernelGGL((hist_i8_kernel<B, C, 1, false, true>), grid, block, 0, s, a); \
    else hipLaunchKernelGGL((hist_i8_kernel<B, C, P, false>), grid, block, 0, s, a);                    \
    return;                                                                                             \
  }
#define FDX_HIST_CASE(B, C)                                                                              \
  if (bt == B && ct == C) { FDX_HIST_NP(B, C, 1) FDX_HIST_NP(B, C, 4) }
  FDX_HIST_CASE(1, 1) FDX_HIST_CASE(1, 2) FDX_HIST_CASE(1, 4) FDX_HIST_CASE(1, 8)
  FDX_HIST_CASE(2, 1) FDX_HIST_CASE(2, 2) FDX_HIST_CASE(2, 4) FDX_HIST_CASE(2, 8)
  FDX_HIST_CASE(4, 1) FDX_HIST_CASE(4, 2) FDX_HIST_CASE(4, 4) FDX_HIST_CASE(4, 8)
#undef FDX_HIST_CASE
#undef FDX_HIST_NP
}

// features per wave of the dense kernel: accumulators FG * BT * CT * 4 registers <= 64. Only the
// 16-bin (BT = 1) hot features are numerous enough (~130) to share the row state of a wave; the
// few wider ones (BT 2 / 4: ~10) take one wave each, otherwise their launches ran ~600 waves on
// 1,024 SIMDs (measured 2.0 -> 0.85 ms for 9 features; 4 instead of 8 16-bin features per wave
// doubled that launch instead: 1.7 -> 3.6 ms).
constexpr int dense_fg(int bt, int ct) {
  return bt > 1 ? 1 : (ct >= 16 ? 1 : 16 / ct > 8 ? 8 : 16 / ct);
}

int dense_features_per_wave(int bt, int ct) { return dense_fg(bt, ct); }
int dense_waves_per_group() { return 1; }

void launch_hist_dense(const DenseHistArgs& a, int bt, int ct, int np, hipStream_t s) {
  if (a.ngroups <= 0 || a.nranges <= 0) return;
  const int per_x = (a.nranges + 7) / 8;                  // ranges per XCD label
  const int64_t waves = (int64_t)per_x * a.ngroups;      // per XCD label
  const dim3 grid((unsigned)(8 * ((waves + 3) / 4))), block(256);
  const bool root = a.slot8 == nullptr;
#define FDX_DENSE_NP(B, C, P)                                                                            \
  if (np == P) {                                                                                        \
    if (root) hipLaunchKernelGGL((hist_dense_kernel<B, 1, P, true, dense_fg(B, 1)>), grid, block, 0, s, a); \
    else hipLaunchKernelGGL((hist_dense_kernel<B, C, P, false, dense_fg(B, C)>), grid, block, 0, s, a);    \
    return;                                                                                             \
  }
#define FDX_DENSE_CASE(B, C)                                                                             \
  if (bt == B && ct == C) { FDX_DENSE_NP(B, C, 1) FDX_DENSE_NP(B, C, 4) }
  FDX_DENSE_CASE(1, 1) FDX_DENSE_CASE(1, 2) FDX_DENSE_CASE(1, 4) FDX_DENSE_CASE(1, 8)
  FDX_DENSE_CASE(2, 1) FDX_DENSE_CASE(2, 2) FDX_DENSE_CASE(2, 4) FDX_DENSE_CASE(2, 8)
  FDX_DENSE_CASE(4, 1) FDX_DENSE_CASE(4, 2) FDX_DENSE_CASE(4, 4) FDX_DENSE_CASE(4, 8)
#undef FDX_DENSE_CASE
#undef FDX_DENSE_NP
}

void launch_hist_subtract(const int64_t* parent, int64_t* cur, const int32_t* dst, const int32_t* par, const int32_t* sib,
                          int32_t n_pairs, int64_t TB, hipStream_t s) {
  if (n_pairs <= 0 || TB <= 0) return;
  const int64_t bx = (TB + 255) / 256;
  hipLaunchKernelGGL(hist_subtract_kernel, dim3((unsigned)(bx < 1024 ? bx : 1024), (unsigned)n_pairs), dim3(256), 0, s,
                     parent, cur, dst, par, sib, n_pairs, TB);
}

void launch_split(const SplitArgs& a, hipStream_t s) {
  const int64_t n = (int64_t)a.num_nodes * a.Fa;
  if (n <= 0) return;
  const unsigned nb = (unsigned)((n + 255) / 256);
  const int64_t waves = (a.wide != nullptr && a.n_wide > 0) ? (int64_t)a.num_nodes * a.n_wide : 0;
  hipLaunchKernelGGL(split_all_kernel, dim3(nb + (unsigned)((waves + 3) / 4)), dim3(256), 0, s, a, nb);
}

static BestPartials best_partials(const SplitArgs* sa) {
  BestPartials bp{};
  if (sa && sa->part_gain) bp = BestPartials{sa->part_gain, sa->part_f, sa->wide, sa->wide ? sa->n_wide : 0};
  return bp;
}

void launch_split_best_plan(const double* gain, const int32_t* bin, const int64_t* left, int32_t nodes, int32_t Fa,
                            int64_t f0, int64_t* out, const LevelPlanArgs& p, unsigned int* ticket, hipStream_t s,
                            const SplitArgs* partials) {
  if (nodes <= 0 || Fa <= 0) {                  // (no candidates: the caller filled out)
    hipLaunchKernelGGL(level_plan_kernel, dim3(1), dim3(64), 0, s, p);
    return;
  }
  hipLaunchKernelGGL(split_best_plan_kernel, dim3(nodes), dim3(kBestThreads), 0, s, gain, bin, left, Fa, f0, out, p,
                     ticket, best_partials(partials));
}

void launch_split_best(const double* gain, const int32_t* bin, const int64_t* left, int32_t nodes, int32_t Fa,
                       int64_t f0, int64_t* out, hipStream_t s, const SplitArgs* partials) {
  if (nodes > 0 && Fa > 0)
    hipLaunchKernelGGL(split_best_kernel, dim3(nodes), dim3(kBestThreads), 0, s, gain, bin, left, Fa, f0, out,
                       best_partials(partials));
}

int64_t split_partials(int32_t nodes, int32_t Fa) {
  return Fa >= kWave ? 2 * (((int64_t)nodes * Fa + 255) / 256) * 4 : 0;     // (every wave of the narrow grid)
}

void launch_partition(const PartitionArgs& a, hipStream_t s) {
  launch_partition_default(a, s);
  if (a.num_items > 0) hipLaunchKernelGGL(partition_column_kernel, dim3(a.num_items), dim3(256), 0, s, a);
}

void launch_level_rows(const LevelRowsArgs& a, hipStream_t s) {
  if (a.nb <= 0) return;
  hipLaunchKernelGGL(level_rows_kernel, dim3((unsigned)((a.nb + 63) / 64)), dim3(64), 0, s, a);
}

void launch_level_plan(const LevelPlanArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(level_plan_kernel, dim3(1), dim3(64), 0, s, a);
}

void launch_partition_cols(const PartitionArgs& a, const int64_t* colptr, const int32_t* cs_feat, const int32_t* n_cs,
                           int32_t max_splits, int32_t wps, hipStream_t s) {
  const auto cols = [&] {
    if (max_splits > 0)
      hipLaunchKernelGGL(partition_cols_kernel, dim3(max_splits * wps), dim3(256), 0, s, a, colptr, cs_feat, n_cs, wps);
  };
  if (a.node_parent != nullptr) cols();   // (column pass first: PartitionArgs node_parent)
  launch_partition_default(a, s);
  if (a.node_parent == nullptr) cols();
}

void launch_level_choose_builds(const LevelChooseArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(level_choose_builds_kernel, dim3(1), dim3(64), 0, s, a);
}

bool partition_counts_ok(int64_t N) {
  return rg_list_rows(N) == 64 * kPartRows && (N + kPartRows - 1) / kPartRows <= 8192ll * 256;
}

void launch_logistic_grad(const double* margin, const float* label, const float* weight, float* g, float* h,
                          int64_t N, hipStream_t s) {
  if (N > 0) hipLaunchKernelGGL(logistic_grad_kernel, dim3(grid_for(N)), dim3(256), 0, s, margin, label, weight, g, h, N);
}

void launch_leaf_values(const int64_t* stats, const int32_t* kexp, int64_t M, double eta, double lambda, double mds,
                        double* out, hipStream_t s) {
  if (M > 0)
    hipLaunchKernelGGL(leaf_values_kernel, dim3((unsigned)((M + 255) / 256)), dim3(256), 0, s, stats, kexp, M, eta,
                       lambda, mds, out);
}

void launch_leaf_update_stats(double* margin, const int32_t* row_node, const int64_t* stats, const int32_t* kexp,
                              double eta, double lambda, double mds, int64_t N, hipStream_t s) {
  if (N > 0)
    hipLaunchKernelGGL(leaf_update_stats_kernel, dim3(grid_for(N)), dim3(256), 0, s, margin, row_node, stats, kexp, eta,
                       lambda, mds, N);
}

void launch_leaf_update(double* margin, const int32_t* row_node, const double* node_value, int64_t N, hipStream_t s) {
  if (N > 0) hipLaunchKernelGGL(leaf_update_kernel, dim3(grid_for(N)), dim3(256), 0, s, margin, row_node, node_value, N);
}

// ------------------------------------------------------------------ lane-batched launchers
// h: the lanes' arguments on the host (grid sizing), d: the same array in device memory
void launch_quant_lanes(const QuantLane* h, const QuantLane* d, int L, hipStream_t s) {
  if (L <= 0) return;
  unsigned gx = 1;
  for (int l = 0; l < L; ++l) {
    const QuantArgs& a = h[l].a;
    FDX_LANES_CHECK(a.atomic_root && a.ticket == nullptr);
    const unsigned nt = a.N > 0 ? grid_for(a.N / kPrologueU + 1, kSlotBlocks) : 1;
    gx = nt > gx ? nt : gx;
  }
  hipLaunchKernelGGL(quant_lanes_kernel, dim3(gx, 1, L), dim3(256), 0, s, d);
}

void launch_hist_lanes(const HistArgs* h, const HistArgs* d, int L, int bt, hipStream_t s) {
  if (L <= 0 || h[0].num_items <= 0) return;
  const int32_t slots = h[0].wave_item ? h[0].num_slots : h[0].num_items;
  const bool listed = h[0].active_list != nullptr, presel = listed && h[0].listed_per_xcd >= 0;
  const bool pack = h[0].rowpack != nullptr;
  unsigned gx = (unsigned)((slots + 3) / 4);
  int32_t ns = 1;
  for (int l = 0; l < L; ++l) {
    FDX_LANES_CHECK((h[l].active_list != nullptr) == listed && (h[l].listed_per_xcd >= 0) == presel &&
                     (h[l].rowpack != nullptr) == pack && h[l].lds);
    ns = h[l].nslots > ns ? h[l].nslots : ns;
  }
  if (presel) {
    int32_t most = 0;
    for (int l = 0; l < L; ++l) most = h[l].listed_per_xcd > most ? h[l].listed_per_xcd : most;
    if (most == 0) return;
    gx = (unsigned)((most + 3) / 4 * 8);
  } else if (listed) {
    hipLaunchKernelGGL(hist_count_zero_lanes_kernel, dim3(1, 1, L), dim3(64), 0, s, d);
    hipLaunchKernelGGL(hist_select_lanes_kernel, dim3((slots + 256 * kSelPerThread - 1) / (256 * kSelPerThread), 1, L),
                       dim3(256), 0, s, d);
    const int32_t waves = slots < kListedWaves ? slots : kListedWaves;
    gx = (unsigned)(((waves + 3) / 4 + 7) / 8 * 8);
  }
  const size_t lds = (size_t)4 * 16 * bt * ns * sizeof(unsigned long long);
  const dim3 grid(gx, 1, L), block(256);
#define FDX_HL(B, P) hipLaunchKernelGGL((hist_lds_lanes_kernel<B, P>), grid, block, lds, s, d)
  if (bt == 1) { if (pack) FDX_HL(1, true); else FDX_HL(1, false); }
  else if (bt == 2) { if (pack) FDX_HL(2, true); else FDX_HL(2, false); }
  else { if (pack) FDX_HL(4, true); else FDX_HL(4, false); }
#undef FDX_HL
}

void launch_split_lanes(const SplitArgs* h, const SplitArgs* d, int L, hipStream_t s) {
  unsigned gx = 0;
  for (int l = 0; l < L; ++l) {
    const int64_t n = (int64_t)h[l].num_nodes * h[l].Fa;
    const int64_t waves = (h[l].wide != nullptr && h[l].n_wide > 0) ? (int64_t)h[l].num_nodes * h[l].n_wide : 0;
    const unsigned g = n > 0 ? (unsigned)((n + 255) / 256) + (unsigned)((waves + 3) / 4) : 0;
    gx = g > gx ? g : gx;
  }
  if (L > 0 && gx > 0) hipLaunchKernelGGL(split_all_lanes_kernel, dim3(gx, 1, L), dim3(256), 0, s, d);
}

void launch_split_best_lanes(const SplitBestLane* h, const SplitBestLane* d, int L, hipStream_t s) {
  int32_t gx = 0;
  for (int l = 0; l < L; ++l) gx = (h[l].Fa > 0 && h[l].nodes > gx) ? h[l].nodes : gx;
  if (L > 0 && gx > 0) hipLaunchKernelGGL(split_best_lanes_kernel, dim3(gx, 1, L), dim3(kBestThreads), 0, s, d);
}

void launch_split_best_plan_lanes(const SplitBestPlanLane* h, const SplitBestPlanLane* d, int L, hipStream_t s) {
  int32_t gx = 0;
  for (int l = 0; l < L; ++l) {
    FDX_LANES_CHECK(h[l].b.nodes > 0 && h[l].b.Fa > 0);
    gx = h[l].b.nodes > gx ? h[l].b.nodes : gx;
  }
  if (L > 0) hipLaunchKernelGGL(split_best_plan_lanes_kernel, dim3(gx, 1, L), dim3(kBestThreads), 0, s, d);
}

void launch_copy_lanes(const CopyLane* h, const CopyLane* d, int L, hipStream_t s) {
  int64_t most = 0;
  for (int l = 0; l < L; ++l) most = h[l].bytes > most ? h[l].bytes : most;
  if (L <= 0 || most <= 0) return;
  const int64_t blocks = (most / 8 + 255) / 256;
  hipLaunchKernelGGL(copy_lanes_kernel, dim3((unsigned)(blocks < 1 ? 1 : (blocks > 64 ? 64 : blocks)), 1, L), dim3(256), 0,
                     s, d);
}

void launch_stage_copy(void* dst, const void* src, int64_t bytes, hipStream_t s) {
  const int64_t n = bytes / 16;
  if (n <= 0) return;
  const int64_t blocks = (n + 255) / 256;
  hipLaunchKernelGGL(stage_copy_kernel, dim3((unsigned)(blocks > 32 ? 32 : blocks)), dim3(256), 0, s,
                     reinterpret_cast<uint4*>(dst), reinterpret_cast<const uint4*>(src), n);
}

void launch_root_send_lanes(const RootSendLane* d, int L, hipStream_t s) {
  if (L > 0) hipLaunchKernelGGL(root_send_lanes_kernel, dim3(1, 1, L), dim3(64), 0, s, d);
}

void launch_level_plan_lanes(const LevelPlanArgs* d, int L, hipStream_t s) {
  if (L > 0) hipLaunchKernelGGL(level_plan_lanes_kernel, dim3(1, 1, L), dim3(64), 0, s, d);
}

void launch_select_groups_lanes(const SelectArgs* h, const SelectArgs* d, int L, hipStream_t s) {
  if (L <= 0 || h[0].n <= 0) return;
  int32_t most = 0;
  for (int g = 0; g < h[0].n; ++g) most = h[0].num_slots[g] > most ? h[0].num_slots[g] : most;
  for (int l = 0; l < L; ++l) FDX_LANES_CHECK(h[l].n == h[0].n);
  if (most <= 0) return;
  hipLaunchKernelGGL(hist_select_groups_lanes_kernel,
                     dim3((most + 256 * kSelPerThread - 1) / (256 * kSelPerThread), h[0].n, L), dim3(256), 0, s, d);
}

void launch_partition_lanes(const PartColsLane* h, const PartColsLane* d, const PartitionArgs* dp, int L,
                            hipStream_t s) {
  if (L <= 0) return;
  int32_t gx = 0;
  for (int l = 0; l < L; ++l) {
    FDX_LANES_CHECK(h[l].a.N == h[0].a.N && (h[l].a.node_parent != nullptr) == (h[0].a.node_parent != nullptr));
    gx = h[l].max_splits * h[l].wps > gx ? h[l].max_splits * h[l].wps : gx;
  }
  const auto cols = [&] {
    if (gx > 0) hipLaunchKernelGGL(partition_cols_lanes_kernel, dim3(gx, 1, L), dim3(256), 0, s, d);
  };
  if (h[0].a.node_parent != nullptr) cols();
  if (h[0].a.N > 0) {
    int mode = 0;                        // (a counting variant if a lane asks for counts)
    for (int l = 0; l < L; ++l) {
      const PartitionArgs& x = h[l].a;
      const int m = x.count_work != nullptr ? 1 : x.rows_out != nullptr ? 3 : x.node_counts != nullptr ? 2 : 0;
      FDX_LANES_CHECK(mode == 0 || m == 0 || m == mode);
      mode = m ? m : mode;
    }
    const dim3 grid(grid_for((h[0].a.N + kPartRows - 1) / kPartRows), 1, L);
    if (mode == 1)
      hipLaunchKernelGGL(partition_default_lanes_kernel<1>, grid, dim3(256), 0, s, dp);
    else if (mode == 3)
      hipLaunchKernelGGL(partition_default_lanes_kernel<3>, grid, dim3(256), 0, s, dp);
    else if (mode == 2)
      hipLaunchKernelGGL(partition_default_lanes_kernel<2>, grid, dim3(256), 0, s, dp);
    else
      hipLaunchKernelGGL(partition_default_lanes_kernel<0>, grid, dim3(256), 0, s, dp);
  }
  if (h[0].a.node_parent == nullptr) cols();
}

}  // namespace fdx

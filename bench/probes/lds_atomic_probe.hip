// LDS atomic / read-modify-write throughput on one MI355X (gfx950): what one wave-instruction of
// each form costs when every CU streams them, for the row-group histogram pass
// (csrc/row_kernels.hip rg_hist_kernel: two ds_add_u64 per entry into 8192-bin int64 tables).
//
//   hipcc --offload-arch=gfx950 -O3 -o bench/probes/lds_atomic_probe bench/probes/lds_atomic_probe.hip
//   bench/probes/lds_atomic_probe            (prints one JSON line per variant)
//
// Every variant: 1024 threads per workgroup (one workgroup per CU holding a 128 KB table, as the
// pass), 2048 workgroups, ITERS wave-instructions per wave. Addresses come from a per-lane hash
// (uniform over the table) unless the variant says otherwise. cycles/instr = CU-cycles spent per
// wave-instruction of the variant = (kernel time * 2.4 GHz * 256 CUs) / (wave-instructions).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

constexpr int kBins = 8192;
constexpr int kThreads = 1024;
constexpr int kIters = 4096;

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}

// mode: 0 ds_add_u64 random | 1 ds_add_u32 random (16K words) | 2 ds_add_u64 conflict-free
// (lane-linear) | 3 ds_add_u64 one address per wave | 4 ds_add_u64, one lane active |
// 5 ds_read_b64 + ds_write_b64 random (no atomicity) | 6 two ds_add_u64 (g, h tables) random |
// 7 ds_add_u64 random over the hottest 256 bins | 8 ds_add_u32 x4 random (split hi/lo of g, h) |
// 9 ds_add_u64 conflict-free only if lanes are banked in 4 groups of 16 (lane l and l + 16 share a
// bank pair) | 10 hot bins with 16 lane replicas: slot (random bin of 128) * 16 + lane % 16 |
// 11 as 10 with 32 replicas over 64 bins (conflict-free for 2 groups of 32 as well)
template <int MODE>
__global__ __launch_bounds__(kThreads) void probe(unsigned long long* out, uint32_t seed) {
  __shared__ unsigned long long hg[kBins];
  __shared__ unsigned long long hh[kBins];
  uint32_t* w32 = reinterpret_cast<uint32_t*>(hg);
  for (int i = threadIdx.x; i < kBins; i += kThreads) { hg[i] = 0; hh[i] = 0; }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  uint32_t h = hash32(seed ^ (blockIdx.x * kThreads + threadIdx.x));
  const unsigned long long v = 3;
  if (MODE == 4 && lane != 0) return;
#pragma unroll 8
  for (int it = 0; it < kIters; ++it) {
    h = hash32(h + it);
    if (MODE == 0) {
      atomicAdd(&hg[h & (kBins - 1)], v);
    } else if (MODE == 1) {
      atomicAdd(&w32[h & (2 * kBins - 1)], 3u);
    } else if (MODE == 2) {
      atomicAdd(&hg[((it & 63) * 64 + lane) & (kBins - 1)], v);
    } else if (MODE == 3) {
      atomicAdd(&hg[(it * 97) & (kBins - 1)], v);
    } else if (MODE == 4) {
      atomicAdd(&hg[h & (kBins - 1)], v);
    } else if (MODE == 5) {
      const uint32_t b = h & (kBins - 1);
      hg[b] = hg[b] + v;
    } else if (MODE == 6) {
      const uint32_t b = h & (kBins - 1);
      atomicAdd(&hg[b], v);
      atomicAdd(&hh[b], v);
    } else if (MODE == 7) {
      atomicAdd(&hg[h & 255], v);
    } else if (MODE == 9) {
      atomicAdd(&hg[((lane & 15) + 32 * (lane >> 4) + 128 * (it & 31)) & (kBins - 1)], v);
    } else if (MODE == 10) {
      atomicAdd(&hg[((h & 127) * 16 + (lane & 15)) & (kBins - 1)], v);
    } else if (MODE == 11) {
      atomicAdd(&hg[((h & 63) * 32 + (lane & 31)) & (kBins - 1)], v);
    } else if (MODE == 8) {
      const uint32_t b = h & (kBins - 1);
      atomicAdd(&w32[2 * b], 3u);
      atomicAdd(&w32[2 * b + 1], 3u);
      atomicAdd(reinterpret_cast<uint32_t*>(hh) + 2 * b, 3u);
      atomicAdd(reinterpret_cast<uint32_t*>(hh) + 2 * b + 1, 3u);
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = hg[seed & (kBins - 1)] + hh[1];
}

template <int MODE>
void run(const char* name, int instr_per_iter, int active_waves_per_wg) {
  const int blocks = 2048;
  unsigned long long* out;
  hipMalloc(&out, blocks * sizeof(unsigned long long));
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  probe<MODE><<<blocks, kThreads>>>(out, 1);      // warm
  hipEventRecord(a);
  probe<MODE><<<blocks, kThreads>>>(out, 7);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  const double instr = (double)blocks * active_waves_per_wg * kIters * instr_per_iter;
  const double cu_cycles = ms * 1e-3 * 2.4e9 * 256;
  printf("{\"variant\": \"%s\", \"ms\": %.3f, \"wave_instr\": %.4g, \"cu_cycles_per_wave_instr\": %.2f}\n", name, ms,
         instr, cu_cycles / instr);
  hipFree(out);
}

int main() {
  run<0>("ds_add_u64 random", 1, 16);
  run<1>("ds_add_u32 random", 1, 16);
  run<2>("ds_add_u64 conflict-free", 1, 16);
  run<3>("ds_add_u64 same address per wave", 1, 16);
  run<4>("ds_add_u64 one active lane", 1, 16);
  run<5>("ds_read_b64+ds_write_b64 random (non-atomic)", 1, 16);
  run<6>("2x ds_add_u64 random (g, h tables)", 2, 16);
  run<7>("ds_add_u64 random over 256 hot bins", 1, 16);
  run<8>("4x ds_add_u32 random (hi/lo g, h)", 4, 16);
  run<9>("ds_add_u64 bank-pair shared by lanes l, l+16", 1, 16);
  run<10>("ds_add_u64 hot bins x16 lane replicas", 1, 16);
  run<11>("ds_add_u64 hot bins x32 lane replicas", 1, 16);
  return 0;
}

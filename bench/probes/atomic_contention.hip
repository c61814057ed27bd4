// Cost of device-scope 64-bit atomics issued once per workgroup to the SAME address versus spread
// over 32 addresses (one per 128-byte line), versus plain per-workgroup stores, for the GBDT round
// prologue (grad_max_kernel / quant_kernel). Each workgroup of 256 threads also streams `rows`
// rows of 20 bytes so the kernels resemble the real passes.
// Build: hipcc --offload-arch=gfx950 -O3 -o /tmp/atomic_contention bench/probes/atomic_contention.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                               \
    }                                                                             \
  } while (0)

// mode 0: no cross-workgroup result; 1: plain store per workgroup; 2: atomic max to one address;
// 3: atomic max spread over 32 lines (blockIdx % 32)
__global__ __launch_bounds__(256) void probe(const double* in, float* out, int64_t n, unsigned long long* dst, int mode) {
  double m = 0.0;
  for (int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x; r < n; r += (int64_t)gridDim.x * 256) {
    const double v = in[r];
    out[r] = (float)v;
    m = fmax(m, fabs(v));
  }
  for (int o = 32; o > 0; o >>= 1) m = fmax(m, __shfl_xor(m, o, 64));
  __shared__ double s[4];
  if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x != 0) return;
  m = fmax(fmax(s[0], s[1]), fmax(s[2], s[3]));
  const unsigned long long bits = (unsigned long long)__double_as_longlong(m);
  if (mode == 1) dst[16 * blockIdx.x] = bits;
  if (mode == 2) { atomicMax(dst, bits); atomicMax(dst + 1, bits); }
  if (mode == 3) { atomicMax(dst + 16 * (blockIdx.x & 31), bits); atomicMax(dst + 16 * (blockIdx.x & 31) + 1, bits); }
}

int main() {
  const int64_t n = 1 << 20;
  double* in;
  float* out;
  unsigned long long* dst;
  CHECK(hipMalloc(&in, n * sizeof(double)));
  CHECK(hipMalloc(&out, n * sizeof(float)));
  CHECK(hipMalloc(&dst, 16 * 8192 * sizeof(unsigned long long)));
  CHECK(hipMemset(in, 0, n * sizeof(double)));
  CHECK(hipMemset(dst, 0, 16 * 8192 * sizeof(unsigned long long)));
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  const char* names[4] = {"none", "store", "atomic_same", "atomic_spread32"};
  for (int blocks : {128, 256, 512, 1024, 2048, 4096}) {
    for (int mode = 0; mode < 4; ++mode) {
      for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(probe, dim3(blocks), dim3(256), 0, 0, in, out, n, dst, mode);
      const int reps = 50;
      CHECK(hipEventRecord(a, 0));
      for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(probe, dim3(blocks), dim3(256), 0, 0, in, out, n, dst, mode);
      CHECK(hipEventRecord(b, 0));
      CHECK(hipEventSynchronize(b));
      float ms = 0.f;
      CHECK(hipEventElapsedTime(&ms, a, b));
      std::printf("{\"rows\": %lld, \"blocks\": %d, \"mode\": \"%s\", \"us_per_launch\": %.2f}\n", (long long)n, blocks,
                  names[mode], 1000.0 * ms / reps);
    }
  }
  CHECK(hipFree(in));
  CHECK(hipFree(out));
  CHECK(hipFree(dst));
  return 0;
}

// Probe: operand / accumulator lane layout of the gfx950 i8 MFMAs used by the histogram engine.
// Hypothesis (same k-map for A and B, so any k permutation cancels in A.B):
//   16x16x64: lane l holds A[r = l&15][k = 16*(l>>4) + j], B[k][c = l&15], j = 0..15 (16 bytes);
//             C[row = 4*(l>>4) + i][col = l&15], i = 0..3.
//   32x32x32: lane l holds A[r = l&31][k = 16*(l>>5) + j], B[k][c = l&31];
//             C[row = (i&3) + 8*(i>>2) + 4*(l>>5)][col = l&31], i = 0..15.
// Random int8 data in [-128,127]; prints PASS/FAIL per shape.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));

__global__ void k16(const int8_t* A, const int8_t* B, int* C) {   // A [16][64], B [64][16], C [16][16]
  const int l = threadIdx.x, r = l & 15, g = l >> 4;
  union { int8_t b[16]; i32x4 v; } a, b;
  for (int j = 0; j < 16; ++j) { a.b[j] = A[r * 64 + 16 * g + j]; b.b[j] = B[(16 * g + j) * 16 + r]; }
  i32x4 acc = {0, 0, 0, 0};
  acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(a.v, b.v, acc, 0, 0, 0);
  for (int i = 0; i < 4; ++i) C[(4 * g + i) * 16 + r] = acc[i];
}

__global__ void k32(const int8_t* A, const int8_t* B, int* C) {   // A [32][32], B [32][32], C [32][32]
  const int l = threadIdx.x, r = l & 31, h = l >> 5;
  union { int8_t b[16]; i32x4 v; } a, b;
  for (int j = 0; j < 16; ++j) { a.b[j] = A[r * 32 + 16 * h + j]; b.b[j] = B[(16 * h + j) * 32 + r]; }
  i32x16 acc = {};
  acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(a.v, b.v, acc, 0, 0, 0);
  for (int i = 0; i < 16; ++i) C[((i & 3) + 8 * (i >> 2) + 4 * h) * 32 + r] = acc[i];
}

static bool run(int M, int K, int N, bool big) {
  std::vector<int8_t> A(M * K), B(K * N);
  srand(M * 7 + K);
  for (auto& x : A) x = (int8_t)(rand() & 255);
  for (auto& x : B) x = (int8_t)(rand() & 255);
  int8_t *dA, *dB; int* dC;
  hipMalloc(&dA, A.size()); hipMalloc(&dB, B.size()); hipMalloc(&dC, M * N * 4);
  hipMemcpy(dA, A.data(), A.size(), hipMemcpyHostToDevice);
  hipMemcpy(dB, B.data(), B.size(), hipMemcpyHostToDevice);
  hipMemset(dC, 0, M * N * 4);
  if (big) hipLaunchKernelGGL(k32, dim3(1), dim3(64), 0, 0, dA, dB, dC);
  else hipLaunchKernelGGL(k16, dim3(1), dim3(64), 0, 0, dA, dB, dC);
  std::vector<int> C(M * N);
  hipMemcpy(C.data(), dC, C.size() * 4, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < M; ++i)
    for (int j = 0; j < N; ++j) {
      int s = 0;
      for (int k = 0; k < K; ++k) s += (int)A[i * K + k] * (int)B[k * N + j];
      if (s != C[i * N + j]) ++bad;
    }
  printf("%s %dx%dx%d: %s (%d mismatches)\n", big ? "mfma_i32_32x32x32_i8" : "mfma_i32_16x16x64_i8", M, N, K,
         bad ? "FAIL" : "PASS", bad);
  hipFree(dA); hipFree(dB); hipFree(dC);
  return bad == 0;
}

int main() {
  const bool a = run(16, 64, 16, false);
  const bool b = run(32, 32, 32, true);
  return (a && b) ? 0 : 1;
}

// i8-MFMA histogram building blocks shared by tree_kernels.hip and blk_kernels.hip (gfx950):
// SWAR one-hot A operands, slot-masked digit B operands, byte transposition, wave-local LDS sync.
// v_mfma_i32_16x16x64_i8 tile: lane l, r = l & 15 (A row / B column), g = l >> 4 (16-entry K group).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fdx {
namespace {
constexpr int kWave = 64;

typedef int i32x4 __attribute__((ext_vector_type(4)));

// 0x80 in every byte of x that is zero, 0x00 elsewhere (SWAR, no carries across bytes).
__device__ __forceinline__ uint32_t zero_bytes80(uint32_t x) {
  const uint32_t y = (x & 0x7f7f7f7fu) + 0x7f7f7f7fu;
  return ~(y | x | 0x7f7f7f7fu);
}
// One-hot A operand bytes (0x80 where the key byte equals the lane's key) when every byte of kv
// and of the key is < 128: 0x80 - (kv ^ key) per byte lies in [1, 128] (no borrow between bytes)
// and has its high bit set iff the bytes are equal. (kv ^ ~key) + 0x80808081 is that difference
// mod 2^32, a single v_xad_u32, so one dword of A costs 2 VALU instead of 5.
__device__ __forceinline__ uint32_t onehot7(uint32_t kv7, uint32_t nkey) {
  return ((kv7 ^ nkey) + 0x80808081u) & 0x80808080u;
}
template <int BT>
__device__ __forceinline__ void onehot_a(uint4 kv, uint32_t key0, bool fast, i32x4 A[BT]) {
  if (fast) {
    const uint4 k7 = make_uint4(kv.x & 0x7f7f7f7fu, kv.y & 0x7f7f7f7fu, kv.z & 0x7f7f7f7fu, kv.w & 0x7f7f7f7fu);
#pragma unroll
    for (int bt = 0; bt < BT; ++bt) {
      const uint32_t nk = ~((key0 + 16u * bt) * 0x01010101u);
      A[bt] = i32x4{(int)onehot7(k7.x, nk), (int)onehot7(k7.y, nk), (int)onehot7(k7.z, nk), (int)onehot7(k7.w, nk)};
    }
  } else {
#pragma unroll
    for (int bt = 0; bt < BT; ++bt) {
      const uint32_t rep = (key0 + 16u * bt) * 0x01010101u;
      A[bt] = i32x4{(int)zero_bytes80(kv.x ^ rep), (int)zero_bytes80(kv.y ^ rep), (int)zero_bytes80(kv.z ^ rep),
                    (int)zero_bytes80(kv.w ^ rep)};
    }
  }
}
// 0xff in every byte of x that is zero
__device__ __forceinline__ uint32_t zero_bytes_ff(uint32_t x) {
  const uint32_t z = zero_bytes80(x);
  return z | (z - (z >> 7));
}
// Slot masks for B with NP = 4 (2 slots per 16-column tile, lane's slot_sub b): a row with slot
// byte s (0..15; 0xff = not built) feeds column tile ct iff s = 2 ct + b. Per K-step the digits
// are masked once to the live rows of parity b (live_parity_mask), then per tile one byte-
// permute table lookup on s >> 1 selects tile ct (ct_select): 2 VALU per dword per tile.
__device__ __forceinline__ uint32_t live_parity_mask(uint32_t s, uint32_t pat) {   // pat = (0x80 | (b ^ 1)) * 0x01010101
  const uint32_t u = (s ^ pat) & 0x81818181u;
  return ((u >> 7) & u & 0x01010101u) * 0xffu;
}
__device__ __forceinline__ uint32_t ct_select(uint32_t sel, int ct) {            // sel = (s >> 1) & 0x07070707
  const uint32_t lo = ct < 4 ? 0xffu << (8 * ct) : 0u, hi = ct < 4 ? 0u : 0xffu << (8 * (ct - 4));
  return __builtin_amdgcn_perm(hi, lo, sel);
}
template <int CT, int NP>
__device__ __forceinline__ void slot_masked_b(uint4 d, uint4 sv, int slot_sub, i32x4 B[CT]) {
  if constexpr (NP == 4) {
    const uint32_t pat = (0x80u | (uint32_t)(slot_sub ^ 1)) * 0x01010101u;
    const uint4 dm = make_uint4(d.x & live_parity_mask(sv.x, pat), d.y & live_parity_mask(sv.y, pat),
                                d.z & live_parity_mask(sv.z, pat), d.w & live_parity_mask(sv.w, pat));
    const uint4 sel = make_uint4((sv.x >> 1) & 0x07070707u, (sv.y >> 1) & 0x07070707u, (sv.z >> 1) & 0x07070707u,
                                 (sv.w >> 1) & 0x07070707u);
#pragma unroll
    for (int ct = 0; ct < CT; ++ct)
      B[ct] = i32x4{(int)(dm.x & ct_select(sel.x, ct)), (int)(dm.y & ct_select(sel.y, ct)),
                    (int)(dm.z & ct_select(sel.z, ct)), (int)(dm.w & ct_select(sel.w, ct))};
  } else {
    constexpr int SPT = 16 / (2 * NP);
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
      const uint32_t rep = (uint32_t)(ct * SPT + slot_sub) * 0x01010101u;
      B[ct] = i32x4{(int)(d.x & zero_bytes_ff(sv.x ^ rep)), (int)(d.y & zero_bytes_ff(sv.y ^ rep)),
                    (int)(d.z & zero_bytes_ff(sv.z ^ rep)), (int)(d.w & zero_bytes_ff(sv.w ^ rep))};
    }
  }
}

// byte p of a, b, c, d -> [a.p, b.p, c.p, d.p]
__device__ __forceinline__ uint32_t gather_byte(uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t p) {
  const uint32_t lo = __builtin_amdgcn_perm(b, a, 0x0c0c0000u | ((4u + p) << 8) | p);
  const uint32_t hi = __builtin_amdgcn_perm(d, c, ((4u + p) << 24) | (p << 16) | 0x0c0cu);
  return lo | hi;
}

__device__ __forceinline__ void lds_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

}  // namespace
}  // namespace fdx

// Device-side MurmurHash3 x64_128 arithmetic for gfx950.
//
// Restates the reference's per-key hash (/root/reference/src/murmurhash3.c:75-160,
// called by shf_make_hash() at /root/reference/src/shf.c:456 with seed 12345) as
// wavefront-friendly pieces:
//   * mix_k1 / mix_k2  -- the independent per-block multiplies (murmurhash3.c:97, :101)
//   * chain_block      -- the serial h1/h2 chain (murmurhash3.c:97-103 after the k mixes)
//   * finish           -- length fold + fmix64 + cross adds (murmurhash3.c:147-159)
// CDNA4 has no 64-bit integer multiply: each u64 x const product lowers to one
// v_mad_u64_u32 (lo x lo, full 64-bit) plus two v_mul_lo_u32 for the cross terms.
// Rotates lower to two v_alignbit_b32; `h * 5 + c` to a shift-add.
#pragma once
#include <stdint.h>

namespace shfhb {

constexpr uint64_t kC1 = 0x87c37b91114253d5ull;  // murmurhash3.c:84
constexpr uint64_t kC2 = 0x4cf5ad432745937full;  // murmurhash3.c:85
constexpr uint64_t kN1 = 0x52dce729ull;          // murmurhash3.c:99
constexpr uint64_t kN2 = 0x38495ab5ull;          // murmurhash3.c:103
constexpr uint64_t kF1 = 0xff51afd7ed558ccdull;  // murmurhash3.c:65
constexpr uint64_t kF2 = 0xc4ceb9fe1a85ec53ull;  // murmurhash3.c:67

typedef uint32_t u32x2_mix __attribute__((ext_vector_type(2)));

// {lo, hi} -> u64 as a register pair. Written as a bit cast: the shift-or form
// lets the compiler split a later 64-bit add into two (one per half, plus a
// zeroed register each), e.g. in rotl64(...) + h2.
__device__ __forceinline__ uint64_t pack64(uint32_t lo, uint32_t hi) {
  return __builtin_bit_cast(uint64_t, (u32x2_mix){lo, hi});
}

// Rotates as two v_alignbit_b32 and `x * 5` as one v_lshl_add_u64, with the
// h1/h2 chain left undistributed (two *5 per block instead of four): k_span
// +7.8 %, k_vround +5.2 % on U[8,512] keys, fixed-length kernels unchanged
// (HBM-bound) -- profiles/r1/ab_asm/. (The compiler's own lowering -- a 64-bit
// shift, a 32-bit shift and an or per rotate, two v_mad_u64_u32 per *5 -- is in
// git history.)
// r is a compile-time constant after inlining.
__device__ __forceinline__ uint64_t rotl64(uint64_t x, int r) {
  const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  if (r < 32)
    return pack64(__builtin_amdgcn_alignbit(lo, hi, 32 - r), __builtin_amdgcn_alignbit(hi, lo, 32 - r));
  return pack64(__builtin_amdgcn_alignbit(hi, lo, 64 - r), __builtin_amdgcn_alignbit(lo, hi, 64 - r));
}
// x * 5 as one v_lshl_add_u64 (x << 2) + x.
__device__ __forceinline__ uint64_t mul5(uint64_t x) {
  uint64_t r;
  asm("v_lshl_add_u64 %0, %1, 2, %1" : "=v"(r) : "v"(x));
  return r;
}

__device__ __forceinline__ uint64_t mix_k1(uint64_t k) { return rotl64(k * kC1, 31) * kC2; }
__device__ __forceinline__ uint64_t mix_k2(uint64_t k) { return rotl64(k * kC2, 33) * kC1; }

struct State {
  uint64_t h1, h2;
};

// One 16-byte body block whose k1/k2 are already mixed (murmurhash3.c:97-103):
//   h1 = (rotl(h1 ^ m1, 27) + h2) * 5 + N1
//   h2 = (rotl(h2 ^ m2, 31) + h1) * 5 + N2
__device__ __forceinline__ void chain_block(State& s, uint64_t m1, uint64_t m2) {
  s.h1 = mul5(rotl64(s.h1 ^ m1, 27) + s.h2) + kN1;
  s.h2 = mul5(rotl64(s.h2 ^ m2, 31) + s.h1) + kN2;
}

__device__ __forceinline__ void body_block(State& s, uint64_t k1, uint64_t k2) {
  chain_block(s, mix_k1(k1), mix_k2(k2));
}

// Tail of 1..15 bytes already assembled little-endian and zero-masked
// (murmurhash3.c:118-138): bytes 8..14 feed k2, bytes 0..7 feed k1.
__device__ __forceinline__ void tail_block(State& s, uint64_t t1, uint64_t t2, uint32_t rem) {
  if (rem > 8) s.h2 ^= mix_k2(t2);
  if (rem > 0) s.h1 ^= mix_k1(t1);
}

__device__ __forceinline__ uint64_t fmix64(uint64_t k) {  // murmurhash3.c:62-71
  k ^= k >> 33;
  k *= kF1;
  k ^= k >> 33;
  k *= kF2;
  k ^= k >> 33;
  return k;
}

// murmurhash3.c:147-156. `len` is the reference's `const int len` widened to
// u64 (sign extension only matters for len >= 2^31, which the ABI rejects).
__device__ __forceinline__ void finish(State& s, uint32_t len) {
  const uint64_t l = (uint64_t)(int64_t)(int32_t)len;
  s.h1 ^= l;
  s.h2 ^= l;
  s.h1 += s.h2;
  s.h2 += s.h1;
  s.h1 = fmix64(s.h1);
  s.h2 = fmix64(s.h2);
  s.h1 += s.h2;
  s.h2 += s.h1;
}

// SHF_HASH fields read by put/find (shf.c:800-803, :893-896), packed in the
// SHF_UID bit order (shf.private.h:170-178) with rnd in the high word.
__device__ __forceinline__ uint64_t uid_parts(const State& s) {
  const uint32_t lo = (uint32_t)s.h1, hi = (uint32_t)(s.h1 >> 32);
  const uint32_t win = lo & 0xffu;
  const uint32_t tab = (lo >> 16) & 0x7ffu;
  const uint32_t row = hi & 0x1ffu;
  const uint32_t rnd = (uint32_t)s.h2 & 0x1fffffu;
  return (uint64_t)(win | (tab << 8) | (row << 19)) | ((uint64_t)rnd << 32);
}

}  // namespace shfhb

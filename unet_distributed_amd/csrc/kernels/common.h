// Shared device helpers for the gfx950 (CDNA4, MI355X) kernels.
//
// Everything here is written for wave64 + MFMA on gfx950 only: no CUDA
// shims, no dual-platform paths.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace unet {

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short short4v __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

#define LDS_PTR(T, p) ((__attribute__((address_space(3))) T*)(p))

__device__ __forceinline__ float bf2f(bf16 x) { return (float)x; }
__device__ __forceinline__ bf16 f2bf(float x) { return (bf16)x; }

__device__ __forceinline__ float bits2f(uint16_t b) {
  return __uint_as_float(((uint32_t)b) << 16);
}

// unpack 8 bf16 held in a 16-byte vector into floats
__device__ __forceinline__ void unpack8(const u32x4& v, float* f) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(v[i] << 16);
    f[2 * i + 1] = __uint_as_float(v[i] & 0xffff0000u);
  }
}

typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

// one v_cvt_pk_bf16_f32 (round-to-nearest-even) for two values
__device__ __forceinline__ uint32_t pack2bf(float a, float b) {
  const f32x2 v = {a, b};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2));
}

__device__ __forceinline__ u32x4 pack8(const float* f) {
  u32x4 r;
#pragma unroll
  for (int i = 0; i < 4; ++i) r[i] = pack2bf(f[2 * i], f[2 * i + 1]);
  return r;
}

// Counter-based dropout hash (murmur3 fmix32 of (index, seed, salt)).  The
// PyTorch reference reproduces it bit-for-bit
// (models/reference.py::_hash_u32) so both paths draw the same keep-mask.
__device__ __forceinline__ uint32_t drop_hash(uint64_t idx, uint32_t seed, uint32_t salt) {
  uint32_t x = (uint32_t)idx ^ (seed * 0x9E3779B9u + salt * 0x85EBCA6Bu);
  x ^= (uint32_t)(idx >> 32) * 0xC2B2AE35u;
  x ^= x >> 16;
  x *= 0x85EBCA6Bu;
  x ^= x >> 13;
  x *= 0xC2B2AE35u;
  x ^= x >> 16;
  return x;
}

__device__ __forceinline__ f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Bijective XCD-aware block remap (cdna_hip_programming.md §5 "XCD swizzle
// must be bijective"): blocks dealt round-robin over 8 XCDs are renumbered so
// every XCD receives a contiguous range of logical tiles (neighbouring tiles
// share operand panels in that XCD's L2).
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg / 8, r = nwg % 8;
  const int xcd = bid % 8, idx = bid / 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

}  // namespace unet

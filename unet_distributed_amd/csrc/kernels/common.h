// Shared device helpers for the gfx950 (CDNA4, MI355X) kernels.
//
// Everything here is written for wave64 + MFMA on gfx950 only: no CUDA
// shims, no dual-platform paths.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "conv_params.h"

// Kernel launch of every launcher (skipped under dry dispatch, conv_params.h)
#define UNET_LAUNCH(...)                                        \
  do {                                                          \
    if (!::unet_types::dry_dispatch()) hipLaunchKernelGGL(__VA_ARGS__); \
  } while (0)

// 16-bit activation / weight-copy element type.  Every kernel TU is compiled twice
// (native/build.py): as bf16 in namespace `unet` and, with -DUNET_FP16
// -Dunet=unet_f16, as IEEE fp16 in namespace `unet_f16`.  The two builds share the
// kernel source; only the element type, its conversions and the MFMA opcode
// (v_mfma_f32_16x16x32_{bf16,f16}, identical operand layouts) differ.
namespace unet {

#ifdef UNET_FP16
typedef _Float16 h16;
#else
typedef __bf16 h16;
#endif
typedef h16 h16x8 __attribute__((ext_vector_type(8)));
typedef h16 h16x4 __attribute__((ext_vector_type(4)));
typedef h16 h16x2 __attribute__((ext_vector_type(2)));
typedef short short4v __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

#ifdef UNET_FP16
constexpr uint32_t kOnes2 = 0x3C003C00u;   // two fp16 1.0
#else
constexpr uint32_t kOnes2 = 0x3F803F80u;   // two bf16 1.0
#endif

#define LDS_PTR(T, p) ((__attribute__((address_space(3))) T*)(p))

// status of the launches a launcher just issued (success under dry dispatch)
inline hipError_t launch_status() { return ::unet_types::dry_dispatch() ? hipSuccess : hipGetLastError(); }

__device__ __forceinline__ float h2f(h16 x) { return (float)x; }
__device__ __forceinline__ h16 f2h(float x) { return (h16)x; }

__device__ __forceinline__ float bits2f(uint16_t b) {
#ifdef UNET_FP16
  return (float)__builtin_bit_cast(_Float16, b);
#else
  return __uint_as_float(((uint32_t)b) << 16);
#endif
}

// unpack 8 16-bit elements held in a 16-byte vector into floats
__device__ __forceinline__ void unpack8(const u32x4& v, float* f) {
#ifdef UNET_FP16
  const f32x8 r = __builtin_convertvector(__builtin_bit_cast(h16x8, v), f32x8);
#pragma unroll
  for (int i = 0; i < 8; ++i) f[i] = r[i];
#else
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(v[i] << 16);
    f[2 * i + 1] = __uint_as_float(v[i] & 0xffff0000u);
  }
#endif
}

// the two 16-bit elements of a 32-bit word as floats
__device__ __forceinline__ f32x2 unpack2(uint32_t w) {
#ifdef UNET_FP16
  return __builtin_convertvector(__builtin_bit_cast(h16x2, w), f32x2);
#else
  return (f32x2){__uint_as_float(w << 16), __uint_as_float(w & 0xffff0000u)};
#endif
}

// one packed convert (round-to-nearest-even) for two values
__device__ __forceinline__ uint32_t pack2h(float a, float b) {
  const f32x2 v = {a, b};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, h16x2));
}

// ReLU of two packed 16-bit floats: the sign bit makes every negative value (and -0)
// a negative int16, so one packed signed max with 0 clamps both
__device__ __forceinline__ uint32_t relu2h(uint32_t w) {
  typedef short s16x2 __attribute__((ext_vector_type(2)));
  const s16x2 v = __builtin_elementwise_max(__builtin_bit_cast(s16x2, w), (s16x2){0, 0});
  return __builtin_bit_cast(uint32_t, v);
}

__device__ __forceinline__ u32x4 pack8(const float* f) {
  u32x4 r;
#pragma unroll
  for (int i = 0; i < 4; ++i) r[i] = pack2h(f[2 * i], f[2 * i + 1]);
  return r;
}

// ReLU masks of 8 packed 16-bit values (bf16 / fp16 alike: > 0 <=> sign bit clear and
// not zero; -0 counts as not positive).  pos_bits: bit e = element e > 0.
__device__ __forceinline__ uint32_t pos_bits(const u32x4& v) {
  // a 16-bit value moved to the top of a word is > 0 as int32 iff its sign bit is clear
  // and it is not zero: one shift / mask and one signed compare per element
  uint32_t b = 0;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    b |= ((int32_t)(v[e] << 16) > 0 ? 1u : 0u) << (2 * e);
    b |= ((int32_t)(v[e] & 0xffff0000u) > 0 ? 1u : 0u) << (2 * e + 1);
  }
  return b;
}
// pos_bits of ReLU outputs (every element +0 or positive, never -0 or negative, e.g.
// relu2h's): nonzero <=> positive, so a packed unsigned min with 1 gives each 16-bit
// half's bit in place and three shift-ors gather them -- 8 VALU instead of ~24.  Bits
// above 7 of the result are not zero (callers store the low byte).
__device__ __forceinline__ uint32_t pos_bits_relu(const u32x4& v) {
  typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
  uint32_t m[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    // (through a scalar copy: __builtin_bit_cast of the vector element lvalue v[e]
    // reads element 0 for every e with this clang)
    const uint32_t w = v[e];
    m[e] = __builtin_bit_cast(uint32_t, __builtin_elementwise_min(__builtin_bit_cast(u16x2, w), (u16x2){1, 1}));
  }
  // bit 2e: element 2e (low half of word e); bit 16 + 2e: element 2e + 1 (high half)
  const uint32_t c = (m[0] | (m[1] << 2)) | ((m[2] | (m[3] << 2)) << 4);
  return c | (c >> 15);
}
// v with element e zeroed unless bit e of `bits` is set
__device__ __forceinline__ u32x4 keep_bits(u32x4 v, uint32_t bits) {
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const uint32_t lo = ((bits >> (2 * e)) & 1u) ? 0xffffu : 0u;
    const uint32_t hi = ((bits >> (2 * e + 1)) & 1u) ? 0xffff0000u : 0u;
    v[e] &= (lo | hi);
  }
  return v;
}
// v with element e zeroed unless element e of the activation m is > 0
__device__ __forceinline__ u32x4 keep_pos(u32x4 v, const u32x4& m) {
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const uint32_t keep_lo = (int32_t)(m[e] << 16) > 0 ? 0xffffu : 0u;
    const uint32_t keep_hi = (int32_t)(m[e] & 0xffff0000u) > 0 ? 0xffff0000u : 0u;
    v[e] &= (keep_lo | keep_hi);
  }
  return v;
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

__device__ __forceinline__ f32x4 mfma16(const h16x8& a, const h16x8& b, const f32x4& c) {
#ifdef UNET_FP16
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
#else
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
#endif
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

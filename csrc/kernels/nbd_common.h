// nbd_common.h — shared device helpers for the gfx950 (CDNA4) kernels of nbdistributed_amd.
//
// Wave64 everywhere (CDNA wavefront = 64 lanes; warpSize folds to 64 on gfx950).  Memory-bound
// kernels move 16 B per lane per access (one dwordx4 = 1 KiB per wave-instruction), the
// coalescing sweet spot on CDNA (cdna_hip_programming.md Guideline 13).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace nbd {

constexpr int kWave = 64;

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));  // MFMA A/B operand: 8 bf16 / f16
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// ---- scalar conversions (bit-exact, round-to-nearest-even; NaN stays NaN) -------------------
__device__ __forceinline__ float bf16_to_f32(uint16_t h) { return __uint_as_float(((uint32_t)h) << 16); }

__device__ __forceinline__ uint16_t f32_to_bf16(float f) {
  // The plain cast lowers to v_cvt_pk_bf16_f32 on gfx950 (keeps NaN a NaN: MI355X_MICROARCH.md,
  // correctness boundaries), unlike the integer rounding trick.
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(uint16_t, b);
}

// Two floats -> one dword of two bf16 (a in the low half) as a single v_cvt_pk_bf16_f32: the
// vector conversion.  Packing two scalar casts with shift / or compiled to 3 instructions a pair
// (the compiler converted each half separately, then merged them with v_and / v_lshl / v_or_sdwa).
typedef float nbd_f2v __attribute__((ext_vector_type(2)));
typedef __bf16 nbd_b2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pack2_bf16(float a, float b) {
  const nbd_f2v f = {a, b};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f, nbd_b2v));
}

__device__ __forceinline__ float f16_to_f32(uint16_t h) { return (float)__builtin_bit_cast(_Float16, h); }
__device__ __forceinline__ uint16_t f32_to_f16(float f) { return __builtin_bit_cast(uint16_t, (_Float16)f); }

// element-type traits: storage type, load-as-float, store-from-float
template <typename T>
struct Elem;
template <>
struct Elem<float> {
  using storage = float;
  static __device__ __forceinline__ float load(const float* p, int64_t i) { return p[i]; }
  static __device__ __forceinline__ void store(float* p, int64_t i, float v) { p[i] = v; }
};
struct bf16_t {
  uint16_t x;
};
struct f16_t {
  uint16_t x;
};
template <>
struct Elem<bf16_t> {
  using storage = uint16_t;
  static __device__ __forceinline__ float load(const bf16_t* p, int64_t i) { return bf16_to_f32(p[i].x); }
  static __device__ __forceinline__ void store(bf16_t* p, int64_t i, float v) { p[i].x = f32_to_bf16(v); }
};
template <>
struct Elem<f16_t> {
  using storage = uint16_t;
  static __device__ __forceinline__ float load(const f16_t* p, int64_t i) { return f16_to_f32(p[i].x); }
  static __device__ __forceinline__ void store(f16_t* p, int64_t i, float v) { p[i].x = f32_to_f16(v); }
};

// ---- 8-element vector load/store as float[8] (16 B or 32 B per lane) ------------------------
template <typename T>
__device__ __forceinline__ void load8(const T* p, float (&v)[8]);
template <>
__device__ __forceinline__ void load8<float>(const float* p, float (&v)[8]) {
  const f32x4 a = *reinterpret_cast<const f32x4*>(p);
  const f32x4 b = *reinterpret_cast<const f32x4*>(p + 4);
  v[0] = a[0]; v[1] = a[1]; v[2] = a[2]; v[3] = a[3];
  v[4] = b[0]; v[5] = b[1]; v[6] = b[2]; v[7] = b[3];
}
template <>
__device__ __forceinline__ void load8<bf16_t>(const bf16_t* p, float (&v)[8]) {
  const u32x4 w = *reinterpret_cast<const u32x4*>(p);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    v[2 * j] = __uint_as_float(w[j] << 16);
    v[2 * j + 1] = __uint_as_float(w[j] & 0xffff0000u);
  }
}
template <>
__device__ __forceinline__ void load8<f16_t>(const f16_t* p, float (&v)[8]) {
  const u32x4 w = *reinterpret_cast<const u32x4*>(p);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    v[2 * j] = f16_to_f32((uint16_t)(w[j] & 0xffffu));
    v[2 * j + 1] = f16_to_f32((uint16_t)(w[j] >> 16));
  }
}

template <typename T>
__device__ __forceinline__ void store8(T* p, const float (&v)[8]);
template <>
__device__ __forceinline__ void store8<float>(float* p, const float (&v)[8]) {
  f32x4 a = {v[0], v[1], v[2], v[3]};
  f32x4 b = {v[4], v[5], v[6], v[7]};
  *reinterpret_cast<f32x4*>(p) = a;
  *reinterpret_cast<f32x4*>(p + 4) = b;
}
template <>
__device__ __forceinline__ void store8<bf16_t>(bf16_t* p, const float (&v)[8]) {
  u32x4 w;
#pragma unroll
  for (int j = 0; j < 4; ++j)
    w[j] = pack2_bf16(v[2 * j], v[2 * j + 1]);
  *reinterpret_cast<u32x4*>(p) = w;
}
template <>
__device__ __forceinline__ void store8<f16_t>(f16_t* p, const float (&v)[8]) {
  u32x4 w;
#pragma unroll
  for (int j = 0; j < 4; ++j)
    w[j] = (uint32_t)f32_to_f16(v[2 * j]) | ((uint32_t)f32_to_f16(v[2 * j + 1]) << 16);
  *reinterpret_cast<u32x4*>(p) = w;
}

// non-temporal loads (a source streamed exactly once)
template <typename T>
__device__ __forceinline__ void load8_nt(const T* p, float (&v)[8]);
template <>
__device__ __forceinline__ void load8_nt<float>(const float* p, float (&v)[8]) {
  const f32x4 a = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p));
  const f32x4 b = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p + 4));
  v[0] = a[0]; v[1] = a[1]; v[2] = a[2]; v[3] = a[3];
  v[4] = b[0]; v[5] = b[1]; v[6] = b[2]; v[7] = b[3];
}
template <>
__device__ __forceinline__ void load8_nt<bf16_t>(const bf16_t* p, float (&v)[8]) {
  const u32x4 w = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    v[2 * j] = __uint_as_float(w[j] << 16);
    v[2 * j + 1] = __uint_as_float(w[j] & 0xffff0000u);
  }
}
template <>
__device__ __forceinline__ void load8_nt<f16_t>(const f16_t* p, float (&v)[8]) {
  const u32x4 w = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    v[2 * j] = f16_to_f32((uint16_t)(w[j] & 0xffffu));
    v[2 * j + 1] = f16_to_f32((uint16_t)(w[j] >> 16));
  }
}

// non-temporal variants (streaming destination: measured +1-3 % on MI355X, copy_bw.hip)
template <typename T>
__device__ __forceinline__ void store8_nt(T* p, const float (&v)[8]);
template <>
__device__ __forceinline__ void store8_nt<float>(float* p, const float (&v)[8]) {
  f32x4 a = {v[0], v[1], v[2], v[3]};
  f32x4 b = {v[4], v[5], v[6], v[7]};
  __builtin_nontemporal_store(a, reinterpret_cast<f32x4*>(p));
  __builtin_nontemporal_store(b, reinterpret_cast<f32x4*>(p + 4));
}
template <>
__device__ __forceinline__ void store8_nt<bf16_t>(bf16_t* p, const float (&v)[8]) {
  u32x4 w;
#pragma unroll
  for (int j = 0; j < 4; ++j)
    w[j] = pack2_bf16(v[2 * j], v[2 * j + 1]);
  __builtin_nontemporal_store(w, reinterpret_cast<u32x4*>(p));
}
template <>
__device__ __forceinline__ void store8_nt<f16_t>(f16_t* p, const float (&v)[8]) {
  u32x4 w;
#pragma unroll
  for (int j = 0; j < 4; ++j)
    w[j] = (uint32_t)f32_to_f16(v[2 * j]) | ((uint32_t)f32_to_f16(v[2 * j + 1]) << 16);
  __builtin_nontemporal_store(w, reinterpret_cast<u32x4*>(p));
}

// ---- wave64 reductions (DPP/permute via __shfl_xor over 64 lanes) ----------------------------
template <typename T, typename Op>
__device__ __forceinline__ T wave_reduce(T v, Op op) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = op(v, __shfl_xor(v, off, kWave));
  return v;
}

}  // namespace nbd

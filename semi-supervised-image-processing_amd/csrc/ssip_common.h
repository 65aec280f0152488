// Shared device/host helpers for the ssip gfx950 kernels.
//
// Element types: every activation kernel is instantiated for two storage
// types, selected at run time by the `dtype` argument of the C ABI
// (include/ssip.h):  SSIP_F32 (float) for the parity path and SSIP_BF16
// (__bf16) for the throughput path.  Accumulation is always fp32.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>
#include <string.h>
#include "../../include/ssip.h"

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) int i32x4;

// ---------------------------------------------------------------------------
// error reporting (thread-local message, negative status codes)
// ---------------------------------------------------------------------------
namespace ssip {
void set_error(const char* fmt, ...);
int check_launch(const char* what);

}  // namespace ssip
#include "stop_event.h"

// Every kernel launch of the library goes through this (hipLaunchKernelGGL's
// arguments).
#define SSIP_KLAUNCH(kernel, grid, block, shm, stream, ...)                                            \
  do {                                                                                                 \
    ::ssip::StopEvent& se_ = ::ssip::stop_event();                                                     \
    if (se_.st != nullptr && (hipStream_t)(stream) == se_.st && ++se_.count == se_.target &&           \
        se_.ev != nullptr) {                                                                           \
      hipExtLaunchKernelGGL(kernel, grid, block, shm, stream, nullptr, se_.ev, 0, __VA_ARGS__);        \
      ++se_.used;                                                                                      \
    } else {                                                                                           \
      hipLaunchKernelGGL(kernel, grid, block, shm, stream, __VA_ARGS__);                               \
    }                                                                                                  \
  } while (0)

#define SSIP_REQUIRE(cond, code, ...)        \
  do {                                       \
    if (!(cond)) {                           \
      ::ssip::set_error(__VA_ARGS__);        \
      return (code);                         \
    }                                        \
  } while (0)

// ---------------------------------------------------------------------------
// scalar conversions
// ---------------------------------------------------------------------------
template <typename T> __device__ __forceinline__ float to_f32(T v);
template <> __device__ __forceinline__ float to_f32<float>(float v) { return v; }
template <> __device__ __forceinline__ float to_f32<__bf16>(__bf16 v) { return (float)v; }

template <typename T> __device__ __forceinline__ T from_f32(float v);
template <> __device__ __forceinline__ float from_f32<float>(float v) { return v; }
template <> __device__ __forceinline__ __bf16 from_f32<__bf16>(float v) { return (__bf16)v; }

// 8-element vector of T, moved as 16 B (bf16) or 2x16 B (f32)
template <typename T> struct Vec8;
template <> struct Vec8<__bf16> {
  i32x4 v;
  __device__ __forceinline__ void zero() { v = (i32x4){0, 0, 0, 0}; }
  __device__ __forceinline__ void load(const __bf16* p) { v = *reinterpret_cast<const i32x4*>(p); }
  __device__ __forceinline__ void store(__bf16* p) const { *reinterpret_cast<i32x4*>(p) = v; }
  __device__ __forceinline__ float get(int j) const {
    const __bf16* e = reinterpret_cast<const __bf16*>(&v);
    return (float)e[j];
  }
  __device__ __forceinline__ void set(int j, float f) {
    __bf16* e = reinterpret_cast<__bf16*>(&v);
    e[j] = (__bf16)f;
  }
};
template <> struct Vec8<float> {
  i32x4 v0, v1;
  __device__ __forceinline__ void zero() { v0 = (i32x4){0, 0, 0, 0}; v1 = v0; }
  __device__ __forceinline__ void load(const float* p) {
    v0 = reinterpret_cast<const i32x4*>(p)[0];
    v1 = reinterpret_cast<const i32x4*>(p)[1];
  }
  __device__ __forceinline__ void store(float* p) const {
    reinterpret_cast<i32x4*>(p)[0] = v0;
    reinterpret_cast<i32x4*>(p)[1] = v1;
  }
  __device__ __forceinline__ float get(int j) const {
    const float* e = j < 4 ? reinterpret_cast<const float*>(&v0) : reinterpret_cast<const float*>(&v1);
    return e[j & 3];
  }
  __device__ __forceinline__ void set(int j, float f) {
    float* e = j < 4 ? reinterpret_cast<float*>(&v0) : reinterpret_cast<float*>(&v1);
    e[j & 3] = f;
  }
};

// 8 consecutive floats (32-B aligned: channel chunks of 8) as two 16-B loads
__device__ __forceinline__ void load_f8(float (&d)[8], const float* p) {
  typedef __attribute__((ext_vector_type(4))) float f4;
  const f4 a = reinterpret_cast<const f4*>(p)[0];
  const f4 b = reinterpret_cast<const f4*>(p)[1];
  d[0] = a[0]; d[1] = a[1]; d[2] = a[2]; d[3] = a[3];
  d[4] = b[0]; d[5] = b[1]; d[6] = b[2]; d[7] = b[3];
}

// ---------------------------------------------------------------------------
// wave reductions (wave64)
// ---------------------------------------------------------------------------
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

static inline int ceil_div(long a, long b) { return (int)((a + b - 1) / b); }

#define SSIP_DISPATCH_DTYPE(dtype, T, ...)                                   \
  do {                                                                       \
    if ((dtype) == SSIP_F32) {                                               \
      typedef float T;                                                       \
      __VA_ARGS__;                                                           \
    } else if ((dtype) == SSIP_BF16) {                                       \
      typedef __bf16 T;                                                      \
      __VA_ARGS__;                                                           \
    } else {                                                                 \
      ::ssip::set_error("unsupported dtype %d", (int)(dtype));               \
      return SSIP_ERR_ARG;                                                   \
    }                                                                        \
  } while (0)

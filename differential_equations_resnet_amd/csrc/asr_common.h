// Shared helpers for the libasr HIP sources (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

#include "../../include/asr.h"

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));

#define ASR_LDS __attribute__((address_space(3)))

namespace asr {

// thread-local error message (asr_last_error)
void set_error(const char* fmt, ...);
int fail(int code, const char* fmt, ...);

inline int hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) return fail(ASR_E_HIP, "%s: %s", what, hipGetErrorString(e));
  return ASR_OK;
}

#define ASR_TRY(expr)            \
  do {                           \
    int _rc = (expr);            \
    if (_rc != ASR_OK) return _rc; \
  } while (0)

#define ASR_LAUNCH_CHECK(name) ASR_TRY(::asr::hip_check(hipGetLastError(), name))

int cu_count();

inline size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

// ---- device helpers --------------------------------------------------------

__device__ __forceinline__ float to_f32(float v) { return v; }
__device__ __forceinline__ float to_f32(bf16 v) { return (float)v; }
template <typename T>
__device__ __forceinline__ T from_f32(float v);
template <>
__device__ __forceinline__ float from_f32<float>(float v) { return v; }
template <>
__device__ __forceinline__ bf16 from_f32<bf16>(float v) { return (bf16)v; }

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

}  // namespace asr

// Internal helpers shared by the mi355_mp HIP translation units (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "../../include/mi355_mp.h"

namespace mp {

void set_error(const char* fmt, ...);

#define MP_CHECK_ARG(cond, ...)        \
  do {                                 \
    if (!(cond)) {                     \
      ::mp::set_error(__VA_ARGS__);    \
      return MP_ERR_ARG;               \
    }                                  \
  } while (0)

// ABI 6: a caller-allocated array passed with its extent in bytes must hold
// what the call writes (or reads); checked before any launch.
#define MP_CHECK_EXTENT(fn, name, have, need)                                                  \
  MP_CHECK_ARG((size_t)(have) >= (size_t)(need), "%s: %s holds %zu bytes, the call needs %zu", \
               fn, name, (size_t)(have), (size_t)(need))

#define MP_CHECK_HIP(expr)                                                   \
  do {                                                                       \
    hipError_t _e = (expr);                                                  \
    if (_e != hipSuccess) {                                                  \
      ::mp::set_error("%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e), \
                      __FILE__, __LINE__);                                   \
      return MP_ERR_HIP;                                                     \
    }                                                                        \
  } while (0)

#define MP_CHECK_LAUNCH() MP_CHECK_HIP(hipGetLastError())

static inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// Entry points enqueue on the caller's stream, on that stream's device: the
// calling thread's current device is switched for the call when it differs
// (a torch stream of cuda:1 while cuda:0 is current) and restored after.
struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(void* stream) {
    if (!stream) return;
    hipDevice_t d;
    int cur;
    if (hipStreamGetDevice(as_stream(stream), &d) != hipSuccess || hipGetDevice(&cur) != hipSuccess) return;
    if (cur != (int)d && hipSetDevice((int)d) == hipSuccess) prev = cur;
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
  DeviceGuard(const DeviceGuard&) = delete;
  DeviceGuard& operator=(const DeviceGuard&) = delete;
};
#define MP_DEVICE_GUARD(stream) DeviceGuard mp_device_guard_(stream)

static inline size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

static inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// Sum over aligned groups of `g` lanes (g a power of two <= 64, wave-uniform)
// with DPP lane permutes (quad_perm, row_half_mirror, row_mirror) fused into
// the adds; every lane of a group ends with the same value (each step adds a
// lane pair in both orders, and fp addition is commutative).
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float group_sum(float t, int g) {
  if (g >= 2) t += dpp<0xB1>(t);   // quad_perm(1,0,3,2)
  if (g >= 4) t += dpp<0x4E>(t);   // quad_perm(2,3,0,1)
  if (g >= 8) t += dpp<0x141>(t);  // row_half_mirror
  if (g >= 16) t += dpp<0x140>(t); // row_mirror
  if (g >= 32) t += __shfl_xor(t, 16);
  if (g >= 64) t += __shfl_xor(t, 32);
  return t;
}

// wave-uniform value helpers
__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

__device__ __forceinline__ int readlane(int v, int l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ float readlane(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}

// Feature fragment: VEC consecutive fp32 owned by one lane.
template <int VEC>
struct Frag {
  float v[VEC];
};

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int VEC>
__device__ __forceinline__ Frag<VEC> load_frag(const float* p) {
  Frag<VEC> r;
  if constexpr (VEC == 4) {
    f32x4 t = *reinterpret_cast<const f32x4*>(p);
    r.v[0] = t.x; r.v[1] = t.y; r.v[2] = t.z; r.v[3] = t.w;
  } else if constexpr (VEC == 2) {
    f32x2 t = *reinterpret_cast<const f32x2*>(p);
    r.v[0] = t.x; r.v[1] = t.y;
  } else {
    r.v[0] = *p;
  }
  return r;
}

template <int VEC>
__device__ __forceinline__ void store_frag(float* p, const Frag<VEC>& f) {
  if constexpr (VEC == 4) {
    f32x4 t = {f.v[0], f.v[1], f.v[2], f.v[3]};
    *reinterpret_cast<f32x4*>(p) = t;
  } else if constexpr (VEC == 2) {
    f32x2 t = {f.v[0], f.v[1]};
    *reinterpret_cast<f32x2*>(p) = t;
  } else {
    *p = f.v[0];
  }
}

template <int VEC>
__device__ __forceinline__ Frag<VEC> load_frag_nt(const float* p) {
  Frag<VEC> r;
  if constexpr (VEC == 4) {
    f32x4 t = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p));
    r.v[0] = t.x; r.v[1] = t.y; r.v[2] = t.z; r.v[3] = t.w;
  } else if constexpr (VEC == 2) {
    f32x2 t = __builtin_nontemporal_load(reinterpret_cast<const f32x2*>(p));
    r.v[0] = t.x; r.v[1] = t.y;
  } else {
    r.v[0] = __builtin_nontemporal_load(p);
  }
  return r;
}

// Fragment load through a buffer resource (32-bit byte offset, range-checked;
// soff: a wave-uniform byte offset added in the soffset field).
template <int VEC, int AUX = 0>  // AUX: cache-policy bits (gfx950: 1 = sc0, 2 = nt, 16 = sc1)
__device__ __forceinline__ Frag<VEC> load_frag_buf(__amdgpu_buffer_rsrc_t r, uint32_t off, uint32_t soff = 0) {
  Frag<VEC> f;
  if constexpr (VEC == 4) {
    f32x4 t = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, soff, AUX));
    f.v[0] = t.x; f.v[1] = t.y; f.v[2] = t.z; f.v[3] = t.w;
  } else if constexpr (VEC == 2) {
    f32x2 t = __builtin_bit_cast(f32x2, __builtin_amdgcn_raw_buffer_load_b64(r, off, soff, AUX));
    f.v[0] = t.x; f.v[1] = t.y;
  } else {
    f.v[0] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, soff, AUX));
  }
  return f;
}

// Non-temporal store of a fragment (output rows are written once and never
// re-read by the kernel; keeping them out of L2/MALL leaves room for the
// gathered x rows).
template <int VEC>
__device__ __forceinline__ void store_frag_nt(float* p, const Frag<VEC>& f) {
  if constexpr (VEC == 4) {
    f32x4 t = {f.v[0], f.v[1], f.v[2], f.v[3]};
    __builtin_nontemporal_store(t, reinterpret_cast<f32x4*>(p));
  } else if constexpr (VEC == 2) {
    f32x2 t = {f.v[0], f.v[1]};
    __builtin_nontemporal_store(t, reinterpret_cast<f32x2*>(p));
  } else {
    __builtin_nontemporal_store(f.v[0], p);
  }
}

}  // namespace mp

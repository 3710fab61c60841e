// Shared host/device definitions for the MI355X (gfx950) hot path.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <string>

#include "../../include/super_rag_mi355x.h"

// SR_WITH_DIAG: 1 in the diagnostic library (libsrmi_diag.so: the product sources plus the
// sr_diag_* entry points of include/super_rag_mi355x_diag.h, timing-only kernel variants and
// the A/B environment knobs); 0 in the product library (libsrmi.so), which exports none of them.
#ifndef SR_WITH_DIAG
#define SR_WITH_DIAG 0
#endif
#if SR_WITH_DIAG
#include <cstdlib>
#include "../../include/super_rag_mi355x_diag.h"
#endif

namespace sr {

// A/B and timing-diagnostic environment knobs: read in the diagnostic library only (the product
// library's knobs are listed in INTEGRATION.md and read with std::getenv where they are used).
inline const char* diag_getenv(const char* name) {
#if SR_WITH_DIAG
  return std::getenv(name);
#else
  (void)name;
  return nullptr;
#endif
}

typedef _Float16 half_t;
typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef _Float16 half4 __attribute__((ext_vector_type(4)));
typedef _Float16 half2_t __attribute__((ext_vector_type(2)));
typedef float float4v __attribute__((ext_vector_type(4)));
typedef short short4v __attribute__((ext_vector_type(4)));

// ---- error plumbing (host) -------------------------------------------------------------------
struct Error : std::runtime_error {
  int code;
  Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

void set_last_error(const std::string& msg);

#define SR_HIP(call)                                                                         \
  do {                                                                                       \
    hipError_t _e = (call);                                                                  \
    if (_e != hipSuccess) {                                                                  \
      throw ::sr::Error(_e == hipErrorOutOfMemory ? SR_ERR_OOM : SR_ERR_HIP,                 \
                        std::string(#call) + ": " + hipGetErrorString(_e) + " at " +         \
                            __FILE__ + ":" + std::to_string(__LINE__));                      \
    }                                                                                        \
  } while (0)

#define SR_CHECK(cond, msg)                                                                   \
  do {                                                                                        \
    if (!(cond)) throw ::sr::Error(SR_ERR_INVALID, std::string(msg));                         \
  } while (0)

#define SR_LAUNCH_CHECK() SR_HIP(hipGetLastError())

// ---- profiling (host) ------------------------------------------------------------------------
// Records a begin/end HIP event pair around a launch when profiling is on.
struct ProfScope {
  const char* name;
  double flops, bytes;
  hipStream_t stream;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  ProfScope(const char* n, hipStream_t s, double f, double b);
  ~ProfScope();
};

// ---- small helpers ---------------------------------------------------------------------------
static inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }
static inline int64_t round_up(int64_t a, int64_t b) { return ceil_div(a, b) * b; }

// Device pointer helpers for LDS address space.
#define SR_LDS(p) ((__attribute__((address_space(3))) void*)(p))

// Buffer resource over `bytes` bytes from `base` (raw buffer: offsets past num_records read as
// zero), for buffer_load ... lds staging with the panel base in SGPRs.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t panel_rsrc(const half_t* base, int64_t bytes) {
  const int nr = bytes > 0x7fffffffLL ? 0x7fffffff : (int)bytes;
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, nr, 0x00020000);
}

// s_waitcnt through the builtin (the compiler's own waitcnt pass then knows the counters are
// satisfied; an asm waitcnt is invisible to it and it re-waits conservatively). gfx9 encoding:
// vmcnt[3:0] | expcnt[6:4] | lgkmcnt[11:8] | vmcnt[5:4] << 14.
#define SR_WAITCNT(vm, lgkm) \
  __builtin_amdgcn_s_waitcnt(((vm) & 15) | (7 << 4) | (((lgkm) & 15) << 8) | (((vm) >> 4) << 14))

// Order-preserving float -> uint32 (larger float -> larger uint).
__device__ __forceinline__ uint32_t ordered_bits(float f) {
  uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float unordered_bits(uint32_t u) {
  return __uint_as_float((u & 0x80000000u) ? (u & 0x7fffffffu) : ~u);
}
// Top-k key: (similarity desc, row asc) <=> key desc.  key == 0 marks "no entry".
__device__ __forceinline__ uint64_t make_key(float sim, uint32_t row) {
  return ((uint64_t)ordered_bits(sim) << 32) | (uint64_t)(0xffffffffu - row);
}
__device__ __forceinline__ float key_sim(uint64_t key) { return unordered_bits((uint32_t)(key >> 32)); }
__device__ __forceinline__ uint32_t key_row(uint64_t key) { return 0xffffffffu - (uint32_t)key; }

// OCP e4m3fn (bias 7, max 448, no infinities), round to nearest even, saturating at +-448.
__device__ __forceinline__ uint32_t e4m3_rne(float v) {
  const uint32_t sign = v < 0.f ? 0x80u : 0u;
  const float a = fminf(fabsf(v), 448.f);
  if (a < 0.015625f) {  // below 2^-6: subnormal steps of 2^-9
    const uint32_t m = (uint32_t)rintf(a * 512.f);  // 0 .. 8 (8 = the smallest normal)
    return sign | m;
  }
  int e;
  (void)frexpf(a, &e);  // a = f * 2^e, f in [0.5, 1)  ->  a = (1 + m / 8) * 2^(e - 1)
  const float m = rintf((ldexpf(a, 1 - e) - 1.f) * 8.f);  // 0 .. 8 (8 carries into the exponent)
  return sign | ((uint32_t)(e - 1 + 7) * 8u + (uint32_t)m);
}

// Four floats -> four e4m3 bytes with v_cvt_pk_fp8_f32 (gfx950: OCP e4m3, round to nearest even;
// bit-identical to e4m3_rne after the clamp, checked on 2^24 values: tools/diag/cvt_fp8.hip).
__device__ __forceinline__ uint32_t e4m3x4(float a, float b, float c, float d) {
  auto cl = [](float x) { return fminf(fmaxf(x, -448.f), 448.f); };
  int w = __builtin_amdgcn_cvt_pk_fp8_f32(cl(a), cl(b), 0, false);
  w = __builtin_amdgcn_cvt_pk_fp8_f32(cl(c), cl(d), w, true);
  return (uint32_t)w;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

}  // namespace sr

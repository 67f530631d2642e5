// Shared device helpers for libclimsr_hip (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "climsr_hip.h"

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

namespace climsr {

void set_error(const char* fmt, ...);
int check_launch(const char* what);
// CU count of the current device (cached per device, thread-safe)
int device_cus();
// hipFuncSetAttribute(MaxDynamicSharedMemorySize) once per (kernel, device), thread-safe, error checked
int lds_opt_in(const void* fn, int bytes);
// dispatcher dry run (climsr_*_kernel name queries): set, the dispatchers record the kernel they would launch in
// g_dry_name and return before launching; dry_run(fmt, ...) records the name and answers whether to return
extern thread_local bool g_dry;
extern thread_local char g_dry_name[96];
bool dry_run(const char* fmt, ...);

__device__ __forceinline__ uint16_t f2bf(float f) {
  __bf16 b = (__bf16)f;  // v_cvt_pk_bf16_f32: RNE, NaN-preserving
  return __builtin_bit_cast(uint16_t, b);
}
__device__ __forceinline__ float bf2f(uint16_t u) { return __uint_as_float(((uint32_t)u) << 16); }

__device__ __forceinline__ float act_apply(float v, int act, float slope) {
  if (act == 1) return v > 0.f ? v : v * slope;
  if (act == 2) return v > 0.f ? v : 0.f;
  return v;
}

// Transposed LDS read: within each 16-lane group, lane 4q+p supplies the address of row q, columns
// 4p..4p+3 (16-bit elements); lane i receives column i of the 4 rows (row q -> element q).
__device__ __forceinline__ s16x4 ds_read_tr16(const void* lds_ptr) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((s16x4 __attribute__((address_space(3)))*)(lds_ptr));
}

// Two transposed reads (rows k..k+3 and k+4..k+7 of one 16-lane column group) as ONE MFMA K-fragment of 8 bf16,
// by vector shuffle: the halves land in adjacent VGPRs without per-element packing (a short[8] temporary made hipcc
// emit v_bfi / v_perm per fragment).
typedef short s16x8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ bf16x8 cat_tr(s16x4 lo, s16x4 hi) {
  const s16x8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, v);
}

// Buffer resource over [base, base + bytes): a raw buffer load whose byte offset is >= bytes returns zeros
// (hardware range check), so halo / padding lanes get zeros without a branch around the load (a branch
// around a load makes hipcc wait vmcnt(0) right there, which serialises a register prefetch).
constexpr uint32_t BUF_OOB = 0x80000000u;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ uint4 buf_load16(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
  return make_uint4(v[0], v[1], v[2], v[3]);
}

// Workgroup barrier for LDS-only hand-offs: orders this wave's LDS accesses (lgkmcnt) but not its global
// loads / stores, so register prefetches and epilogue stores stay in flight across it.  __syncthreads()'s
// release fence waits vmcnt(0), which drains a prefetch issued before it.
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

static inline int ceil_div(long a, long b) { return (int)((a + b - 1) / b); }
static inline int round_up(int a, int b) { return (a + b - 1) / b * b; }

}  // namespace climsr

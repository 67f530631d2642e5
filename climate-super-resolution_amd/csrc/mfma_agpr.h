// MFMA chains whose A operands (weights, read-only for a whole launch) live in AGPRs.
//
// A kernel whose weight fragments exceed the 256 VGPRs keeps them in the accumulator half of the unified register
// file; gfx950 MFMAs read A / B from AGPRs directly (cdna_hip_programming.md §3), but through the builtin hipcc copies
// every AGPR-resident fragment to VGPRs first (4 v_accvgpr_read per MFMA).  These helpers issue the MFMAs from inline
// asm with "a" operands instead.  hipcc sees no MFMA inside the asm, so the hazards are padded here:
//   * each block opens with 4 wait states for a VALU write (e.g. a v_accvgpr_write re-materialising a fragment) of an
//     operand right before it;
//   * a chain may start from a literal 0 accumulator (no VALU zero-fill read as C);
//   * pad_mfma() (18 wait states, tied to the accumulators so no read of them is scheduled ahead of it) must follow
//     the last block before anything else reads the accumulators.
// Dependent MFMAs on one accumulator need no wait states between them.
#pragma once
#include "common.h"

namespace climsr {

// acc (+)= A0 B0 + A1 B1 + A2 B2 (one accumulator, three k-blocks)
template <bool FIRST>
__device__ __forceinline__ void mfma3_agpr(f32x4& acc, const bf16x8& a0, const bf16x8& a1, const bf16x8& a2, const bf16x8& b0,
                                           const bf16x8& b1, const bf16x8& b2) {
  if constexpr (FIRST) {
    asm volatile(
        "s_nop 3\n\t"
        "v_mfma_f32_16x16x32_bf16 %0, %1, %4, 0\n\t"
        "v_mfma_f32_16x16x32_bf16 %0, %2, %5, %0\n\t"
        "v_mfma_f32_16x16x32_bf16 %0, %3, %6, %0"
        : "=&v"(acc)
        : "a"(a0), "a"(a1), "a"(a2), "v"(b0), "v"(b1), "v"(b2));
  } else {
    asm volatile(
        "s_nop 3\n\t"
        "v_mfma_f32_16x16x32_bf16 %0, %1, %4, %0\n\t"
        "v_mfma_f32_16x16x32_bf16 %0, %2, %5, %0\n\t"
        "v_mfma_f32_16x16x32_bf16 %0, %3, %6, %0"
        : "+v"(acc)
        : "a"(a0), "a"(a1), "a"(a2), "v"(b0), "v"(b1), "v"(b2));
  }
}

// the same with the A fragments in VGPRs (for fragments past the 256 AGPRs: a builtin MFMA there would make hipcc
// move the accumulator between the register halves, reading an asm MFMA's result with no wait states)
__device__ __forceinline__ void mfma3_vgpr(f32x4& acc, const bf16x8& a0, const bf16x8& a1, const bf16x8& a2, const bf16x8& b0,
                                           const bf16x8& b1, const bf16x8& b2) {
  asm volatile(
      "s_nop 3\n\t"
      "v_mfma_f32_16x16x32_bf16 %0, %1, %4, %0\n\t"
      "v_mfma_f32_16x16x32_bf16 %0, %2, %5, %0\n\t"
      "v_mfma_f32_16x16x32_bf16 %0, %3, %6, %0"
      : "+v"(acc)
      : "v"(a0), "v"(a1), "v"(a2), "v"(b0), "v"(b1), "v"(b2));
}

// c[t] (+)= A[t] B for t = 0..3 (four accumulators -- four output-channel blocks -- sharing one B fragment); A3V: the
// fourth A fragment is in a VGPR (the 256 AGPRs hold 60 of a 64 -> 64 3x3 conv's 72 fragments)
template <bool FIRST, bool A3V>
__device__ __forceinline__ void mfma4x_agpr(f32x4& c0, f32x4& c1, f32x4& c2, f32x4& c3, const bf16x8& a0, const bf16x8& a1,
                                            const bf16x8& a2, const bf16x8& a3, const bf16x8& b) {
  if constexpr (FIRST) {
    if constexpr (A3V) {
      asm volatile(
          "s_nop 3\n\t"
          "v_mfma_f32_16x16x32_bf16 %0, %4, %8, 0\n\t"
          "v_mfma_f32_16x16x32_bf16 %1, %5, %8, 0\n\t"
          "v_mfma_f32_16x16x32_bf16 %2, %6, %8, 0\n\t"
          "v_mfma_f32_16x16x32_bf16 %3, %7, %8, 0"
          : "=&v"(c0), "=&v"(c1), "=&v"(c2), "=&v"(c3)
          : "a"(a0), "a"(a1), "a"(a2), "v"(a3), "v"(b));
    } else {
      asm volatile(
          "s_nop 3\n\t"
          "v_mfma_f32_16x16x32_bf16 %0, %4, %8, 0\n\t"
          "v_mfma_f32_16x16x32_bf16 %1, %5, %8, 0\n\t"
          "v_mfma_f32_16x16x32_bf16 %2, %6, %8, 0\n\t"
          "v_mfma_f32_16x16x32_bf16 %3, %7, %8, 0"
          : "=&v"(c0), "=&v"(c1), "=&v"(c2), "=&v"(c3)
          : "a"(a0), "a"(a1), "a"(a2), "a"(a3), "v"(b));
    }
  } else {
    if constexpr (A3V) {
      asm volatile(
          "s_nop 3\n\t"
          "v_mfma_f32_16x16x32_bf16 %0, %4, %8, %0\n\t"
          "v_mfma_f32_16x16x32_bf16 %1, %5, %8, %1\n\t"
          "v_mfma_f32_16x16x32_bf16 %2, %6, %8, %2\n\t"
          "v_mfma_f32_16x16x32_bf16 %3, %7, %8, %3"
          : "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3)
          : "a"(a0), "a"(a1), "a"(a2), "v"(a3), "v"(b));
    } else {
      asm volatile(
          "s_nop 3\n\t"
          "v_mfma_f32_16x16x32_bf16 %0, %4, %8, %0\n\t"
          "v_mfma_f32_16x16x32_bf16 %1, %5, %8, %1\n\t"
          "v_mfma_f32_16x16x32_bf16 %2, %6, %8, %2\n\t"
          "v_mfma_f32_16x16x32_bf16 %3, %7, %8, %3"
          : "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3)
          : "a"(a0), "a"(a1), "a"(a2), "a"(a3), "v"(b));
    }
  }
}

// c[t] (+)= A[t] B for t = 0, 1 (two co blocks sharing a B fragment); A1V: the second A fragment is in a VGPR
template <bool FIRST, bool A1V>
__device__ __forceinline__ void mfma2x_agpr(f32x4& c0, f32x4& c1, const bf16x8& a0, const bf16x8& a1, const bf16x8& b) {
  if constexpr (FIRST) {
    if constexpr (A1V) {
      asm volatile("s_nop 3\n\tv_mfma_f32_16x16x32_bf16 %0, %2, %4, 0\n\tv_mfma_f32_16x16x32_bf16 %1, %3, %4, 0"
                   : "=&v"(c0), "=&v"(c1) : "a"(a0), "v"(a1), "v"(b));
    } else {
      asm volatile("s_nop 3\n\tv_mfma_f32_16x16x32_bf16 %0, %2, %4, 0\n\tv_mfma_f32_16x16x32_bf16 %1, %3, %4, 0"
                   : "=&v"(c0), "=&v"(c1) : "a"(a0), "a"(a1), "v"(b));
    }
  } else {
    if constexpr (A1V) {
      asm volatile("s_nop 3\n\tv_mfma_f32_16x16x32_bf16 %0, %2, %4, %0\n\tv_mfma_f32_16x16x32_bf16 %1, %3, %4, %1"
                   : "+v"(c0), "+v"(c1) : "a"(a0), "v"(a1), "v"(b));
    } else {
      asm volatile("s_nop 3\n\tv_mfma_f32_16x16x32_bf16 %0, %2, %4, %0\n\tv_mfma_f32_16x16x32_bf16 %1, %3, %4, %1"
                   : "+v"(c0), "+v"(c1) : "a"(a0), "a"(a1), "v"(b));
    }
  }
}

__device__ __forceinline__ void pad_mfma8(f32x4 (&c)[4][2]) {
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3"
               : "+v"(c[0][0]), "+v"(c[0][1]), "+v"(c[1][0]), "+v"(c[1][1]), "+v"(c[2][0]), "+v"(c[2][1]), "+v"(c[3][0]),
                 "+v"(c[3][1]));
}

__device__ __forceinline__ void pad_mfma(f32x4 (&pn)[4]) {
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" : "+v"(pn[0]), "+v"(pn[1]), "+v"(pn[2]), "+v"(pn[3]));
}
__device__ __forceinline__ void pad_mfma16(f32x4 (&c)[4][4]) {
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3"
               : "+v"(c[0][0]), "+v"(c[0][1]), "+v"(c[0][2]), "+v"(c[0][3]), "+v"(c[1][0]), "+v"(c[1][1]), "+v"(c[1][2]),
                 "+v"(c[1][3]), "+v"(c[2][0]), "+v"(c[2][1]), "+v"(c[2][2]), "+v"(c[2][3]), "+v"(c[3][0]), "+v"(c[3][1]),
                 "+v"(c[3][2]), "+v"(c[3][3]));
}

}  // namespace climsr

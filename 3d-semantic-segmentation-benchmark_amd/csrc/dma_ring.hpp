// LDS-DMA ring helpers shared by the data-gradient (dgrad.hip) and forward (fwd_dma.hip) GEMMs:
// global -> LDS copies with global_load_lds_dwordx4 (no VGPR destination), retired by counted
// `s_waitcnt vmcnt` + raw s_barrier (never __syncthreads(), whose fence would drain the ring;
// cdna_hip_programming.md, glds rules).
#pragma once

#include "pcs_common.hpp"

namespace pcs {

// waitcnt immediate for "vmcnt(n)" alone (gfx9 encoding: vmcnt[3:0] at bits 3:0, vmcnt[5:4] at
// 15:14; expcnt and lgkmcnt left at their maxima)
constexpr int dg_vmcnt(int n) { return (n & 15) | ((n >> 4) << 14) | (7 << 4) | (15 << 8); }

// 16-B chunk swizzle of a 32-float LDS row r (the chunk XOR (r >> 1) & 7 is applied on the SOURCE
// address of the DMA and on every read, so ds_read_b128 over 16 consecutive rows is conflict free)
__device__ __forceinline__ int dg_swz(int r) { return (r >> 1) & 7; }

// one LDS-DMA: 16 B per active lane to LDS byte address dst + 16 * lane, from inline asm so the
// compiler does not track it (it would drain the ring at every LDS read otherwise); M0 is saved
// and restored inside the statement (compiler-reserved)
__device__ __forceinline__ void dg_glds16(const float* gsrc, unsigned dst) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(gsrc), "s"(dst)
                 : "memory");
}

__device__ __forceinline__ unsigned dg_lds_addr(const float* p) {
    return (unsigned)(uintptr_t)((const __attribute__((address_space(3))) float*)p);
}

__device__ __forceinline__ void dg_barrier() { asm volatile("s_barrier" ::: "memory"); }

}  // namespace pcs

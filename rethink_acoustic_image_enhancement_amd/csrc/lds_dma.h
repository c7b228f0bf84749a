// LDS-DMA helpers shared by the ring-pipelined kernels (gdfn.hip, mdta.hip).
//
// global_load_lds moves 16 B per lane from global memory straight into LDS without VGPRs; the LDS
// destination of one wave-instruction is a wave-uniform base + 16 * lane (any swizzle goes on the
// SOURCE address).  It retires on the vector-memory counter like every other VMEM op, and on gfx9
// vmcnt retires IN ORDER and counts stores too, so "wait until the DMA of item k has landed" is
// s_waitcnt vmcnt(<VMEM ops issued after it>).  A __syncthreads() would emit vmcnt(0) and drain
// every DMA in flight, so the ring kernels synchronise with raw s_barrier (see barrier_lds()).
#pragma once
#include <hip/hip_runtime.h>

namespace kdlae {
namespace dma {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) void* gptr_t;
typedef __attribute__((address_space(3))) void* lptr_t;

// s_waitcnt with only a vmcnt limit (gfx9 encoding: vmcnt[3:0] + [15:14], expcnt/lgkmcnt at max)
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

// vmcnt(n) for a wave-uniform runtime n (scalar branch tree); n > 31 waits for everything.
__device__ __forceinline__ void wait_vmcnt_dyn(int n) {
#define KDLAE_VMC(k) \
  case k:            \
    wait_vmcnt<k>(); \
    break;
  switch (n) {
    KDLAE_VMC(0) KDLAE_VMC(1) KDLAE_VMC(2) KDLAE_VMC(3) KDLAE_VMC(4) KDLAE_VMC(5) KDLAE_VMC(6) KDLAE_VMC(7)
    KDLAE_VMC(8) KDLAE_VMC(9) KDLAE_VMC(10) KDLAE_VMC(11) KDLAE_VMC(12) KDLAE_VMC(13) KDLAE_VMC(14)
    KDLAE_VMC(15) KDLAE_VMC(16) KDLAE_VMC(17) KDLAE_VMC(18) KDLAE_VMC(19) KDLAE_VMC(20) KDLAE_VMC(21)
    KDLAE_VMC(22) KDLAE_VMC(23) KDLAE_VMC(24) KDLAE_VMC(25) KDLAE_VMC(26) KDLAE_VMC(27) KDLAE_VMC(28)
    KDLAE_VMC(29) KDLAE_VMC(30) KDLAE_VMC(31)
    default: wait_vmcnt<0>(); break;
  }
#undef KDLAE_VMC
}

__device__ __forceinline__ void dma16(const void* src, f32x4* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)lds_wave_base, 16, 0, 0);
}

// Workgroup barrier that orders LDS (own ds ops complete, then s_barrier) without draining VMEM.
// The empty asm keeps the compiler from hoisting LDS reads above the barrier.
__device__ __forceinline__ void barrier_lds() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Register-staged tile fill for a 256-thread block: item i = tid + 256 k of an N-item f32x4 tile,
// fetched SB items per thread at a time — all SB loads are issued before the first LDS write, so a
// fill costs ceil(N / (256 SB)) memory latencies instead of one per item (a plain strided loop
// compiles to load / s_waitcnt vmcnt(0) / ds_write per item).
template <int N, int SB, typename Fetch>
__device__ __forceinline__ void stage_batched(f32x4* tile, int tid, Fetch&& fetch) {
#pragma unroll 1
  for (int base = 0; base < N; base += 256 * SB) {
    f32x4 v[SB];
#pragma unroll
    for (int k = 0; k < SB; ++k) {
      const int i = base + tid + 256 * k;
      v[k] = i < N ? fetch(i) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int k = 0; k < SB; ++k) {
      const int i = base + tid + 256 * k;
      if (i < N) tile[i] = v[k];
    }
  }
}

}  // namespace dma
}  // namespace kdlae

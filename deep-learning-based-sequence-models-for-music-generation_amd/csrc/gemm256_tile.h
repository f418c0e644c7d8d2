// Device building blocks shared by the 256x256 GEMM tiles (gemm256.hip: the
// per-tile kernel; gemm256p.hip: the persistent kernel). See gemm256.hip for
// the tile structure.
#pragma once
#include "gemm.h"
#include "lds_dma.h"

namespace g256 {

constexpr int NT = 512;
constexpr int HALF = 16384;          // bytes of one half-tile slot
constexpr uint32_t OOB = 0xFFFF0000u;  // voffset past every descriptor's num_records

typedef __attribute__((address_space(3))) char lds_t;

__device__ __forceinline__ int swz_k(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }
__device__ __forceinline__ int gmn(int k) { return ((k & 3) | ((k >> 1) & 4)) << 1; }

__device__ __forceinline__ void vm_wait8() { asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); }
__device__ __forceinline__ void vm_wait0() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
// keeps the compiler from moving VMEM ops across this point (the counted
// vmcnt waits below rely on the issue order DMA halves -> epilogue stores)
__device__ __forceinline__ void order_fence() {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
}
__device__ __forceinline__ void barrier() {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
}

// Per-lane staging state of one operand (both halves, both DMA per half).
template <int KC>
struct Stage {
    uint32_t off[2][2];  // byte offset of this lane's chunk at k0 = 0, [half][j]
    int kk[2];           // k of this lane's chunk relative to k0 (validity), [j]
    bool rv[2][2];       // row / column in range, [half][j]
    uint32_t kstep;      // bytes per unit of k (K-contig: 2, MN-contig: 2*ld)

    __device__ __forceinline__ void init(int64_t r0, int64_t R, int64_t ld, int w, int lane) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int li = (j * 8 + w) * 1024 + lane * 16;  // byte in the half-tile image
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                if (KC) {  // image [128 rows][128 B]
                    const int row = li >> 7, slot = (li >> 4) & 7;
                    const int ch = slot ^ ((row >> 1) & 7);
                    const int64_t gr = r0 + h * 128 + row;
                    rv[h][j] = gr < R;
                    off[h][j] = (uint32_t)((rv[h][j] ? gr : 0) * ld * 2 + ch * 16);
                    kk[j] = ch * 8;
                } else {  // image [64 k][256 B]
                    const int k = li >> 8, slot = (li >> 4) & 15;
                    const int ch = slot ^ gmn(k);
                    const int64_t gc = r0 + h * 128 + ch * 8;
                    rv[h][j] = gc < R;
                    off[h][j] = (uint32_t)((int64_t)k * ld * 2 + (rv[h][j] ? gc : 0) * 2);
                    kk[j] = k;
                }
            }
        }
        kstep = KC ? 2u : (uint32_t)(ld * 2);
    }

    // DMA half h of the K-tile starting at k0 (krem = valid k left from k0)
    __device__ __forceinline__ void issue(__amdgpu_buffer_rsrc_t rs, lds_t* slot, int h, int64_t k0, int64_t krem,
                                          int wu) const {
        const uint32_t kadv = (uint32_t)k0 * kstep;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const uint32_t vo = (rv[h][j] && kk[j] < krem) ? off[h][j] + kadv : OOB;
            lds_dma16(rs, slot + (j * 8 + wu) * 1024, vo);
        }
    }
};

// descriptor from provably wave-uniform words (no waterfall loops, T20)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const char* base, uint32_t bytes) {
    const uint64_t a = (uint64_t)base;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    void* p = (void*)(((uint64_t)hi << 32) | lo);
    return __builtin_amdgcn_make_buffer_rsrc(p, (short)0, (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

__device__ __forceinline__ bf16x8 rd_b128(const lds_t* p) { return *(const bf16x8 __attribute__((address_space(3)))*)p; }
__device__ __forceinline__ bf16x8 rd_tr(const lds_t* p) {
    i16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((i16x4 __attribute__((address_space(3)))*)p);
    i16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((i16x4 __attribute__((address_space(3)))*)(p + 1024));
    union { i16x4 h[2]; bf16x8 v; } u;
    u.h[0] = a;
    u.h[1] = b;
    return u.v;
}

// fragment set of one quadrant-operand: NF 16-row groups x 2 k-steps
template <int KC, int NF>
__device__ __forceinline__ void read_set(bf16x8 (&f)[2][NF], const lds_t* slot, int rbase, const int (&lo)[4]) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int i = 0; i < NF; ++i) {
            if (KC) f[ks][i] = rd_b128(slot + (rbase + i * 16) * 128 + lo[ks]);
            else f[ks][i] = rd_tr(slot + ks * 8192 + lo[i]);
        }
}

}  // namespace g256

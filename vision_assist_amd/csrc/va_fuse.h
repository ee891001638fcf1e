// va_fuse.h -- shared device helpers of the fused multi-layer kernels (va_c2f.hip, va_stem.hip):
// MFMA 16x16x32 bf16 fragments, SiLU epilogues, buffer-descriptor masking, the XCD-aware persistent
// tile schedule.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
typedef __attribute__((ext_vector_type(2))) float f32x2;

namespace fz {

constexpr int FRAG = 512;             // bf16 per MFMA operand fragment (64 lanes x 8)
constexpr int OOB = 0x80000000;       // buffer offset past num_records: a load returns 0, a store is dropped
constexpr int RSRC = 0x00020000;      // buffer descriptor word 3 (gfx9 raw buffer)

// bf16 epilogues: hardware exp and reciprocal (~1 ulp f32, far below the bf16 rounding that follows),
// the same expression as va_seg.hip's unfused layers
__device__ __forceinline__ float silu(float x) { return x * __builtin_amdgcn_rcpf(1.0f + __expf(-x)); }
// four SiLUs with the plain f32 steps packed in pairs (v_pk_mul_f32 / v_pk_add_f32 around the two
// 8-cycle transcendentals): the same operations in the same order as silu(), so bit-identical.  (Briefly
// blamed for va_pw.hip's sporadic non-finite outputs; the cause was that kernel's store hazard)
__device__ __forceinline__ f32x2 silu2(f32x2 x) {
    const f32x2 t = x * (f32x2){-1.4426950408889634f, -1.4426950408889634f};
    const f32x2 e = {__builtin_amdgcn_exp2f(t[0]), __builtin_amdgcn_exp2f(t[1])};
    const f32x2 d = e + (f32x2){1.0f, 1.0f};
    const f32x2 r = {__builtin_amdgcn_rcpf(d[0]), __builtin_amdgcn_rcpf(d[1])};
    return x * r;
}
__device__ __forceinline__ f32x4 act(f32x4 x) {
    const f32x2 lo = silu2((f32x2){x[0], x[1]}), hi = silu2((f32x2){x[2], x[3]});
    return (f32x4){lo[0], lo[1], hi[0], hi[1]};
}

__device__ __forceinline__ f32x4 mma(bf16x8 a, bf16x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// two C fragments (rows 4 fq .. 4 fq + 3 of two 16-row groups) -> one lane's 8 bf16 (P32 order: the
// channel order a consumer's K is permuted to when it takes this as its B fragment)
__device__ __forceinline__ bf16x8 pack(f32x4 lo, f32x4 hi) {
    bf16x8 o;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        o[r] = (__bf16)lo[r];
        o[4 + r] = (__bf16)hi[r];
    }
    return o;
}

__device__ __forceinline__ bf16x8 zero_if(bf16x8 v, bool out) {  // masks whole dwords (packed pairs)
    u32x4 u = (u32x4)v;
#pragma unroll
    for (int r = 0; r < 4; ++r) u[r] = out ? 0u : u[r];
    return (bf16x8)u;
}

// lane id through an opaque asm: stops the compiler hoisting every per-lane address of a persistent
// loop body out of the loop (and spilling them)
__device__ __forceinline__ int lane_id() {
    int l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return l;
}

// k-th tile of workgroup blockIdx.x (or -1): with a grid that is a multiple of 8, the workgroups of one
// XCD (blockIdx mod 8) share a contiguous run of tiles, so neighbouring tiles' halo reads hit its L2
__device__ __forceinline__ int tile(int ntiles, int k) {
    const int G = gridDim.x, b = blockIdx.x;
    if (G % 8) {
        const int t = b + k * G;
        return t < ntiles ? t : -1;
    }
    const int per = G / 8, run = (ntiles + 7) / 8, x = b & 7;
    const int t = x * run + (b >> 3) + k * per;
    return (t < ntiles && t < (x + 1) * run) ? t : -1;
}

// the work-queue schedule of the persistent kernels (va_seg.hip conv3q / stem32, va_stem.hip, va_c2f.hip): the next
// tile from a counter of the plan (va_conv_args.wcnt[0]), or -1; the last workgroup out (counter [1]) zeroes both
// the launchers use it from this many tiles per workgroup: below that (batch-1 shapes) every workgroup runs one or two
// tiles, a late one cannot be helped, and the claims' extra barrier costs (the drop-in call 543-548 calls/s on the
// static schedule against 534-537 with claims, profiles/r05/workq/dropin/)
constexpr int WQ_MIN_TILES_PER_WG = 4;
__device__ __forceinline__ int wq_claim(int* cnt, int ntiles) {
    const int v = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return v < ntiles ? v : -1;
}
// the counter's raw value, for a claim issued well ahead of its use (conv3q, the f32 stem): the range check
// (v < ntiles) is made where the claim is published, so the returning atomic's wait lands there too -- with the
// compiler's atomic optimizer off for the file (Makefile), which would otherwise broadcast the result through a
// readfirstlane and wait for it at once
__device__ __forceinline__ int wq_claim_raw(int* cnt) {
    return __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void wq_release(int* cnt) {
    if (__hip_atomic_fetch_add(cnt + 1, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == (int)gridDim.x - 1) {
        __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(cnt + 1, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

}  // namespace fz

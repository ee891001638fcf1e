// va_diag.h -- out-of-range state a kernel rejected instead of faulting.  The library is built without
// relocatable device code, so each translation unit that includes this header has its own word
// g_diag = {first code, v0, v1, count}; va_diag() (va_handle.hip, include/va355.h) reads and clears them.
//   post (va_post.hip):       11 decode: candidates past the anchor count (v0 = list base, v1 = block's count)
//                             12 NMS: candidate count past the anchor count (v0 = count, v1 = anchors)
//   contour (va_contour.hip): 20 + the CT_OK site code: 22 a traced pixel read outside the framed image, 23 a mark
//                             outside it, 27 a bilinear tap row outside the strip, 30 a fill hit past the lattice
//   nav (va_nav.hip):         31 grid: a rect no frame can hold (v0 = x, v1 = w), treated as no mask
//                             32 A*: start / end node outside the lattice (v0 = start, v1 = end)
//                             33 A*: a popped key outside the open list or the lattice (v0 = node, v1 = open count)
//                             34 A*: a parent chain longer than the lattice (v0 = query slot, v1 = length)
//                             35 dedupe: a found path's length outside 1..nodes (v0 = query k, v1 = length)
//                             36 dedupe: a path node outside the lattice (v0 = query k, v1 = node)
#pragma once
#include <hip/hip_runtime.h>

static __device__ unsigned int g_diag[4];

__device__ inline bool diag_ok(bool c, int code, long long v0, long long v1) {
    if (c) return true;
    if (atomicCAS(&g_diag[0], 0u, (unsigned)code) == 0u) {
        atomicExch(&g_diag[1], (unsigned)v0);
        atomicExch(&g_diag[2], (unsigned)v1);
    }
    atomicAdd(&g_diag[3], 1u);
    return false;
}
#define VA_DIAG_OK(c, code, v0, v1) diag_ok((c), (code), (long long)(v0), (long long)(v1))

// host: this translation unit's word into out4 (after a device synchronisation), then zeroed if clear
static inline int diag_read_tu(unsigned int* out4, int clear) {
    if (hipDeviceSynchronize() != hipSuccess) return -2;
    if (hipMemcpyFromSymbol(out4, HIP_SYMBOL(g_diag), sizeof(unsigned int) * 4) != hipSuccess) return -2;
    if (clear) {
        const unsigned int z[4] = {0, 0, 0, 0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_diag), z, sizeof(z)) != hipSuccess) return -2;
    }
    return 0;
}

int va_diag_post(unsigned int* out4, int clear);
int va_diag_contour(unsigned int* out4, int clear);
int va_diag_nav(unsigned int* out4, int clear);

// va_pw.hip -- pointwise (1x1, stride 1) convolutions with 128 output channels as a streaming GEMM:
// the C2f cv1 / cv2 layers of the P3 blocks (model.4, model.15 of YOLOv8s-seg; block.py C2f.cv1/cv2,
// conv.py Conv with k = 1), run inside YOLO.predict (FrameProcessor.py:322).
//
// These layers move ~200-300 MB per 64 frames for 5-20 GFLOP: HBM-bound.  The LDS-staged GEMM (conv2)
// waits on a full DMA round trip every 64-deep K-step (two or three per tile at K = 128-192), so it
// keeps too few bytes in flight to stream.  Here:
//   * the weights (128 x K, K <= 448) are staged into LDS ONCE per persistent workgroup, in MFMA
//     A-fragment order (one conflict-free ds_read_b128 per fragment), with rows permuted so a lane's
//     fragment pair (2p, 2p + 1) holds 8 consecutive output channels (16-byte epilogue stores);
//   * every wave streams its own 48-pixel tiles: B fragments go straight from HBM into registers
//     (lane (p, q): 16 bytes = channels 8q..8q+7 of pixel p), D 32-deep K-steps ahead in a D-slot
//     register ring (K fully unrolled per instantiation) that runs across tile boundaries -- no LDS for
//     activations, no barrier;
//   * accumulators start from the bias; SiLU epilogue from the accumulators; loads and stores are
//     buffer ops with out-of-range offsets for pixels past M, so none is conditional;
//   * the FPN's upsampled channel prefix (va_conv_args.xu) is read in place like conv2/conv4 do.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "../../include/va355.h"
#include "va_switch.h"
#include "va_dev.h"
#include "va_fuse.h"

namespace {

using fz::mma;

constexpr int PW_NW = 8;    // waves per workgroup
constexpr int PW_NB = 3;    // B fragments (16 pixels each) per wave tile
constexpr int PW_TP = 16 * PW_NB;  // pixels per wave tile
constexpr int PW_NQ = 8;    // 16-channel output groups (Cout = 128)
constexpr int PW_KMAX = 448;

// NK = K / 32 K-steps, fully unrolled; the B fragments run through a ring of D slots (D divides NK, so a
// K-step's slot is a compile-time constant and the next tile's first D steps land in the slots they are
// read from: the ring is carried across tiles without register copies or a full vmcnt drain)
template <int NK, int D>
__global__ __launch_bounds__(PW_NW * 64, 1) void pw_kernel(va_conv_args a, int ntiles) {
    static_assert(NK % D == 0 && D >= 2, "ring");
    extern __shared__ __attribute__((aligned(16))) unsigned char pw_smem[];
    const int tid = threadIdx.x, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    float* bias_s = (float*)(pw_smem + NK * PW_NQ * 1024);
    // weights -> LDS: fragment f = kf * 8 + q, lane l: row perm(q, l & 15), k = 32 kf + 8 (l >> 4)
    {
        const __bf16* W = (const __bf16*)a.w;
        for (int i = tid; i < NK * PW_NQ * 64; i += PW_NW * 64) {
            const int f = i >> 6, l = i & 63, q = f % PW_NQ, kf = f / PW_NQ, r = l & 15;
            const int row = 32 * (q >> 1) + 8 * (r >> 2) + 4 * (q & 1) + (r & 3);
            *(u32x4*)(pw_smem + 16 * i) = *(const u32x4*)(W + (int64_t)row * a.Kpad + 32 * kf + 8 * (l >> 4));
        }
        for (int i = tid; i < 128; i += PW_NW * 64) bias_s[i] = a.bias[i];
    }
    __syncthreads();

    const int lane = fz::lane_id(), fr = lane & 15, fq = lane >> 4;
    const int stride = gridDim.x * PW_NW;
    int t = blockIdx.x * PW_NW + wid;
    if (t >= ntiles) return;  // whole wave (no barrier follows)

    // buffer descriptors over the whole input / output (offsets fit 31 bits: checked by the launcher)
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, (short)0, 0x7fffffff, fz::RSRC);
    const __amdgpu_buffer_rsrc_t ru =
        __builtin_amdgcn_make_buffer_rsrc((void*)(a.xu ? a.xu : a.x), (short)0, 0x7fffffff, fz::RSRC);
    const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc(a.y, (short)0, 0x7fffffff, fz::RSRC);
    const int HW = a.H * a.W, hw2 = (a.H / 2) * (a.W / 2);
    const int cu = a.xu ? a.cu : 0;

    // per tile: the byte offsets of this lane's pixels in x and (upsampled prefix) in xu
    int ox[PW_NB], ou[PW_NB];
    auto tile_offsets = [&](int tt) {
#pragma unroll
        for (int j = 0; j < PW_NB; ++j) {
            const int m = tt * PW_TP + 16 * j + fr;
            if (m < a.M) {
                ox[j] = (m * a.ldx + 8 * fq) * 2;
                const int n = m / HW, p = m - n * HW, h = p / a.W, w = p - h * a.W;
                ou[j] = (((n * hw2) + (h >> 1) * (a.W / 2) + (w >> 1)) * a.ldu + 8 * fq) * 2;
            } else {
                ox[j] = fz::OOB;
                ou[j] = fz::OOB;
            }
        }
    };
    u32x4 bs[D][PW_NB];  // the K-step ring: step kf in slot kf % D
    auto load = [&](int slot, int kf) {
        const int c = 32 * kf;
#pragma unroll
        for (int j = 0; j < PW_NB; ++j)
            bs[slot][j] = c < cu ? __builtin_amdgcn_raw_buffer_load_b128(ru, ou[j] + c * 2, 0, 0)
                                 : __builtin_amdgcn_raw_buffer_load_b128(rx, ox[j] + c * 2, 0, 0);
    };
    tile_offsets(t);
#pragma unroll
    for (int s = 0; s < D; ++s) load(s, s);
    while (true) {
        const int tn = t + stride;
        const bool more = tn < ntiles;
        f32x4 acc[PW_NB][PW_NQ];
#pragma unroll
        for (int q = 0; q < PW_NQ; ++q) {
            const f32x4 b = *(const f32x4*)(bias_s + 32 * (q >> 1) + 8 * fq + 4 * (q & 1));
#pragma unroll
            for (int j = 0; j < PW_NB; ++j) acc[j][q] = b;
        }
        // the weight fragments' LDS address through the opaque lane id, once per tile: keeps the compiler
        // from hoisting all NK * 8 loop-invariant fragment reads out of the tile loop (and spilling them)
        const unsigned char* wl = pw_smem + 16 * fz::lane_id();
        int oy[PW_NB];
#pragma unroll
        for (int j = 0; j < PW_NB; ++j) oy[j] = ox[j] == fz::OOB ? fz::OOB : ((t * PW_TP + 16 * j + fr) * a.ldy + 8 * fq) * 2;
#pragma unroll
        for (int kf = 0; kf < NK; ++kf) {
            // the ring's last D steps of this tile refill with the next tile's first D (past the last tile
            // every offset is out of range: the loads return 0 without touching memory, and stay
            // unconditional so the compiler's vmcnt accounting never has to drain the ring)
            if (kf == NK - D) tile_offsets(tn);
#pragma unroll
            for (int q = 0; q < PW_NQ; ++q) {
                const bf16x8 wa = *(const bf16x8*)(wl + (kf * PW_NQ + q) * 1024);
#pragma unroll
                for (int j = 0; j < PW_NB; ++j) acc[j][q] = mma(wa, (bf16x8)bs[kf % D][j], acc[j][q]);
            }
            if (kf + D < NK) load(kf % D, kf + D);
            else load(kf % D, kf + D - NK);
            // keep each refill right behind the MFMAs that free its slot (the scheduler otherwise sinks all
            // of a tile's refills below the last MFMA and drains the ring to vmcnt(0) every D steps)
            __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int j = 0; j < PW_NB; ++j)
#pragma unroll
            for (int p = 0; p < 4; ++p)
                // the channel offset goes into the voffset (folded into the instruction offset), never into
                // soffset: with an SGPR soffset the compiler treats a VALU write of the 16-byte store data in
                // the next cycle as safe, and on gfx950 it is not (lanes 12-15 of each row group stored the
                // overwritten first dword at p = 2, 3 -- tools/pw_debug.py)
                __builtin_amdgcn_raw_buffer_store_b128(
                    (u32x4)fz::pack(fz::act(acc[j][2 * p]), fz::act(acc[j][2 * p + 1])), ry, oy[j] + 64 * p, 0, 0);
        if (!more) break;
        t = tn;
    }
}

int g_cus = 0;

}  // namespace

// 1x1 / stride 1 / mode 0 / Cout 128 / bf16 in and out, no residual or tail, K = Cin a multiple of 64 up to
// 448 (the weights fit LDS), 16-byte aligned operands, every offset within 31 bits
bool va_pw_eligible(const va_conv_args& a) {
    if (!va_sw().pw) return false;  // VA_PW=0: keep these layers on conv2 (A/B timing, va_switch.h)
    if (a.dtype != VA_DTYPE_BF16 || a.out_f32 || a.kh != 1 || a.kw != 1 || a.stride != 1 || a.pad != 0 ||
        a.mode != 0 || a.w2 || a.res || a.Cout != 128 || a.Cin != a.K || a.K % 64 || a.K > PW_KMAX ||
        a.ldx % 8 || a.ldy % 8 || ((uintptr_t)a.x & 15) || ((uintptr_t)a.y & 15) || ((uintptr_t)a.w & 15) ||
        a.Kpad % 8 || a.Ho != a.H || a.Wo != a.W)
        return false;
    if ((int64_t)a.M * a.ldx * 2 >= 0x7fffffffLL || (int64_t)a.M * a.ldy * 2 >= 0x7fffffffLL) return false;
    if (a.xu && ((int64_t)(a.M / 4 + a.N) * a.ldu * 2 >= 0x7fffffffLL || a.H % 2 || a.W % 2)) return false;
    return true;
}

template <int NK, int D>
hipError_t pw_go(const va_conv_args& a, hipStream_t st, int ntiles, int grid) {
    const int lds = NK * PW_NQ * 1024 + 128 * 4;
    static DevFlag attr;
    if (!attr()) {
        if (hipFuncSetAttribute((const void*)pw_kernel<NK, D>, hipFuncAttributeMaxDynamicSharedMemorySize, lds) !=
            hipSuccess)
            return hipErrorInvalidValue;
        attr() = true;
    }
    hipLaunchKernelGGL((pw_kernel<NK, D>), dim3(grid), dim3(PW_NW * 64), lds, st, a, ntiles);
    return hipGetLastError();
}

hipError_t va_pw_launch(const va_conv_args& a, hipStream_t st) {
    if (g_cus == 0) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&g_cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            return hipErrorInvalidValue;
    }
    const int ntiles = (a.M + PW_TP - 1) / PW_TP;
    int grid = g_cus;
    if ((int64_t)grid * PW_NW > ntiles) grid = (ntiles + PW_NW - 1) / PW_NW;
    switch (a.K / 32) {
        case 2: return pw_go<2, 2>(a, st, ntiles, grid);
        case 4: return pw_go<4, 4>(a, st, ntiles, grid);
        case 6: return pw_go<6, 3>(a, st, ntiles, grid);
        case 8: return pw_go<8, 4>(a, st, ntiles, grid);
        case 10: return pw_go<10, 5>(a, st, ntiles, grid);
        case 12: return pw_go<12, 4>(a, st, ntiles, grid);
        case 14: return pw_go<14, 2>(a, st, ntiles, grid);
        default: return hipErrorInvalidValue;
    }
}

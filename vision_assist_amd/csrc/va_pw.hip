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
//     (lane (p, q): 16 bytes = channels 8q..8q+7 of pixel p), two 32-deep K-steps ahead in a
//     2-slot register ring that runs across tile boundaries -- no LDS for activations, no barrier;
//   * accumulators start from the bias; SiLU epilogue from the accumulators; loads and stores are
//     buffer ops with out-of-range offsets for pixels past M, so none is conditional;
//   * the FPN's upsampled channel prefix (va_conv_args.xu) is read in place like conv2/conv4 do.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "../../include/va355.h"
#include "va_fuse.h"

namespace {

using fz::mma;

constexpr int PW_NW = 8;    // waves per workgroup
constexpr int PW_NB = 3;    // B fragments (16 pixels each) per wave tile
constexpr int PW_TP = 16 * PW_NB;  // pixels per wave tile
constexpr int PW_NQ = 8;    // 16-channel output groups (Cout = 128)
constexpr int PW_KMAX = 448;

__global__ __launch_bounds__(PW_NW * 64, 1) void pw_kernel(va_conv_args a, int ntiles) {
    extern __shared__ __attribute__((aligned(16))) unsigned char pw_smem[];
    const int tid = threadIdx.x, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int nk = a.K / 32;                       // 32-deep K-steps (even: K % 64 == 0)
    float* bias_s = (float*)(pw_smem + nk * PW_NQ * 1024);
    // weights -> LDS: fragment f = kf * 8 + q, lane l: row perm(q, l & 15), k = 32 kf + 8 (l >> 4)
    {
        const __bf16* W = (const __bf16*)a.w;
        for (int i = tid; i < nk * PW_NQ * 64; i += PW_NW * 64) {
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

    // per tile: the byte offsets of this lane's 4 pixels in x and (upsampled prefix) in xu
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
    u32x4 bs[2][PW_NB];  // the K-step ring: slot kf & 1
    auto load = [&](int slot, int kf) {
        const int c = 32 * kf;
#pragma unroll
        for (int j = 0; j < PW_NB; ++j)
            bs[slot][j] = c < cu ? __builtin_amdgcn_raw_buffer_load_b128(ru, ou[j], c * 2, 0)
                                 : __builtin_amdgcn_raw_buffer_load_b128(rx, ox[j], c * 2, 0);
    };
    tile_offsets(t);
    load(0, 0);
    load(1, 1);
    while (true) {
        const int tn = t + stride;
        f32x4 acc[PW_NB][PW_NQ];
#pragma unroll
        for (int q = 0; q < PW_NQ; ++q) {
            const f32x4 b = *(const f32x4*)(bias_s + 32 * (q >> 1) + 8 * fq + 4 * (q & 1));
#pragma unroll
            for (int j = 0; j < PW_NB; ++j) acc[j][q] = b;
        }
        int oy[PW_NB];
#pragma unroll
        for (int j = 0; j < PW_NB; ++j) oy[j] = ox[j] == fz::OOB ? fz::OOB : ((t * PW_TP + 16 * j + fr) * a.ldy + 8 * fq) * 2;
        for (int kp = 0; kp < nk; kp += 2) {
            const bool last = kp + 2 >= nk;
            if (last && tn < ntiles) tile_offsets(tn);  // the ring's next two steps are the next tile's
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int kf = kp + h;
#pragma unroll
                for (int q = 0; q < PW_NQ; ++q) {
                    const bf16x8 wa = *(const bf16x8*)(pw_smem + (kf * PW_NQ + q) * 1024 + 16 * lane);
#pragma unroll
                    for (int j = 0; j < PW_NB; ++j) acc[j][q] = mma(wa, (bf16x8)bs[h][j], acc[j][q]);
                }
                // refill the slot just consumed: two K-steps ahead (the next tile's first two at the end)
                if (!last) load(h, kf + 2);
                else if (tn < ntiles) load(h, h);
            }
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
        if (tn >= ntiles) break;
        t = tn;
    }
}

int g_cus = 0;

}  // namespace

// 1x1 / stride 1 / mode 0 / Cout 128 / bf16 in and out, no residual or tail, K = Cin a multiple of 64 up to
// 448 (the weights fit LDS), 16-byte aligned operands, every offset within 31 bits
bool va_pw_eligible(const va_conv_args& a) {
    const char* e = getenv("VA_PW");  // 0: keep these layers on conv2 (A/B timing; read per call)
    if (e && e[0] == '0') return false;
    if (a.dtype != VA_DTYPE_BF16 || a.out_f32 || a.kh != 1 || a.kw != 1 || a.stride != 1 || a.pad != 0 ||
        a.mode != 0 || a.w2 || a.res || a.Cout != 128 || a.Cin != a.K || a.K % 64 || a.K > PW_KMAX ||
        a.ldx % 8 || a.ldy % 8 || ((uintptr_t)a.x & 15) || ((uintptr_t)a.y & 15) || ((uintptr_t)a.w & 15) ||
        a.Kpad % 8 || a.Ho != a.H || a.Wo != a.W)
        return false;
    if ((int64_t)a.M * a.ldx * 2 >= 0x7fffffffLL || (int64_t)a.M * a.ldy * 2 >= 0x7fffffffLL) return false;
    if (a.xu && ((int64_t)(a.M / 4 + a.N) * a.ldu * 2 >= 0x7fffffffLL || a.H % 2 || a.W % 2)) return false;
    return true;
}

hipError_t va_pw_launch(const va_conv_args& a, hipStream_t st) {
    const int lds = a.K / 32 * PW_NQ * 1024 + 128 * 4;
    if (g_cus == 0) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&g_cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            hipFuncSetAttribute((const void*)pw_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                PW_KMAX / 32 * PW_NQ * 1024 + 128 * 4) != hipSuccess)
            return hipErrorInvalidValue;
    }
    const int ntiles = (a.M + PW_TP - 1) / PW_TP;
    int grid = g_cus;
    if ((int64_t)grid * PW_NW > ntiles) grid = (ntiles + PW_NW - 1) / PW_NW;
    hipLaunchKernelGGL(pw_kernel, dim3(grid), dim3(PW_NW * 64), lds, st, a, ntiles);
    return hipGetLastError();
}

// va_stem.hip -- the network stem as ONE kernel: uint8 BGR frame -> RGB / 255 (LetterBox + ToTensor of
// YOLO.predict at FrameProcessor.py:322, identity for a frame of the network's size) -> model.0 Conv(3, 32,
// 3x3, s2) + SiLU -> model.1 Conv(32, 64, 3x3, s2) + SiLU (ultralytics conv.py Conv.forward, BN folded).
//
// Unfused (va_seg_conv0 + va_seg_conv) the 320 x 320 x 32 model.0 map is written to HBM and read back:
// ~19 MB per frame.  Here a workgroup owns a 16 x 16 tile of the 160 x 160 model.1 output:
//
//   P16   the tile's 67 x 80 input pixels as bf16 (R, G, B, 0) / 255 in LDS (8 bytes a pixel), converted
//         from 48-byte spans of the frame row
//   M0    model.0 on the 33 x 33 pixels the tile's model.1 taps read: k = tap * 4 + channel (36 of two
//         32-deep MFMA steps), a lane's B fragment = two 8-byte P16 pixels; bias + SiLU, zero outside the
//         model.0 map (model.1's padding), stored as two column planes (even / odd columns) so model.1's
//         stride-2 taps read 16 consecutive plane pixels (bank-conflict free with XOR-swizzled chunks)
//   out   model.1: 9 taps x 4 channel groups from M0, bias + SiLU, 16-byte stores of 8 consecutive
//         channels (weight rows permuted on the host)
//
// Persistent (one 512-thread workgroup per CU, XCD-contiguous tile runs); model.0's weights live in
// registers, model.1's in LDS (fragment order); the next tile's frame bytes are loaded into registers at the start of a tile and converted
// into P16 after its model.1, so the load has the whole tile to land.  Rounding matches the unfused layers: model.0 is bias + SiLU in f32
// rounded to bf16 as a stored layer would be.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <type_traits>

#include "../../include/va355.h"
#include "va_dev.h"
#include "va_fuse.h"
#include "va_switch.h"

namespace {

using fz::mma;

constexpr int ST_T = 16;             // model.1 output tile edge
constexpr int ST_NW = 8;             // waves (2 model.1 rows each)
constexpr int ST_M = 2 * ST_T + 1;   // model.0 region edge (33)
constexpr int ST_EW = ST_T + 1, ST_OW = ST_T;  // even / odd column plane widths (17 / 16)
constexpr int ST_PS = 64;            // LDS bytes per model.0 pixel (32 bf16, XOR-swizzled 16-byte chunks)
constexpr int ST_RR = 4 * ST_T + 3;  // input rows of a tile (67)
// P16: the tile's input as bf16 (R, G, B, 0) / 255 pixels, 8 bytes each: columns 4 ox1 - 16 ..
// 4 ox1 + 63 (80 pixels = 5 spans of 16 pixels = 5 x 48 frame bytes, 16-byte aligned in the frame row);
// the first column a window reads (4 ox1 - 3) is P16 column 13
constexpr int ST_PW = 4 * ST_T + 16, ST_SP = ST_PW / 16;  // 80 columns, 5 spans per row
constexpr int ST_NSP = ST_RR * ST_SP;                      // 335 spans per tile (one per thread)
static_assert(ST_NSP <= ST_NW * 64, "one span per thread");
constexpr int ST_G0 = ST_M + ST_M + (ST_M + 15) / 16;  // model.0 groups: even-plane rows, odd-plane rows, column 32
constexpr int ST_NG0 = (ST_G0 + ST_NW - 1) / ST_NW;
// LDS map
constexpr int ST_ME = 0, ST_MO = ST_ME + ST_M * ST_EW * ST_PS, ST_P16 = ST_MO + ST_M * ST_OW * ST_PS;
constexpr int ST_W1 = ST_P16 + ST_RR * ST_PW * 8, ST_BIAS = ST_W1 + 36 * 1024, ST_SINK = ST_BIAS + 96 * 4;
constexpr int ST_LDS = ST_SINK + 64 * 16;
static_assert(ST_LDS + 16 <= 160 * 1024, "LDS (+ the work-queue slots)");
// weight blob (bf16, MFMA A-fragment order): W0 model.0 [2 channel groups][2 K-steps] (k = tap * 4 + c, c =
// R, G, B, 0: 36 of 64; held in registers), W1 model.1 [9 taps][4 groups] (in LDS)
constexpr int ST_FW0 = 0, ST_FW1 = 4 * fz::FRAG, ST_WBLOB = ST_FW1 + 36 * fz::FRAG;
static_assert(ST_WBLOB == 20480, "blob size (seg.py SegNet._pack_stem)");

// chunk c of plane pixel p (XOR swizzle: 16 consecutive pixels' chunk reads and writes are conflict free)
__device__ __forceinline__ int st_addr(int p, int c) { return p * ST_PS + 16 * (c ^ ((p >> 1) & 3)); }

struct StGeom {
    int N, H, W, Ho, Wo, Ho1, Wo1, ldy, tx, tpf, ntiles;
    unsigned long long* trace;  // debug (va_stem_trace): [grid][8 waves][32 tiles][5] real-time stamps, or null
    int* wq;                    // the plan's work counter (va_fuse.h fz::wq_claim), or null: fz::tile's static schedule
};

__global__ __launch_bounds__(ST_NW * 64, 1) void stem_kernel(const uint8_t* __restrict__ frames,
                                                            const __bf16* __restrict__ wf,
                                                            const float* __restrict__ bias, __bf16* __restrict__ Y,
                                                            StGeom g) {
    extern __shared__ __attribute__((aligned(16))) unsigned char st_smem[];
    const int tid = threadIdx.x, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const float* b0 = (const float*)(st_smem + ST_BIAS);  // model.0 [32]
    const float* b1 = b0 + 32;                              // model.1 [64]

    // work queue: tile j's index in LDS slot j & 1, claimed by thread 0 at the start of tile j - 2 and published
    // before its last barrier
    volatile int* slot = (volatile int*)(st_smem + ST_LDS);
    int t, nx;  // this tile, the next
    if (g.wq) {
        if (tid == 0) {
            slot[0] = fz::wq_claim(g.wq, g.ntiles);
            slot[1] = fz::wq_claim(g.wq, g.ntiles);
        }
        __syncthreads();
        t = __builtin_amdgcn_readfirstlane(slot[0]);
        nx = __builtin_amdgcn_readfirstlane(slot[1]);
    } else {
        t = fz::tile(g.ntiles, 0);
        nx = fz::tile(g.ntiles, 1);
    }
    if (t < 0) {
        if (g.wq && tid == 0) fz::wq_release(g.wq);
        return;
    }
    if (tid < 24) *(float4*)(st_smem + ST_BIAS + 16 * tid) = *(const float4*)(bias + 4 * tid);
    for (int i = tid; i < 36 * fz::FRAG / 8; i += ST_NW * 64)
        *(u32x4*)(st_smem + ST_W1 + 16 * i) = *(const u32x4*)(wf + ST_FW1 + 8 * i);
    bf16x8 w0[2][2];
    {
        const int l = tid & 63;
#pragma unroll
        for (int f = 0; f < 4; ++f) w0[f >> 1][f & 1] = *(const bf16x8*)(wf + ST_FW0 + f * fz::FRAG + 8 * l);
    }
    const int fbytes = g.H * g.W * 3;

    // span i (< 335) of tile tt: P16 row i / 5 (frame row 4 oy1 - 3 + row), 16 pixels from column
    // 4 ox1 - 16 + 16 (i % 5): 48 frame bytes in 3 chunks (a chunk is wholly inside or outside the frame)
    u32x4 pf[3];
    auto load_span = [&](int tt) {
        const int n = tt / g.tpf, rr = tt % g.tpf, oy1 = (rr / g.tx) * ST_T, ox1 = (rr % g.tx) * ST_T;
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(frames + (int64_t)n * g.H * g.W * 3), (short)0, fbytes, fz::RSRC);
        const int r = tid / ST_SP, sp = tid - r * ST_SP;
        const int iy = 4 * oy1 - 3 + r, bx = 12 * ox1 - 48 + 48 * sp;
        const bool rok = tid < ST_NSP && (unsigned)iy < (unsigned)g.H;
#pragma unroll
        for (int u = 0; u < 3; ++u) {
            const int b = bx + 16 * u;
            const bool ok = rok && b >= 0 && b < 3 * g.W;
            pf[u] = __builtin_amdgcn_raw_buffer_load_b128(rs, ok ? iy * 3 * g.W + b : fz::OOB, 0, 0);
        }
    };
    // BGR bytes -> (R, G, B, 0) bf16 / 255 (x * (1/255): the bf16 results agree with x / 255 for all 256
    // byte values), two pixels per 16-byte LDS store
    auto store_span = [&]() {
        if (tid >= ST_NSP) return;
        const int r = tid / ST_SP, sp = tid - r * ST_SP;
        unsigned char* dst = st_smem + ST_P16 + (r * ST_PW + 16 * sp) * 8;
        const uint8_t* by = (const uint8_t*)pf;
#pragma unroll
        for (int p = 0; p < 16; p += 2) {
            bf16x8 o;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                o[4 * h + 0] = (__bf16)((float)by[3 * (p + h) + 2] * (1.0f / 255.0f));
                o[4 * h + 1] = (__bf16)((float)by[3 * (p + h) + 1] * (1.0f / 255.0f));
                o[4 * h + 2] = (__bf16)((float)by[3 * (p + h) + 0] * (1.0f / 255.0f));
                o[4 * h + 3] = (__bf16)0.0f;
            }
            *(bf16x8*)(dst + 8 * p) = o;
        }
    };
    load_span(t);
    store_span();
    __syncthreads();

    auto mark = [&](int k, int pt) {  // debug stage stamps (100 MHz clock) of the first 32 tiles
        if (g.trace && k <= 32 && (tid & 63) == 0)
            g.trace[((blockIdx.x * ST_NW + wid) * 32 + k - 1) * 5 + pt] = __builtin_amdgcn_s_memrealtime();
    };
    for (int k = 1; t >= 0; ++k) {
        mark(k, 0);
        const int lane = fz::lane_id(), fr = lane & 15, fq = lane >> 4;
        const int n = t / g.tpf, rr = t % g.tpf, oy1 = (rr / g.tx) * ST_T, ox1 = (rr % g.tx) * ST_T;
        const int tn = nx;
        if (tn >= 0) load_span(tn);  // lands during this tile; converted into P16 after model.1
        int cl = 0;  // the tile after next: claimed here, published before the last barrier (va_fuse.h wq_claim_raw)
        if (g.wq && tid == 0) cl = fz::wq_claim_raw(g.wq);

        // ---- model.0 on the 33 x 33 region (M0 row mr <-> model.0 row 2 oy1 - 1 + mr, column j likewise)
        {
            // this lane's taps: K-step s holds taps 8 s + 2 fq, 8 s + 2 fq + 1 (4 values each); taps past 8
            // (K padding, zero weights) read tap 0's pixel, so every read is unconditional
            int toff[2][2];
#pragma unroll
            for (int st = 0; st < 2; ++st) {
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const int tap = 8 * st + 2 * fq + h;
                    toff[st][h] = tap < 9 ? ((tap / 3) * ST_PW + tap % 3) * 8 : 0;
                }
            }
            const f32x4 c0 = *(const f32x4*)(b0 + 4 * fq), c1 = *(const f32x4*)(b0 + 16 + 4 * fq);
            // group gi: rows of the even plane (gi < 33), of the odd plane (< 66), then column 32 (three
            // groups of 16 rows).  Branch-free bodies (one copy per group count) so the compiler
            // interleaves the groups' LDS reads, MFMAs and SiLU chains.
            auto groups = [&](auto ngc) {
                constexpr int NG = decltype(ngc)::value;
#pragma unroll
                for (int jg = 0; jg < NG; ++jg) {
                    const int gi = wid + ST_NW * jg;
                    const int q = 16 * (gi - 2 * ST_M) + fr;
                    const bool col32 = gi >= 2 * ST_M, valid = !col32 || q < ST_M;
                    const int mr = col32 ? (valid ? q : ST_M - 1) : (gi < ST_M ? gi : gi - ST_M);
                    const int j = col32 ? 2 * ST_T : 2 * fr + (gi >= ST_M ? 1 : 0);
                    // window corner: P16 row 2 mr, column 13 + 2 j
                    const unsigned char* wb = st_smem + ST_P16 + (2 * mr * ST_PW + 13 + 2 * j) * 8;
                    f32x4 a0 = c0, a1 = c1;
#pragma unroll
                    for (int st = 0; st < 2; ++st) {
                        const uint2 lo = *(const uint2*)(wb + toff[st][0]), hi = *(const uint2*)(wb + toff[st][1]);
                        const u32x4 bu = {lo.x, lo.y, hi.x, hi.y};
                        a0 = mma(w0[0][st], (bf16x8)bu, a0);
                        a1 = mma(w0[1][st], (bf16x8)bu, a1);
                    }
                    const int y = 2 * oy1 - 1 + mr, x = 2 * ox1 - 1 + j;
                    const bf16x8 v = fz::zero_if(fz::pack(fz::act(a0), fz::act(a1)),
                                                 (unsigned)y >= (unsigned)g.Ho || (unsigned)x >= (unsigned)g.Wo);
                    const int ad = !valid ? ST_SINK + 16 * lane
                                   : (j & 1) ? ST_MO + st_addr(mr * ST_OW + (j >> 1), fq)
                                             : ST_ME + st_addr(mr * ST_EW + (j >> 1), fq);
                    *(bf16x8*)(st_smem + ad) = v;
                }
            };
            if (wid + ST_NW * (ST_NG0 - 1) < ST_G0)
                groups(std::integral_constant<int, ST_NG0>{});
            else
                groups(std::integral_constant<int, ST_NG0 - 1>{});
        }
        mark(k, 1);
        __syncthreads();
        mark(k, 2);

        // ---- model.1: output rows 2 wid, 2 wid + 1 of the tile; taps read M0 one ahead
        {
            const int r0 = 2 * wid;
            auto boff = [&](int i, int tap) {  // tap (ky, kx): M0 row 2 r + ky, column 2 c + kx
                const int ky = tap / 3, kx = tap % 3, mr = 2 * (r0 + i) + ky;
                return (kx & 1) ? ST_MO + st_addr(mr * ST_OW + fr, fq) : ST_ME + st_addr(mr * ST_EW + fr + (kx >> 1), fq);
            };
            f32x4 acc[2][4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const f32x4 bq = *(const f32x4*)(b1 + 32 * (q >> 1) + 8 * fq + 4 * (q & 1));
                acc[0][q] = bq;
                acc[1][q] = bq;
            }
            bf16x8 wa[2][4], bv[2][2];
            auto fetch = [&](int tap, int sl) {
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    wa[sl][q] = *(const bf16x8*)(st_smem + ST_W1 + (4 * tap + q) * 1024 + 16 * lane);
#pragma unroll
                for (int i = 0; i < 2; ++i) bv[sl][i] = *(const bf16x8*)(st_smem + boff(i, tap));
            };
            fetch(0, 0);
#pragma unroll
            for (int tap = 0; tap < 9; ++tap) {
                if (tap < 8) fetch(tap + 1, (tap + 1) & 1);
#pragma unroll
                for (int q = 0; q < 4; ++q) {
#pragma unroll
                    for (int i = 0; i < 2; ++i) acc[i][q] = mma(wa[tap & 1][q], bv[tap & 1][i], acc[i][q]);
                }
            }
            const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc(
                (void*)(Y + (int64_t)n * g.Ho1 * g.Wo1 * g.ldy), (short)0, g.Ho1 * g.Wo1 * g.ldy * 2, fz::RSRC);
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int y = oy1 + r0 + i, x = ox1 + fr;
                const int off = (y < g.Ho1 && x < g.Wo1) ? ((y * g.Wo1 + x) * g.ldy + 8 * fq) * 2 : fz::OOB;
#pragma unroll
                for (int h = 0; h < 2; ++h)
                    __builtin_amdgcn_raw_buffer_store_b128(
                        (u32x4)fz::pack(fz::act(acc[i][2 * h]), fz::act(acc[i][2 * h + 1])), ry, off, 64 * h, 0);
            }
        }
        mark(k, 3);
        if (tn >= 0) store_span();
        if (g.wq && tid == 0) slot[(k + 1) & 1] = cl < g.ntiles ? cl : -1;
        __syncthreads();
        mark(k, 4);
        nx = g.wq ? __builtin_amdgcn_readfirstlane(slot[(k + 1) & 1]) : fz::tile(g.ntiles, k + 1);
        t = tn;
    }
    if (g.wq && tid == 0) fz::wq_release(g.wq);  // after this workgroup's last (failed) claim
}

int g_cus = 0;
unsigned long long* g_trace = nullptr;

}  // namespace

extern "C" int va_stem_trace(void* buf) {
    g_trace = (unsigned long long*)buf;
    return VA_OK;
}

extern "C" int va_seg_stem(void* stream, const va_conv_args* a) {
    if (!a || !a->x || !a->w || !a->bias || !a->y || a->dtype != VA_DTYPE_BF16 || a->Cin != 32 || a->Cout != 64 ||
        a->N <= 0 || a->H <= 0 || a->W <= 0 || a->W % 16 || a->ldy < 64 || a->ldy % 8 || ((uintptr_t)a->x & 15) ||
        ((uintptr_t)a->y & 15) || ((uintptr_t)a->w & 15) || ((uintptr_t)a->bias & 15))
        return VA_ERR_ARG;
    StGeom g;
    g.N = a->N;
    g.H = a->H;
    g.W = a->W;
    g.Ho = (a->H + 1) / 2;
    g.Wo = (a->W + 1) / 2;
    g.Ho1 = (g.Ho + 1) / 2;
    g.Wo1 = (g.Wo + 1) / 2;
    g.ldy = a->ldy;
    g.trace = g_trace;
    g.wq = a->wcnt && a->ncnt >= 2 && va_sw().conv3q != 2 ? a->wcnt : nullptr;
    // per-frame buffer descriptors: a frame's bytes (and the OOB sentinel above them) must fit 31 bits
    if ((int64_t)a->H * a->W * 3 >= 0x80000000LL || (int64_t)g.Ho1 * g.Wo1 * g.ldy * 2 >= 0x80000000LL)
        return VA_ERR_ARG;
    g.tx = (g.Wo1 + ST_T - 1) / ST_T;
    g.tpf = g.tx * ((g.Ho1 + ST_T - 1) / ST_T);
    const int64_t nt = (int64_t)g.tpf * a->N;
    if (nt > INT32_MAX) return VA_ERR_ARG;
    g.ntiles = (int)nt;
    static DevFlag ready;  // CU count + dynamic-LDS attribute, per device
    if (!ready()) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&g_cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            hipFuncSetAttribute((const void*)stem_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, ST_LDS + 16) !=
                hipSuccess)
            return VA_ERR_HIP;
        ready() = true;
    }
    int grid = g_cus;
    if (grid > g.ntiles) grid = g.ntiles;
    if (g.ntiles < fz::WQ_MIN_TILES_PER_WG * grid) g.wq = nullptr;  // one or two tiles per workgroup: static
    hipLaunchKernelGGL(stem_kernel, dim3(grid), dim3(ST_NW * 64), ST_LDS + 16, (hipStream_t)stream,
                       (const uint8_t*)a->x, (const __bf16*)a->w, a->bias, (__bf16*)a->y, g);
    return hipGetLastError() == hipSuccess ? VA_OK : VA_ERR_HIP;
}

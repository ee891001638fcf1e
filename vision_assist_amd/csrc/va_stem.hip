// va_stem.hip -- the network stem as ONE kernel: uint8 BGR frame -> RGB / 255 (LetterBox + ToTensor of
// YOLO.predict at FrameProcessor.py:322, identity for a frame of the network's size) -> model.0 Conv(3, 32,
// 3x3, s2) + SiLU -> model.1 Conv(32, 64, 3x3, s2) + SiLU (ultralytics conv.py Conv.forward, BN folded).
//
// Unfused (va_seg_conv0 + va_seg_conv) the 320 x 320 x 32 model.0 map is written to HBM and read back:
// ~19 MB per frame.  Here a workgroup owns a 16 x 16 tile of the 160 x 160 model.1 output:
//
//   RAW   the tile's 67 x 67 input pixels (67 rows x 208 bytes of the frame, 16-byte chunks) in LDS
//   M0    model.0 on the 33 x 33 pixels the tile's model.1 taps read: B fragments built from RAW bytes
//         (k = tap * 3 + channel, 27 of one 32-deep MFMA step), bias + SiLU, zero outside the model.0
//         map (model.1's padding), stored as two column planes (even / odd columns) so model.1's
//         stride-2 taps read 16 consecutive plane pixels (bank-conflict free, 96-byte pixel pitch:
//         every tap is a constant offset)
//   out   model.1: 9 taps x 4 channel groups from M0, bias + SiLU, 16-byte stores of 8 consecutive
//         channels (weight rows permuted on the host)
//
// Persistent (one 512-thread workgroup per CU, XCD-contiguous tile runs); the next tile's RAW bytes
// are loaded into registers at the start of a tile and written to LDS after its model.1, so the load
// has the whole tile to land.  Rounding matches the unfused layers: model.0 is bias + SiLU in f32
// rounded to bf16 as a stored layer would be.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "../../include/va355.h"
#include "va_fuse.h"

namespace {

using fz::mma;

constexpr int ST_T = 16;             // model.1 output tile edge
constexpr int ST_NW = 8;             // waves (2 model.1 rows each)
constexpr int ST_M = 2 * ST_T + 1;   // model.0 region edge (33)
constexpr int ST_EW = ST_T + 1, ST_OW = ST_T;  // even / odd column plane widths (17 / 16)
constexpr int ST_PS = 96;            // LDS bytes per model.0 pixel (32 bf16 + padding)
constexpr int ST_RR = 4 * ST_T + 3;  // RAW rows (67)
constexpr int ST_RP = 208;           // RAW row pitch: 13 chunks of 16 bytes; first pixel at byte 7
constexpr int ST_RC = ST_RP / 16;
constexpr int ST_NCH = ST_RR * ST_RC;               // 871 chunks
constexpr int ST_CPT = (ST_NCH + ST_NW * 64 - 1) / (ST_NW * 64);  // chunks per thread (2)
constexpr int ST_G0 = ST_M + ST_M + (ST_M + 15) / 16;  // model.0 groups: even-plane rows, odd-plane rows, column 32
constexpr int ST_NG0 = (ST_G0 + ST_NW - 1) / ST_NW;
// LDS map
constexpr int ST_ME = 0, ST_MO = ST_ME + ST_M * ST_EW * ST_PS, ST_RAW = ST_MO + ST_M * ST_OW * ST_PS;
constexpr int ST_W1 = ST_RAW + ST_RR * ST_RP, ST_BIAS = ST_W1 + 36 * 1024, ST_SINK = ST_BIAS + 96 * 4;
constexpr int ST_LDS = ST_SINK + 64 * 16;
static_assert(ST_LDS <= 160 * 1024, "LDS");
// weight blob (bf16, MFMA A-fragment order): W0 model.0 [2 channel groups], W1 model.1 [9 taps][4 groups]
constexpr int ST_FW0 = 0, ST_FW1 = 2 * fz::FRAG, ST_WBLOB = ST_FW1 + 36 * fz::FRAG;
static_assert(ST_WBLOB == 19456, "blob size (seg.py SegNet._pack_stem)");

struct StGeom {
    int N, H, W, Ho, Wo, Ho1, Wo1, ldy, tx, tpf, ntiles;
};

__global__ __launch_bounds__(ST_NW * 64, 1) void stem_kernel(const uint8_t* __restrict__ frames,
                                                            const __bf16* __restrict__ wf,
                                                            const float* __restrict__ bias, __bf16* __restrict__ Y,
                                                            StGeom g) {
    extern __shared__ __attribute__((aligned(16))) unsigned char st_smem[];
    const int tid = threadIdx.x, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const float* b0 = (const float*)(st_smem + ST_BIAS);  // model.0 [32]
    const float* b1 = b0 + 32;                              // model.1 [64]

    int t = fz::tile(g.ntiles, 0);
    if (t < 0) return;
    for (int i = tid; i < 36 * fz::FRAG / 8; i += ST_NW * 64)
        *(u32x4*)(st_smem + ST_W1 + 16 * i) = *(const u32x4*)(wf + ST_FW1 + 8 * i);
    if (tid < 24) *(float4*)(st_smem + ST_BIAS + 16 * tid) = *(const float4*)(bias + 4 * tid);
    bf16x8 w0[2];
    {
        const int l = tid & 63;
        w0[0] = *(const bf16x8*)(wf + ST_FW0 + 8 * l);
        w0[1] = *(const bf16x8*)(wf + ST_FW0 + fz::FRAG + 8 * l);
    }
    const int fbytes = g.H * g.W * 3;

    // RAW chunk i of tile tt: row i / 13 (frame row 4 oy1 - 3 + row), bytes 12 ox1 - 16 + 16 (i % 13)
    u32x4 pf[ST_CPT];
    auto load_raw = [&](int tt) {
        const int n = tt / g.tpf, rr = tt % g.tpf, oy1 = (rr / g.tx) * ST_T, ox1 = (rr % g.tx) * ST_T;
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(frames + (int64_t)n * g.H * g.W * 3), (short)0, fbytes, fz::RSRC);
#pragma unroll
        for (int u = 0; u < ST_CPT; ++u) {
            const int i = tid + u * ST_NW * 64;
            const int r = i / ST_RC, c = i - r * ST_RC;
            const int iy = 4 * oy1 - 3 + r, bx = 12 * ox1 - 16 + 16 * c;
            const bool ok = i < ST_NCH && (unsigned)iy < (unsigned)g.H && bx >= 0 && bx < 3 * g.W;
            pf[u] = __builtin_amdgcn_raw_buffer_load_b128(rs, ok ? iy * 3 * g.W + bx : fz::OOB, 0, 0);
        }
    };
    auto store_raw = [&]() {
#pragma unroll
        for (int u = 0; u < ST_CPT; ++u) {
            const int i = tid + u * ST_NW * 64;
            if (i < ST_NCH) *(u32x4*)(st_smem + ST_RAW + 16 * i) = pf[u];
        }
    };
    load_raw(t);
    store_raw();
    __syncthreads();

    for (int k = 1; t >= 0; ++k) {
        const int lane = fz::lane_id(), fr = lane & 15, fq = lane >> 4;
        const int n = t / g.tpf, rr = t % g.tpf, oy1 = (rr / g.tx) * ST_T, ox1 = (rr % g.tx) * ST_T;
        const int tn = fz::tile(g.ntiles, k);
        if (tn >= 0) load_raw(tn);  // lands during this tile; written to RAW after model.1
        const bool interior = oy1 >= 1 && ox1 >= 1 && 2 * oy1 + 2 * ST_T <= g.Ho && 2 * ox1 + 2 * ST_T <= g.Wo;

        // ---- model.0 on the 33 x 33 region (M0 row mr <-> model.0 row 2 oy1 - 1 + mr, column j likewise)
        {
            // this lane's k values -> RAW byte offsets from the window corner.  k >= 27 (K padding) reads
            // the corner byte: its weights are zero, so every read is unconditional (no exec-mask branches)
            int koff[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const int kk = 8 * fq + e, tap = kk / 3, ch = kk % 3;  // ch: R, G, B; the frame is BGR
                koff[e] = kk < 27 ? (tap / 3) * ST_RP + (tap % 3) * 3 + (2 - ch) : 0;
            }
            const f32x4 c0 = *(const f32x4*)(b0 + 4 * fq), c1 = *(const f32x4*)(b0 + 16 + 4 * fq);
#pragma unroll
            for (int jg = 0; jg < ST_NG0; ++jg) {
                const int gi = wid + ST_NW * jg;
                if (gi < ST_G0) {
                    int mr, j;
                    bool valid = true;
                    if (gi < ST_M) {
                        mr = gi;
                        j = 2 * fr;
                    } else if (gi < 2 * ST_M) {
                        mr = gi - ST_M;
                        j = 2 * fr + 1;
                    } else {
                        const int q = 16 * (gi - 2 * ST_M) + fr;
                        valid = q < ST_M;
                        mr = valid ? q : ST_M - 1;
                        j = 2 * ST_T;
                    }
                    const unsigned char* wb = st_smem + ST_RAW + 2 * mr * ST_RP + 7 + 6 * j;
                    // x * (1/255) instead of x / 255 (no f32 division): the bf16 results agree for all 256 byte values
                    bf16x8 bfr;
#pragma unroll
                    for (int e = 0; e < 8; ++e)
                        bfr[e] = (__bf16)((float)wb[koff[e]] * (1.0f / 255.0f));
                    bf16x8 v = fz::pack(fz::act(mma(w0[0], bfr, c0)), fz::act(mma(w0[1], bfr, c1)));
                    if (!interior) {
                        const int y = 2 * oy1 - 1 + mr, x = 2 * ox1 - 1 + j;
                        v = fz::zero_if(v, (unsigned)y >= (unsigned)g.Ho || (unsigned)x >= (unsigned)g.Wo);
                    }
                    const int ad = !valid ? ST_SINK + 16 * lane
                                   : (j & 1) ? ST_MO + (mr * ST_OW + (j >> 1)) * ST_PS + 16 * fq
                                             : ST_ME + (mr * ST_EW + (j >> 1)) * ST_PS + 16 * fq;
                    *(bf16x8*)(st_smem + ad) = v;
                }
            }
        }
        __syncthreads();

        // ---- model.1: output rows 2 wid, 2 wid + 1 of the tile; taps read M0 one ahead
        {
            const int r0 = 2 * wid;
            // per row: even-plane and odd-plane address of tap (0, 0) / (0, 1)
            int be[2], bo[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                be[i] = ST_ME + (2 * (r0 + i) * ST_EW + fr) * ST_PS + 16 * fq;
                bo[i] = ST_MO + (2 * (r0 + i) * ST_OW + fr) * ST_PS + 16 * fq;
            }
            auto boff = [&](int i, int tap) {  // tap (ky, kx): M0 row 2 r + ky, column 2 c + kx
                const int ky = tap / 3, kx = tap % 3;
                return (kx & 1) ? bo[i] + ky * ST_OW * ST_PS : be[i] + (ky * ST_EW + (kx >> 1)) * ST_PS;
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
        if (tn >= 0) store_raw();
        __syncthreads();
        t = tn;
    }
}

int g_cus = 0;

}  // namespace

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
    // per-frame buffer descriptors: a frame's bytes (and the OOB sentinel above them) must fit 31 bits
    if ((int64_t)a->H * a->W * 3 >= 0x80000000LL || (int64_t)g.Ho1 * g.Wo1 * g.ldy * 2 >= 0x80000000LL)
        return VA_ERR_ARG;
    g.tx = (g.Wo1 + ST_T - 1) / ST_T;
    g.tpf = g.tx * ((g.Ho1 + ST_T - 1) / ST_T);
    const int64_t nt = (int64_t)g.tpf * a->N;
    if (nt > INT32_MAX) return VA_ERR_ARG;
    g.ntiles = (int)nt;
    if (g_cus == 0) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&g_cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            hipFuncSetAttribute((const void*)stem_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, ST_LDS) !=
                hipSuccess)
            return VA_ERR_HIP;
    }
    int grid = g_cus;
    if (grid > g.ntiles) grid = g.ntiles;
    hipLaunchKernelGGL(stem_kernel, dim3(grid), dim3(ST_NW * 64), ST_LDS, (hipStream_t)stream,
                       (const uint8_t*)a->x, (const __bf16*)a->w, a->bias, (__bf16*)a->y, g);
    return hipGetLastError() == hipSuccess ? VA_OK : VA_ERR_HIP;
}

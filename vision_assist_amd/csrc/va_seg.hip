// va_seg.hip -- YOLOv8-seg forward on MI355X (gfx950): the segmentation half of the hot path
// (YOLO.predict as called at FrameProcessor.py:322; Ultralytics is external).
//
// Activations are NHWC, channel-sliced: every tensor is (pointer to its first channel, channel
// stride of the buffer it lives in), so C2f's chunk/cat, SPPF's cat and the FPN/PAN concats are
// zero-copy -- producers write straight into their slice of the consumer's input buffer.
//
//   seg_preprocess_kernel   uint8 BGR HWC -> RGB/255 NHWC, channels padded to 8 (LetterBox is the
//                           identity for a frame that already has the network's input size)
//   conv_kernel<T, WM, WN>  implicit-GEMM Conv2d (+ folded BN bias, SiLU, residual add) on MFMA:
//                           bf16 -> v_mfma_f32_16x16x32_bf16, f32 (parity mode) -> v_mfma_f32_16x16x4_f32
//                           (exact f32 fma chain).  D[cout][pixel] = W[cout][k] * im2col[k][pixel]:
//                           weights are the MFMA A operand so each lane's accumulator holds 4
//                           consecutive output channels of one pixel (8/16-byte NHWC stores).
//                           mode 1 = ConvTranspose2d(k2, s2) as a 1x1 GEMM with 4*C outputs whose
//                           epilogue scatters the 2x2 sub-pixels (Proto.upsample).
//   sppf_pool_kernel<T>     SPPF's three chained MaxPool2d(5,1,2) as one pass: 5x5, 9x9, 13x13 maxima
//   upsample2x_kernel<T>    nearest x2 into a concat slice
#include <hip/hip_runtime.h>
#include <mutex>
#include <type_traits>
#include <stdint.h>
#include <stdlib.h>

#include "../../include/va355.h"
#include "va_switch.h"
#include "va_dev.h"
#include "va_fuse.h"

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;
// staging registers: a native vector type (HIP's uint4 is a union-based class whose arrays defeat
// SROA and end up in scratch / LDS)
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;

// va_pw.hip: the streaming pointwise kernel for 1x1 / Cout-128 layers
bool va_pw_eligible(const va_conv_args& a);
hipError_t va_pw_launch(const va_conv_args& a, hipStream_t st);
bool va_fp8_conv_ok(const va_conv_args& a);
hipError_t va_fp8_conv_launch(const va_conv_args& a, hipStream_t st);

namespace {

__device__ inline float to_f(float v) { return v; }
__device__ inline float to_f(__bf16 v) { return (float)v; }
template <typename T>
__device__ inline T from_f(float v);
template <>
__device__ inline float from_f<float>(float v) {
    return v;
}
template <>
__device__ inline __bf16 from_f<__bf16>(float v) {
    return (__bf16)v;
}

// bf16-output kernels: hardware exp and reciprocal (~1 ulp f32, far below the bf16 rounding that
// follows); the exact-f32 parity path uses silu_exact
__device__ inline float silu(float x) { return x * __builtin_amdgcn_rcpf(1.0f + __expf(-x)); }
__device__ inline float silu_exact(float x) { return x / (1.0f + expf(-x)); }
// silu() over an array, the plain f32 steps packed in pairs (fz::silu2): bit-identical to silu() per element
template <int N>
__device__ __forceinline__ void silu_n(float (&v)[N]) {
    static_assert(N % 2 == 0, "pairs");
#pragma unroll
    for (int i = 0; i < N; i += 2) {
        const f32x2 r = fz::silu2((f32x2){v[i], v[i + 1]});
        v[i] = r[0];
        v[i + 1] = r[1];
    }
}

// e4m3 weight bytes in the bf16 kernels (va_conv_args.w8, C5's weight-only fp8 form): eight e4m3 values (a uint2,
// element e = byte e) -> the 16-byte bf16 chunk the kernels stage.  Every e4m3 value is exact in bf16 (3 mantissa
// bits, exponents 2^-9 .. 2^8), so nothing is rounded here; the weights' per-output-channel scale multiplies the f32
// accumulator in the epilogue (v_cvt_scalef32_pk_bf16_fp8, scale 1)
// The e4m3 weight rows' K order (va355.h va_conv_args.w8): in every 64-element K block the eight 8-element chunks are
// stored as 0, 4, 1, 5, 2, 6, 3, 7, so a lane's two MFMA K-halves (chunks c and c + 4) are one 16-byte piece; chunk c
// of a row sits at byte 8 w8_pos(c)
__device__ __forceinline__ int w8_pos(int c) { return (c & ~7) | ((c & 3) << 1) | ((c >> 2) & 1); }
__device__ __forceinline__ u32x4 e4m3x8_bf16(uint2 q) {
    typedef __attribute__((ext_vector_type(2))) __bf16 b2;
    const b2 a = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8((int)q.x, 1.0f, false);
    const b2 b = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8((int)q.x, 1.0f, true);
    const b2 c = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8((int)q.y, 1.0f, false);
    const b2 d = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8((int)q.y, 1.0f, true);
    return (u32x4){__builtin_bit_cast(unsigned, a), __builtin_bit_cast(unsigned, b), __builtin_bit_cast(unsigned, c),
                   __builtin_bit_cast(unsigned, d)};
}

// ----------------------------------------------------------------------------------------- preprocess
template <typename T>
__global__ void seg_preprocess_kernel(const uint8_t* __restrict__ frames, int64_t npix, T* __restrict__ out) {
    // frames: [npix][3] BGR; out: [npix][8] (R, G, B, 0, 0, 0, 0, 0) / 255
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < npix; i += (int64_t)gridDim.x * blockDim.x) {
        const uint8_t* p = frames + 3 * i;
        float b = p[0], g = p[1], r = p[2];
        T* o = out + 8 * i;
        o[0] = from_f<T>(r / 255.0f);
        o[1] = from_f<T>(g / 255.0f);
        o[2] = from_f<T>(b / 255.0f);
#pragma unroll
        for (int c = 3; c < 8; ++c) o[c] = from_f<T>(0.0f);
    }
}

// ----------------------------------------------------------------------------------------- conv
constexpr int BK = 32;

template <typename T, int WM, int WN>
struct ConvCfg {
    static constexpr int NT = 64 * WM * WN;           // threads
    static constexpr int BM = 64 * WM;                // pixels per tile
    static constexpr int BN = 64 * WN;                // output channels per tile
    static constexpr int VEC = 16 / sizeof(T);        // elements per 16-byte chunk
    static constexpr int CPR = BK / VEC;              // chunks per tile row
    static constexpr int LDSW = BK + VEC;             // padded LDS row (elements)
    static constexpr int A_CH = BN * CPR / NT;        // weight chunks per thread
    static constexpr int B_CH = BM * CPR / NT;        // pixel chunks per thread
    static_assert(A_CH >= 1 && B_CH >= 1, "tile too small for the block");
};

template <typename T, int WM, int WN, typename OutT>
__global__ __launch_bounds__(64 * WM* WN) void conv_kernel(va_conv_args a) {
    using Cfg = ConvCfg<T, WM, WN>;
    constexpr int NT = Cfg::NT, BM = Cfg::BM, BN = Cfg::BN, VEC = Cfg::VEC, CPR = Cfg::CPR, LDSW = Cfg::LDSW;
    constexpr int A_CH = Cfg::A_CH, B_CH = Cfg::B_CH;
    __shared__ __align__(16) T As[BN * LDSW];
    __shared__ __align__(16) T Bs[BM * LDSW];

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid / WN, wn = wid % WN;
    const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
    const T* __restrict__ X = (const T*)a.x;
    const T* __restrict__ Wt = (const T*)a.w;

    // fixed per-thread k-group and rows
    const int g = tid % CPR;
    int b_row[B_CH], b_hi[B_CH], b_wi[B_CH];
    int64_t b_base[B_CH];
#pragma unroll
    for (int i = 0; i < B_CH; ++i) {
        int r = tid / CPR + (NT / CPR) * i;
        int m = m0 + r;
        b_row[i] = r;
        if (m < a.M) {
            int wo = m % a.Wo, t = m / a.Wo, ho = t % a.Ho, n = t / a.Ho;
            b_hi[i] = ho * a.stride - a.pad;
            b_wi[i] = wo * a.stride - a.pad;
            b_base[i] = (int64_t)n * a.H * a.W;
        } else {
            b_hi[i] = -(1 << 28);  // never in bounds
            b_wi[i] = 0;
            b_base[i] = 0;
        }
    }
    const int a_row0 = tid / CPR;

    u32x4 ra[A_CH], rb[B_CH];
    auto load_tile = [&](int k0) {
#pragma unroll
        for (int i = 0; i < A_CH; ++i) {
            int r = a_row0 + (NT / CPR) * i;
            if (sizeof(T) == 2 && a.w8)  // e4m3 weight bytes (bf16 only): converted as loaded (a fallback kernel)
                ra[i] = e4m3x8_bf16(*(const uint2*)((const uint8_t*)a.w + (int64_t)(n0 + r) * a.Kpad +
                                                    8 * w8_pos((k0 + g * VEC) / 8)));
            else
                ra[i] = *(const u32x4*)(Wt + (int64_t)(n0 + r) * a.Kpad + k0 + g * VEC);
        }
        int k = k0 + g * VEC;
        int tap = k / a.Cin, ci = k - tap * a.Cin;
        int ky = tap / a.kw, kx = tap - ky * a.kw;
        bool kin = k < a.K;
#pragma unroll
        for (int i = 0; i < B_CH; ++i) {
            int hi = b_hi[i] + ky, wi = b_wi[i] + kx;
            if (kin && hi >= 0 && hi < a.H && wi >= 0 && wi < a.W)
                rb[i] = *(const u32x4*)(X + (b_base[i] + (int64_t)hi * a.W + wi) * a.ldx + ci);
            else
                rb[i] = (u32x4){0u, 0u, 0u, 0u};
        }
    };
    auto store_tile = [&]() {
#pragma unroll
        for (int i = 0; i < A_CH; ++i) {
            int r = a_row0 + (NT / CPR) * i;
            *(u32x4*)(As + r * LDSW + g * VEC) = ra[i];
        }
#pragma unroll
        for (int i = 0; i < B_CH; ++i) *(u32x4*)(Bs + b_row[i] * LDSW + g * VEC) = rb[i];
    };

    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

    load_tile(0);
    store_tile();
    __syncthreads();
    const int fr = lane & 15, fq = lane >> 4;
    for (int k0 = 0; k0 < a.Kpad; k0 += BK) {
        const bool more = k0 + BK < a.Kpad;
        if (more) load_tile(k0 + BK);
        if constexpr (sizeof(T) == 2) {
            bf16x8 af[4], bfr[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) af[i] = *(const bf16x8*)(As + (wn * 64 + 16 * i + fr) * LDSW + 8 * fq);
#pragma unroll
            for (int j = 0; j < 4; ++j) bfr[j] = *(const bf16x8*)(Bs + (wm * 64 + 16 * j + fr) * LDSW + 8 * fq);
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
        } else {
#pragma unroll
            for (int kk = 0; kk < BK / 4; ++kk) {
                float af[4], bfr[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) af[i] = As[(wn * 64 + 16 * i + fr) * LDSW + 4 * kk + fq];
#pragma unroll
                for (int j = 0; j < 4; ++j) bfr[j] = Bs[(wm * 64 + 16 * j + fr) * LDSW + 4 * kk + fq];
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], bfr[j], acc[i][j], 0, 0, 0);
            }
        }
        __syncthreads();
        if (more) {
            store_tile();
            __syncthreads();
        }
    }

    // ---- epilogue: bias (+SiLU) (+residual), 4 consecutive channels per lane
    OutT* Y = (OutT*)a.y;
    const T* R = (const T*)a.res;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int m = m0 + wm * 64 + 16 * j + fr;
        if (m >= a.M) continue;
        int64_t obase;
        int wo = 0, ho = 0, n = 0;
        if (a.mode == 1) {
            wo = m % a.Wo;
            int t = m / a.Wo;
            ho = t % a.Ho;
            n = t / a.Ho;
            obase = 0;
        } else {
            obase = (int64_t)m * a.ldy;
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int co = n0 + wn * 64 + 16 * i + 4 * fq;
            if (co >= a.Cout) continue;
            float v[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                float x = (a.w8 ? acc[i][j][r] * a.wscale[co + r] : acc[i][j][r]) + a.bias[co + r];
                if (a.act) x = sizeof(T) == 2 ? silu(x) : silu_exact(x);
                v[r] = x;
            }
            if (R) {
                const T* rp = R + (int64_t)m * a.ldr + co;
#pragma unroll
                for (int r = 0; r < 4; ++r) v[r] += to_f(rp[r]);
            }
            OutT* yp;
            if (a.mode == 1) {
                const int cd = a.Cout / 4;
                const int q = co / cd, c = co - q * cd;
                const int oy = 2 * ho + (q >> 1), ox = 2 * wo + (q & 1);
                yp = Y + (((int64_t)n * 2 * a.Ho + oy) * 2 * a.Wo + ox) * a.ldy + c;
            } else {
                yp = Y + obase + co;
            }
            if (co + 3 < a.Cout) {
                if constexpr (sizeof(OutT) == 2) {
                    __bf16 o4[4] = {(__bf16)v[0], (__bf16)v[1], (__bf16)v[2], (__bf16)v[3]};
                    *(uint2*)yp = *(uint2*)o4;
                } else {
                    *(float4*)yp = make_float4(v[0], v[1], v[2], v[3]);
                }
            } else {
                for (int r = 0; r < 4 && co + r < a.Cout; ++r) yp[r] = from_f<OutT>(v[r]);
            }
        }
    }
}

// ----------------------------------------------------------------------------------------- conv v2 (bf16)
// The bf16 production kernel.
//   * tile: WM x WN waves, each wave 64 pixels x (16*TNS) output channels (TNS = 4 or 2 16-wide
//     MFMA column tiles), BK = 64;
//   * two LDS stages with ONE barrier per K-step (the next stage is written while the current one
//     is read); all LDS is one __shared__ array (a second __shared__ object can make hipcc wait
//     vmcnt(0) before every ds_read, cdna_hip_programming.md §5 "three .s-level traps" (a));
//   * incremental im2col (tap, ci) bookkeeping instead of per-step division; out-of-image and
//     K-padding taps load from the tensor base and are zeroed by a select (a branch around each
//     load makes hipcc wait vmcnt(0) per load);
//   * staging registers are native vectors (HIP's uint4 is a union class whose arrays end up in
//     scratch or get promoted to LDS);
//   * epilogue through LDS: accumulators (+bias, SiLU) are parked as f32 in the freed stage
//     buffers, then every thread writes whole 16-byte runs of consecutive channels of one pixel
//     (+ residual read the same way), so the NHWC stores are row-contiguous;
//   * XCD-aware tile order: blocks b and b+8 share an XCD (MI355X_MICROARCH.md "Workgroup
//     dispatch"), so consecutive virtual tiles -- the N tiles of one pixel tile, then its spatial
//     neighbours -- are dealt to the same XCD and share its L2.
//   * GLDS variant: both operands go global -> LDS by LDS-DMA (global_load_lds_dwordx4, no staging
//     registers, no ds_write pass).  A DMA wave-instruction writes 1 KiB lane-linearly (8 rows x
//     128 B), so rows are unpadded and the bank spread comes from an XOR swizzle applied on BOTH
//     sides (cdna_hip_programming.md §5.4 rule 21): 16-byte chunk c of row r is stored in slot
//     c ^ (r & 7).  Lane l of a DMA instruction therefore fetches chunk (l & 7) ^ (l >> 3) of row
//     l >> 3 -- a per-lane constant, so the incremental im2col state is unchanged -- and a fragment
//     read of chunk c, row r uses slot c ^ (r & 7): each ds_read_b128 lane group of 16 lanes then
//     covers 16 distinct slots of the 256-byte bank row (conflict-free).  Out-of-image / K-tail
//     chunks are fetched from a zeroed device page.
constexpr int BK2 = 64;
__device__ __attribute__((aligned(16))) unsigned int g_zero_page[8];  // 32 zero bytes (conv3t reads two 16-byte words)

// Phase clocks of conv2_kernel (diagnostic build only, -DVA_CONV2_STAMPS, tools/conv2_phases.py): per workgroup the
// shader clock at its start, after the first stage landed, after the K-loop, after the split-K slab and arrival,
// after the combine, at its end, and the 100 MHz real-time clock at start / end; lane 0's vector store.
#ifdef VA_CONV2_STAMPS
constexpr int C2S_BLOCKS = 4096, C2S_PTS = 8;
__device__ unsigned long long g_c2s[C2S_BLOCKS][C2S_PTS];
#define C2S(pt, v)                                                                          \
    do {                                                                                   \
        if (threadIdx.x == 0 && blockIdx.x < C2S_BLOCKS) g_c2s[blockIdx.x][pt] = (v);      \
    } while (0)
#else
#define C2S(pt, v)
#endif
// store sink: masked-out lanes of an epilogue whose store count must stay fixed (counted vmcnt) write here
__device__ __attribute__((aligned(16))) unsigned int g_sink[64 * 4];
typedef __attribute__((ext_vector_type(8))) int i32x8;
typedef __attribute__((address_space(1))) void gvoid_t;
typedef __attribute__((address_space(3))) void lvoid_t;

// T = element type: __bf16 (K-step 64, v_mfma_f32_16x16x32_bf16), float (exact-f32 parity mode: K-step 32,
// four v_mfma_f32_16x16x4_f32 per 16-byte chunk) or uint8_t = e4m3 bytes (the fp8 mode, va355.h
// VA_DTYPE_FP8 with x8: K-step 128, one block-scaled v_mfma_scale_f32_16x16x128_f8f6f4 per fragment pair).  A staged row is 128 bytes = 8 chunks of 16 bytes either way,
// so the LDS layout, the swizzle, the DMA pattern and the im2col bookkeeping are shared.
template <typename T, int WM, int WN, int TNS, bool GLDS = false>
struct Conv2Cfg {
    static constexpr int VEC = 16 / (int)sizeof(T);  // elements per 16-byte chunk
    static constexpr int KS = 8 * VEC;                 // K per stage: 64 bf16 / 32 f32
    static constexpr int NT = 64 * WM * WN, BM = 64 * WM, BN = 16 * TNS * WN, CPR = 8;
    static constexpr int A_CH = BN * CPR / NT, B_CH = BM * CPR / NT, RSTEP = NT / CPR;
    static constexpr int RS = GLDS ? KS : KS + VEC;                  // LDS row stride (elements): 128 / 144 B
    static constexpr int STAGE = (BN + BM) * RS * (int)sizeof(T);  // bytes per stage (A then B)
    static constexpr int CW = BN + 4;                    // epilogue f32 row (floats)
    static constexpr int EPI = BM * CW * 4;
    static constexpr int LDS = (2 * STAGE > EPI ? 2 * STAGE : EPI);
    static_assert(A_CH >= 1 && B_CH >= 1 && (BN * CPR) % NT == 0, "tile/block mismatch");
};

// Output pixel row (NHWC) of GEMM row m: mode 0 -> m; mode 2 (sub-pixel class cls = 2 dy + dx of a
// [N][2Ho][2Wo] map) -> pixel (2 ho + dy, 2 wo + dx).
__device__ __forceinline__ int64_t conv_out_row(const va_conv_args& a, int m, int cls) {
    if (a.mode != 2) return m;
    const int wo = m % a.Wo, t = m / a.Wo, ho = t % a.Ho, n = t / a.Ho;
    return ((int64_t)n * 2 * a.Ho + 2 * ho + (cls >> 1)) * 2 * a.Wo + 2 * wo + (cls & 1);
}

// Fused 1x1 tail (va_conv_args.w2): the 128 x 128 tile of main-conv activations, rounded to bf16
// exactly as the unfused layer would have stored them, goes to LDS as the B operand of a second
// GEMM against the tail's weights (c2 <= 80 rows, read from L2); the tail result is the only write.
constexpr int TAIL_C2F = 5;  // 16-row tail fragments: c2 <= 80

// orow(pl): output row (pixel index of the output tensor) of tile row pl, or -1 when masked
// bias4 (mode 2): the bias row of GEMM row m0 + pl comes from the border table (va355.h va_conv_args.bias4)
template <int NT, int BM, int TNS, typename OutT, typename RowFn>
__device__ __forceinline__ void conv2_tail(const va_conv_args& a, f32x4 (&acc)[TNS][4], unsigned char* smem, int n0,
                                           int wm, int wn, int wid, int fr, int fq, RowFn orow, int m0 = 0,
                                           int cls = 0) {
    constexpr int BN = 128, TW = BN + 8, PS = BM / (NT / 64) / 16;
    __bf16* Ts = (__bf16*)smem;
    int brow[4];  // bias row offset per pixel fragment
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        brow[j] = n0;
        if (a.bias4) {
            const int m = m0 + wm * 64 + 16 * j + fr;
            const int wo = m % a.Wo, ho = (m / a.Wo) % a.Ho;
            const int rf = (cls >> 1) ? ho == a.Ho - 1 : ho == 0, cf = (cls & 1) ? wo == a.Wo - 1 : wo == 0;
            brow[j] = ((cls * 2 + rf) * 2 + cf) * a.Npad + n0;
        }
    }
#pragma unroll
    for (int i = 0; i < TNS; ++i) {
        const int col = wn * 16 * TNS + 16 * i + 4 * fq;
        // w8: the e4m3 weights' per-output-channel scale (class cls's row of the mode-2 table)
        const float4 sv = a.w8 ? *(const float4*)(a.wscale + cls * a.Npad + n0 + col) : make_float4(1.f, 1.f, 1.f, 1.f);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float4 bv = *(const float4*)(a.bias + brow[j] + col);
            float v[4] = {acc[i][j][0] * sv.x + bv.x, acc[i][j][1] * sv.y + bv.y, acc[i][j][2] * sv.z + bv.z,
                          acc[i][j][3] * sv.w + bv.w};
            __bf16 o4[4];
            if (a.act) silu_n(v);
#pragma unroll
            for (int r = 0; r < 4; ++r) o4[r] = (__bf16)v[r];
            *(uint2*)(Ts + (wm * 64 + 16 * j + fr) * TW + col) = *(uint2*)o4;
        }
    }
    __syncthreads();
    const int nc2 = (a.c2 + 15) / 16;
    const __bf16* W2 = (const __bf16*)a.w2;
    f32x4 acc2[TAIL_C2F][PS];
#pragma unroll
    for (int c = 0; c < TAIL_C2F; ++c)
#pragma unroll
        for (int p = 0; p < PS; ++p) acc2[c][p] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kf = 0; kf < BN / 32; ++kf) {
        bf16x8 bfr[PS];
#pragma unroll
        for (int p = 0; p < PS; ++p) bfr[p] = *(const bf16x8*)(Ts + (wid * PS * 16 + 16 * p + fr) * TW + 32 * kf + 8 * fq);
#pragma unroll
        for (int c = 0; c < TAIL_C2F; ++c) {
            if (c < nc2) {
                const bf16x8 af = *(const bf16x8*)(W2 + (16 * c + fr) * BN + 32 * kf + 8 * fq);
#pragma unroll
                for (int p = 0; p < PS; ++p)
                    acc2[c][p] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfr[p], acc2[c][p], 0, 0, 0);
            }
        }
    }
    OutT* Y = (OutT*)a.y;
#pragma unroll
    for (int p = 0; p < PS; ++p) {
        const int64_t orw = orow(wid * PS * 16 + 16 * p + fr);
        if (orw < 0) continue;
#pragma unroll
        for (int c = 0; c < TAIL_C2F; ++c) {
            const int co = 16 * c + 4 * fq;
            if (c >= nc2 || co >= a.c2) continue;
            const float4 bv = *(const float4*)(a.b2 + co);
            float v[4] = {acc2[c][p][0] + bv.x, acc2[c][p][1] + bv.y, acc2[c][p][2] + bv.z, acc2[c][p][3] + bv.w};
            if (a.act2) {
                silu_n(v);
            }
            OutT* yp = Y + orw * a.ldy + co;
            if constexpr (sizeof(OutT) == 2) {
                __bf16 o4[4] = {(__bf16)v[0], (__bf16)v[1], (__bf16)v[2], (__bf16)v[3]};
                *(uint2*)yp = *(uint2*)o4;
            } else {
                *(float4*)yp = make_float4(v[0], v[1], v[2], v[3]);
            }
        }
    }
}

// Shared epilogue of the LDS-staged kernels: bias (+SiLU) -> f32 tile in LDS (the stage buffers are free
// after the last barrier), then 16-byte runs of consecutive channels per pixel (+ residual), row-contiguous
// stores.  Needs BM * (BN + 4) * 4 bytes of LDS.
// orow(pl): output row of tile row pl (mode 1: the linear GEMM row, scattered below), or -1 when masked
// RT: element type of the residual (the activations'); bias4 (mode 2): per-row bias from the border table
// e4m3 (RT / OutT = uint8_t, the fp8 mode): the accumulator is dequantized by wscale before the bias, the residual
// holds r * rscale, the output is stored as sat(y * yscale) (va355.h va_conv_args, VA_DTYPE_FP8)
__device__ __forceinline__ uint2 e4m3_pack8(const float* v, float ys) {
    float c[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) c[e] = fminf(fmaxf(v[e] * ys, -448.0f), 448.0f);
    int lo = __builtin_amdgcn_cvt_pk_fp8_f32(c[0], c[1], 0, false);
    lo = __builtin_amdgcn_cvt_pk_fp8_f32(c[2], c[3], lo, true);
    int hi = __builtin_amdgcn_cvt_pk_fp8_f32(c[4], c[5], 0, false);
    hi = __builtin_amdgcn_cvt_pk_fp8_f32(c[6], c[7], hi, true);
    return make_uint2((unsigned)lo, (unsigned)hi);
}
__device__ __forceinline__ void e4m3_unpack4(unsigned q, float inv, float* v) {
    const f32x2 a = __builtin_amdgcn_cvt_pk_f32_fp8((int)q, false), b = __builtin_amdgcn_cvt_pk_f32_fp8((int)q, true);
    v[0] = a[0] * inv, v[1] = a[1] * inv, v[2] = b[0] * inv, v[3] = b[1] * inv;
}

// epilogue stage 2 (Cs -> global): 16-byte runs of consecutive channels per pixel (+ residual), row-contiguous stores
template <int NT, int BM, int BN, typename OutT, typename RowFn, typename RT>
__device__ __forceinline__ void conv_epilogue_store(const va_conv_args& a, unsigned char* smem, int n0, int tid,
                                                    RowFn orow) {
    constexpr bool F8 = sizeof(RT) == 1;
    constexpr int CW = BN + 4;
    const float* Cs = (const float*)smem;
    constexpr int OV = 16 / sizeof(OutT);
    constexpr int CPRO = BN / OV;
    OutT* Y = (OutT*)a.y;
    const RT* R = (const RT*)a.res;
    constexpr int RV = 16 / (int)sizeof(RT);
    for (int c = tid; c < BM * CPRO; c += NT) {
        const int pl = c / CPRO, cl = (c % CPRO) * OV;
        const int co = n0 + cl;
        const int64_t orw = orow(pl);
        if (orw < 0 || co >= a.Cout) continue;
        float v[OV];
#pragma unroll
        for (int r = 0; r < OV; r += 4) {
            const float4 t = *(const float4*)(Cs + pl * CW + cl + r);
            v[r] = t.x;
            v[r + 1] = t.y;
            v[r + 2] = t.z;
            v[r + 3] = t.w;
        }
        if (R) {
            if constexpr (F8) {  // e4m3 residual: OV (16) bytes
                const float rinv = 1.0f / a.rscale;
                const u32x4 rr = *(const u32x4*)(R + orw * a.ldr + co);
#pragma unroll
                for (int w = 0; w < 4 && 4 * w < OV; ++w) {
                    float rv[4];
                    e4m3_unpack4(rr[w], rinv, rv);
#pragma unroll
                    for (int e = 0; e < 4; ++e) v[4 * w + e] += rv[e];
                }
            } else {
#pragma unroll
                for (int r = 0; r < OV; r += RV) {
                    const u32x4 rr = *(const u32x4*)(R + orw * a.ldr + co + r);
                    const RT* rp = (const RT*)&rr;
#pragma unroll
                    for (int e = 0; e < RV && r + e < OV; ++e) v[r + e] += (float)rp[e];
                }
            }
        }
        OutT* yp;
        if (a.mode == 1) {
            const int m = (int)orw;
            const int wo = m % a.Wo, t = m / a.Wo, ho = t % a.Ho, n = t / a.Ho;
            const int cd = a.Cout / 4, q = co / cd, cc = co - q * cd;
            yp = Y + (((int64_t)n * 2 * a.Ho + 2 * ho + (q >> 1)) * 2 * a.Wo + 2 * wo + (q & 1)) * a.ldy + cc;
        } else {
            yp = Y + orw * a.ldy + co;
        }
        if constexpr (sizeof(OutT) == 1) {  // 16 e4m3 bytes
            const uint2 lo = e4m3_pack8(v, a.yscale), hi = e4m3_pack8(v + 8, a.yscale);
            *(u32x4*)yp = (u32x4){lo.x, lo.y, hi.x, hi.y};
        } else if constexpr (sizeof(OutT) == 2) {
            bf16x8 o;
#pragma unroll
            for (int e = 0; e < 8; ++e) o[e] = (__bf16)v[e];
            *(bf16x8*)yp = o;
        } else {
            *(float4*)yp = make_float4(v[0], v[1], v[2], v[3]);
        }
    }
}

template <int NT, int BM, int BN, int TNS, typename OutT, typename RowFn, typename RT = __bf16>
__device__ __forceinline__ void conv_epilogue(const va_conv_args& a, f32x4 (&acc)[TNS][4], unsigned char* smem, int n0,
                                              int wm, int wn, int tid, int fr, int fq, RowFn orow, int m0 = 0,
                                              int cls = 0) {
    constexpr bool F8 = sizeof(RT) == 1;  // the fp8 mode (e4m3 activations)
    constexpr int CW = BN + 4;
    float* Cs = (float*)smem;
    int brow[4];  // bias row offset per pixel fragment
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        brow[j] = n0;
        if (a.bias4) {
            const int m = m0 + wm * 64 + 16 * j + fr;
            const int wo = m % a.Wo, ho = (m / a.Wo) % a.Ho;
            const int rf = (cls >> 1) ? ho == a.Ho - 1 : ho == 0, cf = (cls & 1) ? wo == a.Wo - 1 : wo == 0;
            brow[j] = ((cls * 2 + rf) * 2 + cf) * a.Npad + n0;
        }
    }
    // bias (and fp8 weight scales) loaded up front: under the a.act branch below each load would otherwise be
    // waited for on its own (vmcnt(0) per fragment)
    float4 bvs[TNS][4], svs[TNS];
    // e4m3 weights in a bf16 conv (w8): the accumulator times the weights' scale of its output channel (class cls's
    // row of the mode-2 table), as the fp8 mode's wscale
    const bool scaled = F8 || (sizeof(RT) == 2 && a.w8);
#pragma unroll
    for (int i = 0; i < TNS; ++i) {
        const int col = wn * 16 * TNS + 16 * i + 4 * fq;
        if (scaled) svs[i] = *(const float4*)(a.wscale + (F8 ? 0 : cls * a.Npad) + n0 + col);
#pragma unroll
        for (int j = 0; j < 4; ++j) bvs[i][j] = *(const float4*)(a.bias + brow[j] + col);  // bias is padded to Npad
    }
#pragma unroll
    for (int i = 0; i < TNS; ++i) {
        const int col = wn * 16 * TNS + 16 * i + 4 * fq;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float4 bv = bvs[i][j];
            f32x4 ac = acc[i][j];
            if (scaled) {
                const float4 sv = svs[i];
                ac = ac * (f32x4){sv.x, sv.y, sv.z, sv.w};
            }
            float v0 = ac[0] + bv.x, v1 = ac[1] + bv.y, v2 = ac[2] + bv.z, v3 = ac[3] + bv.w;
            if (a.act) {
                const f32x2 s01 = fz::silu2((f32x2){v0, v1}), s23 = fz::silu2((f32x2){v2, v3});
                v0 = s01[0];
                v1 = s01[1];
                v2 = s23[0];
                v3 = s23[1];
            }
            *(float4*)(Cs + (wm * 64 + 16 * j + fr) * CW + col) = make_float4(v0, v1, v2, v3);
        }
    }
    __syncthreads();
    conv_epilogue_store<NT, BM, BN, OutT, RowFn, RT>(a, smem, n0, tid, orow);
}

// epilogue stage 1 of the 32x32-fragment form (conv2_kernel SPL 16): acc[ib][jb] is the 32 x 32 block of channels
// wn 16 TNS + 32 ib .. and pixels wm 64 + 32 jb ..; lane l holds pixel l % 32, items q: channel 8 (q / 4) + 4 (l / 32)
// + q % 4 (v_mfma_f32_32x32x16 D layout)
// pcol(c): tile row (pixel) of accumulator column c (0..31) of a 32 x 32 block (the B operand's row order);
// mrow(pl): GEMM row m of tile pixel pl (bias4's border table), or -1 when masked
template <int BN, int TNS, typename MFn, typename PFn>
__device__ __forceinline__ void conv_epilogue32_fill(const va_conv_args& a, f32x16 (&acc)[TNS / 2][2],
                                                     unsigned char* smem, int n0, int wm, int wn, int lane, MFn mrow,
                                                     PFn pcol, int cls) {
    constexpr int CW = BN + 4;
    float* Cs = (float*)smem;
    const int r = lane & 31, g = lane >> 5;
    float4 bvs[2][TNS / 2][4];  // loaded up front (see conv_epilogue)
#pragma unroll
    for (int jb = 0; jb < 2; ++jb) {
        const int pl = wm * 64 + 32 * jb + pcol(r);
        int brow = n0;
        if (a.bias4) {
            const int m = max(mrow(pl), 0);
            const int wo = m % a.Wo, ho = (m / a.Wo) % a.Ho;
            const int rf = (cls >> 1) ? ho == a.Ho - 1 : ho == 0, cf = (cls & 1) ? wo == a.Wo - 1 : wo == 0;
            brow = ((cls * 2 + rf) * 2 + cf) * a.Npad + n0;
        }
#pragma unroll
        for (int ib = 0; ib < TNS / 2; ++ib)
#pragma unroll
            for (int k = 0; k < 4; ++k)
                bvs[jb][ib][k] = *(const float4*)(a.bias + brow + wn * 16 * TNS + 32 * ib + 8 * k + 4 * g);
    }
#pragma unroll
    for (int jb = 0; jb < 2; ++jb) {
        const int pl = wm * 64 + 32 * jb + pcol(r);
#pragma unroll
        for (int ib = 0; ib < TNS / 2; ++ib) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int col = wn * 16 * TNS + 32 * ib + 8 * k + 4 * g;
                const float4 bv = bvs[jb][ib][k];
                float v0 = acc[ib][jb][4 * k] + bv.x, v1 = acc[ib][jb][4 * k + 1] + bv.y,
                      v2 = acc[ib][jb][4 * k + 2] + bv.z, v3 = acc[ib][jb][4 * k + 3] + bv.w;
                if (a.act) {
                    const f32x2 s01 = fz::silu2((f32x2){v0, v1}), s23 = fz::silu2((f32x2){v2, v3});
                    v0 = s01[0];
                    v1 = s01[1];
                    v2 = s23[0];
                    v3 = s23[1];
                }
                *(float4*)(Cs + pl * CW + col) = make_float4(v0, v1, v2, v3);
            }
        }
    }
}

template <int NT, int BM, int BN, int TNS, typename OutT, typename RowFn, typename MFn, typename PFn>
__device__ __forceinline__ void conv_epilogue32(const va_conv_args& a, f32x16 (&acc)[TNS / 2][2], unsigned char* smem,
                                                int n0, int wm, int wn, int tid, int lane, RowFn orow, MFn mrow,
                                                PFn pcol, int cls = 0) {
    conv_epilogue32_fill<BN, TNS>(a, acc, smem, n0, wm, wn, lane, mrow, pcol, cls);
    __syncthreads();
    conv_epilogue_store<NT, BM, BN, OutT, RowFn, float>(a, smem, n0, tid, orow);
}

// FK (LDS-DMA form, Cin % 64 == 0): a 64-deep K-step never straddles a tap, so (ky, kx, channel base) are
// wave-uniform scalars and each staged row keeps a precomputed base pointer: per K-step and row the B
// address is one 64-bit add of a scalar offset plus a bounds select (the general form re-derives the
// im2col coordinates of every lane with 64-bit multiplies).
// UP (FK, 1x1 only): input channels [0, a.cu) come from the half-resolution slice a.xu at (h/2, w/2) -- the
// FPN's Upsample + Concat read in place (va355.h va_conv_args.xu); a K-step is one 64-channel chunk, so
// the source is a wave-uniform choice per K-step.
// f32 as three bf16 terms: h = bf16(x), m = bf16(x - h), l = bf16(x - h - m) (round to nearest even, two elements
// per v_cvt_pk_bf16_f32), x = h + m + l EXACTLY: x - h is a multiple of x's ulp below half of h's bf16 ulp (<= 16
// significant bits, an exact f32 subtraction), likewise (x - h) - m (<= 8 bits, so l is exact in bf16).  Elements
// 0-3 come from c0, 4-7 from c1 -- the same order for both MFMA operands, so the K pairing is kept.
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
__device__ __forceinline__ unsigned cvt_pk_bf16(f32x2 v) {
    return __builtin_bit_cast(unsigned, __builtin_convertvector(v, bf16x2));
}
__device__ __forceinline__ f32x2 unpk_bf16(unsigned p) {
    return (f32x2){__uint_as_float(p << 16), __uint_as_float(p & 0xffff0000u)};
}
__device__ __forceinline__ void split3_bf16(const u32x4& c0, const u32x4& c1, bf16x8 (&t)[3]) {
    unsigned w[3][4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const u32x4& c = e < 2 ? c0 : c1;
        const f32x2 x = {__uint_as_float(c[2 * (e & 1)]), __uint_as_float(c[2 * (e & 1) + 1])};
        w[0][e] = cvt_pk_bf16(x);
        const f32x2 r = x - unpk_bf16(w[0][e]);
        w[1][e] = cvt_pk_bf16(r);
        w[2][e] = cvt_pk_bf16(r - unpk_bf16(w[1][e]));
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) t[k] = __builtin_bit_cast(bf16x8, (u32x4){w[k][0], w[k][1], w[k][2], w[k][3]});
}
// four f32 -> three bf16 planes of 4 values each (split3_bf16's terms)
__device__ __forceinline__ void split3_bf16x4(const f32x4& v, uint2 (&t)[3]) {
#pragma unroll
    for (int e = 0; e < 2; ++e) {
        const f32x2 x = {v[2 * e], v[2 * e + 1]};
        const unsigned h = cvt_pk_bf16(x);
        const f32x2 r = x - unpk_bf16(h);
        const unsigned m = cvt_pk_bf16(r);
        const unsigned l = cvt_pk_bf16(r - unpk_bf16(m));
        (e ? t[0].y : t[0].x) = h;
        (e ? t[1].y : t[1].x) = m;
        (e ? t[2].y : t[2].x) = l;
    }
}

// SPL (T = float only): 0 = exact f32 MFMA (v_mfma_f32_16x16x4_f32, 32 cycles per SIMD); 6 or 9 = the f32
// operands split into three exact bf16 terms (split3_bf16) and multiplied on v_mfma_f32_16x16x32_bf16 (16 cycles
// per SIMD, 8x the K per instruction): the term products h.h, h.m, m.h, h.l, m.m, l.h (+ m.l, l.m, l.l for 9) are
// exact in f32 and accumulated in f32; the three left out at 6 are <= 2^-23 of |a b| together, below one f32
// rounding of the sum.  (The same six products on v_mfma_f32_32x32x16_bf16 measured 2-10 % slower on every layer
// of the s-seg forward, profiles/r03/ab_split_6_16.log.)
// 16-byte write-through (sc1) store of a split-K slab (conv2_kernel's combine): base / bytes = the workspace.  A
// plain __device__ function: the host pass of a kernel template whose body names a buffer builtin can drop the
// kernel's stub (see t3_dma16)
__device__ __forceinline__ void sk_store16(void* base, int64_t bytes, int off, f32x4 v) {
    const __amdgpu_buffer_rsrc_t r =
        __builtin_amdgcn_make_buffer_rsrc(base, 0, (int)(bytes < 0x7fffffff ? bytes : 0x7fffffff), 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, off, 0, 16);
}

// 16-byte buffer_load ... lds of w3 (base, bytes: the descriptor's range; out-of-range offsets load zeros).  A
// plain __device__ function: the host pass of a kernel template whose body names the LDS-DMA buffer builtin drops
// the kernel's stub without a diagnostic (an undefined symbol at load time).
__device__ __forceinline__ void t3_dma16(const void* base, int bytes, void* lds, int voff, int soff) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, bytes, 0x00020000);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lvoid_t*)lds, 16, voff, soff, 0, 0);
}
// f32 fused 1x1 tail (va_conv_args.w2 in f32 mode): the tile's main-conv activations -- every output channel of the
// conv (Cout <= BN), bias + SiLU applied, f32 in Cs [BM][BN + 4] -- contracted with the tail's weights as exact
// three-term products: W2 pre-split on the host ([32 nb][Cout / 8][3][8] bf16, h / m / l per 8-channel group, the
// w3 layout), each activation split here (split3_bf16), the six term products of 32 x 32 x 16 blocks accumulated in
// f32 -- the arithmetic of the unfused 1x1 layer, in another order.  Wave w takes pixels 32 w .. 32 w + 31 and all
// nb = ceil(c2 / 32) blocks of tail channels (c2 <= 96); + b2, SiLU if act2; then through LDS (the activations'
// space, once every wave has read it) to 16-byte runs of consecutive float channels per pixel at a.y / a.ldy.
constexpr int T3_TAIL_C2 = 96;
template <int NT, int BM, int BN, typename RowFn>
__device__ __forceinline__ void conv_tail32(const va_conv_args& a, unsigned char* smem, int tid, int lane,
                                            RowFn orow) {
    static_assert(BM == 32 * (NT / 64), "one 32-pixel block per wave");
    constexpr int CW = BN + 4, CW2 = T3_TAIL_C2 + 4;
    float* Cs = (float*)smem;
    const int w = tid >> 6, r = lane & 31, g = lane >> 5;
    const int K = a.Cout, nb = (a.c2 + 31) >> 5;
    const __bf16* __restrict__ W2 = (const __bf16*)a.w2;
    constexpr int TA[6] = {0, 0, 1, 0, 1, 2}, TB[6] = {0, 1, 0, 2, 1, 0};
    f32x16 acc[3];
#pragma unroll
    for (int ib = 0; ib < 3; ++ib) acc[ib] = (f32x16){};
    for (int k0 = 0; k0 < K; k0 += 16) {
        const float* p = Cs + (32 * w + r) * CW + k0 + 8 * g;
        bf16x8 bt[3];
        split3_bf16(*(const u32x4*)p, *(const u32x4*)(p + 4), bt);
#pragma unroll
        for (int ib = 0; ib < 3; ++ib) {
            if (ib < nb) {  // wave-uniform
                const bf16x8* wp = (const bf16x8*)(W2 + ((int64_t)(32 * ib + r) * (K / 8) + k0 / 8 + g) * 24);
                const bf16x8 at[3] = {wp[0], wp[1], wp[2]};
#pragma unroll
                for (int t = 0; t < 6; ++t)
                    acc[ib] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(at[TA[t]], bt[TB[t]], acc[ib], 0, 0, 0);
            }
        }
    }
    __syncthreads();  // every wave's activation reads are done: the tail's outputs reuse the space
#pragma unroll
    for (int ib = 0; ib < 3; ++ib) {
        if (ib < nb) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int col = 32 * ib + 8 * k + 4 * g;  // v_mfma_f32_32x32x16 D layout: lane (r, g) = pixel r
                const float4 bv = *(const float4*)(a.b2 + col);  // b2 is padded to the tail's Npad
                float v0 = acc[ib][4 * k] + bv.x, v1 = acc[ib][4 * k + 1] + bv.y, v2 = acc[ib][4 * k + 2] + bv.z,
                      v3 = acc[ib][4 * k + 3] + bv.w;
                if (a.act2) {
                    const f32x2 s01 = fz::silu2((f32x2){v0, v1}), s23 = fz::silu2((f32x2){v2, v3});
                    v0 = s01[0];
                    v1 = s01[1];
                    v2 = s23[0];
                    v3 = s23[1];
                }
                *(float4*)(Cs + (32 * w + r) * CW2 + col) = make_float4(v0, v1, v2, v3);
            }
        }
    }
    __syncthreads();
    const int c4 = a.c2 / 4;
    float* Y = (float*)a.y;
    for (int c = tid; c < BM * c4; c += NT) {
        const int pl = c / c4, cl = (c - pl * c4) * 4;
        const int64_t orw = orow(pl);
        if (orw >= 0) *(float4*)(Y + orw * a.ldy + cl) = *(const float4*)(Cs + pl * CW2 + cl);
    }
}

// W8 (T = bf16 only; va_conv_args.w8): the weights are e4m3 bytes [Npad][Kpad] -- 8 bytes per 8-element chunk.  In
// the GLDS forms the A stage holds them as they are: 64-byte rows (a K-step), DMA'd 16 rows per wave instruction (lane
// l: row l >> 2, 16-byte slot l & 3 holding chunk pair (l & 3) ^ ((row >> 2) & 3) -- conflict-free ds_read_b64 of the
// fragments), and each A fragment is converted exactly to bf16 as it is read (e4m3x8_bf16: four
// v_cvt_scalef32_pk_bf16_fp8 per fragment, issued beside the MFMAs).  A form that staged the bytes through registers
// and wrote converted bf16 rows into the stage (the DMA's place) cost 8-16 % per layer: its 64-bit address math, loads,
// conversions and LDS writes sat on every K-step.  The register form (CONV2_LOAD / STORE) converts at the store.  The
// epilogue multiplies by the per-output-channel scale (va_conv_args.wscale)
template <typename T, int WM, int WN, int TNS, typename OutT, bool GLDS = false, bool FK = false, bool UP = false,
          int SPL = 0, bool W8 = false>
__global__ __launch_bounds__(64 * WM* WN) void conv2_kernel(va_conv_args a, int ntn, int ntiles, int ksplit,
                                                           int kper) {
    static_assert(!W8 || sizeof(T) == 2, "e4m3 weights in the bf16 kernel only");
    using Cfg = Conv2Cfg<T, WM, WN, TNS, GLDS>;
    constexpr int NT = Cfg::NT, BM = Cfg::BM, BN = Cfg::BN, CPR = Cfg::CPR;
    constexpr int A_CH = Cfg::A_CH, B_CH = Cfg::B_CH, RSTEP = Cfg::RSTEP, RS = Cfg::RS;
    constexpr int VEC = Cfg::VEC, KS = Cfg::KS;
    __shared__ __align__(16) unsigned char smem[Cfg::LDS];
    auto As = [&](int s) { return (T*)(smem + s * Cfg::STAGE); };
    auto Bs = [&](int s) { return (T*)(smem + s * Cfg::STAGE + BN * RS * (int)sizeof(T)); };

    C2S(0, __builtin_amdgcn_s_memtime());
    C2S(6, __builtin_amdgcn_s_memrealtime());
    // ksplit < 0: split K in the reduce form -- the -ksplit slices only store their slabs, conv2_reduce_kernel sums
    // them and runs the epilogue
    const bool kred = ksplit < 0;
    if (kred) ksplit = -ksplit;
    int bid = blockIdx.x;
    {
        const int nx = 8, q = ntiles / nx, r = ntiles % nx, xcd = bid % nx, j = bid / nx;
        bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + j;
    }
    // split K (ksplit > 1): the ksplit slices of one tile are consecutive virtual blocks (one XCD: the reducer
    // reads its partners' slabs from its own L2); slice sk runs K-steps [sk kper, min(nk, (sk + 1) kper))
    const int sk = bid % ksplit;
    bid /= ksplit;
    const int vt = bid;  // virtual tile (with the sub-pixel class): the arrival counter's index
    // mode 2: the 4 sub-pixel classes of one tile are consecutive virtual tiles (same input, same XCD)
    const int cls = a.mode == 2 ? (bid & 3) : 0;
    if (a.mode == 2) bid >>= 2;
    const int tm = bid / ntn, tn = bid % ntn;
    const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wid / WN, wn = wid % WN;
    const int m0 = tm * BM, n0 = tn * BN;
    const int nk_all = a.Kpad / KS;
    const int kt0 = sk * kper, kt1 = min(nk_all, kt0 + kper);
    const T* __restrict__ X = (const T*)a.x;
    const T* __restrict__ Wt = (const T*)a.w + (int64_t)cls * a.Npad * a.Kpad;
    const uint8_t* __restrict__ W8p = (const uint8_t*)a.w + (int64_t)cls * a.Npad * a.Kpad;  // W8: byte rows
    const int pad_y = a.mode == 2 ? 1 - (cls >> 1) : a.pad, pad_x = a.mode == 2 ? 1 - (cls & 1) : a.pad;
    // fixed 8-element k group of this thread and its first staged row (rows row0 + RSTEP * i); with
    // LDS-DMA, instruction i of wave w covers rows 8 (i NT/64 + w) .. +7, lane l row l >> 3
    const int g = GLDS ? ((lane & 7) ^ (lane >> 3)) : tid % CPR;
    const int row0 = GLDS ? 8 * wid + (lane >> 3) : tid / CPR;

    int b_hi[B_CH], b_wi[B_CH];
    int64_t b_base[B_CH];
    const T* rowu[UP ? B_CH : 1];  // UP: the pixel's row in the half-resolution source (+ lane's chunk)
#pragma unroll
    for (int i = 0; i < B_CH; ++i) {
        const int m = m0 + row0 + RSTEP * i;
        if constexpr (UP) rowu[i] = (const T*)a.xu + VEC * g;
        if (m < a.M) {
            const int wo = m % a.Wo, t = m / a.Wo, ho = t % a.Ho, n = t / a.Ho;
            b_hi[i] = ho * a.stride - pad_y;
            b_wi[i] = wo * a.stride - pad_x;
            b_base[i] = (int64_t)n * a.H * a.W;
            if constexpr (UP)
                rowu[i] = (const T*)a.xu + (((int64_t)n * (a.H / 2) + (ho >> 1)) * (a.W / 2) + (wo >> 1)) * a.ldu + VEC * g;
        } else {
            b_hi[i] = -(1 << 28);
            b_wi[i] = 0;
            b_base[i] = 0;
        }
    }
    // im2col position (tap ky, kx; channel ci) of this thread's 8-element group of K-step kt0
    int kcur = kt0 * KS + VEC * g, ci, ky, kx;
    {
        const int tap = kcur / a.Cin;
        ci = kcur - tap * a.Cin;
        ky = tap / a.kw;
        kx = tap - ky * a.kw;
    }
    // FK state: per-row base pointers (pixel at tap (0, 0), this lane's 8-channel group) and weight rows
    const T* rowp[B_CH];
    const T* wrow[A_CH];
    int fk_ky, fk_kx, fk_c;  // tap and 64-channel chunk of the next K-step (wave-uniform)
    {
        const int tap = kt0 * KS / a.Cin;
        fk_c = kt0 * KS - tap * a.Cin;
        fk_ky = tap / a.kw;
        fk_kx = tap - fk_ky * a.kw;
    }
    const void* zpage = (const void*)g_zero_page;  // hoisted: the asm waits' memory clobbers force a reload
    if constexpr (FK) {
#pragma unroll
        for (int i = 0; i < B_CH; ++i) rowp[i] = X + (b_base[i] + (int64_t)b_hi[i] * a.W + b_wi[i]) * a.ldx + VEC * g;
#pragma unroll
        for (int i = 0; i < A_CH; ++i) wrow[i] = Wt + (int64_t)(n0 + row0 + RSTEP * i) * a.Kpad + VEC * g;
    }

    // no lambdas around the staging arrays: captured by reference they become addressable allocas
    u32x4 ra[A_CH], rb[B_CH];
    uint2 ra8[W8 ? A_CH : 1];  // W8, register form: the e4m3 bytes of this thread's A chunks
#define CONV2_LOAD(k0)                                                                                             \
    {                                                                                                              \
        _Pragma("unroll") for (int i = 0; i < A_CH; ++i) {                                                         \
            if constexpr (W8)                                                                                      \
                ra8[i] = *(const uint2*)(W8p + (int64_t)(n0 + row0 + RSTEP * i) * a.Kpad + (k0) + 8 * w8_pos(g));  \
            else                                                                                                   \
                ra[i] = *(const u32x4*)(Wt + (int64_t)(n0 + row0 + RSTEP * i) * a.Kpad + (k0) + VEC * g);           \
        }                                                                                                          \
        const bool kin = kcur < a.K;                                                                               \
        _Pragma("unroll") for (int i = 0; i < B_CH; ++i) {                                                         \
            const int hi = b_hi[i] + ky, wi = b_wi[i] + kx;                                                        \
            const bool ok = kin && (unsigned)hi < (unsigned)a.H && (unsigned)wi < (unsigned)a.W;                   \
            const int64_t off = ok ? (b_base[i] + (int64_t)hi * a.W + wi) * a.ldx + ci : 0;                       \
            const u32x4 v = *(const u32x4*)(X + off);                                                              \
            rb[i] = ok ? v : (u32x4){0u, 0u, 0u, 0u};                                                              \
        }                                                                                                          \
        kcur += KS;                                                                                               \
        ci += KS;                                                                                                 \
        while (ci >= a.Cin) {                                                                                      \
            ci -= a.Cin;                                                                                           \
            if (++kx == a.kw) {                                                                                    \
                kx = 0;                                                                                            \
                ++ky;                                                                                              \
            }                                                                                                      \
        }                                                                                                          \
    }
#define CONV2_STORE(s)                                                                                             \
    {                                                                                                              \
        T* as_ = As(s);                                                                                       \
        T* bs_ = Bs(s);                                                                                       \
        _Pragma("unroll") for (int i = 0; i < A_CH; ++i) {                                                         \
            if constexpr (W8)                                                                                      \
                *(u32x4*)(as_ + (row0 + RSTEP * i) * RS + VEC * g) = e4m3x8_bf16(ra8[i]);                          \
            else                                                                                                   \
                *(u32x4*)(as_ + (row0 + RSTEP * i) * RS + VEC * g) = ra[i];                                        \
        }                                                                                                          \
        _Pragma("unroll") for (int i = 0; i < B_CH; ++i)* (u32x4*)(bs_ + (row0 + RSTEP * i) * RS + VEC * g) =   \
            rb[i];                                                                                                 \
    }

    // W8 (GLDS): the e4m3 A rows of K-step k0 into stage base AS_ -- BN / 16 wave instructions of 16 rows x 64 bytes,
    // dealt to the waves; lane l fetches 16-byte piece (l & 3) ^ ((row >> 2) & 3) of row l >> 2 -- with the rows'
    // chunk order (w8_pos) piece q holds the K chunks q and q + 4, the two halves of lane group q's fragment, so a
    // fragment is one conflict-free ds_read_b128 (two ds_read_b64 were merged into a read2 that the compiler's wait
    // pass answered with a vmcnt(0) ahead of every step's first MFMA: the next stage's DMA waited out, 8-20 % per layer)
#define CONV2_DMA8(k0, AS_)                                                                                        \
    {                                                                                                              \
        _Pragma("unroll") for (int jj = 0; jj < (BN / 16 + NT / 64 - 1) / (NT / 64); ++jj) {                      \
            const int j8 = wid + (NT / 64) * jj;                                                                   \
            const int r8 = 16 * j8 + (lane >> 2), p8 = (lane & 3) ^ ((r8 >> 2) & 3);                               \
            if (BN / 16 % (NT / 64) == 0 || j8 < BN / 16)                                                          \
                t3_dma16(W8p, a.Npad * a.Kpad, (unsigned char*)(AS_) + 1024 * j8, (n0 + r8) * a.Kpad + 16 * p8,    \
                         (k0));                                                                                    \
        }                                                                                                          \
    }
    // LDS-DMA form of LOAD+STORE: one 1 KiB DMA per operand row block, zero page for masked chunks
#define CONV2_DMA(k0, s)                                                                                           \
    if constexpr (FK) {                                                                                            \
        T* as_ = As(s);                                                                                       \
        T* bs_ = Bs(s);                                                                                       \
        if constexpr (W8) {                                                                                        \
            CONV2_DMA8(k0, as_);                                                                                   \
        } else {                                                                                                   \
            _Pragma("unroll") for (int i = 0; i < A_CH; ++i) __builtin_amdgcn_global_load_lds(                     \
                (gvoid_t*)(wrow[i] + (k0)), (lvoid_t*)(as_ + (RSTEP * i + 8 * wid) * KS), 16, 0, 0);               \
        }                                                                                                          \
        const int soff = (fk_ky * a.W + fk_kx) * a.ldx + fk_c;                                                     \
        _Pragma("unroll") for (int i = 0; i < B_CH; ++i) {                                                         \
            const bool ok = (unsigned)(b_hi[i] + fk_ky) < (unsigned)a.H && (unsigned)(b_wi[i] + fk_kx) < (unsigned)a.W; \
            const T* sp_ = rowp[i] + soff;                                                                    \
            if constexpr (UP) sp_ = fk_c < a.cu ? rowu[i] + fk_c : sp_;                                           \
            const void* src = ok ? (const void*)sp_ : zpage;                                                       \
            __builtin_amdgcn_global_load_lds((gvoid_t*)src, (lvoid_t*)(bs_ + (RSTEP * i + 8 * wid) * KS), 16, 0,  \
                                             0);                                                                   \
        }                                                                                                          \
        fk_c += KS;                                                                                               \
        if (fk_c == a.Cin) {                                                                                       \
            fk_c = 0;                                                                                              \
            if (++fk_kx == a.kw) {                                                                                 \
                fk_kx = 0;                                                                                         \
                ++fk_ky;                                                                                           \
            }                                                                                                      \
        }                                                                                                          \
    } else {                                                                                                       \
        T* as_ = As(s);                                                                                       \
        T* bs_ = Bs(s);                                                                                       \
        if constexpr (W8) {                                                                                        \
            CONV2_DMA8(k0, as_);                                                                                   \
        } else {                                                                                                   \
            _Pragma("unroll") for (int i = 0; i < A_CH; ++i) {                                                     \
                const T* src = Wt + (int64_t)(n0 + row0 + RSTEP * i) * a.Kpad + (k0) + VEC * g;                      \
                __builtin_amdgcn_global_load_lds((gvoid_t*)src, (lvoid_t*)(as_ + (RSTEP * i + 8 * wid) * KS), 16,  \
                                                 0, 0);                                                            \
            }                                                                                                      \
        }                                                                                                          \
        const bool kin = kcur < a.K;                                                                               \
        _Pragma("unroll") for (int i = 0; i < B_CH; ++i) {                                                         \
            const int hi = b_hi[i] + ky, wi = b_wi[i] + kx;                                                        \
            const bool ok = kin && (unsigned)hi < (unsigned)a.H && (unsigned)wi < (unsigned)a.W;                   \
            const void* src = ok ? (const void*)(X + (b_base[i] + (int64_t)hi * a.W + wi) * a.ldx + ci)            \
                                 : (const void*)g_zero_page;                                                       \
            __builtin_amdgcn_global_load_lds((gvoid_t*)src, (lvoid_t*)(bs_ + (RSTEP * i + 8 * wid) * KS), 16, 0,  \
                                             0);                                                                   \
        }                                                                                                          \
        kcur += KS;                                                                                               \
        ci += KS;                                                                                                 \
        while (ci >= a.Cin) {                                                                                      \
            ci -= a.Cin;                                                                                           \
            if (++kx == a.kw) {                                                                                    \
                kx = 0;                                                                                            \
                ++ky;                                                                                              \
            }                                                                                                      \
        }                                                                                                          \
    }

    f32x4 acc[TNS][4];
#pragma unroll
    for (int i = 0; i < TNS; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

    if constexpr (GLDS) {
        CONV2_DMA(kt0 * KS, 0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
        CONV2_LOAD(kt0 * KS);
        CONV2_STORE(0);
    }
    __syncthreads();
    C2S(1, __builtin_amdgcn_s_memtime());
    const int fr = lane & 15, fq = lane >> 4;
    for (int kt = kt0; kt < kt1; ++kt) {
        const int s = (kt - kt0) & 1;
        const bool more = kt + 1 < kt1;
        if constexpr (GLDS) {
            if (more) {
                CONV2_DMA((kt + 1) * KS, s ^ 1);
            }
        } else {
            if (more) CONV2_LOAD((kt + 1) * KS);
        }
        const T* as_ = As(s);
        const T* bs_ = Bs(s);
        {
        // all fragments of the K-step first (the second half's reads overlap the first half's MFMAs)
        u32x4 af[2][TNS], bfr[2][4];
#pragma unroll
        for (int kh = 0; kh < 2; ++kh) {
            // chunk 4 kh + fq of the row; GLDS rows are swizzled (slot = chunk ^ (row & 7), row & 7 == fr & 7)
            const int ch = GLDS ? (((4 * kh + fq) ^ (fr & 7)) * VEC) : 4 * VEC * kh + VEC * fq;
#pragma unroll
            for (int i = 0; i < TNS; ++i) {
                if constexpr (GLDS && W8) {  // the e4m3 row's 8 bytes of this chunk, converted as read
                    const int r8 = wn * 16 * TNS + 16 * i + fr;
                    if (kh == 0) {  // both K halves of the fragment in one 16-byte read
                        const u32x4 q = *(const u32x4*)((const unsigned char*)as_ + r8 * 64 + 16 * (fq ^ ((r8 >> 2) & 3)));
                        af[0][i] = e4m3x8_bf16(make_uint2(q[0], q[1]));
                        af[1][i] = e4m3x8_bf16(make_uint2(q[2], q[3]));
                    }
                } else {
                    af[kh][i] = *(const u32x4*)(as_ + (wn * 16 * TNS + 16 * i + fr) * RS + ch);
                }
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) bfr[kh][j] = *(const u32x4*)(bs_ + (wm * 64 + 16 * j + fr) * RS + ch);
        }
        if constexpr (sizeof(T) == 2) {
#pragma unroll
            for (int kh = 0; kh < 2; ++kh)
#pragma unroll
                for (int i = 0; i < TNS; ++i)
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, af[kh][i]),
                                                                            __builtin_bit_cast(bf16x8, bfr[kh][j]),
                                                                            acc[i][j], 0, 0, 0);
        } else if constexpr (sizeof(T) == 1) {
            // e4m3: lane (fr, fq) holds chunks fq and 4 + fq of row fr -- 32 of the step's 128 K bytes, the same K
            // bytes for A and B, which is all the instruction's lane map asks; E8M0 block scales 2^0 (127)
#pragma unroll
            for (int i = 0; i < TNS; ++i) {
                const i32x8 av = {(int)af[0][i][0], (int)af[0][i][1], (int)af[0][i][2], (int)af[0][i][3],
                                  (int)af[1][i][0], (int)af[1][i][1], (int)af[1][i][2], (int)af[1][i][3]};
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const i32x8 bv = {(int)bfr[0][j][0], (int)bfr[0][j][1], (int)bfr[0][j][2], (int)bfr[0][j][3],
                                      (int)bfr[1][j][0], (int)bfr[1][j][1], (int)bfr[1][j][2], (int)bfr[1][j][3]};
                    acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(av, bv, acc[i][j], 0, 0, 0, 127, 0,
                                                                               127);
                }
            }
        } else if constexpr (SPL > 0) {
            static_assert(SPL == 6 || SPL == 9, "term count");
            // the lane's 8 f32 of a row (chunks fq and 4 + fq) as one 8-deep bf16 operand per term: a 32-deep
            // K-step is one 16x16x32 MFMA per term pair
            bf16x8 at[TNS][3], bt[4][3];
#pragma unroll
            for (int i = 0; i < TNS; ++i) split3_bf16(af[0][i], af[1][i], at[i]);
#pragma unroll
            for (int j = 0; j < 4; ++j) split3_bf16(bfr[0][j], bfr[1][j], bt[j]);
            constexpr int TA[9] = {0, 0, 1, 0, 1, 2, 1, 2, 2}, TB[9] = {0, 1, 0, 2, 1, 0, 2, 1, 2};
#pragma unroll
            for (int t = 0; t < SPL; ++t)
#pragma unroll
                for (int i = 0; i < TNS; ++i)
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(at[i][TA[t]], bt[j][TB[t]], acc[i][j], 0,
                                                                            0, 0);
        } else {
            // f32: element e of lane (fr, fq)'s chunk 4 kh + fq is K index 16 kh + 4 fq + e of the stage -- MFMA
            // (kh, e) sums over fq, so the four MFMAs of a chunk cover its 16 K values (the same permutation of
            // K for both operands: an exact f32 fma chain in another order)
#pragma unroll
            for (int kh = 0; kh < 2; ++kh)
#pragma unroll
                for (int e = 0; e < 4; ++e)
#pragma unroll
                    for (int i = 0; i < TNS; ++i)
#pragma unroll
                        for (int j = 0; j < 4; ++j)
                            // (element e by value: __builtin_bit_cast of a vector-element lvalue reads element 0)
                            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(af[kh][i][e]),
                                                                             __uint_as_float(bfr[kh][j][e]),
                                                                             acc[i][j], 0, 0, 0);
        }
        }
        if constexpr (GLDS) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        } else {
            if (more) CONV2_STORE(s ^ 1);
        }
        __syncthreads();
    }
#undef CONV2_LOAD
#undef CONV2_STORE
#undef CONV2_DMA
#undef CONV2_DMA8
    C2S(2, __builtin_amdgcn_s_memtime());

    {
        if (ksplit > 1) {
            // split-K combine (cdna_hip_programming.md §5 "In-launch split-K reduction", §6 Guideline 16, its sc1
            // form): every slice stores its f32 partial tile write-through (slab [vt][sk][fragment q][thread], 1 KiB
            // per wave-store), drains, and takes an arrival ticket; the slice that draws ksplit - 1 acquires, sums
            // the slabs in slice order (its own read back: the result does not depend on arrival order) and runs the
            // epilogue (a second slab in flight under the adds would cost 64 VGPRs: past 256, one wave per SIMD)
            constexpr int NQ = TNS * 4;
            const int64_t sbase = (int64_t)vt * ksplit * NQ * NT;
#pragma unroll
            for (int q = 0; q < NQ; ++q)
                sk_store16(a.ws, a.ws_bytes, (int)(((sbase + ((int64_t)sk * NQ + q) * NT) + tid) * 16), acc[q / 4][q % 4]);
            if (kred) {
                C2S(3, __builtin_amdgcn_s_memtime());
                C2S(5, __builtin_amdgcn_s_memtime());
                C2S(7, __builtin_amdgcn_s_memrealtime());
                return;
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            int* last_s = (int*)smem;  // the stage buffers are free: the K-loop ended on a barrier
            if (tid == 0) {
                const int prev = __hip_atomic_fetch_add(a.wcnt + vt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const int last = prev == ksplit - 1;
                if (last) {
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    __hip_atomic_store(a.wcnt + vt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // next launch
                }
                last_s[0] = last;
            }
            __syncthreads();
            const bool last = last_s[0] != 0;
            __syncthreads();  // the flag is read before the epilogue reuses the LDS
            C2S(3, __builtin_amdgcn_s_memtime());
            if (!last) {
                C2S(5, __builtin_amdgcn_s_memtime());
                C2S(7, __builtin_amdgcn_s_memrealtime());
                return;
            }
            const f32x4* sl = (const f32x4*)a.ws + sbase + tid;
#pragma unroll
            for (int q = 0; q < NQ; ++q) acc[q / 4][q % 4] = sl[q * NT];
            for (int o = 1; o < ksplit; ++o) {
#pragma unroll
                for (int q = 0; q < NQ; ++q) acc[q / 4][q % 4] += sl[((int64_t)o * NQ + q) * NT];
            }
        }
    }
    C2S(4, __builtin_amdgcn_s_memtime());

    auto orow = [&](int pl) -> int64_t {
        const int m = m0 + pl;
        return m < a.M ? (a.mode == 1 ? (int64_t)m : conv_out_row(a, m, cls)) : -1;
    };
    if constexpr (BN == 128 && sizeof(T) == 2) {
        if (a.w2) {
            conv2_tail<NT, BM, TNS, OutT>(a, acc, smem, n0, wm, wn, wid, fr, fq, orow, m0, cls);
            return;
        }
    }
    conv_epilogue<NT, BM, BN, TNS, OutT, decltype(orow), T>(a, acc, smem, n0, wm, wn, tid, fr, fq, orow, m0, cls);
    C2S(5, __builtin_amdgcn_s_memtime());
    C2S(7, __builtin_amdgcn_s_memrealtime());
}

// ------------------------------------------------------------------------ split-K, reduce form
// conv2_kernel with ksplit < 0 leaves its slices' f32 partial tiles in the workspace (slab [vt][sk][q][thread]: one
// 16-byte accumulator fragment per unit) and this kernel finishes them: a thread per (virtual tile, fragment q,
// thread) unit sums the slices in slice order -- the ticket combine's arithmetic, so the result is bit-identical --
// and applies conv_epilogue's element work (weight scale, bias, SiLU, residual) to its four channels of one pixel,
// stored straight to the output.  The ticket form sums a tile's ks x 64 KiB in ONE workgroup once the last slice
// has arrived (~0.45 us per slice at batch 1) and then runs a 2-6 us LDS epilogue on it
// (profiles/r06/b1/phases_f32_b1.log); here every CU takes a share.  Mode 0 without a fused tail (conv2_red_ok).
constexpr int SK_RED_MAX = 32;  // the reduce form's slice cap (conv2_ksplit)
// FRAG32: conv3t's slabs (v_mfma_f32_32x32x16 accumulators, conv_epilogue32_fill's layout: unit q = 8 ib + 4 jb + c
// of lane l holds pixel wm 64 + 32 jb + l % 32, channels wn 16 TNS + 32 ib + 8 c + 4 (l / 32) ..)
template <typename RT, typename OutT, int WM, int WN, int TNS, bool FRAG32 = false>
__global__ __launch_bounds__(256) void conv2_reduce_kernel(va_conv_args a, int ntn, int ks, int nunits) {
    constexpr int NT = 64 * WM * WN, NQ = TNS * 4, BM = 64 * WM, BN = 16 * TNS * WN;
    const int u = blockIdx.x * 256 + threadIdx.x;
    if (u >= nunits) return;
    const int tid = u % NT, q = (u / NT) % NQ, vt = u / (NT * NQ);
    const int wid = tid >> 6, lane = tid & 63, wm = wid / WN, wn = wid % WN, fr = lane & 15, fq = lane >> 4;
    // conv_epilogue's (conv_epilogue32_fill's) pixel of the unit and its first channel
    const int m = (vt / ntn) * BM + wm * 64 + (FRAG32 ? 32 * ((q >> 2) & 1) + (lane & 31) : 16 * (q % 4) + fr);
    const int co = (vt % ntn) * BN + wn * 16 * TNS +
                   (FRAG32 ? 32 * (q >> 3) + 8 * (q & 3) + 4 * (lane >> 5) : 16 * (q / 4) + 4 * fq);
    if (m >= a.M || co >= a.Cout) return;
    const float4 bv = *(const float4*)(a.bias + co);  // issued ahead of the slabs: one memory latency, not two
    const f32x4* sl = (const f32x4*)a.ws + ((int64_t)vt * ks * NQ + q) * NT + tid;
    // every slab load issued before the first add (ks <= SK_RED_MAX: a loop of eight-load rounds waited one memory
    // latency per round), then added in slice order
    f32x4 t[SK_RED_MAX];
#pragma unroll
    for (int e = 0; e < SK_RED_MAX; ++e)
        if (e < ks) t[e] = sl[(int64_t)e * NQ * NT];
    f32x4 ac = t[0];
#pragma unroll
    for (int e = 1; e < SK_RED_MAX; ++e)
        if (e < ks) ac += t[e];
    if (sizeof(RT) == 2 && a.w8) {
        const float4 sv = *(const float4*)(a.wscale + co);
        ac = ac * (f32x4){sv.x, sv.y, sv.z, sv.w};
    }
    float v[4] = {ac[0] + bv.x, ac[1] + bv.y, ac[2] + bv.z, ac[3] + bv.w};
    if (a.act) {
        const f32x2 s01 = fz::silu2((f32x2){v[0], v[1]}), s23 = fz::silu2((f32x2){v[2], v[3]});
        v[0] = s01[0];
        v[1] = s01[1];
        v[2] = s23[0];
        v[3] = s23[1];
    }
    if (a.res) {
        const RT* rp = (const RT*)a.res + (int64_t)m * a.ldr + co;
        if constexpr (sizeof(RT) == 4) {
            const float4 r = *(const float4*)rp;
            v[0] += r.x, v[1] += r.y, v[2] += r.z, v[3] += r.w;
        } else {
            const uint2 r = *(const uint2*)rp;
            const RT* re = (const RT*)&r;
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] += (float)re[e];
        }
    }
    OutT* yp = (OutT*)a.y + (int64_t)m * a.ldy + co;
    if constexpr (sizeof(OutT) == 2) {
        __attribute__((aligned(8))) __bf16 o[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = (__bf16)v[e];
        *(uint2*)yp = *(const uint2*)o;
    } else {
        *(float4*)yp = make_float4(v[0], v[1], v[2], v[3]);
    }
}

// ------------------------------------------------------------------------ conv3t (f32 mode, three-plane K-loop)
// The f32 conv as six exact bf16 term products (conv2's SPL 6) without the per-wave split in the K-loop: the
// weights arrive pre-split (va_conv_args.w3: [Npad][Kpad/8][3][8] bf16, h / m / l per 8-channel group) and each
// f32 activation is split ONCE per workgroup, while it is staged: a thread loads the 8 channels of one (pixel,
// group) of K-step k + 2 into registers, and splits and stores the three bf16 planes of K-step k + 1 into LDS
// while the MFMAs of step k run.  256-pixel x 128-channel tiles, 8 waves (4 x 2, 64 x 64 each), K-step 16
// channels, three LDS stages (A by LDS-DMA two steps ahead), one workgroup per CU.  The MFMA is
// v_mfma_f32_32x32x16_bf16: lane (r, g) = (lane % 32, lane / 32) feeds row r of a 32-row block with channels
// 8 g .. 8 g + 7 of the step, plane p of a row is one 16-byte read; per 32 x 32 block pair the six products
// h.h, h.m, m.h, h.l, m.m, l.h are six MFMAs (24 per wave per K-step).
// LDS row: 128 bytes = 8 slots of 16 B; chunk c = 3 g + p (c < 6) sits in slot c ^ (r & 7) ^ ((r >> 4) & 1) -- the
// 32-row fragment reads are conflict-free, slots 6-7 of a chunk are DMA'd from the zero page.
constexpr int T3_BN = 128, T3_KS = 16, T3_ROW = 128;
template <int WM, int NSTAGE>
struct T3Cfg {
    static constexpr int BM = 64 * WM, NT = 128 * WM, STAGE = (BM + T3_BN) * T3_ROW;
    static constexpr int EPI = BM * (T3_BN + 4) * 4;
    static constexpr int LDS = NSTAGE * STAGE > EPI ? NSTAGE * STAGE : EPI;
    static constexpr int NA = 16 / (2 * WM);  // A-DMA instructions per wave per K-step (16 KiB of A)
    static_assert(LDS <= 160 * 1024, "LDS");
};

__device__ __forceinline__ int t3_slot(int c, int r) { return c ^ (r & 7) ^ ((r >> 4) & 1); }
template <int N>
__device__ __forceinline__ void t3_waitvm() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// WM = 4, NSTAGE = 3: 256-pixel tiles, 8 waves, one workgroup per CU, A DMA'd two K-steps ahead;
// WM = 2, NSTAGE = 2: 128-pixel tiles, 4 waves, two workgroups per CU, A one K-step ahead.  B registers always
// two K-steps ahead.
template <int WM, int NSTAGE, typename OutT>
__global__ __launch_bounds__(128 * WM) void conv3t_kernel(va_conv_args a, int ntn, int ntiles, int ksplit, int kper) {
    using Cfg = T3Cfg<WM, NSTAGE>;
    extern __shared__ __align__(16) unsigned char smt[];
    constexpr int BM = Cfg::BM, BN = T3_BN, NT = Cfg::NT, WN = 2, TNS = 4, NA = Cfg::NA;
    int bid = blockIdx.x;
    {
        const int nx = 8, q = ntiles / nx, r = ntiles % nx, xcd = bid % nx, j = bid / nx;
        bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + j;
    }
    // split K (ksplit > 1, mode 0, batch-1 shapes): slice sk runs K-steps [sk kper, ..) and stores its partial tile
    // as a slab for conv2_reduce_kernel (conv2's reduce form, the 32 x 32 fragment layout); the slices of a tile are
    // consecutive virtual blocks
    const int sk = bid % ksplit;
    bid /= ksplit;
    const int vt = bid;
    const int cls = a.mode == 2 ? (bid & 3) : 0;
    if (a.mode == 2) bid >>= 2;
    const int tm = bid / ntn, tn = bid % ntn;
    const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wid / WN, wn = wid % WN;
    const int m0 = tm * BM, n0 = tn * BN;
    const float* __restrict__ X = (const float*)a.x;
    const void* WA = (const void*)((const __bf16*)a.w3 + (int64_t)cls * a.Npad * a.Kpad * 3);
    const int pad_y = a.mode == 2 ? 1 - (cls >> 1) : a.pad, pad_x = a.mode == 2 ? 1 - (cls & 1) : a.pad;
    auto stA = [&](int s) { return smt + s * Cfg::STAGE; };
    auto stB = [&](int s) { return smt + s * Cfg::STAGE + BN * T3_ROW; };
    // this slice's K-steps [kb, kb + nk) of the nk_all
    const int nk_all = a.Kpad / T3_KS, kb = sk * kper;
    const int nk = (nk_all - kb < kper ? nk_all - kb : kper);

    // ---- B staging unit of this thread: row br (pixel m0 + br), 8-channel group bg of each K-step; lanes 0-7 of
    // a wave take 8 consecutive rows of one group (conflict-free 16-byte plane stores)
    const int br = (tid & 7) | ((tid >> 4) << 3), bg = (tid >> 3) & 1;
    int b_hi, b_wi;
    int64_t b_base;
    {
        const int m = m0 + br;
        if (m < a.M) {
            const int wo = m % a.Wo, t = m / a.Wo, ho = t % a.Ho, n = t / a.Ho;
            b_hi = ho * a.stride - pad_y;
            b_wi = wo * a.stride - pad_x;
            b_base = (int64_t)n * a.H * a.W;
        } else {
            b_hi = -(1 << 28), b_wi = 0, b_base = 0;
        }
    }
    // ---- A DMA: instructions i = wid + 2 WM j (rows 8 i .. 8 i + 7 of the stage); lane l: row 8 i + (l >> 3),
    // slot l & 7 -> chunk (slot ^ swizzle), whose 16 bytes are bf16 elements 8 chunk .. of the row's K-step run.
    // buffer_load ... lds, not global_load_lds: the compiler's wait pass takes a pending FLAT-encoded LDS DMA as
    // "VM and LGKM out of order" and answers the next register dependency with vmcnt(0), draining the B loads two
    // steps ahead.  Chunks 6-7 (and K-steps past the last) use an offset past the descriptor's range: zeros.
    const void* zpage = (const void*)g_zero_page;
    const int wa_bytes = a.Npad * a.Kpad * 3 * 2;
    constexpr int T3_OOR = 0x7ff00000;
    int aoff[NA];
#pragma unroll
    for (int j = 0; j < NA; ++j) {
        const int row = 8 * (wid + 2 * WM * j) + (lane >> 3);
        const int c = (lane & 7) ^ (row & 7) ^ ((row >> 4) & 1);
        aoff[j] = c < 6 ? ((n0 + row) * a.Kpad * 3 + 8 * c) * 2 : T3_OOR;
    }
    auto dmaA = [&](int k, int s, bool live) {  // this slice's K-step k (channels 16 (kb + k) ..) into stage s
        unsigned char* base = stA(s);
        const int soff = live ? (kb + k) * 96 : T3_OOR;
#pragma unroll
        for (int j = 0; j < NA; ++j)
            t3_dma16(WA, wa_bytes, base + (wid + 2 * WM * j) * 1024, aoff[j], soff);
    };
    // K-step -> (channel group, tap, 16-channel half) of the im2col row, group-major as the w3 runs (seg.py w3_rows: a
    // group's taps in a row, so its input footprint stays in L2 across them; gh = 2 sixteen-channel K-steps per (group,
    // tap) on the stride-2 3x3s -- seg.py w3_group's rule -- so both 64-byte halves of a pixel's 128-byte line are read
    // in consecutive K-steps), advanced per load (uniform)
    const int gh = a.stride == 2 && a.kh * a.kw > 1 && a.Cin % 32 == 0 ? 2 : 1;
    int ld_ky, ld_kx, ld_c, ld_h;
    {
        const int per = a.kh * a.kw * gh, grp = kb / per, r = kb - grp * per, tap = r / gh;
        ld_h = r - tap * gh;
        ld_c = (grp * gh + ld_h) * T3_KS;
        ld_ky = tap / a.kw;
        ld_kx = tap - ld_ky * a.kw;
    }
    u32x4 rb[2][2];  // B registers of two K-steps in flight
    // unconditional: out-of-range taps and the loads past the last K-step read the zero page, so the loop body
    // has no branches and the compiler's own waits on rb see one straight-line load / use pattern
    auto loadB = [&](int slot, bool live) {
        const int hi = b_hi + ld_ky, wi = b_wi + ld_kx;
        const bool ok = live && (unsigned)hi < (unsigned)a.H && (unsigned)wi < (unsigned)a.W;
        const float* p = ok ? X + (b_base + (int64_t)hi * a.W + wi) * a.ldx + ld_c + 8 * bg : (const float*)zpage;
        rb[slot][0] = *(const u32x4*)p;
        rb[slot][1] = *(const u32x4*)(p + 4);
        if (++ld_h < gh) {
            ld_c += T3_KS;
        } else {
            ld_h = 0;
            ld_c -= (gh - 1) * T3_KS;
            if (++ld_kx == a.kw) {
                ld_kx = 0;
                if (++ld_ky == a.kh) {
                    ld_ky = 0;
                    ld_c += gh * T3_KS;
                }
            }
        }
    };
    auto storeB = [&](int slot, int s) {  // split the 8 f32 once, three plane chunks into stage s
        bf16x8 t[3];
        split3_bf16(rb[slot][0], rb[slot][1], t);
        unsigned char* rowp = stB(s) + br * T3_ROW;
#pragma unroll
        for (int p = 0; p < 3; ++p) *(bf16x8*)(rowp + 16 * t3_slot(3 * bg + p, br)) = t[p];
    };

    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = (f32x16){};
    // prologue: A of steps 0 .. NSTAGE - 2 in their stages, B of steps 0 and 1 in registers; step 0 staged
#pragma unroll
    for (int k = 0; k < NSTAGE - 1; ++k) dmaA(k, k, k < nk);
    __builtin_amdgcn_sched_barrier(0);  // the DMAs issue before the loads (the count below assumes it)
    loadB(0, true);
    loadB(1, nk > 1);
    __builtin_amdgcn_sched_barrier(0);
    t3_waitvm<2>();  // everything but step 1's two B loads
    storeB(0, 0);
    __syncthreads();
    const int r32 = lane & 31, g32 = lane >> 5;
    constexpr int TA[6] = {0, 0, 1, 0, 1, 2}, TB[6] = {0, 1, 0, 2, 1, 0};
    // one K-step; LS = the register slot of step k (step k + 2 loads into it, step k + 1 is in 1 - LS): compile-time,
    // so the compiler's own waits on the B registers stay where their data is consumed (a runtime slot index made
    // it wait for every load at once).  Every step issues the same NA DMAs + 2 loads (zero-page sources past the
    // last K-step) and stores the next step's B, so the counted waits are constants and the body has no branch.
    // The step ends in a raw s_barrier (__syncthreads() would add vmcnt(0) and drain the loads two steps ahead).
    auto step = [&](const int k, auto LSc) {
        constexpr int LS = decltype(LSc)::value;
        const int s = k % NSTAGE;
        dmaA(k + NSTAGE - 1, (k + NSTAGE - 1) % NSTAGE, k + NSTAGE - 1 < nk);  // stage last read at step k - 1
        // the counted waits below assume this step's NA DMAs issue BEFORE its two B loads: pinned, not left to the
        // scheduler (an early B load would let vmcnt(2) retire the loads with a DMA still in flight)
        __builtin_amdgcn_sched_barrier(0);
        loadB(LS, k + 2 < nk);  // step k's registers were stored at step k - 1
        __builtin_amdgcn_sched_barrier(0);
        bf16x8 ap[2][3], bp[2][3];
        const unsigned char* as_ = stA(s);
        const unsigned char* bs_ = stB(s);
#pragma unroll
        for (int ib = 0; ib < 2; ++ib) {
            const int row = wn * 64 + 32 * ib + r32;
#pragma unroll
            for (int p = 0; p < 3; ++p) ap[ib][p] = *(const bf16x8*)(as_ + row * T3_ROW + 16 * t3_slot(3 * g32 + p, row));
        }
#pragma unroll
        for (int jb = 0; jb < 2; ++jb) {
            const int row = wm * 64 + 32 * jb + r32;
#pragma unroll
            for (int p = 0; p < 3; ++p) bp[jb][p] = *(const bf16x8*)(bs_ + row * T3_ROW + 16 * t3_slot(3 * g32 + p, row));
        }
#pragma unroll
        for (int t = 0; t < 6; ++t)
#pragma unroll
            for (int ib = 0; ib < 2; ++ib)
#pragma unroll
                for (int jb = 0; jb < 2; ++jb)
                    acc[ib][jb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ap[ib][TA[t]], bp[jb][TB[t]], acc[ib][jb], 0,
                                                                          0, 0);
        // step k + 1's A (DMA'd NSTAGE - 1 steps ago: this step when NSTAGE = 2) and B (loaded one step ago)
        // complete; this step's two B loads stay in flight, and with NSTAGE = 3 this step's DMA too
        t3_waitvm<NSTAGE == 2 ? 2 : NA + 2>();
        storeB(1 - LS, (k + 1) % NSTAGE);  // past the last step: a harmless store into a stage nobody reads
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // stores visible, stage reads retired
    };
    int k = 0;
    for (; k + 1 < nk; k += 2) {
        step(k, std::integral_constant<int, 0>{});
        step(k + 1, std::integral_constant<int, 1>{});
    }
    if (k < nk) step(k, std::integral_constant<int, 0>{});
    t3_waitvm<0>();  // the zero-page DMAs past the last step land before the epilogue reuses the LDS
    if (ksplit > 1) {  // the slab: unit q = 8 ib + 4 jb + c holds acc[ib][jb] items 4 c .. 4 c + 3
        const int64_t sbase = (int64_t)vt * ksplit * 16 * NT;
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const f32x16& v = acc[q >> 3][(q >> 2) & 1];
            const int c = q & 3;
            sk_store16(a.ws, a.ws_bytes, (int)((sbase + ((int64_t)sk * 16 + q) * NT + tid) * 16),
                       (f32x4){v[4 * c], v[4 * c + 1], v[4 * c + 2], v[4 * c + 3]});
        }
        return;
    }
    __syncthreads();

    auto orow = [&](int pl) -> int64_t {
        const int m = m0 + pl;
        return m < a.M ? conv_out_row(a, m, cls) : -1;
    };
    auto mrow = [&](int pl) { return m0 + pl; };
    auto pcol = [](int c) { return c; };
    conv_epilogue32<NT, BM, BN, TNS, OutT>(a, acc, smt, n0, wm, wn, tid, lane, orow, mrow, pcol, cls);
}

// ------------------------------------------------------------------------ conv3h (f32 mode, halo-staged B)
// conv3t's three-term arithmetic for the stride-1 convs with several taps (3x3 / pad 1, and the proto's sub-pixel
// classes: 2x2 taps, mode 2), with the activation operand staged ONCE per 16-channel chunk instead of once per tap.
// conv3t loads B per K-step, i.e. per (tap, chunk): a 3x3 layer moves every input pixel through L2 -> L1 nine
// times and splits it nine times -- the vector-memory return path and the L2 were the wall (TD busy 0.81, TCC busy
// 0.94 on the four largest layers).  conv3h tiles the output as TH x TW pixels of the stacked
// [N * Ho] x Wo map (TW = 4 .. 32 chosen per layer so the tiles cover Wo exactly; TH x TW = 128) and, per chunk of
// 16 input channels, loads the tile's halo -- (TH + kh - 1) x (TW + kw - 1) <= 204 pixels, 1.4-1.6 x the tile --
// once, splits it once into three bf16 planes in LDS, and forms all kh x kw taps from it: per chunk the K-steps
// are the taps, each one A stage (the pre-split weights of (tap, chunk), LDS-DMA two steps ahead, three stages)
// and the B fragments read from the halo at the tap's offset.  A tile that straddles two images of the stacked
// map reads zeros (a zero row) where a tap leaves the pixel's own image, so no tile is ragged.  The next chunk's
// halo is loaded into registers at the chunk's first step (after that step's A DMA: the issue order the counted
// waits assume, pinned by sched_barrier), split and stored into the other halo buffer at its second step (that
// buffer was last read in the previous chunk), and is read from the chunk after.  LDS rows are 96 bytes (16
// channels x 3 planes); chunk c of a weight row r sits in slot c ^ ((r >> 3) & 1), of halo pixel (hy, hx) in
// slot c ^ ((hy ^ (hx >> 3 if TW >= 16)) & 1), and B-block row r holds pixel t3h_perm(r): each ds_read_b128 lane
// group then reads 16 consecutive pixels of one tile row -- conflict-free for every TW and tap
// (tools/lds_conflicts.py).  128 pixels x 128 channels, 4 waves, two workgroups per CU.
constexpr int T3H_ROW = 96, T3H_BM = 128, T3H_NT = 256, T3H_HMAX = 204, T3H_NSA = 3;
constexpr int T3H_HALO = T3H_HMAX * T3H_ROW;  // 19,584 B
constexpr int T3H_NU = 2;                     // halo units (pixel, 8 channels) per thread
static_assert(T3H_NU * T3H_NT >= 2 * T3H_HMAX, "halo units");
// per channel-tile width: TNS = 4 -> 128 output channels (waves 2 x 2, each 64 pixels x 64 channels), TNS = 2 -> 64
// (the narrow layers: waves 2 x 2, each 64 pixels x 32 channels).  TPS = taps per K-step: a stage holds TPS taps'
// weights of the chunk, one BN x 96-byte block per tap.  (TPS = 2 on the narrow tiles -- the wide tiles' 24 MFMAs per
// wave and barrier -- measured neutral, 14.10 vs 14.11 ms per 64-frame forward, profiles/r04/conv3h_tps/; the
// library instantiates TPS = 1 only).  (The A stage as f32 weights split in registers per wave -- 4 instead of 6
// L2 -> LDS bytes per weight -- measured 4-10 % slower and was removed in round 6)
template <int TNS, int TPS = 1>
struct T3HCfg {
    static constexpr int BN = 32 * TNS;
    static constexpr int AROW = T3H_ROW;                          // LDS bytes per weight row of a (tap, chunk)
    static constexpr int ABLK = BN * AROW;                        // one tap's weights of a chunk: 12 / 6 KiB
    static constexpr int ASTAGE = TPS * ABLK;
    static constexpr int NP = ASTAGE / 1024;                      // A-DMA pieces per K-step (12 / 6)
    static constexpr int NAW = (NP + 3) / 4;                      // pieces of the busiest wave (3 / 2)
    static constexpr int ZROW = T3H_NSA * ASTAGE + 2 * T3H_HALO;  // the zero row
    static constexpr int SINK = ZROW + 128;                       // 1 KiB the idle pieces' zero DMAs land in
    static constexpr int LDS0 = NP % 4 ? SINK + 1024 : ZROW + T3H_ROW;
    static constexpr int EPI = T3H_BM * (BN + 4) * 4;
    static constexpr int LDS = LDS0 > EPI ? LDS0 : EPI;
    static_assert(NP * 1024 == ASTAGE && 2 * LDS <= 160 * 1024, "A stage in 1 KiB pieces; two workgroups per CU");
};


// B-block row r (0..31) -> pixel of the block: ds_read_b128's lane groups {0-3, 12-15, 20-27} and {4-11, 16-19,
// 28-31} (MI355X_MICROARCH.md §LDS) take pixels 0..15 and 16..31 in lane order
__device__ __forceinline__ int t3h_perm(int r) {
    return r < 4 ? r : r < 12 ? r + 12 : r < 16 ? r - 8 : r < 20 ? r + 8 : r < 28 ? r - 12 : r;
}

// f(integral_constant<0>) .. f(integral_constant<N - 1>), in order
template <int N, int I = 0, typename F>
__device__ __forceinline__ void t3h_unroll(F&& f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        t3h_unroll<N, I + 1>(f);
    }
}

template <int KH, int KW, int TNS, typename OutT, bool TAIL = false, int TPS = 1>
__global__ __launch_bounds__(T3H_NT) void conv3h_kernel(va_conv_args a, int ntn, int ntiles, int lgw, int tiles_x) {
    extern __shared__ __align__(16) unsigned char smh[];
    using Cfg = T3HCfg<TNS, TPS>;
    constexpr int BM = T3H_BM, BN = Cfg::BN, NT = T3H_NT, WN = 2, CB = TNS / 2, T = KH * KW;
    constexpr int S = (T + TPS - 1) / TPS;  // K-steps per chunk
    static_assert(S >= 2, "the halo is stored at a chunk's second step");
    int bid = blockIdx.x;
    {
        const int nx = 8, q = ntiles / nx, r = ntiles % nx, xcd = bid % nx, j = bid / nx;
        bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + j;
    }
    const int cls = a.mode == 2 ? (bid & 3) : 0;
    if (a.mode == 2) bid >>= 2;
    const int tm = bid / ntn, tn = bid % ntn;
    const int TW = 1 << lgw, TH = BM >> lgw, HW = TW + KW - 1, HHW = (TH + KH - 1) * HW;
    const int ty = tm / tiles_x, tx = tm - ty * tiles_x;
    const int r0 = ty * TH, c0 = tx * TW;  // stacked output row / column of the tile's pixel 0
    const int NR = a.N * a.Ho;
    const int pad_y = a.mode == 2 ? 1 - (cls >> 1) : a.pad, pad_x = a.mode == 2 ? 1 - (cls & 1) : a.pad;
    const int xm = lgw >= 4 ? 1 : 0;
    const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wid / WN, wn = wid % WN;
    const int n0 = tn * BN;
    const int nch = a.Cin / T3_KS;
    const float* __restrict__ X = (const float*)a.x;
    // A source: the pre-split planes (w3); mode 2: the sub-pixel class's matrix
    const void* WA = (const void*)((const __bf16*)a.w3 + (int64_t)cls * a.Npad * a.Kpad * 3);
    auto stA = [&](int s) { return smh + s * Cfg::ASTAGE; };
    auto halo = [&](int b) { return smh + T3H_NSA * Cfg::ASTAGE + b * T3H_HALO; };

    // ---- A DMA: piece P = wid + 4 j of a stage (1 KiB, linear in LDS); lane l writes bytes 16 l of it: row o / 96,
    // slot (o % 96) / 16 -> chunk slot ^ ((row >> 3) & 1) of that weight row's (tap, chunk) run.  Every wave issues
    // NA pieces per K-step (12 over 4 waves; 64-channel tiles: 6, so waves 2-3 send their second piece's zeros to a
    // sink): a fixed count, no branch, so the counted waits and the compiler's own stay exact
    const int wa_bytes = a.Npad * a.Kpad * 3 * 2;
    constexpr int OOR = 0x7ff00000;
    constexpr int NA = Cfg::NAW;
    int aoff[NA];
#pragma unroll
    for (int j = 0; j < NA; ++j) {
        const int o = (1024 * (wid + (NT / 64) * j)) % Cfg::ABLK + 16 * lane;  // offset in the piece's tap block
        const int row = o / T3H_ROW, c = ((o - row * T3H_ROW) >> 4) ^ ((row >> 3) & 1);
        aoff[j] = ((n0 + row) * a.Kpad * 3 + 8 * c) * 2;
    }
    // stage s <- the weights of taps TPS t .. of chunk c (kl_h = chunk * T + tap, or -1: zeros); a piece's tap
    // block is wave-uniform, so the per-tap source offset is a scalar select
    auto dmaA = [&](int kl0, int kl1, int s) {
        unsigned char* base = stA(s);
        constexpr int KLB = 96;  // source bytes of one (tap, chunk) run of a row
        const int so0 = kl0 >= 0 ? kl0 * KLB : OOR, so1 = kl1 >= 0 ? kl1 * KLB : OOR;
#pragma unroll
        for (int j = 0; j < NA; ++j) {
            const int P = wid + (NT / 64) * j;
            const bool real = Cfg::NP % 4 == 0 || P < Cfg::NP;  // wave-uniform: scalar selects, no branch
            const int soff = TPS > 1 && P * 1024 >= Cfg::ABLK ? so1 : so0;
            t3_dma16(WA, wa_bytes, real ? base + P * 1024 : smh + Cfg::SINK, aoff[j], real ? soff : OOR);
        }
    };
    // the w3 run of tap slot h of step t of chunk c (chunk-major, seg.py w3_rows; -1 past the taps or the chunks)
    auto klof = [&](int c, int t, int h) { return (c < nch && TPS * t + h < T) ? c * T + TPS * t + h : -1; };

    // ---- halo units: u = tid + 256 j -> halo pixel u >> 1 (row hy, column hx), channels 8 (u & 1) .. of a chunk
    const void* zpage = (const void*)g_zero_page;
    int64_t hsrc[T3H_NU];  // element offset of the unit's channels in chunk 0, or -1 (outside the map: zeros)
    int hdst[T3H_NU];      // LDS byte offset of the unit's pixel row in a halo buffer, or -1 (no such pixel)
    int hbit[T3H_NU];
#pragma unroll
    for (int j = 0; j < T3H_NU; ++j) {
        const int u = tid + NT * j, hp = u >> 1, g = u & 1;
        const int hy = hp / HW, hx = hp - hy * HW;
        const int R = r0 - pad_y + hy, Xc = c0 - pad_x + hx;
        const bool in = hp < HHW;
        hsrc[j] = in && (unsigned)R < (unsigned)NR && (unsigned)Xc < (unsigned)a.W
                      ? ((int64_t)R * a.W + Xc) * a.ldx + 8 * g : -1;
        hdst[j] = in ? hp * T3H_ROW : -1;
        hbit[j] = (hy ^ ((hx >> 3) & xm)) & 1;
    }
    u32x4 rh[T3H_NU][2];
    auto loadH = [&](int c, bool live) {  // chunk c of every unit into registers (zero page: outside / past the end)
#pragma unroll
        for (int j = 0; j < T3H_NU; ++j) {
            const float* p = live && hsrc[j] >= 0 ? X + hsrc[j] + T3_KS * c : (const float*)zpage;
            rh[j][0] = *(const u32x4*)p;
            rh[j][1] = *(const u32x4*)(p + 4);
        }
    };
    auto storeH = [&](int b) {  // split once, three plane chunks per unit into halo buffer b
        unsigned char* hb = halo(b);
#pragma unroll
        for (int j = 0; j < T3H_NU; ++j) {
            bf16x8 t[3];
            split3_bf16(rh[j][0], rh[j][1], t);
            if (hdst[j] >= 0) {
                const int g = (tid + NT * j) & 1;
#pragma unroll
                for (int p = 0; p < 3; ++p) *(bf16x8*)(hb + hdst[j] + 16 * ((3 * g + p) ^ hbit[j])) = t[p];
            }
        }
    };

    // ---- B fragment rows of this lane: block jb's row r32 is tile pixel (py, px); vy bit ky: the tap row stays in
    // the pixel's own image
    const int r32 = lane & 31, g32 = lane >> 5;
    int bpy[2], bpx[2], vy[2];
#pragma unroll
    for (int jb = 0; jb < 2; ++jb) {
        const int p = wm * 64 + 32 * jb + t3h_perm(r32);
        bpy[jb] = p >> lgw;
        bpx[jb] = p & (TW - 1);
        const int h = (r0 + bpy[jb]) % a.Ho;
        int v = 0;
#pragma unroll
        for (int ky = 0; ky < KH; ++ky) v |= ((unsigned)(h - pad_y + ky) < (unsigned)a.Ho) << ky;
        vy[jb] = v;
    }

    f32x16 acc[CB][2];
#pragma unroll
    for (int i = 0; i < CB; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = (f32x16){};
    // prologue: A of steps 0, 1 of chunk 0, chunk 0's halo staged; the zero row
    dmaA(klof(0, 0, 0), klof(0, 0, 1), 0);
    dmaA(klof(0, 1, 0), klof(0, 1, 1), 1);
    __builtin_amdgcn_sched_barrier(0);
    loadH(0, true);
    __builtin_amdgcn_sched_barrier(0);
    t3_waitvm<0>();
    storeH(0);
    if (tid < T3H_ROW / 16) *(u32x4*)(smh + Cfg::ZROW + 16 * tid) = (u32x4){0u, 0u, 0u, 0u};
    __syncthreads();
    constexpr int TA[6] = {0, 0, 1, 0, 1, 2}, TB[6] = {0, 1, 0, 2, 1, 0};
    // one K-step (chunk c, tap t): A(k + 2) DMA'd first, at t == 0 the next chunk's halo loads, the fragment reads,
    // 24 MFMAs, at t == 1 the next chunk's halo stored; then the counted wait for A(k + 1) and a raw barrier
    auto step = [&](const int c, auto Tc) {
        constexpr int t = decltype(Tc)::value;
        const int k = c * S + t;
        {
            constexpr int t2 = (t + 2) % S, dc = (t + 2) / S;
            dmaA(klof(c + dc, t2, 0), klof(c + dc, t2, 1), (k + 2) % T3H_NSA);  // stage last read at step k - 1
        }
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (t == 0) {
            loadH(c + 1, c + 1 < nch);
            __builtin_amdgcn_sched_barrier(0);
        }
        const unsigned char* hs_ = halo(c & 1);
        t3h_unroll<TPS>([&](auto Hc) {
            constexpr int h = decltype(Hc)::value, tap = TPS * t + h;
            if constexpr (tap < T) {
                constexpr int ky = tap / KW, kx = tap % KW;
                bf16x8 ap[CB][3], bp[2][3];
                const unsigned char* as_ = stA(k % T3H_NSA) + h * Cfg::ABLK;
#pragma unroll
                for (int ib = 0; ib < CB; ++ib) {
                    const int row = wn * 32 * CB + 32 * ib + r32;
                    const int sw = (row >> 3) & 1;
#pragma unroll
                    for (int p = 0; p < 3; ++p)
                        ap[ib][p] = *(const bf16x8*)(as_ + row * T3H_ROW + 16 * ((3 * g32 + p) ^ sw));
                }
#pragma unroll
                for (int jb = 0; jb < 2; ++jb) {
                    const int hy = bpy[jb] + ky, hx = bpx[jb] + kx;
                    const unsigned char* rp = (vy[jb] >> ky) & 1 ? hs_ + (hy * HW + hx) * T3H_ROW : smh + Cfg::ZROW;
                    const int sw = (hy ^ ((hx >> 3) & xm)) & 1;
#pragma unroll
                    for (int p = 0; p < 3; ++p) bp[jb][p] = *(const bf16x8*)(rp + 16 * ((3 * g32 + p) ^ sw));
                }
#pragma unroll
                for (int tt = 0; tt < 6; ++tt)
#pragma unroll
                    for (int ib = 0; ib < CB; ++ib)
#pragma unroll
                        for (int jb = 0; jb < 2; ++jb)
                            acc[ib][jb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ap[ib][TA[tt]], bp[jb][TB[tt]],
                                                                                  acc[ib][jb], 0, 0, 0);
            }
        });
        if constexpr (t == 1) storeH((c + 1) & 1);  // the buffer chunk c - 1 used; past the last chunk: unread zeros
        // A(k + 1) landed: younger than its DMAs are this step's NA DMAs and the halo loads of step t == 0 (issued in
        // this step at t == 0, in the previous one at t == 1)
        t3_waitvm<(t == 0 || t == 1) ? NA + 2 * T3H_NU : NA>();
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    };
    for (int c = 0; c < nch; ++c) t3h_unroll<S>([&](auto Tc) { step(c, Tc); });
    t3_waitvm<0>();  // the zero-page DMAs past the last step land before the epilogue reuses the LDS
    __syncthreads();

    auto mrow = [&](int pl) -> int {
        const int R = r0 + (pl >> lgw), Xc = c0 + (pl & (TW - 1));
        return R < NR && Xc < a.Wo ? R * a.Wo + Xc : -1;
    };
    auto orow = [&](int pl) -> int64_t {
        const int m = mrow(pl);
        return m >= 0 ? conv_out_row(a, m, cls) : -1;
    };
    auto pcol = [](int c) { return t3h_perm(c); };
    if constexpr (TAIL) {  // every channel of the conv is in this tile (ntn == 1): the 1x1 tail runs here
        static_assert(BM * (T3_TAIL_C2 + 4) * 4 <= Cfg::LDS, "tail staging inside the workgroup's LDS");
        conv_epilogue32_fill<BN, TNS>(a, acc, smh, n0, wm, wn, lane, mrow, pcol, cls);
        __syncthreads();
        conv_tail32<NT, BM, BN>(a, smh, tid, lane, orow);
    } else {
        conv_epilogue32<NT, BM, BN, TNS, OutT>(a, acc, smh, n0, wm, wn, tid, lane, orow, mrow, pcol, cls);
    }
}

// ----------------------------------------------------------------------------------------- conv v4 (bf16, Cout >= 256)
// 256 output channels x 256 pixels per workgroup with the phase structure of cdna_hip_programming.md §5
// "The 256² 8-phase template": 8 waves (2 channel halves x 4 pixel quarters; each 128 channels x 64
// pixels, acc[8][4]), BK = 64, two LDS buffers of (A 256 x 64 | B 256 x 64) bf16 = 128 KiB, XOR-swizzled
// rows (conv2's image), one workgroup per CU.  A K-tile runs as four phases, one C quadrant each
// (channel frags 0-3 / 4-7 x pixel frags 0-1 / 2-3); every phase
//   reads its fragments (data published one phase earlier) -> issues one half-tile of the NEXT K-tile by
//   LDS-DMA (A rows 0-127, B rows 0-127, B rows 128-255, A rows 128-255 in phases 0..3) -> s_waitcnt
//   vmcnt(4) (retires exactly the half-tile the next phase reads: two half-tiles of 2 DMAs each stay in
//   flight across the barrier) -> s_barrier -> lgkmcnt(0) -> 16 MFMAs at priority 1 -> s_barrier.
// B (pixels) is gathered im2col-style with conv2's FK addressing (Cin % 64 == 0: wave-uniform tap and
// channel chunk, per-row base pointers).  The weight rows are DMA'd in a channel permutation (LDS row
// 32 p + 16 h + r holds channel 32 p + 8 (r/4) + 4 h + r%4) so that fragments 2p, 2p+1 give each lane 8
// consecutive channels: the epilogue stores 16 bytes per lane straight from the accumulators.
constexpr int C4_NT = 512, C4_BUF = 2 * 256 * BK2 * 2;  // bytes per LDS buffer (A then B)

// W8: e4m3 weight bytes (va_conv_args.w8), staged as they are -- the A image 256 rows x 64 bytes (a K-tile), the
// rows in the same channel permutation, 16-byte piece q of row r at slot q ^ ((r >> 2) & 3), piece q holding the K
// chunks q and q + 4 (the rows' w8_pos order) -- and converted to bf16 as the fragments are read (one ds_read_b128 and
// eight v_cvt_scalef32_pk_bf16_fp8 per fragment pair, beside the MFMAs); the epilogue multiplies by the per-output-
// channel scale.  A half-tile is 128 rows x 64 B = one DMA per wave, issued twice (the same source and destination)
// so every half-tile stays two DMAs per wave and each counted wait below stays exact.  (A form that staged the bytes
// through registers and wrote converted rows measured 6-11 % slower than the bf16 weights on m's 1x1 layers.)
template <typename OutT, bool UP = false, bool W8 = false>  // UP: upsampled channel prefix, as conv2_kernel's UP
__global__ __launch_bounds__(C4_NT, 2) void conv4_kernel(va_conv_args a, int ntn, int ntiles) {
    extern __shared__ __align__(16) unsigned char sm4[];
    int bid = blockIdx.x;
    {
        const int nx = 8, q = ntiles / nx, r = ntiles % nx, xcd = bid % nx, j = bid / nx;
        bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + j;
    }
    const int tn = bid % ntn, tm = bid / ntn;  // channel tile fastest: both channel tiles of a pixel tile
    const int c0 = tn * 256, p0 = tm * 256;    // share the staged pixels through the XCD's L2
    const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wr = wid >> 2, wc = wid & 3;     // channel half, pixel quarter
    const int fr = lane & 15, fq = lane >> 4;
    const __bf16* __restrict__ X = (const __bf16*)a.x;
    const __bf16* __restrict__ Wt = (const __bf16*)a.w;

    // Half-tiles are the rows every wave reads in the same phase: A half 0 = rows 0-63 and 128-191 (channel
    // quarter 0 of both channel halves), A half 1 = 64-127, 192-255; B half 0 = the first 32 rows of each
    // 64-pixel quarter, B half 1 = the second 32.  A DMA instruction writes 8 consecutive rows; wave w
    // issues two per half-tile (u = 0, 1); lane l takes row base + (l >> 3) and fetches chunk
    // (l & 7) ^ (l >> 3) (swizzled slot l & 7).  Staged row of (half, u) for this lane:
    const int g = (lane & 7) ^ (lane >> 3), lr = lane >> 3;
    auto a_row0 = [&](int half, int u) { return 64 * half + 8 * wid + 128 * u; };
    auto b_row0 = [&](int half, int u) { return 64 * ((wid >> 2) + 2 * u) + 32 * half + 8 * (wid & 3); };
    const __bf16* wrow[4];  // [2 half + u]: permuted-channel weight rows
    const __bf16* rowp[4];  // [2 half + u]: pixel rows
    const __bf16* rowu[UP ? 4 : 1];  // UP: the pixel's row in the half-resolution source
    int b_hi[4], b_wi[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int R = a_row0(i >> 1, i & 1) + lr;  // LDS row 0..255 of the A image
        const int pp = R >> 5, hh = (R >> 4) & 1, rr = R & 15;
        const int ch = c0 + 32 * pp + 8 * (rr >> 2) + 4 * hh + (rr & 3);
        wrow[i] = Wt + (int64_t)ch * a.Kpad + 8 * g;
        const int m = p0 + b_row0(i >> 1, i & 1) + lr;
        if (m < a.M) {
            const int wo = m % a.Wo, t = m / a.Wo, ho = t % a.Ho, n = t / a.Ho;
            b_hi[i] = ho * a.stride - a.pad;
            b_wi[i] = wo * a.stride - a.pad;
            rowp[i] = X + (((int64_t)n * a.H + b_hi[i]) * a.W + b_wi[i]) * a.ldx + 8 * g;
            if constexpr (UP)
                rowu[i] = (const __bf16*)a.xu + (((int64_t)n * (a.H / 2) + (ho >> 1)) * (a.W / 2) + (wo >> 1)) * a.ldu + 8 * g;
        } else {
            b_hi[i] = -(1 << 28);
            b_wi[i] = 0;
            rowp[i] = X;
            if constexpr (UP) rowu[i] = (const __bf16*)a.xu;
        }
    }
    // W8: this lane's A DMA of half-tile h -- rows 16 (wave's quarter of the half) .. + 15, lane l row + (l >> 2),
    // fetching piece (l & 3) ^ ((row >> 2) & 3) of its permuted channel's e4m3 row
    const uint8_t* wrow8[2];
    int a8row[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int R = (wid < 4 ? 64 * h + 16 * wid : 128 + 64 * h + 16 * (wid - 4)) + (lane >> 2);
        const int pp = R >> 5, hh = (R >> 4) & 1, rr = R & 15;
        const int ch = c0 + 32 * pp + 8 * (rr >> 2) + 4 * hh + (rr & 3);
        a8row[h] = R - (lane >> 2);
        wrow8[h] = (const uint8_t*)a.w + (int64_t)ch * a.Kpad + 16 * ((lane & 3) ^ ((R >> 2) & 3));
    }
    const void* zpage = (const void*)g_zero_page;
    int fk_ky = 0, fk_kx = 0, fk_c = 0, fk_k = 0;  // tap / channel chunk / k of the tile being staged
    auto adv_k = [&]() {
        fk_k += BK2;
        fk_c += BK2;
        if (fk_c == a.Cin) {
            fk_c = 0;
            if (++fk_kx == a.kw) {
                fk_kx = 0;
                ++fk_ky;
            }
        }
    };
    // half-tile h of the K-tile being staged into buffer b, in the order the phases read them:
    // 0 = A half 0, 1 = B half 0, 2 = B half 1, 3 = A half 1
    auto stage = [&](int b, int h) {
        unsigned char* buf = sm4 + b * C4_BUF;
        const bool isA = h == 0 || h == 3;
        const int half = (h == 0 || h == 1) ? 0 : 1;
        const int soff = (fk_ky * a.W + fk_kx) * a.ldx + fk_c;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int i = 2 * half + u;
            const void* src;
            unsigned char* dst;
            if (isA) {
                if constexpr (W8) {  // the e4m3 half-tile: one DMA per wave, issued twice (u = 0, 1)
                    src = (const void*)(wrow8[half] + fk_k);
                    dst = buf + a8row[half] * 64;
                } else {
                    src = (const void*)(wrow[i] + fk_k);
                    dst = buf + a_row0(half, u) * 128;
                }
            } else {
                const bool ok = (unsigned)(b_hi[i] + fk_ky) < (unsigned)a.H && (unsigned)(b_wi[i] + fk_kx) < (unsigned)a.W;
                const __bf16* sp = rowp[i] + soff;
                if constexpr (UP) sp = fk_c < a.cu ? rowu[i] + fk_c : sp;
                src = ok ? (const void*)sp : zpage;
                dst = buf + 256 * BK2 * 2 + b_row0(half, u) * 128;
            }
            __builtin_amdgcn_global_load_lds((gvoid_t*)src, (lvoid_t*)dst, 16, 0, 0);
        }
    };


    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

    const int nk = a.Kpad / BK2;
    // prologue: K-tile 0 in the order A_lo, B_lo, B_hi, A_hi; phase (0, 0) reads A_lo and B_lo
    stage(0, 0);
    stage(0, 1);
    stage(0, 2);
    stage(0, 3);
    adv_k();
    asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)\n\ts_barrier" ::: "memory");

    bf16x8 fa[4][2], fb01[2][2], fb23[2][2];  // [frag][k half]
    auto read_a = [&](const unsigned char* buf, int quarter) {  // channel frags 4 quarter .. +3 of this wave
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int row = 128 * wr + 64 * quarter + 16 * i + fr;
            if constexpr (W8) {  // both K halves in one 16-byte piece of the e4m3 row, converted here
                const u32x4 q = *(const u32x4*)(buf + row * 64 + 16 * (fq ^ ((row >> 2) & 3)));
                fa[i][0] = __builtin_bit_cast(bf16x8, e4m3x8_bf16(make_uint2(q[0], q[1])));
                fa[i][1] = __builtin_bit_cast(bf16x8, e4m3x8_bf16(make_uint2(q[2], q[3])));
            } else {
#pragma unroll
                for (int kh = 0; kh < 2; ++kh)
                    fa[i][kh] = *(const bf16x8*)(buf + row * 128 + 16 * ((4 * kh + fq) ^ (fr & 7)));
            }
        }
    };
    auto read_b = [&](const unsigned char* buf, int pair, bf16x8(&fb)[2][2]) {  // pixel frags 2 pair, +1
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int row = 64 * wc + 32 * pair + 16 * j + fr;
#pragma unroll
            for (int kh = 0; kh < 2; ++kh)
                fb[j][kh] = *(const bf16x8*)(buf + 256 * BK2 * 2 + row * 128 + 16 * ((4 * kh + fq) ^ (fr & 7)));
        }
    };
    auto mma = [&](int quarter, int pair, bf16x8(&fb)[2][2]) {
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int kh = 0; kh < 2; ++kh)
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    acc[4 * quarter + i][2 * pair + j] =
                        __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][kh], fb[j][kh], acc[4 * quarter + i][2 * pair + j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
    };
// retire the half-tile the next phase reads (two half-tiles = 4 DMAs may stay in flight; none are issued in
// the last K-tile), publish it with the barrier, then wait for this phase's own fragment reads
#define C4_SYNC(more)                                                                        \
    {                                                                                        \
        if (more)                                                                            \
            asm volatile("s_waitcnt vmcnt(4)\n\ts_barrier\n\ts_waitcnt lgkmcnt(0)" ::: "memory"); \
        else                                                                                 \
            asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier\n\ts_waitcnt lgkmcnt(0)" ::: "memory"); \
    }
    for (int t = 0; t < nk; ++t) {
        const unsigned char* buf = sm4 + (t & 1) * C4_BUF;
        const bool more = t + 1 < nk;
        const int nb = (t + 1) & 1;
        // phase 0: A_lo x B_lo
        read_a(buf, 0);
        read_b(buf, 0, fb01);
        if (more) stage(nb, 0);
        C4_SYNC(more);
        mma(0, 0, fb01);
        asm volatile("s_barrier" ::: "memory");
        // phase 1: A_lo x B_hi
        read_b(buf, 1, fb23);
        if (more) stage(nb, 1);
        C4_SYNC(more);
        mma(0, 1, fb23);
        asm volatile("s_barrier" ::: "memory");
        // phase 2: A_hi x B_hi
        read_a(buf, 1);
        if (more) stage(nb, 2);
        C4_SYNC(more);
        mma(1, 1, fb23);
        asm volatile("s_barrier" ::: "memory");
        // phase 3: A_hi x B_lo (no reads)
        if (more) {
            stage(nb, 3);
            adv_k();
        }
        C4_SYNC(more);
        mma(1, 0, fb01);
        asm volatile("s_barrier" ::: "memory");
    }

#undef C4_SYNC
    // epilogue straight from the accumulators: fragments 2p, 2p+1 hold channels c0 + 128 wr + 32 p + 8 fq .. +7
    OutT* Y = (OutT*)a.y;
    const __bf16* R = (const __bf16*)a.res;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int m = p0 + 64 * wc + 16 * j + fr;
        if (m >= a.M) continue;
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            const int co = c0 + 128 * wr + 32 * p + 8 * fq;
            if (co >= a.Cout) continue;
            const float4 b0 = *(const float4*)(a.bias + co), b1 = *(const float4*)(a.bias + co + 4);
            f32x4 t0 = acc[2 * p][j], t1 = acc[2 * p + 1][j];
            if constexpr (W8) {  // the e4m3 weights' per-output-channel scale
                const float4 s0 = *(const float4*)(a.wscale + co), s1 = *(const float4*)(a.wscale + co + 4);
                t0 = t0 * (f32x4){s0.x, s0.y, s0.z, s0.w};
                t1 = t1 * (f32x4){s1.x, s1.y, s1.z, s1.w};
            }
            float v[8] = {t0[0] + b0.x, t0[1] + b0.y, t0[2] + b0.z, t0[3] + b0.w,
                          t1[0] + b1.x, t1[1] + b1.y, t1[2] + b1.z, t1[3] + b1.w};
            if (a.act) {
                silu_n(v);
            }
            if (R) {
                const bf16x8 rr = *(const bf16x8*)(R + (int64_t)m * a.ldr + co);
#pragma unroll
                for (int r = 0; r < 8; ++r) v[r] += (float)rr[r];
            }
            if constexpr (sizeof(OutT) == 2) {
                bf16x8 o;
#pragma unroll
                for (int r = 0; r < 8; ++r) o[r] = (__bf16)v[r];
                *(bf16x8*)(Y + (int64_t)m * a.ldy + co) = o;
            } else {
                *(float4*)(Y + (int64_t)m * a.ldy + co) = make_float4(v[0], v[1], v[2], v[3]);
                *(float4*)(Y + (int64_t)m * a.ldy + co + 4) = make_float4(v[4], v[5], v[6], v[7]);
            }
        }
    }
}

// ----------------------------------------------------------------------------------------- small-N conv
// Narrow layers (Cout <= 64: the C2f bottlenecks of P2/P3, the level-0 box/coef head branches) have
// too little MFMA work per staged activation byte for the LDS-staged kernel: both its LDS traffic
// and its 1-block-per-CU footprint bound them.  Here the whole (small) weight matrix lives in LDS,
// loaded once per workgroup, and every wave streams its activations straight from global memory
// into MFMA B fragments (lane (p, q) loads the 16 bytes of channels [8q, 8q+8) of its pixel's tap:
// 16 pixels x 64 contiguous bytes per instruction for Cin = 32), double-buffered in registers.
// A persistent grid walks 64-pixel tiles per wave, so the weights are read from L2 once per
// workgroup, not once per tile.
//
// Fused 1x1 tail (va_conv_args.w2, TAIL): a wave holds all Cout = 16*TNS activations of its 64 pixels,
// lane (p, q) channels 16i + 4q + r of pixel p.  The tail GEMM contracts over channels in any order,
// so its K fragment kf takes each lane's own 8 values {16(2kf) + 4q + r} u {16(2kf+1) + 4q + r} as
// k = 32kf + 8q + e, and the tail weights are read in that same order (two 8-byte loads per
// fragment): no LDS, no cross-lane traffic, no store of the intermediate layer.
constexpr int DN_TAIL_C2F = 4;  // tail c2 <= 64

// W8: the weights are e4m3 bytes (va_conv_args.w8), converted exactly to bf16 as they are staged into LDS; the
// accumulators are multiplied by their output channel's scale before the bias
template <int TNS, bool TAIL, typename OutT, bool W8 = false>
__global__ __launch_bounds__(256) void conv_dn_kernel(va_conv_args a, int wstride, int ntiles) {
    extern __shared__ __align__(16) __bf16 wsh[];  // [16*TNS][wstride]
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int fr = lane & 15, fq = lane >> 4;
    const __bf16* __restrict__ X = (const __bf16*)a.x;
    // weights -> LDS (rows beyond Cout are zero in the packed matrix: Npad >= 16*TNS)
    const int chunks = a.Kpad / 8;
    for (int i0 = tid; i0 < 16 * TNS * chunks; i0 += 8 * 256) {  // 8 loads in flight per thread
        u32x4 v[8];
        uint2 v8[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int i = i0 + u * 256;
            if (i < 16 * TNS * chunks) {
                const int r = i / chunks, c = i - r * chunks;
                if constexpr (W8)
                    v8[u] = *(const uint2*)((const uint8_t*)a.w + (int64_t)r * a.Kpad + 8 * w8_pos(c));
                else
                    v[u] = *(const u32x4*)((const __bf16*)a.w + (int64_t)r * a.Kpad + 8 * c);
            }
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int i = i0 + u * 256;
            if (i < 16 * TNS * chunks) {
                const int r = i / chunks, c = i - r * chunks;
                if constexpr (W8)
                    *(u32x4*)(wsh + r * wstride + 8 * c) = e4m3x8_bf16(v8[u]);
                else
                    *(u32x4*)(wsh + r * wstride + 8 * c) = v[u];
            }
        }
    }
    __syncthreads();
    float4 wsc[TNS];  // W8: the weights' scale of output channels 16 i + 4 fq ..
#pragma unroll
    for (int i = 0; i < TNS; ++i)
        wsc[i] = W8 ? *(const float4*)(a.wscale + 16 * i + 4 * fq) : make_float4(1.f, 1.f, 1.f, 1.f);
    const int nkf = a.Kpad / 32;
    constexpr int TKF = TAIL ? TNS / 2 : 1;
    bf16x8 w2f[DN_TAIL_C2F][TKF];
    if constexpr (TAIL) {
        static_assert(TNS % 2 == 0, "tail K fragments pair the 16-channel groups");
        const __bf16* W2 = (const __bf16*)a.w2;
#pragma unroll
        for (int c = 0; c < DN_TAIL_C2F; ++c)
#pragma unroll
            for (int kf = 0; kf < TKF; ++kf) {
                const __bf16* r = W2 + (16 * c + fr) * (16 * TNS) + 32 * kf + 4 * fq;
                const uint2 lo = 16 * c < a.c2 ? *(const uint2*)r : make_uint2(0u, 0u);
                const uint2 hi = 16 * c < a.c2 ? *(const uint2*)(r + 16) : make_uint2(0u, 0u);
                w2f[c][kf] = __builtin_bit_cast(bf16x8, (u32x4){lo.x, lo.y, hi.x, hi.y});
            }
    }
    for (int tile = blockIdx.x * 4 + wid; tile < ntiles; tile += gridDim.x * 4) {
        const int m0 = tile * 64;
        int hi0[4], wi0[4];
        int64_t base[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int m = m0 + 16 * j + fr;
            if (m < a.M) {
                const int wo = m % a.Wo, t = m / a.Wo, ho = t % a.Ho, n = t / a.Ho;
                hi0[j] = ho * a.stride - a.pad;
                wi0[j] = wo * a.stride - a.pad;
                base[j] = (int64_t)n * a.H * a.W;
            } else {
                hi0[j] = -(1 << 28);
                wi0[j] = 0;
                base[j] = 0;
            }
        }
        f32x4 acc[4][TNS];
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int i = 0; i < TNS; ++i) acc[j][i] = (f32x4){0.f, 0.f, 0.f, 0.f};
        // k of this lane for K-fragment kf: 32 kf + 8 fq -> (ky, kx, ci), advanced incrementally
        int ci = 8 * fq, ky = 0, kx = 0;
        while (ci >= a.Cin) {
            ci -= a.Cin;
            if (++kx == a.kw) {
                kx = 0;
                ++ky;
            }
        }
        int kcur = 8 * fq;
        u32x4 bcur[4], bnxt[4];
#define DN_LOAD(dst)                                                                                              \
    {                                                                                                             \
        const bool kin = kcur < a.K;                                                                              \
        _Pragma("unroll") for (int j = 0; j < 4; ++j) {                                                           \
            const int hi = hi0[j] + ky, wi = wi0[j] + kx;                                                         \
            const bool ok = kin && (unsigned)hi < (unsigned)a.H && (unsigned)wi < (unsigned)a.W;                  \
            const int64_t off = ok ? (base[j] + (int64_t)hi * a.W + wi) * a.ldx + ci : 0;                        \
            const u32x4 v = *(const u32x4*)(X + off);                                                             \
            dst[j] = ok ? v : (u32x4){0u, 0u, 0u, 0u};                                                            \
        }                                                                                                         \
        kcur += 32;                                                                                               \
        ci += 32;                                                                                                 \
        while (ci >= a.Cin) {                                                                                     \
            ci -= a.Cin;                                                                                          \
            if (++kx == a.kw) {                                                                                   \
                kx = 0;                                                                                           \
                ++ky;                                                                                             \
            }                                                                                                     \
        }                                                                                                         \
    }
        DN_LOAD(bcur);
        for (int kf = 0; kf < nkf; ++kf) {
            if (kf + 1 < nkf) DN_LOAD(bnxt);
            bf16x8 af[TNS];
#pragma unroll
            for (int i = 0; i < TNS; ++i) af[i] = *(const bf16x8*)(wsh + (16 * i + fr) * wstride + 32 * kf + 8 * fq);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const bf16x8 bfr = __builtin_bit_cast(bf16x8, bcur[j]);
#pragma unroll
                for (int i = 0; i < TNS; ++i)
                    acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr, acc[j][i], 0, 0, 0);
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) bcur[j] = bnxt[j];
        }
#undef DN_LOAD
        if constexpr (TAIL) {
            float4 bv[TNS];
#pragma unroll
            for (int i = 0; i < TNS; ++i) bv[i] = *(const float4*)(a.bias + 16 * i + 4 * fq);
            f32x4 acc2[4][DN_TAIL_C2F];
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int c = 0; c < DN_TAIL_C2F; ++c) acc2[j][c] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int kf = 0; kf < TKF; ++kf)
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    bf16x8 b;
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        const int i = 2 * kf + h;
                        float v[4] = {acc[j][i][0] * wsc[i].x + bv[i].x, acc[j][i][1] * wsc[i].y + bv[i].y,
                                      acc[j][i][2] * wsc[i].z + bv[i].z, acc[j][i][3] * wsc[i].w + bv[i].w};
                        if (a.act) silu_n(v);
#pragma unroll
                        for (int r = 0; r < 4; ++r) b[4 * h + r] = (__bf16)v[r];
                    }
#pragma unroll
                    for (int c = 0; c < DN_TAIL_C2F; ++c)
                        acc2[j][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w2f[c][kf], b, acc2[j][c], 0, 0, 0);
                }
            OutT* Y2 = (OutT*)a.y;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int m = m0 + 16 * j + fr;
                if (m >= a.M) continue;
#pragma unroll
                for (int c = 0; c < DN_TAIL_C2F; ++c) {
                    const int co = 16 * c + 4 * fq;
                    if (co >= a.c2) continue;
                    const float4 b2 = *(const float4*)(a.b2 + co);
                    float v[4] = {acc2[j][c][0] + b2.x, acc2[j][c][1] + b2.y, acc2[j][c][2] + b2.z,
                                  acc2[j][c][3] + b2.w};
                    if (a.act2) {
                        silu_n(v);
                    }
                    OutT* yp = Y2 + (int64_t)m * a.ldy + co;
                    if constexpr (sizeof(OutT) == 2) {
                        __bf16 o4[4] = {(__bf16)v[0], (__bf16)v[1], (__bf16)v[2], (__bf16)v[3]};
                        *(uint2*)yp = *(uint2*)o4;
                    } else {
                        *(float4*)yp = make_float4(v[0], v[1], v[2], v[3]);
                    }
                }
            }
            continue;
        }
        __bf16* Y = (__bf16*)a.y;
        const __bf16* R = (const __bf16*)a.res;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int m = m0 + 16 * j + fr;
            if (m >= a.M) continue;
#pragma unroll
            for (int i = 0; i < TNS; ++i) {
                const int co = 16 * i + 4 * fq;
                if (co >= a.Cout) continue;
                const float4 bv = *(const float4*)(a.bias + co);
                float v[4] = {acc[j][i][0] * wsc[i].x + bv.x, acc[j][i][1] * wsc[i].y + bv.y,
                              acc[j][i][2] * wsc[i].z + bv.z, acc[j][i][3] * wsc[i].w + bv.w};
                if (a.act) {
                    silu_n(v);
                }
                if (R) {
                    const uint2 rr = *(const uint2*)(R + (int64_t)m * a.ldr + co);
                    const __bf16* rp = (const __bf16*)&rr;
#pragma unroll
                    for (int r = 0; r < 4; ++r) v[r] += (float)rp[r];
                }
                __bf16 o4[4] = {(__bf16)v[0], (__bf16)v[1], (__bf16)v[2], (__bf16)v[3]};
                *(uint2*)(Y + (int64_t)m * a.ldy + co) = *(uint2*)o4;
            }
        }
    }
}

// ----------------------------------------------------------------------------------------- patch conv
// Narrow stride-1 3x3 convs (Cout 32 / 64, Cin 32 / 64: the C2f bottlenecks of P2/P3 and the head's box /
// coefficient branches).  The im2col kernels fetch every input pixel nine times through L2 (once per tap)
// and are latency-bound on those gathers; here, per 16 x 16 output tile, the 18 x 18-pixel input patch is
// staged ONCE into LDS by LDS-DMA and all nine taps read their B fragments from it, while the whole weight
// matrix stays in LDS for the launch.  Persistent workgroups walk the tiles with two patch buffers: the
// next tile's patch streams in while the current one is computed.  4 waves, wave w = output rows
// 4w .. 4w+3 (four 16-pixel MFMA fragments) x all Cout; no barrier inside a tile.
//
// Patch image: pixel p (row-major in the 18 x 18 patch) holds its Cin channels as CPP = Cin/8 16-byte
// chunks; chunk c of pixel p sits in slot c ^ swz(p) of the pixel's CPP slots, swz(p) = p & 7 (CPP 8) or
// (p ^ p >> 1) & 3 (CPP 4): conflict-free for every tap offset under ds_read_b128's lane groups
// ({0-3, 12-15, 20-27}, ... MI355X_MICROARCH.md §LDS: a group mixes two chunks of 16 pixels).  A DMA
// instruction writes 1 KiB lane-linearly; lane l fetches the chunk its slot holds (the XOR is an
// involution).  Weight rows are padded by 32 bytes: the A-fragment reads are conflict-free too.
constexpr int PT = 16;  // output tile edge
constexpr int PW3 = PT + 2;

template <int CPP>
__device__ __forceinline__ int patch_swz(int p) {
    return CPP == 8 ? (p & 7) : ((p ^ (p >> 1)) & 3);
}
template <int CPP>
__device__ __forceinline__ int patch_off(int p, int c) {
    return p * (CPP * 16) + 16 * (c ^ patch_swz<CPP>(p));
}

// W8 (va_conv_args.w8): e4m3 weight bytes, converted exactly to bf16 as the weight matrix is staged into LDS, the
// accumulators times their channel's scale before the bias
template <int TNS, int CPP, bool TAIL, typename OutT, int NW, int ABL = 0, bool W8 = false>  // NW waves; ABL: diagnosis
__global__ __launch_bounds__(64 * NW) void conv_patch_kernel(va_conv_args a, int wstride, int tiles_x, int tiles_y,
                                                             int ntiles, int patch_bytes) {
    constexpr int NT = 64 * NW, RPW = PT / NW;       // threads, output rows (16-pixel fragments) per wave
    constexpr int NKS = 9 * CPP / 4;               // 32-deep K steps: 9 taps x Cin / 32
    constexpr int PPI = 64 / CPP;                   // patch pixels per DMA instruction
    constexpr int NI = (PW3 * PW3 + PPI - 1) / PPI; // DMA instructions per patch
    extern __shared__ __align__(16) unsigned char smemp[];
    __bf16* wsh = (__bf16*)smemp;                              // [16*TNS][wstride]
    unsigned char* pbuf = smemp + 16 * TNS * wstride * 2;     // 2 x patch_bytes
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int fr = lane & 15, fq = lane >> 4;
    const __bf16* __restrict__ X = (const __bf16*)a.x;

    auto stage_patch = [&](int tile, unsigned char* dst) {
        const int tx = tile % tiles_x, t2 = tile / tiles_x, ty = t2 % tiles_y, n = t2 / tiles_y;
        const int iy0 = PT * ty - 1, ix0 = PT * tx - 1;
        for (int i = wid; i < NI; i += NW) {
            const int off = i * 1024 + 16 * lane;
            const int p = off / (CPP * 16), slot = (off / 16) % CPP;
            const int c = slot ^ patch_swz<CPP>(p);
            const int iy = iy0 + p / PW3, ix = ix0 + p % PW3;
            const bool ok = p < PW3 * PW3 && (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W;
            const void* src = ok ? (const void*)(X + (((int64_t)n * a.H + iy) * a.W + ix) * a.ldx + 8 * c)
                                 : (const void*)g_zero_page;
            __builtin_amdgcn_global_load_lds((gvoid_t*)src, (lvoid_t*)(dst + i * 1024), 16, 0, 0);
        }
    };

    int tile = blockIdx.x;
    if (tile < ntiles) stage_patch(tile, pbuf);
    // weights -> LDS once, rows permuted so that MFMA fragments 2p and 2p + 1 give each lane 8 consecutive
    // output channels (one 16-byte store): LDS row 16 i + r holds channel 32 (i/2) + 8 (r/4) + 4 (i%2) + r%4
    static_assert(TNS % 2 == 0, "fragments pair up");
    // (batches of 8 loads in flight per thread: a load -> store loop would wait out one L2 round trip per chunk)
    const int chunks = NKS * 4;
    for (int i0 = tid; i0 < 16 * TNS * chunks; i0 += 8 * NT) {
        u32x4 v[8];
        uint2 v8[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int i = i0 + u * NT;
            if (i < 16 * TNS * chunks) {
                const int r = i / chunks, c = i - r * chunks;
                const int fi = r / 16, rr = r % 16;
                const int ch = 32 * (fi / 2) + 8 * (rr / 4) + 4 * (fi % 2) + rr % 4;
                if constexpr (W8)
                    v8[u] = *(const uint2*)((const uint8_t*)a.w + (int64_t)ch * a.Kpad + 8 * w8_pos(c));
                else
                    v[u] = *(const u32x4*)((const __bf16*)a.w + (int64_t)ch * a.Kpad + 8 * c);
            }
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int i = i0 + u * NT;
            if (i < 16 * TNS * chunks) {
                const int r = i / chunks, c = i - r * chunks;
                if constexpr (W8)
                    *(u32x4*)(wsh + r * wstride + 8 * c) = e4m3x8_bf16(v8[u]);
                else
                    *(u32x4*)(wsh + r * wstride + 8 * c) = v[u];
            }
        }
    }
    constexpr int TKF = TAIL ? TNS / 2 : 1;
    bf16x8 w2f[TNS][TKF];
    if constexpr (TAIL) {
        // with the row permutation a lane's fragments 2 kf, 2 kf + 1 hold channels 32 kf + 8 fq + (0..7): the
        // tail's K fragment kf in natural order
        const __bf16* W2 = (const __bf16*)a.w2;
#pragma unroll
        for (int c = 0; c < TNS; ++c)
#pragma unroll
            for (int kf = 0; kf < TKF; ++kf)
                w2f[c][kf] = 16 * c < a.c2 ? *(const bf16x8*)(W2 + (16 * c + fr) * (16 * TNS) + 32 * kf + 8 * fq)
                                           : (bf16x8){};
    }
    float4 bv[TNS], sv[TNS];  // bias and (W8) the weights' scale of the lane's channels of fragment i
#pragma unroll
    for (int i = 0; i < TNS; ++i) {
        bv[i] = *(const float4*)(a.bias + 32 * (i / 2) + 8 * fq + 4 * (i % 2));
        sv[i] = W8 ? *(const float4*)(a.wscale + 32 * (i / 2) + 8 * fq + 4 * (i % 2)) : make_float4(1.f, 1.f, 1.f, 1.f);
    }

    for (int it = 0; tile < ntiles; tile += gridDim.x, ++it) {
        unsigned char* cur = pbuf + (it & 1) * patch_bytes;
        // this tile's patch has landed (every wave's DMAs) and every wave is done with the other buffer.  The
        // previous tile's epilogue stores (a fixed NST per wave, issued after that DMA) may stay in flight:
        // vmcnt is in order, so vmcnt(NST) retires the DMA; a raw s_barrier, since __syncthreads() would
        // also drain the stores
        constexpr int NST = TAIL ? RPW * TNS : RPW * TNS / 2;
        static_assert(NST < 64, "vmcnt is 6 bits");
        if (it == 0)
            __builtin_amdgcn_s_waitcnt(0x0070);  // vmcnt(0) expcnt(7) lgkmcnt(0)
        else  // vmcnt(NST): low 4 bits at [3:0], high 2 at [15:14]
            __builtin_amdgcn_s_waitcnt(0x0070 | (NST & 15) | ((NST >> 4) << 14));
        __builtin_amdgcn_s_barrier();
        const int next = tile + gridDim.x;
        if (ABL != 2 && next < ntiles) stage_patch(next, pbuf + ((it + 1) & 1) * patch_bytes);

        f32x4 acc[RPW][TNS];
#pragma unroll
        for (int j = 0; j < RPW; ++j)
#pragma unroll
            for (int i = 0; i < TNS; ++i) acc[j][i] = (f32x4){0.f, 0.f, 0.f, 0.f};
        // fragments are read two steps ahead (three register sets, static indices: the loop is fully
        // unrolled); sched_barrier keeps hipcc from sinking the reads below the MFMAs, which would leave the
        // next step waiting out a whole LDS round trip (lgkmcnt(0)) behind its own reads
        bf16x8 af[3][TNS], bfr[3][RPW];
        auto load_frags = [&](int s, bf16x8(&fa)[TNS], bf16x8(&fb)[RPW]) {
            const int tap = s / (CPP / 4), ky = tap / 3, kx = tap % 3;
            const int c = (s % (CPP / 4)) * 4 + fq;
#pragma unroll
            for (int i = 0; i < TNS; ++i) fa[i] = *(const bf16x8*)(wsh + (16 * i + fr) * wstride + 32 * s + 8 * fq);
#pragma unroll
            for (int j = 0; j < RPW; ++j) {
                const int p = (RPW * wid + j + ky) * PW3 + fr + kx;
                fb[j] = *(const bf16x8*)(cur + patch_off<CPP>(p, c));
            }
        };
        load_frags(0, af[0], bfr[0]);
        load_frags(1, af[1], bfr[1]);
#pragma unroll
        for (int s = 0; s < NKS; ++s) {
            const int b = s % 3;
            if (s + 2 < NKS) load_frags(s + 2, af[(s + 2) % 3], bfr[(s + 2) % 3]);
            __builtin_amdgcn_sched_barrier(0);  // the reads of step s + 2 issue before the MFMAs of step s
            if constexpr (ABL == 1) {
#pragma unroll
                for (int j = 0; j < RPW; ++j) asm volatile("" ::"v"(bfr[b][j]));
#pragma unroll
                for (int i = 0; i < TNS; ++i) asm volatile("" ::"v"(af[b][i]));
                continue;
            }
#pragma unroll
            for (int j = 0; j < RPW; ++j)
#pragma unroll
                for (int i = 0; i < TNS; ++i)
                    acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[b][i], bfr[b][j], acc[j][i], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
        }

        const int tx = tile % tiles_x, t2 = tile / tiles_x, ty = t2 % tiles_y, n = t2 / tiles_y;
        const int ox = PT * tx + fr;
        if constexpr (TAIL) {
            f32x4 acc2[RPW][TNS];
#pragma unroll
            for (int j = 0; j < RPW; ++j)
#pragma unroll
                for (int c = 0; c < TNS; ++c) acc2[j][c] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int kf = 0; kf < TKF; ++kf)
#pragma unroll
                for (int j = 0; j < RPW; ++j) {
                    bf16x8 b;
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        const int i = 2 * kf + h;
                        float v[4] = {acc[j][i][0] * sv[i].x + bv[i].x, acc[j][i][1] * sv[i].y + bv[i].y,
                                      acc[j][i][2] * sv[i].z + bv[i].z, acc[j][i][3] * sv[i].w + bv[i].w};
                        if (a.act) silu_n(v);
#pragma unroll
                        for (int r = 0; r < 4; ++r) b[4 * h + r] = (__bf16)v[r];
                    }
#pragma unroll
                    for (int c = 0; c < TNS; ++c)
                        acc2[j][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w2f[c][kf], b, acc2[j][c], 0, 0, 0);
                }
            OutT* Y2 = (OutT*)a.y;
#pragma unroll
            for (int j = 0; j < RPW; ++j) {
                const int oy = PT * ty + RPW * wid + j;
                const bool pin = oy < a.Ho && ox < a.Wo;
                const int64_t m = pin ? ((int64_t)n * a.Ho + oy) * a.Wo + ox : 0;
#pragma unroll
                for (int c = 0; c < TNS; ++c) {  // every store issues (masked lanes -> g_sink): NST fixed
                    const int co = 16 * c + 4 * fq;
                    const bool ok = pin && co < a.c2;
                    const float4 b2 = ok ? *(const float4*)(a.b2 + co) : make_float4(0.f, 0.f, 0.f, 0.f);
                    float v[4] = {acc2[j][c][0] + b2.x, acc2[j][c][1] + b2.y, acc2[j][c][2] + b2.z,
                                  acc2[j][c][3] + b2.w};
                    if (a.act2) {
                        silu_n(v);
                    }
                    OutT* yp = ok ? Y2 + m * a.ldy + co : (OutT*)(g_sink + 4 * lane);
                    if constexpr (sizeof(OutT) == 2) {
                        __bf16 o4[4] = {(__bf16)v[0], (__bf16)v[1], (__bf16)v[2], (__bf16)v[3]};
                        *(uint2*)yp = *(uint2*)o4;
                    } else {
                        *(float4*)yp = make_float4(v[0], v[1], v[2], v[3]);
                    }
                }
            }
            continue;
        }
        __bf16* Y = (__bf16*)a.y;
        const __bf16* R = (const __bf16*)a.res;
        if (ABL == 3) {
#pragma unroll
            for (int j = 0; j < RPW; ++j)
#pragma unroll
                for (int i = 0; i < TNS; ++i) asm volatile("" ::"v"(acc[j][i]));
            continue;
        }
        // residuals first (one wait for all of them: beside the in-flight patch DMA hipcc drains vmcnt to 0
        // at the first use of a plain load), then bias / SiLU / add and the stores
        bf16x8 rsd[RPW][TNS / 2];
        int64_t mrow[RPW];
        bool pin[RPW];
#pragma unroll
        for (int j = 0; j < RPW; ++j) {
            const int oy = PT * ty + RPW * wid + j;
            pin[j] = oy < a.Ho && ox < a.Wo;  // masked lanes still store (to g_sink): NST fixed
            mrow[j] = pin[j] ? ((int64_t)n * a.Ho + oy) * a.Wo + ox : 0;
            if (R) {
#pragma unroll
                for (int q = 0; q < TNS / 2; ++q)
                    rsd[j][q] = *(const bf16x8*)(pin[j] ? (const void*)(R + mrow[j] * a.ldr + 32 * q + 8 * fq)
                                                        : (const void*)g_zero_page);
            }
        }
#pragma unroll
        for (int j = 0; j < RPW; ++j) {
#pragma unroll
            for (int q = 0; q < TNS / 2; ++q) {
                const int co = 32 * q + 8 * fq;  // 8 consecutive channels: fragments 2q (first 4), 2q + 1
                float v[8];
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const f32x4 t = acc[j][2 * q + h];
                    const float4 b4 = bv[2 * q + h], s4 = sv[2 * q + h];
                    v[4 * h] = t[0] * s4.x + b4.x;
                    v[4 * h + 1] = t[1] * s4.y + b4.y;
                    v[4 * h + 2] = t[2] * s4.z + b4.z;
                    v[4 * h + 3] = t[3] * s4.w + b4.w;
                }
                if (a.act) {
                    silu_n(v);
                }
                if (R) {
#pragma unroll
                    for (int r = 0; r < 8; ++r) v[r] += (float)rsd[j][q][r];
                }
                bf16x8 o;
#pragma unroll
                for (int r = 0; r < 8; ++r) o[r] = (__bf16)v[r];
                *(bf16x8*)(pin[j] ? (void*)(Y + mrow[j] * a.ldy + co) : (void*)(g_sink + 4 * lane)) = o;
            }
        }
    }
}

template <int TNS, bool TAIL, typename OutT, bool W8>
hipError_t launch_conv_dn_w(const va_conv_args& a, hipStream_t st) {
    const int wstride = a.Kpad + 8;  // +16 bytes per row: A-fragment reads spread over the banks
    const size_t lds = (size_t)16 * TNS * wstride * 2;
    static DevFlag attr;
    if (!attr()) {
        if (hipFuncSetAttribute((const void*)conv_dn_kernel<TNS, TAIL, OutT, W8>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) != hipSuccess)
            return hipErrorInvalidValue;
        attr() = true;
    }
    const int ntiles = (a.M + 63) / 64;
    int blocks = (ntiles + 3) / 4;
    const int cap = 256 * (lds <= 40 * 1024 ? 4 : lds <= 80 * 1024 ? 2 : 1);  // resident workgroups
    if (blocks > cap) blocks = cap;
    hipLaunchKernelGGL((conv_dn_kernel<TNS, TAIL, OutT, W8>), dim3(blocks), dim3(256), lds, st, a, wstride, ntiles);
    return hipGetLastError();
}

template <int TNS, bool TAIL = false, typename OutT = __bf16>
hipError_t launch_conv_dn(const va_conv_args& a, hipStream_t st) {
    return a.w8 ? launch_conv_dn_w<TNS, TAIL, OutT, true>(a, st) : launch_conv_dn_w<TNS, TAIL, OutT, false>(a, st);
}

// ----------------------------------------------------------------------------------------- layer 0, f32
// Exact-f32 model.0 with the preprocessing folded in (va355.h va_seg_conv0_f32): one output pixel per lane;
// its 27 inputs (3x3 taps x RGB / 255, zero padding) in registers, every weight a wave-uniform scalar load, so
// the layer is 27 v_fma per output channel.  The results go through LDS: each lane parks its pixel's NCO floats,
// then the wave writes its 64 consecutive pixels as whole 16-byte runs by consecutive lanes (a lane storing its
// own pixel's 128 bytes would put 64 scattered 16-byte pieces in every store instruction) -- the layer is bound
// by that f32 output write (128 B per pixel at Cout 32).
template <int NCO>
__global__ __launch_bounds__(256) void conv0_f32_kernel(const uint8_t* __restrict__ frames, int N, int H, int W,
                                                        const float* __restrict__ w, const float* __restrict__ bias,
                                                        float* __restrict__ y, int ldy) {
    constexpr int RS = NCO + 4;  // LDS row (floats): +4 staggers the 64 rows over the banks
    __shared__ __align__(16) float stage[4][64 * RS];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    float* sw = stage[wid];
    const int Ho = (H + 1) / 2, Wo = (W + 1) / 2;
    const int64_t total = (int64_t)N * Ho * Wo;
    const int64_t nwave = (int64_t)gridDim.x * 4;
    for (int64_t m0 = ((int64_t)blockIdx.x * 4 + wid) * 64; m0 < total; m0 += nwave * 64) {  // wave-uniform
        const int64_t m = m0 + lane;
        if (m < total) {
            const int wo = (int)(m % Wo);
            const int64_t t = m / Wo;
            const int ho = (int)(t % Ho), n = (int)(t / Ho);
            float x[27];
#pragma unroll
            for (int ky = 0; ky < 3; ++ky) {
                const int hi = 2 * ho - 1 + ky;
#pragma unroll
                for (int kx = 0; kx < 3; ++kx) {
                    const int wi = 2 * wo - 1 + kx;
                    const bool in = (unsigned)hi < (unsigned)H && (unsigned)wi < (unsigned)W;
                    const uint8_t* p = frames + (((int64_t)n * H + (in ? hi : 0)) * W + (in ? wi : 0)) * 3;
#pragma unroll
                    for (int c = 0; c < 3; ++c)  // R, G, B = bytes 2, 1, 0
                        x[(ky * 3 + kx) * 3 + c] = in ? (float)p[2 - c] / 255.0f : 0.0f;
                }
            }
#pragma unroll
            for (int co = 0; co < NCO; co += 4) {
                float v[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float* wr = w + (co + r) * 27;
                    float acc = 0.0f;
#pragma unroll
                    for (int k = 0; k < 27; ++k) acc = fmaf(wr[k], x[k], acc);
                    v[r] = silu_exact(acc + bias[co + r]);
                }
                *(float4*)(sw + lane * RS + co) = make_float4(v[0], v[1], v[2], v[3]);
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // the wave's 64 pixels x NCO floats: 16-byte run c of pixel p by lane (p * NCO / 4 + c) % 64
        constexpr int RUNS = NCO / 4;
        for (int i = lane; i < 64 * RUNS; i += 64) {
            const int p = i / RUNS, c = i - p * RUNS;
            if (m0 + p < total) *(float4*)(y + (m0 + p) * ldy + 4 * c) = *(const float4*)(sw + p * RS + 4 * c);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
    }
}

// ----------------------------------------------------------------------------------------- layer 0
// model.0 fused with preprocessing: uint8 BGR frame -> RGB/255 -> Conv(3x3, s2, p1) + folded BN + SiLU
// -> bf16 NHWC.  K = 3x3x3 = 27 (padded to one 32-deep MFMA step), so instead of materialising an
// 8-channel bf16 copy of the frame (16 B/pixel written + read again) each workgroup stages its
// 17 x 129 x 3-byte input patch in LDS and builds the B fragments straight from it.
// Tile: 8 output rows x 64 output columns, 4 waves x 2 rows; weights [Cout][32] bf16 (k = (ky*3+kx)*3 + c,
// c in R, G, B order) stay in registers as the MFMA A operand.
constexpr int C0_TH = 8, C0_TW = 64;
constexpr int C0_PR = 2 * C0_TH + 1;
// patch rows hold frame bytes [6 ox0 - 16, 6 ox0 + 384): 16-byte aligned (W * 3 and 6 * C0_TW are
// multiples of 16), so every 16-byte chunk is wholly inside or wholly outside the frame row; the
// first window pixel (ix0 = 2 ox0 - 1) sits at byte 13
constexpr int C0_PP = 400, C0_OFF = 13;

// OUT8: e4m3 output sat(y * yscale) (the fp8 mode's activation buffers), else bf16
template <int NCO, bool OUT8 = false>
__global__ __launch_bounds__(256) void conv0_kernel(const uint8_t* __restrict__ frames, int N, int H, int W,
                                                    const __bf16* __restrict__ w, const float* __restrict__ bias,
                                                    void* __restrict__ yv, int ldy, float yscale = 0.0f) {
    __bf16* __restrict__ y = (__bf16*)yv;
    __shared__ __align__(16) uint8_t patch[C0_PR * C0_PP];
    const int Ho = (H + 1) / 2, Wo = (W + 1) / 2;
    const int tx = blockIdx.x, ty = blockIdx.y, n = blockIdx.z;
    const int ox0 = tx * C0_TW, oy0 = ty * C0_TH;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const uint8_t* img = frames + (int64_t)n * H * W * 3;
    const int iy0 = 2 * oy0 - 1, rb0 = 6 * ox0 - 16;
    for (int i = tid; i < C0_PR * (C0_PP / 16); i += 256) {
        const int r = i / (C0_PP / 16), c = i - r * (C0_PP / 16);
        const int iy = iy0 + r, rb = rb0 + 16 * c;
        u32x4 v = {0u, 0u, 0u, 0u};
        if ((unsigned)iy < (unsigned)H && rb >= 0 && rb < 3 * W) v = *(const u32x4*)(img + (int64_t)iy * W * 3 + rb);
        *(u32x4*)(patch + r * C0_PP + 16 * c) = v;
    }
    const int fr = lane & 15, fq = lane >> 4;
    // A fragments (weights), rows permuted so that a lane's two 4-channel results of fragments 2p and
    // 2p + 1 are 8 consecutive channels (one 16-byte store): fragment i, row r -> channel
    // 32 (i / 2) + 8 (r / 4) + 4 (i % 2) + r % 4; k = 8 fq .. 8 fq + 7
    bf16x8 af[NCO];
#pragma unroll
    for (int i = 0; i < NCO; ++i) {
        const int co = (NCO % 2 == 0 || i < NCO - 1) ? 32 * (i / 2) + 8 * (fr / 4) + 4 * (i % 2) + fr % 4 : 16 * i + fr;
        af[i] = *(const bf16x8*)(w + co * 32 + 8 * fq);
    }
    // this lane's 8 k values -> patch byte offsets (relative to the pixel's window corner); -1 = K padding
    int koff[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const int k = 8 * fq + e;
        if (k < 27) {
            const int tap = k / 3, c = k % 3;  // c: 0 = R, 1 = G, 2 = B; the frame is BGR
            koff[e] = (tap / 3) * C0_PP + (tap % 3) * 3 + (2 - c);
        } else {
            koff[e] = -1;
        }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 8; ++j) {  // 8 subtiles of 16 pixels per wave: rows 2*wid, 2*wid+1
        const int rl = 2 * wid + (j >> 2), cl = (j & 3) * 16 + fr;
        const int base = (2 * rl) * C0_PP + C0_OFF + 6 * cl;
        // x * (1/255) instead of x / 255 (no f32 division): the bf16 results agree for all 256 byte values
        bf16x8 bfr;
#pragma unroll
        for (int e = 0; e < 8; ++e)
            bfr[e] = koff[e] >= 0 ? (__bf16)((float)patch[base + koff[e]] * (1.0f / 255.0f)) : (__bf16)0.0f;
        const int oy = oy0 + rl, ox = ox0 + cl;
        f32x4 acc[NCO];
#pragma unroll
        for (int i = 0; i < NCO; ++i)
            acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr, (f32x4){0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
        if (oy >= Ho || ox >= Wo) continue;
        if constexpr (OUT8) {
            uint8_t* yp8 = (uint8_t*)yv + (((int64_t)n * Ho + oy) * Wo + ox) * ldy;
#pragma unroll
            for (int p = 0; p < NCO / 2; ++p) {
                const int co = 32 * p + 8 * fq;
                const float4 b0 = *(const float4*)(bias + co), b1 = *(const float4*)(bias + co + 4);
                const float v[8] = {silu(acc[2 * p][0] + b0.x),     silu(acc[2 * p][1] + b0.y),
                                    silu(acc[2 * p][2] + b0.z),     silu(acc[2 * p][3] + b0.w),
                                    silu(acc[2 * p + 1][0] + b1.x), silu(acc[2 * p + 1][1] + b1.y),
                                    silu(acc[2 * p + 1][2] + b1.z), silu(acc[2 * p + 1][3] + b1.w)};
                *(uint2*)(yp8 + co) = e4m3_pack8(v, yscale);
            }
            if constexpr (NCO % 2) {
                const int co = 16 * (NCO - 1) + 4 * fq;
                const float4 bv = *(const float4*)(bias + co);
                const f32x4 t = acc[NCO - 1];
                const float v[8] = {silu(t[0] + bv.x), silu(t[1] + bv.y), silu(t[2] + bv.z), silu(t[3] + bv.w),
                                    0.f, 0.f, 0.f, 0.f};
                *(unsigned*)(yp8 + co) = e4m3_pack8(v, yscale).x;
            }
            continue;
        }
        __bf16* yp = y + (((int64_t)n * Ho + oy) * Wo + ox) * ldy;
#pragma unroll
        for (int p = 0; p < NCO / 2; ++p) {
            const int co = 32 * p + 8 * fq;
            const float4 b0 = *(const float4*)(bias + co), b1 = *(const float4*)(bias + co + 4);
            bf16x8 o;
            o[0] = (__bf16)silu(acc[2 * p][0] + b0.x);
            o[1] = (__bf16)silu(acc[2 * p][1] + b0.y);
            o[2] = (__bf16)silu(acc[2 * p][2] + b0.z);
            o[3] = (__bf16)silu(acc[2 * p][3] + b0.w);
            o[4] = (__bf16)silu(acc[2 * p + 1][0] + b1.x);
            o[5] = (__bf16)silu(acc[2 * p + 1][1] + b1.y);
            o[6] = (__bf16)silu(acc[2 * p + 1][2] + b1.z);
            o[7] = (__bf16)silu(acc[2 * p + 1][3] + b1.w);
            *(bf16x8*)(yp + co) = o;
        }
        if constexpr (NCO % 2) {
            const int co = 16 * (NCO - 1) + 4 * fq;
            const float4 bv = *(const float4*)(bias + co);
            const f32x4 t = acc[NCO - 1];
            __bf16 o4[4] = {(__bf16)silu(t[0] + bv.x), (__bf16)silu(t[1] + bv.y), (__bf16)silu(t[2] + bv.z),
                            (__bf16)silu(t[3] + bv.w)};
            *(uint2*)(yp + co) = *(uint2*)o4;
        }
    }
}

// f32 model.0 on the MFMA (va_conv_args.w3 set on the VA_OP_CONV0 op): conv0_kernel's tiling and LDS patch, with
// the weights as three exact bf16 terms h + m + l ([Cout][4][3][8], split3_bf16 of the [Cout][32] K-padded rows) and
// the B operand the raw frame bytes (0..255: exact in bf16), so each fragment pair is three exact term products
// accumulated in f32 (l first) -- sum_k w_k p_k to f32 accuracy -- and the /255 is applied to the sum: the same
// value as the reference's conv of x / 255 up to f32 rounding.  Epilogue: bias, SiLU (the f32 convs' silu2), f32
// NHWC out, 8 consecutive channels (two 16-byte stores) per lane and fragment pair.  Replaces conv0_f32_kernel's
// 27 v_fma per channel and pixel (VALU-bound).
template <int NCO>
__global__ __launch_bounds__(256) void conv0_f32m_kernel(const uint8_t* __restrict__ frames, int N, int H, int W,
                                                         const __bf16* __restrict__ w3, const float* __restrict__ bias,
                                                         float* __restrict__ y, int ldy) {
    __shared__ __align__(16) uint8_t patch[C0_PR * C0_PP];
    const int Ho = (H + 1) / 2, Wo = (W + 1) / 2;
    const int tx = blockIdx.x, ty = blockIdx.y, n = blockIdx.z;
    const int ox0 = tx * C0_TW, oy0 = ty * C0_TH;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const uint8_t* img = frames + (int64_t)n * H * W * 3;
    const int iy0 = 2 * oy0 - 1, rb0 = 6 * ox0 - 16;
    for (int i = tid; i < C0_PR * (C0_PP / 16); i += 256) {
        const int r = i / (C0_PP / 16), c = i - r * (C0_PP / 16);
        const int iy = iy0 + r, rb = rb0 + 16 * c;
        u32x4 v = {0u, 0u, 0u, 0u};
        if ((unsigned)iy < (unsigned)H && rb >= 0 && rb < 3 * W) v = *(const u32x4*)(img + (int64_t)iy * W * 3 + rb);
        *(u32x4*)(patch + r * C0_PP + 16 * c) = v;
    }
    const int fr = lane & 15, fq = lane >> 4;
    // fragment i, row r -> channel 32 (i / 2) + 8 (r / 4) + 4 (i % 2) + r % 4 (conv0_kernel's permutation)
    bf16x8 af[NCO][3];
#pragma unroll
    for (int i = 0; i < NCO; ++i) {
        const int co = (NCO % 2 == 0 || i < NCO - 1) ? 32 * (i / 2) + 8 * (fr / 4) + 4 * (i % 2) + fr % 4 : 16 * i + fr;
#pragma unroll
        for (int p = 0; p < 3; ++p) af[i][p] = *(const bf16x8*)(w3 + ((co * 4 + fq) * 3 + p) * 8);
    }
    int koff[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const int k = 8 * fq + e;
        if (k < 27) {
            const int tap = k / 3, c = k % 3;  // c: 0 = R, 1 = G, 2 = B; the frame is BGR
            koff[e] = (tap / 3) * C0_PP + (tap % 3) * 3 + (2 - c);
        } else {
            koff[e] = -1;
        }
    }
    __syncthreads();
    constexpr float inv255 = 1.0f / 255.0f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int rl = 2 * wid + (j >> 2), cl = (j & 3) * 16 + fr;
        const int base = (2 * rl) * C0_PP + C0_OFF + 6 * cl;
        bf16x8 bfr;
#pragma unroll
        for (int e = 0; e < 8; ++e) bfr[e] = koff[e] >= 0 ? (__bf16)(float)patch[base + koff[e]] : (__bf16)0.0f;
        const int oy = oy0 + rl, ox = ox0 + cl;
        f32x4 acc[NCO];
#pragma unroll
        for (int i = 0; i < NCO; ++i) {
            acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][2], bfr, (f32x4){0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
            acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][1], bfr, acc[i], 0, 0, 0);
            acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][0], bfr, acc[i], 0, 0, 0);
        }
        if (oy >= Ho || ox >= Wo) continue;
        float* yp = y + (((int64_t)n * Ho + oy) * Wo + ox) * ldy;
#pragma unroll
        for (int p = 0; p < NCO / 2; ++p) {
            const int co = 32 * p + 8 * fq;
            const float4 b0 = *(const float4*)(bias + co), b1 = *(const float4*)(bias + co + 4);
            const f32x4 lo = fz::act((f32x4){acc[2 * p][0] * inv255 + b0.x, acc[2 * p][1] * inv255 + b0.y,
                                             acc[2 * p][2] * inv255 + b0.z, acc[2 * p][3] * inv255 + b0.w});
            const f32x4 hi = fz::act((f32x4){acc[2 * p + 1][0] * inv255 + b1.x, acc[2 * p + 1][1] * inv255 + b1.y,
                                             acc[2 * p + 1][2] * inv255 + b1.z, acc[2 * p + 1][3] * inv255 + b1.w});
            *(f32x4*)(yp + co) = lo;
            *(f32x4*)(yp + co + 4) = hi;
        }
        if constexpr (NCO % 2) {
            const int co = 16 * (NCO - 1) + 4 * fq;
            const float4 bv = *(const float4*)(bias + co);
            const f32x4 t = acc[NCO - 1];
            *(f32x4*)(yp + co) =
                fz::act((f32x4){t[0] * inv255 + bv.x, t[1] * inv255 + bv.y, t[2] * inv255 + bv.z, t[3] * inv255 + bv.w});
        }
    }
}

// Work-queue schedule of the persistent kernels (conv3q, the f32 stem): tiles claimed from a counter of the plan
// (va_conv_args.wcnt[0]) instead of fz::tile's static schedule, so that workgroups that start late (CUs held by a
// kernel of another stream: the headline's two network streams overlap) take fewer tiles instead of stretching the
// launch; the last workgroup out (wcnt[1]) zeroes both counters for the next launch of the plan (the split-K
// counters' contract, va355.h).  Headline 4,951-4,969 (static) -> 5,018-5,045 frames/s with conv3q on it
// (profiles/r05/workq/).

// ----------------------------------------------------------------------------------------- f32 stem
// The f32 stem as ONE launch: uint8 BGR frames -> model.0 Conv(3, 32, 3x3, s2) + SiLU (conv0_f32m's arithmetic: the
// three exact bf16 weight terms x the exact frame bytes on the MFMA, the sum x 1/255 + bias, SiLU) -> model.1 Conv(32,
// 64, 3x3, s2) + SiLU (six exact bf16 term products per f32 product, the weights f32 split in registers) -> f32
// NHWC.  Unfused, model.0's 320 x 320 x 32 f32 map (13 MB per 640 x 640 frame) is written and read back; here it
// never leaves the chip.  Persistent: one workgroup per CU walks 4 x 16 tiles of the model.1 map (XCD-contiguous
// runs), each wave holding its share of model.1's weights in registers, split into the three bf16 terms once per
// workgroup; per tile, model.0 on the 9 x 33 pixels the tile's taps read (zero outside model.0's map: model.1's
// padding) straight into LDS as three bf16 planes (exact: h + m + l = the f32 value), then model.1's K-steps (tap x
// 16-channel chunk) from there with no barrier inside the K-loop; the frame patches of the next two tiles are in
// flight in registers while this tile runs.  (A ring of per-K-step weight stages with a barrier per step: 675 us per 64
// frames; the weights in LDS split per K-step: 700-775 us; the two unfused launches ~750 us: profiles/r05/stem/.)
// LDS: model.0 planes 297 px x 208 B (chunk c, plane p, half g at 96 c + 32 p + 16 g: model.1's stride-2 B reads at
// most 2-way bank conflicted), the frame patch 19 rows x 208 B, a 16 KiB buffer for the K-split's partial sums.  8 waves (two per SIMD): wave w computes the 32 pixels x 32 channels block (wm, wn) = ((w & 3) >> 1,
// w & 1) of model.1 over K-steps 9 (w >> 2) .. 9 (w >> 2) + 8, the six term products in two independent accumulator
// chains; waves 4-7 hand their partial sums to waves 0-3 through LDS.  (One wave per SIMD, the whole K-loop per wave:
// 775 us per 64 frames, profiles/r05/stem/.)
constexpr int S32_TH = 4, S32_TW = 16, S32_NT = 512;
constexpr int S32_MR = 2 * S32_TH + 1, S32_MC = 2 * S32_TW + 1, S32_MP = S32_MR * S32_MC;  // 9 x 33 = 297
constexpr int S32_PS = 208;                           // LDS bytes per model.0 pixel
constexpr int S32_PR = 2 * S32_MR + 1, S32_PP = 208;  // frame patch: 19 rows x 208 bytes (13 chunks of 16)
constexpr int S32_M0 = 0, S32_PATCH = S32_M0 + S32_MP * S32_PS;
constexpr int S32_PART = S32_PATCH + S32_PR * S32_PP, S32_LDS = S32_PART + 4 * 64 * 64;
constexpr int S32_NPC = S32_PR * (S32_PP / 16);       // patch chunks (247 <= threads: one per thread)
static_assert(S32_LDS <= 160 * 1024 && S32_NPC <= S32_NT, "LDS / patch chunks");
// TAIL (model.2.cv1, the C2f's 1x1 64 -> 64, fused): the tile's model.1 activations as three bf16 planes (64 pixels x
// 400 bytes: [chunk 4][plane 3][16 channels] + 16 bytes, conflict-free 16-pixel reads) and cv1's weights pre-split
// once per workgroup (64 rows x 400 bytes, the same layout over K)
constexpr int S32_TP = 400, S32_T = S32_LDS, S32_W1 = S32_T + 64 * S32_TP, S32_LDS_T = S32_W1 + 64 * S32_TP;
static_assert(S32_LDS_T <= 160 * 1024, "LDS with the tail");

// DYN: the work-queue schedule (wq_claim; the tiles' frame patches are loaded two tiles ahead, so the claims run two
// ahead too: tile j's index sits in LDS slot j % 3, claimed by thread 0 at the start of the tile three before it,
// written before that tile's partial-sum barrier and read at the start of the tile before j)
template <bool TAIL, bool DYN>
__global__ __launch_bounds__(S32_NT, 1) void stem32_kernel(const uint8_t* __restrict__ frames, int N, int H, int W,
                                                           const __bf16* __restrict__ w03, const float* __restrict__ b0,
                                                           const float* __restrict__ w1, int Kpad,
                                                           const float* __restrict__ b1, float* __restrict__ y, int ldy,
                                                           int tiles_x, int tiles_y, int ntiles,
                                                           const float* __restrict__ wt, const float* __restrict__ bt,
                                                           int* __restrict__ wq) {
    extern __shared__ __align__(16) unsigned char s32[];
    const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int Ho0 = (H + 1) / 2, Wo0 = (W + 1) / 2, Ho1 = (Ho0 + 1) / 2, Wo1 = (Wo0 + 1) / 2;
    volatile int* slot = (volatile int*)(s32 + (TAIL ? S32_LDS_T : S32_LDS));
    int t, nx;  // this tile, the next
    if constexpr (DYN) {
        if (tid == 0) {
            slot[0] = fz::wq_claim(wq, ntiles);
            slot[1] = fz::wq_claim(wq, ntiles);
            slot[2] = fz::wq_claim(wq, ntiles);
        }
        __syncthreads();
        t = __builtin_amdgcn_readfirstlane(slot[0]);
        nx = __builtin_amdgcn_readfirstlane(slot[1]);
    } else {
        t = fz::tile(ntiles, 0);
        nx = fz::tile(ntiles, 1);
    }
    if (t < 0) {
        if constexpr (DYN) {
            if (tid == 0) fz::wq_release(wq);
        }
        return;
    }
    // the frame patch of tile tt: rows 4 oy0 - 3 .., bytes [12 ox0 - 16, 12 ox0 + 192) (16-byte aligned: W * 3 % 16 == 0)
    auto load_patch = [&](int tt) -> u32x4 {
        u32x4 v = {0u, 0u, 0u, 0u};
        if (tt < 0) return v;
        const int tx = tt % tiles_x, t2 = tt / tiles_x, ty = t2 % tiles_y, n = t2 / tiles_y;
        const int r = tid / (S32_PP / 16), c = tid - r * (S32_PP / 16);
        const int iy = 4 * ty * S32_TH - 3 + r, rb = 12 * tx * S32_TW - 16 + 16 * c;
        if (tid < S32_NPC && (unsigned)iy < (unsigned)H && rb >= 0 && rb < 3 * W)
            v = *(const u32x4*)(frames + (int64_t)n * H * W * 3 + (int64_t)iy * W * 3 + rb);
        return v;
    };
    auto store_patch = [&](const u32x4& v) {
        if (tid < S32_NPC) *(u32x4*)(s32 + S32_PATCH + 16 * tid) = v;  // row r, chunk c at r * 208 + 16 c = 16 tid
    };
    store_patch(load_patch(t));
    u32x4 pf1 = load_patch(nx);  // the next two tiles' patches in flight

    const int fr = lane & 15, fq = lane >> 4;
    // model.0 A fragments (conv0_f32m's permutation: fragment i, row r -> channel 8 (r / 4) + 4 i + r % 4, so lane
    // (fr, fq)'s two results are channels 8 fq .. 8 fq + 7 of pixel fr)
    bf16x8 af[2][3];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int co = 8 * (fr / 4) + 4 * i + fr % 4;
#pragma unroll
        for (int p = 0; p < 3; ++p) af[i][p] = *(const bf16x8*)(w03 + ((co * 4 + fq) * 3 + p) * 8);
    }
    int koff[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const int k = 8 * fq + e;
        const int tap = k / 3, c = k % 3;  // c: 0 = R, 1 = G, 2 = B; the frame is BGR
        koff[e] = k < 27 ? (tap / 3) * S32_PP + (tap % 3) * 3 + (2 - c) : -1;
    }
    const float4 bl = *(const float4*)(b0 + 8 * fq), bh = *(const float4*)(b0 + 8 * fq + 4);
    const int wm = (wid & 3) >> 1, wn = wid & 1, kh = wid >> 2, r32 = lane & 31, g32 = lane >> 5;
    const int py = 2 * wm + (r32 >> 4), px = r32 & 15;  // this lane's model.1 pixel in the tile
    float4 bo[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) bo[j] = *(const float4*)(b1 + 32 * wn + 8 * j + 4 * g32);
    // this wave's model.1 weights, split once: row 32 wn + r32, K-steps 9 kh .. 9 kh + 8, f32 k = 16 kl + 8 g32 ..
    bf16x8 apr[9][3];
    {
        const float* wr = w1 + (int64_t)(32 * wn + r32) * Kpad + 8 * g32 + 16 * 9 * kh;
#pragma unroll
        for (int i = 0; i < 9; ++i) split3_bf16(*(const u32x4*)(wr + 16 * i), *(const u32x4*)(wr + 16 * i + 4), apr[i]);
    }
    if constexpr (TAIL) {  // cv1's [64][64] f32 weights: thread -> row tid / 8, K 8 (tid % 8) .. + 7
        const int r = tid >> 3, q = tid & 7;
        const float* src = wt + r * 64 + 8 * q;
        bf16x8 tw[3];
        split3_bf16(*(const u32x4*)src, *(const u32x4*)(src + 4), tw);
        unsigned char* d = s32 + S32_W1 + r * S32_TP + (q >> 1) * 96 + 16 * (q & 1);
#pragma unroll
        for (int p = 0; p < 3; ++p) *(bf16x8*)(d + 32 * p) = tw[p];
    }
    __syncthreads();

    constexpr float inv255 = 1.0f / 255.0f;
    constexpr int TA[6] = {0, 0, 1, 0, 1, 2}, TB[6] = {0, 1, 0, 2, 1, 0};
    for (int k = 1; t >= 0; ++k) {
        const int tx = t % tiles_x, t2 = t / tiles_x, ty = t2 % tiles_y, n = t2 / tiles_y;
        const int oy0 = ty * S32_TH, ox0 = tx * S32_TW;
        const int tn = nx;
        const int tn2 = DYN ? __builtin_amdgcn_readfirstlane(slot[(k + 1) % 3]) : fz::tile(ntiles, k + 1);
        const u32x4 pf2 = load_patch(tn2);  // two tiles ahead
        int cl = 0;  // DYN: the tile three ahead, claimed here and published after the K-loop (the returning atomic's
        if constexpr (DYN) {  // ~1 us lands during model.0 / model.1 instead of stalling wave 0 before a barrier)
            if (tid == 0) cl = fz::wq_claim_raw(wq);
        }

        // ---- model.0 on the 9 x 33 region: group g = 16 region pixels (the last group ragged); region pixel q <->
        // model.0 (2 oy0 - 1 + q / 33, 2 ox0 - 1 + q % 33); its window starts at patch row 2 (q / 33), byte 6 (q % 33) + 7
        for (int g = wid; g < (S32_MP + 15) / 16; g += S32_NT / 64) {
            const int q = 16 * g + fr;
            const int qi = q < S32_MP ? q / S32_MC : 0, qj = q < S32_MP ? q % S32_MC : 0;
            const int base = S32_PATCH + 2 * qi * S32_PP + 6 * qj + 7;
            bf16x8 bfr;
#pragma unroll
            for (int e = 0; e < 8; ++e) bfr[e] = koff[e] >= 0 ? (__bf16)(float)s32[base + koff[e]] : (__bf16)0.0f;
            f32x4 acc[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][2], bfr, (f32x4){0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
                acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][1], bfr, acc[i], 0, 0, 0);
                acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][0], bfr, acc[i], 0, 0, 0);
            }
            const int Y = 2 * oy0 - 1 + qi, X = 2 * ox0 - 1 + qj;
            const bool in = (unsigned)Y < (unsigned)Ho0 && (unsigned)X < (unsigned)Wo0;
            f32x4 lo = fz::act((f32x4){acc[0][0] * inv255 + bl.x, acc[0][1] * inv255 + bl.y, acc[0][2] * inv255 + bl.z,
                                       acc[0][3] * inv255 + bl.w});
            f32x4 hi = fz::act((f32x4){acc[1][0] * inv255 + bh.x, acc[1][1] * inv255 + bh.y, acc[1][2] * inv255 + bh.z,
                                       acc[1][3] * inv255 + bh.w});
            if (!in) lo = hi = (f32x4){0.f, 0.f, 0.f, 0.f};
            bf16x8 tt3[3];
            split3_bf16(__builtin_bit_cast(u32x4, lo), __builtin_bit_cast(u32x4, hi), tt3);
            if (q < S32_MP) {
                unsigned char* d = s32 + S32_M0 + q * S32_PS + (fq >> 1) * 96 + (fq & 1) * 16;
#pragma unroll
                for (int p = 0; p < 3; ++p) *(bf16x8*)(d + 32 * p) = tt3[p];
            }
        }
        __syncthreads();  // M0 complete; every wave is done with the patch
        store_patch(pf1);  // the next tile's patch (read after the barrier that ends this tile)

        // ---- model.1: wave (wm, wn) = pixels 32 wm .. (tile rows 2 wm, 2 wm + 1) x channels 32 wn ..; K-step kl =
        // tap * 2 + chunk, A from the resident weights, B from M0; two accumulator chains (products 0, 2, 4 / 1, 3, 5)
        f32x16 acc0 = (f32x16){}, acc1 = (f32x16){};
#pragma unroll
        for (int i = 0; i < 9; ++i) {
            const int kl = 9 * kh + i, tap = kl >> 1, ch = kl & 1, ky = tap / 3, kx = tap % 3;
            bf16x8 bp[3];
            const unsigned char* bs = s32 + S32_M0 + ((2 * py + ky) * S32_MC + 2 * px + kx) * S32_PS + ch * 96 + 16 * g32;
#pragma unroll
            for (int p = 0; p < 3; ++p) bp[p] = *(const bf16x8*)(bs + 32 * p);
#pragma unroll
            for (int u = 0; u < 6; u += 2) {
                acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(apr[i][TA[u]], bp[TB[u]], acc0, 0, 0, 0);
                acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(apr[i][TA[u + 1]], bp[TB[u + 1]], acc1, 0, 0, 0);
            }
        }
        // ---- K halves: waves 4-7 hand their partial sums to waves 0-3 (lane-ordered, 64 B per lane); TAIL: the two
        // waves of a K pair swap halves instead -- wave kh finishes channel groups j = 2 kh, 2 kh + 1 (16 B each)
        f32x16 a2 = acc0 + acc1;
        f32x16* part = (f32x16*)(s32 + S32_PART + (wid & 3) * 4096) + lane;
        auto quad = [&](int j) { return (f32x4){a2[4 * j], a2[4 * j + 1], a2[4 * j + 2], a2[4 * j + 3]}; };
        if constexpr (TAIL) {
            f32x4* ph = (f32x4*)part;  // the partner's groups (kh is wave-uniform: a scalar branch, constant indices)
            if (kh) {
                ph[0] = quad(0);
                ph[1] = quad(1);
            } else {
                ph[2] = quad(2);
                ph[3] = quad(3);
            }
        } else {
            if (kh) *part = a2;
        }
        if constexpr (DYN) {
            if (tid == 0) slot[(k + 2) % 3] = cl < ntiles ? cl : -1;  // read at iteration k + 1 (last read at k - 2)
        }
        __syncthreads();
        // ---- epilogue: lane (r32, g32) holds channels 32 wn + 8 j + 4 g32 + (0..3) of its pixel, j = 0..3
        const int oy = oy0 + py, ox = ox0 + px;
        if constexpr (TAIL) {
            // model.1's activations -> the T planes (every pixel of the tile: an outside one is finite and unstored);
            // channel c = 32 wn + 8 j + 4 g32 + e sits in chunk c / 16, at byte 2 (c % 16) of each plane's 32 bytes
            {
                // the K half-0 sum + the half-1 sum, as before (wave kh holds half kh of its own groups)
                const f32x4* ph = (const f32x4*)part;
                unsigned char* tp = s32 + S32_T + (32 * wm + r32) * S32_TP + 8 * g32;
                auto finish = [&](auto KHc) {
                    constexpr int KH = decltype(KHc)::value;
#pragma unroll
                    for (int u = 0; u < 2; ++u) {
                        constexpr int J0 = 2 * KH;
                        const int j = J0 + u;
                        const f32x4 mine = quad(j), oth = ph[j];
                        const f32x4 sm = KH ? oth + mine : mine + oth;
                        uint2 tt3[3];
                        split3_bf16x4(fz::act((f32x4){sm[0] + bo[j].x, sm[1] + bo[j].y, sm[2] + bo[j].z,
                                                      sm[3] + bo[j].w}),
                                      tt3);
                        unsigned char* d = tp + (2 * wn + KH) * 96 + 16 * u;
#pragma unroll
                        for (int p = 0; p < 3; ++p) *(uint2*)(d + 32 * p) = tt3[p];
                    }
                };
                if (kh)
                    finish(std::integral_constant<int, 1>{});
                else
                    finish(std::integral_constant<int, 0>{});
            }
            __syncthreads();  // T complete; M0 and the partial sums free for the next tile; its patch stored
            if (!kh) {
                // cv1 (1x1, 64 -> 64): wave (wm, wn) = pixels 32 wm .. x cv1 channels 32 wn ..; K-step j = model.1
                // channels 16 j .. (four steps), A from the W1 planes, B from T; two accumulator chains
                f32x16 c0 = (f32x16){}, c1 = (f32x16){};
                const unsigned char* wa = s32 + S32_W1 + (32 * wn + r32) * S32_TP + 16 * g32;
                const unsigned char* tb = s32 + S32_T + (32 * wm + r32) * S32_TP + 16 * g32;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    bf16x8 ap[3], bp[3];
#pragma unroll
                    for (int p = 0; p < 3; ++p) {
                        ap[p] = *(const bf16x8*)(wa + j * 96 + 32 * p);
                        bp[p] = *(const bf16x8*)(tb + j * 96 + 32 * p);
                    }
#pragma unroll
                    for (int u = 0; u < 6; u += 2) {
                        c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ap[TA[u]], bp[TB[u]], c0, 0, 0, 0);
                        c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ap[TA[u + 1]], bp[TB[u + 1]], c1, 0, 0, 0);
                    }
                }
                if (oy < Ho1 && ox < Wo1) {
                    const f32x16 cs = c0 + c1;
                    float* yp = y + (((int64_t)n * Ho1 + oy) * Wo1 + ox) * ldy + 32 * wn + 4 * g32;
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const float4 bv = *(const float4*)(bt + 32 * wn + 8 * j + 4 * g32);
                        *(f32x4*)(yp + 8 * j) = fz::act((f32x4){cs[4 * j] + bv.x, cs[4 * j + 1] + bv.y,
                                                                 cs[4 * j + 2] + bv.z, cs[4 * j + 3] + bv.w});
                    }
                }
            }
        } else {
            if (!kh && oy < Ho1 && ox < Wo1) {
                a2 = a2 + *part;
                float* yp = y + (((int64_t)n * Ho1 + oy) * Wo1 + ox) * ldy + 32 * wn + 4 * g32;
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    *(f32x4*)(yp + 8 * j) = fz::act((f32x4){a2[4 * j] + bo[j].x, a2[4 * j + 1] + bo[j].y,
                                                             a2[4 * j + 2] + bo[j].z, a2[4 * j + 3] + bo[j].w});
            }
            __syncthreads();  // M0 and the partial sums free for the next tile; its patch stored
        }
        pf1 = pf2;
        t = tn;
        nx = tn2;
    }
    if constexpr (DYN) {
        if (tid == 0) fz::wq_release(wq);  // after this workgroup's last (failed) claim
    }
}

// channels 4 g .. 4 g + 3 (g = 0..7) of a 32-channel plane pixel at p (208-byte pixel rows: [chunk 2][plane 3][16
// channels]): the three planes' 8-byte pieces
__device__ __forceinline__ void cf32_put4(unsigned char* p, int g, const f32x4& v) {
    uint2 t[3];
    split3_bf16x4(v, t);
    unsigned char* d = p + (g >> 2) * 96 + (g & 3) * 8;
#pragma unroll
    for (int q = 0; q < 3; ++q) *(uint2*)(d + 32 * q) = t[q];
}

// ----------------------------------------------------------------------------------------- f32 32-channel 3x3
// The 32 -> 32 channel stride-1 3x3 f32 layers (model.2's bottleneck convs at 160 x 160 in YOLOv8s-seg, block.py
// Bottleneck; the head's cv4.l.1, head.py Segment) with the stem's structure instead of conv2's im2col tiles, which
// re-read every input pixel nine times through L2 and split both operands per K-step: the whole weight matrix
// (32 x 288) is split into its three exact bf16 terms once per workgroup and held in registers, and per 16 x 16
// output tile the 18 x 18 input halo is read once, split once into three bf16 planes in LDS (208 bytes per pixel:
// [chunk 2][plane 3][16 channels], conflict-free 32-pixel reads) and every tap read from there -- no barrier inside
// the K-loop.  Persistent: one 512-thread workgroup per CU walks the tiles (fz::tile, XCD-contiguous runs), the next
// tile's halo in flight in registers during this one's MFMAs.  Wave w computes output rows 4 (w & 3) .. + 3 of the
// tile (two 32-pixel blocks) x 32 channels over K-steps 9 (w >> 2) .. + 8 (tap x 16-channel chunk), the six term
// products per K-step and block on v_mfma_f32_32x32x16_bf16 (the two blocks are the two accumulator chains); the two
// waves of a row pair swap partial sums through LDS, each finishing one block: bias, SiLU and the residual
// (Bottleneck's shortcut), f32 stores.
constexpr int Q3_T = 16, Q3_HW = Q3_T + 2, Q3_HP = Q3_HW * Q3_HW;  // 16 x 16 tile, 18 x 18 = 324-pixel halo
constexpr int Q3_NT = 512, Q3_PS = 208;
constexpr int Q3_NCH = Q3_HP * 8;                    // 16-byte input chunks (4 channels) per halo: 2592
constexpr int Q3_LD = (Q3_NCH + Q3_NT - 1) / Q3_NT;  // per thread: 6
constexpr int Q3_PART = Q3_HP * Q3_PS, Q3_LDS = Q3_PART + 4 * 2 * 64 * 64;  // planes 66 KiB + partial sums 32 KiB
// TAIL: a fused 1x1 tail (the head's cv4.l.2, 32 -> c2 <= 32, after cv4.l.1: va_conv_args.w2 as conv3h's tail
// planes [32][4][3][8]) in the epilogue; its weights re-laid in LDS once per workgroup so that lane (r, g) reads, for
// tail K-step s, the 8 channels 16 s + 4 g + (0..3) and 16 s + 8 + 4 g + (0..3) -- exactly the 8 channels of the
// main conv's accumulator registers j = 2 s, 2 s + 1 of lane (pixel, g): the B operand is the lane's own split
// activations, no exchange between lanes
constexpr int Q3_W2 = Q3_LDS + 16, Q3_LDS_T = Q3_W2 + 32 * 2 * 3 * 32;
static_assert(Q3_LDS_T <= 160 * 1024, "one workgroup per CU");
// RES (no tail, a.res set: model.2's second bottleneck conv): the tile's residual, 256 pixels x 32 channels f32
// (pixel p at 128 p), DMA'd into LDS as the K-loop starts and read by the epilogue -- its HBM latency used to sit
// between the partial-sum barrier and the stores of every tile (model.2.m.0.cv2 982 us against m.0.cv1's 764)
constexpr int Q3_RES = Q3_LDS + 16, Q3_LDS_R = Q3_RES + 256 * 128;
static_assert(Q3_LDS_R <= 160 * 1024, "one workgroup per CU");

template <bool DYN, bool TAIL = false>
__global__ __launch_bounds__(Q3_NT, 1) void conv3q_kernel(va_conv_args a, int tiles_x, int tiles_y, int ntiles) {
    extern __shared__ __align__(16) unsigned char q3[];
    const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const float* __restrict__ x = (const float*)a.x;
    const int H = a.H, W = a.W, ldx = a.ldx;
    // DYN: the claimed tiles, published by thread 0 in two alternating slots, one tile ahead of their use: iteration
    // k reads slot k & 1 (claimed during iteration k - 1's K-loop, or in the prologue) and writes slot (k + 1) & 1
    volatile int* slot = (volatile int*)(q3 + Q3_LDS);
    int t;
    if constexpr (DYN) {
        if (tid == 0) {
            slot[0] = fz::wq_claim(a.wcnt, ntiles);
            slot[1] = fz::wq_claim(a.wcnt, ntiles);
        }
        __syncthreads();
        t = __builtin_amdgcn_readfirstlane(slot[0]);
    } else {
        t = fz::tile(ntiles, 0);
    }
    if (t < 0) {
        if constexpr (DYN) {
            if (tid == 0) fz::wq_release(a.wcnt);
        }
        return;
    }
    // the 18 x 18 input pixels of tile tt (zero outside the image: the conv's padding), 8 chunks of 4 channels each;
    // chunk c = 8 q + g <-> halo pixel q, channels 4 g .. 4 g + 3
    auto load_halo = [&](int tt, u32x4 (&v)[Q3_LD]) {
        int tx = 0, ty = 0, n = 0;
        if (tt >= 0) {
            tx = tt % tiles_x;
            const int t2 = tt / tiles_x;
            ty = t2 % tiles_y;
            n = t2 / tiles_y;
        }
        const float* xn = x + (int64_t)n * H * W * ldx;
#pragma unroll
        for (int i = 0; i < Q3_LD; ++i) {
            const int c = tid + Q3_NT * i, q = c >> 3, g = c & 7;
            const int iy = ty * Q3_T - 1 + q / Q3_HW, ix = tx * Q3_T - 1 + q % Q3_HW;
            v[i] = (u32x4){0u, 0u, 0u, 0u};
            if (tt >= 0 && c < Q3_NCH && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W)
                v[i] = *(const u32x4*)(xn + ((int64_t)iy * W + ix) * ldx + 4 * g);
        }
    };
    u32x4 hv[Q3_LD];
    load_halo(t, hv);

    const int r32 = lane & 31, g32 = lane >> 5, kh = wid >> 2, pb = wid & 3;
    // this wave's weights, split once: row (output channel) r32, K-steps 9 kh .. 9 kh + 8, f32 k = 16 kl + 8 g32 ..
    bf16x8 apr[9][3];
    {
        const float* wr = (const float*)a.w + (int64_t)r32 * a.Kpad + 8 * g32 + 16 * 9 * kh;
#pragma unroll
        for (int i = 0; i < 9; ++i) split3_bf16(*(const u32x4*)(wr + 16 * i), *(const u32x4*)(wr + 16 * i + 4), apr[i]);
    }
    if constexpr (TAIL) {  // piece (row r, K-step s, plane p, half g): two 8-byte runs of the host planes
        if (tid < 32 * 2 * 3 * 2) {
            const int g = tid & 1, p = (tid >> 1) % 3, s = (tid / 6) & 1, r = tid / 12;
            const unsigned char* src = (const unsigned char*)a.w2 + ((r * 4 + 2 * s) * 3 + p) * 16 + 8 * g;
            const uint2 lo = *(const uint2*)src, hi = *(const uint2*)(src + 48);  // group 2 s, group 2 s + 1
            *(u32x4*)(q3 + Q3_W2 + ((r * 2 + s) * 3 + p) * 32 + 16 * g) = (u32x4){lo.x, lo.y, hi.x, hi.y};
        }
    }
    constexpr int TA[6] = {0, 0, 1, 0, 1, 2}, TB[6] = {0, 1, 0, 2, 1, 0};
    const bool pre_res = !TAIL && a.res != nullptr;  // uniform
    // the residual of tile (ty, tx) of image n into RES: DMA i = wid + 8 u (1 KiB, pixels 8 i ..), lane l -> pixel
    // 8 i + (l >> 3), channels 4 (l & 7) ..; pixels outside the image read zeros (never stored)
    auto dma_res = [&](int n, int ty, int tx) {
        const int rb = H * W * a.ldr * 4;
        const float* rn = (const float*)a.res + (int64_t)n * H * W * a.ldr;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int i = wid + 8 * u, p = 8 * i + (lane >> 3), c = lane & 7;
            const int iy = ty * Q3_T + (p >> 4), ix = tx * Q3_T + (p & 15);
            const int vo = iy < H && ix < W ? ((iy * W + ix) * a.ldr + 4 * c) * 4 : 0x7ff00000;
            t3_dma16(rn, rb, q3 + Q3_RES + 1024 * i, vo, 0);
        }
    };
    for (int k = 1; t >= 0; ++k) {
        const int tx = t % tiles_x, t2 = t / tiles_x, ty = t2 % tiles_y, n = t2 / tiles_y;
#pragma unroll
        for (int i = 0; i < Q3_LD; ++i) {
            const int c = tid + Q3_NT * i;
            if (c < Q3_NCH) cf32_put4(q3 + (c >> 3) * Q3_PS, c & 7, __builtin_bit_cast(f32x4, hv[i]));
        }
        int tn, cl = 0;
        if constexpr (DYN) {
            __syncthreads();  // planes complete; slot k & 1 holds the next tile (claimed an iteration earlier)
            tn = __builtin_amdgcn_readfirstlane(slot[k & 1]);
            load_halo(tn, hv);  // the next tile's halo, in flight during this tile's K-loop
            // the tile after next: the returning atomic (~1 us at the memory side) lands during the K-loop and is
            // published after it, instead of stalling thread 0's wave -- and the barrier -- right here
            if (tid == 0) cl = fz::wq_claim_raw(a.wcnt);
        } else {
            tn = fz::tile(ntiles, k);
            load_halo(tn, hv);
            __syncthreads();  // planes complete
        }
        // (RES was last read by the previous tile's epilogue, before the barrier above)
        if (pre_res) dma_res(n, ty, tx);

        f32x16 acc[2] = {(f32x16){}, (f32x16){}};
#pragma unroll
        for (int i = 0; i < 9; ++i) {
            const int kl = 9 * kh + i, tap = kl >> 1, ch = kl & 1, ky = tap / 3, kx = tap % 3;
            bf16x8 bp[2][3];
#pragma unroll
            for (int b = 0; b < 2; ++b) {
                const unsigned char* bs =
                    q3 + ((4 * pb + 2 * b + (r32 >> 4) + ky) * Q3_HW + (r32 & 15) + kx) * Q3_PS + ch * 96 + 16 * g32;
#pragma unroll
                for (int p = 0; p < 3; ++p) bp[b][p] = *(const bf16x8*)(bs + 32 * p);
            }
#pragma unroll
            for (int u = 0; u < 6; ++u)
#pragma unroll
                for (int b = 0; b < 2; ++b)
                    acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(apr[i][TA[u]], bp[b][TB[u]], acc[b], 0, 0, 0);
        }
        // K halves: wave (pb, kh) hands its partner (pb, 1 - kh) the partial sums of block 1 - kh and finishes block kh
        // (lane-ordered, 64 bytes per lane): the epilogue on all eight waves, one block each (s = the K half-0 sum +
        // the half-1 sum either way: the same f32 addition as one wave finishing both blocks)
        f32x16* part = (f32x16*)(q3 + Q3_PART + pb * 8192) + lane;
        part[64 * (1 - kh)] = kh ? acc[0] : acc[1];
        if constexpr (DYN) {
            // read at iteration k + 1 after its first barrier; last read at iteration k - 1, before this one's
            if (tid == 0) slot[(k + 1) & 1] = cl < ntiles ? cl : -1;
        }
        if (pre_res) t3_waitvm<0>();  // this wave's residual DMAs landed (the halo loads before them long since)
        __syncthreads();  // partial sums complete; every wave is done with this tile's planes; RES complete
        {
            // lane (r32, g32) holds channels 8 j + 4 g32 + (0..3), j = 0..3, of its block's pixel r32
            for (int b = kh, be = kh + 1; b < be; ++b) {  // block kh (a loop for the continue below)
                const f32x16 s = (kh ? acc[1] : acc[0]) + part[64 * b];
                const int oy = ty * Q3_T + 4 * pb + 2 * b + (r32 >> 4), ox = tx * Q3_T + (r32 & 15);
                const bool inside = oy < H && ox < W;
                // (the tail's MFMAs take every lane's operands -- its A rows from lanes of pixels outside the map
                // too -- so only its stores are predicated)
                if (!TAIL && !inside) continue;
                const int64_t pix = ((int64_t)n * H + oy) * W + ox;
                float* yp = (float*)a.y + pix * a.ldy + 4 * g32;
                if constexpr (TAIL) {
                    f32x4 v[4];
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const float4 bv = *(const float4*)(a.bias + 8 * j + 4 * g32);
                        v[j] = (f32x4){s[4 * j] + bv.x, s[4 * j + 1] + bv.y, s[4 * j + 2] + bv.z, s[4 * j + 3] + bv.w};
                        if (a.act) v[j] = fz::act(v[j]);
                    }
                    f32x16 o = (f32x16){};
#pragma unroll
                    for (int st = 0; st < 2; ++st) {
                        bf16x8 bq[3], aq[3];
                        split3_bf16(__builtin_bit_cast(u32x4, v[2 * st]), __builtin_bit_cast(u32x4, v[2 * st + 1]), bq);
#pragma unroll
                        for (int p = 0; p < 3; ++p)
                            aq[p] = *(const bf16x8*)(q3 + Q3_W2 + ((r32 * 2 + st) * 3 + p) * 32 + 16 * g32);
#pragma unroll
                        for (int u = 0; u < 6; ++u)
                            o = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aq[TA[u]], bq[TB[u]], o, 0, 0, 0);
                    }
                    // lane (r32, g32) holds tail channels 8 j + 4 g32 + (0..3) of its pixel
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        if (!inside || 8 * j + 4 * g32 >= a.c2) continue;
                        const float4 bv = *(const float4*)(a.b2 + 8 * j + 4 * g32);
                        f32x4 w = {o[4 * j] + bv.x, o[4 * j + 1] + bv.y, o[4 * j + 2] + bv.z, o[4 * j + 3] + bv.w};
                        if (a.act2) w = fz::act(w);
                        *(f32x4*)(yp + 8 * j) = w;
                    }
                } else {
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const float4 bv = *(const float4*)(a.bias + 8 * j + 4 * g32);
                        f32x4 v = {s[4 * j] + bv.x, s[4 * j + 1] + bv.y, s[4 * j + 2] + bv.z, s[4 * j + 3] + bv.w};
                        if (a.act) v = fz::act(v);
                        if (pre_res)
                            v = v + *(const f32x4*)(q3 + Q3_RES + 128 * ((4 * pb + 2 * b + (r32 >> 4)) * Q3_T + (r32 & 15)) +
                                                    16 * (2 * j + g32));
                        *(f32x4*)(yp + 8 * j) = v;
                    }
                }
            }
        }
        t = tn;
    }
    if constexpr (DYN) {
        if (tid == 0) fz::wq_release(a.wcnt);  // after this workgroup's last (failed) claim
    }
}

// ----------------------------------------------------------------------------------------- SPPF pool
// in: slice 0 of buf (c channels), writes slices 1..3 = MaxPool2d(5,1,2) applied 1, 2, 3 times (-inf padding).
// With -inf padding and stride 1, k chained 5x5 pools equal one (4k+1)x(4k+1) pool clipped to the
// image, and a max pool is separable, so the three outputs are column maxima (radius 2k) of row
// maxima (radius 2k) of the input -- exact, no arithmetic.  One workgroup per (image, 16-byte
// channel group): every thread owns whole 16-byte pixel vectors; the plane and its three row-max
// planes live in LDS ([4][H*W] x 16 B: 25.6 KiB at 20x20, 100 KiB at 40x40).
constexpr int SPPF_MAXPIX = 40 * 40;  // 1280-px input -> 40x40 at stride 32

// e4m3 bytes (sign-magnitude) as order keys, four per word: a positive byte b -> b | 0x80, a negative one -> ~b, so
// the keys compare as unsigned bytes in the order of the values (-0 just below +0); key_e4m3 undoes it
__device__ inline unsigned e4m3_key(unsigned w) { return w ^ (0x80808080u | (((w >> 7) & 0x01010101u) * 0x7Fu)); }
__device__ inline unsigned key_e4m3(unsigned k) { return k ^ (0x80808080u | (((~k >> 7) & 0x01010101u) * 0x7Fu)); }

typedef __attribute__((ext_vector_type(2))) unsigned short u16x2;
// byte-wise unsigned max of two words: even and odd bytes as two packed u16 maxima (v_pk_max_u16)
__device__ inline unsigned bytemax(unsigned a, unsigned b) {
    const u16x2 e = __builtin_elementwise_max(__builtin_bit_cast(u16x2, a & 0x00FF00FFu),
                                              __builtin_bit_cast(u16x2, b & 0x00FF00FFu));
    const u16x2 o = __builtin_elementwise_max(__builtin_bit_cast(u16x2, (a >> 8) & 0x00FF00FFu),
                                              __builtin_bit_cast(u16x2, (b >> 8) & 0x00FF00FFu));
    return __builtin_bit_cast(unsigned, e) | (__builtin_bit_cast(unsigned, o) << 8);
}

// element-wise max of two 16-byte vectors; uint8_t: e4m3 order keys (see e4m3_key)
template <typename T>
__device__ inline u32x4 vmax16(u32x4 a, u32x4 b) {
    if constexpr (sizeof(T) == 1) {
        return (u32x4){bytemax(a[0], b[0]), bytemax(a[1], b[1]), bytemax(a[2], b[2]), bytemax(a[3], b[3])};
    } else {
        constexpr int E = 16 / sizeof(T);
        const T* pa = (const T*)&a;
        const T* pb = (const T*)&b;
        u32x4 r;
        T* pr = (T*)&r;
#pragma unroll
        for (int e = 0; e < E; ++e) pr[e] = to_f(pa[e]) >= to_f(pb[e]) ? pa[e] : pb[e];
        return r;
    }
}

// CGW channel groups per workgroup, the group index fastest over the threads: with CGW = 4 (bf16) a
// pixel's 64 contiguous bytes are read and written by 4 neighbouring lanes (whole 64-byte sectors instead
// of 16-byte pieces spread over 4 workgroups)
template <typename T, int CGW>
__global__ __launch_bounds__(256) void sppf_pool_kernel(T* buf, int H, int W, int c, int ld) {
    extern __shared__ __align__(16) u32x4 sp[];  // [4][H*W][CGW]
    constexpr int CG = 16 / sizeof(T);
    const int groups = c / (CG * CGW);
    const int n = blockIdx.x / groups, cg0 = (blockIdx.x % groups) * CGW;
    const int np = H * W, nq = np * CGW;
    T* base = buf + (int64_t)n * np * ld + cg0 * CG;
    for (int i = threadIdx.x; i < nq; i += blockDim.x) {
        const int p = i / CGW, q = i - p * CGW;
        u32x4 v = *(const u32x4*)(base + (int64_t)p * ld + q * CG);
        if constexpr (sizeof(T) == 1) v = (u32x4){e4m3_key(v[0]), e4m3_key(v[1]), e4m3_key(v[2]), e4m3_key(v[3])};
        sp[i] = v;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < nq; i += blockDim.x) {
        const int p = i / CGW, q = i - p * CGW;
        const int y = p / W, x = p - y * W;
        const u32x4* row = sp + y * W * CGW + q;
        u32x4 m = row[x * CGW];
#pragma unroll
        for (int k = 1; k <= 3; ++k) {
#pragma unroll
            for (int d = 2 * k - 1; d <= 2 * k; ++d) {
                if (x - d >= 0) m = vmax16<T>(m, row[(x - d) * CGW]);
                if (x + d < W) m = vmax16<T>(m, row[(x + d) * CGW]);
            }
            sp[k * nq + i] = m;
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < nq; i += blockDim.x) {
        const int p = i / CGW, q = i - p * CGW;
        const int y = p / W, x = p - y * W;
#pragma unroll
        for (int k = 1; k <= 3; ++k) {
            const u32x4* pl = sp + k * nq + x * CGW + q;
            u32x4 m = pl[y * W * CGW];
            for (int d = 1; d <= 2 * k; ++d) {
                if (y - d >= 0) m = vmax16<T>(m, pl[(y - d) * W * CGW]);
                if (y + d < H) m = vmax16<T>(m, pl[(y + d) * W * CGW]);
            }
            if constexpr (sizeof(T) == 1) m = (u32x4){key_e4m3(m[0]), key_e4m3(m[1]), key_e4m3(m[2]), key_e4m3(m[3])};
            *(u32x4*)(base + (int64_t)p * ld + k * c + q * CG) = m;
        }
    }
}

// nearest x2: src [N,H,W] slice (c channels, ld_s) -> dst [N,2H,2W] slice (ld_d), 16-byte chunks
template <typename T>
__global__ void upsample2x_kernel(const T* src, int ld_s, T* dst, int ld_d, int N, int H, int W, int c) {
    constexpr int VEC = 16 / sizeof(T);
    int cv = c / VEC;
    int64_t total = (int64_t)N * 2 * H * 2 * W * cv;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        int ch = (int)(i % cv) * VEC;
        int64_t p = i / cv;
        int x = (int)(p % (2 * W)), y = (int)((p / (2 * W)) % (2 * H)), n = (int)(p / ((int64_t)4 * W * H));
        const T* s = src + (((int64_t)n * H + y / 2) * W + x / 2) * ld_s + ch;
        *(uint4*)(dst + p * ld_d + ch) = *(const uint4*)s;
    }
}

// ---- optional per-op timing of va_seg_run (HIP events on the caller's stream), see va_prof_*
hipEvent_t* g_ev = nullptr;
int* g_ev_kind = nullptr;
int* g_ev_op = nullptr;
int g_ev_cap = 0, g_ev_used = 0, g_prof_on = 0;

int grid_for(int64_t n, int threads) {
    int64_t b = (n + threads - 1) / threads;
    return (int)(b > 65536 ? 65536 : (b < 1 ? 1 : b));
}

template <typename T, int WM, int WN, typename OutT>
hipError_t launch_conv(const va_conv_args& a, hipStream_t st) {
    using Cfg = ConvCfg<T, WM, WN>;
    dim3 grid((a.M + Cfg::BM - 1) / Cfg::BM, (a.Cout + Cfg::BN - 1) / Cfg::BN);
    hipLaunchKernelGGL((conv_kernel<T, WM, WN, OutT>), grid, dim3(Cfg::NT), 0, st, a);
    return hipGetLastError();
}

// Split-K policy (va_conv_args.ws): a launch of fewer than 128 tiles leaves most of the 256 CUs idle while each
// tile walks its whole K loop, one LDS-DMA round trip + barrier per K-step -- the batch-1 forward's cost.  Cost
// model per tile (us, measured at batch 1, profiles/r03/splitk/): ts per K-step (f32 three-term 1.4, bf16 0.6);
// splitting into ks slices costs, in the ticket form (red = false), a slab write + ticket (1.0) and ~1.5 per slice of
// the combine (one workgroup reads ks x 64 KiB): ks <= 16, tiles x ks <= 256; in the reduce form (red, the default:
// conv2_reduce_kernel) the second launch (3.0) and the slabs' traffic (0.02 per 128 x 128 tile-slice): ks <= 32,
// tiles x ks <= 512.  Pick the ks minimising ceil(nk / ks) ts + tw + tc ks, if it beats the unsplit nk ts by 15 %
// (VA_SPLITK_KS forces a count for sweeps).  VA_SPLITK=0 disables it (A/B timing, va_switch.h).  Returns the slice
// count (1 = no split); *kper = K-steps per slice (every slice non-empty).
int conv2_ksplit(const va_conv_args& a, int tiles, int nk, int bm, int bn, int* kper, bool red) {
    *kper = nk;
    if (!va_sw().splitk || !a.ws || tiles >= 128 || nk < 4) return 1;
    if (!red && (!a.wcnt || tiles > a.ncnt)) return 1;
    // cost model (us): K-steps per slice x ts + tw + tc per slice.  Ticket form swept in round 4 at batch 1 (tc 0.75 /
    // 3, ts x1.43, tiles x ks up to 512): the f32 s-seg and bf16 n-seg forwards within 1-2 % of these constants or
    // slower (profiles/r04/batch1/splitk_sweep.log).  Reduce form: tw = the second launch, tc = the slabs' traffic
    const float ts = a.dtype == VA_DTYPE_F32 ? 1.4f : 0.6f;
    const float tw = red ? 3.0f : 1.0f, tc = red ? 0.02f * tiles * (bm * bn / 16384.0f) : 1.5f;
    const int maxks = red ? SK_RED_MAX : 16, maxb = red ? 512 : 256;
    int best = 1;
    float bt = nk * ts;
    for (int ks = 2; ks <= maxks && ks <= nk / 2 && tiles * ks <= maxb; ++ks) {
        if ((int64_t)tiles * ks * bm * bn * 4 > a.ws_bytes) break;
        const float t = ((nk + ks - 1) / ks) * ts + tw + tc * ks;
        if (va_sw().splitk_ks > 0 ? ks <= va_sw().splitk_ks : t < bt) bt = t, best = ks;
    }
    if (best == 1 || (va_sw().splitk_ks <= 0 && bt > 0.85f * nk * ts)) return 1;
    const int per = (nk + best - 1) / best;
    *kper = per;
    return (nk + per - 1) / per;
}

// split K in the reduce form (conv2_reduce_kernel) where conv2 splits a launch: mode 0 without a fused tail, bf16 / f32
// (not the fp8 conv); VA_SPLITK=ticket keeps the last-arriving-slice combine
template <typename T>
bool conv2_red_ok(const va_conv_args& a) {
    return sizeof(T) != 1 && a.mode == 0 && !a.w2 && va_sw().splitk == 1;
}

template <int WM, int WN, int TNS, typename OutT, typename T = __bf16, int SPL = 0, bool W8 = false>
hipError_t launch_conv2(const va_conv_args& a, hipStream_t st) {
    using Cfg = Conv2Cfg<T, WM, WN, TNS>;
    constexpr int VEC = Cfg::VEC, KS = Cfg::KS;
    const int ntm = (a.M + Cfg::BM - 1) / Cfg::BM, ntn = (a.Cout + Cfg::BN - 1) / Cfg::BN;
    const int ntiles = ntm * ntn * (a.mode == 2 ? 4 : 1);
    // LDS-DMA needs every 16-byte chunk aligned: Cin, ldx multiples of VEC and a 16-byte aligned base
    const bool fk = a.Cin % KS == 0 && a.K == a.kh * a.kw * a.Cin && a.Kpad == a.K;
    int kper = a.Kpad / KS, ks = 1;
    const bool red_ok = conv2_red_ok<T>(a);
    if (a.mode != 1) ks = conv2_ksplit(a, ntiles, a.Kpad / KS, Cfg::BM, Cfg::BN, &kper, red_ok);
    const bool red = ks > 1 && red_ok;
    const int nb = ntiles * ks, kpass = red ? -ks : ks;
    if (a.xu)  // upsampled channel prefix: the FK LDS-DMA form only (checked by va_seg_conv)
        hipLaunchKernelGGL((conv2_kernel<T, WM, WN, TNS, OutT, true, true, true, SPL, W8>), dim3(nb), dim3(Cfg::NT), 0,
                           st, a, ntn, nb, kpass, kper);
    else if (a.Cin % VEC == 0 && a.ldx % VEC == 0 && ((uintptr_t)a.x & 15) == 0 && a.Kpad % VEC == 0) {
        if (fk)
            hipLaunchKernelGGL((conv2_kernel<T, WM, WN, TNS, OutT, true, true, false, SPL, W8>), dim3(nb), dim3(Cfg::NT),
                               0, st, a, ntn, nb, kpass, kper);
        else
            hipLaunchKernelGGL((conv2_kernel<T, WM, WN, TNS, OutT, true, false, false, SPL, W8>), dim3(nb), dim3(Cfg::NT),
                               0, st, a, ntn, nb, kpass, kper);
    }
    else
        hipLaunchKernelGGL((conv2_kernel<T, WM, WN, TNS, OutT, false, false, false, SPL, W8>), dim3(nb), dim3(Cfg::NT), 0,
                           st, a, ntn, nb, kpass, kper);
    if constexpr (sizeof(T) != 1) {
        if (red) {
            const int nunits = ntiles * TNS * 4 * Cfg::NT;
            hipLaunchKernelGGL((conv2_reduce_kernel<T, OutT, WM, WN, TNS>), dim3((nunits + 255) / 256), dim3(256), 0, st,
                               a, ntn, ks, nunits);
        }
    }
    return hipGetLastError();
}

// the bf16 conv2 forms with the weights' storage chosen at run time: e4m3 bytes (va_conv_args.w8) or bf16
template <int WM, int WN, int TNS, typename OutT>
hipError_t launch_conv2_b(const va_conv_args& a, hipStream_t st) {
    return a.w8 ? launch_conv2<WM, WN, TNS, OutT, __bf16, 0, true>(a, st) : launch_conv2<WM, WN, TNS, OutT>(a, st);
}

// VA_CONV_PATCH=0 keeps the narrow 3x3 layers on conv_dn (A/B timing, va_switch.h)
bool use_patch(const va_conv_args& a) {
    if (!va_sw().patch) return false;
    if (a.w2 && a.c2 > a.Cout) return false;  // the tail runs TNS = Cout/16 output fragments
    return a.kh == 3 && a.kw == 3 && a.stride == 1 && a.pad == 1 && a.mode == 0 && (a.Cin == 32 || a.Cin == 64) &&
           (a.Cout == 32 || a.Cout == 64) && a.K == 9 * a.Cin && a.ldx % 8 == 0 && ((uintptr_t)a.x & 15) == 0 &&
           a.Ho == a.H && a.Wo == a.W && (a.w2 ? a.ldy % 4 == 0 : (a.ldy % 8 == 0 && ((uintptr_t)a.y & 15) == 0)) &&
           (!a.res || (a.ldr % 8 == 0 && ((uintptr_t)a.res & 15) == 0));
}

template <int TNS, int CPP, bool TAIL, typename OutT, int NW, bool W8 = false>
hipError_t launch_conv_patch_t(const va_conv_args& a, hipStream_t st) {
    const int K = 9 * CPP * 8;
    const int wstride = K + 16;  // +32 bytes per row: conflict-free A-fragment reads
    constexpr int PPI = 64 / CPP, NI = (PW3 * PW3 + PPI - 1) / PPI;
    const int patch_bytes = NI * 1024;
    const size_t lds = (size_t)16 * TNS * wstride * 2 + 2 * (size_t)patch_bytes;
    static DevFlag attr;
    if (!attr()) {
        if (hipFuncSetAttribute((const void*)conv_patch_kernel<TNS, CPP, TAIL, OutT, NW, 0, W8>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) != hipSuccess)
            return hipErrorInvalidValue;
        attr() = true;
    }
    if (lds > 160 * 1024) return hipErrorInvalidValue;
    const int tiles_x = (a.Wo + PT - 1) / PT, tiles_y = (a.Ho + PT - 1) / PT;
    const int ntiles = a.N * tiles_x * tiles_y;
    const int per_cu = (int)((160 * 1024) / lds);
    int blocks = 256 * (per_cu < 1 ? 1 : per_cu);
    if (blocks > ntiles) blocks = ntiles;
    hipLaunchKernelGGL((conv_patch_kernel<TNS, CPP, TAIL, OutT, NW, 0, W8>), dim3(blocks), dim3(64 * NW), lds, st, a,
                       wstride, tiles_x, tiles_y, ntiles, patch_bytes);
    return hipGetLastError();
}


template <bool TAIL, typename OutT, bool W8>
hipError_t launch_conv_patch_w(const va_conv_args& a, hipStream_t st) {
    if (a.Cin == 32)
        return a.Cout == 32 ? launch_conv_patch_t<2, 4, TAIL, OutT, 8, W8>(a, st)
                            : launch_conv_patch_t<4, 4, TAIL, OutT, 8, W8>(a, st);
    return a.Cout == 32 ? launch_conv_patch_t<2, 8, TAIL, OutT, 8, W8>(a, st)
                        : launch_conv_patch_t<4, 8, TAIL, OutT, 8, W8>(a, st);
}

template <bool TAIL, typename OutT>
hipError_t launch_conv_patch(const va_conv_args& a, hipStream_t st) {
    return a.w8 ? launch_conv_patch_w<TAIL, OutT, true>(a, st) : launch_conv_patch_w<TAIL, OutT, false>(a, st);
}

// The Cout > 128 layers with at least 256 256 x 256 tiles run on conv4 (P3/P4 1x1 and 3x3 layers 2-18 % faster
// than conv2, profiles/r01g); VA_CONV4=0 keeps them on conv2, VA_CONV4=all sends every eligible layer (A/B timing
// and the parity tests, va_switch.h)
bool use_conv4(const va_conv_args& a) {
    const int mn = va_sw().conv4_min;
    if (mn < 0) return false;
    if (a.mode != 0 || a.w2 || a.Cout <= 128 || a.Cin % 64 || a.K != a.kh * a.kw * a.Cin || a.Kpad != a.K ||
        a.ldx % 8 || ((uintptr_t)a.x & 15) || a.ldy % 8 || ((uintptr_t)a.y & 15) || a.Npad % 256 ||
        (a.res && (a.ldr % 8 || ((uintptr_t)a.res & 15))))
        return false;
    // e4m3 weights (w8): the multi-tap layers stay on conv2, whose fragment conversion hides beside its MFMAs --
    // m@1280's 192-channel 3x3s at 160 x 160 took 241 us on conv4 against 207-211 on conv2 (and 228-230 on the bf16
    // conv4); the 1x1s keep conv4 (model.4.cv2 111 against 120 us; profiles/r06/c5/ab_conv4_w8.log)
    if (a.w8 && a.kh * a.kw > 1 && mn > 1) return false;
    const int64_t tiles = (int64_t)((a.M + 255) / 256) * ((a.Cout + 255) / 256);
    return tiles >= mn;
}

template <typename OutT, bool W8>
hipError_t launch_conv4_w(const va_conv_args& a, hipStream_t st) {
    static DevFlag attr;
    if (!attr()) {
        if (hipFuncSetAttribute((const void*)conv4_kernel<OutT, false, W8>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                2 * C4_BUF) != hipSuccess ||
            hipFuncSetAttribute((const void*)conv4_kernel<OutT, true, W8>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                2 * C4_BUF) != hipSuccess)
            return hipErrorInvalidValue;
        attr() = true;
    }
    const int ntn = (a.Cout + 255) / 256, ntiles = ntn * ((a.M + 255) / 256);
    if (a.xu)
        hipLaunchKernelGGL((conv4_kernel<OutT, true, W8>), dim3(ntiles), dim3(C4_NT), 2 * C4_BUF, st, a, ntn, ntiles);
    else
        hipLaunchKernelGGL((conv4_kernel<OutT, false, W8>), dim3(ntiles), dim3(C4_NT), 2 * C4_BUF, st, a, ntn, ntiles);
    return hipGetLastError();
}

template <typename OutT>
hipError_t launch_conv4(const va_conv_args& a, hipStream_t st) {
    return a.w8 ? launch_conv4_w<OutT, true>(a, st) : launch_conv4_w<OutT, false>(a, st);
}

// f32 mode's MFMA form (conv2_kernel SPL): VA_F32_SPLIT = 0 (exact f32 MFMA), 6 (default) or 9 bf16 term
// products (A/B timing, va_switch.h)
int f32_split() { return va_sw().f32_split; }

// VA_CONV3T=0 keeps the wide f32 layers on conv2's three-term form (A/B timing, va_switch.h)
bool conv3t_off() { return va_sw().conv3t == 0; }

// the batch-1 layers conv2 would split over K run on conv3t, split over K as well (its slices' slabs summed by
// conv2_reduce_kernel's 32 x 32 form): the s-seg f32 batch-1 forward 885.7 -> 872.0 us, the 3x3s with K >= 1152
// 9-12 % faster each, the rest within 2 % (profiles/r06/c3s/); VA_CONV3T=nosplit keeps them on conv2 (va_switch.h)
bool conv3t_split_mode() { return va_sw().conv3t == 2; }

// conv3t (three-plane f32 kernel): pre-split weights, Cin a multiple of its 16-channel K-step, wide tiles
bool use_conv3t(const va_conv_args& a) {
    if (!a.w3 || conv3t_off()) return false;
    if (conv3t_split_mode() && a.mode == 0 && conv2_red_ok<float>(a))
        return a.Cin % T3_KS == 0 && a.K == a.kh * a.kw * a.Cin && a.Kpad == a.K && a.Kpad % 32 == 0 &&
               a.Npad % T3_BN == 0 && a.Cout > 64 && a.ldx % 4 == 0 && ((uintptr_t)a.x & 15) == 0 && !a.xu && !a.w2;
    // a layer conv2 would split over K (batch-1 shapes) stays on conv2: on the three-plane kernels instead the batch-1
    // f32 s-seg forward took 1.77 ms (stride-1 3x3s on conv3h) / 2.08 ms (every eligible layer) against 1.29
    // (profiles/r04/batch1/small_ab.log)
    int kper;
    const int t2 = ((a.M + 127) / 128) * ((a.Cout + 127) / 128) * (a.mode == 2 ? 4 : 1);
    if (conv2_ksplit(a, t2, a.Kpad / 32, 128, 128, &kper, conv2_red_ok<float>(a)) > 1) return false;
    return (a.mode == 0 || a.mode == 2) && a.Cin % T3_KS == 0 && a.K == a.kh * a.kw * a.Cin && a.Kpad == a.K &&
           a.Npad % T3_BN == 0 && a.Cout > 64 && a.ldx % 4 == 0 && ((uintptr_t)a.x & 15) == 0 && !a.xu && !a.w2;
}

template <int WM, int NSTAGE, typename OutT>
hipError_t launch_conv3t_v(const va_conv_args& a, hipStream_t st, int ks = 1, int kper = 0) {
    using Cfg = T3Cfg<WM, NSTAGE>;
    if (kper <= 0) kper = a.Kpad / T3_KS;
    static DevFlag attr;
    if (!attr()) {
        if (hipFuncSetAttribute((const void*)conv3t_kernel<WM, NSTAGE, OutT>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, Cfg::LDS) != hipSuccess)
            return hipErrorInvalidValue;
        attr() = true;
    }
    const int ntm = (a.M + Cfg::BM - 1) / Cfg::BM, ntn = (a.Cout + T3_BN - 1) / T3_BN;
    const int ntiles = ntm * ntn * (a.mode == 2 ? 4 : 1);
    hipLaunchKernelGGL((conv3t_kernel<WM, NSTAGE, OutT>), dim3(ntiles * ks), dim3(Cfg::NT), Cfg::LDS, st, a, ntn,
                       ntiles * ks, ks, kper);
    if (ks > 1) {
        static_assert(Cfg::NT == 256, "the reduce form's 32 x 32 layout assumes conv3t's 2 x 2 waves");
        const int nunits = ntiles * 16 * Cfg::NT;
        hipLaunchKernelGGL((conv2_reduce_kernel<float, OutT, 2, 2, 4, true>), dim3((nunits + 255) / 256), dim3(256), 0,
                           st, a, ntn, ks, nunits);
    }
    return hipGetLastError();
}

// VA_CONV3H=0 keeps the multi-tap stride-1 layers on conv3t (A/B timing, va_switch.h)
bool conv3h_off() { return va_sw().conv3h == 0; }

// conv3h's tile width for an output map Wo wide: the TW = 4 .. 32 that covers Wo with the fewest padded columns,
// then the smallest halo, then the widest (longest contiguous halo rows); -1 when no width fits the halo buffer
int conv3h_lgw(const va_conv_args& a) {
    int best = -1, bw = 0, bh = 0;
    for (int lg = 5; lg >= 2; --lg) {
        const int tw = 1 << lg, th = T3H_BM / tw, hh = (th + a.kh - 1) * (tw + a.kw - 1);
        if (hh > T3H_HMAX) continue;
        const int waste = (a.Wo + tw - 1) / tw * tw - a.Wo;
        if (best < 0 || waste < bw || (waste == bw && hh < bh)) best = lg, bw = waste, bh = hh;
    }
    return best;
}

bool conv3h_shape_ok(const va_conv_args& a) {
    if (a.stride != 1 || a.H != a.Ho || a.W != a.Wo) return false;
    const bool taps = a.mode == 0 ? (a.kh == 3 && a.kw == 3 && a.pad == 1) : (a.mode == 2 && a.kh == 2 && a.kw == 2);
    return taps && conv3h_lgw(a) >= 0 && (int64_t)a.N * a.Ho < (1 << 24);
}

bool use_conv3h(const va_conv_args& a) { return !conv3h_off() && conv3h_shape_ok(a); }

template <int KH, int KW, int TNS, typename OutT, bool TAIL = false, int TPS = 1>
hipError_t launch_conv3h_v(const va_conv_args& a, hipStream_t st) {
    using Cfg = T3HCfg<TNS, TPS>;
    static DevFlag attr;
    if (!attr()) {
        if (hipFuncSetAttribute((const void*)conv3h_kernel<KH, KW, TNS, OutT, TAIL, TPS>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, Cfg::LDS) != hipSuccess)
            return hipErrorInvalidValue;
        attr() = true;
    }
    const int lgw = conv3h_lgw(a);
    const int tw = 1 << lgw, th = T3H_BM / tw;
    const int tiles_x = (a.Wo + tw - 1) / tw, tiles_y = (a.N * a.Ho + th - 1) / th;
    const int ntn = (a.Cout + Cfg::BN - 1) / Cfg::BN;
    const int ntiles = tiles_x * tiles_y * ntn * (a.mode == 2 ? 4 : 1);
    hipLaunchKernelGGL((conv3h_kernel<KH, KW, TNS, OutT, TAIL, TPS>), dim3(ntiles), dim3(T3H_NT), Cfg::LDS, st, a,
                       ntn, ntiles, lgw, tiles_x);
    return hipGetLastError();
}

// the narrow f32 3x3 layers (33-64 output channels) on conv3h's 64-channel tiles: the conv3t conditions but Cout,
// and not a layer conv2 would split over K.  (The 32-channel layers stay on conv2: on half-idle 64-channel tiles
// model.2's 32 -> 32 bottleneck at 160 x 160 measured 1.25-1.35x slower, profiles/r04/conv3h_narrow/.)
bool use_conv3h_narrow(const va_conv_args& a) {
    if (!a.w3 || conv3t_off() || a.mode != 0 || a.Cout <= 32 || a.Cout > 64 || !use_conv3h(a)) return false;
    int kper;
    const int t2 = ((a.M + 127) / 128) * ((a.Cout + 63) / 64);
    if (conv2_ksplit(a, t2, a.Kpad / 32, 128, 64, &kper, conv2_red_ok<float>(a)) > 1) return false;
    return a.Cin % T3_KS == 0 && a.K == a.kh * a.kw * a.Cin && a.Kpad == a.K && a.Npad % 64 == 0 && a.ldx % 4 == 0 &&
           ((uintptr_t)a.x & 15) == 0 && !a.xu && !a.w2;
}

template <typename OutT>
hipError_t launch_conv3t(const va_conv_args& a, hipStream_t st) {
    if (conv3t_split_mode() && a.mode == 0 && conv2_red_ok<float>(a)) {
        // the slice count from conv2's model in 32-channel K-steps, two of conv3t's per step
        int kper32;
        const int tiles = ((a.M + 127) / 128) * ((a.Cout + 127) / 128);
        const int ks = conv2_ksplit(a, tiles, a.Kpad / 32, 128, 128, &kper32, true);
        if (ks > 1) return launch_conv3t_v<2, 2, OutT>(a, st, ks, 2 * kper32);
    }
    if (use_conv3h(a)) return a.mode == 2 ? launch_conv3h_v<2, 2, 4, OutT>(a, st) : launch_conv3h_v<3, 3, 4, OutT>(a, st);
    return launch_conv3t_v<2, 2, OutT>(a, st);
}

// f32 fused 1x1 tail (va_conv_args.w2 with w3): the conv on conv3h with the whole channel set in one tile (Cout 64 on
// 64-channel tiles, 128 on 128-channel ones; the proto's sub-pixel fold as mode 2), the tail in its epilogue
bool conv3h_tail_ok(const va_conv_args& a) {
    if (!a.w3 || !a.w2 || !a.b2 || a.res || a.xu || a.c2 <= 0 || a.c2 > T3_TAIL_C2 || a.c2 % 4 || a.ldy % 4 ||
        ((uintptr_t)a.y & 15) || (a.Cout != 64 && a.Cout != 128) || (a.mode == 2 && a.Cout != 128) ||
        !conv3h_shape_ok(a))  // (a planned fused op runs on conv3h whatever VA_CONV3H says: the plan has no other form)
        return false;
    return a.Cin % T3_KS == 0 && a.K == a.kh * a.kw * a.Cin && a.Kpad == a.K && a.Npad % 128 == 0 && a.ldx % 4 == 0 &&
           ((uintptr_t)a.x & 15) == 0;
}

hipError_t launch_conv3h_tail(const va_conv_args& a, hipStream_t st) {
    if (!conv3h_tail_ok(a)) return hipErrorInvalidValue;
    if (a.mode == 2) return launch_conv3h_v<2, 2, 4, float, true>(a, st);
    return a.Cout == 128 ? launch_conv3h_v<3, 3, 4, float, true>(a, st) : launch_conv3h_v<3, 3, 2, float, true>(a, st);
}

// the 32 -> 32 stride-1 3x3 f32 layers on conv3q_kernel (VA_CONV3Q=0: conv2's three-term form) when the launch has
// four tiles per CU or more: a workgroup's first tile carries the weight split and an exposed halo load (~19 us per
// tile when a workgroup runs one or two: batch 4's 400 tiles took 38 us against conv2's 28, batch 1 21 vs 20;
// profiles/r05/conv3q/ab_b1.log, ab_b4.log), at 25 per CU a tile costs ~9 us (batch 64: 220 vs 293 us)
constexpr int Q3_MIN_TILES_PER_CU = 4;
int conv3q_tiles(const va_conv_args& a, int* tx, int* ty) {
    *tx = (a.W + Q3_T - 1) / Q3_T;
    *ty = (a.H + Q3_T - 1) / Q3_T;
    const int64_t nt = (int64_t)a.N * *tx * *ty;
    return nt > INT32_MAX ? -1 : (int)nt;
}
int device_cus() {
    static DevVal<int> n_cu;
    if (!n_cu()) {
        int dev = 0, cus = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            return -1;
        n_cu() = cus;
    }
    return n_cu();
}
bool conv3q_shape_ok(const va_conv_args& a) {
    return a.mode == 0 && a.kh == 3 && a.kw == 3 && a.stride == 1 && a.pad == 1 && a.H == a.Ho && a.W == a.Wo &&
           a.Cin == 32 && a.Cout == 32 && a.K == 288 && a.Kpad == 288 && !a.xu && a.ldx % 4 == 0 && a.ldy % 4 == 0 &&
           ((uintptr_t)a.x & 15) == 0 && ((uintptr_t)a.y & 15) == 0 && ((uintptr_t)a.w & 15) == 0 &&
           ((uintptr_t)a.bias & 15) == 0 &&
           (!a.res || (a.ldr % 4 == 0 && ((uintptr_t)a.res & 15) == 0 && (int64_t)a.H * a.W * a.ldr * 4 < (1ll << 31)));
}
bool use_conv3q(const va_conv_args& a) {
    if (!va_sw().conv3q || a.w2 || !conv3q_shape_ok(a)) return false;
    int tx, ty;
    const int nt = conv3q_tiles(a, &tx, &ty), cus = device_cus();
    return cus > 0 && nt >= Q3_MIN_TILES_PER_CU * cus;
}
// f32 fused 1x1 tail on a 32-channel 3x3 (the head's cv4.l.1 -> cv4.l.2): conv3q's TAIL form, whatever VA_CONV3Q
// says or the tile count (a planned fused op has no other form; the planner fuses where conv3q has a tile per CU)
bool conv3q_tail_ok(const va_conv_args& a) {
    return a.w2 && a.b2 && !a.res && a.c2 > 0 && a.c2 <= 32 && a.c2 % 4 == 0 && ((uintptr_t)a.w2 & 15) == 0 &&
           ((uintptr_t)a.b2 & 15) == 0 && conv3q_shape_ok(a);
}
hipError_t launch_conv3q(const va_conv_args& a, hipStream_t st) {
    static DevFlag attr;
    if (!attr()) {
        if (hipFuncSetAttribute((const void*)conv3q_kernel<false, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                Q3_LDS_R) != hipSuccess ||
            hipFuncSetAttribute((const void*)conv3q_kernel<true, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                Q3_LDS_R) != hipSuccess ||
            hipFuncSetAttribute((const void*)conv3q_kernel<false, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                Q3_LDS_T) != hipSuccess ||
            hipFuncSetAttribute((const void*)conv3q_kernel<true, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                Q3_LDS_T) != hipSuccess)
            return hipErrorInvalidValue;
        attr() = true;
    }
    int tx, ty;
    const int nt = conv3q_tiles(a, &tx, &ty), cus = device_cus();
    if (nt <= 0 || cus <= 0) return hipErrorInvalidValue;
    const dim3 grid(nt < cus ? nt : cus);
    const bool dyn = a.wcnt && a.ncnt >= 2 && va_sw().conv3q != 2 &&  // a work counter of the plan: tiles claimed
                     nt >= fz::WQ_MIN_TILES_PER_WG * (int)grid.x;
    auto go = [&](auto kern, int lds) { hipLaunchKernelGGL(kern, grid, dim3(Q3_NT), lds, st, a, tx, ty, nt); };
    if (a.w2)
        dyn ? go(conv3q_kernel<true, true>, Q3_LDS_T) : go(conv3q_kernel<false, true>, Q3_LDS_T);
    else
        dyn ? go(conv3q_kernel<true, false>, a.res ? Q3_LDS_R : Q3_LDS + 16)
            : go(conv3q_kernel<false, false>, a.res ? Q3_LDS_R : Q3_LDS + 16);
    return hipGetLastError();
}

template <int SPL, typename OutT>
hipError_t launch_conv2_f32(const va_conv_args& a, hipStream_t st) {
    if constexpr (SPL == 6 && sizeof(OutT) == 4) {
        if (use_conv3q(a)) return launch_conv3q(a, st);
    }
    if (SPL == 6 && use_conv3t(a)) return launch_conv3t<OutT>(a, st);
    if (SPL == 6 && use_conv3h_narrow(a)) return launch_conv3h_v<3, 3, 2, OutT>(a, st);
    if (a.mode == 2) return a.Cout > 64 ? launch_conv2<2, 2, 4, OutT, float, SPL>(a, st) : hipErrorInvalidValue;
    if (a.Cout <= 32) return launch_conv2<4, 1, 2, OutT, float, SPL>(a, st);
    if (a.Cout <= 64) return launch_conv2<4, 1, 4, OutT, float, SPL>(a, st);
    return launch_conv2<2, 2, 4, OutT, float, SPL>(a, st);
}

template <typename T, typename OutT>
hipError_t dispatch_conv(const va_conv_args& a, hipStream_t st) {
    if constexpr (sizeof(T) == 2 && sizeof(OutT) == 2) {
        // streaming 1x1, Cout 128 (va_pw.hip); e4m3 weights (w8) go to conv2, which converts them in its A stage
        if (!a.w8 && va_pw_eligible(a)) return va_pw_launch(a, st);
    }
    if (a.w2) {  // fused 1x1 tail: narrow layers (Cout 32 / 64) in registers, Cout 128 through LDS
        if constexpr (sizeof(T) == 2) {
            if ((a.Cout == 32 || a.Cout == 64) && a.mode == 0 && !a.res && a.b2 && a.c2 > 0 &&
                a.c2 <= 16 * DN_TAIL_C2F && a.c2 % 4 == 0 && a.Cin % 8 == 0 && a.ldx % 8 == 0 && a.Kpad % 32 == 0 &&
                (size_t)a.Cout * (a.Kpad + 8) * 2 <= 120 * 1024) {
                if (use_patch(a)) return launch_conv_patch<true, OutT>(a, st);
                return a.Cout == 32 ? launch_conv_dn<2, true, OutT>(a, st) : launch_conv_dn<4, true, OutT>(a, st);
            }
            if (a.Cout == 128 && (a.mode == 0 || a.mode == 2) && !a.res && a.b2 && a.c2 > 0 && a.c2 <= 16 * TAIL_C2F &&
                a.c2 % 4 == 0 &&
                a.Kpad % BK2 == 0 && a.ldy % 4 == 0) {
                return launch_conv2_b<2, 2, 4, OutT>(a, st);
            }
        }
        if constexpr (sizeof(T) == 4) {
            if (a.Cout == 32) return conv3q_tail_ok(a) ? launch_conv3q(a, st) : hipErrorInvalidValue;
            return launch_conv3h_tail(a, st);
        }
        return hipErrorInvalidValue;
    }
    if constexpr (sizeof(T) == 2) {
        if (a.xu) {  // upsampled channel prefix (validated by va_seg_conv): the FK LDS-DMA kernels
            if (use_conv4(a)) return launch_conv4<OutT>(a, st);
            if (a.Cout <= 32) return launch_conv2_b<4, 1, 2, OutT>(a, st);
            if (a.Cout <= 64) return launch_conv2_b<4, 1, 4, OutT>(a, st);
            return launch_conv2_b<2, 2, 4, OutT>(a, st);
        }
        if constexpr (sizeof(OutT) == 2) {
            // narrow layers: weights in LDS, activations straight into MFMA fragments
            if (use_patch(a)) return launch_conv_patch<false, __bf16>(a, st);
            // (a launch of under 4096 pixels goes to conv2 instead: conv_dn stages the whole weight matrix per
            // workgroup, which a handful of tiles cannot amortise -- batch-1 model.16, 23.6 -> 16.7 us,
            // profiles/r03/batch1/)
            if (a.mode == 0 && a.Cout <= 64 && a.Cin % 8 == 0 && a.ldx % 8 == 0 && a.Kpad % 32 == 0 && a.M >= 4096 &&
                (size_t)16 * ((a.Cout + 15) / 16) * (a.Kpad + 8) * 2 <= 120 * 1024) {
                switch ((a.Cout + 15) / 16) {
                    case 1: return launch_conv_dn<1>(a, st);
                    case 2: return launch_conv_dn<2>(a, st);
                    case 3: return launch_conv_dn<3>(a, st);
                    default: return launch_conv_dn<4>(a, st);
                }
            }
        }
        constexpr int OV = 16 / sizeof(OutT);
        if (a.mode == 2) {  // sub-pixel classes: the 128-wide LDS-staged tile only
            if (a.Kpad % BK2 == 0 && a.Cout % OV == 0 && a.ldy % OV == 0 && a.Cout > 64)
                return launch_conv2_b<2, 2, 4, OutT>(a, st);
            return hipErrorInvalidValue;
        }
        if (a.Kpad % BK2 == 0 && a.Cout % OV == 0 && a.ldy % OV == 0 && (a.mode == 0 || (a.Cout / 4) % OV == 0)) {
            if (a.Cout <= 32) return launch_conv2_b<4, 1, 2, OutT>(a, st);
            if (a.Cout <= 64) return launch_conv2_b<4, 1, 4, OutT>(a, st);
            if (use_conv4(a)) return launch_conv4<OutT>(a, st);
            return launch_conv2_b<2, 2, 4, OutT>(a, st);
        }
    }
    if constexpr (sizeof(T) == 4) {
        // exact-f32 parity mode: the three-term forms (conv3t / conv2 SPL 6); VA_F32_SPLIT=0: conv2 on the f32 MFMA
        if (a.Kpad % 32 == 0 && a.Cout % 4 == 0 && a.ldy % 4 == 0 && (a.mode != 1 || (a.Cout / 4) % 4 == 0)) {
            switch (f32_split()) {
                case 6: return launch_conv2_f32<6, OutT>(a, st);
                case 9: return launch_conv2_f32<9, OutT>(a, st);
                default: return launch_conv2_f32<0, OutT>(a, st);
            }
        }
    }
    // generic fallback for shapes outside the fast kernels' constraints (register-staged conv_kernel; small Cout ->
    // tall pixel tiles)
    if (a.Cout <= 64) return launch_conv<T, 4, 1, OutT>(a, st);
    return launch_conv<T, 2, 2, OutT>(a, st);
}

}  // namespace

extern "C" {

#ifdef VA_CONV2_STAMPS
// diagnostic build: copy (and optionally clear) conv2_kernel's phase clocks, [C2S_BLOCKS][8] uint64
int va_conv2_stamps(unsigned long long* out, int clear) {
    if (hipDeviceSynchronize() != hipSuccess) return VA_ERR_HIP;
    if (out && hipMemcpyFromSymbol(out, HIP_SYMBOL(g_c2s), sizeof(g_c2s)) != hipSuccess) return VA_ERR_HIP;
    if (clear) {
        static unsigned long long z[C2S_BLOCKS][C2S_PTS];
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_c2s), z, sizeof(z)) != hipSuccess) return VA_ERR_HIP;
    }
    return VA_OK;
}
#endif

int va_seg_conv(void* stream, const va_conv_args* a) {
    if (!a || !a->x || !a->w || !a->bias || !a->y || a->M <= 0 || a->Kpad % BK || a->Cin <= 0) return VA_ERR_ARG;
    if (a->dtype == VA_DTYPE_FP8) {
        if (!va_fp8_conv_ok(*a) || a->Npad < a->Cout || a->K > a->Kpad) return VA_ERR_ARG;
        hipStream_t st = (hipStream_t)stream;
        // e4m3 input: conv2's LDS-DMA tiles (narrow layers get the tall 256-pixel tiles), e4m3 or float output;
        // a bf16 input (model.0's map) or a bf16 output / residual: va_fp8.hip's register-staged kernel
        const bool c2 = a->x8 && (a->out_f32 || a->yscale > 0.0f) && (!a->res || a->rscale > 0.0f);
        if (c2) {
            const int ov = a->out_f32 ? 4 : 16, cd = a->mode == 1 ? a->Cout / 4 : a->Cout;
            if (a->Cout % ov == 0 && cd % ov == 0 && a->ldy % ov == 0 && ((uintptr_t)a->y & 15) == 0 &&
                (!a->res || (a->ldr % 16 == 0 && ((uintptr_t)a->res & 15) == 0))) {
                hipError_t e;
                if (a->out_f32)
                    e = a->Cout <= 32   ? launch_conv2<4, 1, 2, float, uint8_t>(*a, st)
                        : a->Cout <= 64 ? launch_conv2<4, 1, 4, float, uint8_t>(*a, st)
                                        : launch_conv2<2, 2, 4, float, uint8_t>(*a, st);
                else
                    e = a->Cout <= 32   ? launch_conv2<4, 1, 2, uint8_t, uint8_t>(*a, st)
                        : a->Cout <= 64 ? launch_conv2<4, 1, 4, uint8_t, uint8_t>(*a, st)
                                        : launch_conv2<2, 2, 4, uint8_t, uint8_t>(*a, st);
                return e == hipSuccess ? VA_OK : VA_ERR_HIP;
            }
        }
        return va_fp8_conv_launch(*a, st) == hipSuccess ? VA_OK : VA_ERR_HIP;
    }
    const bool bf = a->dtype == VA_DTYPE_BF16;
    const int vec = bf ? 8 : 4, ks = 8 * vec;  // elements per 16-byte chunk / per conv2 K-step
    if (a->xu && (a->kh != 1 || a->kw != 1 || a->stride != 1 || a->pad != 0 || a->mode != 0 || a->w2 ||
                  a->out_f32 || a->Cin % ks || a->cu <= 0 || a->cu % ks || a->cu >= a->Cin || a->K != a->Cin ||
                  a->Kpad != a->K || a->ldu % vec || ((uintptr_t)a->xu & 15) || a->H % 2 || a->W % 2 ||
                  a->ldx % vec || ((uintptr_t)a->x & 15)))
        return VA_ERR_ARG;
    if (a->Cin % vec || a->ldx % vec || a->Cout % 4 || a->ldy % 4 || (a->res && a->ldr % 4)) return VA_ERR_ARG;
    // e4m3 weight bytes in the bf16 kernels: per-output-channel scales ([4][Npad] for mode 2), 16-byte aligned
    if (a->w8 && (!bf || !a->wscale || ((uintptr_t)a->wscale & 15) || ((uintptr_t)a->w & 15))) return VA_ERR_ARG;
    if (a->Npad % 128 || a->Npad < a->Cout) return VA_ERR_ARG;
    if (a->mode == 2 && (a->kh != 2 || a->kw != 2 || a->stride != 1 || a->res || a->Cout <= 64 || a->Kpad % ks))
        return VA_ERR_ARG;
    // bias4: mode 2 only -- bf16 through conv2's fused-tail path (Cout 128) or its plain epilogue (the wider protos of
    // m / l / x, no tail), f32 through the plain epilogue
    if (a->bias4 && (a->mode != 2 || (bf && a->w2 && a->Cout != 128))) return VA_ERR_ARG;
    // f32 fused tail: conv3h's conditions (launch_conv3h_tail) are checked at dispatch
    if (a->w2 && a->dtype == VA_DTYPE_F32 && a->Cout == 32 && !conv3q_tail_ok(*a)) return VA_ERR_ARG;
    if (a->w2 && a->dtype == VA_DTYPE_F32 && a->Cout != 32 &&
        (!a->w3 || a->res || !a->b2 || a->c2 <= 0 || a->c2 > T3_TAIL_C2 || a->c2 % 4 || a->mode == 1 ||
         (a->Cout != 64 && a->Cout != 128)))
        return VA_ERR_ARG;
    if (a->w2 && a->dtype != VA_DTYPE_F32 && ((a->Cout != 32 && a->Cout != 64 && a->Cout != 128) || a->mode == 1 ||
                  (a->mode == 2 && a->Cout != 128) ||
                  a->res || !a->b2 || a->c2 <= 0 || a->c2 > 16 * (a->Cout == 128 ? TAIL_C2F : DN_TAIL_C2F) ||
                  a->c2 % 4 || a->Kpad % (a->Cout == 128 ? BK2 : 32) ||
                  (a->Cout < 128 && (size_t)a->Cout * (a->Kpad + 8) * 2 > 120 * 1024)))
        return VA_ERR_ARG;
    hipStream_t st = (hipStream_t)stream;
    hipError_t e;
    if (a->dtype == VA_DTYPE_BF16)
        e = a->out_f32 ? dispatch_conv<__bf16, float>(*a, st) : dispatch_conv<__bf16, __bf16>(*a, st);
    else if (a->dtype == VA_DTYPE_F32)
        e = dispatch_conv<float, float>(*a, st);
    else
        return VA_ERR_ARG;
    return e == hipSuccess ? VA_OK : VA_ERR_HIP;
}

int va_seg_preprocess(void* stream, const uint8_t* frames, int32_t B, int32_t H, int32_t W, int32_t dtype,
                      void* out) {
    if (!frames || !out || B <= 0 || H <= 0 || W <= 0) return VA_ERR_ARG;
    int64_t npix = (int64_t)B * H * W;
    hipStream_t st = (hipStream_t)stream;
    if (dtype == VA_DTYPE_BF16)
        hipLaunchKernelGGL(seg_preprocess_kernel<__bf16>, dim3(grid_for(npix, 256)), dim3(256), 0, st, frames, npix,
                           (__bf16*)out);
    else if (dtype == VA_DTYPE_F32)
        hipLaunchKernelGGL(seg_preprocess_kernel<float>, dim3(grid_for(npix, 256)), dim3(256), 0, st, frames, npix,
                           (float*)out);
    else
        return VA_ERR_ARG;
    return hipGetLastError() == hipSuccess ? VA_OK : VA_ERR_HIP;
}

int va_seg_sppf_pool(void* stream, void* buf, int32_t N, int32_t H, int32_t W, int32_t c, int32_t ld,
                     int32_t dtype) {
    const int cg = dtype == VA_DTYPE_FP8 ? 16 : dtype == VA_DTYPE_BF16 ? 8 : 4;  // elements per 16 bytes
    if (!buf || N <= 0 || c <= 0 || ld < 4 * c || c % cg || ld % cg || H * W > SPPF_MAXPIX || ((uintptr_t)buf & 15))
        return VA_ERR_ARG;
    // 2 channel groups per workgroup while the four planes fit 52 KiB of LDS (20 x 20 maps: three
    // workgroups per CU) and the launch still fills the CUs, else one (batch 1: 8 -> 16 workgroups for n-seg)
    const int cgw = ((c / cg) % 2 == 0 && (size_t)4 * H * W * 16 * 2 <= 52 * 1024 && N * (c / cg) >= 512) ? 2 : 1;
    const int blocks = N * (c / cg / cgw);
    const size_t lds = (size_t)4 * H * W * 16 * cgw;
    hipStream_t st = (hipStream_t)stream;
    auto go = [&](auto kern, auto* p) {
        (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), lds, st, p, H, W, c, ld);
    };
    if (dtype == VA_DTYPE_FP8) {
        if (cgw == 2) go(sppf_pool_kernel<uint8_t, 2>, (uint8_t*)buf);
        else go(sppf_pool_kernel<uint8_t, 1>, (uint8_t*)buf);
    } else if (dtype == VA_DTYPE_BF16) {
        if (cgw == 2) go(sppf_pool_kernel<__bf16, 2>, (__bf16*)buf);
        else go(sppf_pool_kernel<__bf16, 1>, (__bf16*)buf);
    } else {
        if (cgw == 2) go(sppf_pool_kernel<float, 2>, (float*)buf);
        else go(sppf_pool_kernel<float, 1>, (float*)buf);
    }
    return hipGetLastError() == hipSuccess ? VA_OK : VA_ERR_HIP;
}

int va_seg_upsample2x(void* stream, const void* src, int32_t ld_s, void* dst, int32_t ld_d, int32_t N, int32_t H,
                      int32_t W, int32_t c, int32_t dtype) {
    const int vec = dtype == VA_DTYPE_FP8 ? 16 : dtype == VA_DTYPE_BF16 ? 8 : 4;
    if (!src || !dst || c % vec || ld_s % vec || ld_d % vec) return VA_ERR_ARG;
    int64_t total = (int64_t)N * 4 * H * W * (c / vec);
    hipStream_t st = (hipStream_t)stream;
    if (dtype == VA_DTYPE_FP8)
        hipLaunchKernelGGL(upsample2x_kernel<uint8_t>, dim3(grid_for(total, 256)), dim3(256), 0, st,
                           (const uint8_t*)src, ld_s, (uint8_t*)dst, ld_d, N, H, W, c);
    else if (dtype == VA_DTYPE_BF16)
        hipLaunchKernelGGL(upsample2x_kernel<__bf16>, dim3(grid_for(total, 256)), dim3(256), 0, st,
                           (const __bf16*)src, ld_s, (__bf16*)dst, ld_d, N, H, W, c);
    else
        hipLaunchKernelGGL(upsample2x_kernel<float>, dim3(grid_for(total, 256)), dim3(256), 0, st, (const float*)src,
                           ld_s, (float*)dst, ld_d, N, H, W, c);
    return hipGetLastError() == hipSuccess ? VA_OK : VA_ERR_HIP;
}

int va_prof_start(int32_t capacity) {
    if (capacity <= 0) return VA_ERR_ARG;
    if (capacity > g_ev_cap) {
        for (int i = 0; i < 2 * g_ev_cap; ++i) (void)hipEventDestroy(g_ev[i]);
        delete[] g_ev;
        delete[] g_ev_kind;
        delete[] g_ev_op;
        g_ev = new hipEvent_t[2 * capacity];
        g_ev_kind = new int[capacity];
        g_ev_op = new int[capacity];
        for (int i = 0; i < 2 * capacity; ++i)
            if (hipEventCreate(&g_ev[i]) != hipSuccess) return VA_ERR_HIP;
        g_ev_cap = capacity;
    }
    g_ev_used = 0;
    g_prof_on = 1;
    return VA_OK;
}

int va_prof_enable(int32_t on) {
    if (!g_ev_cap) return VA_ERR_ARG;
    g_prof_on = on ? 1 : 0;
    return VA_OK;
}

int va_prof_stop_ops(double* ms_by_op, int32_t nops) {
    // per op index of the list (summed over every va_seg_run call recorded); keeps the records
    if (!ms_by_op || nops <= 0) return VA_ERR_ARG;
    for (int k = 0; k < nops; ++k) ms_by_op[k] = 0.0;
    if (g_ev_used && hipEventSynchronize(g_ev[2 * g_ev_used - 1]) != hipSuccess) return VA_ERR_HIP;
    for (int i = 0; i < g_ev_used; ++i) {
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, g_ev[2 * i], g_ev[2 * i + 1]) != hipSuccess) return VA_ERR_HIP;
        if (g_ev_op[i] >= 0 && g_ev_op[i] < nops) ms_by_op[g_ev_op[i]] += ms;
    }
    return g_ev_used;
}

int va_prof_stop(double* ms_by_kind, int64_t* n_by_kind, int32_t nkinds) {
    g_prof_on = 0;
    if (!ms_by_kind || !n_by_kind || nkinds <= 0) return VA_ERR_ARG;
    for (int k = 0; k < nkinds; ++k) {
        ms_by_kind[k] = 0.0;
        n_by_kind[k] = 0;
    }
    if (g_ev_used && hipEventSynchronize(g_ev[2 * g_ev_used - 1]) != hipSuccess) return VA_ERR_HIP;
    for (int i = 0; i < g_ev_used; ++i) {
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, g_ev[2 * i], g_ev[2 * i + 1]) != hipSuccess) return VA_ERR_HIP;
        int k = g_ev_kind[i];
        if (k >= 0 && k < nkinds) {
            ms_by_kind[k] += ms;
            n_by_kind[k] += 1;
        }
    }
    int used = g_ev_used;
    g_ev_used = 0;
    return used;
}

int va_seg_conv0(void* stream, const uint8_t* frames, int32_t N, int32_t H, int32_t W, const void* w,
                 const float* bias, int32_t Cout, void* y, int32_t ldy) {
    if (!frames || !w || !bias || !y || N <= 0 || H <= 0 || W <= 0 || Cout % 16 || Cout > 64 || ldy % 8 ||
        (3 * W) % 16 || ((uintptr_t)frames & 15) || ((uintptr_t)y & 15))
        return VA_ERR_ARG;
    const int Ho = (H + 1) / 2, Wo = (W + 1) / 2;
    dim3 grid((Wo + C0_TW - 1) / C0_TW, (Ho + C0_TH - 1) / C0_TH, N);
    hipStream_t st = (hipStream_t)stream;
    const __bf16* wp = (const __bf16*)w;
    __bf16* yp = (__bf16*)y;
    switch (Cout / 16) {
        case 1: hipLaunchKernelGGL(conv0_kernel<1>, grid, dim3(256), 0, st, frames, N, H, W, wp, bias, yp, ldy); break;
        case 2: hipLaunchKernelGGL(conv0_kernel<2>, grid, dim3(256), 0, st, frames, N, H, W, wp, bias, yp, ldy); break;
        case 3: hipLaunchKernelGGL(conv0_kernel<3>, grid, dim3(256), 0, st, frames, N, H, W, wp, bias, yp, ldy); break;
        default: hipLaunchKernelGGL(conv0_kernel<4>, grid, dim3(256), 0, st, frames, N, H, W, wp, bias, yp, ldy);
    }
    return hipGetLastError() == hipSuccess ? VA_OK : VA_ERR_HIP;
}

int va_seg_conv0_e4m3(void* stream, const uint8_t* frames, int32_t N, int32_t H, int32_t W, const void* w,
                      const float* bias, int32_t Cout, uint8_t* y, int32_t ldy, float yscale) {
    if (!frames || !w || !bias || !y || N <= 0 || H <= 0 || W <= 0 || Cout % 16 || Cout > 64 || ldy % 8 ||
        (3 * W) % 16 || ((uintptr_t)frames & 15) || ((uintptr_t)y & 7) || !(yscale > 0.0f))
        return VA_ERR_ARG;
    const int Ho = (H + 1) / 2, Wo = (W + 1) / 2;
    dim3 grid((Wo + C0_TW - 1) / C0_TW, (Ho + C0_TH - 1) / C0_TH, N);
    hipStream_t st = (hipStream_t)stream;
    const __bf16* wp = (const __bf16*)w;
    switch (Cout / 16) {
        case 1: hipLaunchKernelGGL((conv0_kernel<1, true>), grid, dim3(256), 0, st, frames, N, H, W, wp, bias, y, ldy, yscale); break;
        case 2: hipLaunchKernelGGL((conv0_kernel<2, true>), grid, dim3(256), 0, st, frames, N, H, W, wp, bias, y, ldy, yscale); break;
        case 3: hipLaunchKernelGGL((conv0_kernel<3, true>), grid, dim3(256), 0, st, frames, N, H, W, wp, bias, y, ldy, yscale); break;
        default: hipLaunchKernelGGL((conv0_kernel<4, true>), grid, dim3(256), 0, st, frames, N, H, W, wp, bias, y, ldy, yscale);
    }
    return hipGetLastError() == hipSuccess ? VA_OK : VA_ERR_HIP;
}

int va_seg_conv0_f32(void* stream, const uint8_t* frames, int32_t N, int32_t H, int32_t W, const float* w,
                     const float* bias, int32_t Cout, float* y, int32_t ldy) {
    if (!frames || !w || !bias || !y || N <= 0 || H <= 0 || W <= 0 || Cout % 16 || Cout > 64 || ldy % 4 ||
        ldy < Cout || ((uintptr_t)y & 15))
        return VA_ERR_ARG;
    const int64_t total = (int64_t)N * ((H + 1) / 2) * ((W + 1) / 2);
    const int grid = grid_for(total, 256);
    hipStream_t st = (hipStream_t)stream;
    switch (Cout / 16) {
        case 1: hipLaunchKernelGGL(conv0_f32_kernel<16>, dim3(grid), dim3(256), 0, st, frames, N, H, W, w, bias, y, ldy); break;
        case 2: hipLaunchKernelGGL(conv0_f32_kernel<32>, dim3(grid), dim3(256), 0, st, frames, N, H, W, w, bias, y, ldy); break;
        case 3: hipLaunchKernelGGL(conv0_f32_kernel<48>, dim3(grid), dim3(256), 0, st, frames, N, H, W, w, bias, y, ldy); break;
        default: hipLaunchKernelGGL(conv0_f32_kernel<64>, dim3(grid), dim3(256), 0, st, frames, N, H, W, w, bias, y, ldy);
    }
    return hipGetLastError() == hipSuccess ? VA_OK : VA_ERR_HIP;
}

int va_seg_conv0_f32m(void* stream, const uint8_t* frames, int32_t N, int32_t H, int32_t W, const void* w3,
                      const float* bias, int32_t Cout, float* y, int32_t ldy) {
    if (!frames || !w3 || !bias || !y || N <= 0 || H <= 0 || W <= 0 || Cout % 16 || Cout > 64 || ldy % 4 ||
        ldy < Cout || ((uintptr_t)y & 15) || (W * 3) % 16 || N > 65535)
        return VA_ERR_ARG;
    const int Ho = (H + 1) / 2, Wo = (W + 1) / 2;
    dim3 grid((Wo + C0_TW - 1) / C0_TW, (Ho + C0_TH - 1) / C0_TH, N);
    hipStream_t st = (hipStream_t)stream;
    const __bf16* wp = (const __bf16*)w3;
    switch (Cout / 16) {
        case 1: hipLaunchKernelGGL(conv0_f32m_kernel<1>, grid, dim3(256), 0, st, frames, N, H, W, wp, bias, y, ldy); break;
        case 2: hipLaunchKernelGGL(conv0_f32m_kernel<2>, grid, dim3(256), 0, st, frames, N, H, W, wp, bias, y, ldy); break;
        case 3: hipLaunchKernelGGL(conv0_f32m_kernel<3>, grid, dim3(256), 0, st, frames, N, H, W, wp, bias, y, ldy); break;
        default: hipLaunchKernelGGL(conv0_f32m_kernel<4>, grid, dim3(256), 0, st, frames, N, H, W, wp, bias, y, ldy);
    }
    return hipGetLastError() == hipSuccess ? VA_OK : VA_ERR_HIP;
}

int va_seg_stem_f32(void* stream, const va_conv_args* a) {
    if (!a || !a->x || !a->w3 || !a->bias || !a->w || !a->b2 || !a->y || a->dtype != VA_DTYPE_F32 || a->Cin != 32 ||
        a->Cout != 64 || a->K != 288 || a->Kpad != 288 || a->Npad < 64 || a->N <= 0 || a->H <= 0 || a->W <= 0 ||
        (a->W * 3) % 16 || a->ldy < 64 || a->ldy % 4 || ((uintptr_t)a->y & 15) || ((uintptr_t)a->x & 15) ||
        ((uintptr_t)a->w & 15) || ((uintptr_t)a->bias & 15) || ((uintptr_t)a->b2 & 15) ||
        (int64_t)a->H * a->W * 3 >= 0x80000000LL)
        return VA_ERR_ARG;
    const bool tail = a->w2 != nullptr;
    if (tail && (a->c2 != 64 || a->act2 != 1 || ((uintptr_t)a->w2 & 15))) return VA_ERR_ARG;
    const int Ho0 = (a->H + 1) / 2, Wo0 = (a->W + 1) / 2, Ho1 = (Ho0 + 1) / 2, Wo1 = (Wo0 + 1) / 2;
    const int tiles_x = (Wo1 + S32_TW - 1) / S32_TW, tiles_y = (Ho1 + S32_TH - 1) / S32_TH;
    const int64_t nt = (int64_t)tiles_x * tiles_y * a->N;
    if (nt > INT32_MAX) return VA_ERR_ARG;
    const int cus = device_cus();
    static DevFlag attr;
    if (cus <= 0) return VA_ERR_HIP;
    if (!attr()) {
        if (hipFuncSetAttribute((const void*)stem32_kernel<false, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                S32_LDS + 16) != hipSuccess ||
            hipFuncSetAttribute((const void*)stem32_kernel<false, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                S32_LDS + 16) != hipSuccess ||
            hipFuncSetAttribute((const void*)stem32_kernel<true, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                S32_LDS_T + 16) != hipSuccess ||
            hipFuncSetAttribute((const void*)stem32_kernel<true, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                S32_LDS_T + 16) != hipSuccess)
            return VA_ERR_HIP;
        attr() = true;
    }
    const int grid = (int)(nt < cus ? nt : cus);
    const bool dyn = a->wcnt && a->ncnt >= 2 && va_sw().conv3q != 2 &&  // work-queue schedule (VA_CONV3Q=static: off)
                     nt >= (int64_t)fz::WQ_MIN_TILES_PER_WG * grid;
    const float* wt = tail ? (const float*)a->w2 : nullptr;
    const float* bt = tail ? a->b2 + 64 : nullptr;
    const size_t lds = (tail ? S32_LDS_T : S32_LDS) + 16;
    auto go = [&](auto kern) {
        hipLaunchKernelGGL(kern, dim3(grid), dim3(S32_NT), lds, (hipStream_t)stream, (const uint8_t*)a->x, a->N, a->H,
                           a->W, (const __bf16*)a->w3, a->bias, (const float*)a->w, a->Kpad, a->b2, (float*)a->y,
                           a->ldy, tiles_x, tiles_y, (int)nt, wt, bt, a->wcnt);
    };
    if (tail)
        dyn ? go(stem32_kernel<true, true>) : go(stem32_kernel<true, false>);
    else
        dyn ? go(stem32_kernel<false, true>) : go(stem32_kernel<false, false>);
    return hipGetLastError() == hipSuccess ? VA_OK : VA_ERR_HIP;
}

}  // extern "C"

// ---- lanes of a laned op list (va355.h VA_OP_FORK) ----
// One set of VA_LANES - 1 non-blocking streams + fork / join events per (device, calling stream): two
// pipelines with forwards in flight on two streams never share a lane (no false ordering between them).
// Every wait a list issues points at work already submitted (a fork waits on the calling stream's past, a
// join on the lane's past), so lanes sharing a hardware queue cannot deadlock.
namespace {
struct LaneSet {
    int dev;
    hipStream_t owner;
    hipStream_t s[VA_LANES];
    hipEvent_t fork[VA_LANES], join[VA_LANES];
};
constexpr int VA_LANE_SETS = 32;
LaneSet g_lane_sets[VA_LANE_SETS];
int g_nlane_sets = 0;
std::mutex g_lane_mu;

// -> the calling stream's lane set (created on first use), or nullptr (table full / HIP error: the list then
// runs serially on the calling stream, in list order)
LaneSet* lane_set(hipStream_t owner) {
    const int dev = va_cur_dev();
    std::lock_guard<std::mutex> lk(g_lane_mu);
    for (int i = 0; i < g_nlane_sets; ++i)
        if (g_lane_sets[i].dev == dev && g_lane_sets[i].owner == owner) return &g_lane_sets[i];
    if (g_nlane_sets == VA_LANE_SETS) return nullptr;
    LaneSet& ls = g_lane_sets[g_nlane_sets];
    ls.dev = dev;
    ls.owner = owner;
    for (int l = 1; l < VA_LANES; ++l)
        if (hipStreamCreateWithFlags(&ls.s[l], hipStreamNonBlocking) != hipSuccess ||
            hipEventCreateWithFlags(&ls.fork[l], hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&ls.join[l], hipEventDisableTiming) != hipSuccess)
            return nullptr;
    ++g_nlane_sets;
    return &ls;
}
}  // namespace

extern "C" {

int va_seg_run(void* stream, const va_seg_op* ops, int32_t n) {
    if (!ops || n < 0) return VA_ERR_ARG;
    LaneSet* ls = nullptr;          // resolved at the first fork
    bool serial = g_prof_on;        // live timing brackets every op on the calling stream
    unsigned forked = 0, open = 0;  // lanes forked in this list / with work not yet joined
    for (int i = 0; i < n; ++i) {
        const va_conv_args& a = ops[i].a;
        const int kind = ops[i].kind, lane = ops[i].lane;
        if (lane < 0 || lane >= VA_LANES) return VA_ERR_ARG - 1000 * (i + 1);
        if (kind == VA_OP_FORK || kind == VA_OP_JOIN) {
            const int l = a.N;
            if (l < 1 || l >= VA_LANES || lane != 0 || (kind == VA_OP_JOIN && !(forked >> l & 1)))
                return VA_ERR_ARG - 1000 * (i + 1);
            forked |= 1u << l;
            if (serial) continue;
            if (!ls && !(ls = lane_set((hipStream_t)stream))) {
                serial = true;
                continue;
            }
            const bool fk = kind == VA_OP_FORK;
            hipStream_t from = fk ? (hipStream_t)stream : ls->s[l], to = fk ? ls->s[l] : (hipStream_t)stream;
            hipEvent_t ev = fk ? ls->fork[l] : ls->join[l];
            if (hipEventRecord(ev, from) != hipSuccess || hipStreamWaitEvent(to, ev, 0) != hipSuccess)
                return VA_ERR_HIP - 1000 * (i + 1);
            open = fk ? (open | 1u << l) : (open & ~(1u << l));
            continue;
        }
        if (lane && !(forked >> lane & 1)) return VA_ERR_ARG - 1000 * (i + 1);
        void* st = stream;
        if (lane && !serial) {
            st = ls->s[lane];
            open |= 1u << lane;
        }
        int rc;
        const bool prof = g_prof_on && g_ev_used < g_ev_cap;
        if (prof && hipEventRecord(g_ev[2 * g_ev_used], (hipStream_t)stream) != hipSuccess) return VA_ERR_HIP;
        switch (kind) {
            case VA_OP_CONV:
                rc = va_seg_conv(st, &a);
                break;
            case VA_OP_SPPF:
                rc = va_seg_sppf_pool(st, a.y, a.N, a.H, a.W, a.Cin, a.ldy, a.dtype);
                break;
            case VA_OP_UPSAMPLE:
                rc = va_seg_upsample2x(st, a.x, a.ldx, a.y, a.ldy, a.N, a.H, a.W, a.Cin, a.dtype);
                break;
            case VA_OP_PREPROCESS:
                rc = va_seg_preprocess(st, (const uint8_t*)a.x, a.N, a.H, a.W, a.dtype, a.y);
                break;
            case VA_OP_CONV0:
                rc = a.dtype == VA_DTYPE_F32
                         ? (a.w3 ? va_seg_conv0_f32m(st, (const uint8_t*)a.x, a.N, a.H, a.W, a.w3, a.bias, a.Cout,
                                                     (float*)a.y, a.ldy)
                                 : va_seg_conv0_f32(st, (const uint8_t*)a.x, a.N, a.H, a.W, (const float*)a.w,
                                                    a.bias, a.Cout, (float*)a.y, a.ldy))
                     : a.dtype == VA_DTYPE_FP8
                         ? va_seg_conv0_e4m3(st, (const uint8_t*)a.x, a.N, a.H, a.W, a.w, a.bias, a.Cout,
                                             (uint8_t*)a.y, a.ldy, a.yscale)
                         : va_seg_conv0(st, (const uint8_t*)a.x, a.N, a.H, a.W, a.w, a.bias, a.Cout, a.y, a.ldy);
                break;
            case VA_OP_C2F:
                rc = a.mode == 3 ? va_seg_c2fb(st, &a) : va_seg_c2f(st, &a);
                break;
            case VA_OP_STEM:
                rc = a.dtype == VA_DTYPE_F32 ? va_seg_stem_f32(st, &a) : va_seg_stem(st, &a);
                break;
            default:
                rc = VA_ERR_ARG;
        }
        if (rc != VA_OK) return rc - 1000 * (i + 1);  // encode the failing op index
        if (prof) {
            if (hipEventRecord(g_ev[2 * g_ev_used + 1], (hipStream_t)stream) != hipSuccess) return VA_ERR_HIP;
            g_ev_op[g_ev_used] = i;
            g_ev_kind[g_ev_used++] = kind;
        }
    }
    for (int l = 1; l < VA_LANES; ++l)  // lanes the list left open
        if (open >> l & 1)
            if (hipEventRecord(ls->join[l], ls->s[l]) != hipSuccess ||
                hipStreamWaitEvent((hipStream_t)stream, ls->join[l], 0) != hipSuccess)
                return VA_ERR_HIP;
    return VA_OK;
}

}  // extern "C"

// va_fp8.hip -- the convolutions of YOLOv8-seg on block-scaled fp8 MFMA (gfx950 v_mfma_scale_f32_16x16x128_f8f6f4,
// OCP e4m3 operands): BASELINE.json configs[4], "YOLOv8m-seg 1280x1280 fp8 MFMA weights".
//
// Weights are e4m3 with one scale per output channel (seg.py packs them).  Activations live in HBM as e4m3 bytes
// with one static power-of-two scale per buffer (seg.py SegNet.calibrate_fp8: a concat buffer, and the buffers an
// upsample copies between, share one): every conv reads its input bytes as they are (X8) -- or, for the one bf16
// map (model.0's output), quantizes it while staging -- and writes its output already quantized with the output
// buffer's scale, so SPPF's maxima and the FPN's upsample copies work on the bytes.  With x_q = sat(x * xs),
// W_q = W / sw[co]:
//     y[co] = act(sum_k W_q[co][k] x_q[k] * wscale[co] + bias[co]) (+ r_q / rs),  wscale[co] = sw[co] / xs,
//     stored as sat(y * ys) (e4m3), or bf16 / float,
// the instruction's own E8M0 block scales held at 1.0 (127).  The K order inside a 128-deep step is whatever the
// instruction's lane map is -- the same bytes of a lane feed A and B, so the sum is over the same K either way.
//
//   conv8_kernel<X8>  implicit GEMM, 128 pixels x 128 output channels per 256-thread workgroup (2 x 2 waves of
//                     64 x 64, 16 accumulators each), K-steps of 128 bytes, two LDS stages with register staging
//                     (weights and e4m3 activations: 16-byte loads; bf16 activations: two 16-byte loads per 16
//                     values, clamped in the bf16 domain and converted by v_cvt_scalef32_pk_fp8_bf16),
//                     XCD-aware tile order, the bias / SiLU / residual epilogue (mode 0 and the ConvTranspose2d
//                     scatter of mode 1) with e4m3, bf16 or float output and an e4m3 or bf16 residual.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include "../../include/va355.h"
#include "va_fuse.h"

typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
typedef __attribute__((ext_vector_type(8))) int i32x8;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;

namespace {

constexpr int F8_BM = 128, F8_BN = 128, F8_NT = 256;
constexpr int F8_KS = 128;                   // K (bytes) per stage
constexpr int F8_RS = F8_KS + 16;            // LDS row stride (bytes): +16 spreads the rows over the banks
constexpr int F8_STAGE = (F8_BM + F8_BN) * F8_RS;
constexpr int F8_CW = F8_BN + 4;             // epilogue f32 row (floats)
constexpr int F8_LDS = 2 * F8_STAGE > F8_BM * F8_CW * 4 ? 2 * F8_STAGE : F8_BM * F8_CW * 4;
constexpr float F8_MAX = 448.0f;             // largest e4m3 (OCP e4m3fn)

typedef short v2s __attribute__((ext_vector_type(2)));
typedef __bf16 v2bf __attribute__((ext_vector_type(2)));
typedef unsigned short v2u16 __attribute__((ext_vector_type(2)));

// 16 bf16 (two 16-byte loads) -> 16 e4m3 (one 16-byte LDS chunk): sat(x * s), RNE, with s a power of two.
// v_cvt_scalef32_pk_fp8_bf16 converts two bf16 divided by its scale operand (inv = 1 / s, exact) but turns values
// past the format into NaN, so each pair is first clamped in the bf16 domain: the magnitude bits (a bf16's
// ordering is its integer ordering) capped at lim = 448 / s with one v_pk_min_u16, the sign put back -- four VALU
// ops per two values.
__device__ __forceinline__ u32x4 quant16(u32x4 lo, u32x4 hi, float inv, unsigned lim2) {
    u32x4 out;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const u32x4 v = h ? hi : lo;
#pragma unroll
        for (int q = 0; q < 2; ++q) {  // two u32 (four bf16) -> one u32 (four e4m3)
            unsigned w2[2];
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                const unsigned x = v[2 * q + e];
                const v2u16 m = __builtin_elementwise_min(__builtin_bit_cast(v2u16, x & 0x7FFF7FFFu),
                                                          __builtin_bit_cast(v2u16, lim2));
                w2[e] = (x & 0x80008000u) | __builtin_bit_cast(unsigned, m);
            }
            v2s r = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16((v2s){0, 0}, __builtin_bit_cast(v2bf, w2[0]), inv, false);
            r = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16(r, __builtin_bit_cast(v2bf, w2[1]), inv, true);
            out[2 * h + q] = __builtin_bit_cast(unsigned, r);
        }
    }
    return out;
}

// the clamp bound 448 / s as a pair of bf16 magnitudes (s a power of two: exact)
__device__ __forceinline__ unsigned quant_lim2(float s) {
    const unsigned b = __float_as_uint(F8_MAX / s) >> 16;
    return b | (b << 16);
}

// 8 floats -> 8 e4m3 bytes: sat(v * ys), round to nearest even
__device__ __forceinline__ uint2 pack8_e4m3(const float* v, float ys) {
    float c[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) c[e] = fminf(fmaxf(v[e] * ys, -F8_MAX), F8_MAX);
    int lo = __builtin_amdgcn_cvt_pk_fp8_f32(c[0], c[1], 0, false);
    lo = __builtin_amdgcn_cvt_pk_fp8_f32(c[2], c[3], lo, true);
    int hi = __builtin_amdgcn_cvt_pk_fp8_f32(c[4], c[5], 0, false);
    hi = __builtin_amdgcn_cvt_pk_fp8_f32(c[6], c[7], hi, true);
    return make_uint2((unsigned)lo, (unsigned)hi);
}

// 8 e4m3 bytes -> 8 floats times inv (exact: e4m3 values and power-of-two scales)
__device__ __forceinline__ void unpack8_e4m3(uint2 q, float inv, float* v) {
    typedef __attribute__((ext_vector_type(2))) float f2;
    const f2 a = __builtin_amdgcn_cvt_pk_f32_fp8((int)q.x, false), b = __builtin_amdgcn_cvt_pk_f32_fp8((int)q.x, true);
    const f2 c = __builtin_amdgcn_cvt_pk_f32_fp8((int)q.y, false), d = __builtin_amdgcn_cvt_pk_f32_fp8((int)q.y, true);
    v[0] = a[0] * inv, v[1] = a[1] * inv, v[2] = b[0] * inv, v[3] = b[1] * inv;
    v[4] = c[0] * inv, v[5] = c[1] * inv, v[6] = d[0] * inv, v[7] = d[1] * inv;
}

template <bool X8>
__global__ __launch_bounds__(F8_NT) void conv8_kernel(va_conv_args a, int ntn, int ntiles) {
    __shared__ __align__(16) unsigned char smem[F8_LDS];
    int bid = blockIdx.x;
    {  // XCD-contiguous runs of tiles (blocks are dealt round-robin over the 8 XCDs)
        const int nx = 8, q = ntiles / nx, r = ntiles % nx, xcd = bid % nx, j = bid / nx;
        bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + j;
    }
    const int tm = bid / ntn, tn = bid % ntn;
    const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wid >> 1, wn = wid & 1;
    const int m0 = tm * F8_BM, n0 = tn * F8_BN;
    const uint8_t* __restrict__ Wq = (const uint8_t*)a.w;
    const __bf16* __restrict__ X = (const __bf16*)a.x;
    const uint8_t* __restrict__ X8p = (const uint8_t*)a.x;
    const float inv = 1.0f / a.xscale;  // xscale is a power of two (va_fp8_conv_ok)
    const unsigned lim2 = quant_lim2(a.xscale);
    // staging: chunk c = tid + 256 q (q < 4): row c / 8, 16-byte column g = c % 8 (the same g for all four)
    const int g = tid & 7, row0 = tid >> 3;  // rows row0 + 32 q
    int b_hi[4], b_wi[4];
    int64_t b_base[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int m = m0 + row0 + 32 * q;
        if (m < a.M) {
            const int wo = m % a.Wo, t = m / a.Wo, ho = t % a.Ho, n = t / a.Ho;
            b_hi[q] = ho * a.stride - a.pad;
            b_wi[q] = wo * a.stride - a.pad;
            b_base[q] = (int64_t)n * a.H * a.W;
        } else {
            b_hi[q] = -(1 << 28);
            b_wi[q] = 0;
            b_base[q] = 0;
        }
    }
    int ci = 16 * g, ky = 0, kx = 0, kcur = 16 * g;  // this thread's K position (16 channels, one tap)
    while (ci >= a.Cin) {
        ci -= a.Cin;
        if (++kx == a.kw) {
            kx = 0;
            ++ky;
        }
    }
    u32x4 ra[4], rb[4];
    auto load = [&](int k0) {
#pragma unroll
        for (int q = 0; q < 4; ++q)
            ra[q] = *(const u32x4*)(Wq + (int64_t)(n0 + row0 + 32 * q) * a.Kpad + k0 + 16 * g);
        const bool kin = kcur < a.K;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int hi = b_hi[q] + ky, wi = b_wi[q] + kx;
            const bool ok = kin && (unsigned)hi < (unsigned)a.H && (unsigned)wi < (unsigned)a.W;
            const int64_t off = ok ? (b_base[q] + (int64_t)hi * a.W + wi) * a.ldx + ci : 0;
            if constexpr (X8) {  // already e4m3 with this scale
                const u32x4 v = *(const u32x4*)(X8p + off);
                rb[q] = ok ? v : (u32x4){0u, 0u, 0u, 0u};
            } else {
                const u32x4 lo = *(const u32x4*)(X + off), hi8 = *(const u32x4*)(X + off + 8);
                rb[q] = ok ? quant16(lo, hi8, inv, lim2) : (u32x4){0u, 0u, 0u, 0u};
            }
        }
        kcur += F8_KS;
        ci += F8_KS;
        while (ci >= a.Cin) {
            ci -= a.Cin;
            if (++kx == a.kw) {
                kx = 0;
                ++ky;
            }
        }
    };
    auto store = [&](int s) {
        unsigned char* as_ = smem + s * F8_STAGE;
        unsigned char* bs_ = as_ + F8_BN * F8_RS;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            *(u32x4*)(as_ + (row0 + 32 * q) * F8_RS + 16 * g) = ra[q];
            *(u32x4*)(bs_ + (row0 + 32 * q) * F8_RS + 16 * g) = rb[q];
        }
    };
    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    const int nk = a.Kpad / F8_KS;
    load(0);
    store(0);
    __syncthreads();
    const int fr = lane & 15, fq = lane >> 4;
    for (int kt = 0; kt < nk; ++kt) {
        const int s = kt & 1;
        const bool more = kt + 1 < nk;
        if (more) load((kt + 1) * F8_KS);
        const unsigned char* as_ = smem + s * F8_STAGE;
        const unsigned char* bs_ = as_ + F8_BN * F8_RS;
        // lane (fr, fq): 32 bytes of row fr of each 16-row fragment, bytes 32 fq .. 32 fq + 31 of the step
        i32x8 af[4], bfr[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const unsigned char* p = as_ + (wn * 64 + 16 * i + fr) * F8_RS + 32 * fq;
            const u32x4 x0 = *(const u32x4*)p, x1 = *(const u32x4*)(p + 16);
            af[i] = (i32x8){(int)x0[0], (int)x0[1], (int)x0[2], (int)x0[3], (int)x1[0], (int)x1[1], (int)x1[2],
                            (int)x1[3]};
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const unsigned char* p = bs_ + (wm * 64 + 16 * j + fr) * F8_RS + 32 * fq;
            const u32x4 x0 = *(const u32x4*)p, x1 = *(const u32x4*)(p + 16);
            bfr[j] = (i32x8){(int)x0[0], (int)x0[1], (int)x0[2], (int)x0[3], (int)x1[0], (int)x1[1], (int)x1[2],
                             (int)x1[3]};
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)  // A = weights (format 0: e4m3), B = activations (e4m3), scales 2^0
                acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(af[i], bfr[j], acc[i][j], 0, 0, 0, 127,
                                                                           0, 127);
        if (more) store(s ^ 1);
        __syncthreads();
    }
    // ---- epilogue: dequant scale + bias (+SiLU) -> f32 tile in LDS, then 16-byte runs per pixel (+ residual)
    float* Cs = (float*)smem;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int col = wn * 64 + 16 * i + 4 * fq;
        const float4 bv = *(const float4*)(a.bias + n0 + col);
        const float4 sv = *(const float4*)(a.wscale + n0 + col);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            float v[4] = {acc[i][j][0] * sv.x + bv.x, acc[i][j][1] * sv.y + bv.y, acc[i][j][2] * sv.z + bv.z,
                          acc[i][j][3] * sv.w + bv.w};
            if (a.act) {
                const f32x2 s01 = fz::silu2((f32x2){v[0], v[1]}), s23 = fz::silu2((f32x2){v[2], v[3]});
                v[0] = s01[0], v[1] = s01[1], v[2] = s23[0], v[3] = s23[1];
            }
            *(float4*)(Cs + (wm * 64 + 16 * j + fr) * F8_CW + col) = make_float4(v[0], v[1], v[2], v[3]);
        }
    }
    __syncthreads();
    const bool of32 = a.out_f32 != 0, o8 = a.yscale > 0.0f, r8 = a.rscale > 0.0f;
    const int OV = of32 ? 4 : 8, CPRO = F8_BN / OV;
    const __bf16* R = (const __bf16*)a.res;
    const uint8_t* R8 = (const uint8_t*)a.res;
    const float rinv = r8 ? 1.0f / a.rscale : 0.0f;
    for (int c = tid; c < F8_BM * CPRO; c += F8_NT) {
        const int pl = c / CPRO, cl = (c % CPRO) * OV;
        const int m = m0 + pl, co = n0 + cl;
        if (m >= a.M || co >= a.Cout) continue;
        float v[8];
#pragma unroll
        for (int r = 0; r < 8; r += 4) {
            if (r < OV) {
                const float4 t = *(const float4*)(Cs + pl * F8_CW + cl + r);
                v[r] = t.x, v[r + 1] = t.y, v[r + 2] = t.z, v[r + 3] = t.w;
            }
        }
        if (a.res) {
            if (r8) {  // e4m3 residual (8 channels; not with a float output)
                float rv[8];
                unpack8_e4m3(*(const uint2*)(R8 + (int64_t)m * a.ldr + co), rinv, rv);
#pragma unroll
                for (int e = 0; e < 8; ++e) v[e] += rv[e];
            } else if (of32) {
                const uint2 rr = *(const uint2*)(R + (int64_t)m * a.ldr + co);
                const __bf16* rp = (const __bf16*)&rr;
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] += (float)rp[e];
            } else {
                const u32x4 rr = *(const u32x4*)(R + (int64_t)m * a.ldr + co);
                const __bf16* rp = (const __bf16*)&rr;
#pragma unroll
                for (int e = 0; e < 8; ++e) v[e] += (float)rp[e];
            }
        }
        int64_t yo;
        if (a.mode == 1) {  // ConvTranspose2d(2, 2) as a 1x1 with 4 C outputs: sub-pixel q = co / C
            const int wo = m % a.Wo, t = m / a.Wo, ho = t % a.Ho, n = t / a.Ho;
            const int cd = a.Cout / 4, q = co / cd, cc = co - q * cd;
            yo = (((int64_t)n * 2 * a.Ho + 2 * ho + (q >> 1)) * 2 * a.Wo + 2 * wo + (q & 1)) * a.ldy + cc;
        } else {
            yo = (int64_t)m * a.ldy + co;
        }
        if (of32) {
            *(float4*)((float*)a.y + yo) = make_float4(v[0], v[1], v[2], v[3]);
        } else if (o8) {
            *(uint2*)((uint8_t*)a.y + yo) = pack8_e4m3(v, a.yscale);
        } else {
            bf16x8 o;
#pragma unroll
            for (int e = 0; e < 8; ++e) o[e] = (__bf16)v[e];
            *(bf16x8*)((__bf16*)a.y + yo) = o;
        }
    }
}

}  // namespace

// va_seg_conv's fp8 path (va_seg.hip validates the common fields first)
hipError_t va_fp8_conv_launch(const va_conv_args& a, hipStream_t st) {
    const int ntm = (a.M + F8_BM - 1) / F8_BM, ntn = a.Npad / F8_BN;
    const int ntiles = ntm * ntn;
    if (a.x8) hipLaunchKernelGGL(conv8_kernel<true>, dim3(ntiles), dim3(F8_NT), 0, st, a, ntn, ntiles);
    else hipLaunchKernelGGL(conv8_kernel<false>, dim3(ntiles), dim3(F8_NT), 0, st, a, ntn, ntiles);
    return hipGetLastError();
}

bool va_fp8_conv_ok(const va_conv_args& a) {
    // 16 channels of one tap per staged chunk (16 e4m3 bytes, or two 16-byte bf16 runs); outputs in 8-element runs
    // (e4m3: 8 bytes, bf16: 16 bytes; 4 floats for a float output, which takes no residual); power-of-two scales
    auto pow2 = [](float f) {
        uint32_t b;
        memcpy(&b, &f, sizeof b);
        return f > 0.0f && (b & 0x7FFFFFu) == 0;
    };
    const bool in_ok = a.x8 ? (a.ldx % 16 == 0 && ((uintptr_t)a.x & 15) == 0)
                            : (a.ldx % 8 == 0 && ((uintptr_t)a.x & 15) == 0);
    const bool o8 = a.yscale > 0.0f, r8 = a.rscale > 0.0f;
    bool out_ok;
    if (a.out_f32) {
        out_ok = !o8 && a.Cout % 4 == 0 && a.ldy % 4 == 0 && !a.res;
    } else {
        const int cd = a.mode == 1 ? a.Cout / 4 : a.Cout;
        const int al = o8 ? 8 : 16;  // bytes of an 8-element run
        out_ok = a.Cout % 8 == 0 && cd % 8 == 0 && a.ldy % 8 == 0 && ((uintptr_t)a.y & (al - 1)) == 0 &&
                 (!o8 || pow2(a.yscale));
        if (a.res)
            out_ok = out_ok && a.ldr % 8 == 0 && (r8 ? (pow2(a.rscale) && ((uintptr_t)a.res & 7) == 0)
                                                     : ((uintptr_t)a.res & 15) == 0);
    }
    return a.wscale && pow2(a.xscale) && a.Cin % 16 == 0 && in_ok && a.Kpad % F8_KS == 0 && a.Npad % F8_BN == 0 &&
           (a.mode == 0 || a.mode == 1) && !a.w2 && !a.xu && !a.bias4 && out_ok;
}

// Test probe of the e4m3 conversions (tests/test_gpu_fp8.py): out[2i], out[2i+1] = the staging path's bytes of
// in[i] * s (mode 0), or v_cvt_scalef32_pk_fp8_bf16's bytes with scale s (mode 1).
namespace {
__global__ void fp8_cvt_probe_kernel(const __bf16* in, uint8_t* out, int n, float s, int mode) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (2 * i + 1 >= n) return;
    if (mode == 0) {
        u32x4 lo = {0u, 0u, 0u, 0u};
        lo[0] = (unsigned)__builtin_bit_cast(unsigned short, in[2 * i]) |
                ((unsigned)__builtin_bit_cast(unsigned short, in[2 * i + 1]) << 16);
        const u32x4 q = quant16(lo, (u32x4){0u, 0u, 0u, 0u}, 1.0f / s, quant_lim2(s));
        out[2 * i] = (uint8_t)(q[0] & 0xFF);
        out[2 * i + 1] = (uint8_t)((q[0] >> 8) & 0xFF);
    } else {
        const v2bf src = {in[2 * i], in[2 * i + 1]};
        const v2s r = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16((v2s){0, 0}, src, s, false);
        out[2 * i] = (uint8_t)(r[0] & 0xFF);
        out[2 * i + 1] = (uint8_t)((r[0] >> 8) & 0xFF);
    }
}
}  // namespace

extern "C" int va_fp8_cvt_probe(void* stream, const void* in, void* out, int32_t n, float s, int32_t mode) {
    if (!in || !out || n <= 0 || n % 2) return VA_ERR_ARG;
    hipLaunchKernelGGL(fp8_cvt_probe_kernel, dim3((n / 2 + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                       (const __bf16*)in, (uint8_t*)out, n, s, mode);
    return hipGetLastError() == hipSuccess ? VA_OK : VA_ERR_HIP;
}

// va_c2fb.hip -- a whole YOLOv8 C2f block of any width as ONE launch for small batches (bf16): block.py C2f
// (cv1 -> chunk -> n Bottlenecks -> cat -> cv2), every intermediate in LDS, for the batch-1 forward that
// FrameProcessor.py:322's model.predict runs per frame (C2, BASELINE.json configs[1]).
//
// At batch 1 a C2f block is 4 (n = 1) or 6 (n = 2) dependent launches of a few us each whose MFMA work is tiny
// (model.6 of YOLOv8n-seg at 40 x 40: 0.5 GFLOP), so the block's time is launch boundaries, prologues and store
// tails (DESIGN.md §5's phase clocks).  Here a workgroup owns a T x T output tile and recomputes what the tile needs:
//
//   region IN  (T + 4n)^2 pixels of the block's input (ci channels, zero outside the frame; an FPN upsample prefix
//              is read in place from its half-resolution source, va355.h va_conv_args.xu)
//   cv1        1x1 ci -> 2c over all of IN -> R0 (zero outside the frame: the 3x3s' padding)
//   m.j.cv1    3x3 c -> c: R(2j) -> R(2j+1), one pixel smaller on every side; R(0) means R0's second half (b)
//   m.j.cv2    3x3 c -> c: R(2j+1) -> R(2j+2), + R(2j) at the same pixel (shortcut)
//   cv2        1x1 over [R0 (a | b) | R2 | R4 ...] at the tile's pixels (the concat, read in place) -> y
//
// Each conv is an implicit GEMM over its output region in 16-pixel x 16-channel blocks on
// v_mfma_f32_16x16x32_bf16: the activations (B) from LDS, the weights (A) straight from global memory in
// fragment order (seg.py SegNet._pack_c2fb; L2-resident, eight K-steps loaded ahead), eight waves sharing the
// blocks.  Every intermediate is bias + SiLU (+ shortcut) in f32 rounded to bf16 -- the rounding a stored layer
// gets -- so the block equals the unfused layers up to the f32 summation order inside each conv.  The halo
// recompute (a T = 4 tile of an n = 1 block computes cv1 on 8 x 8 pixels) costs MFMA time the batch-1 forward
// has to spare: a layer there fills a few dozen of the 256 CUs.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/va355.h"
#include "va_dev.h"
#include "va_fuse.h"

namespace {

using fz::mma;

constexpr int XB_NW = 8, XB_NT = 64 * XB_NW;
constexpr int XB_G = 4;       // 16-pixel blocks per work item (one A fragment feeds XB_G MFMAs)
constexpr int XB_KC = 8;      // K-steps of A fragments loaded ahead
constexpr int XB_LDS_MAX = 160 * 1024;
constexpr int XB_TR = 10;     // stage clocks per workgroup in the debug trace: start, after each stage, end
// debug trace: thread 0 stamps the shader clock (s_memtime) at point pt after the workgroup's barrier
#define XB_MARK(g, pt) \
    if ((g).trace && threadIdx.x == 0) (g).trace[blockIdx.x * XB_TR + (pt)] = __builtin_amdgcn_s_memtime()

struct XbGeom {
    const __bf16* x;
    const __bf16* xu;
    __bf16* y;
    const bf16x8* w;  // fragments: conv q at w + 64 * wf[q], [ncb][ks][64 lanes]
    const float* b;   // biases: conv q at b + bo[q], [16 ncb]
    int N, H, W, ci, cu, ldx, ldu, co, ldy;
    int T, tx, tpf;   // tile side, tiles per row, tiles per frame
    int sc;           // Bottleneck shortcut
    int psi;          // LDS bytes per pixel of the input region
    int in_off;       // LDS offset of the input region (R1 .. R2n alias it once cv1 has read it)
    int off_r[5];     // LDS offsets of R0 .. R2n
    int wf[7], bo[7]; // per conv (cv1, m.0.cv1, m.0.cv2, [m.1.cv1, m.1.cv2,] cv2[, the stride-2 prologue])
    // optional stride-2 prologue: input channels [0, cs) are Conv(cis -> cs, 3x3, s2, p1) + SiLU of xs ([N][2H][2W],
    // channel stride ldxs), computed per tile from the source region SR ((2 S0 + 1)^2 pixels) staged at off_sr
    const __bf16* xs;
    int ldxs, cs, cis, lgcis, off_sr, pss;
    unsigned long long* trace;  // debug (va_c2fb_trace): [grid][XB_TR] stage clocks of wave 0, or null
    int off_b, nbias;           // the biases' copy in LDS (off_b) and their count
};

// conv q's shape: output channels, K (elements), K-steps of 32
template <int C, int NB>
struct XbConvShape {
    static __host__ __device__ int nout(int q, int co) { return q == 0 ? 2 * C : q == 2 * NB + 1 ? co : C; }
    static __host__ __device__ int k(int q, int ci) { return q == 0 ? ci : q == 2 * NB + 1 ? (2 + NB) * C : 9 * C; }
};

// LDS pixel strides: 16 bytes past the channels (rows of 16 pixels then spread over the banks)
template <int C>
constexpr int ps0() { return 4 * C + 16; }
template <int C>
constexpr int psc() { return 2 * C + 16; }


// an LDS region: byte offset, width in pixels (regions are square), pixel stride, first channel; off < 0 = none
struct XbIo {
    int off, w, ps, c0;
};

typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;

__device__ __forceinline__ float bf_lo(unsigned u) { return __builtin_bit_cast(float, u << 16); }
__device__ __forceinline__ float bf_hi(unsigned u) { return __builtin_bit_cast(float, u & 0xffff0000u); }

// One conv of the block over an ow x ow output region whose pixel 0 sits at image (oy, ox) of frame n.
// KIND 0: 1x1 over the input region (cv1; src = IN, the same geometry as the output);
// KIND 1: 3x3 from src (one pixel larger on every side), + res at the same pixel (two larger) when res.off >= 0;
// KIND 2: 1x1 over the concat [R0 | R2 | R4 ...] at the tile's pixels (cv2), written to g.y.
// Pixels outside the frame are stored as zero (the next 3x3's padding); KIND 2 skips them.
// every conv's biases into LDS at off_b (issued beside the first stage's loads; read after its barrier)
__device__ __forceinline__ void xb_bias_to_lds(const float* b, int nbias, unsigned char* smem, int off_b) {
    for (int i = 4 * (int)threadIdx.x; i < nbias; i += 4 * XB_NT)
        *(f32x4*)(smem + off_b + 4 * i) = *(const f32x4*)(b + i);
}

// the first XB_KC A fragments of conv q's 16-channel block cb (ks K-steps): what an item's K loop starts on
__device__ __forceinline__ void xb_first(const XbGeom& g, int q, int cb, int ks, int lane, bf16x8 (&a0)[XB_KC]) {
    const bf16x8* wb = g.w + (int64_t)64 * (g.wf[q] + cb * ks) + lane;
#pragma unroll
    for (int i = 0; i < XB_KC; ++i) a0[i] = wb[64 * min(i, ks - 1)];
}

// a conv's shape as its successor's prefetch needs it: index, 16-channel blocks, K-steps (q < 0: none)
struct XbNext {
    int q, ncb, ks;
};

// a0 holds the first chunk of this conv's first item for the wave (issued before the barrier that precedes the
// conv, or by the previous item); the item loop issues the next item's first chunk before its epilogue, and the
// last item the successor conv's (nx) -- so no item and no stage starts on an exposed L2 round trip
template <int C, int NB, int KIND>
__device__ __forceinline__ void xb_conv(const XbGeom& g, unsigned char* smem, int q, int nout, int kel, int ow, int oy,
                                        int ox, int n, XbIo src, XbIo dst, XbIo res, int lane, int wid,
                                        bf16x8 (&a0)[XB_KC], XbNext nx) {
    constexpr int H2 = 2 * NB;
    const int ks = (kel + 31) >> 5, ncb = (nout + 15) >> 4;
    const int P = ow * ow, npb = (P + 15) >> 4, ngr = (npb + XB_G - 1) / XB_G;
    const int items = ngr * ncb;
    const int fr = lane & 15, fq = lane >> 4;
    const int S0 = g.T + 2 * H2;
    for (int it = wid; it < items; it += XB_NW) {
        const int cb = it % ncb, gr = it / ncb;
        const int nb = min(XB_G, npb - gr * XB_G);  // live pixel blocks of this item (wave-uniform)
        int base[XB_G], pr[XB_G], pc[XB_G];
#pragma unroll
        for (int j = 0; j < XB_G; ++j) {
            int p = ((gr * XB_G + j) << 4) + fr;
            p = p < P ? p : P - 1;  // a block's tail lanes read a real pixel; their results are dropped
            const int r = p / ow, c = p - r * ow;
            pr[j] = r;
            pc[j] = c;
            if constexpr (KIND == 0) base[j] = src.off + p * src.ps;
            else if constexpr (KIND == 1) base[j] = src.off + (r * src.w + c) * src.ps + src.c0 * 2;
            else if constexpr (KIND == 3) base[j] = src.off + (2 * r * src.w + 2 * c) * src.ps;
            else base[j] = 0;
        }
        f32x4 acc[XB_G];
#pragma unroll
        for (int j = 0; j < XB_G; ++j) acc[j] = (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
        const bf16x8* wb = g.w + (int64_t)64 * (g.wf[q] + cb * ks) + lane;
        // one K-step: the four blocks' B fragments read together (a block past the item's live ones reads a clamped
        // real pixel), then the live blocks' MFMAs.  (MFMAs on the dead blocks too -- no guard at all -- gave
        // non-finite outputs on the live ones, profiles/r05/c2fb/bisect.log; the guard stays.)
        auto step = [&](int k, bf16x8 a) {
            const int kk = min((k << 5) + (fq << 3), kel - 8);  // past K: the last group (its weights are zero)
            bf16x8 b[XB_G];
#pragma unroll
            for (int j = 0; j < XB_G; ++j) {
                int addr;
                if constexpr (KIND == 0) {
                    addr = base[j] + kk * 2;
                } else if constexpr (KIND == 1) {
                    const int tap = kk / C, ch = kk - tap * C, ky = tap / 3, kx = tap - 3 * ky;
                    addr = base[j] + (ky * src.w + kx) * src.ps + ch * 2;
                } else if constexpr (KIND == 3) {  // stride 2 from SR: output (r, c) reads SR (2r + ky, 2c + kx)
                    const int tap = kk >> g.lgcis, ch = kk - (tap << g.lgcis), ky = tap / 3, kx = tap - 3 * ky;
                    addr = base[j] + (ky * src.w + kx) * src.ps + ch * 2;
                } else if (kk < 2 * C) {
                    addr = g.off_r[0] + ((pr[j] + H2) * S0 + pc[j] + H2) * ps0<C>() + kk * 2;
                } else {
                    const int s = (kk - 2 * C) / C + 1, ch = kk - (s + 1) * C;
                    const int hs = H2 - 2 * s, ws = g.T + 2 * hs;  // R(2s): halo hs
                    addr = g.off_r[2 * s] + ((pr[j] + hs) * ws + pc[j] + hs) * psc<C>() + ch * 2;
                }
                b[j] = *(const bf16x8*)(smem + addr);
            }
            // the reads are used here, ahead of the guards: the compiler cannot sink them into the guarded blocks
            // (where each got a wait of its own); one wait covers the four
#pragma unroll
            for (int j = 0; j < XB_G; ++j) asm volatile("" ::"v"(b[j]));
#pragma unroll
            for (int j = 0; j < XB_G; ++j)
                if (j < nb) acc[j] = mma(a, b[j], acc[j]);
        };
        // A loads unconditional (a chunk past ks re-reads the last step, unused): a fixed count in flight, so the
        // waits before each step count loads instead of draining them all (vmcnt(0))
        bf16x8 a1[XB_KC];
        for (int k0 = 0; k0 < ks; k0 += 2 * XB_KC) {
#pragma unroll
            for (int i = 0; i < XB_KC; ++i) a1[i] = wb[64 * min(k0 + XB_KC + i, ks - 1)];
#pragma unroll
            for (int i = 0; i < XB_KC; ++i)
                if (k0 + i < ks) step(k0 + i, a0[i]);
#pragma unroll
            for (int i = 0; i < XB_KC; ++i) a0[i] = wb[64 * min(k0 + 2 * XB_KC + i, ks - 1)];
#pragma unroll
            for (int i = 0; i < XB_KC; ++i)
                if (k0 + XB_KC + i < ks) step(k0 + XB_KC + i, a1[i]);
        }
        // the next item's first chunk (this conv's, or the successor's first item) in flight under the epilogue
        if (it + XB_NW < items) xb_first(g, q, (it + XB_NW) % ncb, ks, lane, a0);
        else if (nx.q >= 0) xb_first(g, nx.q, wid % nx.ncb, nx.ks, lane, a0);
        // epilogue: the lane holds channels 4 fq .. 4 fq + 3 of block cb for its pixel of each block
        const int co = (cb << 4) + (fq << 2);
        if (co >= nout) continue;
        const f32x4 bias = *(const f32x4*)(smem + g.off_b + (g.bo[q] + co) * 4);  // (a global load here stalled
                                                                                     //  every item's epilogue)
#pragma unroll
        for (int j = 0; j < XB_G; ++j) {
            const int p = ((gr * XB_G + j) << 4) + fr;
            if (j >= nb || p >= P) continue;
            const int r = pr[j], c = pc[j], iy = oy + r, ix = ox + c;
            const bool in = iy >= 0 && iy < g.H && ix >= 0 && ix < g.W;
            f32x4 v = fz::act(acc[j] + bias);
            if (KIND == 1 && res.off >= 0) {  // Bottleneck shortcut, added after the activation (va_seg.hip epilogue)
                const uint2 rr = *(const uint2*)(smem + res.off + ((r + 2) * res.w + c + 2) * res.ps + (res.c0 + co) * 2);
                v += (f32x4){bf_lo(rr.x), bf_hi(rr.x), bf_lo(rr.y), bf_hi(rr.y)};
            }
            bf16x4 o = {(__bf16)v[0], (__bf16)v[1], (__bf16)v[2], (__bf16)v[3]};
            if constexpr (KIND == 2) {
                if (in) *(bf16x4*)(g.y + ((int64_t)(n * g.H + iy) * g.W + ix) * g.ldy + co) = o;
            } else {
                if (!in) o = (bf16x4){(__bf16)0.0f, (__bf16)0.0f, (__bf16)0.0f, (__bf16)0.0f};
                *(bf16x4*)(smem + dst.off + p * dst.ps + (dst.c0 + co) * 2) = o;
            }
        }
    }
    if (wid >= items && nx.q >= 0) xb_first(g, nx.q, wid % nx.ncb, nx.ks, lane, a0);  // idle here: prefetch only
}

template <int C, int NB>
__global__ __launch_bounds__(XB_NT) void c2fb_kernel(XbGeom g) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr int H2 = 2 * NB;
    const int T = g.T, S0 = T + 2 * H2;
    const int t = blockIdx.x, n = t / g.tpf, tt = t - n * g.tpf, ty = tt / g.tx, tx = tt - ty * g.tx;
    const int y0 = ty * T, x0 = tx * T;
    // the wave index as a scalar: item / block / guard arithmetic derived from it stays wave-uniform (scalar branches)
    const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    XB_MARK(g, 0);
    xb_bias_to_lds(g.b, g.nbias, smem, g.off_b);
    // the input region, eight 16-byte loads in flight per thread before their LDS stores
    if (g.cs > 0) {  // the stride-2 prologue's source region, zero outside the source frame
        const int S2 = 2 * S0 + 1, sg = g.cis >> 3, stot = S2 * S2 * sg, sy0 = 2 * (y0 - H2) - 1, sx0 = 2 * (x0 - H2) - 1;
        for (int q0 = tid; q0 < stot; q0 += 8 * XB_NT) {
            u32x4 v[8];
            int dst[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int qq = q0 + i * XB_NT;
                v[i] = (u32x4){0u, 0u, 0u, 0u};
                dst[i] = -1;
                if (qq < stot) {
                    const int px = qq / sg, ch = (qq - px * sg) << 3;
                    const int ry = px / S2, rx = px - ry * S2, iy = sy0 + ry, ix = sx0 + rx;
                    dst[i] = g.off_sr + px * g.pss + ch * 2;
                    if (iy >= 0 && iy < 2 * g.H && ix >= 0 && ix < 2 * g.W)
                        v[i] = *(const u32x4*)(g.xs + ((int64_t)(n * 2 * g.H + iy) * 2 * g.W + ix) * g.ldxs + ch);
                }
            }
#pragma unroll
            for (int i = 0; i < 8; ++i)
                if (dst[i] >= 0) *(u32x4*)(smem + dst[i]) = v[i];
        }
    }
    const int cg = (g.ci - g.cs) >> 3, total = S0 * S0 * cg;  // the channels not produced by the prologue
    for (int q0 = tid; q0 < total; q0 += 8 * XB_NT) {
        u32x4 v[8];
        int dst[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int qq = q0 + i * XB_NT;
            v[i] = (u32x4){0u, 0u, 0u, 0u};
            dst[i] = -1;
            if (qq < total) {
                const int px = qq / cg, ch = g.cs + ((qq - px * cg) << 3);
                const int ry = px / S0, rx = px - ry * S0, iy = y0 - H2 + ry, ix = x0 - H2 + rx;
                dst[i] = g.in_off + px * g.psi + ch * 2;
                if (iy >= 0 && iy < g.H && ix >= 0 && ix < g.W) {
                    if (ch < g.cu)
                        v[i] = *(const u32x4*)(g.xu + ((int64_t)(n * (g.H >> 1) + (iy >> 1)) * (g.W >> 1) + (ix >> 1)) *
                                                          g.ldu + ch);
                    else
                        v[i] = *(const u32x4*)(g.x + ((int64_t)(n * g.H + iy) * g.W + ix) * g.ldx + ch);
                }
            }
        }
#pragma unroll
        for (int i = 0; i < 8; ++i)
            if (dst[i] >= 0) *(u32x4*)(smem + dst[i]) = v[i];
    }
    __syncthreads();
    XB_MARK(g, 1);
    const XbIo none = {-1, 0, 0, 0};
    const XbIo r0 = {g.off_r[0], S0, ps0<C>(), 0}, rin = {g.in_off, S0, g.psi, 0};
    // the convs' shapes for the prefetch chain: cv1 (q 0), m.j.cv1 / cv2 (1 .. 2n), cv2 (2n + 1)
    const XbNext n_cv1 = {0, (2 * C) >> 4, (g.ci + 31) >> 5}, n_m = {1, C >> 4, (9 * C + 31) >> 5};
    const XbNext n_cv2 = {2 * NB + 1, (g.co + 15) >> 4, ((2 + NB) * C + 31) >> 5}, n_end = {-1, 1, 0};
    bf16x8 a0[XB_KC];  // the first chunk of the wave's next item (see xb_conv)
    if (g.cs > 0) {  // IN channels [0, cs) = the stride-2 conv of SR (zero outside the frame)
        xb_first(g, 2 * NB + 2, wid % ((g.cs + 15) >> 4), (9 * g.cis + 31) >> 5, lane, a0);
        xb_conv<C, NB, 3>(g, smem, 2 * NB + 2, g.cs, 9 * g.cis, S0, y0 - H2, x0 - H2, n,
                          XbIo{g.off_sr, 2 * S0 + 1, g.pss, 0}, rin, none, lane, wid, a0, n_cv1);
        __syncthreads();
    } else {
        xb_first(g, 0, wid % n_cv1.ncb, n_cv1.ks, lane, a0);
    }
    XB_MARK(g, 2);
    xb_conv<C, NB, 0>(g, smem, 0, 2 * C, g.ci, S0, y0 - H2, x0 - H2, n, rin, r0, none, lane, wid, a0, n_m);
    __syncthreads();
    XB_MARK(g, 3);
#pragma unroll
    for (int j = 0; j < NB; ++j) {
        const int hs = H2 - 2 * j, ws = T + 2 * hs;  // R(2j): halo hs
        const XbIo rin = j == 0 ? XbIo{g.off_r[0], S0, ps0<C>(), C} : XbIo{g.off_r[2 * j], ws, psc<C>(), 0};
        const XbIo rmid = {g.off_r[2 * j + 1], ws - 2, psc<C>(), 0}, rout = {g.off_r[2 * j + 2], ws - 4, psc<C>(), 0};
        xb_conv<C, NB, 1>(g, smem, 1 + 2 * j, C, 9 * C, ws - 2, y0 - hs + 1, x0 - hs + 1, n, rin, rmid, none, lane, wid,
                          a0, XbNext{2 + 2 * j, n_m.ncb, n_m.ks});
        __syncthreads();
        XB_MARK(g, 4 + 2 * j);
        xb_conv<C, NB, 1>(g, smem, 2 + 2 * j, C, 9 * C, ws - 4, y0 - hs + 2, x0 - hs + 2, n, rmid, rout,
                          g.sc ? rin : none, lane, wid, a0, j + 1 < NB ? XbNext{3 + 2 * j, n_m.ncb, n_m.ks} : n_cv2);
        __syncthreads();
        XB_MARK(g, 5 + 2 * j);
    }
    xb_conv<C, NB, 2>(g, smem, 2 * NB + 1, g.co, (2 + NB) * C, T, y0, x0, n, none, none, none, lane, wid, a0, n_end);
    if (g.trace) {
        __syncthreads();
        XB_MARK(g, XB_TR - 1);
    }
}

// ---- the f32 form (the reference's precision: the drop-in call's batch-1 network, FrameProcessor.py:322) ----
// The same block with every value an f32: the regions hold f32 in LDS, each operand is split on read into three exact
// bf16 terms (x = h + m + l, va_seg.hip split3_bf16) and a product is the six term products h.h, h.m, m.h, h.l, m.m,
// l.h accumulated in f32 on the bf16 MFMA -- the arithmetic of the unfused f32 layers (va_seg.hip §f32), in another
// summation order.  The weights come pre-split (three fragments per 16 x 32 tile).  cv1 reads its operand straight
// from global memory (an f32 input region of the wide blocks would not fit beside R0), computing the b half on all
// of R0's pixels and the a half only at the tile's own pixels (R0a).
constexpr int XF_G = 2;   // 16-pixel blocks per work item
constexpr int XF_KC = 4;  // K-steps loaded ahead

struct XfGeom {
    const float* x;
    const float* xu;
    float* y;
    const bf16x8* w;  // three-term fragments: conv q's tile (cb, k) at w + 192 * (wf[q] + cb * ks + k), [3][64]
    const float* b;
    int N, H, W, ci, cu, ldx, ldu, co, ldy;
    int T, tx, tpf, sc;
    int off_r0a;      // LDS offset of R0a (the a half at the tile's T x T pixels)
    int off_r[5];     // R0b (the b half on all of R0), R1 .. R2n
    int wf[6], bo[6];
    unsigned long long* trace;  // debug (va_c2fb_trace), as XbGeom's
    int off_b, nbias;           // the biases' copy in LDS (off_b) and their count
    int off_stg;                // >= 0: cv1's operand staged in LDS from here (xf_cv1_staged), else read per item
};

// cv1's staged operand (PL): K-chunks of XF_SK input channels of the tile's S0 x S0 pixels, as three bf16 planes per
// pixel (stride XF_SPS); XF_UMAX (pixel, 8-channel) units per thread stage a chunk, XF_IMAX items per wave
constexpr int XF_SK = 64, XF_UPP = XF_SK / 8, XF_SPS = 6 * XF_SK + 16, XF_UMAX = 4, XF_IMAX = 4;

template <int C>
constexpr int pf() { return 4 * C + 16; }
// the f32 form's LDS pixel stride: f32 values, or (PL) the three bf16 term planes h | m | l of C channels each
template <int C, bool PL>
constexpr int xps() { return PL ? 6 * C + 16 : 4 * C + 16; }

__device__ __forceinline__ unsigned xf_pk(f32x2 v) {
    typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
    return __builtin_bit_cast(unsigned, __builtin_convertvector(v, bf16x2));
}
__device__ __forceinline__ f32x2 xf_unpk(unsigned p) {
    return (f32x2){__builtin_bit_cast(float, p << 16), __builtin_bit_cast(float, p & 0xffff0000u)};
}
// eight f32 -> three bf16x8 terms, round to nearest even each (va_seg.hip split3_bf16: the same terms)
__device__ __forceinline__ void xf_split3(const f32x4& lo, const f32x4& hi, bf16x8 (&t)[3]) {
    unsigned w[3][4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const f32x4& c = e < 2 ? lo : hi;
        const f32x2 x = {c[2 * (e & 1)], c[2 * (e & 1) + 1]};
        w[0][e] = xf_pk(x);
        const f32x2 r = x - xf_unpk(w[0][e]);
        w[1][e] = xf_pk(r);
        w[2][e] = xf_pk(r - xf_unpk(w[1][e]));
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) t[k] = __builtin_bit_cast(bf16x8, (u32x4){w[k][0], w[k][1], w[k][2], w[k][3]});
}
// four f32 -> their three bf16 terms, four of each (xf_split3's split)
__device__ __forceinline__ void xf_split3x4(const f32x4& v, uint2 (&t)[3]) {
#pragma unroll
    for (int e = 0; e < 2; ++e) {
        const f32x2 x = {v[2 * e], v[2 * e + 1]};
        const unsigned h = xf_pk(x);
        const f32x2 r = x - xf_unpk(h);
        const unsigned m = xf_pk(r);
        const unsigned l = xf_pk(r - xf_unpk(m));
        (e ? t[0].y : t[0].x) = h;
        (e ? t[1].y : t[1].x) = m;
        (e ? t[2].y : t[2].x) = l;
    }
}

__device__ __forceinline__ f32x4 mma6(const bf16x8 (&a)[3], const bf16x8 (&b)[3], f32x4 c) {
    c = mma(a[0], b[0], c);
    c = mma(a[0], b[1], c);
    c = mma(a[1], b[0], c);
    c = mma(a[0], b[2], c);
    c = mma(a[1], b[1], c);
    return mma(a[2], b[0], c);
}

// One f32 conv of the block (xb_conv's roles): KIND 0 = cv1 rows cb0 * 16 .. from global memory onto dst; 1 = 3x3
// from src (+ res); 2 = cv2 over [R0a | R0b | R2 | R4 ..] at the tile's pixels, to g.y.
// PL: the regions hold each value as its three bf16 terms (planes h | m | l per pixel, split once by the producing
// epilogue) instead of f32 -- B fragments read as they are, no split per read (72 per element of a 128-channel 3x3)
template <int C, int NB, int KIND, bool PL>
__device__ __forceinline__ void xf_conv(const XfGeom& g, unsigned char* smem, int q, int cb0, int nout, int kel, int ow,
                                        int oy, int ox, int n, XbIo src, XbIo dst, XbIo res, int lane, int wid) {
    constexpr int EB = PL ? 2 : 4;  // LDS bytes per channel of a plane / per f32
    constexpr int H2 = 2 * NB;
    const int ks = (kel + 31) >> 5, ncb = (nout + 15) >> 4;
    const int P = ow * ow, npb = (P + 15) >> 4, ngr = (npb + XF_G - 1) / XF_G;
    const int items = ngr * ncb;
    const int fr = lane & 15, fq = lane >> 4;
    const int S0 = g.T + 2 * H2;
    for (int it = wid; it < items; it += XB_NW) {
        const int cb = it % ncb, gr = it / ncb;
        const int nb = min(XF_G, npb - gr * XF_G);
        int pr[XF_G], pc[XF_G], base[XF_G];
        int64_t gx[XF_G], gu[XF_G];  // KIND 0: element offsets of the pixel in x / xu (-1: outside the frame)
#pragma unroll
        for (int j = 0; j < XF_G; ++j) {
            int p = ((gr * XF_G + j) << 4) + fr;
            p = p < P ? p : P - 1;
            const int r = p / ow, c = p - r * ow;
            pr[j] = r;
            pc[j] = c;
            base[j] = KIND == 1 ? src.off + (r * src.w + c) * src.ps : 0;
            if constexpr (KIND == 0) {
                const int iy = oy + r, ix = ox + c;
                const bool in = iy >= 0 && iy < g.H && ix >= 0 && ix < g.W;
                gx[j] = in ? ((int64_t)(n * g.H + iy) * g.W + ix) * g.ldx : -1;
                gu[j] = in ? ((int64_t)(n * (g.H >> 1) + (iy >> 1)) * (g.W >> 1) + (ix >> 1)) * g.ldu : -1;
            }
        }
        f32x4 acc[XF_G];
#pragma unroll
        for (int j = 0; j < XF_G; ++j) acc[j] = (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
        const bf16x8* wb = g.w + (int64_t)192 * (g.wf[q] + (cb0 + cb) * ks) + lane;
        // the lane's B element offset for K-step k of block j (LDS byte offset; KIND 0: handled in load_b)
        auto lds_addr = [&](int k, int j) {
            const int kk = min((k << 5) + (fq << 3), kel - 8);
            if constexpr (KIND == 1) {
                const int tap = kk / C, ch = kk - tap * C, ky = tap / 3, kx = tap - 3 * ky;
                return base[j] + (ky * src.w + kx) * src.ps + ch * EB;
            } else {
                if (kk < C) return g.off_r0a + (pr[j] * g.T + pc[j]) * xps<C, PL>() + kk * EB;
                if (kk < 2 * C) return g.off_r[0] + ((pr[j] + H2) * S0 + pc[j] + H2) * xps<C, PL>() + (kk - C) * EB;
                const int s = (kk - 2 * C) / C + 1, ch = kk - (s + 1) * C;
                const int hs = H2 - 2 * s, ws = g.T + 2 * hs;
                return g.off_r[2 * s] + ((pr[j] + hs) * ws + pc[j] + hs) * xps<C, PL>() + ch * EB;
            }
        };
        // K-steps in chunks of KC, double-buffered: the next chunk's A fragments (and, for cv1, its B operands from
        // global memory) are in flight while this chunk's MFMAs run; B from LDS is read as it is used
        constexpr int KC = KIND == 0 ? 2 : XF_KC;
        bf16x8 a0[KC][3], a1[KC][3];
        f32x4 b0[KC][XF_G][2], b1[KC][XF_G][2];
        // loads unconditional (clamped to the last step / a real pixel, zeros selected after): a fixed count in
        // flight for counted waits
        auto load = [&](bf16x8 (&a)[KC][3], f32x4 (&bv)[KC][XF_G][2], int k0) {
#pragma unroll
            for (int i = 0; i < KC; ++i) {
                const int kc = min(k0 + i, ks - 1);
#pragma unroll
                for (int t = 0; t < 3; ++t) a[i][t] = wb[192 * kc + 64 * t];
                if constexpr (KIND == 0) {
                    const int kk = min((kc << 5) + (fq << 3), kel - 8);
                    const bool up = kk < g.cu;
#pragma unroll
                    for (int j = 0; j < XF_G; ++j) {
                        const int64_t o = up ? gu[j] : gx[j];
                        const float* p = (up ? g.xu : g.x) + (o >= 0 ? o : 0) + kk;
                        const f32x4 z = {0.0f, 0.0f, 0.0f, 0.0f}, v0 = *(const f32x4*)p, v1 = *(const f32x4*)(p + 4);
                        bv[i][j][0] = o >= 0 ? v0 : z;
                        bv[i][j][1] = o >= 0 ? v1 : z;
                    }
                }
            }
        };
        auto compute = [&](const bf16x8 (&a)[KC][3], const f32x4 (&bv)[KC][XF_G][2], int k0) {
#pragma unroll
            for (int i = 0; i < KC; ++i) {
                if (k0 + i < ks) {
                    f32x4 lv[XF_G][2];
                    bf16x8 pv[XF_G][3];
                    if constexpr (KIND != 0 && PL) {  // the blocks' three term fragments, read as they are
#pragma unroll
                        for (int j = 0; j < XF_G; ++j) {
                            const unsigned char* p = smem + lds_addr(k0 + i, j);
#pragma unroll
                            for (int t = 0; t < 3; ++t) pv[j][t] = *(const bf16x8*)(p + 2 * C * t);
                        }
#pragma unroll
                        for (int j = 0; j < XF_G; ++j) asm volatile("" ::"v"(pv[j][0]), "v"(pv[j][1]), "v"(pv[j][2]));
                    } else if constexpr (KIND != 0) {  // the blocks' LDS reads together, then their splits and MFMAs
#pragma unroll
                        for (int j = 0; j < XF_G; ++j) {
                            const unsigned char* p = smem + lds_addr(k0 + i, j);
                            lv[j][0] = *(const f32x4*)p;
                            lv[j][1] = *(const f32x4*)(p + 16);
                        }
#pragma unroll
                        for (int j = 0; j < XF_G; ++j) asm volatile("" ::"v"(lv[j][0]), "v"(lv[j][1]));  // (as xb_conv)
                    }
#pragma unroll
                    for (int j = 0; j < XF_G; ++j) {
                        if (j < nb) {  // (unguarded, the bf16 form's live blocks went non-finite: kept guarded)
                            if constexpr (KIND != 0 && PL) {
                                acc[j] = mma6(a[i], pv[j], acc[j]);
                            } else {
                                bf16x8 bt[3];
                                if constexpr (KIND == 0) xf_split3(bv[i][j][0], bv[i][j][1], bt);
                                else xf_split3(lv[j][0], lv[j][1], bt);
                                acc[j] = mma6(a[i], bt, acc[j]);
                            }
                        }
                    }
                }
            }
        };
        load(a0, b0, 0);
        for (int k0 = 0; k0 < ks; k0 += 2 * KC) {
            load(a1, b1, k0 + KC);
            compute(a0, b0, k0);
            load(a0, b0, k0 + 2 * KC);
            compute(a1, b1, k0 + KC);
        }
        const int co = (cb << 4) + (fq << 2);
        if (co >= nout) continue;
        const f32x4 bias = *(const f32x4*)(smem + g.off_b + (g.bo[q] + 16 * cb0 + co) * 4);
#pragma unroll
        for (int j = 0; j < XF_G; ++j) {
            const int p = ((gr * XF_G + j) << 4) + fr;
            if (j >= nb || p >= P) continue;
            const int r = pr[j], c = pc[j], iy = oy + r, ix = ox + c;
            const bool in = iy >= 0 && iy < g.H && ix >= 0 && ix < g.W;
            f32x4 v = fz::act(acc[j] + bias);
            if (KIND == 1 && res.off >= 0) {
                const unsigned char* rp = smem + res.off + ((r + 2) * res.w + c + 2) * res.ps + (res.c0 + co) * EB;
                if constexpr (PL) {  // (h + m) + l: exact (the split's terms sum back to the value)
                    const uint2 h = *(const uint2*)rp, m = *(const uint2*)(rp + 2 * C), l = *(const uint2*)(rp + 4 * C);
                    const f32x2 h0 = xf_unpk(h.x), h1 = xf_unpk(h.y), m0 = xf_unpk(m.x), m1 = xf_unpk(m.y);
                    const f32x2 l0 = xf_unpk(l.x), l1 = xf_unpk(l.y);
                    v += (f32x4){(h0[0] + m0[0]) + l0[0], (h0[1] + m0[1]) + l0[1], (h1[0] + m1[0]) + l1[0],
                                 (h1[1] + m1[1]) + l1[1]};
                } else {
                    v += *(const f32x4*)rp;
                }
            }
            if constexpr (KIND == 2) {
                if (in) *(f32x4*)(g.y + ((int64_t)(n * g.H + iy) * g.W + ix) * g.ldy + co) = v;
            } else {
                if (!in) v = (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
                unsigned char* dp = smem + dst.off + p * dst.ps + (dst.c0 + co) * EB;
                if constexpr (PL) {  // split once here for every later read
                    uint2 t3[3];
                    xf_split3x4(v, t3);
#pragma unroll
                    for (int t = 0; t < 3; ++t) *(uint2*)(dp + 2 * C * t) = t3[t];
                } else {
                    *(f32x4*)dp = v;
                }
            }
        }
    }
}

// cv1 (both halves: b on all S0 x S0 pixels -> R0b, a on the T x T centre -> R0a) with its operand staged: per K-chunk
// of XF_SK channels the tile's input pixels are loaded from global memory once (the next chunk's in flight under this
// chunk's MFMAs), split once into their three bf16 terms and stored as planes past R0a (R1 .. are not written yet);
// every output-channel item then reads its B fragments from there as they are.  The per-item form (xf_conv KIND 0)
// loads and splits each input element once per 16 output channels: 2C / 16 times.  Items (half, 16 output channels,
// XF_G pixel blocks) as xf_conv's, at most XF_IMAX per wave (the host's condition), their accumulators held across
// the chunks; the same K order, so the same sums.
template <int C, int NB>
__device__ __forceinline__ void xf_cv1_staged(const XfGeom& g, unsigned char* smem, int y0, int x0, int n, XbIo r0b,
                                              XbIo r0a, int lane, int wid) {
    constexpr int H2 = 2 * NB, NCB = C / 16, SKS = XF_SK / 32;
    const int T = g.T, S0 = T + 2 * H2, PB = S0 * S0, PA = T * T;
    const int ngrB = (((PB + 15) >> 4) + XF_G - 1) / XF_G, ngrA = (((PA + 15) >> 4) + XF_G - 1) / XF_G;
    const int itB = ngrB * NCB, items = itB + ngrA * NCB;
    const int fr = lane & 15, fq = lane >> 4, tid = threadIdx.x;
    const int ks = (g.ci + 31) >> 5, nch = (g.ci + XF_SK - 1) / XF_SK;
    unsigned char* stg = smem + g.off_stg;
    f32x4 acc[XF_IMAX][XF_G];
    int sp[XF_IMAX][XF_G];  // the lane's staged pixel per block (its row of the block)
    int nbk[XF_IMAX];       // live blocks of the item (0: no item)
    const bf16x8* wb[XF_IMAX];
#pragma unroll
    for (int i = 0; i < XF_IMAX; ++i) {
        const int it = wid + XB_NW * i;
        const bool hb = it < itB;
        const int loc = hb ? it : it - itB, cb = loc % NCB, gr = loc / NCB;
        const int ow = hb ? S0 : T, P = hb ? PB : PA;
        nbk[i] = it < items ? min(XF_G, ((P + 15) >> 4) - gr * XF_G) : 0;
        wb[i] = g.w + (int64_t)192 * (g.wf[0] + ((hb ? NCB : 0) + cb) * ks) + lane;
#pragma unroll
        for (int j = 0; j < XF_G; ++j) {
            acc[i][j] = (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
            const int p = min(((gr * XF_G + j) << 4) + fr, P - 1), r = p / ow, c = p - r * ow;
            sp[i][j] = hb ? p : (r + H2) * S0 + c + H2;
        }
    }
    // staging units u = tid + XB_NT m: pixel u / XF_UPP, channels 8 (u % XF_UPP) .. of the chunk
    f32x4 rv[XF_UMAX][2];
    auto load_units = [&](int ch) {
#pragma unroll
        for (int m = 0; m < XF_UMAX; ++m) {
            const int u = tid + XB_NT * m, px = u / XF_UPP, k = ch * XF_SK + ((u % XF_UPP) << 3);
            const int r = px / S0, c = px - r * S0, iy = y0 - H2 + r, ix = x0 - H2 + c;
            const bool live = px < PB && k < g.ci && iy >= 0 && iy < g.H && ix >= 0 && ix < g.W;
            const bool up = k < g.cu;
            const int64_t o = live ? (up ? ((int64_t)(n * (g.H >> 1) + (iy >> 1)) * (g.W >> 1) + (ix >> 1)) * g.ldu
                                         : ((int64_t)(n * g.H + iy) * g.W + ix) * g.ldx) + k : 0;
            const float* p = (live && up ? g.xu : g.x) + o;
            const f32x4 z = {0.0f, 0.0f, 0.0f, 0.0f}, v0 = *(const f32x4*)p, v1 = *(const f32x4*)(p + 4);
            rv[m][0] = live ? v0 : z;
            rv[m][1] = live ? v1 : z;
        }
    };
    auto store_units = [&]() {
#pragma unroll
        for (int m = 0; m < XF_UMAX; ++m) {
            const int u = tid + XB_NT * m, px = u / XF_UPP;
            if (px < PB) {
                bf16x8 t3[3];
                xf_split3(rv[m][0], rv[m][1], t3);
                unsigned char* d = stg + px * XF_SPS + ((u % XF_UPP) << 4);
#pragma unroll
                for (int t = 0; t < 3; ++t) *(bf16x8*)(d + 2 * XF_SK * t) = t3[t];
            }
        }
    };
    // item i's A fragments of chunk ch (both K-steps; clamped to the last step: a fixed count in flight)
    bf16x8 a[XF_IMAX][SKS][3];
    auto load_a = [&](int i, int ch) {
#pragma unroll
        for (int s = 0; s < SKS; ++s) {
            const int k = min(ch * SKS + s, ks - 1);
#pragma unroll
            for (int t = 0; t < 3; ++t) a[i][s][t] = wb[i][192 * k + 64 * t];
        }
    };
#pragma unroll
    for (int i = 0; i < XF_IMAX; ++i) load_a(i, 0);
    load_units(0);
    for (int ch = 0; ch < nch; ++ch) {
        // the staged operand, then the next chunk's loads in flight under this chunk's MFMAs: its input pixels, and
        // each item's A fragments as soon as the item is done with this chunk's
        store_units();
        __syncthreads();
        if (ch + 1 < nch) load_units(ch + 1);
#pragma unroll
        for (int i = 0; i < XF_IMAX; ++i) {
            if (nbk[i] == 0) continue;  // wave-uniform
#pragma unroll
            for (int s = 0; s < SKS; ++s) {
                if (ch * SKS + s >= ks) continue;
                bf16x8 pv[XF_G][3];
#pragma unroll
                for (int j = 0; j < XF_G; ++j) {
                    const unsigned char* p = stg + sp[i][j] * XF_SPS + ((s * 32 + 8 * fq) << 1);
#pragma unroll
                    for (int t = 0; t < 3; ++t) pv[j][t] = *(const bf16x8*)(p + 2 * XF_SK * t);
                }
#pragma unroll
                for (int j = 0; j < XF_G; ++j) asm volatile("" ::"v"(pv[j][0]), "v"(pv[j][1]), "v"(pv[j][2]));
#pragma unroll
                for (int j = 0; j < XF_G; ++j)
                    if (j < nbk[i]) acc[i][j] = mma6(a[i][s], pv[j], acc[i][j]);
            }
            load_a(i, ch + 1);
        }
        __syncthreads();  // the chunk read by every item before the next one is stored
    }
    // epilogue (xf_conv's, KIND 0): bias + SiLU, zero outside the frame, split once into the region's planes
#pragma unroll
    for (int i = 0; i < XF_IMAX; ++i) {
        if (nbk[i] == 0) continue;
        const int it = wid + XB_NW * i;
        const bool hb = it < itB;
        const int loc = hb ? it : it - itB, cb = loc % NCB, gr = loc / NCB;
        const int ow = hb ? S0 : T, P = hb ? PB : PA, oy = hb ? y0 - H2 : y0, ox = hb ? x0 - H2 : x0;
        const XbIo dst = hb ? r0b : r0a;
        const int co = (cb << 4) + (fq << 2);
        const f32x4 bias = *(const f32x4*)(smem + g.off_b + (g.bo[0] + (hb ? C : 0) + co) * 4);
#pragma unroll
        for (int j = 0; j < XF_G; ++j) {
            const int p = ((gr * XF_G + j) << 4) + fr;
            if (j >= nbk[i] || p >= P) continue;
            const int r = p / ow, c = p - r * ow, iy = oy + r, ix = ox + c;
            const bool in = iy >= 0 && iy < g.H && ix >= 0 && ix < g.W;
            f32x4 v = fz::act(acc[i][j] + bias);
            if (!in) v = (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
            uint2 t3[3];
            xf_split3x4(v, t3);
            unsigned char* dp = smem + dst.off + p * dst.ps + (dst.c0 + co) * 2;
#pragma unroll
            for (int t = 0; t < 3; ++t) *(uint2*)(dp + 2 * C * t) = t3[t];
        }
    }
}

template <int C, int NB, bool PL>
__global__ __launch_bounds__(XB_NT) void c2fbf_kernel(XfGeom g) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr int H2 = 2 * NB;
    const int T = g.T, S0 = T + 2 * H2;
    const int t = blockIdx.x, n = t / g.tpf, tt = t - n * g.tpf, ty = tt / g.tx, tx = tt - ty * g.tx;
    const int y0 = ty * T, x0 = tx * T;
    // the wave index as a scalar: item / block / guard arithmetic derived from it stays wave-uniform (scalar branches)
    const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const XbIo none = {-1, 0, 0, 0};
    const XbIo r0b = {g.off_r[0], S0, xps<C, PL>(), 0}, r0a = {g.off_r0a, T, xps<C, PL>(), 0};
    XB_MARK(g, 0);
    xb_bias_to_lds(g.b, g.nbias, smem, g.off_b);
    __syncthreads();
    if (PL && g.off_stg >= 0) {  // kernel-uniform
        xf_cv1_staged<C, NB>(g, smem, y0, x0, n, r0b, r0a, lane, wid);
    } else {
        xf_conv<C, NB, 0, PL>(g, smem, 0, C / 16, C, g.ci, S0, y0 - H2, x0 - H2, n, none, r0b, none, lane, wid);
        if (g.trace) {
            __syncthreads();
            XB_MARK(g, 1);
        }
        xf_conv<C, NB, 0, PL>(g, smem, 0, 0, C, g.ci, T, y0, x0, n, none, r0a, none, lane, wid);
    }
    __syncthreads();
    XB_MARK(g, 3);
#pragma unroll
    for (int j = 0; j < NB; ++j) {
        const int hs = H2 - 2 * j, ws = T + 2 * hs;
        const XbIo rin = j == 0 ? r0b : XbIo{g.off_r[2 * j], ws, xps<C, PL>(), 0};
        const XbIo rmid = {g.off_r[2 * j + 1], ws - 2, xps<C, PL>(), 0};
        const XbIo rout = {g.off_r[2 * j + 2], ws - 4, xps<C, PL>(), 0};
        xf_conv<C, NB, 1, PL>(g, smem, 1 + 2 * j, 0, C, 9 * C, ws - 2, y0 - hs + 1, x0 - hs + 1, n, rin, rmid, none, lane,
                          wid);
        __syncthreads();
        XB_MARK(g, 4 + 2 * j);
        xf_conv<C, NB, 1, PL>(g, smem, 2 + 2 * j, 0, C, 9 * C, ws - 4, y0 - hs + 2, x0 - hs + 2, n, rmid, rout,
                          g.sc ? rin : none, lane, wid);
        __syncthreads();
        XB_MARK(g, 5 + 2 * j);
    }
    xf_conv<C, NB, 2, PL>(g, smem, 2 * NB + 1, 0, g.co, (2 + NB) * C, T, y0, x0, n, none, none, none, lane, wid);
    if (g.trace) {
        __syncthreads();
        XB_MARK(g, XB_TR - 1);
    }
}

// f32 LDS layout: [R0b][R0a][R1] .. [R2n]; returns the bytes (or -1)
int xf_layout(int C, int NB, int T, int* off_r0a, int* off_r, bool pl = false) {
    if (T < 1 || T > 64) return -1;
    const int S0 = T + 4 * NB, ps = pl ? 6 * C + 16 : 4 * C + 16;
    int64_t o = (int64_t)S0 * S0 * ps;
    off_r[0] = 0;
    *off_r0a = (int)o;
    o += (int64_t)T * T * ps;
    for (int j = 1; j <= 2 * NB; ++j) {
        const int s = T + 2 * (2 * NB - j);
        off_r[j] = (int)o;
        o += (int64_t)s * s * ps;
    }
    return o > XB_LDS_MAX ? -1 : (int)o;
}

template <int C, int NB>
hipError_t xf_launch(const XfGeom& g, int lds, int ntiles, hipStream_t st, bool pl) {
    static DevFlag attr;
    if (!attr()) {
        if (hipFuncSetAttribute((const void*)c2fbf_kernel<C, NB, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                XB_LDS_MAX) != hipSuccess ||
            hipFuncSetAttribute((const void*)c2fbf_kernel<C, NB, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                XB_LDS_MAX) != hipSuccess)
            return hipErrorInvalidValue;
        attr() = true;
    }
    if (pl)
        hipLaunchKernelGGL((c2fbf_kernel<C, NB, true>), dim3(ntiles), dim3(XB_NT), lds, st, g);
    else
        hipLaunchKernelGGL((c2fbf_kernel<C, NB, false>), dim3(ntiles), dim3(XB_NT), lds, st, g);
    return hipGetLastError();
}

// cv1's operand staged (xf_cv1_staged, term-plane layouts) where its chunk fits from R1 on (moving the biases up if it
// reaches past the regions), its units fit XF_UMAX per thread and its items XF_IMAX per wave: *off_stg (else -1);
// returns the biases' LDS offset
int xf_stage(int C, int NB, int T, bool pl, int lds, int nbias, int off_r1, int* off_stg) {
    const int S0 = T + 4 * NB, pb = S0 * S0;
    auto groups = [](int p) { return ((p + 15) / 16 + XF_G - 1) / XF_G; };
    const int items = (C / 16) * (groups(pb) + groups(T * T));
    const int end = off_r1 + pb * XF_SPS, ob = end > lds ? (end + 15) & ~15 : lds;
    *off_stg = -1;
    if (!pl || pb * XF_UPP > XB_NT * XF_UMAX || items > XB_NW * XF_IMAX || ob + 4 * nbias > XB_LDS_MAX) return lds;
    *off_stg = off_r1;
    return ob;
}

// the f32 form's layout: the term planes where they fit the LDS with the biases, else f32 (*pl says which)
int xf_choose(int C, int NB, int T, int nbias, int* off_r0a, int* off_r, bool* pl) {
    int lds = xf_layout(C, NB, T, off_r0a, off_r, true);
    *pl = lds >= 0 && lds + 4 * nbias <= XB_LDS_MAX;
    if (!*pl) lds = xf_layout(C, NB, T, off_r0a, off_r, false);
    return lds;
}

// LDS layout of one configuration: [R0][IN, later R1 .. R2n]; returns the bytes (or -1)
int xb_layout(int C, int NB, int ci, int T, int* off_r, int* in_off, int* psi, int cis = 0, int* off_sr = nullptr,
              int* pss = nullptr) {
    if (T < 1 || T > 64) return -1;
    const int S0 = T + 4 * NB, S2 = 2 * S0 + 1;
    const int64_t r0 = (int64_t)S0 * S0 * (4 * C + 16);
    int64_t in = (int64_t)S0 * S0 * (2 * ci + 16);
    if (cis > 0) {  // the prologue's source region after IN (both dead once cv1 has run)
        *off_sr = (int)(r0 + in);
        *pss = 2 * cis + 16;
        in += (int64_t)S2 * S2 * (2 * cis + 16);
    }
    int64_t rs = 0;
    off_r[0] = 0;
    for (int j = 1; j <= 2 * NB; ++j) {
        const int s = T + 2 * (2 * NB - j);
        off_r[j] = (int)(r0 + rs);
        rs += (int64_t)s * s * (2 * C + 16);
    }
    *in_off = (int)r0;
    *psi = 2 * ci + 16;
    const int64_t tot = r0 + (in > rs ? in : rs);
    return tot > XB_LDS_MAX ? -1 : (int)tot;
}

// fragment / bias offsets of the blob (seg.py SegNet._pack_c2fb): conv q = cv1, m.0.cv1, m.0.cv2, .., cv2, each
// [ceil(nout / 16)][ceil(K / 32)] fragments and 16 ceil(nout / 16) biases; returns the totals
void xb_blob(int C, int NB, int ci, int co, int* wf, int* bo, int64_t* frags, int64_t* biases, int cs = 0,
             int cis = 0) {
    int64_t f = 0, b = 0;
    for (int q = 0; q < 2 * NB + 2 + (cs > 0); ++q) {
        const int nout = q == 0 ? 2 * C : q == 2 * NB + 1 ? co : q == 2 * NB + 2 ? cs : C;
        const int k = q == 0 ? ci : q == 2 * NB + 1 ? (2 + NB) * C : q == 2 * NB + 2 ? 9 * cis : 9 * C;
        wf[q] = (int)f;
        bo[q] = (int)b;
        f += (int64_t)((nout + 15) / 16) * ((k + 31) / 32);
        b += 16 * ((nout + 15) / 16);
    }
    *frags = f;
    *biases = b;
}

template <int C, int NB>
hipError_t xb_launch(const XbGeom& g, int lds, int ntiles, hipStream_t st) {
    static DevFlag attr;
    if (!attr()) {
        if (hipFuncSetAttribute((const void*)c2fb_kernel<C, NB>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                XB_LDS_MAX) != hipSuccess)
            return hipErrorInvalidValue;
        attr() = true;
    }
    hipLaunchKernelGGL((c2fb_kernel<C, NB>), dim3(ntiles), dim3(XB_NT), lds, st, g);
    return hipGetLastError();
}

// the stride-2 prologue: cs output channels (a multiple of 16, at most ci), cis input channels (a power of two >= 8)
bool xb_s2_ok(int ci, int cs, int cis) {
    return cs > 0 && cs % 16 == 0 && cs <= ci && cis >= 8 && cis <= 512 && (cis & (cis - 1)) == 0;
}

unsigned long long* g_xb_trace = nullptr;  // va_c2fb_trace

bool xb_shape_ok(int C, int NB, bool f32 = false) {
    return (C == 16 || C == 32 || C == 64 || C == 128 || (f32 && C == 256)) && (NB == 1 || NB == 2);
}

}  // namespace

extern "C" int va_c2fb_layout(int32_t c, int32_t n, int32_t ci, int32_t co, int32_t T, int32_t dtype, int32_t cs,
                              int32_t cis, int64_t* out3) {
    const bool f32 = dtype == VA_DTYPE_F32;
    if (!out3 || !xb_shape_ok(c, n, f32) || ci <= 0 || co <= 0 || (!f32 && dtype != VA_DTYPE_BF16) ||
        (cs && (f32 || !xb_s2_ok(ci, cs, cis))))
        return VA_ERR_ARG;
    int off_r[5], in_off, psi, wf[7], bo[7], off_sr, pss;
    int64_t fr, nbias;
    xb_blob(c, n, ci, co, wf, bo, &fr, &nbias, cs, cis);
    bool pl;
    const int lds = f32 ? xf_choose(c, n, T, (int)nbias, &in_off, off_r, &pl)
                        : xb_layout(c, n, ci, T, off_r, &in_off, &psi, cs ? cis : 0, &off_sr, &pss);
    xb_blob(c, n, ci, co, wf, bo, &out3[1], &out3[2], cs, cis);
    if (f32) out3[1] *= 3;  // three term fragments per tile
    int off_stg;
    const int ob = f32 && lds >= 0 ? xf_stage(c, n, T, pl, lds, (int)nbias, off_r[1], &off_stg) : lds;
    out3[0] = lds < 0 ? -1 : ob + 4 * out3[2];  // + the biases' LDS copy
    out3[3] = f32 && pl;
    return lds < 0 || out3[0] > XB_LDS_MAX ? VA_ERR_ARG : VA_OK;
}

static int c2fb_f32(const va_conv_args* a, hipStream_t st);

extern "C" int va_seg_c2fb(void* stream, const va_conv_args* a) {
    if (!a || !a->x || !a->w || !a->bias || !a->y || (a->dtype != VA_DTYPE_BF16 && a->dtype != VA_DTYPE_F32))
        return VA_ERR_ARG;
    if (a->dtype == VA_DTYPE_F32) return c2fb_f32(a, (hipStream_t)stream);
    const int C = a->Npad, NB = a->kh, T = a->stride, ci = a->Cin, co = a->Cout;
    if (!xb_shape_ok(C, NB) || a->N <= 0 || a->H <= 0 || a->W <= 0 || ci % 8 || co % 16 || ci <= 0 || co <= 0 ||
        a->ldx % 8 || a->ldy % 8 || a->ldx < ci || a->ldy < co || ((uintptr_t)a->x & 15) || ((uintptr_t)a->y & 15) ||
        ((uintptr_t)a->w & 15) || ((uintptr_t)a->bias & 15))
        return VA_ERR_ARG;
    if (a->xu && (a->cu <= 0 || a->cu % 8 || a->cu >= ci || a->ldu % 8 || a->ldu < a->cu || a->H % 2 || a->W % 2 ||
                  ((uintptr_t)a->xu & 15)))
        return VA_ERR_ARG;
    // the stride-2 prologue (a.res = its source xs, a.ldr = ldxs, a.c2 = cs, a.K = cis)
    const int cs = a->res ? a->c2 : 0, cis = a->res ? a->K : 0;
    if (cs && (!xb_s2_ok(ci, cs, cis) || a->xu || a->ldr % 8 || a->ldr < cis || ((uintptr_t)a->res & 15)))
        return VA_ERR_ARG;
    XbGeom g;
    const int lds = xb_layout(C, NB, ci, T, g.off_r, &g.in_off, &g.psi, cis, &g.off_sr, &g.pss);
    if (lds < 0) return VA_ERR_ARG;
    int64_t frags, biases;
    xb_blob(C, NB, ci, co, g.wf, g.bo, &frags, &biases, cs, cis);
    g.off_b = lds, g.nbias = (int)biases;  // the biases' LDS copy after the layout (16-byte multiples: biases % 16 == 0)
    const int lds_b = lds + (int)biases * 4;
    if (lds_b > XB_LDS_MAX) return VA_ERR_ARG;
    g.trace = g_xb_trace;
    g.xs = (const __bf16*)a->res;
    g.ldxs = a->ldr, g.cs = cs, g.cis = cis, g.lgcis = cs ? 31 - __builtin_clz(cis) : 0;
    g.x = (const __bf16*)a->x;
    g.xu = (const __bf16*)a->xu;
    g.y = (__bf16*)a->y;
    g.w = (const bf16x8*)a->w;
    g.b = a->bias;
    g.N = a->N, g.H = a->H, g.W = a->W, g.ci = ci, g.cu = a->xu ? a->cu : 0, g.ldx = a->ldx, g.ldu = a->ldu;
    g.co = co, g.ldy = a->ldy, g.T = T, g.sc = a->kw ? 1 : 0;
    g.tx = (a->W + T - 1) / T;
    const int64_t tpf = (int64_t)g.tx * ((a->H + T - 1) / T), nt = tpf * a->N;
    if (nt > INT32_MAX) return VA_ERR_ARG;
    g.tpf = (int)tpf;
    hipStream_t st = (hipStream_t)stream;
    hipError_t rc;
    switch (C * 4 + NB) {
        case 16 * 4 + 1: rc = xb_launch<16, 1>(g, lds_b, (int)nt, st); break;
        case 16 * 4 + 2: rc = xb_launch<16, 2>(g, lds_b, (int)nt, st); break;
        case 32 * 4 + 1: rc = xb_launch<32, 1>(g, lds_b, (int)nt, st); break;
        case 32 * 4 + 2: rc = xb_launch<32, 2>(g, lds_b, (int)nt, st); break;
        case 64 * 4 + 1: rc = xb_launch<64, 1>(g, lds_b, (int)nt, st); break;
        case 64 * 4 + 2: rc = xb_launch<64, 2>(g, lds_b, (int)nt, st); break;
        case 128 * 4 + 1: rc = xb_launch<128, 1>(g, lds_b, (int)nt, st); break;
        default: rc = xb_launch<128, 2>(g, lds_b, (int)nt, st); break;
    }
    return rc == hipSuccess ? VA_OK : VA_ERR_HIP;
}

static int c2fb_f32(const va_conv_args* a, hipStream_t st) {
    const int C = a->Npad, NB = a->kh, T = a->stride, ci = a->Cin, co = a->Cout;
    if (!xb_shape_ok(C, NB, true) || a->N <= 0 || a->H <= 0 || a->W <= 0 || ci % 8 || co % 16 || ci <= 0 || co <= 0 ||
        a->ldx % 4 || a->ldy % 4 || a->ldx < ci || a->ldy < co || ((uintptr_t)a->x & 15) || ((uintptr_t)a->y & 15) ||
        ((uintptr_t)a->w & 15) || ((uintptr_t)a->bias & 15))
        return VA_ERR_ARG;
    // the stride-2 prologue (a->res / c2 / K) is a bf16 form only (va_c2fb_layout rejects cs for f32 as well): an f32
    // call that names one would compute the block from x's first cs channels, which nobody wrote
    if (a->res || a->c2 || a->K) return VA_ERR_ARG;
    if (a->xu && (a->cu <= 0 || a->cu % 8 || a->cu >= ci || a->ldu % 4 || a->ldu < a->cu || a->H % 2 || a->W % 2 ||
                  ((uintptr_t)a->xu & 15)))
        return VA_ERR_ARG;
    XfGeom g;
    int64_t frags, biases;
    xb_blob(C, NB, ci, co, g.wf, g.bo, &frags, &biases);
    bool pl;
    const int lds = xf_choose(C, NB, T, (int)biases, &g.off_r0a, g.off_r, &pl);
    if (lds < 0) return VA_ERR_ARG;
    g.nbias = (int)biases;
    g.off_b = xf_stage(C, NB, T, pl, lds, (int)biases, g.off_r[1], &g.off_stg);
    const int lds_b = g.off_b + (int)biases * 4;
    if (lds_b > XB_LDS_MAX) return VA_ERR_ARG;
    g.trace = g_xb_trace;
    g.x = (const float*)a->x;
    g.xu = (const float*)a->xu;
    g.y = (float*)a->y;
    g.w = (const bf16x8*)a->w;
    g.b = a->bias;
    g.N = a->N, g.H = a->H, g.W = a->W, g.ci = ci, g.cu = a->xu ? a->cu : 0, g.ldx = a->ldx, g.ldu = a->ldu;
    g.co = co, g.ldy = a->ldy, g.T = T, g.sc = a->kw ? 1 : 0;
    g.tx = (a->W + T - 1) / T;
    const int64_t tpf = (int64_t)g.tx * ((a->H + T - 1) / T), nt = tpf * a->N;
    if (nt > INT32_MAX) return VA_ERR_ARG;
    g.tpf = (int)tpf;
    hipError_t rc;
    switch (C * 4 + NB) {
        case 16 * 4 + 1: rc = xf_launch<16, 1>(g, lds_b, (int)nt, st, pl); break;
        case 16 * 4 + 2: rc = xf_launch<16, 2>(g, lds_b, (int)nt, st, pl); break;
        case 32 * 4 + 1: rc = xf_launch<32, 1>(g, lds_b, (int)nt, st, pl); break;
        case 32 * 4 + 2: rc = xf_launch<32, 2>(g, lds_b, (int)nt, st, pl); break;
        case 64 * 4 + 1: rc = xf_launch<64, 1>(g, lds_b, (int)nt, st, pl); break;
        case 64 * 4 + 2: rc = xf_launch<64, 2>(g, lds_b, (int)nt, st, pl); break;
        case 128 * 4 + 1: rc = xf_launch<128, 1>(g, lds_b, (int)nt, st, pl); break;
        case 128 * 4 + 2: rc = xf_launch<128, 2>(g, lds_b, (int)nt, st, pl); break;
        case 256 * 4 + 1: rc = xf_launch<256, 1>(g, lds_b, (int)nt, st, pl); break;
        default: rc = xf_launch<256, 2>(g, lds_b, (int)nt, st, pl); break;
    }
    return rc == hipSuccess ? VA_OK : VA_ERR_HIP;
}

// Debug: stage clocks of the next va_seg_c2fb launches into device memory buf ([grid][10] uint64: s_memtime of thread 0
// at the start, after each stage's barrier, and at the end), or stop (NULL)
extern "C" int va_c2fb_trace(void* buf) {
    g_xb_trace = (unsigned long long*)buf;
    return VA_OK;
}

// va_contour.hip -- the mask -> polygon -> cells boundary of FrameProcessor.py:67-97 on MI355X (gfx950).
//
// The reference reduces the chosen YOLO mask to grid cells through OpenCV (Results.masks.xy = masks2segments
// (findContours RETR_EXTERNAL / CHAIN_APPROX_SIMPLE, the contour with the most points) + scale_coords, then
// max(xy, key=contourArea), np.int32, boundingRect, fillPoly, cell-centre sampling).  OpenCV is third-party and
// absent here; its published algorithms are restated exactly as oracle/contours.py restates them (that module is
// the checker; the cv2 parity itself is unpinned):
//
//   post_contour_kernel  one wave per detection (persistent over the detections): the instance mask --
//                        bilinear x4 of the cropped coef . proto, > 0 (process_mask), or a given binary mask --
//                        as a framed image of three bit planes (mask, traced, traced "right") in LDS, built in strips
//                        of low-res rows; its pixel count and bbox (va_mask_stat); the raster scan of
//                        cvFindNextContour over the rows that hold an unmarked 0 -> 1 transition (no other row
//                        can start an outer border) and Suzuki-Abe border following (icvFetchContour) for every
//                        outer border RETR_EXTERNAL keeps, each contour's CHAIN_APPROX_SIMPLE points written to
//                        one of the instance's two point buffers (the longest stays); cv2.contourArea of the
//                        longest over its float32 scale_coords points (double shoelace in OpenCV's order, the
//                        terms in parallel, summed in order).  -> va_contour_stat.  Three instantiations by
//                        image size: 32 KiB of LDS (several waves per CU), 156 KiB (one per CU), and the
//                        global-memory form for larger regions (full-frame boxes, 1280-pixel inputs).
//   post_fill_kernel     one workgroup per frame: the instance max(area) picks (first maximum; a single detection
//                        is taken as it is), its points as int32 frame points (np.int32 of the float32
//                        scale_coords), boundingRect, and cv2.fillPoly(LINE_8) evaluated only at the cell centres:
//                        a centre is set when an edge's 8-connected Bresenham line (LineIterator + clipLine) passes
//                        through it, or when it lies in a FillEdgeCollection span -- with a = #active edges left of
//                        the pixel and b = #active edges left of its right neighbour (16.16 edge x at that row),
//                        the pixel is inside a pair iff b > a or a is odd, an order-free count the threads
//                        accumulate with LDS atomics.
//
// The image lives in LDS through a pointer the compiler sees as LDS (each size class is its own instantiation): an
// earlier form that selected between an LDS and a global image at run time faulted on gfx950.  The border
// following runs with wave-uniform scalar state (every lane the same pixel): a step is instruction-bound (one
// wave issues at most one instruction per 4 cycles), so the step's work is kept to a few dozen scalar ops.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>
#include <stdlib.h>

#include "../../include/va355.h"
#include "va_switch.h"
#include "va_contour.h"
#include "va_dev.h"
#include "va_diag.h"

namespace {

constexpr int NMC = 32;
constexpr int REG_MAX = 16;
constexpr int CT_THREADS = 64;             // one wave per detection: the scan and the border following are serial
constexpr int FILL_THREADS = 256;
constexpr int CT_STRIP = 1024;             // floats of one strip of low-res rows (4 KiB; >= 2 rows of a 2048-px input)
// The LDS form: 16 waves per workgroup, one workgroup per CU, each wave an independent worker over the detections
// with its image in pages of a shared 160 KiB pool (a 32-bit page map, CAS-allocated), so a CU holds as many
// images as fit instead of one fixed size class per launch.
constexpr int CP_WAVES = 16;
constexpr int CP_THREADS = 64 * CP_WAVES;
constexpr int CP_PAGES = 32;
constexpr int CP_PAGE = 5104;              // bytes (16-aligned): 32 pages + the pool's bookkeeping fit in 160 KiB
constexpr int CP_POOL = CP_PAGES * CP_PAGE;
// chain-code moves (0 = right, counter-clockwise), as 2-bit fields of (d + 1): register arithmetic, not a table
// load (a per-step table load with a lane-varying index is a memory round trip on the trace's critical path)
__device__ __forceinline__ int dir_dx(int s) { return (int)((0x901Au >> (2 * s)) & 3u) - 1; }  // 1 1 0 -1 -1 -1 0 1
__device__ __forceinline__ int dir_dy(int s) { return (int)((0xA901u >> (2 * s)) & 3u) - 1; }  // 0 -1 -1 -1 0 1 1 1
// every lane of the wave holds the same value: make it scalar (uniform branches, SALU arithmetic)
__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }

// Bounds-checked debug build (-DVA_CT_CHECK, tools/ct_check.py): an out-of-range access is skipped and the first
// one recorded as (code, v0, v1) for va_contour_debug instead of faulting.
#ifdef VA_CT_CHECK
__device__ unsigned int g_ct_err[4];
__device__ inline bool ct_ok(bool c, int code, long long v0, long long v1) {
    if (!c && atomicCAS(&g_ct_err[0], 0u, (unsigned)code) == 0u) {
        atomicExch(&g_ct_err[1], (unsigned)v0);
        atomicExch(&g_ct_err[2], (unsigned)v1);
    }
    return c;
}
#define CT_OK(c, code, v0, v1) ct_ok((c), (code), (long long)(v0), (long long)(v1))
// per-detection phase clocks of the contour kernel (s_memtime): build, scan, area; counts: contours, rows
// scanned, positions visited, trace steps
constexpr int CT_PROF_ITEMS = 4096;
__device__ unsigned long long g_ct_prof[CT_PROF_ITEMS][8];
// per frame of the fill kernel: choice + points, edges, fill (s_memtime cycles), the point count, fallback flag
constexpr int CT_FILL_FRAMES = 1024;
__device__ unsigned long long g_ct_fill[CT_FILL_FRAMES][8];
#define CT_PROF(...) __VA_ARGS__
#define CT_STEPS (&nsteps)
#else
// production: the same sites reject the access and record it (va_diag.h: code 20 + site)
#define CT_OK(c, code, v0, v1) VA_DIAG_OK((c), 20 + (code), (v0), (v1))
#define CT_PROF(...)
#define CT_STEPS nullptr
#endif
#if defined(VA_CT_CHECK) && !defined(VA_CT_WATCH)
#define VA_CT_WATCH
#endif
#ifdef VA_CT_WATCH
// hang watch: per (block, wave) of the pool kernel {item, phase, y, counter} in host-mapped memory (system-scope
// stores), readable by the host while a kernel runs (tools/ct_watch.py)
constexpr int CT_WATCH_SLOTS = 256 * 16;
__device__ int* g_ct_watch;
__device__ inline void ct_watch(int f, int v) {
    int* w = g_ct_watch;
    if (!w || (threadIdx.x & 63) != 0) return;
    const int slot = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (slot < CT_WATCH_SLOTS) __hip_atomic_store(w + 4 * slot + f, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
#define CT_WATCH(f, v) ct_watch((f), (int)(v))
#else
#define CT_WATCH(f, v)
#endif

// ------------------------------------------------------------------------------------------ geometry
using Src = CtSrc;
using Frame = CtFrame;
using Scratch = CtScratch;

__device__ inline const float* coef_row(const Src& s, int b, int anchor) {
    const int H = s.Hn, W = s.Wn;
    const int h0 = H / 8, w0 = W / 8, h1 = H / 16, w1 = W / 16, h2 = H / 32, w2 = W / 32;
    const int n0 = h0 * w0, n1 = h1 * w1;
    const int no = 4 * REG_MAX + s.nc + NMC;
    const float* p;
    int local, hw;
    if (anchor < n0) {
        p = s.lv[0], local = anchor, hw = n0;
    } else if (anchor < n0 + n1) {
        p = s.lv[1], local = anchor - n0, hw = n1;
    } else {
        p = s.lv[2], local = anchor - n0 - n1, hw = h2 * w2;
    }
    return p + ((int64_t)b * hw + local) * no + 4 * REG_MAX + s.nc;
}

// process_mask's crop window in low-res pixels (crop_mask: r >= x1 * mw / W && r < x2 * mw / W)
__device__ inline void crop_window(const va_det& d, const Src& s, int* rx0, int* rx1, int* ry0, int* ry1) {
    const float fx1 = d.x1 * ((float)s.mw / (float)s.Wn), fx2 = d.x2 * ((float)s.mw / (float)s.Wn);
    const float fy1 = d.y1 * ((float)s.mh / (float)s.Hn), fy2 = d.y2 * ((float)s.mh / (float)s.Hn);
    *rx0 = max((int)ceilf(fx1), 0);
    *rx1 = min((int)ceilf(fx2) - 1, s.mw - 1);
    *ry0 = max((int)ceilf(fy1), 0);
    *ry1 = min((int)ceilf(fy2) - 1, s.mh - 1);
}

// F.interpolate(bilinear, align_corners=False) taps for output index o (scale = in / out)
__device__ inline void taps(int o, float scale, int in, int* i0, int* i1, float* l0, float* l1) {
    float src = scale * ((float)o + 0.5f) - 0.5f;
    if (src < 0.f) src = 0.f;
    const int x0 = (int)src;
    *l1 = src - (float)x0;
    *l0 = 1.0f - *l1;
    *i0 = x0;
    *i1 = x0 + (x0 < in - 1 ? 1 : 0);
}

// The framed image region of detection (b, k): network pixels [X0, X0 + w) x [Y0, Y0 + h) plus one zero pixel
// around (cv::findContours' border).  Empty (w = 0) when the mask cannot have a positive pixel.
struct Region {
    int X0, Y0, w, h;  // network pixels covered
    int rW, rH, ww;    // framed size in pixels, 32-bit words per plane row (32 pixels each)
    int rx0, rx1, ry0, ry1;
};

__device__ inline Region region_of(const Src& s, int b, int k) {
    Region r{};
    if (s.masks) {
        r.X0 = 0, r.Y0 = 0, r.w = s.Wn, r.h = s.Hn;
    } else {
        const va_det d = s.dets[(int64_t)b * s.max_det + k];
        crop_window(d, s, &r.rx0, &r.rx1, &r.ry0, &r.ry1);
        if (r.rx1 < r.rx0 || r.ry1 < r.ry0) return r;  // w = 0: an all-zero mask
        const float sx = (float)s.mw / (float)s.Wn, sy = (float)s.mh / (float)s.Hn;
        // full-res pixels whose taps can touch the window
        r.X0 = max(0, (int)((r.rx0 - 1) / sx) - 2);
        const int X1 = min(s.Wn - 1, (int)((r.rx1 + 1) / sx) + 2);
        r.Y0 = max(0, (int)((r.ry0 - 1) / sy) - 2);
        const int Y1 = min(s.Hn - 1, (int)((r.ry1 + 1) / sy) + 2);
        r.w = X1 - r.X0 + 1;
        r.h = Y1 - r.Y0 + 1;
    }
    r.rW = r.w + 2;
    r.rH = r.h + 2;
    r.ww = (r.rW + 31) >> 5;
    return r;
}

// the region's fields as scalars (every lane computed the same values from the same loads): scalar branches
__device__ __forceinline__ Region uni_region(const Region& r) {
    Region u;
    u.X0 = uni(r.X0), u.Y0 = uni(r.Y0), u.w = uni(r.w), u.h = uni(r.h);
    u.rW = uni(r.rW), u.rH = uni(r.rH), u.ww = uni(r.ww);
    u.rx0 = uni(r.rx0), u.rx1 = uni(r.rx1), u.ry0 = uni(r.ry0), u.ry1 = uni(r.ry1);
    return u;
}

// 32-bit words of the image: three bit planes per row (+ one spare word, read past by the trace windows)
__device__ inline int64_t image_words(const Region& r) { return (int64_t)r.rH * 3 * r.ww + 1; }

// bytes an instance needs: the image, plus the low-res strip for a head-source mask
__device__ inline int64_t region_need(const Src& s, const Region& r) {
    if (r.w <= 0) return 0;
    return ((image_words(r) * 4 + 15) & ~15ll) + (s.masks ? 0 : CT_STRIP * 4);
}

// float32 scale_coords of a network point (ops.py:784-816)
__device__ inline void scale_pt(const Frame& f, int X, int Y, float* xs, float* ys) {
    *xs = fminf(fmaxf(((float)X - f.padx) / f.gain, 0.0f), (float)f.W0);
    *ys = fminf(fmaxf(((float)Y - f.pady) / f.gain, 0.0f), (float)f.H0);
}

// ------------------------------------------------------------------------------------------ the image
// Three bit planes per framed row y, 32 pixels per word: NZ (plane 0, the mask), N (1: visited by a border trace,
// OpenCV's nbd) and R (2: visited as a "right" border pixel, OpenCV's nbd | -128).  OpenCV's per-visit update
// ("right" -> -126, else 1 -> 2) reaches the value R ? -126 : N ? 2 : NZ in any visit order, so a visit just ORs
// its bit in -- one LDS (or global) atomic OR from lane 0, no read.
__device__ __forceinline__ uint32_t* plane(uint32_t* img, int ww, int y, int p) { return img + (3 * y + p) * ww; }
__device__ __forceinline__ const uint32_t* plane(const uint32_t* img, int ww, int y, int p) {
    return img + (3 * y + p) * ww;
}

// N / R words: the scan reads what the traces wrote.  LDS: plain (one wave, in order); global: coherent.
template <bool LDS>
__device__ __forceinline__ uint32_t ldm(const uint32_t* p) {
    if constexpr (LDS) {
        return *p;
    } else {
        return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// OpenCV's value of a pixel from its three bits
__device__ __forceinline__ int val_bits(uint32_t nz, uint32_t n, uint32_t r) { return r ? -126 : (n ? 2 : (int)nz); }

template <bool LDS>
__device__ __forceinline__ int val_at(const uint32_t* img, int ww, int x, int y) {
    if (!CT_OK(x >= 0 && y >= 0 && (x >> 5) < ww, 2, x, y)) return 0;
    const int w = x >> 5, b = x & 31;
    return val_bits((plane(img, ww, y, 0)[w] >> b) & 1u, (ldm<LDS>(plane(img, ww, y, 1) + w) >> b) & 1u,
                    (ldm<LDS>(plane(img, ww, y, 2) + w) >> b) & 1u);
}

// the value planes of a word: hi = any mark, lo = "right" mark or an unmarked non-zero pixel (value codes
// 0 / 1 / 2 / 3 for 0 / 1 / 2 / -126)
__device__ __forceinline__ void code_planes(uint32_t nz, uint32_t n, uint32_t r, uint32_t& hi, uint32_t& lo) {
    hi = n | r;
    lo = r | (nz & ~n);
}

// The first row in [y, yend) holding a non-zero, unmarked pixel right of a zero pixel -- the only rows where
// cvFindNextContour can start an outer border (traces only mark, so the answer at the row's start holds through
// the row) -- or yend: the rows' words taken 64 at a time across rows (one ballot per 64 words, not one per row).  Exact as a look-ahead: marks only grow and NZ never
// changes, so a row without an unmarked start keeps having none; the scan calls this again after each trace.
template <bool LDS>
__device__ __forceinline__ int next_start_row(const uint32_t* img, int ww, int y, int yend) {
    const int lane = threadIdx.x & 63;
    const int total = (yend - y) * ww;
    for (int i0 = 0; i0 < total; i0 += 64) {
        const int i = i0 + lane;
        bool hit = false;
        if (i < total) {
            const int dy = i / ww, wi = i - dy * ww;
            const uint32_t* nzr = plane(img, ww, y + dy, 0);
            const uint32_t nz = nzr[wi], pnz = wi >= 1 ? nzr[wi - 1] : 0u;
            const uint32_t mk = ldm<LDS>(plane(img, ww, y + dy, 1) + wi) | ldm<LDS>(plane(img, ww, y + dy, 2) + wi);
            hit = (nz & ~mk & ~((nz << 1) | (pnz >> 31))) != 0u;
        }
        const unsigned long long bal = __ballot(hit);
        if (bal) return y + (i0 + __builtin_ctzll(bal)) / ww;
    }
    return yend;
}

// ------------------------------------------------------------------------------------------ building
struct MaskStat {
    int cnt, x0, x1, y0, y1;
};

// The framed image of detection (b, k) into img (region r), by nt threads of the calling block; the mask pixel
// count and bbox accumulate per thread in ms.  Head source: strips of the low-res window of coef . proto in
// `strip`, each evaluating the full-res rows whose taps it holds with the exact per-pixel expression
// wy0 (wx0 v(ya, xa) + wx1 v(ya, xb)) + wy1 (wx0 v(yb, xa) + wx1 v(yb, xb)) > 0.
// the threads building an image: one wave (the contour kernels) or the whole block (post_fill_kernel)
template <bool WAVE>
__device__ __forceinline__ void ct_sync() {
    if constexpr (WAVE) {
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
    } else {
        __syncthreads();
    }
}

// Low-res rows s0 .. s1 of the detection's crop window, coef . proto per pixel, into strip[(y - s0) tw + x - rx0]:
// eight lanes per low-res pixel (its 128 bytes of proto in one coalesced run): lane q's partial sum of 4 channels,
// then the pairwise tree ((p0 + p1) + (p2 + p3)) + ((p4 + p5) + (p6 + p7)) by xor shuffles -- post-processing's
// 8-lane dot (same order, same result).  U pixels' loads in flight per lane before the first is used (the phase is
// latency-bound on them; the block-wide forms have the registers for 8).
template <int U>
__device__ __forceinline__ void strip_dots(const Src& s, int b, const float4& cq, const Region& r, int s0, int s1,
                                           int tw, float* strip, int tid, int nt) {
    const int npx = (s1 - s0 + 1) * tw, ntot = npx * 8;
#pragma unroll 1
    for (int i0 = tid; i0 < ntot; i0 += U * nt) {  // whole 8-lane groups are active together
        float4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int i = i0 + u * nt, px = i >> 3;
            if (i < ntot) {
                const int y = s0 + px / tw, x = r.rx0 + px % tw;
                v[u] = ((const float4*)(s.proto + (((int64_t)b * s.mh + y) * s.mw + x) * NMC))[tid & 7];
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int i = i0 + u * nt;
            if (i < ntot) {
                float part = (cq.x * v[u].x + cq.y * v[u].y) + (cq.z * v[u].z + cq.w * v[u].w);
                part += __shfl_xor(part, 1);
                part += __shfl_xor(part, 2);
                part += __shfl_xor(part, 4);
                if ((tid & 7) == 0) strip[i >> 3] = part;
            }
        }
    }
}

template <bool WAVE, int MEMCLASS = 0>  // MEMCLASS: a distinct instantiation per image memory class (see below)
__device__ __forceinline__ void build_image(const Src& s, int b, int k, const Region& r, uint32_t* img, float* strip,
                                            int tid, int nt, MaskStat& ms, int strip_cap = CT_STRIP,
                                            int sep_cap = 0) {
    auto account = [&](uint32_t w, int x32, int yy) {
        if (!w) return;
        ms.cnt += __builtin_popcount(w);
        const int X = r.X0 + x32 - 1, Y = r.Y0 + yy - 1;
        ms.x0 = min(ms.x0, X + __builtin_ctz(w));
        ms.x1 = max(ms.x1, X + 31 - __builtin_clz(w));
        ms.y0 = min(ms.y0, Y);
        ms.y1 = max(ms.y1, Y);
    };
    // the mark planes and the frame rows start at zero
    for (int i = tid; i < r.rH * r.ww; i += nt) {
        const int y = i / r.ww, w = i % r.ww;
        plane(img, r.ww, y, 1)[w] = 0u;
        plane(img, r.ww, y, 2)[w] = 0u;
        if (y == 0 || y == r.rH - 1) plane(img, r.ww, y, 0)[w] = 0u;
    }
    if (tid == 0) img[image_words(r) - 1] = 0u;
    if (s.masks) {
        const uint8_t* m = s.masks + ((int64_t)b * s.maxn + k) * s.Hn * s.Wn;
        for (int i = tid; i < r.h * r.ww; i += nt) {
            const int y = 1 + i / r.ww, x32 = 32 * (i % r.ww);
            uint32_t w = 0;
#pragma unroll 8
            for (int j = 0; j < 32; ++j) {
                const int x = x32 + j;
                if (x >= 1 && x <= r.w && m[(int64_t)(y - 1) * s.Wn + (x - 1)]) w |= 1u << j;
            }
            account(w, x32, y);
            plane(img, r.ww, y, 0)[x32 >> 5] = w;
        }
        ct_sync<WAVE>();
        return;
    }
    const int anchor = s.dets[(int64_t)b * s.max_det + k].anchor;
    const float4* coef4 = (const float4*)coef_row(s, b, anchor);
    const float4 cq = coef4[tid & 7];  // this lane's 4 of the 32 coefficients (nt is a multiple of 8)
    const int tw = r.rx1 - r.rx0 + 1;
    const int S = strip_cap / tw;  // >= 2: tw <= mw <= CT_STRIP / 2 <= strip_cap / 2 (va_contour_launch)
    const float sx = (float)s.mw / (float)s.Wn, sy = (float)s.mh / (float)s.Hn;
    const int nly = r.ry1 - r.ry0 + 1;
    if (!WAVE && (int64_t)nly * (tw + r.w) <= sep_cap) {  // block-uniform
        // Separable form (the workgroup-per-detection kernel, when the whole window and its rows interpolated to
        // the region's columns fit in LDS): every low-res row's horizontal pass hrow[ly][c] = wx0 A + wx1 B is
        // computed once per column instead of once per full-res pixel, then a pixel is wy0 ha + wy1 hb > 0 of two
        // hrow reads -- the same products and sums in the same order as the per-pixel form, so the same bits.
        float* hrow = strip + nly * tw;
        strip_dots<8>(s, b, cq, r, r.ry0, r.ry1, tw, strip, tid, nt);
        ct_sync<WAVE>();
#pragma unroll 1
        for (int i = tid; i < nly * r.w; i += nt) {
            const int ly = i / r.w, c = i - ly * r.w;
            int xa, xb;
            float wx0, wx1;
            taps(r.X0 + c, sx, s.mw, &xa, &xb, &wx0, &wx1);
            const bool ixa = xa >= r.rx0 && xa <= r.rx1, ixb = xb >= r.rx0 && xb <= r.rx1;
            const float A = ixa ? strip[ly * tw + xa - r.rx0] : 0.f, B = ixb ? strip[ly * tw + xb - r.rx0] : 0.f;
            hrow[i] = wx0 * A + wx1 * B;
        }
        ct_sync<WAVE>();
#pragma unroll 1
        for (int i = tid; i < r.h * r.ww; i += nt) {
            const int yy = 1 + i / r.ww, x32 = 32 * (i % r.ww);
            int ya, yb;
            float wy0, wy1;
            taps(r.Y0 + yy - 1, sy, s.mh, &ya, &yb, &wy0, &wy1);
            const bool oka = ya >= r.ry0 && ya <= r.ry1, okb = yb >= r.ry0 && yb <= r.ry1;
            const int ra = (oka ? ya - r.ry0 : 0) * r.w - 1, rb = (okb ? yb - r.ry0 : 0) * r.w - 1;  // by framed x
            const int j0 = max(0, 1 - x32), j1 = min(31, r.w - x32);  // pixels 1 .. w of the framed row
            uint32_t w = 0;
#pragma unroll 4
            for (int j = j0; j <= j1; ++j) {
                const int x = x32 + j;
                const float ha = oka ? hrow[ra + x] : 0.f, hb = okb ? hrow[rb + x] : 0.f;
                if (wy0 * ha + wy1 * hb > 0.f) w |= 1u << j;
            }
            account(w, x32, yy);
            plane(img, r.ww, yy, 0)[x32 >> 5] = w;
        }
        ct_sync<WAVE>();
        return;
    }
    int next = 1, s0 = r.ry0;     // next framed row to produce; first low-res row of the strip
    while (next <= r.h) {         // block-uniform
        const int s1 = min(s0 + S - 1, r.ry1);
        strip_dots<WAVE ? 4 : 8>(s, b, cq, r, s0, s1, tw, strip, tid, nt);
        ct_sync<WAVE>();
        // the rows whose taps inside the window all lie in s0 .. s1 (taps are non-decreasing in the row)
        int end = next;
        while (end <= r.h) {
            int ya, yb;
            float w0, w1;
            taps(r.Y0 + end - 1, sy, s.mh, &ya, &yb, &w0, &w1);
            const int hi = (yb >= r.ry0 && yb <= r.ry1) ? yb : ((ya >= r.ry0 && ya <= r.ry1) ? ya : -1);
            if (hi > s1) break;
            ++end;
        }
#pragma unroll 1
        for (int i = tid; i < (end - next) * r.ww; i += nt) {
            const int yy = next + i / r.ww, x32 = 32 * (i % r.ww);
            int ya, yb;
            float wy0, wy1;
            taps(r.Y0 + yy - 1, sy, s.mh, &ya, &yb, &wy0, &wy1);
            // val() per tap, its row tests hoisted out of the pixel loop: a tap outside the window reads 0
            const bool oka = ya >= r.ry0 && ya <= r.ry1, okb = yb >= r.ry0 && yb <= r.ry1;
            const int la = (ya - s0) * tw - r.rx0, lb = (yb - s0) * tw - r.rx0;
            if (!CT_OK(!oka || (la + r.rx0 >= 0 && la + r.rx1 < strip_cap), 7, la, tw)) continue;
            if (!CT_OK(!okb || (lb + r.rx0 >= 0 && lb + r.rx1 < strip_cap), 7, lb, tw)) continue;
            const int j0 = max(0, 1 - x32), j1 = min(31, r.w - x32);  // pixels 1 .. w of the framed row
            uint32_t w = 0;
#pragma unroll 4
            for (int j = j0; j <= j1; ++j) {
                int xa, xb;
                float wx0, wx1;
                taps(r.X0 + x32 + j - 1, sx, s.mw, &xa, &xb, &wx0, &wx1);
                const bool ixa = xa >= r.rx0 && xa <= r.rx1, ixb = xb >= r.rx0 && xb <= r.rx1;
                const float A = oka && ixa ? strip[la + xa] : 0.f, B = oka && ixb ? strip[la + xb] : 0.f;
                const float C = okb && ixa ? strip[lb + xa] : 0.f, D = okb && ixb ? strip[lb + xb] : 0.f;
                const float ha = wx0 * A + wx1 * B, hb = wx0 * C + wx1 * D;
                if (wy0 * ha + wy1 * hb > 0.f) w |= 1u << j;
            }
            account(w, x32, yy);
            plane(img, r.ww, yy, 0)[x32 >> 5] = w;
        }
        next = end;
        s0 = s1;  // a later row may need s1 and s1 + 1
        ct_sync<WAVE>();
    }
}

// ------------------------------------------------------------------------------------------ border following
// The trace's view of the NZ plane: the two-word windows (from word c0 = (x - 1) / 32) of rows cy - 1, cy, cy + 1,
// held as wave-uniform scalars.  A step to a neighbour keeps c0 31 times in 32 and shifts the rows on a vertical
// move, so most steps load one row or none (the NZ plane never changes).
struct TraceWin {
    unsigned long long up, md, dn;
    int c0, cy;
};

__device__ __forceinline__ unsigned long long load_win(const uint32_t* img, int ww, int y, int c0) {
    const uint32_t* p = plane(img, ww, y, 0) + c0;
    const uint32_t lo = p[0], hi = p[1];
    return (unsigned long long)(unsigned)uni((int)lo) | ((unsigned long long)(unsigned)uni((int)hi) << 32);
}

__device__ __forceinline__ void win_at(const uint32_t* img, int ww, int x, int y, TraceWin& w) {
    const int c0 = (x - 1) >> 5;
    if (c0 == w.c0 && y == w.cy) return;
    if (c0 == w.c0 && y == w.cy + 1) {
        w.up = w.md, w.md = w.dn, w.dn = load_win(img, ww, y + 1, c0);
    } else if (c0 == w.c0 && y == w.cy - 1) {
        w.dn = w.md, w.md = w.up, w.up = load_win(img, ww, y - 1, c0);
    } else {
        const uint32_t* p = plane(img, ww, y - 1, 0) + c0;
        const int st = 3 * ww;  // one row down, same plane
        const uint32_t a0 = p[0], a1 = p[1], b0 = p[st], b1 = p[st + 1], d0 = p[2 * st], d1 = p[2 * st + 1];
        w.up = (unsigned long long)(unsigned)uni((int)a0) | ((unsigned long long)(unsigned)uni((int)a1) << 32);
        w.md = (unsigned long long)(unsigned)uni((int)b0) | ((unsigned long long)(unsigned)uni((int)b1) << 32);
        w.dn = (unsigned long long)(unsigned)uni((int)d0) | ((unsigned long long)(unsigned)uni((int)d1) << 32);
    }
    w.c0 = c0, w.cy = y;
}

// bit d = the neighbour in direction d (0 = right, counter-clockwise) is non-zero
__device__ __forceinline__ unsigned win_nbrs(const TraceWin& w, int x) {
    const int sh = (x - 1) & 31;
    const unsigned up = (unsigned)(w.up >> sh) & 7u, m = (unsigned)(w.md >> sh) & 7u, dn = (unsigned)(w.dn >> sh) & 7u;
    // up: x-1, x, x+1 -> directions 3, 2, 1 (bit-reversed); md: x+1 -> 0, x-1 -> 4; dn: x-1, x, x+1 -> 5, 6, 7
    return ((m >> 2) & 1u) | (__builtin_bitreverse32(up) >> 28) | ((m & 1u) << 4) | (dn << 5);
}

// the visit's mark of (x, y): "right" -> R, else N (lane 0, one atomic OR)
__device__ __forceinline__ void mark_at(uint32_t* img, int ww, int x, int y, bool right) {
    if ((threadIdx.x & 63) != 0) return;
    if (!CT_OK(x >= 0 && y >= 0 && (x >> 5) < ww, 3, x, y)) return;
    atomicOr(plane(img, ww, y, right ? 2 : 1) + (x >> 5), 1u << (x & 31));
}

// A straight run of the border: with the follow at P_0 = (x, y) having arrived in direction D (s_end = D + 4), the
// number k of consecutive pixels P_j = P_0 + j D (j < 63) at which it leaves in direction D again, i.e. the
// counter-clockwise search from s_end + 1 meets zeros at D + 5, D + 6, D + 7 and a non-zero at D: no point is kept
// there (the direction does not change) and P_j + D = P_(j + 1) is the next position.  Lane j tests P_j (four bits
// of the NZ plane, which no trace changes); k = the ballot's trailing ones.  Lanes whose neighbourhood leaves the
// framed image test false (the border is zero, so a run never reaches it).
__device__ __forceinline__ int border_run(const uint32_t* img, int ww, int rh, int x, int y, int D) {
    const int j = threadIdx.x & 63;
    const int px = x + j * dir_dx(D), py = y + j * dir_dy(D);
    bool run = false;
    if (j < 63 && px >= 1 && py >= 1 && py < rh - 1 && px + 1 < 32 * ww) {
        auto nz = [&](int d) {
            const int qx = px + dir_dx(d & 7), qy = py + dir_dy(d & 7);
            return (plane(img, ww, qy, 0)[qx >> 5] >> (qx & 31)) & 1u;
        };
        run = nz(D) && !(nz(D + 5) | nz(D + 6) | nz(D + 7));
    }
    return __builtin_ctzll(~__ballot(run));
}

// icvFetchContour (CHAIN_APPROX_SIMPLE) from the outer-border start (x0, y0) of the framed image (rh rows), executed
// by the whole wave in lock step (every lane the same pixel, scalar state).  mark(x, y, right) gets a visit's mark,
// mark_run(x, y, D, k, right) the marks of k visits P_0 + j D (j < k) at once, emit(x, y) every kept point in order.
// Where the follow continues in the direction it came (no point kept), the straight run ahead is measured by
// border_run and crossed in one move: a box-like mask's border is a handful of runs instead of one serial step
// (≈ 560 cycles of dependent scalar work) per pixel.  Returns the number of points.
template <typename Mark, typename MarkRun, typename Emit>
__device__ __forceinline__ int follow_border(uint32_t* img, int ww, int rh, bool runs, int x0, int y0, Mark mark,
                                             MarkRun mark_run, Emit emit, int* steps = nullptr) {
    TraceWin w{0ull, 0ull, 0ull, -1, -1};
    win_at(img, ww, x0, y0, w);
    const unsigned nb = win_nbrs(w, x0);
    int s = 4;  // outer border: s_end = s = 4
    const int s_end0 = 4;
    do {
        s = (s - 1) & 7;
    } while (!((nb >> s) & 1) && s != s_end0);
    if (s == s_end0) {  // single pixel domain
        mark(x0, y0, true);
        emit(x0, y0);
        return 1;
    }
    const int x1 = x0 + dir_dx(s), y1 = y0 + dir_dy(s);  // i1
    // the stop test on packed (x | y << 16) positions: framed coordinates are non-negative and below 2^16
    const int p0 = x0 | (y0 << 16), p1 = x1 | (y1 << 16);
    int x3 = x0, y3 = y0;
    int prev_s = s ^ 4, n = 0;
    bool cont1 = false;  // the previous step continued in its direction
    unsigned nb3 = nb;
    while (true) {
        const int s_end = s;
        // counter-clockwise from s_end + 1 to the first non-zero neighbour (one exists: i1 at the latest)
        const unsigned rot = ((nb3 | (nb3 << 8)) >> ((s_end + 1) & 7)) & 0xFFu;
        s = (s_end + 1 + __builtin_ctz(rot)) & 7;
        // s_end = prev_s + 4 always: s == prev_s is a run from (x3, y3) on, k >= 1 (x3 itself continues; the
        // k > 0 test only keeps a broken invariant from stalling the loop).  Measured from the run's second pixel
        // on: noise-like masks' runs are mostly one pixel, where the probe would cost more than the step.
        const bool cont = s == prev_s;
        const int k = runs && cont && cont1 ? border_run(img, ww, rh, x3, y3, s) : 0;
        cont1 = cont;
        if (k > 0) {
            const int dx = dir_dx(s), dy = dir_dy(s);
            const bool right = (unsigned)(s - 1) < (unsigned)s_end;
            // the stop (x3 = i1 and the next position = i0) inside the run: i1 = P_j, j < k, with i1 + D = i0
            const int j1 = dx ? (x1 - x3) * dx : (y1 - y3) * dy;
            if (j1 >= 0 && j1 < k && x3 + j1 * dx == x1 && y3 + j1 * dy == y1 && x1 + dx == x0 && y1 + dy == y0) {
                mark_run(x3, y3, s, j1 + 1, right);
                CT_PROF(if (steps) *steps += j1 + 1);
                break;
            }
            mark_run(x3, y3, s, k, right);
            CT_PROF(if (steps) *steps += k);
            x3 += k * dx;
            y3 += k * dy;
            s = (s + 4) & 7;
            win_at(img, ww, x3, y3, w);
            nb3 = win_nbrs(w, x3);
            continue;
        }
        const int x4 = x3 + dir_dx(s), y4 = y3 + dir_dy(s);
        mark(x3, y3, (unsigned)(s - 1) < (unsigned)s_end);
        if (s != prev_s) {
            emit(x3, y3);
            ++n;
            prev_s = s;
        }
        if ((((x4 | (y4 << 16)) ^ p0) | ((x3 | (y3 << 16)) ^ p1)) == 0) break;
        x3 = x4;
        y3 = y4;
        s = (s + 4) & 7;
        win_at(img, ww, x3, y3, w);
        nb3 = win_nbrs(w, x3);
        CT_PROF(if (steps) ++*steps);
    }
    return n;
}

// the unmarked form (a contour followed again for its points)
template <typename Emit>
__device__ __forceinline__ int fetch_contour(uint32_t* img, int ww, int rh, bool runs, int x0, int y0, Emit emit) {
    return follow_border(img, ww, rh, runs, x0, y0, [](int, int, bool) {}, [](int, int, int, int, bool) {}, emit);
}

// The scan's form: marks and points are collected one per lane in registers (lane i takes record i)
// and written 64 at a time -- a mark is 64 lanes' LDS atomic ORs in one instruction, the points one coalesced
// store -- instead of a lane-0 atomic and a lane-0 store per step on the trace's critical path (the trace reads
// only the mask plane, never the marks, so deferring them changes nothing it sees).  Points go to dst[0, capd)
// as network pixels X | Y << 16.  Returns the number of points.
template <bool LDS>
__device__ __forceinline__ int trace_marked(uint32_t* img, int ww, int rh, bool runs, int x0, int y0, uint32_t* dst,
                                            int capd, int X0, int Y0, int* steps = nullptr) {
    const int lane = threadIdx.x & 63;
    int mrec = 0, nm = 0;   // lane i: pending mark i (x | y << 16 | right << 31)
    int prec = 0, np = 0;   // lane i: pending point i
    auto flush_marks = [&](int cnt) {
        if (lane < cnt) {
            const int x = mrec & 0xFFFF, y = (mrec >> 16) & 0x7FFF;
            if (CT_OK(x >= 0 && y >= 0 && (x >> 5) < ww, 3, x, y))
                atomicOr(plane(img, ww, y, mrec < 0 ? 2 : 1) + (x >> 5), 1u << (x & 31));
        }
    };
    auto flush_points = [&](int base, int cnt) {
        if (lane < cnt && base + lane < capd) dst[base + lane] = (uint32_t)prec;
    };
    const int n = follow_border(
        img, ww, rh, runs, x0, y0,
        [&](int x, int y, bool right) {
            if (lane == (nm & 63)) mrec = x | (y << 16) | (right ? (int)0x80000000 : 0);
            if ((++nm & 63) == 0) flush_marks(64);
        },
        [&](int x, int y, int D, int k, bool right) {  // a run's marks: lane j ORs visit j's bit, now
            if (lane < k) {
                const int px = x + lane * dir_dx(D), py = y + lane * dir_dy(D);
                if (CT_OK(px >= 0 && py >= 0 && (px >> 5) < ww, 3, px, py))
                    atomicOr(plane(img, ww, py, right ? 2 : 1) + (px >> 5), 1u << (px & 31));
            }
        },
        [&](int x, int y) {
            if (lane == (np & 63)) prec = (X0 + x - 1) | ((Y0 + y - 1) << 16);
            if ((++np & 63) == 0) flush_points(np - 64, 64);
        },
        steps);
    flush_marks(nm & 63);
    flush_points(np & ~63, np & 63);
    return n;
}

__device__ __forceinline__ double readlane_f64(double v, int l) {
    const long long bits = __double_as_longlong(v);
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)bits, l);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(bits >> 32), l);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// ------------------------------------------------------------------------------------------ per detection
struct CtArgs {
    Src s;
    Frame f;
    Scratch sc;
    va_contour_stat* cstats;  // [B][max_det]
    int max_det;
    float* polys;             // optional [B][max_det][poly_cap][2]: the best contour in frame coordinates
    int32_t* poly_n;
    int poly_cap;
    int gate;                 // pool kernel: hold new claims while a wave waits for pages
    int runs;                 // border following crosses straight runs in one move (border_run; 0: step by step)
    int64_t pool_max;         // bytes: larger images go to the global-memory form
    int pages;                // pages of the pool kernel's LDS (<= CP_PAGES)
};

__device__ __forceinline__ int wave_sum(int v) {
#pragma unroll
    for (int o = 32; o; o >>= 1) v += __shfl_xor(v, o);
    return v;
}
__device__ __forceinline__ int wave_min(int v) {
#pragma unroll
    for (int o = 32; o; o >>= 1) v = min(v, __shfl_xor(v, o));
    return v;
}
__device__ __forceinline__ int wave_max(int v) {
#pragma unroll
    for (int o = 32; o; o >>= 1) v = max(v, __shfl_xor(v, o));
    return v;
}

// Detection (b, k) with region r, by one wave, its image at img (LDS: a pool page run; else the wave's global
// scratch slot) and, for a head-source mask, the low-res strip at strip.  LDS = the image is in LDS (the
// compiler sees the pointer's address space through the inlining).
template <bool LDS>
__device__ __forceinline__ void contour_scan(const CtArgs& a, int b, int k, const Region& r, uint32_t* img, int item
                                             CT_PROF(, unsigned long long t0, unsigned long long t1));

template <bool LDS>
__device__ __forceinline__ void contour_item(const CtArgs& a, int b, int k, const Region& r, uint32_t* img,
                                             float* strip, int item) {
    const int lane = threadIdx.x & 63;
    const Src& s = a.s;
    const int64_t di = (int64_t)b * a.max_det + k;
    MaskStat ms{0, INT32_MAX, -1, INT32_MAX, -1};
    CT_PROF(const unsigned long long t0 = __builtin_amdgcn_s_memtime());
    CT_WATCH(1, 10);
    build_image<true>(s, b, k, r, img, strip, lane, 64, ms);
    CT_WATCH(1, 11);
    CT_PROF(const unsigned long long t1 = __builtin_amdgcn_s_memtime());
    if (s.stats) {  // pixel count and bbox (process_mask's instance mask)
        const int cnt = wave_sum(ms.cnt);
        const int x0 = wave_min(ms.x1 >= 0 ? ms.x0 : s.Wn), x1 = wave_max(ms.x1);
        const int y0 = wave_min(ms.x1 >= 0 ? ms.y0 : s.Hn), y1 = wave_max(ms.x1 >= 0 ? ms.y1 : -1);
        if (lane == 0) s.stats[di] = va_mask_stat{cnt, x0, y0, x1, y1, {0, 0, 0}};
    }
    if constexpr (!LDS) __threadfence();  // the image before the coherent reads of the scan
    contour_scan<LDS>(a, b, k, r, img, item CT_PROF(, t0, t1));
}

// cvFindNextContour's raster scan (RETR_EXTERNAL) over a built image, the largest contour's area and the
// detection's va_contour_stat -- by one wave (the calling wave)
template <bool LDS>
__device__ __forceinline__ void contour_scan(const CtArgs& a, int b, int k, const Region& r, uint32_t* img, int item
                                             CT_PROF(, unsigned long long t0, unsigned long long t1)) {
    const int lane = threadIdx.x & 63;
    va_contour_stat st{};
    st.ox = st.oy = -1;
    st.X0 = r.X0, st.Y0 = r.Y0;
    const int64_t di = (int64_t)b * a.max_det + k;
    float* poly = a.polys ? a.polys + di * a.poly_cap * 2 : nullptr;
    CT_PROF(unsigned long long nrows = 0, npos = 0; int nsteps = 0; unsigned long long ttr = 0);
    // cvFindNextContour's raster scan (RETR_EXTERNAL); the contour with the most points stays in its half of
    // the instance's point buffer
    uint32_t* cp = a.sc.cpts + di * 2 * a.sc.capd;
    int best_n = 0, best_half = 0, bx = -1, by = -1, ncont = 0, alt = 0;
    for (int y = 1; y < r.rH - 1; ++y) {
        y = next_start_row<LDS>(img, r.ww, y, r.rH - 1);  // skips the rows no outer border can start in
        if (y >= r.rH - 1) break;
        CT_WATCH(2, y);
        CT_PROF(++nrows);
        // OpenCV's skip loop, evaluated a 2048-pixel chunk at a time instead of position by position (the scan's
        // prev is always the value at x - 1, so its stops are the change positions of the current image).  Between
        // two traces nothing changes the image, so the scan's decisions over a chunk follow from the chunk alone
        // and the sign of row[lnbd] carried in: a stop x is an outer-border candidate when row[x - 1] == 0 and
        // row[x] == 1, traced when the last lnbd event before it -- a stop on a mark (lnbd = x), or a hole start
        // after a mark (row[x] == 0, lnbd = x - 1) -- left a non-positive row[lnbd] (marks only grow, 2 -> -126,
        // and a -126 or zero pixel never changes again).  The first traced candidate is taken (every lane finds
        // its word's first by the events below it and the sign carried in from the lanes to its left), then the
        // chunk is re-read from x + 1 with row[lnbd] <= 0 (a traced start does not move lnbd).
        const uint32_t* nzr = plane(img, r.ww, y, 0);
        const uint32_t* nr = plane(img, r.ww, y, 1);
        const uint32_t* rr = plane(img, r.ww, y, 2);
        bool lpos = false;  // row[lnbd] > 0 (lnbd starts on the frame: 0)
        for (int w0 = 0; w0 < r.ww; w0 += 64) {
            const int wi = w0 + lane;
            int from = 32 * w0;
            while (true) {
                CT_PROF(++npos);
                uint32_t chi = 0u, clo = 0u, phi = 0u, plo = 0u;
                if (wi < r.ww) code_planes(nzr[wi], ldm<LDS>(nr + wi), ldm<LDS>(rr + wi), chi, clo);
                if (wi >= 1 && wi <= r.ww)
                    code_planes(nzr[wi - 1], ldm<LDS>(nr + wi - 1), ldm<LDS>(rr + wi - 1), phi, plo);
                // bit j of a word = pixel 32 wi + j; "shifted" = the pixel to its left
                const uint32_t shi = (chi << 1) | (phi >> 31), slo = (clo << 1) | (plo >> 31);
                uint32_t live = 0u;  // positions >= from of this word
                const int fw = from >> 5;
                if (wi < r.ww && wi >= fw) live = wi == fw ? ~0u << (from & 31) : ~0u;
                const uint32_t stop = ((chi ^ shi) | (clo ^ slo)) & live;
                const uint32_t cand = stop & ~chi & clo & ~shi & ~slo;          // 0 -> 1 (unmarked)
                const uint32_t evA = stop & chi;                                  // a stop on a mark
                const uint32_t evB = stop & ~chi & ~clo & shi;                    // 0 after a mark
                const uint32_t ev = evA | evB;
                const uint32_t evpos = (evA & ~clo) | (evB & ~slo);               // row[lnbd] == 2 after it
                // the sign carried into this word: the last event of the lanes to the left, else the chunk's
                const unsigned long long hasb = __ballot(ev != 0u);
                const int topb = ev ? 31 - __builtin_clz(ev) : 0;
                const int lastpos = (int)((evpos >> topb) & 1u);
                const unsigned long long below = hasb & ((1ull << lane) - 1ull);
                const int src = below ? 63 - __builtin_clzll(below) : lane;
                const int fromleft = __shfl(lastpos, src);
                const bool cin = below ? fromleft != 0 : lpos;
                // this word's first candidate whose last event below it (or cin) leaves row[lnbd] <= 0
                int okbit = -1;
                for (uint32_t c = cand; c; c &= c - 1u) {
                    const int j = __builtin_ctz(c);
                    const uint32_t eb = ev & ((1u << j) - 1u);
                    const bool pos = eb ? ((evpos >> (31 - __builtin_clz(eb))) & 1u) != 0u : cin;
                    if (!pos) {
                        okbit = j;
                        break;
                    }
                }
                const unsigned long long okb = __ballot(okbit >= 0);
                if (!okb) {  // no trace in the rest of the chunk: carry the last event's sign on
                    if (hasb) lpos = __builtin_amdgcn_readlane(lastpos, 63 - __builtin_clzll(hasb)) != 0;
                    break;
                }
                const int l = __builtin_ctzll(okb);
                const int x = 32 * (w0 + l) + __builtin_amdgcn_readlane(okbit, l);
                CT_PROF(const unsigned long long ta = __builtin_amdgcn_s_memtime());
                const int n = trace_marked<LDS>(img, r.ww, r.rH, a.runs, x, y, cp + alt * a.sc.capd, a.sc.capd,
                                                r.X0, r.Y0, CT_STEPS);
                CT_PROF(ttr += __builtin_amdgcn_s_memtime() - ta);
                ++ncont;
                CT_WATCH(3, ncont);
                if (n > best_n) {
                    best_n = n, best_half = alt, bx = x, by = y;
                    alt ^= 1;
                }
                if constexpr (!LDS) __threadfence();  // the marks before the scan reads on
                lpos = false;
                from = x + 1;
            }
        }
    }
    st.npts = best_n;
    st.ncont = ncont;
    st.half = best_half;
    CT_PROF(const unsigned long long t2 = __builtin_amdgcn_s_memtime());
    if (best_n > 0) {
        st.ox = bx, st.oy = by;
        // cv2.contourArea of the float32 scale_coords points: a00 += prev.x * y - prev.y * x from the last
        // point on, in order (terms in parallel, summed in order); the polygon itself if asked for
        double acc = 0.0;
        if (best_n <= a.sc.capd) {
            __threadfence();  // lane 0's point stores before every lane reads them
            const uint32_t* P = cp + best_half * a.sc.capd;
            const uint32_t plast = P[best_n - 1];
            for (int b0 = 0; b0 < best_n; b0 += 64) {
                const int i = b0 + lane;
                double term = 0.0;
                if (i < best_n) {
                    const uint32_t q = P[i], pq = i == 0 ? plast : P[i - 1];
                    float xs, ys, pxs, pys;
                    scale_pt(a.f, (int)(q & 0xFFFFu), (int)(q >> 16), &xs, &ys);
                    scale_pt(a.f, (int)(pq & 0xFFFFu), (int)(pq >> 16), &pxs, &pys);
                    term = (double)pxs * (double)ys - (double)pys * (double)xs;
                    if (poly && i < a.poly_cap) {
                        poly[2 * i] = xs;
                        poly[2 * i + 1] = ys;
                    }
                }
                const int m = min(64, best_n - b0);
                for (int j = 0; j < m; ++j) acc += readlane_f64(term, j);
            }
        } else {  // longer than the buffer: followed again from the image (marks off)
            int lx = 0, ly = 0;
            fetch_contour(img, r.ww, r.rH, a.runs, bx, by, [&](int px, int py) { lx = px, ly = py; });
            float pxs, pys;
            scale_pt(a.f, r.X0 + lx - 1, r.Y0 + ly - 1, &pxs, &pys);
            int i = 0;
            fetch_contour(img, r.ww, r.rH, a.runs, bx, by, [&](int qx, int qy) {
                float xs, ys;
                scale_pt(a.f, r.X0 + qx - 1, r.Y0 + qy - 1, &xs, &ys);
                acc += (double)pxs * (double)ys - (double)pys * (double)xs;
                pxs = xs, pys = ys;
                if (poly && i < a.poly_cap && lane == 0) {
                    poly[2 * i] = xs;
                    poly[2 * i + 1] = ys;
                }
                ++i;
            });
        }
        st.area = fabs(acc * 0.5);
    }
    if (lane == 0) {
        if (a.poly_n) a.poly_n[di] = best_n;
        a.cstats[di] = st;
        CT_PROF(if (item < CT_PROF_ITEMS) {
            const unsigned long long t3 = __builtin_amdgcn_s_memtime();
            unsigned long long* pr = g_ct_prof[item];
            pr[0] = t1 - t0, pr[1] = t2 - t1, pr[2] = t3 - t2, pr[3] = (unsigned long long)ncont;
            pr[4] = nrows, pr[5] = npos, pr[6] = (unsigned long long)nsteps, pr[7] = ttr;
        });
    }
    CT_PROF((void)item);
}

// the empty record of a detection whose crop window holds no low-res pixel
__device__ __forceinline__ void contour_empty(const CtArgs& a, int b, int k, const Region& r) {
    if ((threadIdx.x & 63) != 0) return;
    const int64_t di = (int64_t)b * a.max_det + k;
    va_contour_stat st{};
    st.ox = st.oy = -1;
    st.X0 = r.X0, st.Y0 = r.Y0;
    if (a.s.stats) a.s.stats[di] = va_mask_stat{0, 0, 0, -1, -1, {0, 0, 0}};
    if (a.poly_n) a.poly_n[di] = 0;
    a.cstats[di] = st;
}

// The LDS form.  Block g takes detections g, g + G, ...; its 16 waves claim them one at a time from an LDS counter
// and each runs its own detection in a page run of the pool (first fit on the page map, CAS).  A wave that finds
// no free run counts itself into the gate, and no wave claims a new detection while any wave waits, so the pool
// drains towards the waiting waves (which hold no pages: no deadlock); each leaves the count once it has its run
// (a count, not a flag: the first of two waiting waves to get pages does not reopen claims for the other, ADVICE
// r2).  Detections needing more than the pool are left to post_contour_global_kernel.
__global__ __launch_bounds__(CP_THREADS) void post_contour_pool_kernel(CtArgs a) {
    extern __shared__ __align__(16) uint32_t cp_pool[];
    __shared__ unsigned s_map;
    __shared__ int s_next, s_gate;
    const int lane = threadIdx.x & 63;
    if (threadIdx.x == 0) s_map = 0u, s_next = 0, s_gate = 0;
    __syncthreads();
    const Src& s = a.s;
    const int total = s.B * a.max_det;
    const int G = gridDim.x;
    int spins = 0;
    // Every lane runs the bookkeeping (no lane-0-only regions): the claim adds 1 from lane 0 and 0 from the others
    // (lane 0 gets the claim), the page-map CAS is issued by all lanes with the same operands (one succeeds), the
    // release and the gate are idempotent.  An earlier form with `if (lane == 0)` regions and `continue` was
    // compiled into a loop that re-ran a skipped detection without claiming a new one (hung).
    for (int item = 0; item < total;) {
        while (uni(__hip_atomic_load(&s_gate, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP)) != 0)
            __builtin_amdgcn_s_sleep(2);
        item = blockIdx.x + uni(atomicAdd(&s_next, lane == 0 ? 1 : 0)) * G;
        CT_WATCH(0, item);
        CT_WATCH(1, 1);
        bool run_it = false;
        Region r{};
        int b = 0, k = 0;
        if (item < total) {
            b = item / a.max_det, k = item % a.max_det;
            if (k < uni(s.ndet[b])) {
                r = uni_region(region_of(s, b, k));
                if (r.w <= 0) contour_empty(a, b, k, r);
                else run_it = region_need(s, r) <= a.pool_max;  // else the global kernel's
            }
        }
        if (run_it) {
            const int np = (int)((region_need(s, r) + CP_PAGE - 1) / CP_PAGE);
            const unsigned run = np >= 32 ? ~0u : ((1u << np) - 1u);
            CT_WATCH(1, 2);
            int page = -1;
            bool gated = false;
            while (true) {
                const unsigned cur = uni((int)__hip_atomic_load(&s_map, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP));
                int q = -1;
                for (int t = 0; t + np <= a.pages; ++t)
                    if (!(cur & (run << t))) {
                        q = t;
                        break;
                    }
                if (q >= 0) {  // a failed CAS (the map changed under us) looks again at once
                    const unsigned old = atomicCAS(&s_map, cur, cur | (run << q));
                    if (__ballot(old == cur) != 0ull) {
                        page = q;
                        break;
                    }
                } else {
                    if (!gated && a.gate) {  // one more waiting wave (lane 0 adds, the others add 0)
                        atomicAdd(&s_gate, lane == 0 ? 1 : 0);
                        gated = true;
                    }
                    ++spins;
                    __builtin_amdgcn_s_sleep(4);
                }
            }
            if (gated) atomicAdd(&s_gate, lane == 0 ? -1 : 0);  // claims resume when no wave waits
            CT_WATCH(1, 3);
            CT_WATCH(2, page);
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            uint32_t* img = cp_pool + page * (CP_PAGE / 4);
            float* strip = (float*)(img + ((image_words(r) + 3) & ~3ll));
            contour_item<true>(a, b, k, r, img, strip, item);
            CT_WATCH(1, 4);
            ct_sync<true>();
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");  // this wave's image accesses before the release
            atomicAnd(&s_map, ~(run << page));
        }
    }
    CT_WATCH(1, 5);
    CT_WATCH(3, spins);
    (void)spins;
}

// The global-memory form for the regions the pool cannot hold (full-frame boxes of 1280-pixel inputs): one wave
// per block, the image in the block's scratch slot.
__global__ __launch_bounds__(CT_THREADS) void post_contour_global_kernel(CtArgs a) {
    const Src& s = a.s;
    unsigned char* slot = a.sc.base + (int64_t)blockIdx.x * a.sc.slot_bytes;
    const int total = s.B * a.max_det;
    for (int item = blockIdx.x; item < total; item += gridDim.x) {
        const int b = item / a.max_det, k = item % a.max_det;
        if (k >= uni(s.ndet[b])) continue;
        const Region r = uni_region(region_of(s, b, k));
        if (r.w <= 0 || region_need(s, r) <= a.pool_max) continue;
        contour_item<false>(a, b, k, r, (uint32_t*)(slot + a.sc.img_off), (float*)slot, item);
        __syncthreads();  // the slot is reused by the next item
    }
}

// Small batches (every detection of the launch has its own scratch slot: B x max_det <= slots): ONE WORKGROUP per
// detection, the image built by all its waves in the detection's global slot (build_image with the block's
// threads), then the scan / trace by wave 0 as in the other forms.  The pool kernel builds an image with one
// wave, which a few large compact masks (batch 1: 1-5 detections, the whole GPU otherwise idle) leave as the
// network-to-answer path's longest serial stage.
constexpr int CT_WG_THREADS = 512;
constexpr int CT_WG_LDS = CP_POOL;  // the image (+ strip) of a region up to the pool's size lives in LDS
template <bool LDS>
__device__ __forceinline__ void contour_wg_item(const CtArgs& a, int b, int k, const Region& r, uint32_t* img,
                                                float* strip, int strip_cap, int item, int* s_ms) {
    const Src& s = a.s;
    MaskStat ms{0, INT32_MAX, -1, INT32_MAX, -1};
    CT_PROF(const unsigned long long t0 = __builtin_amdgcn_s_memtime());
    // its own build instantiation per memory class: one body serving an LDS and a global image through one pointer
    // faulted on gfx950 (an aperture violation, §4.2 of DESIGN.md)
    build_image<false, LDS ? 1 : 2>(s, b, k, r, img, strip, threadIdx.x, CT_WG_THREADS, ms, strip_cap,
                                    LDS ? strip_cap : 0);
    CT_PROF(const unsigned long long t1 = __builtin_amdgcn_s_memtime());
    const int lane = threadIdx.x & 63;
    if (s.stats) {  // pixel count and bbox: per wave, then across the block
        const int cnt = wave_sum(ms.cnt);
        const int x0 = wave_min(ms.x1 >= 0 ? ms.x0 : s.Wn), x1 = wave_max(ms.x1);
        const int y0 = wave_min(ms.x1 >= 0 ? ms.y0 : s.Hn), y1 = wave_max(ms.x1 >= 0 ? ms.y1 : -1);
        if (lane == 0) {
            atomicAdd(&s_ms[0], cnt);
            atomicMin(&s_ms[1], x0);
            atomicMax(&s_ms[2], x1);
            atomicMin(&s_ms[3], y0);
            atomicMax(&s_ms[4], y1);
        }
    }
    if constexpr (!LDS) __threadfence();  // every wave's image words before wave 0's scan reads them
    __syncthreads();
    if (threadIdx.x < 64) {
        if (s.stats && lane == 0)
            s.stats[(int64_t)b * a.max_det + k] = va_mask_stat{s_ms[0], s_ms[1], s_ms[3], s_ms[2], s_ms[4], {0, 0, 0}};
        contour_scan<LDS>(a, b, k, r, img, item CT_PROF(, t0, t1));
    }
}

__global__ __launch_bounds__(CT_WG_THREADS) void post_contour_wg_kernel(CtArgs a) {
    extern __shared__ __align__(16) uint32_t wg_img[];
    const Src& s = a.s;
    const int item = blockIdx.x;
    const int b = item / a.max_det, k = item % a.max_det;
    if (k >= s.ndet[b]) return;  // block-uniform
    const Region r = region_of(s, b, k);
    if (r.w <= 0) {
        contour_empty(a, b, k, r);
        return;
    }
    __shared__ int s_ms[5];
    if (threadIdx.x == 0) s_ms[0] = 0, s_ms[1] = INT32_MAX, s_ms[2] = -1, s_ms[3] = INT32_MAX, s_ms[4] = -1;
    __syncthreads();
    if (region_need(s, r) <= CT_WG_LDS) {  // block-uniform: the image and the strip in LDS, the trace on LDS
        // the strip takes the rest of the LDS: the whole low-res window of a typical detection in one strip (one
        // round of proto loads and one barrier instead of one per CT_STRIP floats)
        const int64_t img4 = (image_words(r) + 3) & ~3ll;
        float* strip = (float*)(wg_img + img4);
        contour_wg_item<true>(a, b, k, r, wg_img, strip, (int)(CT_WG_LDS / 4 - img4), item, s_ms);
    } else {  // a larger region: the detection's global slot
        unsigned char* slot = a.sc.base + (int64_t)item * a.sc.slot_bytes;
        contour_wg_item<false>(a, b, k, r, (uint32_t*)(slot + a.sc.img_off), (float*)slot, CT_STRIP, item, s_ms);
    }
}

// Batches past the per-detection launch (B x max_det > the scratch slots: the headline's B = 256): the same
// workgroup form, persistent -- one 160 KiB workgroup per CU claims the batch's detections one at a time from a
// counter (ct_prefix_kernel's exclusive prefix of ndet over the frames maps a claim to its (frame, detection)), so
// each detection gets the block-wide separable build instead of one wave's per-pixel build in the pool form.
// buf (the last scratch slot): [0] claim counter, [1 .. B] prefix, [B + 1] total.  A region past the LDS uses the
// workgroup's own slot (blockIdx.x < nslots - 1).
__global__ __launch_bounds__(1024) void ct_prefix_kernel(const int32_t* __restrict__ ndet, int B, int max_det,
                                                          int32_t* __restrict__ buf) {
    __shared__ int part[1024];
    const int tid = threadIdx.x, per = (B + 1023) / 1024, b0 = tid * per, b1 = min(B, b0 + per);
    auto nd = [&](int b) { return min(max(ndet[b], 0), max_det); };
    int sum = 0;
    for (int b = b0; b < b1; ++b) sum += nd(b);
    part[tid] = sum;
    __syncthreads();
    if (tid == 0) {
        int acc = 0;
        for (int i = 0; i < 1024; ++i) {
            const int v = part[i];
            part[i] = acc;
            acc += v;
        }
        buf[0] = 0;
        buf[1 + B] = acc;
    }
    __syncthreads();
    int acc = part[tid];
    for (int b = b0; b < b1; ++b) {
        buf[1 + b] = acc;
        acc += nd(b);
    }
}

// A round takes up to eight claimed detections whose images fit the LDS side by side: each is built by the whole
// block in turn (its strip / separable rows in the LDS past the images), then wave w scans / traces detection w --
// eight independent scans at once, as the pool form's waves run them, instead of one wave scanning while seven
// wait.  A detection whose image cannot share the LDS runs alone (in the workgroup's slot if it exceeds the LDS).
constexpr int WGP_D = CT_WG_THREADS / 64;

__global__ __launch_bounds__(CT_WG_THREADS) void post_contour_wgp_kernel(CtArgs a, int32_t* buf, int lds_bytes) {
    extern __shared__ __align__(16) uint32_t wg_img[];
    __shared__ int s_ms[WGP_D][5], s_j, s_b[WGP_D], s_k[WGP_D], s_off[WGP_D], s_item[WGP_D];
    const Src& s = a.s;
    const int B = s.B, total = buf[1 + B];
    const int32_t* pre = buf + 1;
    const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63;
    unsigned char* slot = a.sc.base + (int64_t)blockIdx.x * a.sc.slot_bytes;
    int qn = 0, qe = 0;  // claimed, not yet taken: [qn, qe) (block-uniform)
    while (true) {
        if (qn == qe) {
            if (tid == 0) s_j = atomicAdd(&buf[0], WGP_D);
            __syncthreads();
            qn = s_j;
            qe = min(qn + WGP_D, total);
            __syncthreads();  // s_j read by every thread before the next claim writes it
            if (qn >= total) break;  // block-uniform
        }
        int nd = 0;
        int64_t used = 0;  // LDS words held by this round's images
        while (qn < qe && nd < WGP_D) {
            const int j = qn;
            int lo = 0, hi = B - 1;  // the frame: the last b with pre[b] <= j
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (pre[mid] <= j) lo = mid;
                else hi = mid - 1;
            }
            const int b = lo, k = j - pre[lo];
            const Region r = region_of(s, b, k);
            if (r.w <= 0) {
                if (tid < 64) contour_empty(a, b, k, r);
                ++qn;
                continue;
            }
            const int64_t img4 = (image_words(r) + 3) & ~3ll;
            if ((used + img4) * 4 + CT_STRIP * 4 > lds_bytes) {  // block-uniform
                if (nd > 0) break;  // scan this round's detections first
                // alone and still too large for the LDS: the workgroup's slot, wave 0's scan
                if (tid == 0) s_ms[0][0] = 0, s_ms[0][1] = INT32_MAX, s_ms[0][2] = -1, s_ms[0][3] = INT32_MAX, s_ms[0][4] = -1;
                __syncthreads();
                contour_wg_item<false>(a, b, k, r, (uint32_t*)(slot + a.sc.img_off), (float*)slot, CT_STRIP, j,
                                       s_ms[0]);
                __syncthreads();
                ++qn;
                continue;
            }
            if (tid == 0) {
                s_ms[nd][0] = 0, s_ms[nd][1] = INT32_MAX, s_ms[nd][2] = -1, s_ms[nd][3] = INT32_MAX, s_ms[nd][4] = -1;
                s_b[nd] = b, s_k[nd] = k, s_off[nd] = (int)used, s_item[nd] = j;
            }
            uint32_t* img = wg_img + used;
            const int cap = (int)(lds_bytes / 4 - used - img4);
            MaskStat ms{0, INT32_MAX, -1, INT32_MAX, -1};
            build_image<false, 1>(s, b, k, r, img, (float*)(img + img4), tid, CT_WG_THREADS, ms, cap, cap);
            if (s.stats) {
                const int cnt = wave_sum(ms.cnt);
                const int x0 = wave_min(ms.x1 >= 0 ? ms.x0 : s.Wn), x1 = wave_max(ms.x1);
                const int y0 = wave_min(ms.x1 >= 0 ? ms.y0 : s.Hn), y1 = wave_max(ms.x1 >= 0 ? ms.y1 : -1);
                if (lane == 0) {
                    atomicAdd(&s_ms[nd][0], cnt);
                    atomicMin(&s_ms[nd][1], x0);
                    atomicMax(&s_ms[nd][2], x1);
                    atomicMin(&s_ms[nd][3], y0);
                    atomicMax(&s_ms[nd][4], y1);
                }
            }
            __syncthreads();  // the image complete (and its scratch free for the next build)
            used += img4;
            ++nd;
            ++qn;
        }
        if (wid < nd) {  // wave w: detection w of the round
            const int b = s_b[wid], k = s_k[wid];
            const Region r = uni_region(region_of(s, b, k));
            if (s.stats && lane == 0)
                s.stats[(int64_t)b * a.max_det + k] =
                    va_mask_stat{s_ms[wid][0], s_ms[wid][1], s_ms[wid][3], s_ms[wid][2], s_ms[wid][4], {0, 0, 0}};
            contour_scan<true>(a, b, k, r, wg_img + s_off[wid], s_item[wid] CT_PROF(, 0ull, 0ull));
        }
        __syncthreads();  // the round's images and records free
    }
}

// ------------------------------------------------------------------------------------------ per frame
struct FillArgs {
    Src s;
    Frame f;
    Scratch sc;
    const va_contour_stat* cstats;
    int max_det;
    const uint8_t* plant_cells;
    const int32_t* plant_rects;
    int plant_mode;
    uint8_t* cells;   // [B][H0/20][W0/20]
    int32_t* rects;   // [B][4]
    int32_t* chosen;  // [B]
    int32_t* status;  // [B] or NULL: 0 ok (no failure mode left: long contours are taken in chunks)
    int runs;         // as CtArgs::runs
};

constexpr int FILL_MAX_CELLS = 64 * 64;  // lattice of a 1280 x 1280 frame
constexpr int FILL_MAX_ROWS = 64, FILL_MAX_COLS = 64;
constexpr int FILL_LDS = 120 * 1024;  // dynamic LDS of the fill kernel (its static arrays take ~37 KiB)

// cv::clipLine(Size(W, H), pt1, pt2): false when the segment misses the image
__device__ bool clip_line(int W, int H, long long& x1, long long& y1, long long& x2, long long& y2) {
    const long long right = W - 1, bottom = H - 1;
    int c1 = (x1 < 0) + (x1 > right) * 2 + (y1 < 0) * 4 + (y1 > bottom) * 8;
    int c2 = (x2 < 0) + (x2 > right) * 2 + (y2 < 0) * 4 + (y2 > bottom) * 8;
    if ((c1 & c2) == 0 && (c1 | c2) != 0) {
        long long t;
        if (c1 & 12) {
            t = c1 < 8 ? 0 : bottom;
            x1 += (long long)((double)(t - y1) * (double)(x2 - x1) / (double)(y2 - y1));
            y1 = t;
            c1 = (x1 < 0) + (x1 > right) * 2;
        }
        if (c2 & 12) {
            t = c2 < 8 ? 0 : bottom;
            x2 += (long long)((double)(t - y2) * (double)(x2 - x1) / (double)(y2 - y1));
            y2 = t;
            c2 = (x2 < 0) + (x2 > right) * 2;
        }
        if ((c1 & c2) == 0 && (c1 | c2) != 0) {
            if (c1) {
                t = c1 == 1 ? 0 : right;
                y1 += (long long)((double)(t - x1) * (double)(y2 - y1) / (double)(x2 - x1));
                x1 = t;
                c1 = 0;
            }
            if (c2) {
                t = c2 == 1 ? 0 : right;
                y2 += (long long)((double)(t - x2) * (double)(y2 - y1) / (double)(x2 - x1));
                x2 = t;
                c2 = 0;
            }
        }
    }
    return (c1 | c2) == 0;
}

__global__ __launch_bounds__(FILL_THREADS) void post_fill_kernel(FillArgs a) {
    extern __shared__ __align__(16) uint32_t fill_lds[];  // FILL_LDS bytes: the chosen instance's image
    __shared__ int s_k, s_n, s_edges, s_px, s_py, s_lx, s_ly;
    __shared__ int s_minx, s_miny, s_maxx, s_maxy;
    __shared__ unsigned long long s_exmin, s_exmax;  // edge x extremes, biased by 2^62
    __shared__ int s_eymin, s_eymax;
    __shared__ unsigned char hit[FILL_MAX_CELLS];
    __shared__ int cnt_a[FILL_MAX_ROWS * (FILL_MAX_COLS + 1)], cnt_b[FILL_MAX_ROWS * (FILL_MAX_COLS + 1)];
    const int tid = threadIdx.x, nt = blockDim.x;
    const Src& s = a.s;
    const int H0 = a.f.H0, W0 = a.f.W0, LR = H0 / VA_GRID, LC = W0 / VA_GRID;
    unsigned char* slot = a.sc.base + (int64_t)blockIdx.x * a.sc.slot_bytes;
    int32_t* pts = (int32_t*)(slot + a.sc.pts_off);
    for (int b = blockIdx.x; b < s.B; b += gridDim.x) {
        uint8_t* out = a.cells + (int64_t)b * LR * LC;
        if (tid == 0) {
            const int nd = s.ndet[b];
            int k = -1;
            if (nd == 1) {
                k = 0;
            } else if (nd > 1) {  // max(xy, key=cv2.contourArea): the first maximum
                double best = -1.0;
                for (int i = 0; i < nd; ++i) {
                    const double ar = a.cstats[(int64_t)b * a.max_det + i].area;
                    if (ar > best) best = ar, k = i;
                }
            }
            if (a.plant_mode == 2 || (nd == 0 && a.plant_mode == 1)) k = -2;  // planted
            s_k = k;
            a.chosen[b] = k;
            if (a.status) a.status[b] = 0;
        }
        __syncthreads();
        const int k = s_k;
        CT_PROF(const unsigned long long f0 = __builtin_amdgcn_s_memtime(); int fb = 0);
        if (k == -2) {
            for (int i = tid; i < LR * LC; i += nt) out[i] = a.plant_cells[(int64_t)b * LR * LC + i];
            if (tid < 4) a.rects[4 * b + tid] = a.plant_rects[4 * b + tid];
            __syncthreads();
            continue;
        }
        for (int i = tid; i < LR * LC; i += nt) {
            hit[i] = 0;
            out[i] = 0;
        }
        for (int i = tid; i < LR * (LC + 1); i += nt) cnt_a[i] = cnt_b[i] = 0;
        if (k < 0) {  // no mask (results.masks is None): no grid
            if (tid < 4) a.rects[4 * b + tid] = 0;
            __syncthreads();
            continue;
        }
        const int64_t di = (int64_t)b * a.max_det + k;
        const va_contour_stat st = a.cstats[di];
        const int n = st.npts;
        if (tid == 0) {
            s_minx = s_miny = INT32_MAX;
            s_maxx = s_maxy = INT32_MIN;
            s_edges = 0;
            s_exmin = ~0ull;
            s_exmax = 0ull;
            s_eymin = INT32_MAX;
            s_eymax = INT32_MIN;
        }
        __syncthreads();
        CT_PROF(const unsigned long long f1 = __builtin_amdgcn_s_memtime(); fb = st.npts > a.sc.capd);
        // boundingRect + the edges of points pts[0, n) (int32 frame points, np.int32 of scale_coords: truncation,
        // >= 0): lines through cell centres, span counts at the sampled rows.  Every term is order-free (min / max,
        // hit flags, counts), so a contour longer than the point buffer is taken a chunk at a time.
        auto edges = [&](const int n, const int px, const int py) {
            for (int i = tid; i < n; i += nt) {
                const int x1i = pts[2 * i], y1i = pts[2 * i + 1];
                // CollectPolyEdges: pt0 = v[count - 1], then v[0], v[1], ...: the predecessor of the chunk's first
                // point is (px, py) -- the contour's last point for the first chunk
                const int x0i = i == 0 ? px : pts[2 * (i - 1)], y0i = i == 0 ? py : pts[2 * (i - 1) + 1];
                atomicMin(&s_minx, x1i);
                atomicMin(&s_miny, y1i);
                atomicMax(&s_maxx, x1i);
                atomicMax(&s_maxy, y1i);
                // cv::Line(img, t0, t1, color, LINE_8): LineIterator(8, leftToRight) after clipLine
                {
                    long long lx1 = x0i, ly1 = y0i, lx2 = x1i, ly2 = y1i;
                    bool ok = true;
                    if (!(lx1 >= 0 && lx1 < W0 && lx2 >= 0 && lx2 < W0 && ly1 >= 0 && ly1 < H0 && ly2 >= 0 && ly2 < H0))
                        ok = clip_line(W0, H0, lx1, ly1, lx2, ly2);
                    if (ok) {  // inside the frame now: int arithmetic
                        int x1 = (int)lx1, y1 = (int)ly1, x2 = (int)lx2, y2 = (int)ly2;
                        int dx = x2 - x1, dy = y2 - y1, sy = 1;
                        if (dx < 0) {
                            dx = -dx, dy = -dy;
                            int t = x1;
                            x1 = x2, x2 = t;
                            t = y1;
                            y1 = y2, y2 = t;
                        }
                        if (dy < 0) dy = -dy, sy = -1;
                        const bool vert = dy > dx;
                        if (vert) {
                            const int t = dx;
                            dx = dy, dy = t;
                        }
                        // The walk (err = dx - 2 dy; per step err -= 2 dy, += 2 dx on a minor step when err < 0)
                        // has taken m_t = (2 dy t + dx - 1) / (2 dx) minor steps after t major ones (exact, checked
                        // against the step-by-step walk for every dy <= dx < 300); only positions on a cell centre
                        // (x = y = 10 mod 20) are kept, so only the major-axis steps landing on 10 mod 20 are
                        // evaluated: dx / 20 of them instead of dx serial 64-bit steps per edge.
                        constexpr int h = VA_GRID / 2;
                        const int m0 = vert ? sy * (h - y1) : h - x1;
                        for (int t = (m0 % VA_GRID + VA_GRID) % VA_GRID; t <= dx; t += VA_GRID) {
                            const int m = dx ? (2 * dy * t + dx - 1) / (2 * dx) : 0;
                            const int x = vert ? x1 + m : x1 + t, y = vert ? y1 + sy * t : y1 + sy * m;
                            if (x >= 0 && y >= 0 && x < W0 && y < H0 && (vert ? x : y) % VA_GRID == h &&
                                CT_OK((y / VA_GRID) * LC + x / VA_GRID < FILL_MAX_CELLS, 10, x, y))
                                hit[(y / VA_GRID) * LC + x / VA_GRID] = 1;
                        }
                    }
                }
                // PolyEdge (CollectPolyEdges, shift 0, line_type < CV_AA)
                if (y0i != y1i) {
                    long long p0x = (long long)x0i << 16, p0y = y0i, p1x = (long long)x1i << 16, p1y = y1i;
                    long long c0x = p0x, c0y = p0y, c1x = p1x, c1y = p1y;
                    if (!(x0i >= 0 && x0i < W0 && x1i >= 0 && x1i < W0 && y0i >= 0 && y0i < H0 && y1i >= 0 && y1i < H0)) {
                        long long t0x = x0i, t0y = y0i, t1x = x1i, t1y = y1i;
                        clip_line(W0, H0, t0x, t0y, t1x, t1y);
                        if (t0y != t1y) {
                            c0y = t0y, c1y = t1y;
                            c0x = t0x << 16, c1x = t1x << 16;
                        }
                    } else {
                        c0x += 1 << 15;
                        c1x += 1 << 15;
                    }
                    const long long edx = (c1x - c0x) / (c1y - c0y);  // C++ truncating division
                    int ey0, ey1;
                    long long ex;
                    if (p0y < p1y) {
                        ey0 = (int)p0y, ey1 = (int)p1y, ex = c0x + (p0y - c0y) * edx;
                    } else {
                        ey0 = (int)p1y, ey1 = (int)p0y, ex = c1x + (p1y - c1y) * edx;
                    }
                    atomicAdd(&s_edges, 1);
                    const long long xend = ex + (long long)(ey1 - ey0) * edx;
                    atomicMin(&s_eymin, ey0);
                    atomicMax(&s_eymax, ey1);
                    constexpr unsigned long long BIAS = 1ull << 62;
                    atomicMin(&s_exmin, (unsigned long long)min(ex, xend) + BIAS);
                    atomicMax(&s_exmax, (unsigned long long)max(ex, xend) + BIAS);
                    // sampled rows cy = 20 r + 10 with ey0 <= cy < ey1
                    int r0 = ey0 <= VA_GRID / 2 ? 0 : (ey0 - VA_GRID / 2 + VA_GRID - 1) / VA_GRID;
                    for (int rr = r0; rr < LR; ++rr) {
                        const int cy = VA_GRID * rr + VA_GRID / 2;
                        if (cy >= ey1) break;
                        const long long xx = ex + (long long)(cy - ey0) * edx;
                        const long long xi = xx >> 16;
                        const long long qa = xi - VA_GRID / 2, qb = xi - VA_GRID / 2 - 1;
                        const long long ca = qa < 0 ? 0 : qa / VA_GRID + 1, cb = qb < 0 ? 0 : qb / VA_GRID + 1;
                        if (ca < LC) atomicAdd(&cnt_a[rr * (LC + 1) + ca], 1);
                        if (cb < LC) atomicAdd(&cnt_b[rr * (LC + 1) + cb], 1);
                    }
                }
            }
            __syncthreads();
        };
        if (st.npts > 0 && st.npts <= a.sc.capd) {
            // the chosen instance's best contour, kept by the contour kernel
            const uint32_t* P = a.sc.cpts + (di * 2 + st.half) * a.sc.capd;
            for (int i = tid; i < st.npts; i += nt) {
                const uint32_t q = P[i];
                float xs, ys;
                scale_pt(a.f, (int)(q & 0xFFFFu), (int)(q >> 16), &xs, &ys);
                pts[2 * i] = (int)xs;
                pts[2 * i + 1] = (int)ys;
            }
            __syncthreads();
            edges(st.npts, pts[2 * (st.npts - 1)], pts[2 * (st.npts - 1) + 1]);
        } else if (st.npts > 0) {
            // longer than the kept buffer: the image rebuilt (in LDS if it fits) and the contour followed again,
            // once per chunk of sc.cap points (pass p stores points [p cap, (p + 1) cap), the point before the
            // chunk and the contour's last point) -- no length limit (a capped buffer dropped the grid)
            const Region r = uni_region(region_of(s, b, k));
            MaskStat ms{0, INT32_MAX, -1, INT32_MAX, -1};
            auto retrace = [&](uint32_t* img, float* strip) {
                build_image<false>(s, b, k, r, img, strip, tid, nt, ms);
                for (int lo = 0;; lo += a.sc.cap) {
                    if (tid < 64) {
                        int i = 0;
                        fetch_contour(img, r.ww, r.rH, a.runs, st.ox, st.oy, [&](int qx, int qy) {
                            if (tid == 0) {
                                float xs, ys;
                                scale_pt(a.f, r.X0 + qx - 1, r.Y0 + qy - 1, &xs, &ys);
                                if (i >= lo && i < lo + a.sc.cap) {
                                    pts[2 * (i - lo)] = (int)xs;
                                    pts[2 * (i - lo) + 1] = (int)ys;
                                }
                                if (i == lo - 1) s_px = (int)xs, s_py = (int)ys;
                                s_lx = (int)xs, s_ly = (int)ys;
                            }
                            ++i;
                        });
                        if (tid == 0) s_n = i;
                    }
                    __syncthreads();
                    const int total = s_n;
                    if (lo >= total) break;
                    const int cnt = total - lo < a.sc.cap ? total - lo : a.sc.cap;
                    edges(cnt, lo == 0 ? s_lx : s_px, lo == 0 ? s_ly : s_py);
                    if (lo + cnt >= total) break;
                }
            };
            // two call sites, each with its own pointer (an LDS / global select would make the accesses flat)
            if (region_need(s, r) <= FILL_LDS) retrace(fill_lds, (float*)(fill_lds + ((image_words(r) + 3) & ~3ll)));
            else retrace((uint32_t*)(slot + a.sc.img_off), (float*)slot);
        }
        CT_PROF(const unsigned long long f2 = __builtin_amdgcn_s_memtime());
        // FillEdgeCollection's early outs: fewer than 2 edges, or all edges outside the image
        constexpr unsigned long long BIAS = 1ull << 62;
        const long long exmin = (long long)(s_exmin - BIAS), exmax = (long long)(s_exmax - BIAS);
        const bool spans = s_edges >= 2 && !(s_eymax < 0 || s_eymin >= H0 || exmax < 0 ||
                                             exmin >= ((long long)W0 << 16));
        for (int rr = tid; rr < LR; rr += nt) {
            int ra = 0, rb = 0;
            for (int c = 0; c < LC; ++c) {
                ra += cnt_a[rr * (LC + 1) + c];
                rb += cnt_b[rr * (LC + 1) + c];
                const bool in = spans && (rb > ra || (ra & 1));
                out[rr * LC + c] = (in || hit[rr * LC + c]) ? 1 : 0;
            }
        }
        if (tid == 0) {
            if (n == 0) {
                a.rects[4 * b + 0] = a.rects[4 * b + 1] = a.rects[4 * b + 2] = a.rects[4 * b + 3] = 0;
            } else {
                a.rects[4 * b + 0] = s_minx;
                a.rects[4 * b + 1] = s_miny;
                a.rects[4 * b + 2] = s_maxx - s_minx + 1;
                a.rects[4 * b + 3] = s_maxy - s_miny + 1;
            }
            CT_PROF(if (b < CT_FILL_FRAMES) {
                unsigned long long* pr = g_ct_fill[b];
                pr[0] = f1 - f0, pr[1] = f2 - f1, pr[2] = __builtin_amdgcn_s_memtime() - f2;
                pr[3] = (unsigned long long)n, pr[4] = (unsigned long long)fb;
            });
        }
        __syncthreads();
    }
}

}  // namespace

// Contour + fill launch for va_post_run and the C-ABI entry points below (internal linkage across the library's
// translation units; not part of va355.h).
hipError_t va_contour_launch(const CtSrc& src, const CtFrame& f, const CtScratch& sc, va_contour_stat* cstats, int max_det,
                             const uint8_t* plant_cells, const int32_t* plant_rects, int plant_mode, uint8_t* cells,
                             int32_t* rects, int32_t* chosen, int32_t* status, float* polys, int32_t* poly_n,
                             int poly_cap, hipStream_t st) {
    static DevFlag pool_attr;  // per device: the pool and fill kernels' dynamic LDS
    if (!pool_attr()) {
        if (hipFuncSetAttribute((const void*)post_contour_pool_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                CP_POOL) != hipSuccess ||
            hipFuncSetAttribute((const void*)post_contour_wg_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                CT_WG_LDS) != hipSuccess ||
            hipFuncSetAttribute((const void*)post_contour_wgp_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                CT_WG_LDS) != hipSuccess ||
            hipFuncSetAttribute((const void*)post_fill_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                FILL_LDS) != hipSuccess)
            return hipErrorInvalidValue;
        pool_attr() = true;
    }
    if (src.mw > CT_STRIP / 2) return hipErrorInvalidValue;  // a strip holds >= 2 low-res rows
    CtArgs ca;
    ca.s = src;
    ca.f = f;
    ca.sc = sc;
    ca.cstats = cstats;
    ca.max_det = max_det;
    ca.polys = polys;
    ca.poly_n = poly_n;
    ca.poly_cap = poly_cap;
    ca.gate = 1;
    ca.runs = va_sw().ct_runs ? 1 : 0;  // VA_CT_RUNS=0: border following pixel by pixel (A/B, va_switch.h)
    ca.pages = CP_PAGES;                // the pool form's LDS: all 32 pages (160 KiB)
    ca.pool_max = (int64_t)CP_PAGES * CP_PAGE;
    const int64_t items = (int64_t)src.B * max_det;
    static DevVal<int> n_cu;  // per device: one pool block per CU
    if (n_cu() <= 0) {
        int dev = 0, cus = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            return hipErrorInvalidValue;
        n_cu() = cus;
    }
    const int pgrid = (int)(items < n_cu() ? items : n_cu());
    const int grid = (int)(items < sc.nslots ? items : sc.nslots);
    // a slot per detection (small batches): the workgroup-per-detection form
    // larger batches: the persistent workgroup form, one 160 KiB workgroup per CU (VA_CT_WGP=0 keeps the pool form,
    // A/B, va_switch.h); its claim counter and frame prefix live in the last scratch slot
    int32_t* cbuf = (int32_t*)(sc.base + (int64_t)(sc.nslots - 1) * sc.slot_bytes);
    if (items <= sc.nslots) {
        hipLaunchKernelGGL(post_contour_wg_kernel, dim3((int)items), dim3(CT_WG_THREADS), CT_WG_LDS, st, ca);
    } else if (va_sw().ct_wgp && sc.nslots >= 2 && (int64_t)(src.B + 2) * 4 <= sc.slot_bytes) {
        hipLaunchKernelGGL(ct_prefix_kernel, dim3(1), dim3(1024), 0, st, src.ndet, src.B, max_det, cbuf);
        const int lds = CT_WG_LDS;
        const int g = n_cu() < sc.nslots - 1 ? n_cu() : sc.nslots - 1;
        hipLaunchKernelGGL(post_contour_wgp_kernel, dim3(g), dim3(CT_WG_THREADS), lds, st, ca, cbuf, lds);
    } else {
        hipLaunchKernelGGL(post_contour_pool_kernel, dim3(pgrid), dim3(CP_THREADS), (size_t)ca.pages * CP_PAGE, st,
                           ca);
        hipLaunchKernelGGL(post_contour_global_kernel, dim3(grid), dim3(CT_THREADS), 0, st, ca);
    }
    if (hipGetLastError() != hipSuccess) return hipErrorLaunchFailure;
    if (!cells) return hipSuccess;
    FillArgs fa;
    fa.s = src;
    fa.f = f;
    fa.sc = sc;
    fa.cstats = cstats;
    fa.max_det = max_det;
    fa.plant_cells = plant_cells;
    fa.plant_rects = plant_rects;
    fa.plant_mode = plant_mode;
    fa.cells = cells;
    fa.rects = rects;
    fa.chosen = chosen;
    fa.status = status;
    fa.runs = ca.runs;
    const int fgrid = src.B < sc.nslots ? src.B : sc.nslots;
    hipLaunchKernelGGL(post_fill_kernel, dim3(fgrid), dim3(FILL_THREADS), FILL_LDS, st, fa);
    return hipGetLastError();
}

namespace {
bool frame_ok(int H0, int W0) {
    return H0 > 0 && W0 > 0 && H0 % VA_GRID == 0 && W0 % VA_GRID == 0 && H0 / VA_GRID <= FILL_MAX_ROWS &&
           W0 / VA_GRID <= FILL_MAX_COLS;
}
}  // namespace

extern "C" {

int va_contour_scratch_bytes(int32_t Hn, int32_t Wn, int32_t nslots, int32_t cap, int64_t* slot_bytes,
                             int64_t* img_off, int64_t* pts_off) {
    if (Hn <= 0 || Wn <= 0 || Hn % 4 || Wn % 4 || nslots <= 0 || cap <= 0) return VA_ERR_ARG;
    const int64_t strip = (int64_t)CT_STRIP * 4;
    const int64_t img = (((int64_t)(Hn + 2) * 3 * (((Wn + 2) + 31) / 32) + 1) * 4 + 255) & ~255ll;
    const int64_t pts = (int64_t)cap * 8;
    *img_off = strip;
    *pts_off = strip + img;
    *slot_bytes = strip + img + pts;
    return VA_OK;
}

int va_post_select_masks(void* stream, const va_mask_select_args* m) {
    if (!m || !m->masks || !m->nmask || m->B <= 0 || m->maxn <= 0 || m->Hn <= 0 || m->Wn <= 0 || !m->scratch ||
        m->nslots <= 0 || m->cap <= 0 || !m->cstats || !frame_ok(m->H0, m->W0) || !(m->gain > 0.0f) ||
        (m->cells && (!m->rects || !m->chosen)) || m->Hn % 4 || m->Wn % 4 || m->Hn > 65535 || m->Wn > 65535 ||
        !m->cpts || m->cpts_cap <= 0 || m->cpts_cap > m->cap)
        return VA_ERR_ARG;
    Src src{};
    src.masks = m->masks;
    src.maxn = m->maxn;
    src.ndet = m->nmask;
    src.B = m->B;
    src.Hn = m->Hn;
    src.Wn = m->Wn;
    src.mh = m->Hn / 4;
    src.mw = m->Wn / 4;
    src.max_det = m->maxn;
    Frame f{m->H0, m->W0, m->gain, m->padx, m->pady};
    Scratch sc{(unsigned char*)m->scratch, 0, 0, 0, m->nslots, m->cap, m->cpts, m->cpts_cap};
    if (va_contour_scratch_bytes(m->Hn, m->Wn, m->nslots, m->cap, &sc.slot_bytes, &sc.img_off, &sc.pts_off) != VA_OK)
        return VA_ERR_ARG;
    const hipError_t e = va_contour_launch(src, f, sc, m->cstats, m->maxn, nullptr, nullptr, 0, m->cells, m->rects,
                                           m->chosen, m->status, m->polys, m->poly_n, m->poly_cap,
                                           (hipStream_t)stream);
    return e == hipSuccess ? VA_OK : VA_ERR_HIP;
}

}  // extern "C"

#ifdef VA_CT_CHECK
extern "C" int va_contour_prof(unsigned long long* out, int n) {
    if (hipDeviceSynchronize() != hipSuccess) return VA_ERR_HIP;
    if (n > CT_PROF_ITEMS) n = CT_PROF_ITEMS;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ct_prof), sizeof(unsigned long long) * 8 * n) != hipSuccess)
        return VA_ERR_HIP;
    return VA_OK;
}

extern "C" int va_contour_fill_prof(unsigned long long* out, int n) {
    if (hipDeviceSynchronize() != hipSuccess) return VA_ERR_HIP;
    if (n > CT_FILL_FRAMES) n = CT_FILL_FRAMES;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ct_fill), sizeof(unsigned long long) * 8 * n) != hipSuccess)
        return VA_ERR_HIP;
    return VA_OK;
}

extern "C" int va_contour_debug(unsigned int* out4, int reset) {
    if (hipDeviceSynchronize() != hipSuccess) return VA_ERR_HIP;
    if (hipMemcpyFromSymbol(out4, HIP_SYMBOL(g_ct_err), sizeof(unsigned int) * 4) != hipSuccess) return VA_ERR_HIP;
    if (reset) {
        const unsigned int z[4] = {0, 0, 0, 0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_ct_err), z, sizeof(z)) != hipSuccess) return VA_ERR_HIP;
    }
    return VA_OK;
}
#endif

#ifdef VA_CT_WATCH
extern "C" int va_contour_watch(void** host) {
    static int* h = nullptr;
    if (!h) {
        if (hipHostMalloc((void**)&h, sizeof(int) * 4 * CT_WATCH_SLOTS, hipHostMallocMapped | hipHostMallocCoherent) !=
            hipSuccess)
            return VA_ERR_HIP;
        memset(h, 0xFF, sizeof(int) * 4 * CT_WATCH_SLOTS);
        int* d = nullptr;
        if (hipHostGetDevicePointer((void**)&d, h, 0) != hipSuccess) return VA_ERR_HIP;
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_ct_watch), &d, sizeof(d)) != hipSuccess) return VA_ERR_HIP;
    }
    *host = h;
    return VA_OK;
}
#endif

int va_diag_contour(unsigned int* out4, int clear) { return diag_read_tu(out4, clear); }

// va_contour.hip -- the mask -> polygon -> cells boundary of FrameProcessor.py:67-97 on MI355X (gfx950).
//
// The reference reduces the chosen YOLO mask to grid cells through OpenCV (Results.masks.xy = masks2segments
// (findContours RETR_EXTERNAL / CHAIN_APPROX_SIMPLE, the contour with the most points) + scale_coords, then
// max(xy, key=contourArea), np.int32, boundingRect, fillPoly, cell-centre sampling).  OpenCV is third-party and
// absent here; its published algorithms are restated exactly as oracle/contours.py restates them (that module is
// the checker; the cv2 parity itself is unpinned):
//
//   post_contour_kernel  one wave per detection (persistent over slots): the instance mask -- bilinear x4 of the
//                        cropped coef . proto, > 0 (or a given binary mask) -- as a framed byte image in the slot's
//                        scratch (global memory: a few KiB to 400 KiB, L2-resident while it is followed; a
//                        generic pointer that may point into LDS faulted on gfx950 under the atomics below); the
//                        raster scan of cvFindNextContour and Suzuki-Abe border following (icvFetchContour) for
//                        every outer border RETR_EXTERNAL keeps; the contour with the most CHAIN_APPROX_SIMPLE
//                        points, re-followed once for its cv2.contourArea over the float32 scale_coords points
//                        (double shoelace in OpenCV's order).  -> va_contour_stat.
//   post_fill_kernel     one workgroup per frame: the instance max(area) picks (first maximum; a single detection
//                        is taken as it is), its best contour followed again into int32 frame points
//                        (np.int32 of the float32 scale_coords), boundingRect, and cv2.fillPoly(LINE_8) evaluated
//                        only at the cell centres: a centre is set when an edge's 8-connected Bresenham line
//                        (LineIterator + clipLine) passes through it, or when it lies in a FillEdgeCollection span --
//                        with a = #active edges left of the pixel and b = #active edges left of its right neighbour
//                        (16.16 edge x at that row), the pixel is inside a pair iff b > a or a is odd, an
//                        order-free count the threads accumulate with LDS atomics.
//
// Pixel states of the byte image: bit 0 = non-zero mask pixel, bit 1 = traced border pixel (OpenCV's nbd = 2),
// bit 2 = traced "right" border pixel (OpenCV's nbd | -128).  A border visit ORs its bit in (atomicOr on the
// pixel's word): OpenCV's per-visit update "cond ? -126 : (v == 1 ? 2 : v)" reaches the same final value in any
// visit order, so a trace never has to read back its own marks.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/va355.h"
#include "va_contour.h"
#include "va_dev.h"

namespace {

constexpr int NMC = 32;
constexpr int REG_MAX = 16;
constexpr int CT_THREADS = 64;       // one wave per detection: the scan and the border following are serial
constexpr int FILL_THREADS = 256;
__constant__ int c_dx[8] = {1, 1, 0, -1, -1, -1, 0, 1};
__constant__ int c_dy[8] = {0, -1, -1, -1, 0, 1, 1, 1};

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
#else
#define CT_OK(c, code, v0, v1) true
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
    int rW, rH, ww;    // framed size in pixels, words per row
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
        // full-res pixels whose taps can touch the window (post_mask_kernel's footprint)
        r.X0 = max(0, (int)((r.rx0 - 1) / sx) - 2);
        const int X1 = min(s.Wn - 1, (int)((r.rx1 + 1) / sx) + 2);
        r.Y0 = max(0, (int)((r.ry0 - 1) / sy) - 2);
        const int Y1 = min(s.Hn - 1, (int)((r.ry1 + 1) / sy) + 2);
        r.w = X1 - r.X0 + 1;
        r.h = Y1 - r.Y0 + 1;
    }
    r.rW = r.w + 2;
    r.rH = r.h + 2;
    r.ww = (r.rW + 3) / 4;
    return r;
}

// ------------------------------------------------------------------------------------------ the byte image
// word i holds pixels 4 (i % ww) .. +3 of row i / ww (byte j = pixel 4 (i % ww) + j)
struct Img {
    uint32_t* p;
    int ww, nw;  // words per row, words
    __device__ inline bool in(int x, int y, int code) const {
        return CT_OK(x >= 0 && y >= 0 && (x >> 2) < ww && y * ww + (x >> 2) < nw, code, x, y);
    }
    __device__ inline int nz(int x, int y) const {  // bit 0 never changes: plain load
        if (!in(x, y, 1)) return 0;
        return (p[y * ww + (x >> 2)] >> (8 * (x & 3))) & 1;
    }
    __device__ inline int val(int x, int y) const {  // OpenCV's value of the pixel (marks: coherent load)
        if (!in(x, y, 2)) return 0;
        const uint32_t w = __hip_atomic_load(p + y * ww + (x >> 2), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int v = (int)((w >> (8 * (x & 3))) & 0xFF);
        return (v & 4) ? -126 : (v & 2) ? 2 : (v & 1);
    }
    __device__ inline void mark(int x, int y, bool right) const {
        if (!in(x, y, 3)) return;
        atomicOr(p + y * ww + (x >> 2), (right ? 4u : 2u) << (8 * (x & 3)));
    }
};

// Build the framed image of detection (b, k) into img (region r) with nt threads of the calling block.
// lowres: scratch of (ry1 - ry0 + 1) x (rx1 - rx0 + 1) floats (head source only).
__device__ void build_image(const Src& s, int b, int k, const Region& r, Img img, float* lowres, int tid, int nt) {
    const int nwords = r.rH * r.ww;
    if (s.masks) {
        const uint8_t* m = s.masks + ((int64_t)b * s.maxn + k) * s.Hn * s.Wn;
        for (int i = tid; i < nwords; i += nt) {
            const int y = i / r.ww, x4 = 4 * (i % r.ww);
            uint32_t w = 0;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int x = x4 + j;
                if (y >= 1 && y <= r.h && x >= 1 && x <= r.w && m[(int64_t)(y - 1) * s.Wn + (x - 1)]) w |= 1u << (8 * j);
            }
            if (CT_OK(i < img.nw, 4, i, img.nw)) img.p[i] = w;
        }
        __syncthreads();
        return;
    }
    // low-res window of coef . proto: 8 lanes per pixel, one 16-byte run of its 32 channels each (the dot of
    // post_mask_kernel, same partial sums and reduction order)
    const int anchor = s.dets[(int64_t)b * s.max_det + k].anchor;
    [[maybe_unused]] const int na = (s.Hn / 8) * (s.Wn / 8) + (s.Hn / 16) * (s.Wn / 16) + (s.Hn / 32) * (s.Wn / 32);
    if (!CT_OK(anchor >= 0 && anchor < na, 13, anchor, na)) return;  // (debug build only)
    const float* coef = coef_row(s, b, anchor);
    const int tw = r.rx1 - r.rx0 + 1, th = r.ry1 - r.ry0 + 1;
    const int sub = tid & 7;
    const float4 cq = *(const float4*)(coef + 4 * sub);
    for (int i = tid >> 3; i < tw * th; i += nt / 8) {
        const int y = r.ry0 + i / tw, x = r.rx0 + i % tw;
        if (!CT_OK(y >= 0 && y < s.mh && x >= 0 && x < s.mw, 5, x, y)) continue;  // (debug build only)
        const float4 v = *(const float4*)(s.proto + (((int64_t)b * s.mh + y) * s.mw + x) * NMC + 4 * sub);
        float sdot = (cq.x * v.x + cq.y * v.y) + (cq.z * v.z + cq.w * v.w);
        sdot += __shfl_xor(sdot, 1, 8);
        sdot += __shfl_xor(sdot, 2, 8);
        sdot += __shfl_xor(sdot, 4, 8);
        if (sub == 0 && CT_OK(i < s.mh * s.mw, 6, i, tw)) lowres[i] = sdot;
    }
    __syncthreads();
    const float sx = (float)s.mw / (float)s.Wn, sy = (float)s.mh / (float)s.Hn;
    auto val = [&](int yy, int xx) -> float {
        if (xx < r.rx0 || xx > r.rx1 || yy < r.ry0 || yy > r.ry1) return 0.f;
        const int li = (yy - r.ry0) * tw + (xx - r.rx0);
        if (!CT_OK(li >= 0 && li < s.mh * s.mw, 7, li, tw)) return 0.f;
        return lowres[li];
    };
    for (int i = tid; i < nwords; i += nt) {
        const int y = i / r.ww, x4 = 4 * (i % r.ww);
        uint32_t w = 0;
        if (y >= 1 && y <= r.h) {
            const int Y = r.Y0 + y - 1;
            int ya, yb;
            float wy0, wy1;
            taps(Y, sy, s.mh, &ya, &yb, &wy0, &wy1);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int x = x4 + j;
                if (x < 1 || x > r.w) continue;
                const int X = r.X0 + x - 1;
                int xa, xb;
                float wx0, wx1;
                taps(X, sx, s.mw, &xa, &xb, &wx0, &wx1);
                const float A = val(ya, xa), B = val(ya, xb), C = val(yb, xa), D = val(yb, xb);
                const float ha = wx0 * A + wx1 * B, hb = wx0 * C + wx1 * D;
                if (wy0 * ha + wy1 * hb > 0.f) w |= 1u << (8 * j);
            }
        }
        if (CT_OK(i < img.nw, 8, i, img.nw)) img.p[i] = w;
    }
    __syncthreads();
}

// ------------------------------------------------------------------------------------------ border following
// icvFetchContour (CHAIN_APPROX_SIMPLE) from the outer-border start (x0, y0) of the framed image, executed by the
// whole wave in lock step (lanes 0-7 fetch the 8 neighbours of the current pixel).  emit(x, y) gets every kept
// point in order; mark = whether to write the traced pixels' marks.  Returns the number of points.
template <typename Emit>
__device__ int fetch_contour(Img img, int x0, int y0, bool mark, Emit emit) {
    const int lane = threadIdx.x & 63;
    const int ld = lane & 7;
    auto nbrs = [&](int x, int y) -> unsigned {  // bit d = neighbour in direction d is non-zero
        const int nzv = lane < 8 ? img.nz(x + c_dx[ld], y + c_dy[ld]) : 0;
        return (unsigned)(__ballot(nzv != 0) & 0xFFull);
    };
    unsigned nb = nbrs(x0, y0);
    int s = 4;  // outer border: s_end = s = 4
    const int s_end0 = 4;
    do {
        s = (s - 1) & 7;
    } while (!((nb >> s) & 1) && s != s_end0);
    if (s == s_end0) {  // single pixel domain
        if (mark && lane == 0) img.mark(x0, y0, true);
        emit(x0, y0);
        return 1;
    }
    const int x1 = x0 + c_dx[s], y1 = y0 + c_dy[s];  // i1
    int x3 = x0, y3 = y0;
    int prev_s = s ^ 4, n = 0;
    int px = x0, py = y0;
    unsigned nb3 = nb;
    while (true) {
        const int s_end = s;
        // counter-clockwise from s_end + 1 to the first non-zero neighbour
        int t = s_end + 1;
        while (!((nb3 >> (t & 7)) & 1)) ++t;
        s = t & 7;
        const int x4 = x3 + c_dx[s], y4 = y3 + c_dy[s];
        if (mark && lane == 0) img.mark(x3, y3, (unsigned)(s - 1) < (unsigned)s_end);
        if (s != prev_s) {
            emit(px, py);
            ++n;
            prev_s = s;
        }
        px += c_dx[s];
        py += c_dy[s];
        if (x4 == x0 && y4 == y0 && x3 == x1 && y3 == y1) break;
        x3 = x4;
        y3 = y4;
        s = (s + 4) & 7;
        nb3 = nbrs(x3, y3);
    }
    return n;
}

// The first position >= x of row y whose value differs from prev (OpenCV's skip loop), or width.  Wave-wide.
__device__ inline int next_stop(Img img, int y, int x, int width, int prev) {
    const int lane = threadIdx.x & 63;
    while (x < width) {
        const int xx = x + lane;
        const bool d = xx < width && img.val(xx, y) != prev;
        const unsigned long long m = __ballot(d);
        if (m) return x + __builtin_ctzll(m);
        x += 64;
    }
    return width;
}

// float32 scale_coords of a network point (ops.py:784-816)
__device__ inline void scale_pt(const Frame& f, int X, int Y, float* xs, float* ys) {
    *xs = fminf(fmaxf(((float)X - f.padx) / f.gain, 0.0f), (float)f.W0);
    *ys = fminf(fmaxf(((float)Y - f.pady) / f.gain, 0.0f), (float)f.H0);
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
};

__global__ __launch_bounds__(CT_THREADS) void post_contour_kernel(CtArgs a) {
    __shared__ unsigned char rowflag[4096];
    const int tid = threadIdx.x;
    const Src& s = a.s;
    unsigned char* slot = a.sc.base + (int64_t)blockIdx.x * a.sc.slot_bytes;
    const int total = s.B * a.max_det;
    for (int item = blockIdx.x; item < total; item += gridDim.x) {
        const int b = item / a.max_det, k = item % a.max_det;
        const int nd = s.ndet[b];
        if (k >= nd) continue;  // block-uniform
        va_contour_stat st{};
        st.ox = st.oy = -1;
        const Region r = region_of(s, b, k);
        if (r.w > 0 && r.rH <= 4096) {
            Img img{(uint32_t*)(slot + a.sc.img_off), r.ww, r.rH * r.ww};
            build_image(s, b, k, r, img, (float*)slot, tid, CT_THREADS);
            // rows with a 0 -> 1 transition (no other row can start a border): per word, bit 0 of each byte
            // against the byte before it
            for (int y = tid; y < r.rH; y += CT_THREADS) rowflag[y] = 0;
            __syncthreads();
            for (int i = tid; i < r.rH * r.ww; i += CT_THREADS) {
                const int y = i / r.ww, wx = i % r.ww;
                const uint32_t cur = img.p[i] & 0x01010101u;
                const uint32_t before = (cur << 8) | (wx ? (img.p[i - 1] >> 24) & 1u : 0u);
                if (cur & ~before) rowflag[y] = 1;
            }
            __syncthreads();
            // cvFindNextContour's raster scan (RETR_EXTERNAL); best = the contour with the most points
            int best_n = 0, bx = -1, by = -1, blx = 0, bly = 0, ncont = 0;
            for (int y = 1; y < r.rH - 1; ++y) {
                if (!rowflag[y]) continue;
                int x = 1, prev = 0, lnbd = 0;
                while (true) {
                    x = next_stop(img, y, x, r.rW, prev);
                    if (x >= r.rW) break;
                    const int p = img.val(x, y);
                    if (prev == 0 && p == 1) {
                        if (img.val(lnbd, y) <= 0) {
                            int lx = 0, ly = 0;
                            const int n = fetch_contour(img, x, y, true, [&](int px, int py) { lx = px, ly = py; });
                            ++ncont;
                            if (n > best_n) {
                                best_n = n, bx = x, by = y, blx = lx, bly = ly;
                            }
                            __threadfence();  // the marks (atomics at L2) before the scan reads on
                            prev = img.val(x, y);
                            ++x;
                            continue;
                        }
                    } else if (p == 0 && prev >= 1) {
                        if (prev & -2) lnbd = x - 1;
                    }
                    prev = p;
                    if (p & -2) lnbd = x;
                    ++x;
                }
            }
            st.npts = best_n;
            st.ncont = ncont;
            if (best_n > 0) {
                st.ox = bx, st.oy = by;
                // cv2.contourArea of the float32 scale_coords points, from the last point on (OpenCV's order)
                float pxs, pys;
                scale_pt(a.f, r.X0 + blx - 1, r.Y0 + bly - 1, &pxs, &pys);
                double a00 = 0.0;
                float* poly = a.polys ? a.polys + ((int64_t)b * a.max_det + k) * a.poly_cap * 2 : nullptr;
                int i = 0;
                fetch_contour(img, bx, by, false, [&](int qx, int qy) {
                    float xs, ys;
                    scale_pt(a.f, r.X0 + qx - 1, r.Y0 + qy - 1, &xs, &ys);
                    a00 += (double)pxs * (double)ys - (double)pys * (double)xs;
                    pxs = xs, pys = ys;
                    if (poly && i < a.poly_cap && tid == 0) {
                        poly[2 * i] = xs;
                        poly[2 * i + 1] = ys;
                    }
                    ++i;
                });
                st.area = fabs(a00 * 0.5);
                if (a.poly_n && tid == 0) a.poly_n[(int64_t)b * a.max_det + k] = best_n;
            } else if (a.poly_n && tid == 0) {
                a.poly_n[(int64_t)b * a.max_det + k] = 0;
            }
            st.X0 = r.X0, st.Y0 = r.Y0;
        } else {
            st.status = r.w > 0 ? 1 : 0;  // 1: region taller than the row-flag table
            if (a.poly_n && tid == 0) a.poly_n[(int64_t)b * a.max_det + k] = 0;
        }
        if (tid == 0) a.cstats[(int64_t)b * a.max_det + k] = st;
        __syncthreads();  // the slot image is reused by the next item
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
    int32_t* status;  // [B] or NULL: 0 ok, 1 contour larger than the point buffer
};

constexpr int FILL_MAX_CELLS = 64 * 64;  // lattice of a 1280 x 1280 frame
constexpr int FILL_MAX_ROWS = 64, FILL_MAX_COLS = 64;

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
    __shared__ int s_k, s_n, s_edges;
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
        const va_contour_stat st = a.cstats[(int64_t)b * a.max_det + k];
        if (st.npts > a.sc.cap) {
            if (tid == 0 && a.status) a.status[b] = 1;
            if (tid < 4) a.rects[4 * b + tid] = 0;
            __syncthreads();
            continue;
        }
        // the chosen instance's best contour, followed again into int32 frame points (np.int32 of scale_coords)
        if (st.npts > 0) {
            const Region r = region_of(s, b, k);
            Img img{(uint32_t*)(slot + a.sc.img_off), r.ww, r.rH * r.ww};
            build_image(s, b, k, r, img, (float*)slot, tid, nt);
            if (tid < 64) {
                int i = 0;
                fetch_contour(img, st.ox, st.oy, false, [&](int qx, int qy) {
                    float xs, ys;
                    scale_pt(a.f, r.X0 + qx - 1, r.Y0 + qy - 1, &xs, &ys);
                    if (tid == 0 && i < a.sc.cap && CT_OK(xs >= 0.f && ys >= 0.f, 9, xs, ys)) {
                        pts[2 * i] = (int)xs;  // np.int32: truncation (the values are >= 0)
                        pts[2 * i + 1] = (int)ys;
                    }
                    ++i;
                });
                if (tid == 0) s_n = i;
            }
        } else if (tid == 0) {
            s_n = 0;
        }
        if (tid == 0) {
            s_minx = s_miny = INT32_MAX;
            s_maxx = s_maxy = INT32_MIN;
            s_edges = 0;
            s_exmin = ~0ull;
            s_exmax = 0ull;
            s_eymin = INT32_MAX;
            s_eymax = INT32_MIN;
        }
        __threadfence_block();
        __syncthreads();
        const int n = s_n;
        // boundingRect + the edges: lines through cell centres, span counts at the sampled rows
        for (int i = tid; i < n; i += nt) {
            const int x1i = pts[2 * i], y1i = pts[2 * i + 1];
            const int j = i == 0 ? n - 1 : i - 1;  // CollectPolyEdges: pt0 = v[count - 1], then v[0], v[1], ...
            const int x0i = pts[2 * j], y0i = pts[2 * j + 1];
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
                if (ok) {
                    long long dx = lx2 - lx1, dy = ly2 - ly1;
                    long long sy = 1;
                    if (dx < 0) {
                        dx = -dx, dy = -dy;
                        long long t = lx1;
                        lx1 = lx2, lx2 = t;
                        t = ly1;
                        ly1 = ly2, ly2 = t;
                    }
                    if (dy < 0) dy = -dy, sy = -1;
                    const bool vert = dy > dx;
                    if (vert) {
                        const long long t = dx;
                        dx = dy, dy = t;
                    }
                    long long err = dx - (dy + dy);
                    const long long plus = dx + dx, minus = -(dy + dy);
                    long long x = lx1, y = ly1;
                    for (long long st2 = 0; st2 <= dx; ++st2) {
                        if (x % VA_GRID == VA_GRID / 2 && y % VA_GRID == VA_GRID / 2 && x >= 0 && y >= 0 && x < W0 &&
                            y < H0)
                            if (CT_OK((y / VA_GRID) * LC + x / VA_GRID < FILL_MAX_CELLS, 10, x, y))
                                hit[(y / VA_GRID) * LC + x / VA_GRID] = 1;
                        const bool minor = err < 0;
                        err += minus + (minor ? plus : 0);
                        if (vert) {
                            y += sy;
                            x += minor ? 1 : 0;
                        } else {
                            x += 1;
                            y += minor ? sy : 0;
                        }
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
                    if (ca < LC && CT_OK(ca >= 0, 11, ca, rr)) atomicAdd(&cnt_a[rr * (LC + 1) + ca], 1);
                    if (cb < LC && CT_OK(cb >= 0, 12, cb, rr)) atomicAdd(&cnt_b[rr * (LC + 1) + cb], 1);
                }
            }
        }
        __syncthreads();
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
    CtArgs ca;
    ca.s = src;
    ca.f = f;
    ca.sc = sc;
    ca.cstats = cstats;
    ca.max_det = max_det;
    ca.polys = polys;
    ca.poly_n = poly_n;
    ca.poly_cap = poly_cap;
    const int64_t items = (int64_t)src.B * max_det;
    const int grid = (int)(items < sc.nslots ? items : sc.nslots);
    hipLaunchKernelGGL(post_contour_kernel, dim3(grid), dim3(CT_THREADS), 0, st, ca);
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
    const int fgrid = src.B < sc.nslots ? src.B : sc.nslots;
    hipLaunchKernelGGL(post_fill_kernel, dim3(fgrid), dim3(FILL_THREADS), 0, st, fa);
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
    const int64_t lowres = ((int64_t)(Hn / 4) * (Wn / 4) * 4 + 255) & ~255ll;
    const int64_t img = ((int64_t)(Hn + 2) * (((Wn + 2) + 3) / 4) * 4 + 255) & ~255ll;
    const int64_t pts = (int64_t)cap * 8;
    *img_off = lowres;
    *pts_off = lowres + img;
    *slot_bytes = lowres + img + pts;
    return VA_OK;
}

}  // extern "C"

extern "C" {

int va_post_select_masks(void* stream, const va_mask_select_args* m) {
    if (!m || !m->masks || !m->nmask || m->B <= 0 || m->maxn <= 0 || m->Hn <= 0 || m->Wn <= 0 || !m->scratch ||
        m->nslots <= 0 || m->cap <= 0 || !m->cstats || !frame_ok(m->H0, m->W0) || !(m->gain > 0.0f) ||
        (m->cells && (!m->rects || !m->chosen)) || m->Hn + 2 > 4096 || m->Hn % 4 || m->Wn % 4)
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
    Scratch sc{(unsigned char*)m->scratch, 0, 0, 0, m->nslots, m->cap};
    if (va_contour_scratch_bytes(m->Hn, m->Wn, m->nslots, m->cap, &sc.slot_bytes, &sc.img_off, &sc.pts_off) != VA_OK)
        return VA_ERR_ARG;
    const hipError_t e = va_contour_launch(src, f, sc, m->cstats, m->maxn, nullptr, nullptr, 0, m->cells, m->rects,
                                           m->chosen, m->status, m->polys, m->poly_n, m->poly_cap,
                                           (hipStream_t)stream);
    return e == hipSuccess ? VA_OK : VA_ERR_HIP;
}

}  // extern "C"

#ifdef VA_CT_CHECK
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

// va_nav.hip -- grid-level hot path of vision-assist on MI355X (gfx950).
//
// Kernels (one HIP launch each, all on the caller's stream):
//   nav_sample_kernel   mask pixels -> cell-lattice samples         FrameProcessor.py:88-97
//   nav_grid_kernel     one 256-thread workgroup per frame:
//                         grid list + artificial rows (Q9/Q10 list semantics)  FrameProcessor.py:50-171
//                         easy segments + per-cell penalties                   PenaltyCalculator.py:26-142
//                         implicit 4-neighbour graph (+ duplicate-row lists)  FrameProcessor.py:184-207
//                         top-row protrusion peaks                             ProtrusionDetector.py:38-158,419-535
//                         start / end cells                                    utils.py:6-32
//   nav_astar_kernel    one wave64 per A* query, whole search state in LDS     PathFinder.py:119-186
//   nav_validate_kernel serial check of the speculative angle-cache rounds     PathFinder.py:32 (global cache)
//   nav_dedupe_kernel   one wave per frame: Jaccard / subset path filter       FrameProcessor.py:209-271
//
// Bit-exactness notes:
//   * all float64 arithmetic is written in the reference's operation order and the
//     file is compiled with -ffp-contract=off (no FMA contraction);
//   * A* pops argmin (push-time f, x, y) with no decrease-key (Q4); the angle term
//     uses the O(1) newest-window rule (Q3) and the 128-entry table of
//     va_angle_table.h (Q1/Q5);
//   * the process-global angle cache makes queries depend on every earlier query
//     (Q2).  Queries of a batch run speculatively in parallel against the seen set
//     at batch start; nav_validate_kernel finds the first query whose newly-missed
//     keys were already added by an earlier query, and the driver re-runs from
//     there with the corrected set.  Every round adds >= 1 key, so a process needs
//     at most 128 re-run rounds in its whole lifetime.
#include <hip/hip_runtime.h>
#include <map>
#include <mutex>
#include <stdint.h>
#include <string.h>

#include "../../include/va355.h"
#include "va_dev.h"
#include "va_diag.h"
#include "va_angle_table.h"

#define VA_MAX_LAT 64          // max lattice rows / cols (1280 px)
#define VA_NAV_THREADS 256

__constant__ double c_angle_pen[128];
__constant__ int8_t c_prev_idx[7 * 7];  // (dx+3)*7 + (dy+3) -> prev index or -1
__constant__ int8_t c_next_idx[5 * 5];  // (dx+2)*5 + (dy+2) -> next index or -1

namespace {

struct Dims {
    int H, W, LR, LC, start_y, NART, PMAX, MAXPK, NODES;
    int64_t frame_bytes, off_hdr, off_peaks, off_pos_obj, off_pos_y, off_pos_attr, off_cell_flags, off_cell_pen,
        off_node_flags, off_node_pen, query_bytes, off_q_hdr, off_q_path;
};

__host__ __device__ inline int64_t align16(int64_t v) { return (v + 15) & ~int64_t(15); }

bool make_dims(int H, int W, Dims* d) {
    if (H <= 0 || W <= 0 || H % VA_GRID || W % VA_GRID) return false;
    d->H = H;
    d->W = W;
    d->LR = H / VA_GRID;
    d->LC = W / VA_GRID;
    if (d->LR > VA_MAX_LAT || d->LC > VA_MAX_LAT) return false;
    int sy = (7 * H) / 8;  // int(H * 0.875): H*0.875 is exact in binary64
    sy = sy + (VA_GRID - sy % VA_GRID) % VA_GRID;
    d->start_y = sy;
    d->NART = sy < H ? (H - sy) / VA_GRID : 0;
    d->PMAX = d->LR + d->NART;
    d->MAXPK = (d->LC + 1) / 2;
    d->NODES = d->LR * d->LC;
    int64_t o = 0;
    d->off_hdr = o;
    o = align16(o + (int64_t)sizeof(va_frame_hdr));
    d->off_peaks = o;
    o = align16(o + 4 * 4 * (int64_t)d->MAXPK);
    d->off_pos_obj = o;
    o = align16(o + 2 * (int64_t)d->PMAX);
    d->off_pos_y = o;
    o = align16(o + 2 * (int64_t)d->PMAX);
    d->off_pos_attr = o;
    o = align16(o + 2 * (int64_t)d->PMAX);
    d->off_cell_flags = o;
    o = align16(o + (int64_t)d->PMAX * d->LC);
    d->off_cell_pen = o;
    o = align16(o + 8 * (int64_t)d->PMAX * d->LC);
    d->off_node_flags = o;
    o = align16(o + (int64_t)d->NODES);
    d->off_node_pen = o;
    o = align16(o + 8 * (int64_t)d->NODES);
    d->frame_bytes = o;
    d->off_q_hdr = 0;
    d->off_q_path = align16(sizeof(va_query_hdr));
    d->query_bytes = align16(d->off_q_path + 2 * (int64_t)d->NODES);
    return true;
}

// ---------------------------------------------------------------------------------------------
// workspace: [B frame records][B*MAXPK query records][starts int32[B*MAXPK]][ends][ctrl int32[16]]
struct Work {
    uint8_t* frames;
    uint8_t* queries;
    int32_t* starts;
    int32_t* ends;
    int32_t* ctrl;  // [0] rerun slot (-1 = none)
};

int64_t work_bytes(const Dims& d, int B, Work* w, uint8_t* base) {
    int64_t nslots = (int64_t)B * d.MAXPK;
    int64_t o = 0;
    int64_t off_frames = o;
    o = align16(o + (int64_t)B * d.frame_bytes);
    int64_t off_q = o;
    o = align16(o + nslots * d.query_bytes);
    int64_t off_s = o;
    o = align16(o + 4 * nslots);
    int64_t off_e = o;
    o = align16(o + 4 * nslots);
    int64_t off_c = o;
    o = align16(o + 64);
    if (w && base) {
        w->frames = base + off_frames;
        w->queries = base + off_q;
        w->starts = (int32_t*)(base + off_s);
        w->ends = (int32_t*)(base + off_e);
        w->ctrl = (int32_t*)(base + off_c);
    }
    return o;
}

// ---------------------------------------------------------------------------------------------
// block helpers
__device__ inline unsigned long long block_min_u64(unsigned long long v, unsigned long long* scratch) {
    // 256 threads = 4 waves
    for (int o = 32; o > 0; o >>= 1) {
        unsigned long long w = __shfl_xor(v, o, 64);
        v = w < v ? w : v;
    }
    int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    __syncthreads();
    if (lane == 0) scratch[wid] = v;
    __syncthreads();
    unsigned long long r = scratch[0];
    for (int i = 1; i < (int)(blockDim.x >> 6); ++i) r = scratch[i] < r ? scratch[i] : r;
    __syncthreads();
    return r;
}

// ---------------------------------------------------------------------------------------------
__global__ void nav_sample_kernel(const uint8_t* __restrict__ masks, int64_t pitch, int B, int H, int W,
                                  uint8_t* __restrict__ cells) {
    int LR = H / VA_GRID, LC = W / VA_GRID;
    int64_t n = (int64_t)B * LR * LC;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        int64_t b = i / (LR * LC);
        int r = (int)((i / LC) % LR), c = (int)(i % LC);
        cells[i] = masks[(b * H + (int64_t)(VA_GRID * r + VA_GRID / 2)) * pitch + VA_GRID * c + VA_GRID / 2] != 0;
    }
}

// ---------------------------------------------------------------------------------------------
// nav_grid_kernel: one workgroup per frame.
struct GridArgs {
    const uint8_t* cells;
    const int32_t* rects;
    uint8_t* frames;
    int32_t* starts;
    int32_t* ends;
    uint8_t* queries;
    Dims d;
};

__global__ __launch_bounds__(VA_NAV_THREADS) void nav_grid_kernel(GridArgs a) {
    const Dims& d = a.d;
    const int f = blockIdx.x;
    const int tid = threadIdx.x, nt = blockDim.x;
    const int LR = d.LR, LC = d.LC, NART = d.NART, NOBJ = d.LR + d.NART;
    uint8_t* rec = a.frames + (int64_t)f * d.frame_bytes;
    va_frame_hdr* hdr = (va_frame_hdr*)(rec + d.off_hdr);
    int32_t* peak_x = (int32_t*)(rec + d.off_peaks);
    int32_t* peak_y = peak_x + d.MAXPK;
    int32_t* end_p = peak_y + d.MAXPK;
    int32_t* end_c = end_p + d.MAXPK;
    int16_t* g_pos_obj = (int16_t*)(rec + d.off_pos_obj);
    int16_t* g_pos_y = (int16_t*)(rec + d.off_pos_y);
    int16_t* g_pos_attr = (int16_t*)(rec + d.off_pos_attr);
    uint8_t* g_cell_flags = rec + d.off_cell_flags;
    double* g_cell_pen = (double*)(rec + d.off_cell_pen);
    uint8_t* g_node_flags = rec + d.off_node_flags;
    double* g_node_pen = (double*)(rec + d.off_node_pen);
    const uint8_t* cells = a.cells + (int64_t)f * LR * LC;

    extern __shared__ __align__(16) uint8_t smem[];
    unsigned long long* red = (unsigned long long*)smem;       // 8 words
    int* sh = (int*)(smem + 64);                                // scalars
    int16_t* pos_obj = (int16_t*)(smem + 256);                  // [PMAX]
    int16_t* obj_pos = pos_obj + d.PMAX;                        // [NOBJ]
    int16_t* er_first = obj_pos + NOBJ;                         // [PMAX]
    int16_t* er_last = er_first + d.PMAX;
    int16_t* ec_first = er_last + d.PMAX;                       // [LC]
    int16_t* ec_last = ec_first + LC;
    uint8_t* obj_flags = (uint8_t*)(ec_last + LC);              // [NOBJ][LC]
    uint8_t* node_fl = obj_flags + NOBJ * LC;                   // [LR*LC]
    uint8_t* occ = node_fl + LR * LC;                           // [LC]

    enum { S_STATUS, S_X0, S_Y0, S_C, S_RM, S_P, S_ANY, S_MINY, S_NPK };
    // slot queries of this frame: default none
    for (int k = tid; k < d.MAXPK; k += nt) {
        a.starts[f * d.MAXPK + k] = -1;
        a.ends[f * d.MAXPK + k] = -1;
        va_query_hdr* q = (va_query_hdr*)(a.queries + ((int64_t)f * d.MAXPK + k) * d.query_bytes);
        q->status = VA_QUERY_NONE;
        q->len = 0;
        q->cost = 0.0;
        q->miss[0] = q->miss[1] = 0;
        q->frame = f;
        q->k = k;
        q->expansions = 0;
        q->unique = 0;
        q->order = -1;
    }
    if (tid == 0) {
        int x = a.rects[4 * f + 0], y = a.rects[4 * f + 1], w = a.rects[4 * f + 2], h = a.rects[4 * f + 3];
        int status = VA_FRAME_OK;
        if (w <= 0 || h <= 0) status = VA_FRAME_NO_MASK;
        // a boundingRect lies in the frame (points are clipped to it): anything far outside is not a rect the
        // mask choice wrote -- rejected (no mask) before the arithmetic below could overflow
        constexpr int LIM = 1 << 24;
        if (status == VA_FRAME_OK &&
            !VA_DIAG_OK(x > -LIM && x < LIM && y > -LIM && y < LIM && w < LIM && h < LIM, 31, x, w))
            status = VA_FRAME_NO_MASK;
        // FrameProcessor.py:79-83 (only w is clamped to the frame, Q14)
        x = x - (x % VA_GRID);
        y = y - (y % VA_GRID);
        w = (w % VA_GRID != 0) ? w + (VA_GRID - w % VA_GRID) : w;
        w = w > d.W ? d.W : w;
        h = (h % VA_GRID != 0) ? h + (VA_GRID - h % VA_GRID) : h;
        // :94-97 index mask_img at every cell centre of the snapped rect: a centre past the frame (a polygon
        // clipped onto x = W0 / y = H0 by scale_coords, then rounded up to whole cells) is numpy's IndexError
        if (status == VA_FRAME_OK && (x < 0 || y < 0)) status = VA_FRAME_NO_MASK;  // (never: points are >= 0)
        if (status == VA_FRAME_OK && (x + w > d.W || y + h > d.H)) status = VA_FRAME_INDEX_ERROR;
        sh[S_STATUS] = status;
        sh[S_X0] = x;
        sh[S_Y0] = y;
        sh[S_C] = status == VA_FRAME_OK ? w / VA_GRID : 0;
        sh[S_RM] = status == VA_FRAME_OK ? h / VA_GRID : 0;
        sh[S_ANY] = 0;
        sh[S_NPK] = 0;
    }
    __syncthreads();
    const int x0 = sh[S_X0], y0 = sh[S_Y0], C = sh[S_C], Rm = sh[S_RM];
    const int xi0 = x0 / VA_GRID, yi0 = y0 / VA_GRID, ay0 = d.start_y / VA_GRID;
    // ---- main objects (FrameProcessor.py:104-124): empty = mask not set at the cell centre
    int any = 0;
    for (int i = tid; i < Rm * C; i += nt) {
        int r = i / C, c = i % C;
        bool in = cells[(yi0 + r) * LC + xi0 + c] != 0;
        obj_flags[r * LC + c] = in ? 0 : VA_CELL_EMPTY;
        any |= in;
    }
    if (any) atomicOr(&sh[S_ANY], 1);
    __syncthreads();
    if (tid == 0 && sh[S_STATUS] == VA_FRAME_OK) {
        if (!sh[S_ANY]) {
            sh[S_STATUS] = VA_FRAME_EMPTY;  // :99-101
        } else {
            // artificial-row list emulation (:130-165), python list semantics
            int P = Rm;
            for (int p = 0; p < Rm; ++p) pos_obj[p] = (int16_t)p;
            for (int aa = 0; aa < NART; ++aa) {
                int ri = (ay0 + aa) - yi0;  // (i - y) // grid_size, exact
                if (ri < P - 1) {
                    if (ri < -P) {
                        sh[S_STATUS] = VA_FRAME_INDEX_ERROR;
                        break;
                    }
                    pos_obj[ri >= 0 ? ri : P + ri] = (int16_t)(LR + aa);
                } else {
                    pos_obj[P++] = (int16_t)(LR + aa);
                }
            }
            sh[S_P] = P;
        }
    }
    __syncthreads();
    const int status = sh[S_STATUS];
    if (status != VA_FRAME_OK) {
        if (tid == 0) {
            hdr->status = status;
            hdr->x0 = x0;
            hdr->y0 = y0;
            hdr->C = C;
            hdr->Rm = Rm;
            hdr->P = 0;
            hdr->npeaks = 0;
            hdr->start_p = hdr->start_c = -1;
            hdr->min_y = -1;
            hdr->rounds = 0;
        }
        return;
    }
    const int P = sh[S_P];
    // ---- artificial objects (:133-160) + inverse position map
    const int art_lo = d.W / 2 - VA_GRID * 8;  // artifical_grid_column_xs (:60-65)
    for (int i = tid; i < NART * C; i += nt) {
        int aa = i / C, c = i % C;
        int yi = ay0 + aa;
        bool prev_empty = true;  // grid_lookup.get((j, i)) before this row is written: a main object or nothing
        if (yi >= yi0 && yi < yi0 + Rm) prev_empty = (obj_flags[(yi - yi0) * LC + c] & VA_CELL_EMPTY) != 0;
        int xr = x0 + VA_GRID * c - art_lo;
        bool art_col = xr >= 0 && xr < VA_GRID * 17 && xr % VA_GRID == 0;
        uint8_t fl;
        if (prev_empty)
            fl = art_col ? VA_CELL_ARTIFICIAL : VA_CELL_EMPTY;
        else
            fl = 0;
        obj_flags[(LR + aa) * LC + c] = fl;
    }
    for (int o = tid; o < NOBJ; o += nt) obj_pos[o] = -1;
    __syncthreads();
    for (int p = tid; p < P; p += nt) obj_pos[pos_obj[p]] = (int16_t)p;
    __syncthreads();
    auto obj_y = [&](int o) -> int { return o < LR ? yi0 + o : ay0 + (o - LR); };       // lattice row
    auto obj_attr = [&](int o) -> int { return o < LR ? o : (ay0 + (o - LR)) - yi0; };  // Grid.row
    // ---- lookup lattice (grid_lookup after the whole build; artificial rows written last)
    for (int i = tid; i < LR * LC; i += nt) {
        int yi = i / LC, xi = i % LC;
        int c = xi - xi0;
        int o = -1;
        if (c >= 0 && c < C) {
            if (yi >= ay0 && yi - ay0 < NART)
                o = LR + (yi - ay0);
            else if (yi >= yi0 && yi < yi0 + Rm)
                o = yi - yi0;
        }
        uint8_t fl = 0;
        if (o >= 0) {
            fl |= VA_NODE_EXISTS;
            if (!(obj_flags[o * LC + c] & VA_CELL_EMPTY)) fl |= VA_NODE_NONEMPTY;
            if (obj_flags[o * LC + c] & VA_CELL_ARTIFICIAL) fl |= VA_NODE_ARTIFICIAL;
            if (obj_pos[o] >= 0) fl |= VA_NODE_IN_GRIDS;
            // graph multiplicity: non-empty objects of self.grids at these coords (Q19)
            int m = 0;
            if (yi >= yi0 && yi < yi0 + Rm) {
                int om = yi - yi0;
                if (obj_pos[om] >= 0 && !(obj_flags[om * LC + c] & VA_CELL_EMPTY)) ++m;
            }
            if (yi >= ay0 && yi - ay0 < NART) {
                int oa = LR + (yi - ay0);
                if (obj_pos[oa] >= 0 && !(obj_flags[oa * LC + c] & VA_CELL_EMPTY)) ++m;
            }
            fl |= (uint8_t)(m << VA_NODE_MULT_SHIFT);
        }
        node_fl[i] = fl;
        g_node_flags[i] = fl;
    }
    // ---- position table + cell flags to the record
    for (int p = tid; p < d.PMAX; p += nt) {
        int o = p < P ? pos_obj[p] : -1;
        g_pos_obj[p] = (int16_t)o;
        g_pos_y[p] = (int16_t)(o >= 0 ? obj_y(o) : -1);
        g_pos_attr[p] = (int16_t)(o >= 0 ? obj_attr(o) : 0);
    }
    for (int i = tid; i < P * C; i += nt) {
        int p = i / C, c = i % C;
        g_cell_flags[p * LC + c] = obj_flags[pos_obj[p] * LC + c];
    }
    // ---- easy segments (PenaltyCalculator.py:26-55), keyed by list position
    for (int p = tid; p < P; p += nt) {
        const uint8_t* fl = obj_flags + pos_obj[p] * LC;
        int first = -1, last = -1, cnt = 0;
        for (int c = 0; c < C; ++c)
            if (!(fl[c] & VA_CELL_EMPTY)) {
                if (first < 0) first = c;
                last = c;
                ++cnt;
            }
        bool easy = cnt > 0 && last - first == cnt - 1;
        er_first[p] = (int16_t)(easy ? first : -1);
        er_last[p] = (int16_t)(easy ? last : -1);
    }
    for (int c = tid; c < C; c += nt) {
        int first = -1, last = -1, cnt = 0;
        for (int p = 0; p < P; ++p)
            if (!(obj_flags[pos_obj[p] * LC + c] & VA_CELL_EMPTY)) {
                if (first < 0) first = p;
                last = p;
                ++cnt;
            }
        bool easy = cnt > 0 && last - first == cnt - 1;
        ec_first[c] = (int16_t)(easy ? first : -1);
        ec_last[c] = (int16_t)(easy ? last : -1);
    }
    __syncthreads();
    // ---- penalties (PenaltyCalculator.py:57-142) for every non-empty object in self.grids
    auto lk_open = [&](int yi, int xi) -> bool {  // (x, y) in grid_lookup and not .empty
        if (yi < 0 || yi >= LR || xi < 0 || xi >= LC) return false;
        return (node_fl[yi * LC + xi] & (VA_NODE_EXISTS | VA_NODE_NONEMPTY)) == (VA_NODE_EXISTS | VA_NODE_NONEMPTY);
    };
    for (int i = tid; i < P * C; i += nt) {
        int p = i / C, c = i % C;
        int o = pos_obj[p];
        double pen = 0.0;
        if (!(obj_flags[o * LC + c] & VA_CELL_EMPTY)) {
            const int sx = x0 + VA_GRID * c, syy = VA_GRID * obj_y(o);
            // row
            int attr = obj_attr(o), lx, rx;
            if (attr >= 0 && attr < P && er_first[attr] >= 0) {
                lx = x0 + VA_GRID * er_first[attr];
                rx = x0 + VA_GRID * er_last[attr];
            } else {
                int yi = obj_y(o), xl = xi0 + c, xr = xi0 + c;
                while (lk_open(yi, xl - 1)) --xl;
                while (lk_open(yi, xr + 1)) ++xr;
                lx = VA_GRID * xl;
                rx = VA_GRID * xr;
            }
            int den = rx - lx;
            double ratio = den == 0 ? 0.5 : (double)(sx - lx) / (double)den;
            double rp = 2.0 * fabs(ratio - 0.5);
            // column
            int ty, by;
            if (ec_first[c] >= 0) {
                ty = VA_GRID * obj_y(pos_obj[ec_first[c]]);
                by = VA_GRID * obj_y(pos_obj[ec_last[c]]);
            } else {
                int xi = xi0 + c, yt = obj_y(o), yb = obj_y(o);
                while (lk_open(yt - 1, xi)) --yt;
                while (lk_open(yb + 1, xi)) ++yb;
                ty = VA_GRID * yt;
                by = VA_GRID * yb;
            }
            den = by - ty;
            ratio = den == 0 ? 0.5 : (double)(syy - ty) / (double)den;
            double cp = 2.0 * fabs(ratio - 0.5);
            if (rp > 0.99 || cp > 0.99) {
                pen = 1.0;
            } else {
                double total = rp + cp;
                if (total == 0.0) {
                    pen = 0.0;
                } else {
                    double dom = fabs(rp - cp) / total;
                    double rw = 0.5 + (rp > cp ? 0.25 * dom : -(0.25 * dom));
                    double cw = 1.0 - rw;
                    pen = (rp * rw) + (cp * cw);
                }
            }
        }
        g_cell_pen[p * LC + c] = pen;
    }
    __syncthreads();
    // node penalty = Grid.penalty of grid_lookup[(x, y)] (None -> 0 for empty objects and orphans)
    for (int i = tid; i < LR * LC; i += nt) {
        uint8_t fl = node_fl[i];
        double pen = 0.0;
        if ((fl & (VA_NODE_EXISTS | VA_NODE_NONEMPTY | VA_NODE_IN_GRIDS)) ==
            (VA_NODE_EXISTS | VA_NODE_NONEMPTY | VA_NODE_IN_GRIDS)) {
            int yi = i / LC, c = i % LC - xi0;
            int o = (yi >= ay0 && yi - ay0 < NART) ? LR + (yi - ay0) : yi - yi0;
            pen = g_cell_pen[obj_pos[o] * LC + c];
        }
        g_node_pen[i] = pen;
    }
    // ---- protrusion (ProtrusionDetector.py:38-99): top-most non-empty row of self.grids
    unsigned long long mn = ~0ull;
    for (int i = tid; i < P * C; i += nt) {
        int p = i / C, c = i % C;
        if (!(obj_flags[pos_obj[p] * LC + c] & VA_CELL_EMPTY)) {
            unsigned long long v = (unsigned long long)obj_y(pos_obj[p]);
            mn = v < mn ? v : mn;
        }
    }
    mn = block_min_u64(mn, red);
    const int min_yi = (int)mn;
    for (int c = tid; c < LC; c += nt) occ[c] = 0;
    __syncthreads();
    for (int i = tid; i < P * C; i += nt) {
        int p = i / C, c = i % C;
        int o = pos_obj[p];
        if (obj_y(o) == min_yi && !(obj_flags[o * LC + c] & VA_CELL_EMPTY)) occ[c] = 1;
    }
    __syncthreads();
    if (tid == 0) {
        // runs of occupied columns: pixel runs [x, min(x_last+20, W-1)] split at gaps > 5
        int npk = 0;
        int c = 0;
        while (c < C) {
            if (!occ[c]) {
                ++c;
                continue;
            }
            int ca = c;
            while (c + 1 < C && occ[c + 1]) ++c;
            int xa = x0 + VA_GRID * ca;
            int xe = x0 + VA_GRID * c + VA_GRID;
            if (xe > d.W - 1) xe = d.W - 1;
            int len = xe - xa + 1;
            if (npk < d.MAXPK) {
                peak_x[npk] = xa + len / 2;
                peak_y[npk] = VA_GRID * min_yi;
            }
            ++npk;
            ++c;
        }
        sh[S_NPK] = npk < d.MAXPK ? npk : d.MAXPK;
    }
    __syncthreads();
    const int npk = sh[S_NPK];
    // ---- start / end cells (utils.py:6-32): first minimum of the squared distance, row-major
    int sp = -1, sc = -1;
    for (int t = -1; t < npk; ++t) {
        int px = t < 0 ? d.W / 2 : peak_x[t];
        int py = t < 0 ? d.H : peak_y[t];
        unsigned long long best = ~0ull;
        for (int i = tid; i < P * C; i += nt) {
            int p = i / C, c = i % C;
            int o = pos_obj[p];
            if (obj_flags[o * LC + c] & VA_CELL_EMPTY) continue;
            long long dx = px - (x0 + VA_GRID * c + VA_GRID / 2);
            long long dy = py - (VA_GRID * obj_y(o) + VA_GRID / 2);
            unsigned long long key = ((unsigned long long)(dx * dx + dy * dy) << 24) | (unsigned long long)i;
            best = key < best ? key : best;
        }
        best = block_min_u64(best, red);
        int i = (int)(best & 0xFFFFFF);
        if (t < 0) {
            sp = i / C;
            sc = i % C;
        } else if (tid == 0) {
            end_p[t] = i / C;
            end_c[t] = i % C;
            int so = pos_obj[sp], eo = pos_obj[i / C];
            a.starts[f * d.MAXPK + t] = obj_y(so) * LC + xi0 + sc;
            a.ends[f * d.MAXPK + t] = obj_y(eo) * LC + xi0 + (i % C);
        }
    }
    if (tid == 0) {
        hdr->status = VA_FRAME_OK;
        hdr->x0 = x0;
        hdr->y0 = y0;
        hdr->C = C;
        hdr->Rm = Rm;
        hdr->P = P;
        hdr->npeaks = npk;
        hdr->start_p = sp;
        hdr->start_c = sc;
        hdr->min_y = VA_GRID * min_yi;
        hdr->rounds = 0;
    }
}

// ---------------------------------------------------------------------------------------------
// A*: one wave64 per query.  LDS: the angle tables (1.1 KiB), then per node g f64 | parent u16 | hist u16 |
// state u8, and per open-list slot its node u16, push-time f (key bits, u64) and (x, y) tie key u32: 27 B per
// node, 28.7 KiB at 640x640.  The node penalties stay in global memory (8 KiB per frame, L1/L2-resident; a
// query wave sharing a CU with two conv2 workgroups must fit beside them): a pop issues the four neighbours'
// penalty loads first, so their latency runs under the pop's LDS work.  One wave per workgroup: no block
// barrier is needed between the lanes' LDS accesses (a wave's LDS operations complete in order), only a
// compiler-level ordering point (WAVE_SYNC).
constexpr int ASTAR_TABLES = 128 * 8 + 64 + 32;  // angle penalties f64, prev / next index tables
#define ST_EXISTS 1u
#define ST_MULT_SHIFT 1  // bits 1-2
#define ST_HASG 8u
#define ST_INOPEN 16u
#define ST_CLOSED 32u
#define HD_DEPTH_SHIFT 12  // hist: 6 moves x 2 bits in bits 0-11, saturated depth (0..7) in bits 12-14

struct AstarArgs {
    const uint8_t* node_flags;  // base; query slot q uses base + (q / qpf) * node_stride
    const double* node_pen;     // same indexing (stride in bytes)
    int64_t node_stride;
    int qpf;
    const int32_t* starts;
    const int32_t* ends;
    uint8_t* qwork;
    int64_t query_bytes, off_q_path;
    int LR, LC, nslots;
    int slot0;                  // first slot to (re)run
    const uint64_t* seen;       // base seen set of this round
};

#define WAVE_SYNC()                                            \
    do {                                                       \
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); \
        __builtin_amdgcn_wave_barrier();                       \
    } while (0)

extern "C" __device__ __attribute__((const)) unsigned long long __ockl_wfred_min_u64(unsigned long long);
extern "C" __device__ __attribute__((const)) unsigned int __ockl_wfred_min_u32(unsigned int);

// lexicographic (fb, sec) minimum over the wave: two DPP-based wave reductions (ockl) instead of a
// 6-step xor-shuffle butterfly of three ds_bpermute each
__device__ inline void wave_argmin(unsigned long long& fb, unsigned& sec) {
    const unsigned long long m = __ockl_wfred_min_u64(fb);
    const unsigned s2 = __ockl_wfred_min_u32(fb == m ? sec : ~0u);
    fb = m;
    sec = s2;
}

__global__ __launch_bounds__(64) void nav_astar_kernel(AstarArgs a) {
    const int q = blockIdx.x;
    const int lane = threadIdx.x;
    if (q < a.slot0 || q >= a.nslots) return;
    const int s = a.starts[q], e = a.ends[q];
    va_query_hdr* qh = (va_query_hdr*)(a.qwork + (int64_t)q * a.query_bytes);
    if (s < 0 || e < 0) return;  // empty slot (status already VA_QUERY_NONE)
    const int LC = a.LC, N = a.LR * a.LC;
    if (!VA_DIAG_OK(s < N && e < N, 32, s, e)) return;  // never written by the grid kernel: rejected
    const int fr = q / a.qpf;
    const uint8_t* nflags = (const uint8_t*)((const uint8_t*)a.node_flags + (int64_t)fr * a.node_stride);
    const double* npen = (const double*)((const uint8_t*)a.node_pen + (int64_t)fr * a.node_stride);

    extern __shared__ __align__(16) uint8_t smem[];
    double* apen = (double*)smem;                 // [128] angle penalties
    int8_t* pidx = (int8_t*)(apen + 128);         // [49] (+ pad)
    int8_t* nidx = pidx + 64;                     // [25] (+ pad)
    double* g = (double*)(smem + ASTAR_TABLES);
    unsigned long long* okey = (unsigned long long*)(g + N);  // per open slot: push-time f bits
    uint32_t* osec = (uint32_t*)(okey + N);       // per open slot: x << 24 | y << 16
    uint16_t* par = (uint16_t*)(osec + N);
    uint16_t* hd = par + N;
    uint16_t* open = hd + N;                      // (unused slot array: the popped node comes from osec)
    uint8_t* st = (uint8_t*)(open + N);
    const double* __restrict__ pen = npen;  // global (see above)

    for (int i = lane; i < 128; i += 64) apen[i] = c_angle_pen[i];
    if (lane < 49) pidx[lane] = c_prev_idx[lane];
    if (lane < 25) nidx[lane] = c_next_idx[lane];
    for (int i = lane; i < N; i += 64) {
        uint8_t fl = nflags[i];
        uint8_t v = 0;
        if (fl & VA_NODE_EXISTS) v |= ST_EXISTS;
        v |= (uint8_t)(((fl >> VA_NODE_MULT_SHIFT) & 3u) << ST_MULT_SHIFT);
        st[i] = v;
    }
    unsigned long long seen0 = a.seen[0], seen1 = a.seen[1];
    unsigned long long miss0 = 0, miss1 = 0;
    const int ex = e % LC, ey = e / LC;
    WAVE_SYNC();
    if (lane == 0) {
        g[s] = 0.0;
        int sx = s % LC, sy = s / LC;
        hd[s] = 0;
        st[s] |= ST_HASG | ST_INOPEN;
        okey[0] = (unsigned long long)__double_as_longlong((double)(VA_GRID * (abs(sx - ex) + abs(sy - ey))));
        osec[0] = ((unsigned)sx << 24) | ((unsigned)sy << 16);
    }
    int open_n = 1;
    int found = 0, expansions = 0;
    WAVE_SYNC();
    // neighbour order of FrameProcessor.py:195-200: right, left, down, up
    const int ndx = lane == 0 ? 1 : lane == 1 ? -1 : 0;
    const int ndy = lane == 2 ? 1 : lane == 3 ? -1 : 0;
    while (open_n > 0) {
        // ---- pop argmin (push-time f, x, y)
        unsigned long long fb = ~0ull;
        unsigned sec = ~0u;
        for (int i = lane; i < open_n; i += 64) {
            const unsigned long long kb = okey[i];
            const unsigned ks = osec[i] | (unsigned)i;
            if (kb < fb || (kb == fb && ks < sec)) {
                fb = kb;
                sec = ks;
            }
        }
        wave_argmin(fb, sec);
        // the popped node straight from its key (osec holds x << 24 | y << 16): no dependent read of open[]
        const int slot = (int)(sec & 0xFFFFu);
        const int cx = (int)(sec >> 24), cy = (int)((sec >> 16) & 0xFFu);
        const int cur = cy * LC + cx;
        // the popped key must name a live open slot and a lattice node (it indexes the global penalties below):
        // anything else is open-list state no push wrote -- recorded and the query ends (wave-uniform values)
        if (!VA_DIAG_OK(slot < open_n && cx < LC && cy < a.LR, 33, cur, open_n)) break;
        // the neighbours (lanes 0..3) and their penalties, loaded now and consumed by the relaxation
        int nb = -1;
        if (lane < 4) {
            const int nx = cx + ndx, ny = cy + ndy;
            if (nx >= 0 && nx < LC && ny >= 0 && ny < a.LR) nb = ny * LC + nx;
        }
        const double pnb = pen[nb >= 0 ? nb : cur];  // unconditional: the wait lands at the use
        const uint8_t snb = st[nb >= 0 ? nb : cur];   // with it: closing cur below never touches a neighbour
        WAVE_SYNC();
        if (lane == 0) {
            const int last = open_n - 1;
            okey[slot] = okey[last];
            osec[slot] = osec[last];
        }
        --open_n;
        ++expansions;
        if (cur == e) {
            found = 1;
            break;
        }
        const double gcur = g[cur];
        const unsigned hcur = hd[cur];
        const unsigned mult = (st[cur] >> ST_MULT_SHIFT) & 3u;
        WAVE_SYNC();
        if (lane == 0) st[cur] |= ST_CLOSED;
        WAVE_SYNC();
        const bool valid = nb >= 0 && (snb & ST_EXISTS) && !(snb & ST_CLOSED);
        unsigned long long vb = __ballot(valid);
        // angle penalty of the first non-closed neighbour (newest-window rule, Q3)
        double ap = 0.0;
        const unsigned depth = hcur >> HD_DEPTH_SHIFT;
        if (mult > 0 && vb != 0 && depth >= 6) {
            // moves m_d .. m_{d-5} in bits [1:0] .. [11:10]
            auto mvx = [](int m) { return m == 0 ? 1 : m == 1 ? -1 : 0; };
            auto mvy = [](int m) { return m == 2 ? 1 : m == 3 ? -1 : 0; };
            int m0 = hcur & 3, m1 = (hcur >> 2) & 3, m3 = (hcur >> 6) & 3, m4 = (hcur >> 8) & 3,
                m5 = (hcur >> 10) & 3;
            int nxv = mvx(m0) + mvx(m1), nyv = mvy(m0) + mvy(m1);
            int pxv = mvx(m3) + mvx(m4) + mvx(m5), pyv = mvy(m3) + mvy(m4) + mvy(m5);
            int pi = pidx[(pxv + 3) * 7 + (pyv + 3)];
            int ni = nidx[(nxv + 2) * 5 + (nyv + 2)];
            if (pi >= 0 && ni >= 0) {
                int key = pi * 8 + ni;
                unsigned long long bit = 1ull << (key & 63);
                bool hit = key < 64 ? (seen0 & bit) : (seen1 & bit);
                if (!hit) {
                    ap = apen[key];
                    if (key < 64) {
                        seen0 |= bit;
                        miss0 |= bit;
                    } else {
                        seen1 |= bit;
                        miss1 |= bit;
                    }
                }
            }
        }
        const int first = vb ? __ffsll((long long)vb) - 1 : -1;
        for (unsigned pass = 0; pass < mult; ++pass) {
            bool push = false;
            double t = 0.0, fnew = 0.0;
            unsigned secn = 0;
            if (valid) {
                double apj = (pass == 0 && lane == first) ? ap : 0.0;
                double pm = (1.0 + (0.5 * pnb)) + (apj * 1.5);
                t = gcur + (20.0 * pm);
                uint8_t sv = st[nb];
                if (!(sv & ST_HASG) || t < g[nb]) {
                    g[nb] = t;
                    par[nb] = (uint16_t)cur;
                    unsigned dnew = depth < 7 ? depth + 1 : 7;
                    hd[nb] = (uint16_t)((dnew << HD_DEPTH_SHIFT) | (((hcur << 2) | (unsigned)lane) & 0xFFFu));
                    if (!(sv & ST_INOPEN)) {
                        push = true;
                        const int nx = nb % LC, ny = nb / LC;
                        fnew = t + (double)(VA_GRID * (abs(nx - ex) + abs(ny - ey)));
                        secn = ((unsigned)nx << 24) | ((unsigned)ny << 16);
                        st[nb] = sv | ST_HASG | ST_INOPEN;
                    } else {
                        st[nb] = sv | ST_HASG;
                    }
                }
            }
            unsigned long long pb = __ballot(push);
            if (push) {
                const int pos = open_n + __popcll(pb & ((1ull << lane) - 1ull));
                okey[pos] = (unsigned long long)__double_as_longlong(fnew);
                osec[pos] = secn;
            }
            open_n += __popcll(pb);
            WAVE_SYNC();
        }
    }
    // ---- result
    if (lane == 0) {
        qh->expansions = expansions;
        qh->miss[0] = miss0;
        qh->miss[1] = miss1;
        qh->unique = 0;
        qh->order = -1;
        int len = 1;
        if (found) {  // the parent chain from e must reach s within the lattice (the record holds N nodes)
            int c = e;
            while (c != s && len <= N) {
                c = par[c];
                ++len;
                if (c >= N) len = N + 1;
            }
            found = VA_DIAG_OK(len <= N, 34, q, len);
        }
        if (found) {
            uint16_t* path = (uint16_t*)((uint8_t*)qh + a.off_q_path);
            int c = e;
            for (int i = len - 1; i >= 0; --i) {
                path[i] = (uint16_t)c;
                if (i) c = par[c];
            }
            qh->status = VA_QUERY_FOUND;
            qh->len = len;
            qh->cost = g[e];
        } else {
            qh->status = VA_QUERY_NO_PATH;
            qh->len = 0;
            qh->cost = __builtin_inf();
        }
    }
}

// validation of one speculative round (see file header): the first slot q >= slot0 whose
// newly-missed keys intersect base | (misses of the slots before it).  One 1024-thread workgroup:
// chunked exclusive OR-scan of the 128-bit miss masks in slot order.
constexpr int VAL_THREADS = 1024;

__global__ __launch_bounds__(VAL_THREADS) void nav_validate_kernel(const int32_t* starts, const uint8_t* qwork,
                                                                   int64_t query_bytes, int nslots, int slot0,
                                                                   uint64_t* seen, int32_t* ctrl) {
    __shared__ unsigned long long s0[VAL_THREADS], s1[VAL_THREADS];
    __shared__ int first;
    __shared__ unsigned long long acc0, acc1;
    const int tid = threadIdx.x;
    if (tid == 0) {
        first = INT32_MAX;
        acc0 = seen[0];
        acc1 = seen[1];
    }
    __syncthreads();
    for (int base = slot0; base < nslots; base += VAL_THREADS) {
        const int q = base + tid;
        unsigned long long m0 = 0, m1 = 0;
        if (q < nslots && starts[q] >= 0) {
            const va_query_hdr* qh = (const va_query_hdr*)(qwork + (int64_t)q * query_bytes);
            m0 = qh->miss[0];
            m1 = qh->miss[1];
        }
        s0[tid] = m0;
        s1[tid] = m1;
        __syncthreads();
        for (int off = 1; off < VAL_THREADS; off <<= 1) {  // inclusive OR-scan (Hillis-Steele)
            unsigned long long a0 = tid >= off ? s0[tid - off] : 0, a1 = tid >= off ? s1[tid - off] : 0;
            __syncthreads();
            s0[tid] |= a0;
            s1[tid] |= a1;
            __syncthreads();
        }
        unsigned long long p0 = acc0 | (tid ? s0[tid - 1] : 0), p1 = acc1 | (tid ? s1[tid - 1] : 0);
        if (((m0 & p0) | (m1 & p1)) != 0) atomicMin(&first, q);
        __syncthreads();
        if (first != INT32_MAX) {
            // seen = base | misses of the slots before the first conflict
            const int fq = first - base;
            if (tid == 0) {
                seen[0] = acc0 | (fq ? s0[fq - 1] : 0);
                seen[1] = acc1 | (fq ? s1[fq - 1] : 0);
                ctrl[0] = first;
            }
            return;
        }
        if (tid == 0) {
            acc0 |= s0[VAL_THREADS - 1];
            acc1 |= s1[VAL_THREADS - 1];
        }
        __syncthreads();
    }
    if (tid == 0) {
        seen[0] = acc0;
        seen[1] = acc1;
        ctrl[0] = -1;
    }
}

// Jaccard / subset filter of FrameProcessor._find_paths (:255-269), one wave per frame.
__global__ __launch_bounds__(64) void nav_dedupe_kernel(uint8_t* qwork, int64_t query_bytes, int64_t off_q_path,
                                                        int qpf, int nodes) {
    const int f = blockIdx.x, lane = threadIdx.x;
    const int words = (nodes + 63) / 64;
    extern __shared__ __align__(16) uint8_t smem[];
    unsigned long long* bits = (unsigned long long*)smem;  // [qpf][words]
    int* order = (int*)(bits + (int64_t)qpf * words);      // [qpf] query k by rank
    int* keep = order + qpf;
    auto qhdr = [&](int k) { return (va_query_hdr*)(qwork + ((int64_t)f * qpf + k) * query_bytes); };
    for (int i = lane; i < qpf * words; i += 64) bits[i] = 0;
    __syncthreads();
    for (int k = 0; k < qpf; ++k) {
        va_query_hdr* qh = qhdr(k);
        if (qh->status != VA_QUERY_FOUND) continue;
        const uint16_t* path = (const uint16_t*)((uint8_t*)qh + off_q_path);
        const int len = VA_DIAG_OK(qh->len > 0 && qh->len <= nodes, 35, k, qh->len) ? qh->len : 0;
        for (int i = lane; i < len; i += 64) {
            int nd = path[i];
            if (VA_DIAG_OK(nd < nodes, 36, k, nd)) atomicOr(&bits[(int64_t)k * words + nd / 64], 1ull << (nd % 64));
        }
    }
    __syncthreads();
    if (lane == 0) {
        // stable sort by length, descending (list.sort(key=len, reverse=True) keeps equal keys in order)
        int n = 0;
        for (int k = 0; k < qpf; ++k) {
            va_query_hdr* qh = qhdr(k);
            if (qh->status != VA_QUERY_FOUND) continue;
            int pos = n;
            while (pos > 0 && qhdr(order[pos - 1])->len < qh->len) {
                order[pos] = order[pos - 1];
                --pos;
            }
            order[pos] = k;
            ++n;
        }
        int nkeep = 0;
        for (int r = 0; r < n; ++r) {
            int k = order[r];
            int la = qhdr(k)->len;
            bool unique = true;
            for (int u = 0; u < nkeep && unique; ++u) {
                int j = keep[u];
                int lb = qhdr(j)->len;
                int inter = 0;
                for (int w = 0; w < words; ++w)
                    inter += __popcll(bits[(int64_t)k * words + w] & bits[(int64_t)j * words + w]);
                double sim;
                if (inter == la || inter == lb)
                    sim = 1.0;
                else
                    sim = (double)inter / (double)(la + lb - inter);
                if (sim >= 0.90) unique = false;
            }
            qhdr(k)->unique = unique ? 1 : 0;
            qhdr(k)->order = unique ? nkeep : -1;
            if (unique) keep[nkeep++] = k;
        }
    }
}

// ---------------------------------------------------------------------------------------------
DevFlag g_tables_ready;  // the __constant__ tables live in each device's copy of the module

hipError_t ensure_tables() {
    if (g_tables_ready()) return hipSuccess;
    int8_t prev_idx[49], next_idx[25];
    memset(prev_idx, -1, sizeof prev_idx);
    memset(next_idx, -1, sizeof next_idx);
    for (int i = 0; i < 16; ++i) prev_idx[(VA_PREV_VEC[i][0] + 3) * 7 + (VA_PREV_VEC[i][1] + 3)] = (int8_t)i;
    for (int i = 0; i < 8; ++i) next_idx[(VA_NEXT_VEC[i][0] + 2) * 5 + (VA_NEXT_VEC[i][1] + 2)] = (int8_t)i;
    hipError_t e;
    if ((e = hipMemcpyToSymbol(HIP_SYMBOL(c_angle_pen), VA_ANGLE_PEN, sizeof VA_ANGLE_PEN)) != hipSuccess) return e;
    if ((e = hipMemcpyToSymbol(HIP_SYMBOL(c_prev_idx), prev_idx, sizeof prev_idx)) != hipSuccess) return e;
    if ((e = hipMemcpyToSymbol(HIP_SYMBOL(c_next_idx), next_idx, sizeof next_idx)) != hipSuccess) return e;
    g_tables_ready() = true;
    return hipSuccess;
}

// pinned verdict word of (current device, stream); allocated once, kept for the process
volatile int32_t* verdict_word(hipStream_t st) {
    static std::mutex mu;
    static std::map<std::pair<int, hipStream_t>, int32_t*> words;
    std::lock_guard<std::mutex> lock(mu);
    int32_t*& w = words[{va_cur_dev(), st}];
    if (!w && hipHostMalloc((void**)&w, 64, hipHostMallocDefault) != hipSuccess) {
        w = nullptr;
        return nullptr;
    }
    return w;
}

size_t astar_lds(int nodes) { return ASTAR_TABLES + (size_t)nodes * (8 + 8 + 4 + 2 + 2 + 2 + 1) + 16; }

// the Jaccard / subset filter of a va_nav_run batch (nav_dedupe_kernel's launch)
struct DedupeLaunch {
    uint8_t* queries;
    int64_t query_bytes, off_q_path;
    int B, qpf, nodes;
    size_t lds;
};

// the records of a va_nav_run copied to the caller's host memory (va_nav_run_rb)
struct ReadBack {
    void* dst;
    const void* src;
    int64_t bytes;
};

// speculative rounds over `nslots` query slots.  With `dd` the dedupe kernel is enqueued behind every round's
// validation, before the host waits for the round's verdict: a round that is final (the common case) then needs no
// launch after the wait; a round that is re-run gets its dedupe again behind the next one (the filter reads the
// query records afresh and rewrites every unique / order field, so only the last round's counts).  With `rb` the
// records are copied to the host behind every round's kernels and ahead of its verdict copy, so the verdict wait
// also covers them: a final round (the common case) returns with the records on the host; a re-run round copies
// them again
int astar_rounds(hipStream_t st, AstarArgs a, int32_t* ctrl, uint64_t* seen, int32_t* rounds_out,
                 const DedupeLaunch* dd = nullptr, const ReadBack* rb = nullptr) {
    size_t lds = astar_lds(a.LR * a.LC);
    if (lds > 65536 &&
        hipFuncSetAttribute((const void*)nav_astar_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) !=
            hipSuccess)
        return VA_ERR_HIP;
    // the round's verdict is read through a pinned host word, copied on the launch stream behind the validation
    // kernel and waited for on that stream -- never a pageable copy, whose staging the runtime orders on its own.
    // One word per (device, stream), handed out under a mutex: two host threads running va_nav_run on different
    // streams never share one (a shared word let one caller's verdict end another's rounds early)
    volatile int32_t* rerun_h = verdict_word(st);
    if (!rerun_h) return VA_ERR_HIP;
    int slot0 = 0, rounds = 0;
    while (true) {
        ++rounds;
        a.slot0 = slot0;
        a.seen = seen;
        hipLaunchKernelGGL(nav_astar_kernel, dim3(a.nslots), dim3(64), lds, st, a);
        if (hipGetLastError() != hipSuccess) return VA_ERR_HIP;
        hipLaunchKernelGGL(nav_validate_kernel, dim3(1), dim3(VAL_THREADS), 0, st, a.starts, a.qwork, a.query_bytes,
                           a.nslots, slot0, seen, ctrl);
        if (hipGetLastError() != hipSuccess) return VA_ERR_HIP;
        if (dd) {
            hipLaunchKernelGGL(nav_dedupe_kernel, dim3(dd->B), dim3(64), dd->lds, st, dd->queries, dd->query_bytes,
                               dd->off_q_path, dd->qpf, dd->nodes);
            if (hipGetLastError() != hipSuccess) return VA_ERR_HIP;
        }
        if (rb && hipMemcpyAsync(rb->dst, rb->src, (size_t)rb->bytes, hipMemcpyDeviceToHost, st) != hipSuccess)
            return VA_ERR_HIP;
        *rerun_h = -2;
        if (hipMemcpyAsync((void*)rerun_h, ctrl, sizeof(int32_t), hipMemcpyDeviceToHost, st) != hipSuccess)
            return VA_ERR_HIP;
        if (hipStreamSynchronize(st) != hipSuccess) return VA_ERR_HIP;
        const int32_t rerun = *rerun_h;
        if (rerun == -1) break;
        // the first conflicting slot lies after this round's first slot; anything else (or the -2 the copy
        // should have overwritten) means the copy did not see the validation's result: refuse, never launch on it
        if (rerun <= slot0 || rerun >= a.nslots) return VA_ERR_RANGE;
        if (rounds > 130) return VA_ERR_RANGE;  // impossible: every round adds a key (<= 128)
        slot0 = rerun;
    }
    if (rounds_out) *rounds_out = rounds;
    return VA_OK;
}

void fill_dims(const Dims& d, va_nav_dims* o) {
    o->H = d.H;
    o->W = d.W;
    o->LR = d.LR;
    o->LC = d.LC;
    o->start_y = d.start_y;
    o->NART = d.NART;
    o->PMAX = d.PMAX;
    o->MAXPK = d.MAXPK;
    o->NODES = d.NODES;
    o->pad = 0;
    o->frame_bytes = d.frame_bytes;
    o->off_hdr = d.off_hdr;
    o->off_peaks = d.off_peaks;
    o->off_pos_obj = d.off_pos_obj;
    o->off_pos_y = d.off_pos_y;
    o->off_pos_attr = d.off_pos_attr;
    o->off_cell_flags = d.off_cell_flags;
    o->off_cell_pen = d.off_cell_pen;
    o->off_node_flags = d.off_node_flags;
    o->off_node_pen = d.off_node_pen;
    o->query_bytes = d.query_bytes;
    o->off_q_hdr = d.off_q_hdr;
    o->off_q_path = d.off_q_path;
    o->off_queries_per_frame = d.frame_bytes;
}

size_t grid_lds(const Dims& d) {
    int NOBJ = d.LR + d.NART;
    return 256 + 2 * (size_t)(d.PMAX + NOBJ + 2 * d.PMAX + 2 * d.LC) + (size_t)NOBJ * d.LC + (size_t)d.LR * d.LC +
           d.LC + 64;
}

}  // namespace

// =============================================================================================== C ABI
extern "C" {

int va_nav_dims_for(int32_t H, int32_t W, va_nav_dims* out) {
    Dims d;
    if (!out || !make_dims(H, W, &d)) return VA_ERR_ARG;
    fill_dims(d, out);
    return VA_OK;
}

int64_t va_nav_workspace_bytes(int32_t B, int32_t H, int32_t W) {
    Dims d;
    if (B <= 0 || !make_dims(H, W, &d)) return VA_ERR_ARG;
    return work_bytes(d, B, nullptr, nullptr);
}

int va_nav_sample_cells(void* stream, const uint8_t* masks, int64_t pitch, int32_t B, int32_t H, int32_t W,
                        uint8_t* cells) {
    Dims d;
    if (!masks || !cells || B <= 0 || pitch < W || !make_dims(H, W, &d)) return VA_ERR_ARG;
    int64_t n = (int64_t)B * d.LR * d.LC;
    int blocks = (int)((n + 255) / 256);
    if (blocks > 65535) blocks = 65535;
    hipLaunchKernelGGL(nav_sample_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, masks, pitch, B, H, W,
                       cells);
    return hipGetLastError() == hipSuccess ? VA_OK : VA_ERR_HIP;
}

int64_t va_nav_records_bytes(int32_t B, int32_t H, int32_t W) {
    Dims d;
    if (B <= 0 || !make_dims(H, W, &d)) return VA_ERR_ARG;
    return align16(align16((int64_t)B * d.frame_bytes) + (int64_t)B * d.MAXPK * d.query_bytes);
}

int va_nav_run(void* stream, const uint8_t* cells, const int32_t* rects, int32_t B, int32_t H, int32_t W,
               uint64_t* seen, void* work, int32_t* rounds) {
    return va_nav_run_rb(stream, cells, rects, B, H, W, seen, work, rounds, nullptr, 0);
}

int va_nav_run_rb(void* stream, const uint8_t* cells, const int32_t* rects, int32_t B, int32_t H, int32_t W,
                  uint64_t* seen, void* work, int32_t* rounds, void* host_records, int64_t host_bytes) {
    Dims d;
    if (!cells || !rects || !seen || !work || B <= 0 || !make_dims(H, W, &d)) return VA_ERR_ARG;
    const int64_t rec_bytes = va_nav_records_bytes(B, H, W);
    if (host_records && host_bytes < rec_bytes) return VA_ERR_ARG;
    if (ensure_tables() != hipSuccess) return VA_ERR_HIP;
    hipStream_t st = (hipStream_t)stream;
    Work w;
    work_bytes(d, B, &w, (uint8_t*)work);
    GridArgs ga{cells, rects, w.frames, w.starts, w.ends, w.queries, d};
    hipLaunchKernelGGL(nav_grid_kernel, dim3(B), dim3(VA_NAV_THREADS), grid_lds(d), st, ga);
    if (hipGetLastError() != hipSuccess) return VA_ERR_HIP;
    AstarArgs aa{};
    aa.node_flags = (const uint8_t*)(w.frames + d.off_node_flags);
    aa.node_pen = (const double*)(w.frames + d.off_node_pen);
    aa.node_stride = d.frame_bytes;
    aa.qpf = d.MAXPK;
    aa.starts = w.starts;
    aa.ends = w.ends;
    aa.qwork = w.queries;
    aa.query_bytes = d.query_bytes;
    aa.off_q_path = d.off_q_path;
    aa.LR = d.LR;
    aa.LC = d.LC;
    aa.nslots = B * d.MAXPK;
    const int words = (d.NODES + 63) / 64;
    const DedupeLaunch dd{w.queries, d.query_bytes, d.off_q_path, B, d.MAXPK, d.NODES,
                          (size_t)d.MAXPK * words * 8 + 8 * (size_t)d.MAXPK + 16};
    int32_t r = 0;
    const ReadBack rb{host_records, work, rec_bytes};
    int rc = astar_rounds(st, aa, w.ctrl, seen, &r, &dd, host_records ? &rb : nullptr);
    if (rc != VA_OK) return rc;
    if (rounds) *rounds = r;
    return VA_OK;
}

int64_t va_nav_query_bytes(int32_t nodes) {
    if (nodes <= 0 || nodes > VA_MAX_LAT * VA_MAX_LAT) return VA_ERR_ARG;
    return align16(align16(sizeof(va_query_hdr)) + 2 * (int64_t)nodes);
}

int64_t va_astar_workspace_bytes(int32_t Q, int32_t nodes) {
    int64_t qb = va_nav_query_bytes(nodes);
    if (qb < 0 || Q <= 0) return VA_ERR_ARG;
    return align16((int64_t)Q * qb) + 64;
}

int va_astar_run(void* stream, const uint8_t* node_flags, const double* node_pen, int32_t LR, int32_t LC,
                 const int32_t* starts, const int32_t* ends, int32_t Q, uint64_t* seen, void* qwork,
                 int32_t* rounds) {
    if (!node_flags || !node_pen || !starts || !ends || !seen || !qwork || Q <= 0 || LR <= 0 || LC <= 0 ||
        LR > VA_MAX_LAT || LC > VA_MAX_LAT)
        return VA_ERR_ARG;
    if (ensure_tables() != hipSuccess) return VA_ERR_HIP;
    hipStream_t st = (hipStream_t)stream;
    int64_t qb = va_nav_query_bytes(LR * LC);
    uint8_t* base = (uint8_t*)qwork;
    int32_t* ctrl = (int32_t*)(base + align16((int64_t)Q * qb));
    // clear the records (a slot with start < 0 keeps VA_QUERY_NONE)
    if (hipMemsetAsync(base, 0, (size_t)Q * qb, st) != hipSuccess) return VA_ERR_HIP;
    AstarArgs aa{};
    aa.node_flags = node_flags;
    aa.node_pen = node_pen;
    aa.node_stride = 0;
    aa.qpf = Q;
    aa.starts = starts;
    aa.ends = ends;
    aa.qwork = base;
    aa.query_bytes = qb;
    aa.off_q_path = align16(sizeof(va_query_hdr));
    aa.LR = LR;
    aa.LC = LC;
    aa.nslots = Q;
    return astar_rounds(st, aa, ctrl, seen, rounds);
}

int va_abi_struct_sizes(int64_t* out, int32_t n) {
    const int64_t sz[] = {(int64_t)sizeof(va_nav_dims), (int64_t)sizeof(va_frame_hdr), (int64_t)sizeof(va_query_hdr),
                          (int64_t)sizeof(va_conv_args), (int64_t)sizeof(va_seg_op),    (int64_t)sizeof(va_cand),
                          (int64_t)sizeof(va_det),       (int64_t)sizeof(va_mask_stat), (int64_t)sizeof(va_post_args),
                          (int64_t)sizeof(va_contour_stat), (int64_t)sizeof(va_mask_select_args)};
    int k = (int)(sizeof sz / sizeof sz[0]);
    if (!out) return k;
    for (int i = 0; i < n && i < k; ++i) out[i] = sz[i];
    return k < n ? k : n;
}

const char* va_version(void) { return "libva355 0.4 gfx950 abi 4 (" __DATE__ ")"; }

}  // extern "C"

int va_diag_nav(unsigned int* out4, int clear) { return diag_read_tu(out4, clear); }

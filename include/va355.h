/*
 * va355.h -- C ABI of libva355.so, the MI355X (gfx950) implementation of
 * vision-assist's per-frame hot path:
 *
 *     frame -> YOLOv8-seg -> mask -> grid (+penalties) -> protrusions -> A*
 *
 * Every entry point is extern "C", takes plain pointers and sizes (device
 * pointers for bulk data, a hipStream_t passed as void*), allocates nothing,
 * and returns an int status (VA_OK = 0, < 0 = error).  No C++ exception crosses
 * this boundary.  All device buffers are caller-owned (PyTorch tensors in the
 * Python host layer, see INTEGRATION.md for ctypes / cffi bindings).
 *
 * Reference interfaces each group replaces (paths under the reference repo):
 *   va_nav_*   FrameProcessor._extract_grid_information     FrameProcessor.py:50-171
 *              FrameProcessor._calculate_penalties          FrameProcessor.py:173-182
 *                + PenaltyCalculator.calculate_penalty      PenaltyCalculator.py:26-142
 *              FrameProcessor._create_graph                 FrameProcessor.py:184-207
 *              ProtrusionDetector.__call__                  ProtrusionDetector.py:419-535
 *              FrameProcessor._find_paths                   FrameProcessor.py:230-271
 *                + utils.get_closest_grid_to_point          utils.py:6-32
 *                + PathFinder.find_path                     PathFinder.py:119-186
 *   va_seg_*   YOLO.predict (Ultralytics, external) as called at FrameProcessor.py:322:
 *              letterbox/normalise, YOLOv8-seg forward, NMS, process_mask,
 *              masks.xy -> largest mask -> fillPoly          FrameProcessor.py:67-86
 */
#ifndef VA355_H
#define VA355_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------------------------------------------------------- status */
#define VA_OK 0
#define VA_ERR_ARG (-1)       /* bad argument (shape not a multiple of 20, null ptr, ...) */
#define VA_ERR_HIP (-2)       /* a HIP runtime call failed */
#define VA_ERR_RANGE (-3)     /* input outside the compiled limits */

/* per-frame nav status (va_frame_hdr.status) */
#define VA_FRAME_OK 0
#define VA_FRAME_EMPTY 1      /* no cell centre inside the mask: FrameProcessor.py:99-101 -> __call__ returns [] */
#define VA_FRAME_INDEX_ERROR 2 /* the reference raises IndexError */
#define VA_FRAME_NO_MASK 3    /* no mask at all (no detection): FrameProcessor.py:68-69 */

/* per-query status (va_query_hdr.status) */
#define VA_QUERY_NONE 0       /* no query in this slot */
#define VA_QUERY_FOUND 1
#define VA_QUERY_NO_PATH 2    /* find_path returned ([], inf): "No path found." FrameProcessor.py:252-253 */

#define VA_GRID 20            /* config.py:1 grid_size */

/* ---------------------------------------------------------------- nav layout */
/* Geometry of one frame size.  "lattice" = the H/20 x W/20 cell lattice on
 * which every grid coordinate of the reference lies (x, y multiples of 20).
 * A lattice node index is yi * LC + xi. */
typedef struct va_nav_dims {
    int32_t H, W;          /* frame size in pixels (multiples of 20) */
    int32_t LR, LC;        /* lattice rows / cols */
    int32_t start_y;       /* first artificial row y: FrameProcessor.py:126-127 */
    int32_t NART;          /* number of artificial rows (start_y .. H-20) */
    int32_t PMAX;          /* max list positions in self.grids = LR + NART */
    int32_t MAXPK;         /* max protrusion peaks (= queries) per frame */
    int32_t NODES;         /* LR * LC */
    int32_t pad;
    /* byte offsets inside one frame record */
    int64_t frame_bytes;
    int64_t off_hdr, off_peaks, off_pos_obj, off_pos_y, off_pos_attr;
    int64_t off_cell_flags, off_cell_pen, off_node_flags, off_node_pen;
    /* byte offsets inside one query record */
    int64_t query_bytes;
    int64_t off_q_hdr, off_q_path;
    /* workspace = B frame records | B*MAXPK query records | control block */
    int64_t off_queries_per_frame; /* = frame_bytes (queries start after all frames) */
} va_nav_dims;

typedef struct va_frame_hdr {
    int32_t status;        /* VA_FRAME_* */
    int32_t x0, y0;        /* snapped rect origin (pixels): FrameProcessor.py:79-80 */
    int32_t C, Rm;         /* columns (len(j_vals)), main rows (len(i_vals)) */
    int32_t P;             /* len(self.grids) after the artificial-row loop */
    int32_t npeaks;        /* protrusion peaks = A* queries */
    int32_t start_p, start_c; /* start Grid = self.grids[start_p][start_c] (utils.py:6-32) */
    int32_t min_y;         /* y of the top-most non-empty row (pixels) */
    int32_t rounds;        /* speculative A* rounds this frame took part in */
    int32_t pad[5];
} va_frame_hdr;            /* 64 bytes; followed by int32 peak_x/peak_y/end_p/end_c[MAXPK] */

/* cell flag bits (per list position p, column c): the Grid object self.grids[p][c] */
#define VA_CELL_EMPTY 1u
#define VA_CELL_ARTIFICIAL 2u
/* node flag bits (per lattice node): the object self.grid_lookup[(x, y)] */
#define VA_NODE_EXISTS 1u      /* (x, y) in grid_lookup */
#define VA_NODE_NONEMPTY 2u    /* grid_lookup[(x, y)].empty == False */
#define VA_NODE_IN_GRIDS 4u    /* that object is also in self.grids (not an orphan) */
#define VA_NODE_MULT_SHIFT 3   /* bits 3-4: len(graph[(x, y)]) / 4 (duplicate rows, Q19) */
#define VA_NODE_ARTIFICIAL 32u /* grid_lookup[(x, y)].artificial */

typedef struct va_query_hdr {
    int32_t status;        /* VA_QUERY_* */
    int32_t len;           /* path length (Grid count) */
    double cost;           /* total_cost (g of the end node) */
    uint64_t miss[2];      /* angle keys this query added to the seen set */
    int32_t frame, k;      /* frame index, peak index */
    int32_t expansions;    /* A* pops */
    int32_t unique;        /* 1 = kept by the Jaccard/subset filter (FrameProcessor.py:256-269) */
    int32_t order;         /* index in the returned path list (-1 if dropped) */
    int32_t pad;
} va_query_hdr;            /* 56 bytes; followed by uint16 path[NODES] (lattice nodes, start..end) */

/* Fill *out for an H x W frame.  Returns VA_ERR_ARG unless H, W are positive
 * multiples of 20 and within the compiled limits (W/20, H/20 <= 64). */
int va_nav_dims_for(int32_t H, int32_t W, va_nav_dims* out);

/* Bytes of device workspace va_nav_run needs for B frames. */
int64_t va_nav_workspace_bytes(int32_t B, int32_t H, int32_t W);

/* Sample the cell lattice of B filled masks: cells[b][yi][xi] = mask[b][20*yi+10][20*xi+10] != 0
 * (FrameProcessor.py:88-97 samples exactly these pixels).  masks: uint8 [B][H][pitch]. */
int va_nav_sample_cells(void* stream, const uint8_t* masks, int64_t pitch, int32_t B, int32_t H, int32_t W,
                        uint8_t* cells);

/* The whole grid-level hot path for B frames of size H x W.
 *   cells   device uint8 [B][H/20][W/20]: lattice samples of the filled mask (cv2.fillPoly result)
 *   rects   device int32 [B][4]: cv2.boundingRect (x, y, w, h) of the mask polygon; w <= 0 = no mask
 *   seen    device uint64 [2] in/out: PathFinder.angle_cache key set (128 bits, key = prev*8+next;
 *           the process-global cache of PathFinder.py:32, never cleared).  Queries are ordered
 *           (frame, peak) exactly as the reference issues them; the result is bit-identical to
 *           running them one after the other.
 *   work    device workspace of va_nav_workspace_bytes(B, H, W) bytes: frame + query records.
 *   rounds  host out (may be NULL): speculative A* rounds needed (1 = no re-run).
 * Synchronises `stream` once per speculative round (to read the round's verdict). */
int va_nav_run(void* stream, const uint8_t* cells, const int32_t* rects, int32_t B, int32_t H, int32_t W,
               uint64_t* seen, void* work, int32_t* rounds);

/* The records va_nav_run leaves at the start of its workspace for B frames: B frame records of
 * va_nav_dims.frame_bytes, then (16-byte aligned) B * MAXPK query records of query_bytes -- bytes
 * [0, va_nav_records_bytes) of `work`. */
int64_t va_nav_records_bytes(int32_t B, int32_t H, int32_t W);

/* va_nav_run with the records read back: host_records (host memory of >= va_nav_records_bytes(B, H, W) bytes;
 * pinned, or the copy is staged and synchronous) receives them on `stream` behind each speculative round's
 * kernels and ahead of that round's verdict copy, so the call returns with the final round's records on the
 * host and the caller needs no second synchronisation (FrameProcessor.py:325-347 reads every one of them on the
 * host right after).  host_records NULL = va_nav_run. */
int va_nav_run_rb(void* stream, const uint8_t* cells, const int32_t* rects, int32_t B, int32_t H, int32_t W,
                  uint64_t* seen, void* work, int32_t* rounds, void* host_records, int64_t host_bytes);

/* Standalone A* over an explicit lattice (PathFinder.find_path surface, PathFinder.py:119-186)
 * for Q queries that share one lattice of LR x LC nodes.
 *   node_flags  device uint8 [LR*LC] (VA_NODE_* bits; multiplicity in bits 3-4)
 *   node_pen    device double [LR*LC] (Grid.penalty of grid_lookup[(x, y)], None -> 0)
 *   starts/ends device int32 [Q] lattice node indices
 *   seen        device uint64 [2] in/out
 *   qwork       device workspace of va_astar_workspace_bytes(Q, LR*LC) bytes: Q query records of
 *               va_nav_query_bytes(LR*LC) bytes each, then a 64-byte control block */
int64_t va_nav_query_bytes(int32_t nodes);
int64_t va_astar_workspace_bytes(int32_t Q, int32_t nodes);
int va_astar_run(void* stream, const uint8_t* node_flags, const double* node_pen, int32_t LR, int32_t LC,
                 const int32_t* starts, const int32_t* ends, int32_t Q, uint64_t* seen, void* qwork,
                 int32_t* rounds);


/* ---------------------------------------------------------------- segmentation (YOLOv8-seg) */
#define VA_DTYPE_BF16 1
#define VA_DTYPE_F32 2
#define VA_DTYPE_FP8 3   /* e4m3 MFMA convolutions (va_seg_conv: e4m3 weights + per-channel scales, e4m3 or bf16
                            activations, va_conv_args.xscale...); va_seg_sppf_pool / va_seg_upsample2x: e4m3 byte
                            buffers (one power-of-two scale per buffer, unchanged by max and copy) */

/* One Conv2d (+ folded BN bias, optional SiLU, optional residual add) as an implicit GEMM on MFMA.
 * Replaces the Conv / Bottleneck / C2f / SPPF / Detect / Proto convolutions Ultralytics runs inside
 * YOLO.predict (FrameProcessor.py:322; modules conv.py:54, block.py:237-239, head.py per the
 * reference's profile.svg).  Activations are NHWC channel slices: element (n, h, w, c) of a tensor
 * lives at ptr[((n*H + h)*W + w)*ld + c]. */
typedef struct va_conv_args {
    const void* x;          /* input slice (dtype) */
    int32_t N, H, W, Cin, ldx;
    int32_t kh, kw, stride, pad;
    int32_t Ho, Wo;
    const void* w;          /* packed weights (dtype) [Npad][Kpad], K ordered (ky, kx, ci), zero padded */
    const float* bias;      /* [Npad] */
    int32_t Cout, Npad, K, Kpad; /* K = kh*kw*Cin; Kpad % 32 == 0; Npad % 128 == 0 */
    void* y;                /* output slice (dtype, or float if out_f32) */
    int32_t ldy;
    const void* res;        /* residual slice (dtype) added after the activation, or NULL */
    int32_t ldr;
    int32_t act;            /* 1 = SiLU */
    int32_t mode;           /* 0 = conv, 1 = ConvTranspose2d(k=2, s=2) packed as a 1x1 conv with Cout = 4*C,
                               2 = sub-pixel classes (bf16, Cout > 64): ConvTranspose2d(k=2, s=2) followed by a
                               3x3 / pad 1 conv, folded: for each class c = 2 dy + dx a 2x2 conv (kh = kw = 2,
                               stride 1) with pads (1 - dy, 1 - dx) and weights w + c * Npad * Kpad, writing
                               pixel (2 ho + dy, 2 wo + dx) of a [N][2 Ho][2 Wo] map; M = N * Ho * Wo */
    int32_t M;              /* N * Ho * Wo */
    int32_t dtype;          /* VA_DTYPE_BF16 (MFMA bf16, f32 accumulate) or VA_DTYPE_F32 (exact f32 MFMA) */
    int32_t out_f32;        /* bf16 inputs with a float output (head logits) */
    int32_t bias4;          /* mode 2 only (bf16: with a fused tail): bias is a border table [4 classes][2][2][Npad],
                               entry [c][rf][cf] for output pixels whose class-c taps miss the map's first /
                               last row (rf) or column (cf) -- the folded deconv bias depends on which taps
                               fall inside the map, so no constant-1 input channel is needed */
    /* Optional fused 1x1 tail conv (bf16, mode 0, no residual; Cout == 128 with c2 <= 80, or Cout 32 / 64 with
     * c2 <= 64 and the weights fitting 120 KiB of LDS): when w2 != NULL the main conv's activations (bias + act,
     * rounded to bf16 as a stored layer would be) never leave the chip and feed y2 = act2(W2 . a + b2);
     * y / ldy / out_f32 then describe the TAIL output (c2 channels, c2 % 4 == 0).  Replaces a 1x1 layer that
     * only consumes this one (proto.cv2 -> proto.cv3, head cv2/cv3/cv4 .l.1 -> .l.2).
     * f32 (VA_DTYPE_F32 with w3): a stride-1 3x3 / pad 1 conv (or the mode-2 fold) with Cout 64 or 128 (128 for
     * mode 2), c2 <= 96, no residual; w2 = the tail's weights as three exact bf16 terms [32 ceil(c2 / 32)][Cout / 8]
     * [3][8] (w3's layout), the main activations kept in f32 and contracted as six exact term products; the tail
     * output is float. */
    const void* w2;         /* bf16: [>= ceil16(c2)][Cout], K contiguous; f32: the three-term planes above */
    const float* b2;        /* [>= ceil16(c2)] */
    int32_t c2;
    int32_t act2;           /* 1 = SiLU */
    /* Optional nearest-x2 upsampled channel prefix (the FPN's Upsample + Concat read in place, Ultralytics
     * nn.Upsample + Concat of YOLOv8's head): when xu != NULL, input channels [0, cu) of pixel (n, h, w) are
     * read from xu at (n, h/2, w/2) -- an [N][H/2][W/2] slice with channel stride ldu -- and channels
     * [cu, Cin) from x as usual (x's first cu channels are never read).  bf16, 1x1 / stride 1 / mode 0 without
     * a tail, Cin and cu multiples of 64, H and W even. */
    const void* xu;
    int32_t ldu;
    int32_t cu;
    /* VA_DTYPE_FP8: w is e4m3 [Npad][Kpad] (Kpad % 128 == 0); the input holds sat(x * xscale) as e4m3 bytes
     * (x8 = 1: an fp8 activation buffer, ldx % 16 == 0) or is bf16 quantized so on the fly (x8 = 0); the
     * accumulator is dequantized by wscale[co] (= the weights' per-channel scale / xscale) before bias and act.
     * Output: e4m3 sat(y * yscale) when yscale > 0 (ldy % 8 == 0), else bf16 (or float with out_f32); an e4m3
     * residual holds r * rscale (rscale > 0), else bf16.  Scales are powers of two.  Mode 0 / 1, Cin % 16 == 0,
     * no tail / xu / bias4 (BASELINE.json configs[4]: "fp8 MFMA weights"). */
    const float* wscale;    /* [Npad] */
    float xscale;
    int32_t x8;
    float yscale;
    float rscale;
    /* VA_DTYPE_F32 only: the weights pre-split into their three exact bf16 terms h, m, l (x = h + m + l, each the
     * round-to-nearest bf16 of what remains), [Npad][Kpad / 8][3][8] -- per 8-channel K group the 8 h, then the
     * 8 m, then the 8 l -- with K ordered group-major: G-channel group, then tap, then channel (K' = (c / G) taps G +
     * G tap + c % G; G = 32 when stride == 2, kh kw > 1 and Cin % 32 == 0, else 16; a K-step is one 96-byte run of 16
     * channels; seg.py w3_rows / w3_group).  When set (and Cin % 16 == 0, Npad % 128 == 0, K == Kpad, mode 0 or 2) the
     * conv runs on the three-plane kernels (va_seg.hip conv3t_kernel / conv3h_kernel); NULL keeps conv2's in-loop
     * split. */
    const void* w3;
    /* Optional split-K workspace (any dtype; conv2's LDS-DMA form, mode 0 / 2): when ws != NULL and the layer has
     * too few output tiles to fill the chip (a batch-1 forward's 40 x 40 and 20 x 20 layers), the dispatcher may
     * split the K loop of each tile over up to 16 workgroups.  Each writes its f32 partial tile to ws, the last
     * to arrive (per-tile arrival counter in wcnt, agent-scope release / acquire) sums them and runs the usual
     * epilogue -- same operands, same per-split f32 accumulation, then one f32 sum of the partials.  The
     * dispatcher only splits when tiles * splits * 64 KiB <= ws_bytes and tiles <= ncnt.  wcnt must be zero
     * before the first call; every split launch leaves it zero again.  A plan's ops run in order on one
     * stream, so one workspace serves them all; two streams need two.  The persistent kernels (the f32 32-channel
     * 3x3 conv3q, va_seg_stem / va_seg_stem_f32, va_seg_c2f) use wcnt[0..1] (ncnt >= 2) as a work counter when it
     * is given: tiles claimed as workgroups start, not a static schedule, and both counters zero again when the
     * launch ends (VA_CONV3Q=static: the static schedule). */
    void* ws;
    int64_t ws_bytes;
    int32_t* wcnt;
    int32_t ncnt;
    /* VA_DTYPE_BF16 only -- C5's weight-only fp8 form (BASELINE.json configs[4] "fp8 MFMA weights" on bf16
     * activations): w8 = 1 means w holds e4m3 bytes [Npad][Kpad] (mode 2: [4][Npad][Kpad]) and wscale the weights'
     * scale per output channel, float [Npad] (mode 2: [4][Npad]), 16-byte aligned.  K order inside every 64-element
     * block of a row: the eight 8-element chunks stored as 0, 4, 1, 5, 2, 6, 3, 7 (chunk c at byte 8 (2 (c % 4) +
     * c / 4)), so one 16-byte piece holds both K halves of an MFMA fragment.  The bf16 kernels (conv2, conv4, conv_dn,
     * the patch kernel and the generic fallback) convert the bytes exactly to bf16 -- conv2 as it reads its A
     * fragments, the others as they stage them -- and multiply the f32 accumulator by wscale[co] before the bias; the
     * streaming 1x1 (pw), which has no A stage, is skipped for these ops.  A fused tail's w2 stays bf16.  Replaces the
     * host-side dequantization into bf16 weights (round 5's w8a16 form), so HBM holds 1 byte per weight. */
    int32_t w8;
} va_conv_args;

int va_seg_conv(void* stream, const va_conv_args* a);

/* One C2f block with n = 1 and a shortcut, 64 -> 64 channels (block.py C2f / Bottleneck, hidden 32):
 * cv1 (1x1) -> chunk -> m.0.cv1 (3x3) -> m.0.cv2 (3x3) + residual -> cat -> cv2 (1x1), every conv with
 * folded BN bias + SiLU, as ONE launch whose intermediates never leave the chip (bf16 only).  Uses
 * a.x / a.ldx (input, 64 channels), a.N / H / W, a.Cin = a.Cout = 64, a.y / a.ldy (output), a.dtype and:
 *   a.w    bf16 weight blob in MFMA fragment order (28672 values; layout: seg.py SegNet._pack_c2f)
 *   a.bias float [192] = cv1 [64] | m.0.cv1 [32] | m.0.cv2 [32] | cv2 [64]
 * ldx, ldy % 8 == 0; x, y, w, bias 16-byte aligned.  Replaces the four va_seg_conv calls of the
 * block (the reference's model.2 in YOLOv8s-seg). */
int va_seg_c2f(void* stream, const va_conv_args* a);
/* The stem (bf16) as ONE launch: uint8 BGR frames [N][H][W][3] -> RGB / 255 -> model.0 Conv(3, 32, 3x3, s2)
 * + SiLU -> model.1 Conv(32, 64, 3x3, s2) + SiLU -> a.y [N][ceil(H/4)][ceil(W/4)] (channel stride a.ldy), the
 * 32-channel model.0 map never leaving the chip.  Replaces va_seg_conv0 + the model.1 va_seg_conv.  Uses
 * a.x (frames), a.N / H / W (frame size, W % 16 == 0), a.Cin = 32, a.Cout = 64, a.y / a.ldy (ldy % 8 == 0),
 * a.dtype = VA_DTYPE_BF16 and:
 *   a.w    bf16 weight blob in MFMA fragment order (20480 values; layout: seg.py SegNet._pack_stem)
 *   a.bias float [96] = model.0 [32] | model.1 [64] */
int va_seg_stem(void* stream, const va_conv_args* a);
/* Any C2f block of YOLOv8n/s-seg as ONE launch for small batches (bf16; the batch-1 latency path, C2):
 * cv1 (1x1, ci -> 2c) -> chunk -> n Bottlenecks (3x3 c -> c, 3x3 c -> c, + shortcut when set) -> cat -> cv2 (1x1,
 * (2 + n) c -> co), every conv with folded BN bias + SiLU, each intermediate rounded to bf16 as a stored layer
 * would be.  A workgroup owns a T x T output tile and recomputes the 2n-pixel halo its 3x3s need; nothing but the
 * block's output leaves the chip.  Fields: a.x / a.ldx / a.Cin = ci (input, ci % 8 == 0; with a.xu / a.ldu /
 * a.cu the first cu channels are the nearest-x2 upsample of a half-resolution slice, read in place as for
 * va_seg_conv), a.y / a.ldy / a.Cout = co (co % 16 == 0), a.N / H / W, a.dtype = VA_DTYPE_BF16, a.mode = 3, and
 *   a.Npad   hidden width c (16, 32, 64 or 128)
 *   a.kh     n, Bottlenecks (1 or 2);  a.kw  shortcut (1 / 0)
 *   a.stride tile side T (the LDS layout must fit: va_c2fb_layout)
 *   a.w      bf16 A fragments (seg.py SegNet._pack_c2fb): per conv (cv1, m.0.cv1, m.0.cv2, .., cv2) the packed
 *            [Cout][K] weights (K ordered (ky, kx, ci)) zero padded to 16-row x 32-column tiles, in tile order
 *            [Cout / 16][K / 32], each tile as 64 lanes x 8 (lane 16 q + r: row r, columns 8 q .. 8 q + 7)
 *   a.bias   float, per conv its biases zero padded to a multiple of 16, in the same order
 * Optional stride-2 prologue (bf16; a.res != NULL): the block's input channels [0, cs) are Conv(cis -> cs, 3x3,
 * stride 2, pad 1) + bias + SiLU of a.res ([N][2H][2W], channel stride a.ldr), computed per tile from its (2(T + 4n)
 * + 1)^2 source pixels -- the backbone's / PAN's stride-2 convs (model.3 / 5 / 7 / 16 / 19) whose only consumer is
 * the block; a.c2 = cs (% 16 == 0, <= ci), a.K = cis (a power of two, 8 .. 512), the conv's tiles and biases after
 * cv2's in a.w / a.bias; x's first cs channels are not read; no xu.
 * ldx, ldy, ldu % 8 == 0; x, xu, y, w, bias 16-byte aligned.  Replaces the block's 2n + 2 va_seg_conv calls
 * (block.py C2f, Bottleneck) inside YOLO.predict (FrameProcessor.py:322).  VA_OP_C2F with a.mode == 3.
 * a.dtype = VA_DTYPE_F32 (the reference's precision; c up to 256): float activations (ldx, ldy, ldu % 4 == 0), every
 * product as six exact bf16 term products (va_seg_conv's f32 arithmetic), a.w = the same tiles as three fragments
 * each (h, m, l: the exact three-term bf16 split of the f32 weights, [tile][3][64 lanes][8]).  Its intermediates sit in
 * LDS as their three bf16 terms (split once by the producing conv's epilogue) where that layout fits, else as f32
 * split per read (va_c2fb_layout out[3]). */
int va_seg_c2fb(void* stream, const va_conv_args* a);
/* va_seg_c2fb's sizes for hidden width c, n Bottlenecks, ci / co channels, tile side T, dtype and the stride-2
 * prologue's cs / cis channels (0, 0: none): out[0] = LDS bytes per workgroup, out[1] = A fragments (64 lanes x 8
 * bf16) of the weight blob, out[2] = floats of the bias blob, out[3] = 1 when the f32 form keeps its intermediates as
 * bf16 term planes (else 0).  VA_ERR_ARG when the shape is not covered or the layout exceeds the 160 KiB of LDS
 * (out[1], out[2] still set for a covered shape).  out holds 4 values. */
int va_c2fb_layout(int32_t c, int32_t n, int32_t ci, int32_t co, int32_t T, int32_t dtype, int32_t cs, int32_t cis,
                   int64_t* out);
/* The stem in f32 (the headline's precision) as ONE launch: uint8 BGR frames [N][H][W][3] -> model.0 (the
 * three exact bf16 terms of its weights x the frame bytes, x 1/255, + bias, SiLU) -> model.1 Conv(32, 64, 3x3, s2)
 * + SiLU as six exact bf16 term products -> float a.y [N][ceil(H/4)][ceil(W/4)] (channel stride a.ldy % 4 == 0);
 * the 32-channel f32 model.0 map never leaves the chip.  Replaces va_seg_conv0_f32m + the model.1 va_seg_conv.
 * a.dtype = VA_DTYPE_F32, a.Cin = 32, a.Cout = 64, (W * 3) % 16 == 0, and:
 *   a.w3   model.0's K-padded weights as three exact bf16 terms [32][4][3][8] (va_seg_conv0_f32m's w3)
 *   a.bias model.0's bias float [32]
 *   a.w    model.1's packed f32 weights [Npad][Kpad], K = Kpad = 288 ordered (ky, kx, ci)
 *   a.b2   model.1's bias float [64]
 * Optional tail (a.w2 != NULL): model.2.cv1, the C2f's 1x1 Conv(64, 64) + SiLU, in the epilogue -- model.1's map
 * stays on the chip too and a.y receives cv1's output: a.w2 = its f32 weights [>= 64][64], a.b2 = [model.1 bias 64 |
 * cv1 bias 64], a.c2 = 64, a.act2 = 1.  Replaces the model.2.cv1 va_seg_conv as well. */
int va_seg_stem_f32(void* stream, const va_conv_args* a);
/* Debug: record per-wave stage clocks (s_memtime) of the first 32 tiles of every workgroup of the next
 * va_seg_c2f launches into device memory buf ([grid][8][32][6] uint64), or stop (buf = NULL). */
int va_c2f_trace(void* buf);
/* Debug: per-workgroup stage clocks of the next va_seg_c2fb launches into device memory buf ([grid][10] uint64: thread
 * 0's s_memtime at the start, after each stage's barrier and at the end; unused points keep their contents), or stop
 * (buf = NULL). */
int va_c2fb_trace(void* buf);
/* Debug: the same for va_seg_stem ([grid][8][32][5] uint64 of the 100 MHz real-time counter). */
int va_stem_trace(void* buf);

/* uint8 BGR frames [B][H][W][3] -> RGB / 255 NHWC with 8 channels (3 used), dtype VA_DTYPE_*. */
int va_seg_preprocess(void* stream, const uint8_t* frames, int32_t B, int32_t H, int32_t W, int32_t dtype, void* out);

/* model.0 fused with the preprocessing (bf16): uint8 BGR [N][H][W][3] -> RGB/255 -> Conv2d(3, Cout, 3, s2, p1)
 * + folded BN bias + SiLU -> bf16 NHWC [N][H/2][W/2] with channel stride ldy.  w: bf16 [Cout][32], k =
 * (ky*3 + kx)*3 + c with c in R, G, B order, k >= 27 zero; Cout in {16, 32, 48, 64}; W % 16 == 0, ldy % 8 == 0,
 * frames and y 16-byte aligned. */
int va_seg_conv0(void* stream, const uint8_t* frames, int32_t N, int32_t H, int32_t W, const void* w,
                 const float* bias, int32_t Cout, void* y, int32_t ldy);

/* The same layer in exact f32 (the parity / headline mode): uint8 BGR -> RGB / 255 (f32 division) ->
 * Conv2d(3, Cout, 3, s2, p1) + folded BN bias + SiLU (x / (1 + exp(-x))) -> f32 NHWC [N][H/2][W/2] with channel
 * stride ldy, on the vector ALU (K = 27: one output pixel per lane, the weights wave-uniform).  w: f32 [Cout][27],
 * k = (ky*3 + kx)*3 + c with c in R, G, B order; Cout in {16, 32, 48, 64}; ldy % 4 == 0, y 16-byte aligned. */
/* va_seg_conv0 with an e4m3 output sat(y * yscale) (the fp8 mode's first activation buffer; bf16 weights and
 * arithmetic as va_seg_conv0, yscale a power of two). */
int va_seg_conv0_e4m3(void* stream, const uint8_t* frames, int32_t N, int32_t H, int32_t W, const void* w,
                      const float* bias, int32_t Cout, uint8_t* y, int32_t ldy, float yscale);

int va_seg_conv0_f32(void* stream, const uint8_t* frames, int32_t N, int32_t H, int32_t W, const float* w,
                     const float* bias, int32_t Cout, float* y, int32_t ldy);

/* The f32 layer on the MFMA: the [Cout][32] (K-padded) weights as three exact bf16 terms w3 = bf16 [Cout][4][3][8]
 * (per 8-element group h, m, l with h + m + l == w exactly), the frame bytes as exact bf16 operands, three term
 * products accumulated in f32 per fragment pair, then * (1/255) + bias and SiLU (exp2 / rcp form of the f32 convs)
 * -> f32 NHWC as va_seg_conv0_f32 (max |diff| against it at f32 rounding level: tests/test_gpu_seg.py).  The
 * VA_OP_CONV0 op takes this form when a.w3 is set.  W * 3 % 16 == 0 (the 16-byte patch loads). */
int va_seg_conv0_f32m(void* stream, const uint8_t* frames, int32_t N, int32_t H, int32_t W, const void* w3,
                      const float* bias, int32_t Cout, float* y, int32_t ldy);

/* SPPF (block.py SPPF): slice 0 (c channels) of an NHWC buffer of channel stride ld >= 4c -> slices 1..3
 * = MaxPool2d(5, 1, 2) applied once, twice, three times (dtype F32 / BF16 / FP8: e4m3 bytes, ordered as the
 * values they encode). */
int va_seg_sppf_pool(void* stream, void* buf, int32_t N, int32_t H, int32_t W, int32_t c, int32_t ld, int32_t dtype);

/* nn.Upsample(scale_factor=2, mode="nearest") from a slice into a concat slice. */
int va_seg_upsample2x(void* stream, const void* src, int32_t ld_s, void* dst, int32_t ld_d, int32_t N, int32_t H,
                      int32_t W, int32_t c, int32_t dtype);

/* A whole forward as a list of ops executed back-to-back on one stream by ONE call (no per-layer
 * host round trip; the list is built once per (batch, frame size) by the host planner), optionally with
 * independent branches on lanes (VA_OP_FORK). */
#define VA_OP_CONV 1        /* conv: all fields of .a */
#define VA_OP_SPPF 2        /* sppf pool: a.y = buffer, a.N/H/W, a.Cin = c, a.ldy = ld, a.dtype */
#define VA_OP_UPSAMPLE 3    /* upsample2x: a.x/a.ldx -> a.y/a.ldy, a.N/H/W (source size), a.Cin = c, a.dtype */
#define VA_OP_PREPROCESS 4  /* preprocess: a.x = uint8 frames, a.y = out, a.N/H/W, a.dtype */
#define VA_OP_CONV0 5       /* preprocess fused into model.0: a.x = uint8 frames, a.N/H/W (input), a.w, a.bias,
                               a.Cout, a.y, a.ldy, a.dtype (FP8: e4m3 output with a.yscale; F32 with a.w3: the
                               MFMA form) -- see va_seg_conv0 / va_seg_conv0_f32(m) / va_seg_conv0_e4m3 */
#define VA_OP_C2F 6         /* fused C2f block: see va_seg_c2f (a.mode == 3: va_seg_c2fb) */
#define VA_OP_STEM 7        /* fused preprocess + model.0 + model.1: va_seg_stem (bf16), va_seg_stem_f32 (f32) */
/* Branch-parallel lists (small batches, where one layer does not fill the 256 CUs): an op with lane L > 0
 * is issued on auxiliary stream L of the calling stream (VA_LANES - 1 of them, created on first use per
 * (device, calling stream) and kept for the process).  FORK (a.N = L): lane L waits for everything issued
 * so far on the calling stream; JOIN (a.N = L): the calling stream waits for everything issued so far on
 * lane L.  An op on lane L needs an earlier FORK of L in the same list; lanes still open at the end of the
 * list are joined by the call, so the calling stream covers the whole list when it returns (and a graph
 * captured on it holds the lanes as parallel branches).  While va_prof_* recording is on, lanes are
 * ignored (every op on the calling stream, in list order -- a valid serial order of any laned list). */
#define VA_OP_FORK 8
#define VA_OP_JOIN 9
#define VA_LANES 4
typedef struct va_seg_op {
    int32_t kind;
    int32_t lane; /* 0 = the calling stream; 1 .. VA_LANES - 1 (see VA_OP_FORK) */
    va_conv_args a;
} va_seg_op;

int va_seg_run(void* stream, const va_seg_op* ops, int32_t n);

/* Optional live timing of va_seg_run: while enabled every op is bracketed by a pair of HIP events on
 * the launch stream (capacity = max ops recorded).  va_prof_stop waits for the last event and returns,
 * per op kind (VA_OP_*, index = kind), the summed milliseconds and the launch count; returns the number
 * of ops recorded. */
int va_prof_start(int32_t capacity);
int va_prof_stop(double* ms_by_kind, int64_t* n_by_kind, int32_t nkinds);
/* Per op-list index instead of per kind (call before va_prof_stop, which clears the records). */
int va_prof_stop_ops(double* ms_by_op, int32_t nops);
/* Suspend (on = 0) / resume (on = 1) the recording between va_prof_start and va_prof_stop, keeping the
 * records: lets a caller sample some forwards of a timed run (each event pair is a GPU-side packet). */
int va_prof_enable(int32_t on);

/* ---------------------------------------------------------------- segmentation post-processing */
typedef struct va_cand { float x1, y1, x2, y2, score; int32_t cls, anchor, pad; } va_cand;  /* NMS candidate */
typedef struct va_det { float x1, y1, x2, y2, score; int32_t cls, anchor, pad; } va_det;    /* kept detection */
typedef struct va_mask_stat { int32_t count, x0, y0, x1, y1, pad[3]; } va_mask_stat;        /* mask pixels, bbox */
/* Per instance mask: its Results.masks.xy polygon as FrameProcessor consumes it (masks2segments 'largest' +
 * scale_coords; oracle/contours.py restates OpenCV's algorithms). */
typedef struct va_contour_stat {
    int32_t npts;     /* CHAIN_APPROX_SIMPLE points of the largest external contour (0: empty mask) */
    int32_t ox, oy;   /* its start pixel in the instance's framed region image */
    int32_t ncont;    /* external contours found (RETR_EXTERNAL) */
    int32_t X0, Y0;   /* the region's origin in network pixels (framed image pixel (x, y) = (X0 + x - 1, Y0 + y - 1)) */
    int32_t status;   /* 0 ok */
    int32_t half;     /* which half of the instance's point buffer (cpts) holds that contour */
    double area;      /* cv2.contourArea of the float32 scale_coords points */
} va_contour_stat;

/* Everything YOLO.predict does after the forward, for B frames, plus the mask choice of
 * FrameProcessor.py:67-97 with OpenCV's algorithms restated (oracle/contours.py; parity with cv2 unpinned):
 *   decode (DFL, dist2bbox, sigmoid) -> conf filter -> max_nms cut -> class-offset greedy NMS (IoU > iou) -> max_det
 *   -> process_mask (coef . proto, crop, bilinear x4, > 0) -> per-instance pixel count / bbox (stats), the
 *      largest external contour (findContours RETR_EXTERNAL, CHAIN_APPROX_SIMPLE) and its contourArea over
 *      the float32 scale_coords points (cstats)
 *   -> (if cells != NULL) the instance of
 *      max area (first maximum; a single one as it is), np.int32 of its polygon, boundingRect, and
 *      fillPoly(LINE_8) sampled at the 20-px cell centres of the H0 x W0 frame -> the (cells, rects) input of
 *      va_nav_run.
 * plant_mode: 0 = never plant; 1 = use plant_cells/plant_rects for frames with no detection; 2 = always. */
typedef struct va_post_args {
    const float* levels[3];     /* float [B][H/s][W/s][64 + nc + 32], s = 8, 16, 32 */
    const float* proto;         /* float [B][H/4][W/4][32] */
    int32_t B, H, W, nc;
    float conf, iou;            /* 0.5 (FrameProcessor.py:322), 0.7 (Ultralytics default) */
    int32_t max_det;            /* 300 */
    int32_t plant_mode;
    va_cand* cand;              /* scratch [B][A] */
    int32_t* cand_count;        /* scratch [B] */
    unsigned long long* keys;   /* scratch [B][A] */
    va_det* dets;               /* out [B][max_det] */
    int32_t* ndet;              /* out [B] */
    va_mask_stat* stats;        /* out [B][max_det] */
    const uint8_t* plant_cells; /* [B][H/20][W/20] or NULL */
    const int32_t* plant_rects; /* [B][4] or NULL */
    uint8_t* cells;             /* out [B][H/20][W/20] or NULL (skip the mask choice) */
    int32_t* rects;             /* out [B][4] */
    int32_t* chosen;            /* out [B]: chosen detection, -1 none, -2 planted */
    /* The frame the network input was letterboxed from (va_letterbox): cells / rects refer to the H0 x W0
     * frame; polygon points are mapped back as ops.scale_coords does in float32: (p - pad) / gain, clipped to
     * [0, W0] x [0, H0], with gain = min(H/H0, W/W0) and pad = ((W - W0 gain) / 2, (H - H0 gain) / 2) rounded
     * to float32 (numpy's float32 arithmetic).  H0 = 0: the frame is the network input (gain 1, pad 0). */
    int32_t H0, W0;
    float sc_gain, sc_padx, sc_pady;
    /* contour scratch: cslots slots of va_contour_scratch_bytes(H, W, cslots, ccap) bytes each */
    void* cscratch;
    int32_t cslots, ccap;
    va_contour_stat* cstats;    /* out [B][max_det] */
    int32_t* cstatus;           /* out [B] or NULL: 0 (a chosen contour longer than cpts_cap is filled in chunks) */
    /* per instance two buffers of cpts_cap contour points (network pixel x | y << 16): the contour being
     * followed and the longest so far; a longer contour is followed again from the image instead */
    uint32_t* cpts;             /* scratch [B][max_det][2][cpts_cap] */
    /* non_max_suppression's max_nms (ops.py:332-333): a candidate list longer than this is cut to its
     * max_nms highest scores before NMS.  <= 0: VA_MAX_NMS (Ultralytics' 30000). */
    int32_t max_nms;
    int32_t cpts_cap;
} va_post_args;

#define VA_MAX_NMS 30000

/* LetterBox(new_shape, auto=True, stride 32) of uint8 BGR frames [B][H][W][3] into [B][Hn][Wn][3]:
 * bilinear resize to newh x neww (cv2.INTER_LINEAR fixed-point form; a copy when the size is unchanged)
 * placed at (top, left), the border filled with 114.  Replaces the LetterBox call inside YOLO.predict
 * (FrameProcessor.py:322; Ultralytics data/augment.py LetterBox). */
int va_letterbox(void* stream, const uint8_t* src, int32_t B, int32_t H, int32_t W, uint8_t* dst, int32_t Hn,
                 int32_t Wn, int32_t top, int32_t left, int32_t newh, int32_t neww);

/* Number of anchors A for an H x W input (strides 8, 16, 32), or < 0. */
int va_post_anchors(int32_t H, int32_t W);
/* cells == NULL and cstats == NULL: decode + NMS only (the contour pass and its buffers are not touched). */
int va_post_run(void* stream, const va_post_args* p);

/* Bytes of one contour scratch slot for an H x W network input with point capacity cap, and the offsets of its
 * image and point areas.  The caller allocates nslots x *slot_bytes. */
int va_contour_scratch_bytes(int32_t H, int32_t W, int32_t nslots, int32_t cap, int64_t* slot_bytes, int64_t* img_off,
                             int64_t* pts_off);

/* The same mask -> polygon -> cells boundary for given binary masks (test / harness entry point): masks uint8
 * [B][maxn][Hn][Wn] (non-zero = set), nmask[b] masks for frame b.  polys (optional) [B][maxn][poly_cap][2] float
 * receives each mask's Results.masks.xy polygon (poly_n[b * maxn + k] points). */
typedef struct va_mask_select_args {
    const uint8_t* masks;
    const int32_t* nmask;
    int32_t B, maxn, Hn, Wn, H0, W0;
    float gain, padx, pady;
    void* scratch;
    int32_t nslots, cap;
    va_contour_stat* cstats;    /* out [B][maxn] */
    uint8_t* cells;             /* out [B][H0/20][W0/20] or NULL */
    int32_t* rects;             /* out [B][4] */
    int32_t* chosen;            /* out [B] */
    int32_t* status;            /* out [B] or NULL */
    float* polys;               /* out or NULL */
    int32_t* poly_n;
    uint32_t* cpts;             /* scratch [B][maxn][2][cpts_cap] (va_post_args.cpts) */
    int32_t poly_cap, cpts_cap;
} va_mask_select_args;
int va_post_select_masks(void* stream, const va_mask_select_args* m);

/* Results.masks.xy for the detections of the last va_post_run on the same buffers (p as passed to it, with
 * cstats): per detection its largest external contour in frame coordinates, float [B][max_det][poly_cap][2],
 * poly_n [B][max_det] points (truncated to poly_cap). */
int va_post_polygons(void* stream, const va_post_args* p, float* polys, int32_t* poly_n, int32_t poly_cap);

/* ABI self-check: writes sizeof() of va_nav_dims, va_frame_hdr, va_query_hdr, va_conv_args, va_seg_op,
 * va_cand, va_det, va_mask_stat, va_post_args, va_contour_stat, va_mask_select_args (in that order) into
 * out[0..n-1]; returns how many. */
int va_abi_struct_sizes(int64_t* out, int32_t n);

/* Device-bound handle.  va_create binds to HIP device `device` (a gfx950; flags must be 0);
 * the kernels' own entry points stay stateless.  va_frame runs one batch through the whole hot path on the
 * handle's device (made current for the call, the caller's restored after it): va_seg_run(ops) ->
 * va_post_run(post) -> va_nav_run(post->cells, post->rects, post->B, H0, W0, seen, nav_work, rounds) -- the
 * reference's FrameProcessor.__call__ (FrameProcessor.py:301-360) up to the PathAnalyser, for post->B frames of
 * H0 x W0 (the frame size the cells and rects are in).  Returns the first failing stage's status. */
typedef struct va_handle_s* va_handle;
int va_create(int32_t device, uint32_t flags, va_handle* out);
int va_destroy(va_handle h);
int va_handle_device(va_handle h, int32_t* device);
int va_frame(va_handle h, void* stream, const va_seg_op* ops, int32_t nops, const va_post_args* post, int32_t H0,
             int32_t W0, uint64_t* seen, void* nav_work, int32_t* rounds);
/* va_frame whose grid stage is va_nav_run_rb: the nav records land in host_records (NULL = va_frame). */
int va_frame_rb(va_handle h, void* stream, const va_seg_op* ops, int32_t nops, const va_post_args* post, int32_t H0,
                int32_t W0, uint64_t* seen, void* nav_work, int32_t* rounds, void* host_records,
                int64_t host_bytes);

/* Out-of-range state the kernels rejected instead of faulting (a rect no frame holds, an A* node outside the
 * lattice, a traced pixel outside its image, candidate counts past the anchors -- csrc/va_diag.h lists the
 * codes): out[4 i .. 4 i + 3] = {first code, v0, v1, count} for the units post, contour, nav (n >= 12); the
 * words are zeroed when clear != 0.  Synchronises the current device.  Debug / test surface. */
int va_diag(uint32_t* out, int32_t n, int32_t clear);

/* The library's A/B switches (environment variables VA_F32_SPLIT, VA_CONV3H, VA_CONV3T, VA_SPLITK, VA_CONV_PATCH,
 * VA_CONV4, VA_PW, VA_CT_RUNS, VA_CT_WGP) are read once per process, at the first launch that
 * consults them.  va_switches_reload re-reads them (a test comparing two kernel forms inside one process). */
int va_switches_reload(void);

/* Library version / build info string; "abi 3": va_post_args as above (sc_* floats, cpts / cpts_cap / max_nms;
 * round 2 changed its layout from round 1's int pad_x / pad_y) -- check va_abi_struct_sizes as well. */
const char* va_version(void);

#ifdef __cplusplus
}
#endif
#endif /* VA355_H */

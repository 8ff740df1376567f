// lbm_layout.hpp -- device data layout and kernel argument blocks shared by
// the HIP kernels (lbm_kernels.hip, lbm_step2.hip) and the engine
// (lbm_engine.hip).
//
// Lattice (one per ping-pong side, per sub-domain of w x h cells): SoA with a
// ghost ring gr cells wide (engine: gr = max(2, halo width of the kernel in
// use), at most MAX_GR).  Kernels address it through an ORIGIN pointer
// o = &f[plane 0][cell (0,0)]:
//     cell (x, y), -2 <= x < w+2, -2 <= y < h+2, speed k  ->  o[k*plane + y*pitch + x]
// Default layout (row-interleaved): the nine planes of a lattice row are
// adjacent, plane = rf, pitch = 9*rf, rf = roundup(w + xoff + gr + 2, 64); the
// planar layout (plane = rows*rf + pad, pitch = rf) is kept for A/B.  The
// interior row start sits XOFF = 4 floats into each plane row, so every
// interior float4 is 16-byte aligned.
//
// Speeds (main/include/LatticeBoltzmannUtils.hpp:20-22):
//   0 M, 1 E(+1,0), 2 N(0,+1), 3 W(-1,0), 4 S(0,-1),
//   5 NE(+1,+1), 6 NW(-1,+1), 7 SW(-1,-1), 8 SE(+1,-1)
// Pull streaming: s_k(x,y) = f_old[k](x - cx_k, y - cy_k)   (LastChance.cpp:203-211)
//
// Halo directions d = 0..7 use the velocity of speed d+1: E, N, W, S, NE, NW, SW, SE.
// Two halo formats:
//   W1 (one-step kernels): the populations that leave through side d
//       (PLANES[d]) of the outermost cell row/column, ghost ring width 1.
//   WG (multi-step kernels, width g = steps per launch): all nine
//       populations of the g outermost cell rows/columns (g x g cells at
//       corners) -- a fused S-step launch pulls from up to S cells out.
//       (The fused two-step kernel is the g = 2 case, historically "W2".)
#pragma once

#include <cstdint>

namespace lbm {

constexpr int Q = 9;
constexpr int XOFF = 4;   // interior column 0 offset inside a plane row
constexpr int MAX_GR = 10;  // widest ghost ring (rows/columns) any kernel needs (stream kernel: S <= 10, tolerance)
// smallest interior column offset: an odd-S strip reads S + 1 columns left of
// column 0 (float2 alignment), and rows must stay 16-B aligned
constexpr int MIN_XOFF = (MAX_GR + 2 + 3) / 4 * 4;
constexpr int BLOCK = 256;  // 4 wave64s
constexpr int MAX_RECTS = 4;
constexpr int MAX_SRECTS = 32;  // stream kernels: guided per-XCD row bands (lbm_engine.hip stream_split)

// fused two-step tile shapes (cells).  v1 (step2): LDS intermediate
// 9 x (TH+2) x (TW+2) floats, 256 threads.  v2 (step2w): one wave per tile
// row, TW = 64, planes 0/1/3 in registers, LDS 6 x (TH+2) x 66 floats.
// The two shapes that won their A/B (profiles/r01/ab_step2_tiles.log): v2
// 64x8 with 8 waves while the lattice pair lives in the Infinity Cache, v1
// 64x8 once it streams from HBM (the other eight shapes were removed).
enum Tile2 : int { T2_64x8 = 0, T2V_64x8_W8 = 1 };
constexpr int NUM_TILE2 = 2;
constexpr int T2_W[NUM_TILE2] = {64, 64};
constexpr int T2_H[NUM_TILE2] = {8, 8};

enum Dir : int { DE = 0, DN = 1, DW = 2, DS = 3, DNE = 4, DNW = 5, DSW = 6, DSE = 7 };

// d -> (dx, dy)
constexpr int DIR_X[8] = {1, 0, -1, 0, 1, -1, -1, 1};
constexpr int DIR_Y[8] = {0, 1, 0, -1, 1, 1, -1, -1};
constexpr int OPP_DIR[8] = {DW, DS, DE, DN, DSW, DSE, DNE, DNW};
// W1: populations leaving through direction d (-1 = unused slot)
constexpr int PLANES[8][3] = {{1, 5, 8}, {2, 5, 6}, {3, 6, 7}, {4, 7, 8},
                              {5, -1, -1}, {6, -1, -1}, {7, -1, -1}, {8, -1, -1}};
constexpr int NPLANES[8] = {3, 3, 3, 3, 1, 1, 1, 1};

enum HaloMode : int { HALO_W1 = 1, HALO_WG = 2 };

// A rectangle of the sub-domain processed by one step launch, in work units
// (one-step kernels: x0/y0 in cells, wc = width in lanes' chunks, hr = rows;
//  two-step kernel: everything in tiles).
struct Rect {
    int x0, y0, wc, hr;
};

// W1 destination of one direction: value of plane slot i at edge position p
// -> p[i][pos * ps]   (own ghost ring, or a contiguous send buffer)
struct EdgeDst {
    float *p[3];
    int ps;
    int pad;
};

// WG destination of one direction: value of speed k at strip coordinates
// (a, b) -> base[k*ks + a*s1 + b*s2].  (a, b) = (strip column, row) for E/W,
// (strip row, column) for N/S, (strip row, strip column) for corners.
struct Dst2 {
    float *base;
    long long ks;
    int s1, s2;
};

// Average-velocity bookkeeping lives in device memory (ctl):
//   ctl[0] = steps whose block partials are pending (0, 1 or 2)
//   ctl[1] = next av_local index
//   ctl[2] = partials per pending step, ctl[3] = stride between steps
// Block 0 of every reducing launch folds the pending steps in a fixed order,
// so no host sync or extra launch is needed per step (and graphs replay it).

struct StepArgs {
    const float *fin;       // input lattice origin
    float *fout;            // output lattice origin
    const uint8_t *obst;    // uint8[h][w]
    long long plane;        // plane stride in floats
    int pitch;              // row stride in floats
    int w, h;               // sub-domain size
    int accel_row;          // local row carrying the folded acceleration, -1 if none
    float omega, omo, w1, w2;
    int nrect;
    int total;              // total tiles (BLOCK work items each) over all rects
    Rect rect[MAX_RECTS];
    int rect_begin[MAX_RECTS];  // first tile of each rect (INT_MAX when unused); a tile never spans rects
    EdgeDst dst[8];
    // average-velocity reduction
    float *partials_out;        // this launch writes partials_out[blockIdx.x]
    const float *partials_prev; // previous launch's block partials (reduced by block 0)
    float *av_local;            // per-step local sums of |u|
    int *ctl;
    int n_total, stride;        // written to ctl by the reducing launch's block 0
};

struct Step2Args {
    const float *fin;
    float *fout;
    const uint8_t *obst_g;  // ghosted obstacles, (y+1)*ogp + (x+1), -1 <= x <= w, -1 <= y <= h
    long long plane;
    int pitch, ogp;
    int w, h;
    int gy0, ny, accel_g;   // global row of local row 0, global ny, global accelerated row (-1: none)
    float omega, omo, w1, w2;
    int tile;               // Tile2 shape
    int nrect, total;       // rects in tile units; total tiles
    Rect rect[MAX_RECTS];
    int rect_begin[MAX_RECTS];
    Dst2 dst[8];
    float *partials_out;        // step s of this launch: partials_out[s*stride + blockIdx.x]
    const float *partials_prev;
    float *av_local;
    int *ctl;
    int n_total, stride;
};

// S-step streaming kernels (lbm_stream.hip, lbm_stream2.hip): a rect of
// output cells is cut into strips of ow columns (one wave each; ow = 64 - 2S
// with one column per lane, 128 - 2S or 126 - 2S with two) and segments of
// hs rows.
struct SRect {
    int x0, y0, w, h;   // output cells
    int nstrip, hs;     // strips across, rows per segment
    int ow;             // owned columns per strip
};

struct StreamArgs {
    const float *fin;
    float *fout;
    const uint8_t *obst_g;  // ghosted obstacles, (y+og)*ogp + (x+og)
    long long plane;
    int pitch, ogp, og;
    int w, h, xmax;         // xmax: last column inside the row allocation (>= w + gr + 1)
    int hw;                 // WG halo width of the dst tables (the engine's steps per launch; >= S of any launch)
    int gy0, ny, accel_g;
    float omega, omo, w1, w2;
    float tc0, tc1, tc2;    // LBM_FLAG_TOLERANCE collision: 4 omega / 9, omega / 9, omega / 36
    int nrect, total;       // total work units (strip x segment)
    SRect rect[MAX_SRECTS];
    int rect_begin[MAX_SRECTS];
    Dst2 dst[8];            // WG halo destinations, g = S
    const Dst2 *dstg;       // the same eight in device memory (read only where a halo cell is stored)
    const uint8_t *uobst;   // v3: per work unit, 1 = reads an obstacle cell (nullptr: every unit may)
    const int *uperm;       // v3: dispatch slot -> work unit (nullptr: identity)
    unsigned long long *trace;  // diagnostics (LBM_STREAM_TRACE): per unit {start, end} s_memrealtime, or null
    float *partials_out;    // step s of this launch: partials_out[s*stride + blockIdx.x]
    const float *partials_prev;
    float *av_local;
    int *ctl;
    int n_total, stride;
};

// Lattice-resident persistent kernel (lbm_resident.hip): tiles of RES_TW
// columns x RES_TH[variant] rows, one workgroup each, all co-resident; every
// step of a run in one launch.  Edge populations move between neighbouring
// tiles as 8-byte {value, tag} granules: halo[2][ntiles][8 dirs][3][RES_GW].
// v1 (scalar, one column per lane): 64-column tiles, any grid.  v2 (packed
// fp32, a column pair per lane): 128-column tiles, even nx only.
constexpr int RES_TW = 64;
constexpr int RES2_TW = 128;
// (v3, register-resident, and v4, AA-pattern LDS addressing, lost their A/B
// to v2 -- DESIGN.md section 4 -- and were removed in round 3.)
enum ResVariant : int {
    RES_64 = 0, RES_32 = 1, RES_16 = 2, RES_16x4 = 3, RES_8 = 4, RES_4 = 5,           // v1
    RES2_32 = 6, RES2_16 = 7, RES2_8 = 8, RES2_4 = 9, RES2_2 = 10,                    // v2
    RES2_16x8 = 11                                                                      // v2, 8 waves: 2 tiles per CU
};
// (v5, a two-cell ring with one hand-off per two steps, lost its A/B to v2 in
// round 4 -- 4.4 vs 4.0 us per step, DESIGN.md section 4.4,
// profiles/r04/res5/ -- and was removed from the sources in round 5.)
constexpr int NUM_RES = 12;
constexpr int RES_TH[NUM_RES] = {64, 32, 16, 16, 8, 4, 32, 16, 8, 4, 2, 16};
constexpr int RES_TWV[NUM_RES] = {64, 64, 64, 64, 64, 64, 128, 128, 128, 128, 128, 128};
constexpr int RES_VER[NUM_RES] = {1, 1, 1, 1, 1, 1, 2, 2, 2, 2, 2, 2};
// granule values per (tile, direction, position): three planes
constexpr int RES_GV[NUM_RES] = {3, 3, 3, 3, 3, 3, 3, 3, 3, 3, 3, 3};
constexpr int RES_GW = 128;  // granule positions per (tile, direction, plane), both versions

struct ResidentArgs {
    const float *fin;       // input lattice origin (interior read, ring from periodic images)
    float *fout;            // output lattice origin (interior written at the end)
    const uint8_t *obst;    // uint8[ny][nx]
    long long plane;
    int pitch;
    int nx, ny, tiles_x, tiles_y;
    int steps;
    unsigned tag0;          // granule tags of this run: tag0 + 1 .. tag0 + steps
    int accel_row;          // global row with the folded acceleration (-1: none)
    float omega, omo, w1, w2;
    float tc0, tc1, tc2;    // LBM_FLAG_TOLERANCE collision: 4 omega / 9, omega / 9, omega / 36
    unsigned long long *halo;
    float *partials;        // [steps][ntiles]
    int *status;            // set to 1 when a neighbour hand-off timed out
    long long timeout_ticks;  // wall-clock ticks a poll may wait
    long long *trace;       // LBM_RES_TRACE diagnostics: [step][5] wall-clock stamps of tile 0, wave 0 (or null)
    int trace_steps;
    unsigned long long *htrace;  // LBM_RES_TRACE=2: [step][tile][2] latest wave's collision end, ring ready
    int early_poll;         // v2: poll the ring after the first work item instead of after the last
    // LBM_DEBUG_RES_STALL_TILE / _STEP (debug knobs, tests/test_gpu_resident_recovery.py):
    // tile stall_tile leaves the step loop at step stall_step without publishing,
    // as a tile that never became resident would -- a deterministic residency failure
    int stall_tile, stall_step;
};

// Halo pack (edge -> dst) after load / accelerate, and unpack (recv -> ghost
// ring) after every exchange; both in either format.
struct HaloArgs {
    float *f;               // lattice origin
    long long plane;
    int pitch, w, h;
    unsigned mask;          // directions to process
    int mode;               // HALO_W1 / HALO_WG
    int g;                  // WG width
    EdgeDst dst[8];         // W1 pack destinations
    Dst2 dst2[8];           // WG pack destinations
    Dst2 ghost2[8];         // WG unpack: ghost region of side e
    const float *recv[8];   // unpack: receive buffer per direction
};

// message sizes (floats)
inline int edge_len(int d, int w, int h) { return d < 4 ? ((d & 1) ? w : h) : 1; }
inline long long msg_floats(int mode, int d, int w, int h, int g) {
    return mode == HALO_WG ? (d < 4 ? (long long)g * Q * edge_len(d, w, h) : (long long)g * g * Q)
                           : (long long)NPLANES[d] * edge_len(d, w, h);
}

}  // namespace lbm

// lbm_layout.hpp -- device data layout and kernel argument blocks shared by
// the HIP kernels (lbm_kernels.hip) and the engine (lbm_engine.hip).
//
// Lattice: SoA f[9][h+2][pitch] per sub-domain, one-cell ghost ring.
//   interior cell (x, y), 0<=x<w, 0<=y<h  ->  f[k*plane + (y+1)*pitch + XOFF + x]
//   ghost column x=-1 sits at XOFF-1, ghost column x=w at XOFF+w,
//   ghost rows y=-1 / y=h are rows 0 / h+1.
// XOFF = 4 keeps every interior row 16-byte aligned for float4 access
// (pitch and plane are multiples of 64 floats).
//
// Speeds (main/include/LatticeBoltzmannUtils.hpp:20-22):
//   0 M, 1 E(+1,0), 2 N(0,+1), 3 W(-1,0), 4 S(0,-1),
//   5 NE(+1,+1), 6 NW(-1,+1), 7 SW(-1,-1), 8 SE(+1,-1)
// Pull streaming: s_k(x,y) = f_old[k](x - cx_k, y - cy_k)   (LastChance.cpp:203-211)
//
// Halo directions d = 0..7 use the velocity of speed d+1: E, N, W, S, NE, NW, SW, SE.
// The populations that leave a sub-domain through direction d are the
// planes whose velocity has d's non-zero components (PLANES[d]); the
// receiving neighbour stores them in its ghost region on the opposite side.
#pragma once

#include <cstdint>

namespace lbm {

constexpr int Q = 9;
constexpr int XOFF = 4;
constexpr int BLOCK = 256;  // 4 wave64s
constexpr int MAX_RECTS = 4;

enum Dir : int { DE = 0, DN = 1, DW = 2, DS = 3, DNE = 4, DNW = 5, DSW = 6, DSE = 7 };

// d -> (dx, dy)
constexpr int DIR_X[8] = {1, 0, -1, 0, 1, -1, -1, 1};
constexpr int DIR_Y[8] = {0, 1, 0, -1, 1, 1, -1, -1};
constexpr int OPP_DIR[8] = {DW, DS, DE, DN, DSW, DSE, DNE, DNW};
// populations leaving through direction d (-1 = unused slot)
constexpr int PLANES[8][3] = {{1, 5, 8}, {2, 5, 6}, {3, 6, 7}, {4, 7, 8},
                              {5, -1, -1}, {6, -1, -1}, {7, -1, -1}, {8, -1, -1}};
constexpr int NPLANES[8] = {3, 3, 3, 3, 1, 1, 1, 1};

// A rectangle of the sub-domain processed by one step launch.
// x0/y0 in cells (local), wc = width in work items (chunks of VEC cells),
// hr = rows.
struct Rect {
    int x0, y0, wc, hr;
};

// Where the values of one halo direction go: either this lattice's own ghost
// ring (periodic wrap inside one sub-domain) or a contiguous send buffer.
// Value of plane slot i at edge position p  ->  p[i][pos * ps]
struct EdgeDst {
    float *p[3];
    int ps;
    int pad;
};

struct StepArgs {
    const float *fin;       // input lattice, plane 0 base
    float *fout;            // output lattice, plane 0 base
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
    const float *partials_prev; // previous step's block partials (reduced by block 0)
    int n_prev;
    float *av_local;            // per-step local sums of |u|
    int *ctl;                   // ctl[0] = previous step pending, ctl[1] = next av index
};

// Halo pack (edge -> dst) used after load / accelerate, and unpack
// (recv buffers -> ghost ring) used after every exchange.
struct HaloArgs {
    float *f;               // lattice, plane 0 base
    long long plane;
    int pitch, w, h;
    unsigned mask;          // directions to process
    EdgeDst dst[8];         // pack: destination per direction
    const float *recv[8];   // unpack: receive buffer per direction
};

}  // namespace lbm

// lbm_kernels.hip -- hand-written gfx950 kernels of the D2Q9-BGK hot path.
//
// One fused kernel per step does what the reference splits into
// accelerate_flow -> propagate -> rebound -> collision -> av_velocity
// (main/LastChance.cpp:185-266; IPU vertex LbmTimeStepVertex,
// main/codelets/D2Q9Codelets.cpp:94-191,226-268):
//   * pull-stream the nine populations from the ghosted SoA lattice,
//   * rebound on obstacle cells, BGK collision elsewhere,
//   * fold the acceleration into the outputs of row ny-2,
//   * accumulate |u| (pre-collision velocity) of fluid cells into a
//     deterministic per-block partial,
//   * write the outgoing edge populations either into the lattice's own ghost
//     ring (periodic wrap inside one sub-domain) or into the halo send
//     buffers (fused pack for the RCCL exchange).
// Block 0 of the reducing launch also sums the previous step's block partials
// into av_local (the reference's reduceWithOutput + AppendReducedSum +
// IncrementIndex, main/LbmAoS.cpp:25-93), so no extra launch or host sync is
// needed per step.
//
// Arithmetic is IEEE fp32 evaluated exactly as the reference writes it
// (compiled with -ffp-contract=off, correctly rounded division and sqrt), so
// the lattice is bitwise identical to the CPU oracle.
//
// This is a bandwidth-bound stencil (72 algorithmic bytes per cell update,
// ~1 flop/byte): no MFMA.  The SoA pull scheme reads every population exactly
// once, so there is no inter-cell reuse to stage in LDS; the +-1 column shift
// of six planes is resolved in registers by a cross-lane shuffle of the
// neighbouring lane's float4 instead (one exec-masked scalar load at each
// wave/row boundary).

#include <hip/hip_runtime.h>

#include <climits>
#include <cstdint>

#include "lbm_layout.hpp"

namespace lbm {

__device__ __forceinline__ float4 ld4(const float *p) { return *reinterpret_cast<const float4 *>(p); }
__device__ __forceinline__ void st4(float *p, float4 v) { *reinterpret_cast<float4 *>(p) = v; }

// Bijective XCD-aware block remap (blocks b and b+8 share an XCD): blocks on
// one XCD get consecutive logical ids, so neighbouring chunks -- which share
// the cache line at their boundary -- are fetched through one L2.
__device__ __forceinline__ int xcd_remap(int b, int nb) {
    const int xcd = b & 7;
    const int q = nb >> 3, r = nb & 7;
    const int start = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
    return start + (b >> 3);
}

// 256-thread block sum in a fixed order (result valid in thread 0).
__device__ __forceinline__ float block_sum(float v, float *lds) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    __syncthreads();
    if (lane == 0) lds[wid] = v;
    __syncthreads();
    float r = 0.f;
    if (threadIdx.x == 0) r = ((lds[0] + lds[1]) + lds[2]) + lds[3];
    return r;
}

// Block 0: fold the previous step's partials into av_local[ctl[1]++].
__device__ __forceinline__ void reduce_prev(const StepArgs &a, float *lds) {
    const int pending = a.ctl[0];
    if (!pending) return;
    float v = 0.f;
    for (int i = threadIdx.x; i < a.n_prev; i += BLOCK) v += a.partials_prev[i];
    const float s = block_sum(v, lds);
    if (threadIdx.x == 0) {
        const int idx = a.ctl[1];
        a.av_local[idx] = s;
        a.ctl[1] = idx + 1;
    }
    __syncthreads();
}

// Collision of one cell from its nine pulled populations; expression order is
// main/LastChance.cpp:226-262 verbatim.  Obstacle cells rebound
// (LastChance.cpp:213-223).  Returns |u| for fluid cells, 0 for obstacles.
__device__ __forceinline__ float collide(const float (&s)[Q], float (&o)[Q], bool obst, float accf,
                                         float omega, float omo, float w1, float w2) {
    const float rho = s[0] + s[1] + s[2] + s[3] + s[4] + s[5] + s[6] + s[7] + s[8];
    const float ux = (s[1] + s[5] + s[8] - (s[3] + s[6] + s[7])) / rho;
    const float uy = (s[2] + s[5] + s[6] - (s[4] + s[7] + s[8])) / rho;
    const float usq = ux * ux + uy * uy;
    const float csq = 1.00f - usq * 1.50f;
    const float ld0 = 4.00f / 9.00f * rho * omega;
    const float ld1 = rho / 9.00f * omega;
    const float ld2 = rho / 36.00f * omega;
    const float us = ux + uy;
    const float ud = -ux + uy;
    const float c0 = s[0] * omo + ld0 * csq;
    const float c1 = s[1] * omo + ld1 * ((4.50f * ux) * (2.00f / 3.00f + ux) + csq);
    const float c2 = s[2] * omo + ld1 * ((4.50f * uy) * (2.00f / 3.00f + uy) + csq);
    const float c3 = s[3] * omo + ld1 * ((-4.50f * ux) * (2.00f / 3.00f - ux) + csq);
    const float c4 = s[4] * omo + ld1 * ((-4.50f * uy) * (2.00f / 3.00f - uy) + csq);
    const float c5 = s[5] * omo + ld2 * ((4.50f * us) * (2.00f / 3.00f + us) + csq);
    const float c6 = s[6] * omo + ld2 * ((4.50f * ud) * (2.00f / 3.00f + ud) + csq);
    const float c7 = s[7] * omo + ld2 * ((-4.50f * us) * (2.00f / 3.00f - us) + csq);
    const float c8 = s[8] * omo + ld2 * ((-4.50f * ud) * (2.00f / 3.00f - ud) + csq);
    o[0] = obst ? s[0] : c0;
    o[1] = obst ? s[3] : c1 + accf * w1;
    o[2] = obst ? s[4] : c2;
    o[3] = obst ? s[1] : c3 - accf * w1;
    o[4] = obst ? s[2] : c4;
    o[5] = obst ? s[7] : c5 + accf * w2;
    o[6] = obst ? s[8] : c6 - accf * w2;
    o[7] = obst ? s[5] : c7 - accf * w2;
    o[8] = obst ? s[6] : c8 + accf * w2;
    return obst ? 0.f : sqrtf(usq);
}

struct RectPos {
    int x0, y, cxi, wc;
    bool active;
};

// Tile t (BLOCK work items, wave-uniform) -> rect; lane -> (column chunk, row).
// Every tile lies inside one rect, so the rect lookup stays scalar.
__device__ __forceinline__ RectPos locate(const StepArgs &a, int t, int tid) {
    int r = 0;
#pragma unroll
    for (int i = 1; i < MAX_RECTS; ++i) r = (t >= a.rect_begin[i]) ? i : r;
    r = __builtin_amdgcn_readfirstlane(r);
    const Rect R = a.rect[r];
    const int items = R.wc * R.hr;
    int lc = (t - a.rect_begin[r]) * BLOCK + tid;
    const bool active = lc < items;
    lc = active ? lc : items - 1;
    const int yy = lc / R.wc;
    const int cxi = lc - yy * R.wc;
    return RectPos{R.x0, R.y0 + yy, cxi, R.wc, active};
}

// --------------------------------------------------------------------------
// Fast path: 4 consecutive cells per lane, float4 loads/stores.
// Requires w % 4 == 0 and every rect aligned to 4 columns.
// --------------------------------------------------------------------------
template <bool kReduce>
__global__ __launch_bounds__(BLOCK) void step_vec4(StepArgs a) {
    __shared__ float lds[4];
    if (kReduce && blockIdx.x == 0) reduce_prev(a, lds);

    const int tid = threadIdx.x, lane = tid & 63;
    const long long P = a.plane;
    const int pitch = a.pitch;
    const int nb = gridDim.x;
    const int lb = xcd_remap(blockIdx.x, nb);
    float tot = 0.f;

    for (int t = lb; t < a.total; t += nb) {
        const RectPos rp = locate(a, t, tid);
        const bool active = rp.active;
        const int x0 = rp.x0 + 4 * rp.cxi;
        const int y = rp.y;
        const bool ldir = (lane == 0) || (rp.cxi == 0);
        const bool rdir = (lane == 63) || (rp.cxi == rp.wc - 1);

        const float *r0 = a.fin + (long long)(y + 1) * pitch + XOFF + x0;  // row y
        const float *rm = r0 - pitch;                                      // row y-1
        const float *rp1 = r0 + pitch;                                     // row y+1

        const float4 v0 = ld4(r0);
        const float4 v1 = ld4(r0 + 1 * P);
        const float4 v2 = ld4(rm + 2 * P);
        const float4 v3 = ld4(r0 + 3 * P);
        const float4 v4 = ld4(rp1 + 4 * P);
        const float4 v5 = ld4(rm + 5 * P);
        const float4 v6 = ld4(rm + 6 * P);
        const float4 v7 = ld4(rp1 + 7 * P);
        const float4 v8 = ld4(rp1 + 8 * P);
        const uint32_t ob = *reinterpret_cast<const uint32_t *>(a.obst + (long long)y * a.w + x0);

        float e1 = 0.f, e5 = 0.f, e8 = 0.f, e3 = 0.f, e6 = 0.f, e7 = 0.f;
        if (ldir) {
            e1 = r0[1 * P - 1];
            e5 = rm[5 * P - 1];
            e8 = rp1[8 * P - 1];
        }
        if (rdir) {
            e3 = r0[3 * P + 4];
            e6 = rm[6 * P + 4];
            e7 = rp1[7 * P + 4];
        }
        // x-1 neighbour of this lane's first cell = previous lane's last cell
        float l1 = __shfl_up(v1.w, 1, 64), l5 = __shfl_up(v5.w, 1, 64), l8 = __shfl_up(v8.w, 1, 64);
        // x+4 neighbour of this lane's last cell = next lane's first cell
        float q3 = __shfl_down(v3.x, 1, 64), q6 = __shfl_down(v6.x, 1, 64), q7 = __shfl_down(v7.x, 1, 64);
        l1 = ldir ? e1 : l1;
        l5 = ldir ? e5 : l5;
        l8 = ldir ? e8 : l8;
        q3 = rdir ? e3 : q3;
        q6 = rdir ? e6 : q6;
        q7 = rdir ? e7 : q7;

        const float accf = (y == a.accel_row) ? 1.00f : 0.00f;
        float o[4][Q];
        {
            const float s[Q] = {v0.x, l1, v2.x, v3.y, v4.x, l5, v6.y, v7.y, l8};
            const float u = collide(s, o[0], (ob & 0xffu) != 0, accf, a.omega, a.omo, a.w1, a.w2);
            if (active) tot += u;
        }
        {
            const float s[Q] = {v0.y, v1.x, v2.y, v3.z, v4.y, v5.x, v6.z, v7.z, v8.x};
            const float u = collide(s, o[1], (ob & 0xff00u) != 0, accf, a.omega, a.omo, a.w1, a.w2);
            if (active) tot += u;
        }
        {
            const float s[Q] = {v0.z, v1.y, v2.z, v3.w, v4.z, v5.y, v6.w, v7.w, v8.y};
            const float u = collide(s, o[2], (ob & 0xff0000u) != 0, accf, a.omega, a.omo, a.w1, a.w2);
            if (active) tot += u;
        }
        {
            const float s[Q] = {v0.w, v1.z, v2.w, q3, v4.w, v5.z, q6, q7, v8.z};
            const float u = collide(s, o[3], (ob & 0xff000000u) != 0, accf, a.omega, a.omo, a.w1, a.w2);
            if (active) tot += u;
        }

        if (active) {
            float *w0 = a.fout + (long long)(y + 1) * pitch + XOFF + x0;
#pragma unroll
            for (int k = 0; k < Q; ++k) st4(w0 + k * P, make_float4(o[0][k], o[1][k], o[2][k], o[3][k]));

            // ---- edge populations: own ghost ring or halo send buffers ----
            const bool east = (x0 + 3 == a.w - 1), west = (x0 == 0);
            const bool north = (y == a.h - 1), south = (y == 0);
            if (east) {
                const EdgeDst &d = a.dst[DE];
                d.p[0][y * d.ps] = o[3][1];
                d.p[1][y * d.ps] = o[3][5];
                d.p[2][y * d.ps] = o[3][8];
            }
            if (west) {
                const EdgeDst &d = a.dst[DW];
                d.p[0][y * d.ps] = o[0][3];
                d.p[1][y * d.ps] = o[0][6];
                d.p[2][y * d.ps] = o[0][7];
            }
            if (north) {
                const EdgeDst &d = a.dst[DN];
                st4(d.p[0] + x0, make_float4(o[0][2], o[1][2], o[2][2], o[3][2]));
                st4(d.p[1] + x0, make_float4(o[0][5], o[1][5], o[2][5], o[3][5]));
                st4(d.p[2] + x0, make_float4(o[0][6], o[1][6], o[2][6], o[3][6]));
                if (east) a.dst[DNE].p[0][0] = o[3][5];
                if (west) a.dst[DNW].p[0][0] = o[0][6];
            }
            if (south) {
                const EdgeDst &d = a.dst[DS];
                st4(d.p[0] + x0, make_float4(o[0][4], o[1][4], o[2][4], o[3][4]));
                st4(d.p[1] + x0, make_float4(o[0][7], o[1][7], o[2][7], o[3][7]));
                st4(d.p[2] + x0, make_float4(o[0][8], o[1][8], o[2][8], o[3][8]));
                if (west) a.dst[DSW].p[0][0] = o[0][7];
                if (east) a.dst[DSE].p[0][0] = o[3][8];
            }
        }
    }

    const float s = block_sum(tot, lds);
    if (threadIdx.x == 0) {
        a.partials_out[blockIdx.x] = s;
        if (kReduce && blockIdx.x == 0) a.ctl[0] = 1;
    }
}

// --------------------------------------------------------------------------
// General path: one cell per lane, any sub-domain width.
// --------------------------------------------------------------------------
template <bool kReduce>
__global__ __launch_bounds__(BLOCK) void step_scalar(StepArgs a) {
    __shared__ float lds[4];
    if (kReduce && blockIdx.x == 0) reduce_prev(a, lds);

    const int tid = threadIdx.x;
    const long long P = a.plane;
    const int pitch = a.pitch;
    const int nb = gridDim.x;
    const int lb = xcd_remap(blockIdx.x, nb);
    float tot = 0.f;

    for (int t = lb; t < a.total; t += nb) {
        const RectPos rp = locate(a, t, tid);
        if (!rp.active) continue;
        const int x = rp.x0 + rp.cxi;
        const int y = rp.y;
        const float *r0 = a.fin + (long long)(y + 1) * pitch + XOFF + x;
        const float *rm = r0 - pitch;
        const float *rp1 = r0 + pitch;
        const float s[Q] = {r0[0],         r0[1 * P - 1], rm[2 * P],     r0[3 * P + 1], rp1[4 * P],
                            rm[5 * P - 1], rm[6 * P + 1], rp1[7 * P + 1], rp1[8 * P - 1]};
        const bool obst = a.obst[(long long)y * a.w + x] != 0;
        const float accf = (y == a.accel_row) ? 1.00f : 0.00f;
        float o[Q];
        tot += collide(s, o, obst, accf, a.omega, a.omo, a.w1, a.w2);

        float *w0 = a.fout + (long long)(y + 1) * pitch + XOFF + x;
#pragma unroll
        for (int k = 0; k < Q; ++k) w0[k * P] = o[k];

        const bool east = (x == a.w - 1), west = (x == 0);
        const bool north = (y == a.h - 1), south = (y == 0);
        if (east) {
            const EdgeDst &d = a.dst[DE];
            d.p[0][y * d.ps] = o[1];
            d.p[1][y * d.ps] = o[5];
            d.p[2][y * d.ps] = o[8];
        }
        if (west) {
            const EdgeDst &d = a.dst[DW];
            d.p[0][y * d.ps] = o[3];
            d.p[1][y * d.ps] = o[6];
            d.p[2][y * d.ps] = o[7];
        }
        if (north) {
            const EdgeDst &d = a.dst[DN];
            d.p[0][x] = o[2];
            d.p[1][x] = o[5];
            d.p[2][x] = o[6];
            if (east) a.dst[DNE].p[0][0] = o[5];
            if (west) a.dst[DNW].p[0][0] = o[6];
        }
        if (south) {
            const EdgeDst &d = a.dst[DS];
            d.p[0][x] = o[4];
            d.p[1][x] = o[7];
            d.p[2][x] = o[8];
            if (west) a.dst[DSW].p[0][0] = o[7];
            if (east) a.dst[DSE].p[0][0] = o[8];
        }
    }

    const float s = block_sum(tot, lds);
    if (threadIdx.x == 0) {
        a.partials_out[blockIdx.x] = s;
        if (kReduce && blockIdx.x == 0) a.ctl[0] = 1;
    }
}

// Fold the last step's partials (end of a run).
__global__ __launch_bounds__(BLOCK) void finalize_av(const float *partials, int n, float *av_local, int *ctl) {
    __shared__ float lds[4];
    if (ctl[0] == 0) return;
    float v = 0.f;
    for (int i = threadIdx.x; i < n; i += BLOCK) v += partials[i];
    const float s = block_sum(v, lds);
    if (threadIdx.x == 0) {
        const int idx = ctl[1];
        av_local[idx] = s;
        ctl[1] = idx + 1;
        ctl[0] = 0;
    }
}

// One-time conditional accelerate of row `row` (LastChance.cpp:161-183,
// D2Q9Codelets.cpp:71-93).  In place on the current lattice.
__global__ __launch_bounds__(BLOCK) void accelerate_row(float *f, const uint8_t *obst, long long P, int pitch,
                                                       int w, int row, float w1, float w2) {
    const int x = blockIdx.x * BLOCK + threadIdx.x;
    if (x >= w) return;
    float *c = f + (long long)(row + 1) * pitch + XOFF + x;
    if (!obst[(long long)row * w + x] && (c[3 * P] - w1) > 0.f && (c[6 * P] - w2) > 0.f &&
        (c[7 * P] - w2) > 0.f) {
        c[1 * P] += w1;
        c[5 * P] += w2;
        c[8 * P] += w2;
        c[3 * P] -= w1;
        c[6 * P] -= w2;
        c[7 * P] -= w2;
    }
}

// Equilibrium at rest over the whole allocation, ghosts included
// (LatticeBoltzmannUtils.hpp:137-157).
__global__ __launch_bounds__(BLOCK) void init_equilibrium(float *f, long long P, float c0, float c1, float c2) {
    const long long i = (long long)blockIdx.x * BLOCK + threadIdx.x;
    if (i >= P) return;
    f[i] = c0;
    f[1 * P + i] = c1;
    f[2 * P + i] = c1;
    f[3 * P + i] = c1;
    f[4 * P + i] = c1;
    f[5 * P + i] = c2;
    f[6 * P + i] = c2;
    f[7 * P + i] = c2;
    f[8 * P + i] = c2;
}

// AoS [h][w][9] staging <-> SoA ghosted lattice.
__global__ __launch_bounds__(BLOCK) void aos_to_soa(const float *aos, float *f, long long P, int pitch, int w, int h) {
    const long long i = (long long)blockIdx.x * BLOCK + threadIdx.x;
    if (i >= (long long)w * h) return;
    const int y = (int)(i / w), x = (int)(i - (long long)y * w);
    float *d = f + (long long)(y + 1) * pitch + XOFF + x;
#pragma unroll
    for (int k = 0; k < Q; ++k) d[k * P] = aos[i * Q + k];
}

__global__ __launch_bounds__(BLOCK) void soa_to_aos(const float *f, float *aos, long long P, int pitch, int w, int h) {
    const long long i = (long long)blockIdx.x * BLOCK + threadIdx.x;
    if (i >= (long long)w * h) return;
    const int y = (int)(i / w), x = (int)(i - (long long)y * w);
    const float *s = f + (long long)(y + 1) * pitch + XOFF + x;
#pragma unroll
    for (int k = 0; k < Q; ++k) aos[i * Q + k] = s[k * P];
}

// Edge cell of direction d at edge position p (local coordinates).
__device__ __forceinline__ void edge_cell(int d, int p, int w, int h, int &x, int &y) {
    switch (d) {
        case DE: x = w - 1; y = p; break;
        case DW: x = 0; y = p; break;
        case DN: x = p; y = h - 1; break;
        case DS: x = p; y = 0; break;
        case DNE: x = w - 1; y = h - 1; break;
        case DNW: x = 0; y = h - 1; break;
        case DSW: x = 0; y = 0; break;
        default: x = w - 1; y = 0; break;  // DSE
    }
}

// Ghost cell of direction e at position p.
__device__ __forceinline__ void ghost_cell(int e, int p, int w, int h, int &x, int &y) {
    switch (e) {
        case DE: x = w; y = p; break;
        case DW: x = -1; y = p; break;
        case DN: x = p; y = h; break;
        case DS: x = p; y = -1; break;
        case DNE: x = w; y = h; break;
        case DNW: x = -1; y = h; break;
        case DSW: x = -1; y = -1; break;
        default: x = w; y = -1; break;  // DSE
    }
}

__device__ __forceinline__ int edge_len(int d, int w, int h) { return d < 4 ? ((d & 1) ? w : h) : 1; }

// Pack: the outgoing populations of every direction in `mask` from the
// current lattice to their destination (own ghost ring or send buffer).
// Grid: (ceil(max(w,h)/BLOCK), 8).
__global__ __launch_bounds__(BLOCK) void halo_pack(HaloArgs a) {
    const int d = blockIdx.y;
    if (!((a.mask >> d) & 1u)) return;
    const int p = blockIdx.x * BLOCK + threadIdx.x;
    if (p >= edge_len(d, a.w, a.h)) return;
    int x, y;
    edge_cell(d, p, a.w, a.h, x, y);
    const float *src = a.f + (long long)(y + 1) * a.pitch + XOFF + x;
    const EdgeDst &dst = a.dst[d];
    const int pos = d < 4 ? p : 0;
    for (int i = 0; i < 3; ++i) {
        const int k = PLANES[d][i];
        if (k < 0) break;
        dst.p[i][(long long)pos * dst.ps] = src[k * a.plane];
    }
}

// Unpack: receive buffer of direction e -> ghost region e (planes arriving
// from the neighbour on that side = PLANES[OPP_DIR[e]]).
__global__ __launch_bounds__(BLOCK) void halo_unpack(HaloArgs a) {
    const int e = blockIdx.y;
    if (!((a.mask >> e) & 1u)) return;
    const int p = blockIdx.x * BLOCK + threadIdx.x;
    const int len = edge_len(e, a.w, a.h);
    if (p >= len) return;
    int x, y;
    ghost_cell(e, p, a.w, a.h, x, y);
    float *g = a.f + (long long)(y + 1) * a.pitch + XOFF + x;
    const int od = OPP_DIR[e];
    for (int i = 0; i < 3; ++i) {
        const int k = PLANES[od][i];
        if (k < 0) break;
        g[k * a.plane] = a.recv[e][(long long)i * len + p];
    }
}

// ---- host-side launch wrappers (called from lbm_engine.hip) ---------------

hipError_t launch_step(const StepArgs &a, int blocks, bool vec4, bool reduce, hipStream_t s) {
    if (vec4) {
        if (reduce)
            hipLaunchKernelGGL(step_vec4<true>, dim3(blocks), dim3(BLOCK), 0, s, a);
        else
            hipLaunchKernelGGL(step_vec4<false>, dim3(blocks), dim3(BLOCK), 0, s, a);
    } else {
        if (reduce)
            hipLaunchKernelGGL(step_scalar<true>, dim3(blocks), dim3(BLOCK), 0, s, a);
        else
            hipLaunchKernelGGL(step_scalar<false>, dim3(blocks), dim3(BLOCK), 0, s, a);
    }
    return hipGetLastError();
}

hipError_t launch_finalize(const float *partials, int n, float *av_local, int *ctl, hipStream_t s) {
    hipLaunchKernelGGL(finalize_av, dim3(1), dim3(BLOCK), 0, s, partials, n, av_local, ctl);
    return hipGetLastError();
}

hipError_t launch_accelerate(float *f, const uint8_t *obst, long long P, int pitch, int w, int row, float w1,
                             float w2, hipStream_t s) {
    hipLaunchKernelGGL(accelerate_row, dim3((w + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, s, f, obst, P, pitch, w, row,
                       w1, w2);
    return hipGetLastError();
}

hipError_t launch_init_equilibrium(float *f, long long P, float c0, float c1, float c2, hipStream_t s) {
    hipLaunchKernelGGL(init_equilibrium, dim3((unsigned)((P + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, s, f, P, c0, c1,
                       c2);
    return hipGetLastError();
}

hipError_t launch_aos_to_soa(const float *aos, float *f, long long P, int pitch, int w, int h, hipStream_t s) {
    const long long n = (long long)w * h;
    hipLaunchKernelGGL(aos_to_soa, dim3((unsigned)((n + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, s, aos, f, P, pitch, w,
                       h);
    return hipGetLastError();
}

hipError_t launch_soa_to_aos(const float *f, float *aos, long long P, int pitch, int w, int h, hipStream_t s) {
    const long long n = (long long)w * h;
    hipLaunchKernelGGL(soa_to_aos, dim3((unsigned)((n + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, s, f, aos, P, pitch, w,
                       h);
    return hipGetLastError();
}

hipError_t launch_halo_pack(const HaloArgs &a, hipStream_t s) {
    const int m = a.w > a.h ? a.w : a.h;
    hipLaunchKernelGGL(halo_pack, dim3((m + BLOCK - 1) / BLOCK, 8), dim3(BLOCK), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_halo_unpack(const HaloArgs &a, hipStream_t s) {
    const int m = a.w > a.h ? a.w : a.h;
    hipLaunchKernelGGL(halo_unpack, dim3((m + BLOCK - 1) / BLOCK, 8), dim3(BLOCK), 0, s, a);
    return hipGetLastError();
}

}  // namespace lbm

// lbm_kernels.hip -- hand-written gfx950 kernels of the D2Q9-BGK hot path.
//
// The fused step does what the reference splits into
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
// Block 0 of the reducing launch also folds the previous launch's block
// partials into av_local (the reference's reduceWithOutput + AppendReducedSum
// + IncrementIndex, main/LbmAoS.cpp:25-93): no extra launch or host sync per
// step.
//
// Two one-step kernels live here:
//   step_vec4   4 consecutive cells per lane (float4 pulls, x+-1 shifts by
//               cross-lane shuffle) -- the fast path;
//   step_scalar one cell per lane, any width;
// lbm_step2.hip adds the fused two-step kernel.
//
// Arithmetic is IEEE fp32 evaluated exactly as the reference writes it
// (compiled with -ffp-contract=off, correctly rounded division and sqrt), so
// the lattice is bitwise identical to the CPU oracle.
//
// This is a bandwidth-bound stencil (72 algorithmic bytes per cell update,
// ~1 flop/byte): no MFMA.

#include <algorithm>

#include "lbm_device.hpp"

namespace lbm {

// --------------------------------------------------------------------------
// One step, 4 consecutive cells per lane, float4 loads/stores.
// Requires w % 4 == 0 and every rect aligned to 4 columns.  Macroscopic
// values per cell first, then each plane (or rebound pair) is finished and
// stored, so input and output registers retire early (no spills).
// --------------------------------------------------------------------------
template <bool kReduce>
__global__ __launch_bounds__(BLOCK) void step_vec4(StepArgs a) {
    __shared__ float lds[4];
    if (kReduce && blockIdx.x == 0) reduce_pending(a.ctl, a.partials_prev, a.av_local, lds);

    const int tid = threadIdx.x, lane = tid & 63;
    const long long P = a.plane;
    const int pitch = a.pitch;
    const int nb = gridDim.x;
    const int lb = xcd_remap(blockIdx.x, nb);
    float tot = 0.f;

    for (int t = lb; t < a.total; t += nb) {
        const RectPos rp = locate(a.rect, a.rect_begin, t, tid);
        const bool active = rp.active;
        const int x0 = rp.x0 + 4 * rp.cxi;
        const int y = rp.y;
        const bool ldir = (lane == 0) || (rp.cxi == 0);
        const bool rdir = (lane == 63) || (rp.cxi == rp.wc - 1);

        const float *r0 = a.fin + (long long)y * pitch + x0;  // row y
        const float *rm = r0 - pitch;                           // row y-1
        const float *rp1 = r0 + pitch;                          // row y+1

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
        const float S[Q][4] = {{v0.x, v0.y, v0.z, v0.w}, {l1, v1.x, v1.y, v1.z}, {v2.x, v2.y, v2.z, v2.w},
                               {v3.y, v3.z, v3.w, q3},   {v4.x, v4.y, v4.z, v4.w}, {l5, v5.x, v5.y, v5.z},
                               {v6.y, v6.z, v6.w, q6},   {v7.y, v7.z, v7.w, q7},   {l8, v8.x, v8.y, v8.z}};
        Macro m[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float s[Q] = {S[0][j], S[1][j], S[2][j], S[3][j], S[4][j], S[5][j], S[6][j], S[7][j], S[8][j]};
            m[j] = macro(s, ((ob >> (8 * j)) & 0xffu) != 0, a.omega);
            if (active) tot += m[j].u;
        }
        const float omo = a.omo, w1 = a.w1, w2 = a.w2, omega = a.omega;
        float *w0 = a.fout + (long long)y * pitch + x0;
        const bool east = (x0 + 3 == a.w - 1), west = (x0 == 0);
        const bool north = (y == a.h - 1), south = (y == 0);
        // rest
        {
            float o[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) o[j] = out0(S[0][j], m[j], omo, omega);
            if (active) st4(w0, make_float4(o[0], o[1], o[2], o[3]));
        }
        // E / W pair
        {
            float o1[4], o3[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) out13(S[1][j], S[3][j], m[j], omo, accf, w1, o1[j], o3[j]);
            if (active) {
                st4(w0 + 1 * P, make_float4(o1[0], o1[1], o1[2], o1[3]));
                st4(w0 + 3 * P, make_float4(o3[0], o3[1], o3[2], o3[3]));
                if (east) a.dst[DE].p[0][(long long)y * a.dst[DE].ps] = o1[3];
                if (west) a.dst[DW].p[0][(long long)y * a.dst[DW].ps] = o3[0];
            }
        }
        // N / S pair
        {
            float o2[4], o4[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) out24(S[2][j], S[4][j], m[j], omo, o2[j], o4[j]);
            const float4 k2 = make_float4(o2[0], o2[1], o2[2], o2[3]);
            const float4 k4 = make_float4(o4[0], o4[1], o4[2], o4[3]);
            if (active) {
                st4(w0 + 2 * P, k2);
                st4(w0 + 4 * P, k4);
                if (north) st4(a.dst[DN].p[0] + x0, k2);
                if (south) st4(a.dst[DS].p[0] + x0, k4);
            }
        }
        // NE / SW pair
        {
            float o5[4], o7[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) out57(S[5][j], S[7][j], m[j], omo, accf, w2, o5[j], o7[j]);
            const float4 k5 = make_float4(o5[0], o5[1], o5[2], o5[3]);
            const float4 k7 = make_float4(o7[0], o7[1], o7[2], o7[3]);
            if (active) {
                st4(w0 + 5 * P, k5);
                st4(w0 + 7 * P, k7);
                if (east) a.dst[DE].p[1][(long long)y * a.dst[DE].ps] = o5[3];
                if (west) a.dst[DW].p[2][(long long)y * a.dst[DW].ps] = o7[0];
                if (north) {
                    st4(a.dst[DN].p[1] + x0, k5);
                    if (east) a.dst[DNE].p[0][0] = o5[3];
                }
                if (south) {
                    st4(a.dst[DS].p[1] + x0, k7);
                    if (west) a.dst[DSW].p[0][0] = o7[0];
                }
            }
        }
        // NW / SE pair
        {
            float o6[4], o8[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) out68(S[6][j], S[8][j], m[j], omo, accf, w2, o6[j], o8[j]);
            const float4 k6 = make_float4(o6[0], o6[1], o6[2], o6[3]);
            const float4 k8 = make_float4(o8[0], o8[1], o8[2], o8[3]);
            if (active) {
                st4(w0 + 6 * P, k6);
                st4(w0 + 8 * P, k8);
                if (east) a.dst[DE].p[2][(long long)y * a.dst[DE].ps] = o8[3];
                if (west) a.dst[DW].p[1][(long long)y * a.dst[DW].ps] = o6[0];
                if (north) {
                    st4(a.dst[DN].p[2] + x0, k6);
                    if (west) a.dst[DNW].p[0][0] = o6[0];
                }
                if (south) {
                    st4(a.dst[DS].p[2] + x0, k8);
                    if (east) a.dst[DSE].p[0][0] = o8[3];
                }
            }
        }
    }

    const float s = block_sum(tot, lds);
    if (threadIdx.x == 0) {
        a.partials_out[blockIdx.x] = s;
        if (kReduce && blockIdx.x == 0) publish_pending(a.ctl, 1, a.n_total, a.stride);
    }
}

// --------------------------------------------------------------------------
// One step, one cell per lane, any sub-domain width.
// --------------------------------------------------------------------------
template <bool kReduce>
__global__ __launch_bounds__(BLOCK) void step_scalar(StepArgs a) {
    __shared__ float lds[4];
    if (kReduce && blockIdx.x == 0) reduce_pending(a.ctl, a.partials_prev, a.av_local, lds);

    const int tid = threadIdx.x;
    const long long P = a.plane;
    const int pitch = a.pitch;
    const int nb = gridDim.x;
    const int lb = xcd_remap(blockIdx.x, nb);
    float tot = 0.f;

    for (int t = lb; t < a.total; t += nb) {
        const RectPos rp = locate(a.rect, a.rect_begin, t, tid);
        if (!rp.active) continue;
        const int x = rp.x0 + rp.cxi;
        const int y = rp.y;
        const float *r0 = a.fin + (long long)y * pitch + x;
        const float *rm = r0 - pitch;
        const float *rp1 = r0 + pitch;
        const float s[Q] = {r0[0],         r0[1 * P - 1], rm[2 * P],     r0[3 * P + 1], rp1[4 * P],
                            rm[5 * P - 1], rm[6 * P + 1], rp1[7 * P + 1], rp1[8 * P - 1]};
        const bool obst = a.obst[(long long)y * a.w + x] != 0;
        const float accf = (y == a.accel_row) ? 1.00f : 0.00f;
        float o[Q];
        tot += collide(s, o, obst, accf, a.omega, a.omo, a.w1, a.w2);

        float *w0 = a.fout + (long long)y * pitch + x;
#pragma unroll
        for (int k = 0; k < Q; ++k) w0[k * P] = o[k];

        const bool east = (x == a.w - 1), west = (x == 0);
        const bool north = (y == a.h - 1), south = (y == 0);
        if (east) {
            const EdgeDst &d = a.dst[DE];
            d.p[0][(long long)y * d.ps] = o[1];
            d.p[1][(long long)y * d.ps] = o[5];
            d.p[2][(long long)y * d.ps] = o[8];
        }
        if (west) {
            const EdgeDst &d = a.dst[DW];
            d.p[0][(long long)y * d.ps] = o[3];
            d.p[1][(long long)y * d.ps] = o[6];
            d.p[2][(long long)y * d.ps] = o[7];
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
        if (kReduce && blockIdx.x == 0) publish_pending(a.ctl, 1, a.n_total, a.stride);
    }
}

// Fold the last launch's pending partials (end of a run).
__global__ __launch_bounds__(BLOCK) void finalize_av(const float *partials, float *av_local, int *ctl) {
    __shared__ float lds[4];
    reduce_pending(ctl, partials, av_local, lds);
    if (threadIdx.x == 0) ctl[0] = 0;
}

// One-time conditional accelerate of row `row` (LastChance.cpp:161-183,
// D2Q9Codelets.cpp:71-93).  In place on the current lattice (origin f).
__global__ __launch_bounds__(BLOCK) void accelerate_row(float *f, const uint8_t *obst, long long P, int pitch,
                                                       int w, int row, float w1, float w2) {
    const int x = blockIdx.x * BLOCK + threadIdx.x;
    if (x >= w) return;
    float *c = f + (long long)row * pitch + x;
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

// Equilibrium at rest over every row of the allocation, ghosts included
// (LatticeBoltzmannUtils.hpp:137-157).  base = allocation start, rf = floats
// per plane row.
__global__ __launch_bounds__(BLOCK) void init_equilibrium(float *base, long long rows, int rf, int pitch, long long P,
                                                         float c0, float c1, float c2) {
    const long long i = (long long)blockIdx.x * BLOCK + threadIdx.x;
    if (i >= rows * rf) return;
    const long long r = i / rf, x = i - r * rf;
    float *d = base + r * pitch + x;
    d[0] = c0;
    d[1 * P] = c1;
    d[2 * P] = c1;
    d[3 * P] = c1;
    d[4 * P] = c1;
    d[5 * P] = c2;
    d[6 * P] = c2;
    d[7 * P] = c2;
    d[8 * P] = c2;
}

// AoS [h][w][9] staging <-> SoA ghosted lattice (origin f).
__global__ __launch_bounds__(BLOCK) void aos_to_soa(const float *aos, float *f, long long P, int pitch, int w, int h) {
    const long long i = (long long)blockIdx.x * BLOCK + threadIdx.x;
    if (i >= (long long)w * h) return;
    const int y = (int)(i / w), x = (int)(i - (long long)y * w);
    float *d = f + (long long)y * pitch + x;
#pragma unroll
    for (int k = 0; k < Q; ++k) d[k * P] = aos[i * Q + k];
}

// LBM_NAN_CHECK / lbm_nonfinite_count: populations of the w x h interior
// that are NaN or +-Inf (SURVEY §5 "NaN scan of f in debug mode").  One
// 64-bit atomic per block that found any.
__global__ __launch_bounds__(BLOCK) void count_nonfinite(const float *f, long long P, int pitch, int w, int h,
                                                         unsigned long long *out) {
    __shared__ unsigned blk;
    if (threadIdx.x == 0) blk = 0;
    __syncthreads();
    const long long n = (long long)w * h;
    unsigned mine = 0;
    for (long long i = (long long)blockIdx.x * BLOCK + threadIdx.x; i < n; i += (long long)gridDim.x * BLOCK) {
        const long long y = i / w, x = i - y * w;
        const float *c = f + y * pitch + x;
#pragma unroll
        for (int k = 0; k < Q; ++k) mine += __builtin_isfinite(c[k * P]) ? 0u : 1u;
    }
    if (mine) atomicAdd(&blk, mine);
    __syncthreads();
    if (threadIdx.x == 0 && blk) atomicAdd(out, (unsigned long long)blk);
}

__global__ __launch_bounds__(BLOCK) void soa_to_aos(const float *f, float *aos, long long P, int pitch, int w, int h) {
    const long long i = (long long)blockIdx.x * BLOCK + threadIdx.x;
    if (i >= (long long)w * h) return;
    const int y = (int)(i / w), x = (int)(i - (long long)y * w);
    const float *s = f + (long long)y * pitch + x;
#pragma unroll
    for (int k = 0; k < Q; ++k) aos[i * Q + k] = s[k * P];
}

// W1: edge cell of direction d at edge position p; ghost cell of side e.
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

// WG: strip cell (a, b) of direction d (width g) -> cell coordinates.
__device__ __forceinline__ void strip_cell(int d, int a, int b, int w, int h, int g, int &x, int &y) {
    switch (d) {
        case DE: x = w - g + a; y = b; break;
        case DW: x = a; y = b; break;
        case DN: x = b; y = h - g + a; break;
        case DS: x = b; y = a; break;
        case DNE: x = w - g + b; y = h - g + a; break;
        case DNW: x = b; y = h - g + a; break;
        case DSW: x = b; y = a; break;
        default: x = w - g + b; y = a; break;  // DSE
    }
}

__device__ __forceinline__ int dev_edge_len(int d, int w, int h) { return d < 4 ? ((d & 1) ? w : h) : 1; }

// Pack the outgoing halo of every direction in `mask` from the current
// lattice to its destination (own ghost ring or send buffer).
// Grid: (ceil(max(3, g)*max(w,h)/BLOCK), 8).
__global__ __launch_bounds__(BLOCK) void halo_pack(HaloArgs a) {
    const int d = blockIdx.y;
    if (!((a.mask >> d) & 1u)) return;
    const int i = blockIdx.x * BLOCK + threadIdx.x;
    if (a.mode == HALO_W1) {
        if (i >= dev_edge_len(d, a.w, a.h)) return;
        int x, y;
        edge_cell(d, i, a.w, a.h, x, y);
        const float *src = a.f + (long long)y * a.pitch + x;
        const EdgeDst &dst = a.dst[d];
        const int pos = d < 4 ? i : 0;
        for (int s = 0; s < 3; ++s) {
            const int k = PLANES[d][s];
            if (k < 0) break;
            dst.p[s][(long long)pos * dst.ps] = src[k * a.plane];
        }
    } else {
        const int len = d < 4 ? dev_edge_len(d, a.w, a.h) : a.g;
        if (i >= a.g * len) return;
        const int sa = i / len, sb = i - sa * len;
        int x, y;
        strip_cell(d, sa, sb, a.w, a.h, a.g, x, y);
        const float *src = a.f + (long long)y * a.pitch + x;
        const Dst2 &dst = a.dst2[d];
        float *o = dst.base + (long long)sa * dst.s1 + (long long)sb * dst.s2;
#pragma unroll
        for (int k = 0; k < Q; ++k) o[k * dst.ks] = src[k * a.plane];
    }
}

// Unpack: receive buffer of side e -> ghost region e.
__global__ __launch_bounds__(BLOCK) void halo_unpack(HaloArgs a) {
    const int e = blockIdx.y;
    if (!((a.mask >> e) & 1u)) return;
    const int i = blockIdx.x * BLOCK + threadIdx.x;
    if (a.mode == HALO_W1) {
        const int len = dev_edge_len(e, a.w, a.h);
        if (i >= len) return;
        int x, y;
        ghost_cell(e, i, a.w, a.h, x, y);
        float *g = a.f + (long long)y * a.pitch + x;
        const int od = OPP_DIR[e];  // populations arriving from side e left the neighbour through OPP(e)
        for (int s = 0; s < 3; ++s) {
            const int k = PLANES[od][s];
            if (k < 0) break;
            g[k * a.plane] = a.recv[e][(long long)s * len + i];
        }
    } else {
        // the neighbour on side e sent its strip of direction OPP(e), laid out
        // [9][g][len] (edges) or [9][g][g] (corners)
        const int len = e < 4 ? dev_edge_len(e, a.w, a.h) : a.g;
        if (i >= a.g * len) return;
        const int sa = i / len, sb = i - sa * len;
        const Dst2 &g = a.ghost2[e];
        float *o = g.base + (long long)sa * g.s1 + (long long)sb * g.s2;
        const float *r = a.recv[e] + (long long)sa * len + sb;
#pragma unroll
        for (int k = 0; k < Q; ++k) o[k * g.ks] = r[(long long)k * a.g * len];
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

// Debug-only stall (LBM_DEBUG_DELAY_*, engines' ordering regression tests):
// one lane spins on the 100 MHz constant clock for `ticks` ticks.  Queued on
// one sub-domain's stream it holds that stream back while the other
// sub-domains run ahead, which makes a missing cross-stream wait show every
// time instead of once in a few hundred runs.
__global__ void debug_spin(long long ticks) {
    const long long end = (long long)wall_clock64() + ticks;
    while ((long long)wall_clock64() < end) __builtin_amdgcn_s_sleep(8);
}

hipError_t launch_debug_spin(int microseconds, hipStream_t s) {
    if (microseconds <= 0) return hipSuccess;
    hipLaunchKernelGGL(debug_spin, dim3(1), dim3(1), 0, s, (long long)microseconds * 100);
    return hipGetLastError();
}

hipError_t launch_finalize(const float *partials, float *av_local, int *ctl, hipStream_t s) {
    hipLaunchKernelGGL(finalize_av, dim3(1), dim3(BLOCK), 0, s, partials, av_local, ctl);
    return hipGetLastError();
}

hipError_t launch_accelerate(float *f, const uint8_t *obst, long long P, int pitch, int w, int row, float w1,
                             float w2, hipStream_t s) {
    hipLaunchKernelGGL(accelerate_row, dim3((w + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, s, f, obst, P, pitch, w, row,
                       w1, w2);
    return hipGetLastError();
}

hipError_t launch_init_equilibrium(float *base, long long rows, int rf, int pitch, long long P, float c0, float c1,
                                   float c2, hipStream_t s) {
    const long long n = rows * rf;
    hipLaunchKernelGGL(init_equilibrium, dim3((unsigned)((n + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, s, base, rows,
                       rf, pitch, P, c0, c1, c2);
    return hipGetLastError();
}

hipError_t launch_count_nonfinite(const float *f, long long P, int pitch, int w, int h, unsigned long long *out,
                                  hipStream_t s) {
    const long long n = (long long)w * h;
    const unsigned blocks = (unsigned)std::min<long long>(4096, (n + BLOCK - 1) / BLOCK);
    hipLaunchKernelGGL(count_nonfinite, dim3(std::max(blocks, 1u)), dim3(BLOCK), 0, s, f, P, pitch, w, h, out);
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
    const int m = (a.g > 3 ? a.g : 3) * (a.w > a.h ? a.w : a.h);
    hipLaunchKernelGGL(halo_pack, dim3((m + BLOCK - 1) / BLOCK, 8), dim3(BLOCK), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_halo_unpack(const HaloArgs &a, hipStream_t s) {
    const int m = (a.g > 3 ? a.g : 3) * (a.w > a.h ? a.w : a.h);
    hipLaunchKernelGGL(halo_unpack, dim3((m + BLOCK - 1) / BLOCK, 8), dim3(BLOCK), 0, s, a);
    return hipGetLastError();
}

}  // namespace lbm

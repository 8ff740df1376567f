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

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float4 ld4(const float *p) { return *reinterpret_cast<const float4 *>(p); }
__device__ __forceinline__ void st4(float *p, float4 v) { *reinterpret_cast<float4 *>(p) = v; }

// Streaming (non-temporal) variants: the lattice is touched once per step
// and is far larger than L2 / the Infinity Cache at the roofline sizes.
template <bool kNT>
__device__ __forceinline__ float4 ld4s(const float *p) {
    if constexpr (kNT) {
        const f32x4 v = __builtin_nontemporal_load(reinterpret_cast<const f32x4 *>(p));
        return make_float4(v.x, v.y, v.z, v.w);
    } else {
        return ld4(p);
    }
}
template <bool kNT>
__device__ __forceinline__ void st4s(float *p, float4 v) {
    if constexpr (kNT) {
        f32x4 u = {v.x, v.y, v.z, v.w};
        __builtin_nontemporal_store(u, reinterpret_cast<f32x4 *>(p));
    } else {
        st4(p, v);
    }
}

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

// Sum n block partials in a fixed order (depends on n only): float4 loads,
// four independent accumulators per thread so the loads overlap, then the
// block tree.  Result valid in thread 0.
__device__ __forceinline__ float sum_partials(const float *p, int n, float *lds) {
    const int n4 = n >> 2;
    const float4 *p4 = reinterpret_cast<const float4 *>(p);
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    int i = threadIdx.x;
    for (; i + 3 * BLOCK < n4; i += 4 * BLOCK) {
        const float4 x0 = p4[i], x1 = p4[i + BLOCK], x2 = p4[i + 2 * BLOCK], x3 = p4[i + 3 * BLOCK];
        a0 += (x0.x + x0.y) + (x0.z + x0.w);
        a1 += (x1.x + x1.y) + (x1.z + x1.w);
        a2 += (x2.x + x2.y) + (x2.z + x2.w);
        a3 += (x3.x + x3.y) + (x3.z + x3.w);
    }
    for (; i < n4; i += BLOCK) {
        const float4 x0 = p4[i];
        a0 += (x0.x + x0.y) + (x0.z + x0.w);
    }
    for (int k = 4 * n4 + threadIdx.x; k < n; k += BLOCK) a1 += p[k];
    return block_sum((a0 + a1) + (a2 + a3), lds);
}

// Block 0: fold the previous step's partials into av_local[ctl[1]++].
__device__ __forceinline__ void reduce_prev(const StepArgs &a, float *lds) {
    const int pending = a.ctl[0];
    if (!pending) return;
    const float s = sum_partials(a.partials_prev, a.n_prev, lds);
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
// kFlags: bit 0 = non-temporal stores, bit 1 = non-temporal loads.
// kMinWaves: occupancy request (waves per SIMD) passed to the register allocator.
template <bool kReduce, int kFlags, int kMinWaves>
__global__ __launch_bounds__(BLOCK, kMinWaves) void step_vec4(StepArgs a) {
    constexpr bool kNTS = (kFlags & 1) != 0;
    constexpr bool kNTL = (kFlags & 2) != 0;
    constexpr bool kPlaneOrder = (kFlags & 4) != 0;
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

        const float4 v0 = ld4s<kNTL>(r0);
        const float4 v1 = ld4s<kNTL>(r0 + 1 * P);
        const float4 v2 = ld4s<kNTL>(rm + 2 * P);
        const float4 v3 = ld4s<kNTL>(r0 + 3 * P);
        const float4 v4 = ld4s<kNTL>(rp1 + 4 * P);
        const float4 v5 = ld4s<kNTL>(rm + 5 * P);
        const float4 v6 = ld4s<kNTL>(rm + 6 * P);
        const float4 v7 = ld4s<kNTL>(rp1 + 7 * P);
        const float4 v8 = ld4s<kNTL>(rp1 + 8 * P);
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
        if constexpr (kPlaneOrder) {
            // Macroscopic values per cell first, then each plane (or rebound
            // pair) is finished and stored, so inputs and outputs retire early.
            const float S[Q][4] = {{v0.x, v0.y, v0.z, v0.w}, {l1, v1.x, v1.y, v1.z}, {v2.x, v2.y, v2.z, v2.w},
                                   {v3.y, v3.z, v3.w, q3},   {v4.x, v4.y, v4.z, v4.w}, {l5, v5.x, v5.y, v5.z},
                                   {v6.y, v6.z, v6.w, q6},   {v7.y, v7.z, v7.w, q7},   {l8, v8.x, v8.y, v8.z}};
            float rho[4], ux[4], uy[4], csq[4], ld1[4], ld2[4];
            bool obf[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                obf[j] = ((ob >> (8 * j)) & 0xffu) != 0;
                rho[j] = S[0][j] + S[1][j] + S[2][j] + S[3][j] + S[4][j] + S[5][j] + S[6][j] + S[7][j] + S[8][j];
                ux[j] = (S[1][j] + S[5][j] + S[8][j] - (S[3][j] + S[6][j] + S[7][j])) / rho[j];
                uy[j] = (S[2][j] + S[5][j] + S[6][j] - (S[4][j] + S[7][j] + S[8][j])) / rho[j];
                const float usq = ux[j] * ux[j] + uy[j] * uy[j];
                csq[j] = 1.00f - usq * 1.50f;
                ld1[j] = rho[j] / 9.00f * a.omega;
                ld2[j] = rho[j] / 36.00f * a.omega;
                const float u = obf[j] ? 0.f : sqrtf(usq);
                if (active) tot += u;
            }
            const float omo = a.omo, w1 = a.w1, w2 = a.w2;
            float *w0 = a.fout + (long long)(y + 1) * pitch + XOFF + x0;
            const bool east = (x0 + 3 == a.w - 1), west = (x0 == 0);
            const bool north = (y == a.h - 1), south = (y == 0);
            float4 ok;
            // plane 0
            {
                float o[4];
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    o[j] = obf[j] ? S[0][j] : S[0][j] * omo + 4.00f / 9.00f * rho[j] * a.omega * csq[j];
                ok = make_float4(o[0], o[1], o[2], o[3]);
                if (active) st4s<kNTS>(w0, ok);
            }
            // E / W pair
            {
                float o1[4], o3[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const float c1 = S[1][j] * omo + ld1[j] * ((4.50f * ux[j]) * (2.00f / 3.00f + ux[j]) + csq[j]);
                    const float c3 = S[3][j] * omo + ld1[j] * ((-4.50f * ux[j]) * (2.00f / 3.00f - ux[j]) + csq[j]);
                    o1[j] = obf[j] ? S[3][j] : c1 + accf * w1;
                    o3[j] = obf[j] ? S[1][j] : c3 - accf * w1;
                }
                if (active) {
                    st4s<kNTS>(w0 + 1 * P, make_float4(o1[0], o1[1], o1[2], o1[3]));
                    st4s<kNTS>(w0 + 3 * P, make_float4(o3[0], o3[1], o3[2], o3[3]));
                    if (east) a.dst[DE].p[0][y * a.dst[DE].ps] = o1[3];
                    if (west) a.dst[DW].p[0][y * a.dst[DW].ps] = o3[0];
                }
            }
            // N / S pair
            {
                float o2[4], o4[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const float c2 = S[2][j] * omo + ld1[j] * ((4.50f * uy[j]) * (2.00f / 3.00f + uy[j]) + csq[j]);
                    const float c4 = S[4][j] * omo + ld1[j] * ((-4.50f * uy[j]) * (2.00f / 3.00f - uy[j]) + csq[j]);
                    o2[j] = obf[j] ? S[4][j] : c2;
                    o4[j] = obf[j] ? S[2][j] : c4;
                }
                const float4 k2 = make_float4(o2[0], o2[1], o2[2], o2[3]);
                const float4 k4 = make_float4(o4[0], o4[1], o4[2], o4[3]);
                if (active) {
                    st4s<kNTS>(w0 + 2 * P, k2);
                    st4s<kNTS>(w0 + 4 * P, k4);
                    if (north) st4(a.dst[DN].p[0] + x0, k2);
                    if (south) st4(a.dst[DS].p[0] + x0, k4);
                }
            }
            // NE / SW pair
            {
                float o5[4], o7[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const float us = ux[j] + uy[j];
                    const float c5 = S[5][j] * omo + ld2[j] * ((4.50f * us) * (2.00f / 3.00f + us) + csq[j]);
                    const float c7 = S[7][j] * omo + ld2[j] * ((-4.50f * us) * (2.00f / 3.00f - us) + csq[j]);
                    o5[j] = obf[j] ? S[7][j] : c5 + accf * w2;
                    o7[j] = obf[j] ? S[5][j] : c7 - accf * w2;
                }
                const float4 k5 = make_float4(o5[0], o5[1], o5[2], o5[3]);
                const float4 k7 = make_float4(o7[0], o7[1], o7[2], o7[3]);
                if (active) {
                    st4s<kNTS>(w0 + 5 * P, k5);
                    st4s<kNTS>(w0 + 7 * P, k7);
                    if (east) a.dst[DE].p[1][y * a.dst[DE].ps] = o5[3];
                    if (west) a.dst[DW].p[2][y * a.dst[DW].ps] = o7[0];
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
                for (int j = 0; j < 4; ++j) {
                    const float ud = -ux[j] + uy[j];
                    const float c6 = S[6][j] * omo + ld2[j] * ((4.50f * ud) * (2.00f / 3.00f + ud) + csq[j]);
                    const float c8 = S[8][j] * omo + ld2[j] * ((-4.50f * ud) * (2.00f / 3.00f - ud) + csq[j]);
                    o6[j] = obf[j] ? S[8][j] : c6 - accf * w2;
                    o8[j] = obf[j] ? S[6][j] : c8 + accf * w2;
                }
                const float4 k6 = make_float4(o6[0], o6[1], o6[2], o6[3]);
                const float4 k8 = make_float4(o8[0], o8[1], o8[2], o8[3]);
                if (active) {
                    st4s<kNTS>(w0 + 6 * P, k6);
                    st4s<kNTS>(w0 + 8 * P, k8);
                    if (east) a.dst[DE].p[2][y * a.dst[DE].ps] = o8[3];
                    if (west) a.dst[DW].p[1][y * a.dst[DW].ps] = o6[0];
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
            (void)ok;
        } else {
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
                for (int k = 0; k < Q; ++k) st4s<kNTS>(w0 + k * P, make_float4(o[0][k], o[1][k], o[2][k], o[3][k]));

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
    const float s = sum_partials(partials, n, lds);
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

// Equilibrium at rest over every row of the allocation, ghosts included
// (LatticeBoltzmannUtils.hpp:137-157).  rf = floats per plane row.
__global__ __launch_bounds__(BLOCK) void init_equilibrium(float *f, long long rows, int rf, int pitch, long long P,
                                                         float c0, float c1, float c2) {
    const long long i = (long long)blockIdx.x * BLOCK + threadIdx.x;
    if (i >= rows * rf) return;
    const long long r = i / rf, x = i - r * rf;
    float *d = f + r * pitch + x;
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

template <bool R, int F>
static void launch_vec4_w(const StepArgs &a, int blocks, int min_waves, hipStream_t s) {
    switch (min_waves) {
        case 5: hipLaunchKernelGGL((step_vec4<R, F, 5>), dim3(blocks), dim3(BLOCK), 0, s, a); break;
        case 6: hipLaunchKernelGGL((step_vec4<R, F, 6>), dim3(blocks), dim3(BLOCK), 0, s, a); break;
        default: hipLaunchKernelGGL((step_vec4<R, F, 1>), dim3(blocks), dim3(BLOCK), 0, s, a); break;
    }
}

template <bool R>
static void launch_vec4_f(const StepArgs &a, int blocks, int flags, int min_waves, hipStream_t s) {
    switch (flags & 7) {
        case 1: launch_vec4_w<R, 1>(a, blocks, min_waves, s); break;
        case 2: launch_vec4_w<R, 2>(a, blocks, min_waves, s); break;
        case 3: launch_vec4_w<R, 3>(a, blocks, min_waves, s); break;
        case 4: launch_vec4_w<R, 4>(a, blocks, min_waves, s); break;
        case 5: launch_vec4_w<R, 5>(a, blocks, min_waves, s); break;
        case 6: launch_vec4_w<R, 6>(a, blocks, min_waves, s); break;
        case 7: launch_vec4_w<R, 7>(a, blocks, min_waves, s); break;
        default: launch_vec4_w<R, 0>(a, blocks, min_waves, s); break;
    }
}

hipError_t launch_step(const StepArgs &a, int blocks, bool vec4, bool reduce, int flags, int min_waves,
                       hipStream_t s) {
    if (vec4) {
        if (reduce)
            launch_vec4_f<true>(a, blocks, flags, min_waves, s);
        else
            launch_vec4_f<false>(a, blocks, flags, min_waves, s);
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

hipError_t launch_init_equilibrium(float *f, long long rows, int rf, int pitch, long long P, float c0, float c1,
                                   float c2, hipStream_t s) {
    const long long n = rows * rf;
    hipLaunchKernelGGL(init_equilibrium, dim3((unsigned)((n + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, s, f, rows, rf,
                       pitch, P, c0, c1, c2);
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

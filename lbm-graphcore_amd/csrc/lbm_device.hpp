// lbm_device.hpp -- device helpers shared by the step kernels.
//
// The per-cell arithmetic is split into macro() (density, velocity, |u|)
// and the per-pair outputs so kernels can finish and store one rebound pair
// at a time; collide() composes them for one cell.  Every expression follows
// main/LastChance.cpp:226-262 verbatim (same operand order, same constants),
// which together with -ffp-contract=off makes the lattice bitwise identical
// to the CPU oracle.
#pragma once

#include <hip/hip_runtime.h>

#include <climits>
#include <cstdint>

#include "lbm_layout.hpp"

namespace lbm {

__device__ __forceinline__ float4 ld4(const float *p) { return *reinterpret_cast<const float4 *>(p); }
__device__ __forceinline__ void st4(float *p, float4 v) { *reinterpret_cast<float4 *>(p) = v; }

// Bijective XCD-aware block remap (blocks b and b+8 share an XCD): blocks on
// one XCD get consecutive logical ids, so neighbouring tiles -- which share
// cache lines at their seams -- are fetched through one L2.
__device__ __forceinline__ int xcd_remap(int b, int nb) {
    const int xcd = b & 7;
    const int q = nb >> 3, r = nb & 7;
    const int start = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
    return start + (b >> 3);
}

// Block sum over NW waves in a fixed order (result valid in thread 0).
template <int NW>
__device__ __forceinline__ float block_sum_n(float v, float *lds) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    __syncthreads();
    if (lane == 0) lds[wid] = v;
    __syncthreads();
    float r = 0.f;
    if (threadIdx.x == 0) {
        r = lds[0];
#pragma unroll
        for (int i = 1; i < NW; ++i) r += lds[i];
    }
    return r;
}

__device__ __forceinline__ float block_sum(float v, float *lds) { return block_sum_n<BLOCK / 64>(v, lds); }

// Sum n block partials in a fixed order (depends on n and NT only): float4
// loads, four independent accumulators per thread so the loads overlap, then
// the block tree.  p must be 16-byte aligned.  Result valid in thread 0.
template <int NT>
__device__ __forceinline__ float sum_partials_n(const float *p, int n, float *lds) {
    const int n4 = n >> 2;
    const float4 *p4 = reinterpret_cast<const float4 *>(p);
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    int i = threadIdx.x;
    for (; i + 3 * NT < n4; i += 4 * NT) {
        const float4 x0 = p4[i], x1 = p4[i + NT], x2 = p4[i + 2 * NT], x3 = p4[i + 3 * NT];
        a0 += (x0.x + x0.y) + (x0.z + x0.w);
        a1 += (x1.x + x1.y) + (x1.z + x1.w);
        a2 += (x2.x + x2.y) + (x2.z + x2.w);
        a3 += (x3.x + x3.y) + (x3.z + x3.w);
    }
    for (; i < n4; i += NT) {
        const float4 x0 = p4[i];
        a0 += (x0.x + x0.y) + (x0.z + x0.w);
    }
    for (int k = 4 * n4 + threadIdx.x; k < n; k += NT) a1 += p[k];
    return block_sum_n<NT / 64>((a0 + a1) + (a2 + a3), lds);
}

// Block 0 of a reducing launch (NT threads): fold every pending step of the
// previous launch (ctl[0] steps of ctl[2] partials, ctl[3] apart) into
// av_local[ctl[1]...] and advance ctl[1].
template <int NT>
__device__ __forceinline__ void reduce_pending_n(int *ctl, const float *partials, float *av_local, float *lds) {
    const int pending = ctl[0];
    if (pending <= 0) return;
    const int n = ctl[2], stride = ctl[3];
    const int idx = ctl[1];
    for (int s = 0; s < pending; ++s) {
        const float v = sum_partials_n<NT>(partials + (long long)s * stride, n, lds);
        if (threadIdx.x == 0) av_local[idx + s] = v;
    }
    __syncthreads();
    if (threadIdx.x == 0) ctl[1] = idx + pending;
    __syncthreads();
}

__device__ __forceinline__ void reduce_pending(int *ctl, const float *partials, float *av_local, float *lds) {
    reduce_pending_n<BLOCK>(ctl, partials, av_local, lds);
}

__device__ __forceinline__ void publish_pending(int *ctl, int steps, int n, int stride) {
    ctl[0] = steps;
    ctl[2] = n;
    ctl[3] = stride;
}

// Store the nine populations of one cell at strip coordinates (sa, sb) of a
// wide-halo destination (own ghost ring or send buffer, lbm_layout.hpp Dst2).
// The destination is global memory: stores through a generic (flat) pointer
// would make every later vmcnt wait a full drain (flat operations complete
// out of order), including the prefetched rows of the stream kernels.
__device__ __forceinline__ void store2(const Dst2 &d, int sa, int sb, const float (&o)[Q]) {
    __attribute__((address_space(1))) float *p =
        (__attribute__((address_space(1))) float *)d.base + (long long)sa * d.s1 + (long long)sb * d.s2;
#pragma unroll
    for (int k = 0; k < Q; ++k) p[k * d.ks] = o[k];
}

// ---- per-cell physics -----------------------------------------------------

struct Macro {
    float rho, ux, uy, csq, ld1, ld2, u;
    bool obst;
};

// Density, velocity and the relaxation factors of one cell from its nine
// pulled populations (LastChance.cpp:226-242); u = |u| for fluid cells, 0 for
// obstacles (av_velocity counts fluid cells only, :262).
__device__ __forceinline__ Macro macro(const float (&s)[Q], bool obst, float omega) {
    Macro m;
    m.obst = obst;
    m.rho = s[0] + s[1] + s[2] + s[3] + s[4] + s[5] + s[6] + s[7] + s[8];
    m.ux = (s[1] + s[5] + s[8] - (s[3] + s[6] + s[7])) / m.rho;
    m.uy = (s[2] + s[5] + s[6] - (s[4] + s[7] + s[8])) / m.rho;
    const float usq = m.ux * m.ux + m.uy * m.uy;
    m.csq = 1.00f - usq * 1.50f;
    m.ld1 = m.rho / 9.00f * omega;
    m.ld2 = m.rho / 36.00f * omega;
    m.u = obst ? 0.f : sqrtf(usq);
    return m;
}

// Outputs (LastChance.cpp:243-261): obstacle cells rebound (out_k = s_opp(k),
// :213-223), fluid cells relax, the folded acceleration (accf = 1 on row
// ny-2) adds +-w1/w2.
__device__ __forceinline__ float out0(float s0, const Macro &m, float omo, float omega) {
    return m.obst ? s0 : s0 * omo + 4.00f / 9.00f * m.rho * omega * m.csq;
}

__device__ __forceinline__ void out13(float s1, float s3, const Macro &m, float omo, float accf, float w1, float &o1,
                                      float &o3) {
    const float c1 = s1 * omo + m.ld1 * ((4.50f * m.ux) * (2.00f / 3.00f + m.ux) + m.csq);
    const float c3 = s3 * omo + m.ld1 * ((-4.50f * m.ux) * (2.00f / 3.00f - m.ux) + m.csq);
    o1 = m.obst ? s3 : c1 + accf * w1;
    o3 = m.obst ? s1 : c3 - accf * w1;
}

__device__ __forceinline__ void out24(float s2, float s4, const Macro &m, float omo, float &o2, float &o4) {
    const float c2 = s2 * omo + m.ld1 * ((4.50f * m.uy) * (2.00f / 3.00f + m.uy) + m.csq);
    const float c4 = s4 * omo + m.ld1 * ((-4.50f * m.uy) * (2.00f / 3.00f - m.uy) + m.csq);
    o2 = m.obst ? s4 : c2;
    o4 = m.obst ? s2 : c4;
}

__device__ __forceinline__ void out57(float s5, float s7, const Macro &m, float omo, float accf, float w2, float &o5,
                                      float &o7) {
    const float us = m.ux + m.uy;
    const float c5 = s5 * omo + m.ld2 * ((4.50f * us) * (2.00f / 3.00f + us) + m.csq);
    const float c7 = s7 * omo + m.ld2 * ((-4.50f * us) * (2.00f / 3.00f - us) + m.csq);
    o5 = m.obst ? s7 : c5 + accf * w2;
    o7 = m.obst ? s5 : c7 - accf * w2;
}

__device__ __forceinline__ void out68(float s6, float s8, const Macro &m, float omo, float accf, float w2, float &o6,
                                      float &o8) {
    const float ud = -m.ux + m.uy;
    const float c6 = s6 * omo + m.ld2 * ((4.50f * ud) * (2.00f / 3.00f + ud) + m.csq);
    const float c8 = s8 * omo + m.ld2 * ((-4.50f * ud) * (2.00f / 3.00f - ud) + m.csq);
    o6 = m.obst ? s8 : c6 - accf * w2;
    o8 = m.obst ? s6 : c8 + accf * w2;
}

// Whole cell: returns |u| (0 for obstacles).
__device__ __forceinline__ float collide(const float (&s)[Q], float (&o)[Q], bool obst, float accf, float omega,
                                         float omo, float w1, float w2) {
    const Macro m = macro(s, obst, omega);
    o[0] = out0(s[0], m, omo, omega);
    out13(s[1], s[3], m, omo, accf, w1, o[1], o[3]);
    out24(s[2], s[4], m, omo, o[2], o[4]);
    out57(s[5], s[7], m, omo, accf, w2, o[5], o[7]);
    out68(s[6], s[8], m, omo, accf, w2, o[6], o[8]);
    return m.u;
}

// ---- work decomposition -----------------------------------------------------

struct RectPos {
    int x0, y, cxi, wc;
    bool active;
};

// Tile t (BLOCK work items, wave-uniform) -> rect; lane -> (column chunk, row).
// Every tile lies inside one rect, so the rect lookup stays scalar.
template <int N>
__device__ __forceinline__ int rect_of(const int (&rect_begin)[N], int t) {
    int r = 0;
#pragma unroll
    for (int i = 1; i < N; ++i) r = (t >= rect_begin[i]) ? i : r;
    return __builtin_amdgcn_readfirstlane(r);
}

__device__ __forceinline__ RectPos locate(const Rect (&rect)[MAX_RECTS], const int (&rect_begin)[MAX_RECTS], int t,
                                          int tid) {
    const int r = rect_of(rect_begin, t);
    const Rect R = rect[r];
    const int items = R.wc * R.hr;
    int lc = (t - rect_begin[r]) * BLOCK + tid;
    const bool active = lc < items;
    lc = active ? lc : items - 1;
    const int yy = lc / R.wc;
    const int cxi = lc - yy * R.wc;
    return RectPos{R.x0, R.y0 + yy, cxi, R.wc, active};
}

}  // namespace lbm

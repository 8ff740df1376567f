// lbm3d.hip -- D3Q19-BGK engine (include/lbm3d_hip.h): BASELINE config 5,
// SURVEY 8f rank 4.  The reference has no 3-D code; this is the 3-D analogue
// of its fused D2Q9 step (main/LastChance.cpp:192-266) on the same machinery
// as the D2Q9 engine: SoA lattice pair, one fused pull-stream / bounce-back /
// BGK / body-force / |u| kernel, device-side per-step |u| partials, slab
// decomposition with halos over RCCL (or device copies), boundary planes on a
// high-priority stream so the exchange overlaps the interior.
//
// Layout per slab of nzs planes: f[z + 2][k][y][px] for -2 <= z <= nzs + 1 (two
// ghost planes below and above: the one-step kernels read the inner ones, the
// two-step kernel both); speeds ordered so that the five that cross
// the top face (c_z = +1: 9..13) and the five that cross the bottom face
// (c_z = -1: 14..18) are each ONE contiguous block of a plane -- the halo
// message of a face is a single contiguous range of the lattice, sent and
// received in place (no pack / unpack kernels).  x and y wrap in-kernel.
//
// Bandwidth-bound: 152 algorithmic bytes per cell update (19 fp32 loads + 19
// stores); no MFMA.  Arithmetic in IEEE fp32 evaluated in the order of
// oracle/lbm_oracle3d.c (-ffp-contract=off, correctly rounded / and sqrt), so
// the lattice is bitwise equal to the CPU restatement.

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <array>
#include <vector>
#include <type_traits>

#include "lbm3d_hip.h"
#include "lbm_packed.hpp"

#ifndef LBM3D_XCD_REMAP
#define LBM3D_XCD_REMAP 1  // 0: the hardware's block order (A/B builds only)
#endif

namespace lbm {

constexpr int Q3 = 19;
constexpr int B3X = 64, B3Y = 4;  // block: 64 x-columns (one wave) x 4 rows

struct Step3Args {
    const float *fin;        // origin (plane z = 0) of the lattice read
    float *fout;             // origin of the lattice written
    const uint8_t *obst;     // [nzs][ny][nx]
    long long PL, KS;        // plane stride, speed stride (floats)
    int px, nx, ny;
    int z0;                  // first plane of this launch
    float omega, omo, w1, w2;
    float *partials;         // this launch writes partials[block]
};

__global__ __launch_bounds__(B3X * B3Y) void step3d(Step3Args a) {
    __shared__ float lds[B3X * B3Y / 64];
    const int x = blockIdx.x * B3X + threadIdx.x;
    const int y = blockIdx.y * B3Y + threadIdx.y;
    const int z = a.z0 + blockIdx.z;
    float usum = 0.f;
    if (x < a.nx && y < a.ny) {
        const int xw = x == 0 ? a.nx - 1 : x - 1, xe = x == a.nx - 1 ? 0 : x + 1;
        const int ys = y == 0 ? a.ny - 1 : y - 1, yn = y == a.ny - 1 ? 0 : y + 1;
        const long long PL = a.PL, KS = a.KS;
        const int px = a.px;
        // pulled populations s_k = f_k(x - cx, y - cy, z - cz)
        const float *p0 = a.fin + (long long)z * PL;  // plane z
        const float *pm = p0 - PL;                     // plane z-1 (c_z = +1 pulls from below)
        const float *pp = p0 + PL;                     // plane z+1
        const long long ry = (long long)y * px, rs = (long long)ys * px, rn = (long long)yn * px;
        float s[Q3];
        s[0] = p0[0 * KS + ry + x];
        s[1] = p0[1 * KS + ry + xw];
        s[2] = p0[2 * KS + ry + xe];
        s[3] = p0[3 * KS + rs + x];
        s[4] = p0[4 * KS + rn + x];
        s[5] = p0[5 * KS + rs + xw];
        s[6] = p0[6 * KS + rn + xe];
        s[7] = p0[7 * KS + rn + xw];
        s[8] = p0[8 * KS + rs + xe];
        s[9] = pm[9 * KS + ry + x];
        s[10] = pm[10 * KS + ry + xw];
        s[11] = pm[11 * KS + ry + xe];
        s[12] = pm[12 * KS + rs + x];
        s[13] = pm[13 * KS + rn + x];
        s[14] = pp[14 * KS + ry + x];
        s[15] = pp[15 * KS + ry + xe];
        s[16] = pp[16 * KS + ry + xw];
        s[17] = pp[17 * KS + rn + x];
        s[18] = pp[18 * KS + rs + x];
        float o[Q3];
        const bool ob = a.obst[((long long)blockIdx.z * a.ny + y) * a.nx + x] != 0;
        if (ob) {  // bounce-back: out_k = s_opp(k)
            o[0] = s[0];
            o[1] = s[2];
            o[2] = s[1];
            o[3] = s[4];
            o[4] = s[3];
            o[5] = s[6];
            o[6] = s[5];
            o[7] = s[8];
            o[8] = s[7];
#pragma unroll
            for (int i = 0; i < 5; ++i) {
                o[9 + i] = s[14 + i];
                o[14 + i] = s[9 + i];
            }
        } else {
            const float rho = s[0] + s[1] + s[2] + s[3] + s[4] + s[5] + s[6] + s[7] + s[8] + s[9] + s[10] + s[11] +
                              s[12] + s[13] + s[14] + s[15] + s[16] + s[17] + s[18];
            const float ux = ((s[1] + s[5] + s[7] + s[10] + s[16]) - (s[2] + s[6] + s[8] + s[11] + s[15])) / rho;
            const float uy = ((s[3] + s[5] + s[8] + s[12] + s[18]) - (s[4] + s[6] + s[7] + s[13] + s[17])) / rho;
            const float uz = ((s[9] + s[10] + s[11] + s[12] + s[13]) - (s[14] + s[15] + s[16] + s[17] + s[18])) / rho;
            const float usq = ux * ux + uy * uy + uz * uz;
            const float c = 1.00f - usq * 1.50f;
            const float ld0 = rho / 3.00f * a.omega;
            const float ld1 = rho / 18.00f * a.omega;
            const float ld2 = rho / 36.00f * a.omega;
            const float pxy = ux + uy, mxy = ux - uy, pxz = ux + uz, mxz = -ux + uz, pyz = uy + uz, myz = -uy + uz;
            const float e[Q3] = {0.f, ux, -ux, uy, -uy, pxy, -pxy, mxy, -mxy, uz, pxz, mxz, pyz, myz,
                                 -uz, -pxz, -mxz, -pyz, -myz};
            const float omo = a.omo;
            o[0] = s[0] * omo + ld0 * c;
#pragma unroll
            for (int k = 1; k < Q3; ++k) {
                const float ld = (k <= 4 || k == 9 || k == 14) ? ld1 : ld2;
                o[k] = s[k] * omo + ld * ((4.50f * e[k]) * (2.00f / 3.00f + e[k]) + c);
            }
            const float w1 = a.w1, w2 = a.w2;
            o[1] = o[1] + w1;
            o[2] = o[2] - w1;
            o[5] = o[5] + w2;
            o[6] = o[6] - w2;
            o[7] = o[7] + w2;
            o[8] = o[8] - w2;
            o[10] = o[10] + w2;
            o[11] = o[11] - w2;
            o[15] = o[15] - w2;
            o[16] = o[16] + w2;
            usum = sqrtf(usq);
        }
        float *d = a.fout + (long long)z * PL + ry + x;
#pragma unroll
        for (int k = 0; k < Q3; ++k) d[k * KS] = o[k];
    }
    // block partial in a fixed order (waves in threadIdx order)
    float v = usum;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
    const int t = threadIdx.y * B3X + threadIdx.x;
    if ((t & 63) == 0) lds[t >> 6] = v;
    __syncthreads();
    if (t == 0) {
        float b = lds[0];
#pragma unroll
        for (int i = 1; i < B3X * B3Y / 64; ++i) b += lds[i];
        a.partials[((long long)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x] = b;
    }
}

// One D3Q19 cell: pulled populations s -> outputs o (the order of
// oracle/lbm_oracle3d.c cell3d); returns |u| (0 for an obstacle).
__device__ __forceinline__ float cell3d(const float (&s)[Q3], float (&o)[Q3], bool ob, float omega, float omo,
                                        float w1, float w2) {
    if (ob) {
        o[0] = s[0];
        o[1] = s[2];
        o[2] = s[1];
        o[3] = s[4];
        o[4] = s[3];
        o[5] = s[6];
        o[6] = s[5];
        o[7] = s[8];
        o[8] = s[7];
#pragma unroll
        for (int i = 0; i < 5; ++i) {
            o[9 + i] = s[14 + i];
            o[14 + i] = s[9 + i];
        }
        return 0.f;
    }
    const float rho = s[0] + s[1] + s[2] + s[3] + s[4] + s[5] + s[6] + s[7] + s[8] + s[9] + s[10] + s[11] + s[12] +
                      s[13] + s[14] + s[15] + s[16] + s[17] + s[18];
    // correctly rounded divisions for every input (lbm_packed.hpp header):
    // the velocity components by the compiler's IEEE sequence; x/3 by the
    // short sequence (exhaustively exact for every float x); x/18 and x/36
    // by it for x >= 2^-120 (exhaustive: exact from 2^-125 / 2^-124 up), by
    // IEEE division in a wave holding a smaller density (never in physical states)
    auto cdiv = [](float x, float d, float y) {
        const float q = x * y;
        return __builtin_fmaf(__builtin_fmaf(-d, q, x), y, q);
    };
    const float ux = ((s[1] + s[5] + s[7] + s[10] + s[16]) - (s[2] + s[6] + s[8] + s[11] + s[15])) / rho;
    const float uy = ((s[3] + s[5] + s[8] + s[12] + s[18]) - (s[4] + s[6] + s[7] + s[13] + s[17])) / rho;
    const float uz = ((s[9] + s[10] + s[11] + s[12] + s[13]) - (s[14] + s[15] + s[16] + s[17] + s[18])) / rho;
    const float usq = ux * ux + uy * uy + uz * uz;
    const float c = 1.00f - usq * 1.50f;
    const float ld0 = cdiv(rho, 3.00f, 1.00f / 3.00f) * omega;
    float r18 = cdiv(rho, 18.00f, 1.00f / 18.00f), r36 = cdiv(rho, 36.00f, 1.00f / 36.00f);
    if (__builtin_expect(__builtin_amdgcn_ballot_w64(!(rho >= 0x1p-120f)) != 0, 0)) {
        r18 = rho / 18.00f;
        r36 = rho / 36.00f;
    }
    const float ld1 = r18 * omega;
    const float ld2 = r36 * omega;
    const float pxy = ux + uy, mxy = ux - uy, pxz = ux + uz, mxz = -ux + uz, pyz = uy + uz, myz = -uy + uz;
    const float e[Q3] = {0.f, ux, -ux, uy, -uy, pxy, -pxy, mxy, -mxy, uz, pxz, mxz, pyz, myz,
                         -uz, -pxz, -mxz, -pyz, -myz};
    o[0] = s[0] * omo + ld0 * c;
#pragma unroll
    for (int k = 1; k < Q3; ++k) {
        const float ld = (k <= 4 || k == 9 || k == 14) ? ld1 : ld2;
        o[k] = s[k] * omo + ld * ((4.50f * e[k]) * (2.00f / 3.00f + e[k]) + c);
    }
    o[1] = o[1] + w1;
    o[2] = o[2] - w1;
    o[5] = o[5] + w2;
    o[6] = o[6] - w2;
    o[7] = o[7] + w2;
    o[8] = o[8] - w2;
    o[10] = o[10] + w2;
    o[11] = o[11] - w2;
    o[15] = o[15] - w2;
    o[16] = o[16] + w2;
    return __builtin_amdgcn_sqrtf(usq);  // |u| feeds av_vels only (<= 1 ulp, as lbm_packed.hpp sqrt_av)
}

// LBM_FLAG_TOLERANCE form of cell3d (the 2-D collide2t's reassociation in
// 3-D): one reciprocal of rho (v_rcp_f32, 1 ulp, no Newton step) for the velocity,
// carried scaled (v = 3u), rho * (omega / 3 | 18 | 36), and per pair of
// opposite speeds out_k = fma(s_k, 1 - omega, P) +- Q with P = ld (v^2 / 2 +
// c), c = 1 - |v|^2 / 6, Q = ld v (+ the body-force weight of the pair, which
// enters the two outputs with opposite signs).  Not bitwise equal to
// oracle/lbm_oracle3d.c; checked against it within a stated tolerance
// (tests/test_d3q19.py test_d3q19_tolerance_*).  k = {1 - omega, omega/3,
// omega/18, omega/36}.
__device__ __forceinline__ float cell3dt(const float (&s)[Q3], float (&o)[Q3], bool ob, float omo, float k0, float k1,
                                         float k2, float w1, float w2) {
    if (ob) {
        o[0] = s[0];
        o[1] = s[2];
        o[2] = s[1];
        o[3] = s[4];
        o[4] = s[3];
        o[5] = s[6];
        o[6] = s[5];
        o[7] = s[8];
        o[8] = s[7];
#pragma unroll
        for (int i = 0; i < 5; ++i) {
            o[9 + i] = s[14 + i];
            o[14 + i] = s[9 + i];
        }
        return 0.f;
    }
    const float ax = s[1] + s[5] + s[7] + s[10] + s[16], bx = s[2] + s[6] + s[8] + s[11] + s[15];
    const float ay = s[3] + s[5] + s[8] + s[12] + s[18], by = s[4] + s[6] + s[7] + s[13] + s[17];
    const float az = s[9] + s[10] + s[11] + s[12] + s[13], bz = s[14] + s[15] + s[16] + s[17] + s[18];
    // ax + bx holds speeds 1, 2, 5-8, 10, 11, 15, 16; the rest of the 19 here
    const float rho = ((s[0] + (s[3] + s[4])) + (ax + bx)) + ((s[9] + s[12] + s[13]) + (s[14] + s[17] + s[18]));
    const float r = __builtin_amdgcn_rcpf(rho);
    const float r3 = r * 3.00f;
    const float vx = (ax - bx) * r3, vy = (ay - by) * r3, vz = (az - bz) * r3;  // 3 u
    const float h = __builtin_fmaf(vx, vx, __builtin_fmaf(vy, vy, vz * vz));   // 9 |u|^2
    const float c = __builtin_fmaf(h, -1.00f / 6.00f, 1.00f);
    const float ld1 = rho * k1, ld2 = rho * k2;
    o[0] = __builtin_fmaf(s[0], omo, (rho * k0) * c);
    // q: the pair's +- term, w: its body-force weight (+w on kp, -w on km)
    auto pair = [&](int kp, int km, float v, float ld, float w) {
        const float p = ld * __builtin_fmaf(v * v, 0.50f, c), q = __builtin_fmaf(ld, v, w);
        o[kp] = __builtin_fmaf(s[kp], omo, p) + q;
        o[km] = __builtin_fmaf(s[km], omo, p) - q;
    };
    auto pair0 = [&](int kp, int km, float v, float ld) {  // no body force on this pair
        const float p = ld * __builtin_fmaf(v * v, 0.50f, c);
        o[kp] = __builtin_fmaf(ld, v, __builtin_fmaf(s[kp], omo, p));
        o[km] = __builtin_fmaf(-ld, v, __builtin_fmaf(s[km], omo, p));
    };
    pair(1, 2, vx, ld1, w1);
    pair0(3, 4, vy, ld1);
    pair0(9, 14, vz, ld1);
    pair(5, 6, vx + vy, ld2, w2);
    pair(7, 8, vx - vy, ld2, w2);
    pair(10, 15, vx + vz, ld2, w2);
    pair(11, 16, vz - vx, ld2, -w2);
    pair0(12, 17, vy + vz, ld2);
    pair0(13, 18, vz - vy, ld2);
    return __builtin_amdgcn_sqrtf(h) * (1.00f / 3.00f);  // |u|, av_vels only
}

// Two cells per lane (a column pair, nx even): every load and store is a
// float2 (512 B per wave instruction instead of 256); the x-shifted pulls
// take the neighbour column from the adjacent lane by DPP, and the first /
// last pair of a wave (or of a row, with the periodic wrap) loads it
// directly.  Each block walks ZB planes, so the per-step |u| partials are
// ZB times fewer.  Bitwise equal to step3d (same cell3d arithmetic).
template <int ZB, bool NT>
__global__ __launch_bounds__(B3X * B3Y) void step3d_pair(Step3Args a, int planes) {
    __shared__ float lds[B3X * B3Y / 64];
    const int lane = threadIdx.x;
    const int xa = blockIdx.x * (2 * B3X) + 2 * lane;
    const int y = blockIdx.y * B3Y + threadIdx.y;
    const bool active = xa < a.nx && y < a.ny;
    float usum = 0.f;
    const long long PL = a.PL, KS = a.KS;
    const int px = a.px, nx = a.nx;
    const int yc = min(y, a.ny - 1);  // inactive rows read a valid row
    const int ys = yc == 0 ? a.ny - 1 : yc - 1, yn = yc + 1 >= a.ny ? 0 : yc + 1;
    const long long ry = (long long)yc * px, rs = (long long)ys * px, rn = (long long)yn * px;
    const int xc = min(xa, nx - 2);  // clamped pair base for inactive lanes
    const bool first = lane == 0 || xa == 0;
    const bool last = lane == B3X - 1 || xa + 2 >= nx;
    const int xl = xa == 0 ? nx - 1 : xa - 1;   // column left of the pair (periodic)
    const int xr = xa + 2 >= nx ? 0 : xa + 2;   // column right of the pair
    const int zb0 = blockIdx.z * ZB;
    for (int zi = 0; zi < ZB; ++zi) {
        const int zl = zb0 + zi;
        if (zl >= planes) break;
        const int z = a.z0 + zl;
        const float *p0 = a.fin + (long long)z * PL;
        const float *pm = p0 - PL, *pp = p0 + PL;
        auto L2 = [&](const float *base, int k, long long row) {
            return *reinterpret_cast<const f2 *>(base + k * KS + row + xc);
        };
        f2 s2[Q3];
        s2[0] = L2(p0, 0, ry);
        s2[1] = left2(L2(p0, 1, ry));
        s2[2] = right2(L2(p0, 2, ry));
        s2[3] = L2(p0, 3, rs);
        s2[4] = L2(p0, 4, rn);
        s2[5] = left2(L2(p0, 5, rs));
        s2[6] = right2(L2(p0, 6, rn));
        s2[7] = left2(L2(p0, 7, rn));
        s2[8] = right2(L2(p0, 8, rs));
        s2[9] = L2(pm, 9, ry);
        s2[10] = left2(L2(pm, 10, ry));
        s2[11] = right2(L2(pm, 11, ry));
        s2[12] = L2(pm, 12, rs);
        s2[13] = L2(pm, 13, rn);
        s2[14] = L2(pp, 14, ry);
        s2[15] = right2(L2(pp, 15, ry));
        s2[16] = left2(L2(pp, 16, ry));
        s2[17] = L2(pp, 17, rn);
        s2[18] = L2(pp, 18, rs);
        if (first && active) {  // pulls from x - 1: speeds 1, 5, 7, 10, 16
            s2[1].x = p0[1 * KS + ry + xl];
            s2[5].x = p0[5 * KS + rs + xl];
            s2[7].x = p0[7 * KS + rn + xl];
            s2[10].x = pm[10 * KS + ry + xl];
            s2[16].x = pp[16 * KS + ry + xl];
        }
        if (last && active) {   // pulls from x + 1: speeds 2, 6, 8, 11, 15
            s2[2].y = p0[2 * KS + ry + xr];
            s2[6].y = p0[6 * KS + rn + xr];
            s2[8].y = p0[8 * KS + rs + xr];
            s2[11].y = pm[11 * KS + ry + xr];
            s2[15].y = pp[15 * KS + ry + xr];
        }
        if (active) {
            const uint16_t ob2 = *reinterpret_cast<const uint16_t *>(a.obst + ((long long)zl * a.ny + y) * nx + xa);
            float sa[Q3], sb[Q3], oa[Q3], obv[Q3];
#pragma unroll
            for (int k = 0; k < Q3; ++k) {
                sa[k] = s2[k].x;
                sb[k] = s2[k].y;
            }
            usum += cell3d(sa, oa, (ob2 & 0xffu) != 0, a.omega, a.omo, a.w1, a.w2);
            usum += cell3d(sb, obv, (ob2 >> 8) != 0, a.omega, a.omo, a.w1, a.w2);
            float *d = a.fout + (long long)z * PL + ry + xa;
#pragma unroll
            for (int k = 0; k < Q3; ++k) {
                if (NT)
                    __builtin_nontemporal_store(f2{oa[k], obv[k]}, reinterpret_cast<f2 *>(d + k * KS));
                else
                    *reinterpret_cast<f2 *>(d + k * KS) = f2{oa[k], obv[k]};
            }
        }
    }
    float v = usum;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
    const int t = threadIdx.y * B3X + threadIdx.x;
    if ((t & 63) == 0) lds[t >> 6] = v;
    __syncthreads();
    if (t == 0) {
        float b = lds[0];
#pragma unroll
        for (int i = 1; i < B3X * B3Y / 64; ++i) b += lds[i];
        a.partials[((long long)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x] = b;
    }
}

// ---------------------------------------------------------------------------
// Two time steps per pass over the lattice (one slab, z periodic): 2.5-D
// temporal blocking.  A block of 64 columns (one wave, one column per lane) x
// TH rows (one wave per row) walks a segment of z planes; as input plane j
// arrives (step t, 19 coalesced loads per lane), level 1 computes plane j-1 at
// t+1 and level 2 computes plane j-2 at t+2 from level 1's planes, so the
// lattice crosses HBM once per two steps.  Owned outputs: the inner 60 x
// (TH - 4) cells (a two-cell ring in x and y is recomputed).
// Pulls, per level, for the centre plane z (input plane z+1 just arrived):
//   own row, x +- 1 by DPP:   speeds 0,1,2 of plane z, 9,10,11 of plane z-1
//                             (registers kept from earlier iterations),
//                             14,15,16 of plane z+1;
//   rows y +- 1 through LDS:  3..8 of plane z (one slot set, read into
//                             registers the iteration plane z arrives),
//                             12,13 of plane z-1 (ring of 3), 17,18 of z+1.
// Two barriers per iteration (one per level) order every slot's writes and
// reads (each slot is rewritten only after the barrier that follows its last
// read).  Algorithmic traffic per cell update: (19 loads x 64 TH / (60 (TH-4))
// + 19 stores) x 4 B / 2 = 98.8 B at TH = 12, 92.3 B at TH = 16, instead of
// 152.  Same cell3d arithmetic: bitwise equal to the one-step kernels.
// ---------------------------------------------------------------------------
// TH = rows per block (waves), a template parameter (LBM3D_TH): two levels of
// 14 plane slots of 64 x TH floats take 7 x TH KB of LDS (TH <= 16: one
// block of 16 waves per CU, 4 per SIMD).
// SKIP: a wave whose row no level-2 (level-1) cell depends on skips that
// level's collision (rows 0 and TH-1 at level 1; rows 0, 1, TH-2, TH-1 at
// level 2) -- it still writes and reads its LDS slots and barriers, and the
// skipped values are never read (level 2 of rows 2 .. TH-3 pulls from level-1
// rows 1 .. TH-2).
constexpr int T3W = 64;
constexpr int T3OX = T3W - 4;  // owned columns
// Z (speeds 3..8 of the newest plane) is single-buffered: each thread reads
// its six y +- 1 pulls right after the barrier that publishes them and keeps
// them in registers (zr) until the next iteration, when that plane is the
// centre plane -- 14 slots per level instead of 20 (round 3), so blocks of
// 16 rows fit (owned 60 x 12 of 64 x 16 loaded: 92 B per update instead of
// 98.8 for 12 rows).
template <int TH>
struct T3 {
    static constexpr int C = T3W * TH;                    // cells per plane slot
    static constexpr int LDS = (2 + 6 + 3 * 2) * C;       // floats per level: M, Z[6], P[3][2]
    static constexpr int OY = TH - 4;                     // owned rows
};

// XCD-aware block order for the multi-step passes (as the 2-D stream
// kernel's xcd_remap, lbm_device.hpp): the hardware deals workgroups to the
// eight XCDs round robin, so consecutive blocks -- x neighbours, whose
// windows overlap by six columns, and y neighbours, overlapping by six rows
// -- landed on different XCDs and read their shared cells from HBM twice.
// Here each XCD takes one contiguous range of (x fastest, then y, then z)
// blocks, so neighbours run side by side on one XCD and the overlap comes
// from its L2.  Blocks keep their logical index for the |u| partials.
struct Blk3 {
    int x, y, z;
};
__device__ __forceinline__ Blk3 blk3_remap() {
    const int nb = gridDim.x * gridDim.y * gridDim.z;
    const int lin = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
    const int l = LBM3D_XCD_REMAP ? xcd_remap(lin, nb) : lin;
    const int yz = l / gridDim.x;
    return Blk3{l - yz * (int)gridDim.x, yz % (int)gridDim.y, yz / (int)gridDim.y};
}

struct Two3Args {
    const float *fin;   // origin of the lattice read (ghost planes -2, -1, nz, nz + 1 filled)
    float *fout;
    const uint8_t *obst;  // plane 0 of [nz + 6][ny][nx]: three planes of neighbour / periodic images each side
    long long PL, KS;
    int px, nx, ny, nz, seg;
    int z0, zn;           // output planes [z0, zn) of this launch, in segments of seg planes
    float omega, omo, w1, w2;
    float k0, k1, k2;     // tolerance collision: omega / 3, omega / 18, omega / 36
    float *partials;      // [2][nblocks]: |u| of step t+1, then t+2, at blk0 + this launch's block
    int nblocks, blk0;
};

// One level for centre plane jz - 1, input plane jz (in).  Must be reached by
// every thread of the block (it holds a barrier).  live (wave-uniform): some
// later level or output needs this row's result.
template <int TH, bool TOL>
__device__ __forceinline__ float level3(const float (&in)[Q3], float (&out)[Q3], float *lds, int jz, float (&r0)[3],
                                        float (&r9a)[3], float (&r9b)[3], float (&zr)[6], int lane, int wy, bool ob,
                                        bool live, const Two3Args &a) {
    constexpr int T3C = T3<TH>::C;
    float *M = lds, *Z = lds + 2 * T3C, *P = lds + 8 * T3C;
    const int c = wy * T3W + lane;
    const int pw = ((jz % 3) + 3) % 3;  // P slot of plane jz
    M[c] = in[17];
    M[T3C + c] = in[18];
#pragma unroll
    for (int i = 0; i < 6; ++i) Z[i * T3C + c] = in[3 + i];
    P[(pw * 2) * T3C + c] = in[12];
    P[(pw * 2 + 1) * T3C + c] = in[13];
    __syncthreads();
    const int wm = max(wy - 1, 0) * T3W, wp = min(wy + 1, TH - 1) * T3W;
    const int lm = max(lane - 1, 0), lp = min(lane + 1, T3W - 1);
    const float *p = P + ((((jz - 2) % 3) + 3) % 3) * 2 * T3C;  // plane jz - 2
    float s[Q3];
    s[0] = r0[0];
    s[1] = dpp_from_left(r0[1]);
    s[2] = dpp_from_right(r0[2]);
#pragma unroll
    for (int i = 0; i < 6; ++i) s[3 + i] = zr[i];  // plane jz - 1's pulls, read one iteration ago
    // plane jz's y +- 1 pulls of speeds 3..8, for the next iteration (the slot
    // is rewritten only after the next barrier of this level's other half)
    zr[0] = Z[0 * T3C + wm + lane];
    zr[1] = Z[1 * T3C + wp + lane];
    zr[2] = Z[2 * T3C + wm + lm];
    zr[3] = Z[3 * T3C + wp + lp];
    zr[4] = Z[4 * T3C + wp + lm];
    zr[5] = Z[5 * T3C + wm + lp];
    s[9] = r9b[0];
    s[10] = dpp_from_left(r9b[1]);
    s[11] = dpp_from_right(r9b[2]);
    s[12] = p[0 * T3C + wm + lane];
    s[13] = p[1 * T3C + wp + lane];
    s[14] = in[14];
    s[15] = dpp_from_right(in[15]);
    s[16] = dpp_from_left(in[16]);
    s[17] = M[wp + lane];
    s[18] = M[T3C + wm + lane];
    float u = 0.f;
    if (live) {
        if constexpr (TOL)
            u = cell3dt(s, out, ob, a.omo, a.k0, a.k1, a.k2, a.w1, a.w2);
        else
            u = cell3d(s, out, ob, a.omega, a.omo, a.w1, a.w2);
    } else {
#pragma unroll
        for (int k = 0; k < Q3; ++k) out[k] = 0.f;
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        r9b[i] = r9a[i];
        r9a[i] = in[9 + i];
        r0[i] = in[i];
    }
    return u;
}

// PD: input planes in flight -- 1: plane j+1 while j is computed; 2: also j+2
// (19 more VGPRs; one 768..960-thread block per CU keeps few loads in flight);
// 0: plane j+1 is loaded into the input registers once level 1 has consumed
// them, in flight across level 2 only (19 VGPRs fewer: blocks of 16 rows fit
// 128 VGPRs).
template <int TH, bool SKIP, int PD, bool TOL = false>
__global__ __launch_bounds__(T3W * TH) void step3d_two(Two3Args a) {
    __shared__ float lds1[T3<TH>::LDS], lds2[T3<TH>::LDS];
    __shared__ float red[2][TH];
    const int lane = threadIdx.x, wy = __builtin_amdgcn_readfirstlane(threadIdx.y);
    const Blk3 B = blk3_remap();
    const int ox = B.x * T3OX, oy = B.y * T3<TH>::OY;
    const bool live1 = !SKIP || (wy >= 1 && wy < TH - 1), live2 = !SKIP || (wy >= 2 && wy < TH - 2);
    const int x = (((ox - 2 + lane) % a.nx) + a.nx) % a.nx;
    const int y = (((oy - 2 + wy) % a.ny) + a.ny) % a.ny;
    const bool own = lane >= 2 && lane < T3W - 2 && wy >= 2 && wy < TH - 2 && ox + lane - 2 < a.nx &&
                     oy + wy - 2 < a.ny;
    const int zs = a.z0 + B.z * a.seg, ze = min(zs + a.seg, a.zn);
    const long long row = (long long)y * a.px + x;
    float r0a[3] = {0.f, 0.f, 0.f}, r9aa[3] = {0.f, 0.f, 0.f}, r9ba[3] = {0.f, 0.f, 0.f};
    float r0b[3] = {0.f, 0.f, 0.f}, r9ab[3] = {0.f, 0.f, 0.f}, r9bb[3] = {0.f, 0.f, 0.f};
    float zra[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, zrb[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    float u1 = 0.f, u2 = 0.f;
    auto obz = [&](int zz) {  // planes zs-4 .. ze are asked for; only zs-1 .. ze are used
        zz = min(max(zz, -2), a.nz + 1);
        return a.obst[((long long)zz * a.ny + y) * a.nx + x] != 0;
    };
    // input planes are prefetched PD iterations ahead (their loads stay in
    // flight across the two barriers of the current iteration)
    float in[Q3], far[Q3];
    bool ob1 = obz(zs - 3), ob2 = obz(zs - 4);
    {
        const float *pl = a.fin + (long long)(zs - 2) * a.PL + row;
#pragma unroll
        for (int k = 0; k < Q3; ++k) in[k] = pl[k * a.KS];
        if (PD == 2) {
            const float *pf = a.fin + (long long)min(zs - 1, ze + 1) * a.PL + row;
#pragma unroll
            for (int k = 0; k < Q3; ++k) far[k] = pf[k * a.KS];
        }
    }
    for (int j = zs - 2; j <= ze + 1; ++j) {
        float nin[Q3];
        const float *pn = a.fin + (long long)min(j + (PD == 0 ? 1 : PD), ze + 1) * a.PL + row;
        if (PD == 0) {
        } else if (PD == 2) {
#pragma unroll
            for (int k = 0; k < Q3; ++k) nin[k] = far[k];
#pragma unroll
            for (int k = 0; k < Q3; ++k) far[k] = pn[k * a.KS];
        } else {
#pragma unroll
            for (int k = 0; k < Q3; ++k) nin[k] = pn[k * a.KS];
        }
        ob2 = ob1;
        ob1 = obz(j - 1);
        float o1[Q3], o2[Q3];
        const float v1 = level3<TH, TOL>(in, o1, lds1, j, r0a, r9aa, r9ba, zra, lane, wy, ob1, live1, a);
        if (own && j - 1 >= zs && j - 1 < ze) u1 += v1;
        if (PD == 0) {  // level 1 is done with plane j: its registers take plane j + 1
#pragma unroll
            for (int k = 0; k < Q3; ++k) in[k] = pn[k * a.KS];
        }
        const float v2 = level3<TH, TOL>(o1, o2, lds2, j - 1, r0b, r9ab, r9bb, zrb, lane, wy, ob2, live2, a);
        if (own && j - 2 >= zs && j - 2 < ze) {
            u2 += v2;
            float *d = a.fout + (long long)(j - 2) * a.PL + row;
#pragma unroll
            for (int k = 0; k < Q3; ++k) __builtin_nontemporal_store(o2[k], d + k * a.KS);
        }
        if (PD != 0) {
#pragma unroll
            for (int k = 0; k < Q3; ++k) in[k] = nin[k];
        }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        u1 += __shfl_down(u1, off, 64);
        u2 += __shfl_down(u2, off, 64);
    }
    if (lane == 0) {
        red[0][wy] = u1;
        red[1][wy] = u2;
    }
    __syncthreads();
    if (lane == 0 && wy == 0) {
        float b1 = red[0][0], b2 = red[1][0];
#pragma unroll
        for (int i = 1; i < TH; ++i) {
            b1 += red[0][i];
            b2 += red[1][i];
        }
        const int blk = a.blk0 + (B.z * gridDim.y + B.y) * gridDim.x + B.x;
        a.partials[blk] = b1;
        a.partials[a.nblocks + blk] = b2;
    }
}

// ---------------------------------------------------------------------------
// step3d_three: three time steps per pass (single slab).  The same 64 x 12
// block and level3 building block with a third level: level 1 computes plane
// j-1 at t+1, level 2 plane j-2 at t+2, level 3 plane j-3 at t+3 as input
// plane j arrives.  A three-cell ring in x and y is recomputed: owned 58 x 6
// of 64 x 12 loaded cells, three levels of 14 plane slots = 126 KB of LDS (one
// block per CU, three waves per SIMD).  Algorithmic traffic per cell update:
// (19 x 768 loads + 19 x 348 stores) x 4 B / (3 x 348) = 81.2 B instead of
// 98.8 for two steps per pass (152 for one).  Input planes zs-3 .. ze+2: the
// lattice carries three ghost planes each side (GZ3), refreshed from the
// periodic images before every pass.  Same cell3d / cell3dt arithmetic as the
// other passes: bitwise equal to them (and the oracle) in bitwise mode.
constexpr int T3OX3 = T3W - 6;  // owned columns
constexpr int T3TH3 = 12;       // rows (waves) per block
constexpr int T3OY3 = T3TH3 - 6;
constexpr int GZ3 = 3;  // ghost planes each side of every slab lattice (and obst_g)

// Per-level delay lines of the three-step pass in two register sets used on
// alternate planes (the plane loop runs two planes per iteration, set P = 0
// then 1): r0[P ^ 1] / zr[P ^ 1] hold what the previous plane left (speeds 0,
// 1, 2 of the centre plane; its y +- 1 pulls of speeds 3..8), r0[P] / zr[P]
// take this plane's; r9[P] holds the speeds 9, 10, 11 of the plane two back
// and takes this plane's.  (One set per delay line, rotated by copies, cost
// ~45 moves per plane iteration plus ~40 loop-carried copies at the back edge.)
struct Lv3 {
    float r0[2][3], r9[2][3], zr[2][6];
};

// per-thread LDS offsets (floats) of a level's slots, loop-invariant
struct Lds3 {
    int c, ym, yp, ymxm, ypxp, ypxm, ymxp;  // own cell; y-1; y+1; (y-1,x-1); (y+1,x+1); (y+1,x-1); (y-1,x+1)
};

// level3 for the three-step pass: level L (centre plane jz - 1, input plane
// jz), register set P as above, for a wave whose row is live for the first D
// levels (SKIP: D = min(row, 11 - row, 3); every row D = 3 without it).
// Level L publishes its input only while some live row reads it (L <= D + 1:
// the rows beside a live row are live one level less) and computes only
// while live (L <= D); every level meets its barrier.  Liveness is static per
// instantiation, so no path merges a computed with a skipped result (the
// merges had cost a register move per population and level).
// pin / pold: P-ring slots of planes jz and jz - 2 (wave-uniform).
template <int P, int L, int D, bool TOL>
__device__ __forceinline__ float level3p(const float (&in)[Q3], float (&out)[Q3], float *lds, int pin, int pold,
                                         Lv3 &st, const Lds3 &d, bool ob, const Two3Args &a) {
    constexpr int C = T3<T3TH3>::C;
    float *M = lds, *Z = lds + 2 * C, *Pr = lds + 8 * C;
    if constexpr (L <= D + 1) {
        M[d.c] = in[17];
        M[C + d.c] = in[18];
#pragma unroll
        for (int i = 0; i < 6; ++i) Z[i * C + d.c] = in[3 + i];
        Pr[(pin * 2) * C + d.c] = in[12];
        Pr[(pin * 2 + 1) * C + d.c] = in[13];
    }
    __syncthreads();
    if constexpr (L > D) {
        return 0.f;
    } else {
        const float *pp = Pr + pold * 2 * C;  // plane jz - 2
        float s[Q3];
        s[0] = st.r0[P ^ 1][0];
        s[1] = dpp_from_left(st.r0[P ^ 1][1]);
        s[2] = dpp_from_right(st.r0[P ^ 1][2]);
#pragma unroll
        for (int i = 0; i < 6; ++i) s[3 + i] = st.zr[P ^ 1][i];
        // plane jz's y +- 1 pulls of speeds 3..8, for the next plane (each
        // slot is rewritten only after the next barrier of this level)
        st.zr[P][0] = Z[0 * C + d.ym];
        st.zr[P][1] = Z[1 * C + d.yp];
        st.zr[P][2] = Z[2 * C + d.ymxm];
        st.zr[P][3] = Z[3 * C + d.ypxp];
        st.zr[P][4] = Z[4 * C + d.ypxm];
        st.zr[P][5] = Z[5 * C + d.ymxp];
        s[9] = st.r9[P][0];
        s[10] = dpp_from_left(st.r9[P][1]);
        s[11] = dpp_from_right(st.r9[P][2]);
        s[12] = pp[d.ym];
        s[13] = pp[C + d.yp];
        s[14] = in[14];
        s[15] = dpp_from_right(in[15]);
        s[16] = dpp_from_left(in[16]);
        s[17] = M[d.yp];
        s[18] = M[C + d.ym];
        float u;
        if constexpr (TOL)
            u = cell3dt(s, out, ob, a.omo, a.k0, a.k1, a.k2, a.w1, a.w2);
        else
            u = cell3d(s, out, ob, a.omega, a.omo, a.w1, a.w2);
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            st.r9[P][i] = in[9 + i];
            st.r0[P][i] = in[i];
        }
        return u;
    }
}

// The plane loop of one wave (rows live for D levels, see level3p); input
// planes zs-3 .. ze+2, two per iteration (register sets 0 and 1).  Every
// plane base and speed offset is wave-uniform: loads and stores are buffer
// operations on a per-plane descriptor with the speed offset in soffset and
// the lane's cell in voffset (no per-access 64-bit address arithmetic; the
// engine keeps Q3 x KS x 4 B below 2^31 for this pass).
template <int D, bool TOL>
__device__ __forceinline__ void three_rows(const Two3Args &a, const Lds3 &d, float *lds1, float *lds2, float *lds3,
                                           int x, int y, unsigned rowb, bool own, int zs, int ze, float &u1,
                                           float &u2, float &u3) {
    Lv3 s1{}, s2{}, s3{};
    const unsigned nrec = (unsigned)(Q3 * a.KS * 4);
    const int ks4 = (int)(a.KS * 4);
    auto rsrc = [&](const float *base) {
        return __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(base), 0, (int)nrec, 0x00020000);
    };
    auto obz = [&](int zz) {  // planes zs-6 .. ze+1 are asked for; only zs-2 .. ze+1 are used
        zz = min(max(zz, -3), a.nz + 2);
        return a.obst[((long long)zz * a.ny + y) * a.nx + x] != 0;
    };
    float in[Q3];
    auto load = [&](int pl) {
        const auto r = rsrc(a.fin + (long long)pl * a.PL);
#pragma unroll
        for (int k = 0; k < Q3; ++k) in[k] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, (int)rowb, k * ks4, 0));
    };
    bool ob1 = obz(zs - 4), ob2 = obz(zs - 5), ob3 = obz(zs - 6);
    load(zs - 3);
    // P-ring slots (planes mod 3): level L publishes plane j - L + 1 and reads
    // plane j - L - 1 of input plane j
    int sj = (((zs - 3) % 3) + 3) % 3;  // slot of plane j
    auto plane = [&](auto PC, int j) __attribute__((always_inline)) {
        constexpr int P = decltype(PC)::value;
        const int sm1 = sj == 0 ? 2 : sj - 1, sm2 = sj == 2 ? 0 : sj + 1;  // slots of j - 1, j - 2 (j - 3: sj)
        if constexpr (D >= 1) {
            ob3 = ob2;
            ob2 = ob1;
            ob1 = obz(j - 1);
        }
        float o1[Q3], o2[Q3], o3[Q3];
        const float v1 = level3p<P, 1, D, TOL>(in, o1, lds1, sj, sm2, s1, d, ob1, a);
        if (D == 3 && own && j - 1 >= zs && j - 1 < ze) u1 += v1;
        load(min(j + 1, ze + 2));
        const float v2 = level3p<P, 2, D, TOL>(o1, o2, lds2, sm1, sj, s2, d, ob2, a);
        if (D == 3 && own && j - 2 >= zs && j - 2 < ze) u2 += v2;
        const float v3 = level3p<P, 3, D, TOL>(o2, o3, lds3, sm2, sm1, s3, d, ob3, a);
        if constexpr (D == 3) {
            if (own && j - 3 >= zs && j - 3 < ze) {
                u3 += v3;
                const auto r = rsrc(a.fout + (long long)(j - 3) * a.PL);
#pragma unroll
                // plain (temporal) stores: x-neighbouring blocks run on one XCD
                // and each writes a 232-B unaligned row segment, which the L2
                // merges into whole lines before they leave (non-temporal
                // stores: 2.11-2.30 vs 2.07 ms per step at 512^3 tolerance,
                // profiles/r06/d3store/)
                for (int k = 0; k < Q3; ++k) __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(o3[k]), r, (int)rowb, k * ks4, 0);
            }
        }
        sj = sj == 2 ? 0 : sj + 1;
    };
    int j = zs - 3;
    for (; j + 1 <= ze + 2; j += 2) {
        plane(std::integral_constant<int, 0>{}, j);
        plane(std::integral_constant<int, 1>{}, j + 1);
    }
    if (j <= ze + 2) plane(std::integral_constant<int, 0>{}, j);
}

// SKIP: rows no later level reads skip the collision (level 1: rows 1..10,
// level 2: 2..9, level 3: 3..8 live), as step3d_two's SKIP -- each wave runs
// the plane loop instantiated for its row's live depth.
template <bool TOL, bool SKIP>
__global__ __launch_bounds__(T3W *T3TH3) void step3d_three(Two3Args a) {
    __shared__ float lds1[T3<T3TH3>::LDS], lds2[T3<T3TH3>::LDS], lds3[T3<T3TH3>::LDS];
    __shared__ float red[3][T3TH3];
    const int lane = threadIdx.x, wy = __builtin_amdgcn_readfirstlane(threadIdx.y);
    const Blk3 B = blk3_remap();
    const int ox = B.x * T3OX3, oy = B.y * T3OY3;
    const int x = (((ox - 3 + lane) % a.nx) + a.nx) % a.nx;
    const int y = (((oy - 3 + wy) % a.ny) + a.ny) % a.ny;
    const bool own = lane >= 3 && lane < T3W - 3 && wy >= 3 && wy < T3TH3 - 3 && ox + lane - 3 < a.nx &&
                     oy + wy - 3 < a.ny;
    const int zs = a.z0 + B.z * a.seg, ze = min(zs + a.seg, a.zn);
    const unsigned rowb = (unsigned)(y * a.px + x) * 4u;  // byte offset of the lane's cell in a speed plane
    Lds3 d;
    {
        const int wm = max(wy - 1, 0) * T3W, wp = min(wy + 1, T3TH3 - 1) * T3W;
        const int lm = max(lane - 1, 0), lp = min(lane + 1, T3W - 1);
        d.c = wy * T3W + lane;
        d.ym = wm + lane;
        d.yp = wp + lane;
        d.ymxm = wm + lm;
        d.ypxp = wp + lp;
        d.ypxm = wp + lm;
        d.ymxp = wm + lp;
    }
    float u1 = 0.f, u2 = 0.f, u3 = 0.f;
    const int depth = SKIP ? min(min(wy, T3TH3 - 1 - wy), 3) : 3;  // wave-uniform
    switch (depth) {
        case 0: three_rows<0, TOL>(a, d, lds1, lds2, lds3, x, y, rowb, own, zs, ze, u1, u2, u3); break;
        case 1: three_rows<1, TOL>(a, d, lds1, lds2, lds3, x, y, rowb, own, zs, ze, u1, u2, u3); break;
        case 2: three_rows<2, TOL>(a, d, lds1, lds2, lds3, x, y, rowb, own, zs, ze, u1, u2, u3); break;
        default: three_rows<3, TOL>(a, d, lds1, lds2, lds3, x, y, rowb, own, zs, ze, u1, u2, u3); break;
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        u1 += __shfl_down(u1, off, 64);
        u2 += __shfl_down(u2, off, 64);
        u3 += __shfl_down(u3, off, 64);
    }
    if (lane == 0) {
        red[0][wy] = u1;
        red[1][wy] = u2;
        red[2][wy] = u3;
    }
    __syncthreads();
    if (lane == 0 && wy == 0) {
        float b1 = red[0][0], b2 = red[1][0], b3 = red[2][0];
#pragma unroll
        for (int i = 1; i < T3TH3; ++i) {
            b1 += red[0][i];
            b2 += red[1][i];
            b3 += red[2][i];
        }
        const int blk = a.blk0 + (B.z * gridDim.y + B.y) * gridDim.x + B.x;
        a.partials[blk] = b1;
        a.partials[a.nblocks + blk] = b2;
        a.partials[2 * a.nblocks + blk] = b3;
    }
}

__global__ __launch_bounds__(BLOCK) void reduce3d(const float *partials, int n, float *av_local, int t) {
    __shared__ float lds[BLOCK / 64];
    const float v = sum_partials_n<BLOCK>(partials, n, lds);
    if (threadIdx.x == 0) av_local[t] = v;
}

// every plane (ghosts included) at rest equilibrium
__global__ __launch_bounds__(BLOCK) void init3d(float *base, long long planes, long long KS, long long PL, float c0,
                                               float c1, float c2) {
    const long long i = (long long)blockIdx.x * BLOCK + threadIdx.x;
    if (i >= planes * KS) return;
    const long long z = i / KS, r = i - z * KS;
    float *d = base + z * PL + r;
    d[0] = c0;
#pragma unroll
    for (int k = 1; k < Q3; ++k) d[k * KS] = (k <= 4 || k == 9 || k == 14) ? c1 : c2;
}

// AoS [nzs][ny][nx][19] staging <-> lattice interior
__global__ __launch_bounds__(BLOCK) void aos_to_soa3d(const float *aos, float *f, long long PL, long long KS, int px,
                                                     int nx, int ny, long long n) {
    const long long i = (long long)blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    const long long zy = i / nx;
    const int x = (int)(i - zy * nx);
    const int y = (int)(zy % ny);
    const long long z = zy / ny;
    float *d = f + z * PL + (long long)y * px + x;
#pragma unroll
    for (int k = 0; k < Q3; ++k) d[k * KS] = aos[i * Q3 + k];
}

__global__ __launch_bounds__(BLOCK) void soa_to_aos3d(const float *f, float *aos, long long PL, long long KS, int px,
                                                     int nx, int ny, long long n) {
    const long long i = (long long)blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    const long long zy = i / nx;
    const int x = (int)(i - zy * nx);
    const int y = (int)(zy % ny);
    const long long z = zy / ny;
    const float *s = f + z * PL + (long long)y * px + x;
#pragma unroll
    for (int k = 0; k < Q3; ++k) aos[i * Q3 + k] = s[k * KS];
}

hipError_t launch_debug_spin(int microseconds, hipStream_t s);  // lbm_kernels.hip
}  // namespace lbm

using namespace lbm;

namespace {

// The ordered posts of one z slab's ghost exchange (RCCL pairs them by
// order inside one ncclGroupStart/End): send up (dir 0, +z) to rank+1, send
// down (dir 1, -z) to rank-1, receive the below ghosts (dir 1) from rank-1,
// receive the above ghosts (dir 0) from rank+1 -- periodic in z.  `floats`
// per message: 5 speed planes for a one-step launch, n whole planes (all 19
// speeds) for an n-step pass.  exchange() / exchange_planes() post exactly
// this list; lbm3d_exchange_schedule exports it.
std::array<lbm_xfer, 4> slab_posts(int rank, int world, long long floats) {
    const int up = (rank + 1) % world, down = (rank + world - 1) % world;
    return {lbm_xfer{LBM_XFER_SEND, 0, up, 0, floats}, lbm_xfer{LBM_XFER_SEND, 1, down, 0, floats},
            lbm_xfer{LBM_XFER_RECV, 1, down, 0, floats}, lbm_xfer{LBM_XFER_RECV, 0, up, 0, floats}};
}

struct fail3 : std::runtime_error {
    int code;
    fail3(int c, const std::string &m) : std::runtime_error(m), code(c) {}
};

#define H3(expr)                                                                                          \
    do {                                                                                                  \
        hipError_t e_ = (expr);                                                                           \
        if (e_ != hipSuccess) throw fail3(LBM_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)
#define N3(expr)                                                                                          \
    do {                                                                                                  \
        ncclResult_t r_ = (expr);                                                                         \
        if (r_ != ncclSuccess) throw fail3(LBM_E_RCCL, std::string(#expr) + ": " + ncclGetErrorString(r_)); \
    } while (0)

struct Slab {
    int id = 0, dev = 0, z0 = 0, nzs = 0;
    float *f[2] = {nullptr, nullptr};  // allocations (ghost plane below first)
    bool f_joint = false;              // f[1] lies in f[0]'s allocation (LBM_LATTICE_PAD)
    float *o[2] = {nullptr, nullptr};  // origins: plane z = 0
    uint8_t *obst = nullptr;
    uint8_t *obst_g = nullptr;   // [nzs + 6][ny][nx]: obst with three image planes each side (two/three-step kernels)
    float *partials = nullptr;
    int nblk_all = 0, nblk_bnd = 0, nblk_int = 0;
    float *partials2 = nullptr;  // two-step kernel: [2][nblk_two]
    int nblk_two = 0;
    float *partials3 = nullptr;  // three-step kernel (single slab): [3][nblk_three]
    int nblk_three = 0;
    float *av_local = nullptr;
    int av_cap = 0;
    int cur = 0;
    hipStream_t s_comp = nullptr, s_bnd = nullptr, s_comm = nullptr;
    hipEvent_t ev_b = nullptr, ev_i = nullptr, ev_x = nullptr, ev_end = nullptr;
};

}  // namespace

struct lbm3d_handle {
    lbm3d_params p{};
    int parts = 1, transport = LBM_TRANSPORT_LOCAL, rank = 0, world = 1;
    int px = 0;
    long long KS = 0, PL = 0;
    bool pair = true;  // column-pair kernel (nx even; LBM3D_PAIR=0 forces the one-cell kernel)
    // tuned at 512^3 (profiles/r01/d3q19/ab_zb_nt.log): 2 planes per block,
    // non-temporal stores (the lattice written now is read a whole step later)
    int zb = 2;        // LBM3D_ZB: planes per block of the pair kernel (1, 2, 4, 8)
    bool nt = true;    // LBM3D_NT: non-temporal output stores
    bool two = true;   // LBM3D_TWO: two steps per pass (step3d_two), single slab or z slabs
    // LBM3D_THREE: three steps per pass (step3d_three), one slab or z slabs of
    // >= 6 planes (needs two);
    // default (-1): both modes since round 4 (with skip3) -- 512^3, skip3 on:
    // tolerance 55.4-55.6 GLUPS, bitwise 51.2-51.3 vs 44.1-45.2 for two-step
    // passes (profiles/r04/d3q19/ab_skip3.log); round 3, skip3 off, had kept
    // bitwise on two-step passes (43.9-44.1 vs 44.6-45.0: the divisions made
    // the third level's recompute VALU-bound)
    int three = -1;
    int seg3 = 64;     // LBM3D_SEG3: z planes per block of the three-step kernel
    int seg = 64;      // LBM3D_SEG: z planes per block of the two-step kernel (32-128 equal within noise at 512^3)
    int th = 12;       // LBM3D_TH: rows (waves) per block of the two-step kernel (12 only since round 3)
    bool skip = false; // LBM3D_SKIP: waves skip the collisions of rows no later level reads (not faster)
    // LBM3D_SKIP3: the same in the three-step pass -- there it pays (default on):
    // the live rows per level (10, 8, 6 of 12) spread over the 4 SIMDs as
    // 3 + 2 + 2 wave-collisions on the busiest SIMD instead of 3 + 3 + 3;
    // 512^3 tolerance 55.4-55.6 vs 45.6-50.0 GLUPS, bitwise 51.2-51.3 vs 43.7-43.9
    bool skip3 = true;
    // LBM3D_PD: input planes in flight in the two-step kernel -- 0 (default): the
    // next plane loaded once level 1 has consumed the current one (44.7 vs
    // 38.6-42.5 GLUPS at 512^3 for 1, profiles/r03/d3q19/ab_pd.log); 1, 2
    int pd = 0;
    long long kspad = 0;  // LBM3D_KSPAD: floats appended to each speed plane (multiple of 64)
    const char *lattice_pad = nullptr;  // LBM_LATTICE_PAD (debug knob)
    bool poison = false;  // LBM_POISON=1: fresh allocations filled with NaN bytes
    int probe_tries = 6;  // LBM3D_PLACEMENT_TRIES: lattice pairs the placement probe times (1 = off)
    long long probe_min_cells = 1LL << 26;  // LBM3D_PROBE_MIN_CELLS: smallest single slab probed
    bool probe_three = true;                 // LBM3D_PROBE_THREE=0: three-step engines skip the probe (A/B)
    bool probe_log = false;  // LBM_PLACEMENT_LOG: print the probe's per-pair times
    // ordering regression knobs (debug only, tests/test_gpu_ordering.py): slab
    // LBM_DEBUG_DELAY_SUB's boundary and interior launches are each preceded
    // by a stall of LBM_DEBUG_DELAY_US on their stream
    int delay_sub = -1, delay_us = 0;
    bool tolerance = false;  // LBM_FLAG_TOLERANCE: the two-step passes use cell3dt (not bitwise)
    std::vector<Slab> slabs;
    std::vector<int> all_z0, all_nz;
    ncclComm_t comm = nullptr;
    int64_t free_cells = 0;
    bool loaded = false;
    int last_steps = 0;
    double last_seconds = 0.0;
    hipEvent_t t0 = nullptr, t1 = nullptr;
    std::string err;

    // several slabs, or RCCL transport (then even one rank sends its faces to
    // itself through RCCL: the exchange path is testable on one GPU)
    bool multi() const { return parts > 1 || transport == LBM_TRANSPORT_RCCL; }
    float w1() const { return p.density * p.accel / 18.f; }
    float w2() const { return p.density * p.accel / 36.f; }

    void create(const lbm3d_params *prm, const uint8_t *obstacles, const lbm_config &cfg) {
        p = *prm;
        if (p.nx <= 0 || p.ny <= 0 || p.nz <= 0 || p.max_iters < 0)
            throw fail3(LBM_E_INVALID, "nx, ny, nz must be > 0 and max_iters >= 0");
        if (!obstacles) throw fail3(LBM_E_INVALID, "obstacles must not be NULL");
        parts = cfg.parts > 0 ? cfg.parts : 1;
        transport = cfg.transport;
        tolerance = (cfg.flags & LBM_FLAG_TOLERANCE) != 0;
        if (parts > p.nz) throw fail3(LBM_E_INVALID, "more z slabs than planes");
        int ndev = 0;
        H3(hipGetDeviceCount(&ndev));
        if (ndev <= 0) throw fail3(LBM_E_HIP, "no HIP device visible");
        const long long cells = (long long)p.nx * p.ny * p.nz;
        free_cells = 0;
        for (long long i = 0; i < cells; ++i) free_cells += obstacles[i] ? 0 : 1;
        px = (p.nx + 15) / 16 * 16;  // 64-byte rows
        // tuning knobs only with LBM_DEBUG_KNOBS=1 (as the 2-D engine); LBM_POISON always
        const char *dk = getenv("LBM_DEBUG_KNOBS");
        const bool knobs = dk && *dk && atoi(dk) != 0;
        const char *po = getenv("LBM_POISON");
        poison = po && *po && atoi(po) != 0;
        auto knob = [&](const char *name) -> const char * {
            const char *v = knobs ? getenv(name) : nullptr;
            return (v && *v) ? v : nullptr;
        };
        const char *pe = knob("LBM3D_PAIR");
        pair = p.nx % 2 == 0 && !(pe && atoi(pe) == 0);
        if (const char *z = knob("LBM3D_ZB")) zb = (atoi(z) == 1 || atoi(z) == 4 || atoi(z) == 8) ? atoi(z) : 2;
        if (const char *n = knob("LBM3D_NT")) nt = atoi(n) != 0;
        if (const char *t = knob("LBM3D_TWO")) two = atoi(t) != 0;
        if (const char *g = knob("LBM3D_SEG")) seg = std::max(1, atoi(g));
        if (const char *t = knob("LBM3D_THREE")) three = atoi(t) != 0 ? 1 : 0;
        if (const char *g = knob("LBM3D_SEG3")) seg3 = std::max(1, atoi(g));
        if (const char *h = knob("LBM3D_TH")) th = atoi(h);
        if (const char *k = knob("LBM3D_SKIP")) skip = atoi(k) != 0;
        if (const char *k = knob("LBM3D_SKIP3")) skip3 = atoi(k) != 0;
        if (const char *d = knob("LBM3D_PD")) pd = atoi(d);
        if (const char *k = knob("LBM3D_KSPAD")) kspad = (std::max(0LL, atoll(k)) + 63) / 64 * 64;
        lattice_pad = knob("LBM_LATTICE_PAD");
        if (const char *t = knob("LBM3D_PLACEMENT_TRIES")) probe_tries = std::max(1, atoi(t));
        if (const char *m = knob("LBM3D_PROBE_MIN_CELLS")) probe_min_cells = std::max(0LL, atoll(m));
        if (const char *pt = knob("LBM3D_PROBE_THREE")) probe_three = atoi(pt) != 0;
        probe_log = knob("LBM_PLACEMENT_LOG") != nullptr;
        if (const char *d = knob("LBM_DEBUG_DELAY_SUB")) delay_sub = atoi(d);
        if (const char *d = knob("LBM_DEBUG_DELAY_US")) delay_us = std::min(std::max(atoi(d), 0), 100000);
        if (tolerance) {  // the tolerance pass exists for the default block only
            th = 12;
            skip = false;
            pd = 0;
        }
        // the two-step kernel is instantiated for these (rows, skip, prefetch)
        // combinations only; anything else is rejected here, never launched as
        // a different template (blocks of 64 x th threads, at most 960)
        if (two_variant(th, skip, pd) < 0)
            throw fail3(LBM_E_INVALID, "unsupported two-step block: LBM3D_TH " + std::to_string(th) + ", SKIP " +
                                           std::to_string(skip ? 1 : 0) + ", PD " + std::to_string(pd));
        KS = (long long)p.ny * px + kspad;
        PL = (long long)Q3 * KS;
        // round-robin z extents (StructuredGridUtils.hpp:161-165 rule, in z)
        all_z0.assign(parts, 0);
        all_nz.assign(parts, p.nz / parts);
        for (int i = 0; i < p.nz % parts; ++i) all_nz[i]++;
        for (int i = 1; i < parts; ++i) all_z0[i] = all_z0[i - 1] + all_nz[i - 1];
        std::vector<int> mine;
        if (transport == LBM_TRANSPORT_RCCL) {
            if (cfg.world != parts || cfg.rank < 0 || cfg.rank >= parts)
                throw fail3(LBM_E_INVALID, "RCCL transport needs world == parts and 0 <= rank < world");
            if (!cfg.rccl_unique_id) throw fail3(LBM_E_INVALID, "RCCL transport needs rccl_unique_id");
            rank = cfg.rank;
            world = cfg.world;
            mine.push_back(rank);
        } else if (transport == LBM_TRANSPORT_LOCAL) {
            for (int i = 0; i < parts; ++i) mine.push_back(i);
        } else {
            throw fail3(LBM_E_INVALID, "unknown transport");
        }
        slabs.resize(mine.size());
        for (size_t k = 0; k < mine.size(); ++k) {
            Slab &s = slabs[k];
            s.id = mine[k];
            s.z0 = all_z0[s.id];
            s.nzs = all_nz[s.id];
            if (transport == LBM_TRANSPORT_RCCL)
                s.dev = (cfg.devices && cfg.num_devices > 0) ? cfg.devices[0] : rank % ndev;
            else
                s.dev = (cfg.devices && cfg.num_devices > 0) ? cfg.devices[s.id % cfg.num_devices] : s.id % ndev;
            if (s.dev < 0 || s.dev >= ndev) throw fail3(LBM_E_INVALID, "device index out of range");
            alloc(s, obstacles);
        }
        if (transport == LBM_TRANSPORT_RCCL) {
            ncclUniqueId id;
            memcpy(&id, cfg.rccl_unique_id, sizeof(id));
            H3(hipSetDevice(slabs[0].dev));
            N3(ncclCommInitRank(&comm, world, id, rank));
        } else if (slabs.size() > 1) {
            for (auto &a : slabs)
                for (auto &b : slabs)
                    if (a.dev != b.dev) {
                        int can = 0;
                        H3(hipDeviceCanAccessPeer(&can, a.dev, b.dev));
                        if (can) {
                            H3(hipSetDevice(a.dev));
                            hipError_t e = hipDeviceEnablePeerAccess(b.dev, 0);
                            if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) H3(e);
                            (void)hipGetLastError();
                        }
                    }
        }
        ensure_av(std::max(p.max_iters, 1));
        H3(hipSetDevice(slabs[0].dev));
        H3(hipEventCreate(&t0));
        H3(hipEventCreate(&t1));
        placement_probe();
    }

    // Placement probe (the D3Q19 counterpart of lbm_engine.hip's; DESIGN.md
    // §4.9): the two-step pass runs at an engine-to-engine spread of about
    // +-5 % at 512^3 fixed by where the lattices land (39.9-44.2 GLUPS over
    // six engines in one process, profiles/r03/d3q19/spread.log).  A single
    // slab of at least 2^26 cells allocates up to probe_tries lattice pairs
    // (at most 128 GB held at once: six at 512^3), times the engine's passes
    // on each (constant populations; one warm-up round, then the best of two
    // interleaved rounds), keeps the fastest pair and frees the rest; the kept
    // pair is filled as a fresh allocation is, so the engine's state is as if
    // the probe had not run.  Failures inside free every extra candidate and
    // restore the original pair.
    // Scope: single-slab engines; each candidate is timed with the engine's
    // own pass form (three-step passes, the default in both numerics since
    // round 4, or two-step ones).  Round 4 first timed two-step passes for
    // three-step engines and gained nothing (profiles/r04/prof1/d3_probe.log);
    // timing their own three-step passes it keeps the fast placement
    // (7.1-7.2 vs 7.4-7.8 ms per tolerance pass): 55.0-55.9 GLUPS over four
    // engines against 51.5-55.4 unprobed (profiles/r04/d3q19/ab_probe3.log).
    // LBM3D_PROBE_THREE=0 skips the probe for three-step engines (A/B).
    void placement_probe() {
        if (multi() || !use_two() || (use_three() && !probe_three) || slabs.size() != 1) return;
        Slab &s = slabs[0];
        if ((long long)p.nx * p.ny * p.nz < probe_min_cells || s.f_joint) return;
        const size_t floats = (size_t)(s.nzs + 2 * GZ3) * PL;
        const size_t pair_bytes = 2 * sizeof(float) * floats;
        const int cap = (int)std::max<size_t>(1, (128ull << 30) / pair_bytes);
        const int tries = std::min({probe_tries, 8, cap});
        if (tries <= 1) return;
        H3(hipSetDevice(s.dev));
        std::vector<std::array<float *, 2>> cand{{s.f[0], s.f[1]}};
        size_t keep = 0;
        auto set_pair = [&](size_t c) {
            for (int k = 0; k < 2; ++k) {
                s.f[k] = cand[c][k];
                s.o[k] = s.f[k] + GZ3 * PL;
            }
            s.cur = 0;
        };
        hipEvent_t e0 = nullptr, e1 = nullptr;
        const bool three_probe = use_three();
        try {
            for (int c = 1; c < tries; ++c) {
                std::array<float *, 2> f{nullptr, nullptr};
                if (hipMalloc(&f[0], sizeof(float) * floats) != hipSuccess) { (void)hipGetLastError(); break; }
                if (hipMalloc(&f[1], sizeof(float) * floats) != hipSuccess) {
                    (void)hipGetLastError();
                    (void)hipFree(f[0]);
                    break;
                }
                cand.push_back(f);
            }
            for (auto &f : cand)  // 0.05f everywhere: rho = 0.95, no tiny-density path
                for (float *q : f) H3(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(q), 0x3d4ccccd, floats, s.s_comp));
            H3(hipEventCreate(&e0));
            H3(hipEventCreate(&e1));
            std::vector<float> best(cand.size(), 1e30f);
            for (int round = 0; round < 3; ++round)
                for (size_t c = 0; c < cand.size(); ++c) {
                    set_pair(c);
                    H3(hipEventRecord(e0, s.s_comp));
                    for (int i = 0; i < 2; ++i) {  // the engine's own pass form
                        if (three_probe)
                            launch_three(s, 0, s.nzs, 0, s.s_comp);
                        else
                            launch_two(s, 0, s.nzs, 0, s.s_comp);
                        s.cur ^= 1;
                    }
                    H3(hipEventRecord(e1, s.s_comp));
                    H3(hipEventSynchronize(e1));
                    float ms = 0.f;
                    H3(hipEventElapsedTime(&ms, e0, e1));
                    if (round > 0) best[c] = std::min(best[c], ms / 2);  // round 0: clock warm-up
                }
            for (size_t c = 1; c < cand.size(); ++c)
                if (best[c] < best[keep]) keep = c;
            if (probe_log) {
                fprintf(stderr, "lbm3d placement probe (%dx%dx%d): ms per %s-step pass", p.nx, p.ny, p.nz,
                        three_probe ? "three" : "two");
                for (float v : best) fprintf(stderr, " %.4f", v);
                fprintf(stderr, "; kept pair %zu\n", keep);
            }
            for (size_t c = 0; c < cand.size(); ++c)
                if (c != keep)
                    for (float *&q : cand[c]) {
                        (void)hipFree(q);
                        q = nullptr;
                    }
            set_pair(keep);
            for (float *q : s.f) fill_fresh(q, sizeof(float) * floats, s.s_comp);
            H3(hipEventDestroy(e0));
            H3(hipEventDestroy(e1));
        } catch (...) {
            // the handle keeps exactly one pair: the original while it exists, else the kept one
            const size_t own = cand[0][0] ? 0 : keep;
            for (size_t c = 0; c < cand.size(); ++c)
                if (c != own)
                    for (float *&q : cand[c])
                        if (q) {
                            (void)hipFree(q);
                            q = nullptr;
                        }
            set_pair(own);
            if (e0) (void)hipEventDestroy(e0);
            if (e1) (void)hipEventDestroy(e1);
            throw;
        }
    }

    int blocks_for(int planes) const {
        if (pair)
            return ((p.nx + 2 * B3X - 1) / (2 * B3X)) * ((p.ny + B3Y - 1) / B3Y) * ((std::max(planes, 0) + zb - 1) / zb);
        return ((p.nx + B3X - 1) / B3X) * ((p.ny + B3Y - 1) / B3Y) * std::max(planes, 0);
    }

    void alloc(Slab &s, const uint8_t *obstacles) {
        H3(hipSetDevice(s.dev));
        // streams first: every initial fill below is ordered on s_comp (a
        // null-stream hipMemset is not ordered with these non-blocking streams)
        H3(hipStreamCreateWithFlags(&s.s_comp, hipStreamNonBlocking));
        H3(hipStreamCreateWithFlags(&s.s_comm, hipStreamNonBlocking));
        int lo = 0, hi = 0;
        H3(hipDeviceGetStreamPriorityRange(&lo, &hi));
        H3(hipStreamCreateWithPriority(&s.s_bnd, hipStreamNonBlocking, hi));
        for (hipEvent_t *e : {&s.ev_b, &s.ev_i, &s.ev_x, &s.ev_end}) H3(hipEventCreateWithFlags(e, hipEventDisableTiming));
        // three ghost planes below and above (the three-step kernel reads all of them)
        const size_t floats = (size_t)(s.nzs + 2 * GZ3) * PL;
        const char *lp = lattice_pad;
        if (lp && *lp) {
            // both lattices in one allocation, the second pad bytes (rounded to
            // 256 B) after the end of the first (see lbm_engine.hip alloc_sub)
            const size_t second = floats + (size_t)(std::max(0LL, atoll(lp)) + 255) / 256 * 64;
            const size_t n = (second + floats) * sizeof(float);
            H3(hipMalloc(&s.f[0], n));
            fill_fresh(s.f[0], n, s.s_comp);
            s.f[1] = s.f[0] + second;
            s.f_joint = true;
        } else {
            for (int k = 0; k < 2; ++k) {
                H3(hipMalloc(&s.f[k], floats * sizeof(float)));
                fill_fresh(s.f[k], floats * sizeof(float), s.s_comp);
            }
        }
        for (int k = 0; k < 2; ++k) s.o[k] = s.f[k] + GZ3 * PL;
        const size_t ob = (size_t)s.nzs * p.ny * p.nx, plane = (size_t)p.ny * p.nx;
        H3(hipMalloc(&s.obst, ob + 256));
        H3(hipMemcpy(s.obst, obstacles + (size_t)s.z0 * plane, ob, hipMemcpyHostToDevice));
        H3(hipMalloc(&s.obst_g, (size_t)(s.nzs + 2 * GZ3) * plane + 256));
        for (int z = -GZ3; z < s.nzs + GZ3; ++z) {  // global periodic images (the neighbour slabs' planes)
            const int gz = ((s.z0 + z) % p.nz + p.nz) % p.nz;
            H3(hipMemcpy(s.obst_g + (size_t)(z + GZ3) * plane, obstacles + (size_t)gz * plane, plane,
                         hipMemcpyHostToDevice));
        }
        // multi: two one-plane boundary launches, then the interior launch
        s.nblk_bnd = multi() ? (s.nzs >= 2 ? 2 : 1) * blocks_for(1) : 0;
        s.nblk_int = multi() ? blocks_for(s.nzs - 2) : 0;
        s.nblk_all = multi() ? s.nblk_bnd + s.nblk_int : blocks_for(s.nzs);
        H3(hipMalloc(&s.partials, sizeof(float) * (size_t)(s.nblk_all + 64)));
        fill_fresh(s.partials, sizeof(float) * (size_t)(s.nblk_all + 64), s.s_comp);
        s.nblk_two = 0;
        for (const auto &r : two_ranges(s)) s.nblk_two += two_blocks(r.first, r.second);
        H3(hipMalloc(&s.partials2, sizeof(float) * (2 * (size_t)std::max(s.nblk_two, 1) + 64)));
        fill_fresh(s.partials2, sizeof(float) * (2 * (size_t)std::max(s.nblk_two, 1) + 64), s.s_comp);
        s.nblk_three = 0;
        for (const auto &r : three_ranges(s)) s.nblk_three += three_blocks(r.first, r.second);
        if (s.nblk_three > 0) {
            H3(hipMalloc(&s.partials3, sizeof(float) * (3 * (size_t)s.nblk_three + 64)));
            fill_fresh(s.partials3, sizeof(float) * (3 * (size_t)s.nblk_three + 64), s.s_comp);
        }
    }

    // Initial fill of a fresh allocation on `st`, waited for: zero, or with
    // LBM_POISON=1 all-ones bytes (NaN floats) -- a read of anything the
    // engine did not write then shows up as NaN (tests/test_poison.py).
    void fill_fresh(void *ptr, size_t bytes, hipStream_t st) const {
        H3(hipMemsetAsync(ptr, poison ? 0xFF : 0, bytes, st));
        H3(hipStreamSynchronize(st));
    }

    // Output plane ranges of one two-step pass of slab s, in launch order.
    // Single slab: all planes.  z slabs: the two boundary pairs [0, 2) and
    // [nzs-2, nzs) first (their outputs are the next pass's exchanged ghost
    // planes), then the interior [2, nzs-2), which reads no ghost plane and
    // runs while the exchange moves.
    std::vector<std::pair<int, int>> two_ranges(const Slab &s) const {
        if (!multi() || s.nzs < 4) return {{0, s.nzs}};
        std::vector<std::pair<int, int>> r = {{0, 2}, {s.nzs - 2, s.nzs}};
        if (s.nzs > 4) r.push_back({2, s.nzs - 2});
        return r;
    }
    // switch key of the instantiated step3d_two<TH, SKIP, PD> variants, -1 if none:
    // 12 rows without skip, late load (default) or one plane prefetched.  Blocks
    // of 14-16 rows, the row skip and two prefetched planes were measured and
    // removed (profiles/r02/d3q19/ab_two_th_skip_pd.log, profiles/r03/d3q19/ab_pd.log).
    static int two_variant(int th, bool skip, int pd) {
        return (th == 12 && !skip && (pd == 0 || pd == 1)) ? pd : -1;
    }
    int two_blocks(int z0, int zn) const {
        return ((p.nx + T3OX - 1) / T3OX) * ((p.ny + th - 5) / (th - 4)) * ((zn - z0 + seg - 1) / seg);
    }
    // two-step passes: one slab, or z slabs of at least 4 planes (ghosts are 2 planes of the neighbours)
    bool use_two() const {
        if (!two) return false;
        if (!multi()) return true;
        for (int n : all_nz)
            if (n < 4) return false;
        return true;
    }

    void launch_two(Slab &s, int z0, int zn, int blk0, hipStream_t st) {
        if (zn <= z0) return;
        Two3Args a{};
        a.fin = s.o[s.cur];
        a.fout = s.o[1 - s.cur];
        a.obst = s.obst_g + (size_t)GZ3 * p.ny * p.nx;
        a.PL = PL;
        a.KS = KS;
        a.px = px;
        a.nx = p.nx;
        a.ny = p.ny;
        a.nz = s.nzs;
        a.seg = seg;
        a.z0 = z0;
        a.zn = zn;
        a.omega = p.omega;
        a.omo = 1 - p.omega;
        a.w1 = w1();
        a.w2 = w2();
        a.k0 = p.omega * (1.f / 3.f);
        a.k1 = p.omega * (1.f / 18.f);
        a.k2 = p.omega * (1.f / 36.f);
        a.partials = s.partials2;
        a.nblocks = s.nblk_two;
        a.blk0 = blk0;
        const dim3 g((p.nx + T3OX - 1) / T3OX, (p.ny + th - 5) / (th - 4), (zn - z0 + seg - 1) / seg);
        const dim3 b(T3W, th);
        if (tolerance) {  // the default block only (12 rows, no skip, late load)
            hipLaunchKernelGGL((step3d_two<12, false, 0, true>), g, b, 0, st, a);
            H3(hipGetLastError());
            return;
        }
        switch (two_variant(th, skip, pd)) {
            case 0: hipLaunchKernelGGL((step3d_two<12, false, 0>), g, b, 0, st, a); break;
            case 1: hipLaunchKernelGGL((step3d_two<12, false, 1>), g, b, 0, st, a); break;
            default: throw fail3(LBM_E_INTERNAL, "unvalidated two-step variant");
        }
        H3(hipGetLastError());
    }

    // three-step passes: one slab, or z slabs of at least 6 planes (ghosts are
    // 3 planes of the neighbours, exchanged once per pass)
    bool use_three() const {
        if (three == 0 || !use_two()) return false;
        // step3d_three addresses a plane's speeds by 32-bit buffer offsets
        if ((long long)Q3 * KS * 4 >= (1LL << 31)) return false;
        if (!multi()) return true;
        for (int n : all_nz)
            if (n < 6) return false;
        return true;
    }
    int three_blocks(int z0, int zn) const {
        return ((p.nx + T3OX3 - 1) / T3OX3) * ((p.ny + T3OY3 - 1) / T3OY3) * ((zn - z0 + seg3 - 1) / seg3);
    }
    // output plane ranges of one three-step pass, in launch order (as two_ranges)
    std::vector<std::pair<int, int>> three_ranges(const Slab &s) const {
        if (!multi() || s.nzs < 6) return {{0, s.nzs}};
        std::vector<std::pair<int, int>> r = {{0, 3}, {s.nzs - 3, s.nzs}};
        if (s.nzs > 6) r.push_back({3, s.nzs - 3});
        return r;
    }

    void launch_three(Slab &s, int z0, int zn, int blk0, hipStream_t st) {
        if (zn <= z0) return;
        Two3Args a{};
        a.fin = s.o[s.cur];
        a.fout = s.o[1 - s.cur];
        a.obst = s.obst_g + (size_t)GZ3 * p.ny * p.nx;
        a.PL = PL;
        a.KS = KS;
        a.px = px;
        a.nx = p.nx;
        a.ny = p.ny;
        a.nz = s.nzs;
        a.seg = seg3;
        a.z0 = z0;
        a.zn = zn;
        a.omega = p.omega;
        a.omo = 1 - p.omega;
        a.w1 = w1();
        a.w2 = w2();
        a.k0 = p.omega * (1.f / 3.f);
        a.k1 = p.omega * (1.f / 18.f);
        a.k2 = p.omega * (1.f / 36.f);
        a.partials = s.partials3;
        a.nblocks = s.nblk_three;
        a.blk0 = blk0;
        const dim3 g((p.nx + T3OX3 - 1) / T3OX3, (p.ny + T3OY3 - 1) / T3OY3, (zn - z0 + seg3 - 1) / seg3);
        const dim3 b(T3W, T3TH3);
        if (tolerance && skip3)
            hipLaunchKernelGGL((step3d_three<true, true>), g, b, 0, st, a);
        else if (tolerance)
            hipLaunchKernelGGL((step3d_three<true, false>), g, b, 0, st, a);
        else if (skip3)
            hipLaunchKernelGGL((step3d_three<false, true>), g, b, 0, st, a);
        else
            hipLaunchKernelGGL((step3d_three<false, false>), g, b, 0, st, a);
        H3(hipGetLastError());
    }

    // three-step pass (single slab): ghost planes -3..-1, nz..nz+2 of the
    // current lattice (periodic images, all 19 speeds), step3d_three, then the
    // three steps' |u|
    void reduce_three(Slab &s, int t, hipStream_t st) {
        for (int l = 0; l < 3; ++l)
            hipLaunchKernelGGL(reduce3d, dim3(1), dim3(BLOCK), 0, st, s.partials3 + (size_t)l * s.nblk_three,
                               s.nblk_three, s.av_local, t + l);
        H3(hipGetLastError());
    }

    // Three steps of every slab (z slabs): as step_two_multi with three-plane
    // boundary ranges and a three-plane exchange.
    void step_three_multi(int t) {
        for (auto &s : slabs) {
            H3(hipSetDevice(s.dev));
            H3(hipStreamWaitEvent(s.s_bnd, s.ev_i, 0));
            wait_x(s, s.s_bnd);
            stall(s, s.s_bnd);
            const auto r = three_ranges(s);
            int blk = 0;
            for (size_t i = 0; i < r.size() && i < 2; ++i) {
                launch_three(s, r[i].first, r[i].second, blk, s.s_bnd);
                blk += three_blocks(r[i].first, r[i].second);
            }
            H3(hipEventRecord(s.ev_b, s.s_bnd));
        }
        exchange_planes(1 - slabs[0].cur, 3, true);
        for (auto &s : slabs) {
            H3(hipSetDevice(s.dev));
            const auto r = three_ranges(s);
            stall(s, s.s_comp);
            if (r.size() > 2)
                launch_three(s, r[2].first, r[2].second,
                             three_blocks(r[0].first, r[0].second) + three_blocks(r[1].first, r[1].second), s.s_comp);
            H3(hipStreamWaitEvent(s.s_comp, s.ev_b, 0));
            reduce_three(s, t, s.s_comp);
            H3(hipEventRecord(s.ev_i, s.s_comp));
            s.cur ^= 1;
        }
    }

    void step_three(int t) {
        if (multi()) {
            step_three_multi(t);
            return;
        }
        Slab &s = slabs[0];
        const size_t bytes = sizeof(float) * (size_t)PL;
        float *o = s.o[s.cur];
        for (int g : {-3, -2, -1, s.nzs, s.nzs + 1, s.nzs + 2}) {
            const int src = ((g % s.nzs) + s.nzs) % s.nzs;
            H3(hipMemcpyAsync(o + (long long)g * PL, o + (long long)src * PL, bytes, hipMemcpyDeviceToDevice, s.s_comp));
        }
        launch_three(s, 0, s.nzs, 0, s.s_comp);
        reduce_three(s, t, s.s_comp);
        s.cur ^= 1;
        exchange(s.cur, false);  // faces for a one-step launch that may follow
    }

    void reduce_two(Slab &s, int t, hipStream_t st) {
        hipLaunchKernelGGL(reduce3d, dim3(1), dim3(BLOCK), 0, st, s.partials2, s.nblk_two, s.av_local, t);
        hipLaunchKernelGGL(reduce3d, dim3(1), dim3(BLOCK), 0, st, s.partials2 + s.nblk_two, s.nblk_two, s.av_local,
                           t + 1);
        H3(hipGetLastError());
    }

    // n-plane ghost exchange of lattice l (all 19 speeds; n = 2 for two-step,
    // 3 for three-step passes): planes nzs-n .. nzs-1 go up into the next
    // slab's ghosts -n .. -1; planes 0 .. n-1 go down into the previous slab's
    // ghosts nzs .. nzs+n-1.  Every rank posts send up, send down, recv from
    // below, recv from above (RCCL matches by order).
    void exchange2(int l, bool use_comm) { exchange_planes(l, 2, use_comm); }
    void exchange_planes(int l, int n, bool use_comm) {
        const size_t n2 = (size_t)n * PL;
        auto top = [&](const Slab &s) { return s.o[l] + (long long)(s.nzs - n) * PL; };
        auto bottom = [&](const Slab &s) { return s.o[l]; };
        auto ghost_lo = [&](const Slab &s) { return s.o[l] - n * PL; };
        auto ghost_hi = [&](const Slab &s) { return s.o[l] + (long long)s.nzs * PL; };
        if (transport == LBM_TRANSPORT_RCCL) {
            Slab &s = slabs[0];
            H3(hipSetDevice(s.dev));
            hipStream_t st = use_comm ? s.s_comm : s.s_comp;
            H3(hipStreamWaitEvent(st, s.ev_b, 0));
            N3(ncclGroupStart());
            for (const lbm_xfer &x : slab_posts(rank, world, (long long)n2)) {
                if (x.op == LBM_XFER_SEND)
                    N3(ncclSend(x.dir == 0 ? top(s) : bottom(s), (size_t)x.floats, ncclFloat, x.peer, comm, st));
                else
                    N3(ncclRecv(x.dir == 1 ? ghost_lo(s) : ghost_hi(s), (size_t)x.floats, ncclFloat, x.peer, comm, st));
            }
            N3(ncclGroupEnd());
            H3(hipEventRecord(s.ev_x, st));
            return;
        }
        for (auto &s : slabs) {  // LOCAL: each slab pulls its two ghost pairs
            H3(hipSetDevice(s.dev));
            hipStream_t st = use_comm ? s.s_comm : s.s_comp;
            Slab *below = local((s.id + parts - 1) % parts), *above = local((s.id + 1) % parts);
            H3(hipStreamWaitEvent(st, below->ev_b, 0));
            H3(hipStreamWaitEvent(st, above->ev_b, 0));
            const size_t bytes = sizeof(float) * n2;
            if (below->dev == s.dev)
                H3(hipMemcpyAsync(ghost_lo(s), top(*below), bytes, hipMemcpyDeviceToDevice, st));
            else
                H3(hipMemcpyPeerAsync(ghost_lo(s), s.dev, top(*below), below->dev, bytes, st));
            if (above->dev == s.dev)
                H3(hipMemcpyAsync(ghost_hi(s), bottom(*above), bytes, hipMemcpyDeviceToDevice, st));
            else
                H3(hipMemcpyPeerAsync(ghost_hi(s), s.dev, bottom(*above), above->dev, bytes, st));
            H3(hipEventRecord(s.ev_x, st));
        }
    }

    // Two steps of every slab (z slabs): B(t) = the boundary pairs on the
    // high-priority stream after I(t-1) and the exchange that filled our
    // ghosts; X(t) = their planes to the neighbours on the comm stream; I(t) =
    // the interior on the compute stream, overlapping X(t); then both steps'
    // |u| folds.  (Mirrors step_once's one-plane schedule.)
    void step_two_multi(int t) {
        for (auto &s : slabs) {
            H3(hipSetDevice(s.dev));
            H3(hipStreamWaitEvent(s.s_bnd, s.ev_i, 0));
            wait_x(s, s.s_bnd);
            stall(s, s.s_bnd);
            const auto r = two_ranges(s);
            int blk = 0;
            for (size_t i = 0; i < r.size() && i < 2; ++i) {
                launch_two(s, r[i].first, r[i].second, blk, s.s_bnd);
                blk += two_blocks(r[i].first, r[i].second);
            }
            H3(hipEventRecord(s.ev_b, s.s_bnd));
        }
        exchange2(1 - slabs[0].cur, true);
        for (auto &s : slabs) {
            H3(hipSetDevice(s.dev));
            const auto r = two_ranges(s);
            stall(s, s.s_comp);
            if (r.size() > 2) launch_two(s, r[2].first, r[2].second, two_blocks(r[0].first, r[0].second) +
                                                                          two_blocks(r[1].first, r[1].second), s.s_comp);
            H3(hipStreamWaitEvent(s.s_comp, s.ev_b, 0));
            reduce_two(s, t, s.s_comp);
            H3(hipEventRecord(s.ev_i, s.s_comp));
            s.cur ^= 1;
        }
    }

    // two-step pass: ghost planes -2, -1, nz, nz + 1 of the current lattice
    // (periodic images, all 19 speeds), then step3d_two, then both steps' |u|
    void step_two(int t) {
        if (multi()) {
            step_two_multi(t);
            return;
        }
        Slab &s = slabs[0];
        const size_t bytes = sizeof(float) * (size_t)PL;
        float *o = s.o[s.cur];
        for (int g : {-2, -1, s.nzs, s.nzs + 1}) {
            const int src = ((g % s.nzs) + s.nzs) % s.nzs;
            H3(hipMemcpyAsync(o + (long long)g * PL, o + (long long)src * PL, bytes, hipMemcpyDeviceToDevice, s.s_comp));
        }
        launch_two(s, 0, s.nzs, 0, s.s_comp);
        reduce_two(s, t, s.s_comp);
        s.cur ^= 1;
        exchange(s.cur, false);  // faces for a one-step launch that may follow
    }

    void ensure_av(int n) {
        for (auto &s : slabs) {
            if (s.av_cap >= n) continue;
            H3(hipSetDevice(s.dev));
            if (s.av_local) H3(hipFree(s.av_local));
            s.av_cap = std::max(n, 1);
            H3(hipMalloc(&s.av_local, sizeof(float) * (size_t)s.av_cap));
            fill_fresh(s.av_local, sizeof(float) * (size_t)s.av_cap, s.s_comp);
        }
    }

    Slab *local(int id) {
        for (auto &s : slabs)
            if (s.id == id) return &s;
        return nullptr;
    }

    // one contiguous face block: speeds 9..13 of the top plane (goes up) or
    // 14..18 of the bottom plane (goes down); ghost targets likewise
    float *up_src(const Slab &s, int l) const { return s.o[l] + (long long)(s.nzs - 1) * PL + 9 * KS; }
    float *down_src(const Slab &s, int l) const { return s.o[l] + 14 * KS; }
    float *below_ghost(const Slab &s, int l) const { return s.o[l] - PL + 9 * KS; }
    float *above_ghost(const Slab &s, int l) const { return s.o[l] + (long long)s.nzs * PL + 14 * KS; }

    // Fill the ghost planes of lattice l of every slab (on `st` of each slab,
    // after event `after` of the source slabs).  Single slab: periodic self copies.
    void exchange(int l, bool use_comm) {
        const size_t bytes = sizeof(float) * 5 * (size_t)KS;
        if (!multi()) {
            Slab &s = slabs[0];
            H3(hipSetDevice(s.dev));
            H3(hipMemcpyAsync(below_ghost(s, l), up_src(s, l), bytes, hipMemcpyDeviceToDevice, s.s_comp));
            H3(hipMemcpyAsync(above_ghost(s, l), down_src(s, l), bytes, hipMemcpyDeviceToDevice, s.s_comp));
            return;
        }
        if (transport == LBM_TRANSPORT_RCCL) {
            Slab &s = slabs[0];
            H3(hipSetDevice(s.dev));
            hipStream_t st = use_comm ? s.s_comm : s.s_comp;
            H3(hipStreamWaitEvent(st, s.ev_b, 0));
            N3(ncclGroupStart());
            // same posting order on every rank: send up, send down, recv from below, recv from above
            for (const lbm_xfer &x : slab_posts(rank, world, 5 * KS)) {
                if (x.op == LBM_XFER_SEND)
                    N3(ncclSend(x.dir == 0 ? up_src(s, l) : down_src(s, l), (size_t)x.floats, ncclFloat, x.peer, comm,
                                st));
                else
                    N3(ncclRecv(x.dir == 1 ? below_ghost(s, l) : above_ghost(s, l), (size_t)x.floats, ncclFloat,
                                x.peer, comm, st));
            }
            N3(ncclGroupEnd());
            H3(hipEventRecord(s.ev_x, st));
            return;
        }
        for (auto &s : slabs) {  // LOCAL: each slab pulls its two ghost blocks
            H3(hipSetDevice(s.dev));
            hipStream_t st = use_comm ? s.s_comm : s.s_comp;
            Slab *below = local((s.id + parts - 1) % parts), *above = local((s.id + 1) % parts);
            H3(hipStreamWaitEvent(st, below->ev_b, 0));
            H3(hipStreamWaitEvent(st, above->ev_b, 0));
            if (below->dev == s.dev)
                H3(hipMemcpyAsync(below_ghost(s, l), up_src(*below, l), bytes, hipMemcpyDeviceToDevice, st));
            else
                H3(hipMemcpyPeerAsync(below_ghost(s, l), s.dev, up_src(*below, l), below->dev, bytes, st));
            if (above->dev == s.dev)
                H3(hipMemcpyAsync(above_ghost(s, l), down_src(*above, l), bytes, hipMemcpyDeviceToDevice, st));
            else
                H3(hipMemcpyPeerAsync(above_ghost(s, l), s.dev, down_src(*above, l), above->dev, bytes, st));
            H3(hipEventRecord(s.ev_x, st));
        }
    }

    void stall(const Slab &s, hipStream_t st) {
        if (delay_us > 0 && s.id == delay_sub) H3(launch_debug_spin(delay_us, st));
    }

    // st waits for this slab's last exchange and (LOCAL) its neighbours' (they read our faces)
    void wait_x(Slab &s, hipStream_t st) {
        H3(hipStreamWaitEvent(st, s.ev_x, 0));
        if (transport == LBM_TRANSPORT_LOCAL && multi()) {
            H3(hipStreamWaitEvent(st, local((s.id + parts - 1) % parts)->ev_x, 0));
            H3(hipStreamWaitEvent(st, local((s.id + 1) % parts)->ev_x, 0));
        }
    }

    void launch(Slab &s, int zfirst, int planes, float *partials, hipStream_t st) {
        if (planes <= 0) return;
        Step3Args a{};
        a.fin = s.o[s.cur];
        a.fout = s.o[1 - s.cur];
        a.obst = s.obst + (size_t)zfirst * p.ny * p.nx;
        a.PL = PL;
        a.KS = KS;
        a.px = px;
        a.nx = p.nx;
        a.ny = p.ny;
        a.z0 = zfirst;
        a.omega = p.omega;
        a.omo = 1 - p.omega;
        a.w1 = w1();
        a.w2 = w2();
        a.partials = partials;
        if (pair) {
            dim3 grid((p.nx + 2 * B3X - 1) / (2 * B3X), (p.ny + B3Y - 1) / B3Y, (planes + zb - 1) / zb);
            auto k = zb == 1 ? (nt ? step3d_pair<1, true> : step3d_pair<1, false>)
                   : zb == 2 ? (nt ? step3d_pair<2, true> : step3d_pair<2, false>)
                   : zb == 8 ? (nt ? step3d_pair<8, true> : step3d_pair<8, false>)
                             : (nt ? step3d_pair<4, true> : step3d_pair<4, false>);
            hipLaunchKernelGGL(k, grid, dim3(B3X, B3Y), 0, st, a, planes);
        } else {
            dim3 grid((p.nx + B3X - 1) / B3X, (p.ny + B3Y - 1) / B3Y, planes);
            hipLaunchKernelGGL(step3d, grid, dim3(B3X, B3Y), 0, st, a);
        }
        H3(hipGetLastError());
    }

    // one step of every slab: reads lattice cur, writes 1 - cur and its ghosts
    void step_once(int t) {
        if (!multi()) {
            Slab &s = slabs[0];
            launch(s, 0, s.nzs, s.partials, s.s_comp);
            exchange(1 - s.cur, false);
            hipLaunchKernelGGL(reduce3d, dim3(1), dim3(BLOCK), 0, s.s_comp, s.partials, s.nblk_all, s.av_local, t);
            H3(hipGetLastError());
            s.cur ^= 1;
            return;
        }
        // B(t): faces, after I(t-1) and the exchanges that filled / read our ghosts and faces
        for (auto &s : slabs) {
            H3(hipSetDevice(s.dev));
            H3(hipStreamWaitEvent(s.s_bnd, s.ev_i, 0));
            wait_x(s, s.s_bnd);
            stall(s, s.s_bnd);
            launch(s, 0, 1, s.partials, s.s_bnd);
            if (s.nzs >= 2) launch(s, s.nzs - 1, 1, s.partials + blocks_for(1), s.s_bnd);
            H3(hipEventRecord(s.ev_b, s.s_bnd));
        }
        // X(t): faces of the new lattice -> neighbours' ghost planes, on the comm streams
        exchange(1 - slabs[0].cur, true);
        // I(t): interior planes, after B(t) (reduction needs its partials; the
        // interior reads the faces B(t-1) wrote, already ordered by ev_b)
        for (auto &s : slabs) {
            H3(hipSetDevice(s.dev));
            stall(s, s.s_comp);
            launch(s, 1, s.nzs - 2, s.partials + s.nblk_bnd, s.s_comp);
            H3(hipStreamWaitEvent(s.s_comp, s.ev_b, 0));
            hipLaunchKernelGGL(reduce3d, dim3(1), dim3(BLOCK), 0, s.s_comp, s.partials, s.nblk_all, s.av_local, t);
            H3(hipGetLastError());
            H3(hipEventRecord(s.ev_i, s.s_comp));
            s.cur ^= 1;
        }
    }

    void sync_all() {
        for (auto &s : slabs) {
            H3(hipSetDevice(s.dev));
            H3(hipStreamSynchronize(s.s_comp));
            H3(hipStreamSynchronize(s.s_bnd));
            H3(hipStreamSynchronize(s.s_comm));
        }
    }

    // ghost planes of the current lattice, from its faces (after load / init)
    void refresh() {
        if (multi()) {
            for (auto &s : slabs) {
                H3(hipSetDevice(s.dev));
                H3(hipEventRecord(s.ev_b, s.s_comp));
            }
            exchange(slabs[0].cur, false);
        } else {
            exchange(slabs[0].cur, false);
        }
        sync_all();
    }

    void run_steps(int steps) {
        if (!loaded) throw fail3(LBM_E_STATE, "lattice not initialised (lbm3d_load_cells / lbm3d_init_equilibrium)");
        if (steps < 0) throw fail3(LBM_E_INVALID, "steps must be >= 0");
        ensure_av(std::max(steps, 1));
        sync_all();
        Slab &s0 = slabs[0];
        H3(hipSetDevice(s0.dev));
        H3(hipEventRecord(t0, s0.s_comp));
        for (auto &s : slabs) {  // every stream starts after t0 and the last refresh
            H3(hipSetDevice(s.dev));
            H3(hipStreamWaitEvent(s.s_comp, t0, 0));
            H3(hipEventRecord(s.ev_i, s.s_comp));
            H3(hipEventRecord(s.ev_x, s.s_comp));
        }
        int t = 0;
        if (use_two() && steps >= 2) {
            if (multi()) {  // two- / three-plane ghosts of the current lattice (a one-step launch leaves only its five speeds)
                for (auto &s : slabs) {
                    H3(hipSetDevice(s.dev));
                    H3(hipEventRecord(s.ev_b, s.s_comp));
                }
                exchange_planes(slabs[0].cur, use_three() && steps >= 3 ? 3 : 2, false);
            }
            if (use_three())
                for (; t + 3 <= steps; t += 3) step_three(t);
            for (; t + 2 <= steps; t += 2) step_two(t);
        }
        for (; t < steps; ++t) step_once(t);
        for (auto &s : slabs) {
            H3(hipSetDevice(s.dev));
            H3(hipStreamWaitEvent(s.s_comp, s.ev_x, 0));
            H3(hipEventRecord(s.ev_end, s.s_comp));
        }
        H3(hipSetDevice(s0.dev));
        for (auto &s : slabs) H3(hipStreamWaitEvent(s0.s_comp, s.ev_end, 0));
        H3(hipEventRecord(t1, s0.s_comp));
        H3(hipEventSynchronize(t1));
        float ms = 0.f;
        H3(hipEventElapsedTime(&ms, t0, t1));
        last_seconds = ms * 1e-3;
        last_steps = steps;
        sync_all();
    }

    void init_equilibrium() {
        const float c0 = p.density / 3.f, c1 = p.density / 18.f, c2 = p.density / 36.f;
        for (auto &s : slabs) {
            H3(hipSetDevice(s.dev));
            s.cur = 0;
            const long long planes = s.nzs + 2 * GZ3;
            hipLaunchKernelGGL(init3d, dim3((unsigned)((planes * KS + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, s.s_comp,
                               s.f[0], planes, KS, PL, c0, c1, c2);
            H3(hipGetLastError());
        }
        sync_all();
        loaded = true;
    }

    void load_cells(const float *aos) {
        if (!aos) throw fail3(LBM_E_INVALID, "cells must not be NULL");
        for (auto &s : slabs) {
            H3(hipSetDevice(s.dev));
            const long long n = (long long)s.nzs * p.ny * p.nx;
            float *stage = nullptr;
            H3(hipMalloc(&stage, sizeof(float) * Q3 * (size_t)n));
            H3(hipMemcpy(stage, aos + (size_t)s.z0 * p.ny * p.nx * Q3, sizeof(float) * Q3 * (size_t)n,
                         hipMemcpyHostToDevice));
            s.cur = 0;
            hipLaunchKernelGGL(aos_to_soa3d, dim3((unsigned)((n + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, s.s_comp, stage,
                               s.o[0], PL, KS, px, p.nx, p.ny, n);
            H3(hipGetLastError());
            H3(hipStreamSynchronize(s.s_comp));
            H3(hipFree(stage));
        }
        refresh();
        loaded = true;
    }

    void store(float *aos, float *av, int n_av) {
        if (!loaded) throw fail3(LBM_E_STATE, "nothing to store");
        sync_all();
        if (aos)
            for (auto &s : slabs) {
                H3(hipSetDevice(s.dev));
                const long long n = (long long)s.nzs * p.ny * p.nx;
                float *stage = nullptr;
                H3(hipMalloc(&stage, sizeof(float) * Q3 * (size_t)n));
                hipLaunchKernelGGL(soa_to_aos3d, dim3((unsigned)((n + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, s.s_comp,
                                   s.o[s.cur], stage, PL, KS, px, p.nx, p.ny, n);
                H3(hipGetLastError());
                H3(hipStreamSynchronize(s.s_comp));
                H3(hipMemcpy(aos + (size_t)s.z0 * p.ny * p.nx * Q3, stage, sizeof(float) * Q3 * (size_t)n,
                             hipMemcpyDeviceToHost));
                H3(hipFree(stage));
            }
        if (av && n_av > 0) {
            const int n = std::min(n_av, last_steps);
            std::vector<float> per((size_t)parts * std::max(n, 1), 0.f);
            if (n > 0) {
                if (transport == LBM_TRANSPORT_RCCL) {
                    Slab &s = slabs[0];
                    H3(hipSetDevice(s.dev));
                    float *g = nullptr;
                    H3(hipMalloc(&g, sizeof(float) * (size_t)n * world));
                    N3(ncclAllGather(s.av_local, g, (size_t)n, ncclFloat, comm, s.s_comm));
                    H3(hipStreamSynchronize(s.s_comm));
                    H3(hipMemcpy(per.data(), g, sizeof(float) * (size_t)n * world, hipMemcpyDeviceToHost));
                    H3(hipFree(g));
                } else {
                    for (auto &s : slabs) {
                        H3(hipSetDevice(s.dev));
                        H3(hipMemcpy(per.data() + (size_t)s.id * n, s.av_local, sizeof(float) * (size_t)n,
                                     hipMemcpyDeviceToHost));
                    }
                }
            }
            const float fc = (float)free_cells;
            for (int t = 0; t < n_av; ++t) {
                if (t >= n) {
                    av[t] = 0.f;
                    continue;
                }
                float tot = 0.f;
                for (int r = 0; r < parts; ++r) tot += per[(size_t)r * n + t];  // fixed slab order
                av[t] = tot / fc;
            }
        }
    }

    void destroy() {
        for (auto &s : slabs) {
            if (hipSetDevice(s.dev) != hipSuccess) continue;
            (void)hipDeviceSynchronize();
            for (int k = 0; k < 2; ++k)
                if (s.f[k] && !(k == 1 && s.f_joint)) (void)hipFree(s.f[k]);
            if (s.obst) (void)hipFree(s.obst);
            if (s.obst_g) (void)hipFree(s.obst_g);
            if (s.partials) (void)hipFree(s.partials);
            if (s.partials2) (void)hipFree(s.partials2);
            if (s.partials3) (void)hipFree(s.partials3);
            if (s.av_local) (void)hipFree(s.av_local);
            for (hipStream_t st : {s.s_comp, s.s_bnd, s.s_comm})
                if (st) (void)hipStreamDestroy(st);
            for (hipEvent_t e : {s.ev_b, s.ev_i, s.ev_x, s.ev_end})
                if (e) (void)hipEventDestroy(e);
        }
        if (comm) (void)ncclCommDestroy(comm);
        if (t0) (void)hipEventDestroy(t0);
        if (t1) (void)hipEventDestroy(t1);
    }
};

namespace {
thread_local std::string g_err3;

template <class F>
int guard3(lbm3d_handle *h, F &&f) {
    try {
        f();
        return LBM_OK;
    } catch (const fail3 &e) {
        if (h) h->err = e.what();
        return e.code;
    } catch (const std::bad_alloc &) {
        if (h) h->err = "host allocation failed";
        return LBM_E_NOMEM;
    } catch (const std::exception &e) {
        if (h) h->err = e.what();
        return LBM_E_INTERNAL;
    } catch (...) {
        if (h) h->err = "unknown failure";
        return LBM_E_INTERNAL;
    }
}
}  // namespace

extern "C" {

int lbm3d_create(const lbm3d_params *params, const uint8_t *obstacles, const lbm_config *config, lbm3d_handle **out) {
    if (!params || !out) return LBM_E_INVALID;
    *out = nullptr;
    auto *h = new (std::nothrow) lbm3d_handle();
    if (!h) return LBM_E_NOMEM;
    lbm_config dflt{};
    dflt.parts = 1;
    const int rc = guard3(h, [&] { h->create(params, obstacles, config ? *config : dflt); });
    if (rc != LBM_OK) {
        g_err3 = h->err;
        h->destroy();
        delete h;
        return rc;
    }
    *out = h;
    return LBM_OK;
}

int lbm3d_init_equilibrium(lbm3d_handle *h) {
    if (!h) return LBM_E_INVALID;
    return guard3(h, [&] { h->init_equilibrium(); });
}

int lbm3d_load_cells(lbm3d_handle *h, const float *cells_aos) {
    if (!h) return LBM_E_INVALID;
    return guard3(h, [&] { h->load_cells(cells_aos); });
}

int lbm3d_run_steps(lbm3d_handle *h, int32_t steps) {
    if (!h) return LBM_E_INVALID;
    return guard3(h, [&] { h->run_steps(steps); });
}

int lbm3d_store(lbm3d_handle *h, float *cells_aos, float *av_vels, int32_t n_av) {
    if (!h) return LBM_E_INVALID;
    return guard3(h, [&] { h->store(cells_aos, av_vels, n_av); });
}

int lbm3d_last_run_seconds(lbm3d_handle *h, double *seconds) {
    if (!h || !seconds) return LBM_E_INVALID;
    *seconds = h->last_seconds;
    return LBM_OK;
}

int64_t lbm3d_total_free_cells(lbm3d_handle *h) { return h ? h->free_cells : -1; }

int lbm3d_local_slabs(lbm3d_handle *h, int32_t *z0, int32_t *nz, int32_t max_slabs, int32_t *n_out) {
    if (!h) return LBM_E_INVALID;
    const int n = (int)h->slabs.size();
    if (n_out) *n_out = n;
    for (int i = 0; i < n && i < max_slabs; ++i) {
        if (z0) z0[i] = h->slabs[i].z0;
        if (nz) nz[i] = h->slabs[i].nzs;
    }
    return LBM_OK;
}

int lbm3d_exchange_schedule(int32_t nx, int32_t ny, int32_t nz, int32_t parts, int32_t rank, int32_t planes,
                            lbm_xfer *out, int32_t max_out, int32_t *n_out) {
    if (!n_out || nx < 1 || ny < 1 || parts < 1 || parts > nz || rank < 0 || rank >= parts || planes < 1 ||
        planes > 3)
        return LBM_E_INVALID;
    const long long KS = (long long)ny * ((nx + 15) / 16 * 16);  // the engine's speed stride (64-byte rows)
    const auto v = slab_posts(rank, parts, planes == 1 ? 5 * KS : (long long)planes * Q3 * KS);
    *n_out = (int32_t)v.size();
    if (out) {
        if (max_out < (int32_t)v.size()) return LBM_E_INVALID;
        for (size_t i = 0; i < v.size(); ++i) out[i] = v[i];
    }
    return LBM_OK;
}

const char *lbm3d_last_error(lbm3d_handle *h) { return h ? h->err.c_str() : g_err3.c_str(); }

void lbm3d_destroy(lbm3d_handle *h) {
    if (!h) return;
    try {
        h->destroy();
    } catch (...) {
    }
    delete h;
}

}  // extern "C"

// lbm_packed.hpp -- packed fp32 (two cells per lane) D2Q9 collision shared by
// the two-column stream kernel (lbm_stream2.hip) and the packed resident
// kernel (lbm_resident.hip).
//
// Bitwise parity with the one-step kernels and the CPU oracle: every
// expression is evaluated in the order of LastChance.cpp:226-262 with one
// rounding per operation (packed ops round each lane like their scalar
// forms; no contraction).  Divisions stay correctly rounded for EVERY input:
//   * n / rho: the compiler's IEEE sequence (v_div_scale, v_rcp, four fma,
//     v_div_fmas, v_div_fixup).  A shorter sequence without the scale / fixup
//     wrappers (round 1) is exact only while rho, n and n/rho stay clear of
//     the exponent limits (tools/check_fastdiv.c --probe); on states with
//     tiny densities it produced NaN where the oracle did not
//     (tests/test_gpu_parity.py test_division_adversarial_states_bitwise);
//   * x / 9: q = x*y, r = fma(-9, q, x), q' = fma(r, y, q) with y = RN(1/9) --
//     exhaustively equal to RN(x/9) for every float x;
//   * x / 36: the same sequence is exact for x >= 2^-124 (exhaustive); a wave
//     holding a smaller density takes the compiler's IEEE division instead
//     (a wave-uniform branch, never taken in physical states).
// |u| = sqrt(u^2) feeds only av_vels and uses v_sqrt_f32 (sqrt_av below).
// (The shared-reciprocal n / rho was measured as library variants in round 4:
// +10 % unguarded but not exact for every input, no gain guarded -- DESIGN.md
// section 9, profiles/r04/fastdiv/; removed from the sources in round 5.)
#pragma once

#include "lbm_device.hpp"

namespace lbm {
typedef float f2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f2 fma2(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ f2 mk2(float v) { return f2{v, v}; }

// lanes shifted in from outside the wave read 0 (bound_ctrl); no old-value init move
__device__ __forceinline__ float dpp_from_left(float v) {  // lane - 1
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x138 /* wave_shr:1 */, 0xf, 0xf, true));
}
__device__ __forceinline__ float dpp_from_right(float v) {  // lane + 1
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x130 /* wave_shl:1 */, 0xf, 0xf, true));
}
// (x-1) and (x+1) neighbours of a lane's column pair (A = .x, B = .y)
__device__ __forceinline__ f2 left2(f2 v) { return f2{dpp_from_left(v.y), v.x}; }
__device__ __forceinline__ f2 right2(f2 v) { return f2{v.y, dpp_from_right(v.x)}; }

// The same shifts in place: the shifted pair is kept SWAPPED in its registers
// ({B', A'} for the in-order {A', B'} above), so the half that stays is
// already where it belongs and the shift is one DPP move over the other half
// (the in-order forms cost a DPP move plus a copy of the staying half).
// Readers take it through unswap(), which the packed instructions absorb as
// op_sel (free); the empty asm keeps the swapped pair in one register pair
// (without it the element picks cancel before register allocation and the
// copy comes back).
__device__ __forceinline__ f2 pin2(f2 v) {
    asm("" : "+v"(v));
    return v;
}
__device__ __forceinline__ f2 left2x(f2 v) { return pin2(f2{v.x, dpp_from_left(v.y)}); }
__device__ __forceinline__ f2 right2x(f2 v) { return pin2(f2{dpp_from_right(v.x), v.y}); }
__device__ __forceinline__ f2 unswap(f2 u) { return __builtin_shufflevector(u, u, 1, 0); }

// RN(x / d) for d = 9 or 36 (see header)
template <int D>
__device__ __forceinline__ f2 div_const(f2 x) {
    constexpr float y = 1.0f / (float)D;
    const f2 q = x * mk2(y);
    const f2 r = fma2(mk2(-(float)D), q, x);
    return fma2(r, mk2(y), q);
}

// RN(x / 36) for every x: the short sequence unless some lane of the wave
// holds x < 2^-120 (or a negative / NaN x), then IEEE division (see header)
__device__ __forceinline__ f2 div36_exact(f2 x) {
    const bool tiny = __builtin_amdgcn_ballot_w64(!(x.x >= 0x1p-120f) || !(x.y >= 0x1p-120f)) != 0;
    if (__builtin_expect(tiny, 0)) return x / mk2(36.0f);
    return div_const<36>(x);
}

// |u| for av_vels only (never fed back into the lattice): v_sqrt_f32, within
// 1 ulp of the correctly rounded sqrtf.  The av_vels sum already differs
// from the reference's by summation order; this costs < 1e-7 relative per
// term and saves the 16-instruction correction per cell pair
// (profiles/r01/final/ab_sqrt.log: +1 % at 8192^2, +5 % resident 1024^2).
__device__ __forceinline__ float sqrt_av(float x) { return __builtin_amdgcn_sqrtf(x); }

// One cell pair: pulled populations s -> post-collision o; returns |u| per cell (0 for obstacles).
// any_obst (wave-uniform): some lane of the wave has an obstacle cell in this
// row; without one the rebound selects are skipped (same values).
__device__ __forceinline__ f2 collide2(const f2 (&s)[Q], f2 (&o)[Q], bool oa, bool ob, bool any_obst, float accf,
                                       float omega, float omo, float w1, float w2) {
    const f2 rho = s[0] + s[1] + s[2] + s[3] + s[4] + s[5] + s[6] + s[7] + s[8];
    const f2 ux = (s[1] + s[5] + s[8] - (s[3] + s[6] + s[7])) / rho;
    const f2 uy = (s[2] + s[5] + s[6] - (s[4] + s[7] + s[8])) / rho;
    const f2 usq = ux * ux + uy * uy;
    const f2 csq = mk2(1.00f) - usq * mk2(1.50f);
    const f2 ld1 = div_const<9>(rho) * mk2(omega);
    const f2 ld2 = div36_exact(rho) * mk2(omega);
    const f2 OMO = mk2(omo);
    const f2 c23 = mk2(2.00f / 3.00f);
    const f2 c45 = mk2(4.50f), n45 = mk2(-4.50f);

    const f2 c0 = s[0] * OMO + mk2(4.00f / 9.00f) * rho * mk2(omega) * csq;
    const f2 c1 = s[1] * OMO + ld1 * ((c45 * ux) * (c23 + ux) + csq);
    const f2 c3 = s[3] * OMO + ld1 * ((n45 * ux) * (c23 - ux) + csq);
    const f2 c2 = s[2] * OMO + ld1 * ((c45 * uy) * (c23 + uy) + csq);
    const f2 c4 = s[4] * OMO + ld1 * ((n45 * uy) * (c23 - uy) + csq);
    const f2 us = ux + uy;
    const f2 c5 = s[5] * OMO + ld2 * ((c45 * us) * (c23 + us) + csq);
    const f2 c7 = s[7] * OMO + ld2 * ((n45 * us) * (c23 - us) + csq);
    const f2 ud = -ux + uy;
    const f2 c6 = s[6] * OMO + ld2 * ((c45 * ud) * (c23 + ud) + csq);
    const f2 c8 = s[8] * OMO + ld2 * ((n45 * ud) * (c23 - ud) + csq);
    const f2 a1 = mk2(accf * w1), a2 = mk2(accf * w2);
    const f2 f1 = c1 + a1, f3 = c3 - a1, f5 = c5 + a2, f6 = c6 - a2, f7 = c7 - a2, f8 = c8 + a2;
    if (!any_obst) {
        o[0] = c0;
        o[1] = f1;
        o[3] = f3;
        o[2] = c2;
        o[4] = c4;
        o[5] = f5;
        o[7] = f7;
        o[6] = f6;
        o[8] = f8;
        return f2{sqrt_av(usq.x), sqrt_av(usq.y)};
    }
    // obstacle cells rebound: out_k = s_opp(k)
    o[0] = f2{oa ? s[0].x : c0.x, ob ? s[0].y : c0.y};
    o[1] = f2{oa ? s[3].x : f1.x, ob ? s[3].y : f1.y};
    o[3] = f2{oa ? s[1].x : f3.x, ob ? s[1].y : f3.y};
    o[2] = f2{oa ? s[4].x : c2.x, ob ? s[4].y : c2.y};
    o[4] = f2{oa ? s[2].x : c4.x, ob ? s[2].y : c4.y};
    o[5] = f2{oa ? s[7].x : f5.x, ob ? s[7].y : f5.y};
    o[7] = f2{oa ? s[5].x : f7.x, ob ? s[5].y : f7.y};
    o[6] = f2{oa ? s[8].x : f6.x, ob ? s[8].y : f6.y};
    o[8] = f2{oa ? s[6].x : f8.x, ob ? s[6].y : f8.y};
    return f2{oa ? 0.f : sqrt_av(usq.x), ob ? 0.f : sqrt_av(usq.y)};
}

// collide2 for a wave whose pair row is uniform: the folded acceleration
// accel * w is added on EVERY row, as LastChance.cpp:253-261 does (accel = 0
// adds 0 * w, which turns a -0.0 population into +0.0 -- skipping the add off
// the accelerated row would not), with accel * w formed on the scalar unit
// (accrow is wave-uniform), and |u|^2 is returned for the caller to take the
// square root only where the row counts towards av_vels.
__device__ __forceinline__ f2 collide2u(const f2 (&s)[Q], f2 (&o)[Q], bool oa, bool ob, bool any_obst, bool accrow,
                                        float omega, float omo, float w1, float w2) {
    const f2 rho = s[0] + s[1] + s[2] + s[3] + s[4] + s[5] + s[6] + s[7] + s[8];
    const f2 ux = (s[1] + s[5] + s[8] - (s[3] + s[6] + s[7])) / rho;
    const f2 uy = (s[2] + s[5] + s[6] - (s[4] + s[7] + s[8])) / rho;
    const f2 usq = ux * ux + uy * uy;
    const f2 csq = mk2(1.00f) - usq * mk2(1.50f);
    const f2 ld1 = div_const<9>(rho) * mk2(omega);
    const f2 ld2 = div36_exact(rho) * mk2(omega);
    const f2 OMO = mk2(omo);
    const f2 c23 = mk2(2.00f / 3.00f);
    const f2 c45 = mk2(4.50f), n45 = mk2(-4.50f);

    f2 c[Q];
    c[0] = s[0] * OMO + mk2(4.00f / 9.00f) * rho * mk2(omega) * csq;
    c[1] = s[1] * OMO + ld1 * ((c45 * ux) * (c23 + ux) + csq);
    c[3] = s[3] * OMO + ld1 * ((n45 * ux) * (c23 - ux) + csq);
    c[2] = s[2] * OMO + ld1 * ((c45 * uy) * (c23 + uy) + csq);
    c[4] = s[4] * OMO + ld1 * ((n45 * uy) * (c23 - uy) + csq);
    const f2 us = ux + uy;
    c[5] = s[5] * OMO + ld2 * ((c45 * us) * (c23 + us) + csq);
    c[7] = s[7] * OMO + ld2 * ((n45 * us) * (c23 - us) + csq);
    const f2 ud = -ux + uy;
    c[6] = s[6] * OMO + ld2 * ((c45 * ud) * (c23 + ud) + csq);
    c[8] = s[8] * OMO + ld2 * ((n45 * ud) * (c23 - ud) + csq);
    {
        const float accf = accrow ? 1.00f : 0.00f;
        const f2 a1 = mk2(accf * w1), a2 = mk2(accf * w2);
        c[1] = c[1] + a1;
        c[3] = c[3] - a1;
        c[5] = c[5] + a2;
        c[6] = c[6] - a2;
        c[7] = c[7] - a2;
        c[8] = c[8] + a2;
    }
    if (!any_obst) {
#pragma unroll
        for (int k = 0; k < Q; ++k) o[k] = c[k];
        return usq;
    }
    // obstacle cells rebound: out_k = s_opp(k)
    constexpr int OPP[Q] = {0, 3, 4, 1, 2, 7, 8, 5, 6};
#pragma unroll
    for (int k = 0; k < Q; ++k) o[k] = f2{oa ? s[OPP[k]].x : c[k].x, ob ? s[OPP[k]].y : c[k].y};
    return usq;
}

// LBM_FLAG_TOLERANCE collision: the same BGK step as collide2u, reassociated
// for fewer VALU instructions (54 packed + 2 v_rcp_f32 per cell pair against
// 95 packed + 63 scalar in the bitwise form).  Not bitwise equal to
// LastChance.cpp:226-262 -- within the tolerance lbm_hip.h states:
//   * 1/rho once per cell (v_rcp_f32, 1 ulp; round 5 dropped the Newton step), shared by
//     u_x and u_y, instead of two correctly rounded divisions; the velocities
//     are carried scaled, v = 3u = (m / rho) * 3;
//   * rho/9 * omega and rho/36 * omega as rho * (omega/9), rho * (omega/36);
//   * out_k = s_k (1 - omega) + ld ((+-4.5 u)(2/3 +- u) + c) written as
//     fma(+-ld, v, fma(s_k, 1 - omega, P)) with P = ld (v^2 / 2 + c) shared by
//     each pair of opposite speeds and c = 1 - (vx^2 + vy^2) / 6 (the
//     3 ld u term rides in the outer fma instead of its own multiply);
//   * the folded acceleration only on the accelerated row (adding 0 * w
//     elsewhere changes nothing but the sign of a zero).
// Returns vx^2 + vy^2 = 9 |u|^2: the callers sum its square root and scale
// the sum by TOL_USQ_ROOT = 1/3 once, where the |u| partials are written.
// k = {1 - omega, 4 omega / 9, omega / 9, omega / 36}: wave-uniform scalars
// (kernel arguments, formed on the host), so they live in SGPRs, not VGPRs.
struct TolK {
    float omo, c0, c1, c2;
};
constexpr float TOL_USQ_ROOT = 1.00f / 3.00f;
// STAGED (the stream kernel): the speed pairs stage by stage (below);
// false (the resident tiles, 16 waves per CU = 128 VGPRs): pair by pair --
// the staged order holds more values at once and spilled 7 VGPRs there
// (1024^2 tolerance 240 vs 262 GLUPS).  The same operations either way: the
// two orders give the same lattice bit for bit.
template <bool STAGED = true>
__device__ __forceinline__ f2 collide2t(const f2 (&s)[Q], f2 (&o)[Q], bool oa, bool ob, bool any_obst, bool accrow,
                                        const TolK &k, float w1, float w2) {
    const f2 a = s[1] + s[5] + s[8], b = s[3] + s[6] + s[7];
    const f2 c = s[2] + s[5] + s[6], d = s[4] + s[7] + s[8];
    const f2 rho = (s[0] + s[2] + s[4]) + (a + b);
    f2 r = f2{__builtin_amdgcn_rcpf(rho.x), __builtin_amdgcn_rcpf(rho.y)};
    // (no Newton step: the hardware reciprocal's 1 ulp is inside the stated
    // tolerance, and dropping the two packed FMAs per cell pair and level ran
    // the S = 10 launch 2.6 % faster, profiles/r05/ab/)
    const f2 r3 = r * mk2(3.00f);
    const f2 vx = (a - b) * r3, vy = (c - d) * r3;  // 3 u
    const f2 hx = vx * vx, hy = vy * vy;
    const f2 h = hx + hy;                             // 9 |u|^2
    const f2 csq = fma2(h, mk2(-1.00f / 6.00f), mk2(1.00f));
    const f2 ld1 = rho * mk2(k.c1), ld2 = rho * mk2(k.c2);
    const f2 omo = mk2(k.omo);
    const f2 half = mk2(0.50f);
    f2 cc[Q];
    // the four pairs' chains written stage by stage, not pair by pair:
    // consecutive packed instructions are then independent, where the
    // pair-by-pair order made the compiler place them back to back and pad
    // each dependent pair with an s_nop (81 -> 3 in the S = 10 LP loop,
    // 244 -> 254 VGPRs; S = 10 launch -2 %, S = 8 -10 %, the same lattice bit
    // for bit: profiles/r05/ab/ab_ilv.log)
    if constexpr (!STAGED) {
        cc[0] = fma2(s[0], omo, (rho * mk2(k.c0)) * csq);
        {
            const f2 p = ld1 * fma2(hx, half, csq);
            cc[1] = fma2(ld1, vx, fma2(s[1], omo, p));
            cc[3] = fma2(-ld1, vx, fma2(s[3], omo, p));
        }
        {
            const f2 p = ld1 * fma2(hy, half, csq);
            cc[2] = fma2(ld1, vy, fma2(s[2], omo, p));
            cc[4] = fma2(-ld1, vy, fma2(s[4], omo, p));
        }
        {
            const f2 ws = vx + vy;
            const f2 p = ld2 * fma2(ws * ws, half, csq);
            cc[5] = fma2(ld2, ws, fma2(s[5], omo, p));
            cc[7] = fma2(-ld2, ws, fma2(s[7], omo, p));
        }
        {
            const f2 wd = vy - vx;
            const f2 p = ld2 * fma2(wd * wd, half, csq);
            cc[6] = fma2(ld2, wd, fma2(s[6], omo, p));
            cc[8] = fma2(-ld2, wd, fma2(s[8], omo, p));
        }
    } else {
    const f2 ws = vx + vy, wd = vy - vx;
    const f2 w5 = ws * ws, w6 = wd * wd;
    const f2 q1 = fma2(hx, half, csq), q2 = fma2(hy, half, csq);
    const f2 q5 = fma2(w5, half, csq), q6 = fma2(w6, half, csq);
    const f2 p1 = ld1 * q1, p2 = ld1 * q2, p5 = ld2 * q5, p6 = ld2 * q6;
    const f2 t1 = fma2(s[1], omo, p1), t2 = fma2(s[2], omo, p2), t5 = fma2(s[5], omo, p5),
             t6 = fma2(s[6], omo, p6);
    const f2 t3 = fma2(s[3], omo, p1), t4 = fma2(s[4], omo, p2), t7 = fma2(s[7], omo, p5),
             t8 = fma2(s[8], omo, p6);
    cc[0] = fma2(s[0], omo, (rho * mk2(k.c0)) * csq);
    cc[1] = fma2(ld1, vx, t1);
    cc[2] = fma2(ld1, vy, t2);
    cc[5] = fma2(ld2, ws, t5);
    cc[6] = fma2(ld2, wd, t6);
    cc[3] = fma2(-ld1, vx, t3);
    cc[4] = fma2(-ld1, vy, t4);
    cc[7] = fma2(-ld2, ws, t7);
    cc[8] = fma2(-ld2, wd, t8);
    }
    if (accrow) {
        // a real (wave-uniform) branch: without this barrier to speculation
        // the compiler if-converts it into 6 adds + 12 selects on EVERY row
        // (and holds their results in registers)
        asm volatile("" ::: "memory");
        const f2 a1 = mk2(w1), a2 = mk2(w2);
        cc[1] = cc[1] + a1;
        cc[3] = cc[3] - a1;
        cc[5] = cc[5] + a2;
        cc[6] = cc[6] - a2;
        cc[7] = cc[7] - a2;
        cc[8] = cc[8] + a2;
    }
    if (!any_obst) {
#pragma unroll
        for (int i = 0; i < Q; ++i) o[i] = cc[i];
        return h;
    }
    constexpr int OPP[Q] = {0, 3, 4, 1, 2, 7, 8, 5, 6};
#pragma unroll
    for (int i = 0; i < Q; ++i) o[i] = f2{oa ? s[OPP[i]].x : cc[i].x, ob ? s[OPP[i]].y : cc[i].y};
    return h;
}

}  // namespace lbm

/*
 * lbm_oracle3d.c -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the D3Q19-BGK extension (include/lbm3d_hip.h), the
 * parity checker of the HIP D3Q19 kernels.  Only tests/, smoke() and bench.py
 * use it; the product never links it.
 *
 * PARITY UNPINNED with respect to the reference: thorbenlouw/lbm-graphcore has
 * no 3-D code (BASELINE config 5).  The model is the
 * 3-D analogue of the reference's fused step (main/LastChance.cpp:192-266):
 * pull streaming with periodic wrap, bounce-back on obstacle cells, BGK
 * collision in the reference's expression form
 *     out_k = s_k (1 - omega) + ld_k ((4.5 e.u)(2/3 + e.u) + (1 - 1.5 |u|^2)),
 * and a body force folded into the fluid cells' outputs with the reference's
 * accelerate weights (density accel / 18 on the x-axis speeds, / 36 on the
 * diagonals with c_x != 0).  What pins it instead: mass conservation, a
 * Poiseuille profile between wall planes (tests/test_d3q19.py), and the D2Q9
 * limit of the same expression form (which IS pinned by the reference).
 *
 * Layout at this interface: AoS float[nz][ny][nx][19] (speed order in
 * include/lbm3d_hip.h), obstacles uint8[nz][ny][nx].  IEEE fp32 with
 * -ffp-contract=off, the same expression order as the HIP kernel.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define Q3 19

typedef struct {
    int32_t nx, ny, nz, max_iters;
    float density, accel, omega;
} oracle3d_params;

static const int CX[Q3] = {0, 1, -1, 0, 0, 1, -1, 1, -1, 0, 1, -1, 0, 0, 0, -1, 1, 0, 0};
static const int CY[Q3] = {0, 0, 0, 1, -1, 1, -1, -1, 1, 0, 0, 0, 1, -1, 0, 0, 0, -1, 1};
static const int CZ[Q3] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1};
static const int OPP[Q3] = {0, 2, 1, 4, 3, 6, 5, 8, 7, 14, 15, 16, 17, 18, 9, 10, 11, 12, 13};

void oracle3d_init_equilibrium(const oracle3d_params *p, float *cells)
{
    const float c0 = p->density / 3.f, c1 = p->density / 18.f, c2 = p->density / 36.f;
    const size_t n = (size_t)p->nx * p->ny * p->nz;
    for (size_t i = 0; i < n; i++) {
        float *c = cells + i * Q3;
        c[0] = c0;
        for (int k = 1; k < Q3; k++) c[k] = (k <= 4 || k == 9 || k == 14) ? c1 : c2;
    }
}

int64_t oracle3d_free_cells(const oracle3d_params *p, const uint8_t *obst)
{
    int64_t n = 0;
    const size_t total = (size_t)p->nx * p->ny * p->nz;
    for (size_t i = 0; i < total; i++) n += obst[i] ? 0 : 1;
    return n;
}

/* One cell from its 19 pulled populations; |u| for fluid, -1 for obstacles. */
static inline float cell3d(const float s[Q3], float o[Q3], int obstacle, float omega, float omo, float w1, float w2)
{
    if (obstacle) {
        for (int k = 0; k < Q3; k++) o[k] = s[OPP[k]];
        return -1.f;
    }
    const float rho = s[0] + s[1] + s[2] + s[3] + s[4] + s[5] + s[6] + s[7] + s[8] + s[9] + s[10] + s[11] + s[12] +
                      s[13] + s[14] + s[15] + s[16] + s[17] + s[18];
    const float ux = ((s[1] + s[5] + s[7] + s[10] + s[16]) - (s[2] + s[6] + s[8] + s[11] + s[15])) / rho;
    const float uy = ((s[3] + s[5] + s[8] + s[12] + s[18]) - (s[4] + s[6] + s[7] + s[13] + s[17])) / rho;
    const float uz = ((s[9] + s[10] + s[11] + s[12] + s[13]) - (s[14] + s[15] + s[16] + s[17] + s[18])) / rho;
    const float usq = ux * ux + uy * uy + uz * uz;
    const float c = 1.00f - usq * 1.50f;
    const float ld0 = rho / 3.00f * omega;
    const float ld1 = rho / 18.00f * omega;
    const float ld2 = rho / 36.00f * omega;
    const float pxy = ux + uy, mxy = ux - uy, pxz = ux + uz, mxz = -ux + uz, pyz = uy + uz, myz = -uy + uz;
    const float e[Q3] = {0.f, ux, -ux, uy, -uy, pxy, -pxy, mxy, -mxy, uz, pxz, mxz, pyz, myz,
                         -uz, -pxz, -mxz, -pyz, -myz};
    o[0] = s[0] * omo + ld0 * c;
    for (int k = 1; k < Q3; k++) {
        const float ld = (k <= 4 || k == 9 || k == 14) ? ld1 : ld2;
        o[k] = s[k] * omo + ld * ((4.50f * e[k]) * (2.00f / 3.00f + e[k]) + c);
    }
    /* body force along +x (c_x = +1: 1, 5, 7, 10, 16; c_x = -1: 2, 6, 8, 11, 15) */
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
    return sqrtf(usq);
}

/* One periodic step; returns the row-major (z, y, x) sum of |u| over fluid cells. */
float oracle3d_step(const oracle3d_params *p, const float *old, float *out, const uint8_t *obst)
{
    const int nx = p->nx, ny = p->ny, nz = p->nz;
    const float omega = p->omega, omo = 1 - p->omega;
    const float w1 = p->density * p->accel / 18.f, w2 = p->density * p->accel / 36.f;
    float tot = 0.00f;
    for (int z = 0; z < nz; z++)
        for (int y = 0; y < ny; y++)
            for (int x = 0; x < nx; x++) {
                float s[Q3];
                for (int k = 0; k < Q3; k++) {
                    const int xs = (x - CX[k] + nx) % nx, ys = (y - CY[k] + ny) % ny, zs = (z - CZ[k] + nz) % nz;
                    s[k] = old[(((size_t)zs * ny + ys) * nx + xs) * Q3 + k];
                }
                const size_t idx = ((size_t)z * ny + y) * nx + x;
                const float u = cell3d(s, out + idx * Q3, obst[idx], omega, omo, w1, w2);
                if (u >= 0.f) tot += u;
            }
    return tot;
}

/* `iters` steps in place; av_vels[t] = tot / fluid cells.  0 or -1 (allocation). */
int oracle3d_run(const oracle3d_params *p, float *cells, const uint8_t *obst, int iters, float *av_vels)
{
    const size_t n = (size_t)p->nx * p->ny * p->nz * Q3;
    float *tmp = (float *)malloc(n * sizeof(float));
    if (!tmp) return -1;
    const float fc = (float)oracle3d_free_cells(p, obst);
    float *a = cells, *b = tmp;
    for (int t = 0; t < iters; t++) {
        const float tot = oracle3d_step(p, a, b, obst);
        if (av_vels) av_vels[t] = tot / fc;
        float *sw = a;
        a = b;
        b = sw;
    }
    if (a != cells) memcpy(cells, a, n * sizeof(float));
    free(tmp);
    return 0;
}

/*
 * Same step on a z slab of nzs planes with one ghost plane below and above:
 * `old` is AoS [(nzs+2)][ny][nx][19] (ghost planes at 0 and nzs+1, only the
 * speeds that cross into the slab need be valid: 9..13 below, 14..18 above),
 * `out` is [nzs][ny][nx][19]; x and y wrap.  Used by the multi-rank
 * decomposition test (tests/test_d3q19_gloo.py).
 */
float oracle3d_step_slab(const oracle3d_params *p, int nzs, const float *old, float *out, const uint8_t *obst)
{
    const int nx = p->nx, ny = p->ny;
    const float omega = p->omega, omo = 1 - p->omega;
    const float w1 = p->density * p->accel / 18.f, w2 = p->density * p->accel / 36.f;
    float tot = 0.00f;
    for (int z = 0; z < nzs; z++)
        for (int y = 0; y < ny; y++)
            for (int x = 0; x < nx; x++) {
                float s[Q3];
                for (int k = 0; k < Q3; k++) {
                    const int xs = (x - CX[k] + nx) % nx, ys = (y - CY[k] + ny) % ny, zs = z + 1 - CZ[k];
                    s[k] = old[(((size_t)zs * ny + ys) * nx + xs) * Q3 + k];
                }
                const size_t idx = ((size_t)z * ny + y) * nx + x;
                const float u = cell3d(s, out + idx * Q3, obst[idx], omega, omo, w1, w2);
                if (u >= 0.f) tot += u;
            }
    return tot;
}

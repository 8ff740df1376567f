/*
 * lbm_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference D2Q9-BGK hot path, used exclusively as the
 * parity checker by tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg.  Nothing in the product (lbm-graphcore_amd/) links,
 * loads or calls this file.
 *
 * Algorithm followed (thorbenlouw/lbm-graphcore @ v0):
 *   - equilibrium initialisation      main/LastChance.cpp:428-450
 *                                     (= main/include/LatticeBoltzmannUtils.hpp:137-157)
 *   - one-time conditional accelerate main/LastChance.cpp:156-183
 *                                     (= main/codelets/D2Q9Codelets.cpp:71-93)
 *   - fused pull-stream / rebound / BGK collision / folded accelerate /
 *     |u| accumulation                main/LastChance.cpp:185-266
 *                                     (= main/codelets/D2Q9Codelets.cpp:94-191)
 *   - av_vels[t] = tot_u / free cells main/LastChance.cpp:266, :486-493
 *   - Reynolds number                 main/include/LatticeBoltzmannUtils.hpp:202-205
 *   - av_velocity of a state          main/LastChance.cpp:290-339
 *   - UNFUSED pipeline: per step accelerate_flow ->
 *     propagate -> rebound -> collision -> av_velocity as separate passes,
 *     main/LbmPoplibs.cpp:225-233 + :23-95 (timestep / averageVelocity), the
 *     conditional accelerate every step (LastChance.cpp:161-183,
 *     D2Q9CodeletsOld.cpp:52-80), the textbook BGK CollisionVertex
 *     (main/codelets/D2Q9CodeletsOptimised.cpp:102-212) and
 *     AppendReducedSum total / count (D2Q9Codelets.cpp:18-38)
 *
 * Parity pin: tests/test_oracle.py checks this restatement against the
 * reference's committed check/*.dat fixtures (copied, gzipped, into
 * tests/golden/check/) and, when /root/reference is present, bit-for-bit
 * against oracle/_ref/lastchance built from the reference's own source.
 *
 * Floating point: IEEE fp32, compiled with -ffp-contract=off so that every
 * expression is evaluated exactly as written (no FMA contraction).  The HIP
 * kernels are compiled the same way, which makes the lattice bitwise
 * comparable.
 *
 * Layout at this interface: AoS float[ny][nx][9], speed order
 *   0 M, 1 E, 2 N, 3 W, 4 S, 5 NE, 6 NW, 7 SW, 8 SE
 * (main/include/LatticeBoltzmannUtils.hpp:20-22); obstacles uint8[ny][nx].
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define Q 9

typedef struct {
    int32_t nx, ny, max_iters, reynolds_dim;
    float density, accel, omega;
} oracle_params;

/* LastChance.cpp:428-450 */
void oracle_init_equilibrium(const oracle_params *p, float *cells)
{
    const float c0 = p->density * 4.f / 9.f;
    const float c1 = p->density / 9.f;
    const float c2 = p->density / 36.f;
    const size_t n = (size_t)p->nx * (size_t)p->ny;
    for (size_t i = 0; i < n; i++) {
        float *c = cells + i * Q;
        c[0] = c0;
        c[1] = c1; c[2] = c1; c[3] = c1; c[4] = c1;
        c[5] = c2; c[6] = c2; c[7] = c2; c[8] = c2;
    }
}

/* LastChance.cpp:486-493 */
int64_t oracle_free_cells(const oracle_params *p, const uint8_t *obst)
{
    int64_t n = 0;
    const size_t total = (size_t)p->nx * (size_t)p->ny;
    for (size_t i = 0; i < total; i++) n += obst[i] ? 0 : 1;
    return n;
}

/* One-time accelerate of row ny-2 with positivity guard: LastChance.cpp:161-183. */
void oracle_accelerate(const oracle_params *p, float *cells, const uint8_t *obst)
{
    if (p->ny < 2) return;
    const float w1 = p->density * p->accel / 9.f;
    const float w2 = p->density * p->accel / 36.f;
    const int row = p->ny - 2;
    for (int x = 0; x < p->nx; x++) {
        const size_t idx = (size_t)row * p->nx + x;
        float *c = cells + idx * Q;
        if (!obst[idx] && (c[3] - w1) > 0.f && (c[6] - w2) > 0.f && (c[7] - w2) > 0.f) {
            c[1] += w1; c[5] += w2; c[8] += w2;
            c[3] -= w1; c[6] -= w2; c[7] -= w2;
        }
    }
}

/*
 * Per-cell update from the nine pulled populations s[0..8] (already streamed).
 * Writes out[0..8]; returns |u| for a fluid cell and -1 for an obstacle.
 * Expression order mirrors LastChance.cpp:213-262 exactly.
 */
static inline float cell_update(const float s[Q], float out[Q], int obstacle,
                                float accel_flag, float omega, float one_minus_omega,
                                float w1, float w2)
{
    if (obstacle) {
        /* rebound: out_k = s_opp(k)   (LastChance.cpp:213-223) */
        out[0] = s[0]; out[1] = s[3]; out[2] = s[4]; out[3] = s[1]; out[4] = s[2];
        out[5] = s[7]; out[6] = s[8]; out[7] = s[5]; out[8] = s[6];
        return -1.f;
    }
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
    const float o0 = s[0] * one_minus_omega + ld0 * csq;
    const float o1 = s[1] * one_minus_omega + ld1 * ((4.50f * ux) * (2.00f / 3.00f + ux) + csq);
    const float o2 = s[2] * one_minus_omega + ld1 * ((4.50f * uy) * (2.00f / 3.00f + uy) + csq);
    const float o3 = s[3] * one_minus_omega + ld1 * ((-4.50f * ux) * (2.00f / 3.00f - ux) + csq);
    const float o4 = s[4] * one_minus_omega + ld1 * ((-4.50f * uy) * (2.00f / 3.00f - uy) + csq);
    const float o5 = s[5] * one_minus_omega + ld2 * ((4.50f * us) * (2.00f / 3.00f + us) + csq);
    const float o6 = s[6] * one_minus_omega + ld2 * ((4.50f * ud) * (2.00f / 3.00f + ud) + csq);
    const float o7 = s[7] * one_minus_omega + ld2 * ((-4.50f * us) * (2.00f / 3.00f - us) + csq);
    const float o8 = s[8] * one_minus_omega + ld2 * ((-4.50f * ud) * (2.00f / 3.00f - ud) + csq);
    /* folded acceleration, unconditional on the accelerated row (LastChance.cpp:253-261) */
    out[0] = o0;
    out[1] = o1 + accel_flag * w1;
    out[2] = o2;
    out[3] = o3 - accel_flag * w1;
    out[4] = o4;
    out[5] = o5 + accel_flag * w2;
    out[6] = o6 - accel_flag * w2;
    out[7] = o7 - accel_flag * w2;
    out[8] = o8 + accel_flag * w2;
    return sqrtf(usq);
}

/*
 * One fused periodic step over the whole domain (LastChance.cpp:192-265).
 * Returns tot_u = sum over fluid cells of |u| (pre-collision velocity),
 * accumulated in row-major order like the reference.
 */
float oracle_step(const oracle_params *p, const float *old, float *out_cells, const uint8_t *obst)
{
    const int nx = p->nx, ny = p->ny;
    const float w1 = p->density * p->accel / 9.f;
    const float w2 = p->density * p->accel / 36.f;
    const float omega = p->omega;
    const float omo = 1 - p->omega; /* LastChance.cpp:388 */
    float tot_u = 0.00f;
    for (int y = 0; y < ny; y++) {
        const int yn = (y + 1) % ny;
        const int ys = (y == 0) ? ny - 1 : y - 1;
        const float accel_flag = (y == ny - 2) ? 1.00f : 0.00f;
        for (int x = 0; x < nx; x++) {
            const int xe = (x + 1) % nx;
            const int xw = (x == 0) ? nx - 1 : x - 1;
            float s[Q];
#define AT(xx, yy, k) old[((size_t)(yy) * nx + (xx)) * Q + (k)]
            s[0] = AT(x, y, 0);
            s[1] = AT(xw, y, 1);
            s[2] = AT(x, ys, 2);
            s[3] = AT(xe, y, 3);
            s[4] = AT(x, yn, 4);
            s[5] = AT(xw, ys, 5);
            s[6] = AT(xe, ys, 6);
            s[7] = AT(xe, yn, 7);
            s[8] = AT(xw, yn, 8);
#undef AT
            const size_t idx = (size_t)y * nx + x;
            const float u = cell_update(s, out_cells + idx * Q, obst[idx], accel_flag,
                                        omega, omo, w1, w2);
            if (u >= 0.f) tot_u += u;
        }
    }
    return tot_u;
}

/*
 * Same update on a ghosted sub-block: `old` is AoS [(h+2)][(w+2)][9] with a
 * one-cell ghost ring already filled; `out_cells` is AoS [h][w][9].
 * `accel_row` is the local row index that carries the folded acceleration
 * (or -1).  Used by the multi-rank decomposition tests: the same arithmetic
 * as oracle_step, only the neighbour addressing differs
 * (cf. main/include/GraphcoreUtils.hpp:119-127 stitchHalos and
 * main/codelets/D2Q9Codelets.cpp:102-123 OLD_OFFSET).
 */
float oracle_step_ghosted(const oracle_params *p, int w, int h, const float *old,
                          float *out_cells, const uint8_t *obst, int accel_row)
{
    const float w1 = p->density * p->accel / 9.f;
    const float w2 = p->density * p->accel / 36.f;
    const float omega = p->omega;
    const float omo = 1 - p->omega;
    const int gw = w + 2;
    float tot_u = 0.00f;
    for (int y = 0; y < h; y++) {
        const float accel_flag = (y == accel_row) ? 1.00f : 0.00f;
        for (int x = 0; x < w; x++) {
            float s[Q];
#define G(dx, dy, k) old[((size_t)(y + 1 + (dy)) * gw + (x + 1 + (dx))) * Q + (k)]
            s[0] = G(0, 0, 0);
            s[1] = G(-1, 0, 1);
            s[2] = G(0, -1, 2);
            s[3] = G(1, 0, 3);
            s[4] = G(0, 1, 4);
            s[5] = G(-1, -1, 5);
            s[6] = G(1, -1, 6);
            s[7] = G(1, 1, 7);
            s[8] = G(-1, 1, 8);
#undef G
            const size_t idx = (size_t)y * w + x;
            const float u = cell_update(s, out_cells + idx * Q, obst[idx], accel_flag,
                                        omega, omo, w1, w2);
            if (u >= 0.f) tot_u += u;
        }
    }
    return tot_u;
}

/*
 * Full run as program 1 of the reference (main/LbmRunner.cpp:102-104 /
 * LastChance.cpp:156-267): first accelerate, then `iters` fused steps with
 * ping-pong buffers.  `cells` is updated in place with the final state; if
 * `av_vels` is non-NULL it receives tot_u / free_cells for every step.
 * Returns 0, or -1 on allocation failure.
 */
int oracle_run(const oracle_params *p, float *cells, const uint8_t *obst, int iters,
               float *av_vels)
{
    const size_t n = (size_t)p->nx * (size_t)p->ny * Q;
    float *tmp = (float *)malloc(n * sizeof(float));
    if (!tmp) return -1;
    const float free_cells = (float)oracle_free_cells(p, obst);
    oracle_accelerate(p, cells, obst);
    float *a = cells, *b = tmp;
    for (int t = 0; t < iters; t++) {
        const float tot = oracle_step(p, a, b, obst);
        if (av_vels) av_vels[t] = tot / free_cells;
        float *s = a; a = b; b = s;
    }
    if (a != cells) memcpy(cells, a, n * sizeof(float));
    free(tmp);
    return 0;
}

/* Average velocity of a state, LastChance.cpp:290-339. */
float oracle_av_velocity(const oracle_params *p, const float *cells, const uint8_t *obst)
{
    int tot_cells = 0;
    float tot_u = 0.f;
    const size_t total = (size_t)p->nx * (size_t)p->ny;
    for (size_t i = 0; i < total; i++) {
        if (obst[i]) continue;
        const float *c = cells + i * Q;
        float rho = 0.f;
        for (int k = 0; k < Q; k++) rho += c[k];
        const float ux = (c[1] + c[5] + c[8] - (c[3] + c[6] + c[7])) / rho;
        const float uy = (c[2] + c[5] + c[6] - (c[4] + c[7] + c[8])) / rho;
        tot_u += sqrtf((ux * ux) + (uy * uy));
        ++tot_cells;
    }
    return tot_u / (float)tot_cells;
}

/* LatticeBoltzmannUtils.hpp:202-205 */
float oracle_reynolds(const oracle_params *p, float av_velocity)
{
    const float viscosity = 1.f / 6.f * (2.f / p->omega - 1.f);
    return av_velocity * (float)p->reynolds_dim / viscosity;
}

/* ---- unfused pipeline (main/LbmPoplibs.cpp timestep + averageVelocity) ---- */

/* propagate: tmp[k](x, y) = cells[k](x - cx_k, y - cy_k), periodic
 * (LbmPoplibs.cpp:134-175 PropagateVertex with wrap-around halos). */
void oracle_pipe_propagate(const oracle_params *p, const float *cells, float *tmp)
{
    const int nx = p->nx, ny = p->ny;
    for (int y = 0; y < ny; y++) {
        const int yn = (y + 1) % ny, ys = (y == 0) ? ny - 1 : y - 1;
        for (int x = 0; x < nx; x++) {
            const int xe = (x + 1) % nx, xw = (x == 0) ? nx - 1 : x - 1;
            float *t = tmp + ((size_t)y * nx + x) * Q;
#define AT(xx, yy, k) cells[((size_t)(yy) * nx + (xx)) * Q + (k)]
            t[0] = AT(x, y, 0);
            t[1] = AT(xw, y, 1);
            t[2] = AT(x, ys, 2);
            t[3] = AT(xe, y, 3);
            t[4] = AT(x, yn, 4);
            t[5] = AT(xw, ys, 5);
            t[6] = AT(xe, ys, 6);
            t[7] = AT(xe, yn, 7);
            t[8] = AT(xw, yn, 8);
#undef AT
        }
    }
}

/* rebound on obstacle cells: cells_k = tmp_opp(k) (CollisionVertex rebound
 * branch, D2Q9CodeletsOptimised.cpp:141-149; speed 0 keeps its value). */
void oracle_pipe_rebound(const oracle_params *p, const float *tmp, float *cells, const uint8_t *obst)
{
    const size_t n = (size_t)p->nx * (size_t)p->ny;
    for (size_t i = 0; i < n; i++) {
        if (!obst[i]) continue;
        const float *s = tmp + i * Q;
        float *o = cells + i * Q;
        o[0] = s[0]; o[1] = s[3]; o[2] = s[4]; o[3] = s[1]; o[4] = s[2];
        o[5] = s[7]; o[6] = s[8]; o[7] = s[5]; o[8] = s[6];
    }
}

/* Textbook BGK on fluid cells (D2Q9CodeletsOptimised.cpp:150-205, every
 * expression in its order): returns the sum of |u| (pre-collision) over the
 * fluid cells in row-major order; *count receives their number. */
float oracle_pipe_collision(const oracle_params *p, const float *tmp, float *cells, const uint8_t *obst,
                            int64_t *count)
{
    const float c_sq = 1.f / 3.f;
    const float cc2 = (2.f * c_sq * c_sq);
    const float w0 = 4.f / 9.f, w1 = 1.f / 9.f, w2 = 1.f / 36.f;
    const float o = p->omega;
    const size_t n = (size_t)p->nx * (size_t)p->ny;
    float tot = 0.f;
    int64_t cnt = 0;
    for (size_t i = 0; i < n; i++) {
        if (obst[i]) continue;
        const float *in = tmp + i * Q;
        float *out = cells + i * Q;
        float local_density = 0.f;
        for (int kk = 0; kk < Q; kk++) local_density += in[kk];
        const float u_x = ((in[1] + in[5] + in[8]) - (in[3] + in[6] + in[7])) / local_density;
        const float u_y = ((in[2] + in[5] + in[6]) - (in[4] + in[7] + in[8])) / local_density;
        const float u_sq = u_x * u_x + u_y * u_y;
        tot += sqrtf(u_sq);
        cnt++;
        const float u[Q] = {0, u_x, u_y, -u_x, -u_y, u_x + u_y, -u_x + u_y, -u_x - u_y, u_x - u_y};
        const float u_over_2csq = u_sq / (2.f * c_sq);
        float d_equ[Q];
        d_equ[0] = w0 * local_density * (1.f - u_over_2csq);
        for (int k = 1; k < Q; k++) {
            const float wk = k < 5 ? w1 : w2;
            d_equ[k] = wk * local_density * (1.f + u[k] / c_sq + (u[k] * u[k]) / cc2 - u_over_2csq);
        }
        for (int kk = 0; kk < Q; kk++) out[kk] = in[kk] + o * (d_equ[kk] - in[kk]);
    }
    if (count) *count = cnt;
    return tot;
}

/* accelerate_flow -> propagate -> rebound -> collision -> av_velocity,
 * `iters` times (LbmPoplibs.cpp:362-365: Repeat(maxIters, {timestep,
 * averageVelocity}); the accelerate runs at the start of EVERY step).
 * av_vels[t] = total / count (AppendReducedSum).  Returns 0 or -1. */
int oracle_pipe_run(const oracle_params *p, float *cells, const uint8_t *obst, int iters, float *av_vels)
{
    const size_t n = (size_t)p->nx * (size_t)p->ny * Q;
    float *tmp = (float *)malloc(n * sizeof(float));
    if (!tmp) return -1;
    for (int t = 0; t < iters; t++) {
        oracle_accelerate(p, cells, obst);
        oracle_pipe_propagate(p, cells, tmp);
        oracle_pipe_rebound(p, tmp, cells, obst);
        int64_t cnt = 0;
        const float tot = oracle_pipe_collision(p, tmp, cells, obst, &cnt);
        if (av_vels) av_vels[t] = tot / (float)cnt;
    }
    free(tmp);
    return 0;
}

/*
 * Multi-threaded run for the informational all-cores CPU baseline (bench.py
 * aux.cpu_baseline_threads): the same per-cell update as oracle_step with the
 * rows split over `threads` OpenMP threads.  The lattice is bitwise the same;
 * the per-step |u| sum is added per row and then over rows in row order, so
 * av_vels can differ from oracle_run in the last bits.
 */
int oracle_run_mt(const oracle_params *p, float *cells, const uint8_t *obst, int iters, float *av_vels, int threads)
{
    const size_t n = (size_t)p->nx * (size_t)p->ny * Q;
    float *tmp = (float *)malloc(n * sizeof(float));
    float *rows = (float *)malloc((size_t)p->ny * sizeof(float));
    if (!tmp || !rows) {
        free(tmp);
        free(rows);
        return -1;
    }
    const float free_cells = (float)oracle_free_cells(p, obst);
    oracle_accelerate(p, cells, obst);
    const int nx = p->nx, ny = p->ny;
    const float w1 = p->density * p->accel / 9.f, w2 = p->density * p->accel / 36.f;
    const float omega = p->omega, omo = 1 - p->omega;
    float *a = cells, *b = tmp;
    for (int t = 0; t < iters; t++) {
#pragma omp parallel for num_threads(threads) schedule(static)
        for (int y = 0; y < ny; y++) {
            const int yn = (y + 1) % ny, ys = (y == 0) ? ny - 1 : y - 1;
            const float accel_flag = (y == ny - 2) ? 1.00f : 0.00f;
            float row_u = 0.00f;
            for (int x = 0; x < nx; x++) {
                const int xe = (x + 1) % nx, xw = (x == 0) ? nx - 1 : x - 1;
                float s[Q];
#define AT(xx, yy, k) a[((size_t)(yy) * nx + (xx)) * Q + (k)]
                s[0] = AT(x, y, 0);
                s[1] = AT(xw, y, 1);
                s[2] = AT(x, ys, 2);
                s[3] = AT(xe, y, 3);
                s[4] = AT(x, yn, 4);
                s[5] = AT(xw, ys, 5);
                s[6] = AT(xe, ys, 6);
                s[7] = AT(xe, yn, 7);
                s[8] = AT(xw, yn, 8);
#undef AT
                const size_t idx = (size_t)y * nx + x;
                const float u = cell_update(s, b + idx * Q, obst[idx], accel_flag, omega, omo, w1, w2);
                if (u >= 0.f) row_u += u;
            }
            rows[y] = row_u;
        }
        float tot = 0.00f;
        for (int y = 0; y < ny; y++) tot += rows[y];
        if (av_vels) av_vels[t] = tot / free_cells;
        float *sw = a;
        a = b;
        b = sw;
    }
    if (a != cells) memcpy(cells, a, n * sizeof(float));
    free(tmp);
    free(rows);
    return 0;
}

/*
 * lbm3d_hip.h -- C ABI of the D3Q19-BGK engine in liblbm_hip.so (BASELINE
 * config 5 / SURVEY 8f rank 4: "D3Q19 512^3 fp32 on 8 x MI355X, same
 * SoA / halo machinery").
 *
 * The reference has NO 3-D code: this is the stretch extension of its D2Q9
 * hot path, kept as close to it as a third dimension allows, and its parity
 * is pinned only against our own CPU restatement (oracle/lbm_oracle3d.c,
 * bitwise) plus physics checks (mass conservation, Poiseuille profile) --
 * "parity unpinned" with respect to the reference.
 *
 * Model (mirrors main/LastChance.cpp:192-266 in 3-D):
 *   * pull streaming, periodic in x, y and z; obstacle cells bounce back
 *     (out_k = s_opp(k));
 *   * BGK collision out_k = s_k (1 - omega) + ld_k ((4.5 e.u)(2/3 + e.u) + c),
 *     c = 1 - 1.5 |u|^2, ld = rho w_k omega with w = 1/3, 1/18, 1/36;
 *   * body force along +x folded into every fluid cell's outputs: +-w1 on
 *     the two x-axis speeds, +-w2 on the eight speeds with c_x != 0
 *     (w1 = density accel / 18, w2 = density accel / 36 -- the reference's
 *     D2Q9 accelerate_flow weights ρa/9, ρa/36 in 3-D), which drives a
 *     Poiseuille flow between wall planes;
 *   * av_vels[t] = sum over fluid cells of |u| (pre-collision) / fluid cells.
 *
 * Speed order (chosen so the populations that cross a z face are adjacent
 * in memory: one contiguous RCCL message per face):
 *    0 ( 0, 0, 0)
 *    1 (+1, 0, 0)   2 (-1, 0, 0)   3 ( 0,+1, 0)   4 ( 0,-1, 0)
 *    5 (+1,+1, 0)   6 (-1,-1, 0)   7 (+1,-1, 0)   8 (-1,+1, 0)
 *    9 ( 0, 0,+1)  10 (+1, 0,+1)  11 (-1, 0,+1)  12 ( 0,+1,+1)  13 ( 0,-1,+1)
 *   14 ( 0, 0,-1)  15 (-1, 0,-1)  16 (+1, 0,-1)  17 ( 0,-1,-1)  18 ( 0,+1,-1)
 *   opposite: 1<->2, 3<->4, 5<->6, 7<->8, 9+i <-> 14+i (i = 0..4).
 *
 * Layout at the boundary: AoS float[nz][ny][nx][19]; obstacles uint8[nz][ny][nx].
 * Inside: per z plane all 19 populations, f[z+3][k][y][px], with three ghost
 * planes below and above; the domain is cut into z slabs (one per rank /
 * sub-domain); one-step launches move each slab's top plane speeds 9..13 and
 * bottom plane speeds 14..18 to the neighbour's ghost planes, two-step passes
 * two whole planes each way, three-step passes (the default for one slab or
 * slabs of >= 6 planes, both numerics) three planes each way (a single slab's
 * ghost planes refreshed from the periodic images).
 *
 * Placement reuses lbm_config (lbm_hip.h): parts = z slabs, transport LOCAL
 * (all slabs in this process, device copies) or RCCL (one slab per rank);
 * kernel / graph fields are ignored; flags may carry LBM_FLAG_TOLERANCE: the
 * two- and three-step passes then use the reciprocal collision (one v_rcp_f32 without a Newton
 * step for u, FMA contraction; not bitwise equal to the restatement, within
 * the tolerance tests/test_d3q19.py states), one-step launches stay bitwise.
 */
#ifndef LBM3D_HIP_H
#define LBM3D_HIP_H

#include <stdint.h>

#include "lbm_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

#define LBM3D_Q 19

typedef struct lbm3d_params {
    int32_t nx, ny, nz;
    int32_t max_iters;
    float density;
    float accel;
    float omega;
} lbm3d_params;

typedef struct lbm3d_handle lbm3d_handle;

/* Create the engine: obstacles uint8[nz][ny][nx] (full domain).
 * Single-slab engines of >= 2^26 cells run a placement probe here (DESIGN.md
 * section 4.9): up to six candidate lattice pairs timed with the engine's own
 * pass form, at most 128 GB of device memory held transiently (about 124 GB
 * at 512^3), the fastest kept and the rest freed before the call returns. */
int lbm3d_create(const lbm3d_params *params, const uint8_t *obstacles, const lbm_config *config,
                 lbm3d_handle **out);

/* Equilibrium at rest: f_k = density * w_k. */
int lbm3d_init_equilibrium(lbm3d_handle *h);

/* Host AoS float[nz][ny][nx][19] (full domain) -> device. */
int lbm3d_load_cells(lbm3d_handle *h, const float *cells_aos);

/* `steps` steps (blocking); av_vels of these steps stay on the device. */
int lbm3d_run_steps(lbm3d_handle *h, int32_t steps);

/* Device -> host AoS (full-domain array; RCCL: this rank's slab only) and
 * av_vels[n_av] of the last run, combined over all ranks.  Either may be NULL. */
int lbm3d_store(lbm3d_handle *h, float *cells_aos, float *av_vels, int32_t n_av);

/* Device-event seconds of the last lbm3d_run_steps. */
int lbm3d_last_run_seconds(lbm3d_handle *h, double *seconds);

/* Fluid (non-obstacle) cells of the full domain. */
int64_t lbm3d_total_free_cells(lbm3d_handle *h);

/* Local slab z ranges: z0[i], nz[i] for i < *n_out (LOCAL: all; RCCL: this rank's). */
int lbm3d_local_slabs(lbm3d_handle *h, int32_t *z0, int32_t *nz, int32_t max_slabs, int32_t *n_out);

/*
 * The ordered ghost-exchange posts of z slab `rank` of `parts` (host-only;
 * the engine's RCCL exchanges iterate the same list, lbm3d.hip slab_posts):
 * send up (dir 0, +z), send down (dir 1), receive the below ghosts (dir 1),
 * receive the above ghosts (dir 0), periodic in z.  planes = 1: the five
 * speed planes leaving a face (one-step launches); 2 / 3: that many whole
 * planes, all 19 speeds (two- / three-step passes).  floats use the engine's
 * default plane layout (rows padded to 16 floats).  Writes 4 lbm_xfer
 * (lbm_hip.h) to out (may be NULL) and *n_out = 4.
 */
int lbm3d_exchange_schedule(int32_t nx, int32_t ny, int32_t nz, int32_t parts, int32_t rank, int32_t planes,
                            lbm_xfer *out, int32_t max_out, int32_t *n_out);

const char *lbm3d_last_error(lbm3d_handle *h);

void lbm3d_destroy(lbm3d_handle *h);

#ifdef __cplusplus
}
#endif

#endif /* LBM3D_HIP_H */

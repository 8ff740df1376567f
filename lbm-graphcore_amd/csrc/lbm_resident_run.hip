// lbm_resident_run.hip -- host side of the lattice-resident kernel (lbm_resident.hip):
// tile choice, the launch, and the residency-failure fallback to STEP2.

#include "lbm_engine.hpp"

// Pick the resident tile height (smallest with at most one tile per CU,
// or LBM_RES_TH) and allocate the granule buffer.  false: does not fit.
bool lbm_handle::setup_resident(const Sub &s) {
    set_device(s);
    int cus = 0;
    HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, s.dev));
    // v2 (packed pairs, 128-column tiles) needs an even width; v1 takes any grid
    std::vector<int> order;
    // (smallest tile height with one tile per CU first, except that 2-row
    // tiles are slower than 4-row ones on every grid measured:
    // profiles/r01/resident/)
    if (p.nx % 2 == 0 && (res_version == 0 || res_version == 2))
        order.insert(order.end(), {RES2_4, RES2_8, RES2_16, RES2_32, RES2_2, RES2_16x8});
    if (res_version == 0 || res_version == 1) order.insert(order.end(), {RES_4, RES_8, RES_16, RES_32, RES_64, RES_16x4});
    res_variant = -1;
    for (int v : order) {
        if (res_th_env > 0 && RES_TH[v] != res_th_env) continue;
        const int tx = (p.nx + RES_TWV[v] - 1) / RES_TWV[v];
        const int ty = (p.ny + RES_TH[v] - 1) / RES_TH[v];
        int cap = 0;
        HIP_CHECK(resident_capacity(v, s.dev, tolerance && RES_VER[v] >= 2, cap));
        const long long n = (long long)tx * ty;
        // LBM_DEBUG_RES_OVERSUBSCRIBE=1: take the first tile shape whatever
        // the capacity -- a grid that cannot be co-resident (tests)
        if ((n <= cap && n <= (long long)res_per_cu * cus) || res_oversubscribe) {
            res_variant = v;
            res_tx = tx;
            res_ty = ty;
            break;
        }
    }
    if (res_variant < 0) return false;
    const size_t granules = 2ull * res_tx * res_ty * 8 * RES_GV[res_variant] * RES_GW;
    // granules validate by their step tag (== the expected step, never 0 or
    // all-ones in a run): the poison pattern reads as "not there yet"
    HIP_CHECK(hipMalloc(&res_halo, granules * sizeof(unsigned long long)));
    fill_fresh(res_halo, granules * sizeof(unsigned long long), s.s_comp);
    HIP_CHECK(hipMalloc(&res_status, 64));
    fill_zero(res_status, 64, s.s_comp);
    int khz = 0;
    HIP_CHECK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, s.dev));
    res_timeout = (long long)std::max(khz, 1000) * res_timeout_ms;  // 2 s of wall clock per poll phase
    return true;
}

// Every step of the run in one cooperative launch (lbm_resident.hip),
// then the fixed-order |u| fold.  The ghost ring of the result is not
// maintained (the resident kernel reads the periodic images itself; a
// STEP2 fallback rebuilds it).  Returns false when a neighbour hand-off
// timed out (the tiles were not all co-resident): the kernel only reads
// s.o[s.cur] and writes the other lattice, so the input lattice -- with
// the first accelerate applied -- is intact, and s.cur, res_tag and
// last_steps are left as they were.
bool lbm_handle::run_resident(int steps, bool accelerate_first) {
    Sub &s = subs[0];
    set_device(s);
    const int ntiles = res_tx * res_ty;
    if ((long long)steps * ntiles > res_partials_cap) {
        if (res_partials) HIP_CHECK(hipFree(res_partials));
        res_partials = nullptr;
        res_partials_cap = (long long)std::max(steps, 1) * ntiles;
        HIP_CHECK(hipMalloc(&res_partials, sizeof(float) * (size_t)res_partials_cap));
    }
    HIP_CHECK(hipMemsetAsync(res_status, 0, 64, s.s_comp));
    HIP_CHECK(hipEventRecord(t0, s.s_comp));
    if (accelerate_first && s.accel_row >= 0) {
        const float w1 = p.density * p.accel / 9.f;
        const float w2 = p.density * p.accel / 36.f;
        timed(s, s.s_comp, "accelerate_row", [&] {
            HIP_CHECK(launch_accelerate(s.o[s.cur], s.obst, s.plane, s.pitch, s.w, s.accel_row, w1, w2, s.s_comp));
        });
    }
    if (steps > 0) {
        ResidentArgs a{};
        a.fin = s.o[s.cur];
        a.fout = s.o[1 - s.cur];
        a.obst = s.obst;
        a.plane = s.plane;
        a.pitch = s.pitch;
        a.nx = p.nx;
        a.ny = p.ny;
        a.tiles_x = res_tx;
        a.tiles_y = res_ty;
        a.steps = steps;
        a.tag0 = res_tag;
        a.accel_row = p.ny >= 2 ? p.ny - 2 : -1;
        a.omega = p.omega;
        a.omo = 1 - p.omega;
        a.w1 = p.density * p.accel / 9.f;
        a.w2 = p.density * p.accel / 36.f;
        a.tc0 = p.omega * (4.f / 9.f);
        a.tc1 = p.omega * (1.f / 9.f);
        a.tc2 = p.omega * (1.f / 36.f);
        a.halo = res_halo;
        a.partials = res_partials;
        a.status = res_status;
        a.timeout_ticks = res_timeout;
        a.early_poll = res_early_poll;
        a.stall_tile = res_stall_tile;
        a.stall_step = res_stall_step;
        long long *trace = nullptr;
        unsigned long long *htrace = nullptr;
        const int trace_steps = std::min(steps, 256);
        const int trace_mode = knob("LBM_RES_TRACE", 0);
        if (trace_mode) {
            HIP_CHECK(hipMalloc(&trace, sizeof(long long) * 5 * trace_steps));
            HIP_CHECK(hipMemsetAsync(trace, 0, sizeof(long long) * 5 * trace_steps, s.s_comp));
            a.trace = trace;
            a.trace_steps = trace_steps;
        }
        if (trace_mode >= 2) {
            const size_t n = sizeof(unsigned long long) * 2 * trace_steps * ntiles;
            HIP_CHECK(hipMalloc(&htrace, n));
            HIP_CHECK(hipMemsetAsync(htrace, 0, n, s.s_comp));
            a.htrace = htrace;
        }
        bool rejected = false;  // the cooperative launch refused the grid: a residency failure too
        timed(s, s.s_comp, std::string("resident_steps (all steps, one launch)") + (tolerance && RES_VER[res_variant] >= 2 ? " tolerance" : ""),
              [&] {
                  const hipError_t e = launch_resident(a, res_variant, tolerance && RES_VER[res_variant] >= 2,
                                                       res_coop, s.s_comp);
                  if (e == hipErrorCooperativeLaunchTooLarge) {
                      (void)hipGetLastError();
                      rejected = true;
                  } else {
                      HIP_CHECK(e);
                  }
              });
        if (rejected) HIP_CHECK(hipMemsetAsync(res_status, 0xff, sizeof(int), s.s_comp));
        if (htrace) {  // per tile and step: wait for the slowest neighbour, then the hop itself
            std::vector<unsigned long long> hv((size_t)2 * trace_steps * ntiles);
            HIP_CHECK(hipMemcpyAsync(hv.data(), htrace, hv.size() * 8, hipMemcpyDeviceToHost, s.s_comp));
            HIP_CHECK(hipStreamSynchronize(s.s_comp));
            HIP_CHECK(hipFree(htrace));
            double wait = 0, hop = 0, step = 0, hop_max = 0;
            long long cnt = 0;
            for (int t = 2; t + 1 < trace_steps; ++t)
                for (int tl = 0; tl < ntiles; ++tl) {
                    const int tx = tl % res_tx, ty = tl / res_tx;
                    unsigned long long nbmax = 0;
                    for (int dy = -1; dy <= 1; ++dy)
                        for (int dx = -1; dx <= 1; ++dx) {
                            if (!dx && !dy) continue;
                            const int nt = ((ty + dy + res_ty) % res_ty) * res_tx + (tx + dx + res_tx) % res_tx;
                            nbmax = std::max(nbmax, hv[((size_t)t * ntiles + nt) * 2]);
                        }
                    const unsigned long long own = hv[((size_t)t * ntiles + tl) * 2];
                    const unsigned long long ready = hv[((size_t)t * ntiles + tl) * 2 + 1];
                    wait += (double)nbmax - (double)own;
                    hop += (double)ready - (double)nbmax;
                    hop_max = std::max(hop_max, (double)ready - (double)nbmax);
                    step += (double)hv[((size_t)(t + 1) * ntiles + tl) * 2] - (double)own;
                    ++cnt;
                }
            int khz = 1;
            HIP_CHECK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, s.dev));
            const double us = 1e3 / khz;
            fprintf(stderr, "[resident hop] %dx%d tile-height %d early_poll %d: per tile-step (us) own collision end -> "
                    "slowest neighbour's %.3f, -> ring ready %.3f (max %.3f), collision end to next %.3f\n", p.nx,
                    p.ny, RES_TH[res_variant], res_early_poll, wait / cnt * us, hop / cnt * us, hop_max * us,
                    step / cnt * us);
        }
        if (trace) {  // mean phase durations over the traced steps (skipping the first)
            std::vector<long long> tv((size_t)5 * trace_steps);
            HIP_CHECK(hipMemcpyAsync(tv.data(), trace, tv.size() * sizeof(long long), hipMemcpyDeviceToHost, s.s_comp));
            HIP_CHECK(hipStreamSynchronize(s.s_comp));
            HIP_CHECK(hipFree(trace));
            double ph[5] = {0, 0, 0, 0, 0};
            int n = 0;
            for (int t = 1; t + 1 < trace_steps; ++t, ++n) {
                const long long *r = &tv[(size_t)5 * t];
                ph[0] += (double)(r[1] - r[0]);
                ph[1] += (double)(r[2] - r[1]);
                ph[2] += (double)(r[3] - r[2]);
                ph[3] += (double)(r[4] - r[3]);
                ph[4] += (double)(tv[(size_t)5 * (t + 1)] - r[0]);
            }
            int khz = 1;
            HIP_CHECK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, s.dev));
            const double us = 1e3 / khz / std::max(n, 1);
            fprintf(stderr, "[resident trace] %dx%d tile-height %d: per step (us) pull+barrier %.3f collide+publish %.3f "
                    "poll %.3f barrier %.3f total %.3f\n", p.nx, p.ny, RES_TH[res_variant], ph[0] * us, ph[1] * us,
                    ph[2] * us, ph[3] * us, ph[4] * us);
        }
        timed(s, s.s_comp, "resident_reduce",
              [&] { HIP_CHECK(launch_resident_reduce(res_partials, s.av_local, steps, ntiles, s.s_comp)); });
    }
    HIP_CHECK(hipEventRecord(t1, s.s_comp));
    HIP_CHECK(hipEventSynchronize(t1));
    float ms = 0.f;
    HIP_CHECK(hipEventElapsedTime(&ms, t0, t1));
    int status = 0;
    HIP_CHECK(hipMemcpy(&status, res_status, sizeof(int), hipMemcpyDeviceToHost));
    prof_collect();
    if (status != 0) return false;
    if (steps > 0) {
        res_tag += (unsigned)steps;
        s.cur ^= 1;
    }
    last_seconds = ms * 1e-3;
    last_steps = steps;
    return true;
}

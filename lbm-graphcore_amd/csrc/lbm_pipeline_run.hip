// lbm_pipeline_run.hip -- step loop of the unfused per-stage pipeline (lbm_pipeline.hip,
// LbmPoplibs.cpp:225-233).

#include "lbm_engine.hpp"

// Unfused pipeline, one kernel per stage (lbm_pipeline.hip): every step
// accelerates row ny-2 (conditionally), refreshes the W1 ghost ring of
// the current lattice (exchanging across sub-domains), propagates into
// the other lattice, rebounds / collides back, and folds the |u|
// partials into av_local[t].  The current lattice never changes parity.
void lbm_handle::run_pipeline(int steps) {
    const float w1 = p.density * p.accel / 9.f;
    const float w2 = p.density * p.accel / 36.f;
    Sub &s0 = subs[0];
    set_device(s0);
    HIP_CHECK(hipEventRecord(t0, s0.s_comp));
    for (size_t k = 1; k < subs.size(); ++k) {
        set_device(subs[k]);
        HIP_CHECK(hipStreamWaitEvent(subs[k].s_comp, t0, 0));
    }
    for (int t = 0; t < steps; ++t) {
        for (auto &s : subs) {
            if (s.accel_row < 0 || p.ny < 2) continue;
            set_device(s);
            timed(s, s.s_comp, "accelerate_row", [&] {
                HIP_CHECK(launch_accelerate(s.o[s.cur], s.obst, s.plane, s.pitch, s.w, s.accel_row, w1, w2, s.s_comp));
            });
        }
        refresh_halos();
        for (auto &s : subs) {
            set_device(s);
            float *cells = s.o[s.cur], *tmp = s.o[1 - s.cur];
            debug_delay(s, s.s_comp);
            timed(s, s.s_comp, "pipe_propagate",
                  [&] { HIP_CHECK(launch_pipe_propagate(cells, tmp, s.plane, s.pitch, s.w, s.h, s.s_comp)); });
            timed(s, s.s_comp, "pipe_rebound",
                  [&] { HIP_CHECK(launch_pipe_rebound(tmp, cells, s.obst, s.plane, s.pitch, s.w, s.h, s.s_comp)); });
            timed(s, s.s_comp, "pipe_collision", [&] {
                HIP_CHECK(launch_pipe_collision(tmp, cells, s.obst, s.plane, s.pitch, s.w, s.h, p.omega,
                                                s.pipe_partials, s.s_comp));
            });
            timed(s, s.s_comp, "pipe_av", [&] {
                HIP_CHECK(launch_pipe_av(s.pipe_partials, pipe_blocks(s.w, s.h), s.av_local, t, s.s_comp));
            });
        }
    }
    for (auto &s : subs) {
        set_device(s);
        HIP_CHECK(hipEventRecord(s.ev_end, s.s_comp));
    }
    set_device(s0);
    for (size_t k = 1; k < subs.size(); ++k) HIP_CHECK(hipStreamWaitEvent(s0.s_comp, subs[k].ev_end, 0));
    HIP_CHECK(hipEventRecord(t1, s0.s_comp));
    HIP_CHECK(hipEventSynchronize(t1));
    float ms = 0.f;
    HIP_CHECK(hipEventElapsedTime(&ms, t0, t1));
    last_seconds = ms * 1e-3;
    last_steps = steps;
    sync_all();
    prof_collect();
}

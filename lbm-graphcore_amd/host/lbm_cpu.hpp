// lbm_cpu.hpp -- host CPU backend of lbm_runner (--device cpu), the
// counterpart of the reference's non-IPU device choice (main/LbmRunner.cpp:18,
// --device ipu|ipumodel; SURVEY.md §5 "Config / flags").  Product code: the
// same fused D2Q9-BGK step as the GPU engine's bitwise mode, for hosts
// without a GPU and for runs too small to be worth one.
//
// Numerics: the per-cell arithmetic of main/LastChance.cpp:192-262 in its
// own operand order (no reassociation, -ffp-contract=off), so the lattice is
// bit-identical to the GPU engine's bitwise mode and to the reference for any
// step count; av_vels sum |u| per row and then the rows in order (the
// reference sums sequentially over the whole grid), so they agree to summation
// order, as the GPU engine's do.
//
// Layout: two planar SoA lattices f[k][ny][nx] (ping-pong) built from the
// boundary's AoS cells on load; rows are split across OpenMP threads, each
// row pulls from rows y-1, y, y+1 with the periodic wrap of
// LastChance.cpp:196-200.
#pragma once

#include <chrono>
#include <cmath>
#include <cstdint>
#include <vector>

#ifdef _OPENMP
#include <omp.h>
#endif

namespace lbmcpu {

constexpr int Q = 9;

class Engine {
  public:
    Engine(int nx, int ny, float density, float accel, float omega, const std::vector<uint8_t> &obstacles)
        : nx_(nx), ny_(ny), density_(density), accel_(accel), omega_(omega), obst_(obstacles) {
        for (auto &l : f_) l.assign((size_t)Q * nx_ * ny_, 0.f);
        row_u_.assign(ny_, 0.f);
        for (uint8_t o : obst_) free_cells_ += o ? 0 : 1;
    }

    static int threads() {
#ifdef _OPENMP
        return omp_get_max_threads();
#else
        return 1;
#endif
    }

    // run(0): AoS float[ny][nx][9] -> planar lattice 0
    void load(const std::vector<float> &aos) {
        cur_ = 0;
        float *f = f_[0].data();
        const size_t n = (size_t)nx_ * ny_;
        for (size_t i = 0; i < n; ++i)
            for (int k = 0; k < Q; ++k) f[k * n + i] = aos[i * Q + k];
    }

    // run(2): the current lattice back to AoS
    void store(std::vector<float> &aos) const {
        const float *f = f_[cur_].data();
        const size_t n = (size_t)nx_ * ny_;
        aos.resize(n * Q);
        for (size_t i = 0; i < n; ++i)
            for (int k = 0; k < Q; ++k) aos[i * Q + k] = f[k * n + i];
    }

    // run(1): the conditional first acceleration (LastChance.cpp:161-183),
    // then `steps` fused steps; av_vels[t] per step.  Returns wall seconds of
    // the step loop.
    double run(int steps, std::vector<float> &av_vels) {
        av_vels.assign(steps, 0.f);
        const auto t0 = std::chrono::steady_clock::now();
        accelerate_first();
        for (int t = 0; t < steps; ++t) {
            step(f_[cur_].data(), f_[1 - cur_].data());
            cur_ = 1 - cur_;
            float tot = 0.f;
            for (int y = 0; y < ny_; ++y) tot += row_u_[y];
            av_vels[t] = tot / (float)free_cells_;
        }
        return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    }

  private:
    float w1() const { return density_ * accel_ / 9.f; }
    float w2() const { return density_ * accel_ / 36.f; }

    void accelerate_first() {
        if (ny_ < 2) return;
        const size_t n = (size_t)nx_ * ny_;
        float *f = f_[cur_].data();
        const int y = ny_ - 2;
        const float a1 = w1(), a2 = w2();
        for (int x = 0; x < nx_; ++x) {
            const size_t c = (size_t)y * nx_ + x;
            if (obst_[c] || !(f[3 * n + c] - a1 > 0.f) || !(f[6 * n + c] - a2 > 0.f) || !(f[7 * n + c] - a2 > 0.f))
                continue;
            f[1 * n + c] += a1;
            f[5 * n + c] += a2;
            f[8 * n + c] += a2;
            f[3 * n + c] -= a1;
            f[6 * n + c] -= a2;
            f[7 * n + c] -= a2;
        }
    }

    void step(const float *src, float *dst) {
        const size_t n = (size_t)nx_ * ny_;
        const float omega = omega_, omo = 1 - omega_;
        const float a1 = w1(), a2 = w2();
#pragma omp parallel for schedule(static)
        for (int y = 0; y < ny_; ++y) {
            const int yn = y + 1 == ny_ ? 0 : y + 1, ys = y == 0 ? ny_ - 1 : y - 1;
            const size_t r = (size_t)y * nx_, rn = (size_t)yn * nx_, rs = (size_t)ys * nx_;
            const float acc = (y == ny_ - 2) ? 1.00f : 0.00f;
            float tot = 0.f;
            for (int x = 0; x < nx_; ++x) {
                const int xe = x + 1 == nx_ ? 0 : x + 1, xw = x == 0 ? nx_ - 1 : x - 1;
                float s[Q];
                s[0] = src[0 * n + r + x];
                s[1] = src[1 * n + r + xw];
                s[2] = src[2 * n + rs + x];
                s[3] = src[3 * n + r + xe];
                s[4] = src[4 * n + rn + x];
                s[5] = src[5 * n + rs + xw];
                s[6] = src[6 * n + rs + xe];
                s[7] = src[7 * n + rn + xe];
                s[8] = src[8 * n + rn + xw];
                float o[Q];
                if (obst_[r + x]) {
                    static constexpr int opp[Q] = {0, 3, 4, 1, 2, 7, 8, 5, 6};
                    for (int k = 0; k < Q; ++k) o[k] = s[opp[k]];
                } else {
                    const float rho = s[0] + s[1] + s[2] + s[3] + s[4] + s[5] + s[6] + s[7] + s[8];
                    const float ux = (s[1] + s[5] + s[8] - (s[3] + s[6] + s[7])) / rho;
                    const float uy = (s[2] + s[5] + s[6] - (s[4] + s[7] + s[8])) / rho;
                    const float usq = ux * ux + uy * uy;
                    const float c = 1.00f - usq * 1.50f;
                    const float ld0 = 4.00f / 9.00f * rho * omega;
                    const float ld1 = rho / 9.00f * omega;
                    const float ld2 = rho / 36.00f * omega;
                    const float us = ux + uy, ud = -ux + uy;
                    auto eq = [&](float ld, float v, float k45, float k23v) { return ld * ((k45 * v) * k23v + c); };
                    o[0] = s[0] * omo + ld0 * c;
                    o[1] = s[1] * omo + eq(ld1, ux, 4.50f, 2.00f / 3.00f + ux) + acc * a1;
                    o[2] = s[2] * omo + eq(ld1, uy, 4.50f, 2.00f / 3.00f + uy);
                    o[3] = s[3] * omo + eq(ld1, ux, -4.50f, 2.00f / 3.00f - ux) - acc * a1;
                    o[4] = s[4] * omo + eq(ld1, uy, -4.50f, 2.00f / 3.00f - uy);
                    o[5] = s[5] * omo + eq(ld2, us, 4.50f, 2.00f / 3.00f + us) + acc * a2;
                    o[6] = s[6] * omo + eq(ld2, ud, 4.50f, 2.00f / 3.00f + ud) - acc * a2;
                    o[7] = s[7] * omo + eq(ld2, us, -4.50f, 2.00f / 3.00f - us) - acc * a2;
                    o[8] = s[8] * omo + eq(ld2, ud, -4.50f, 2.00f / 3.00f - ud) + acc * a2;
                    tot += std::sqrt(usq);
                }
                for (int k = 0; k < Q; ++k) dst[k * n + r + x] = o[k];
            }
            row_u_[y] = tot;
        }
    }

    int nx_, ny_;
    float density_, accel_, omega_;
    std::vector<uint8_t> obst_;
    std::vector<float> f_[2];
    std::vector<float> row_u_;
    int cur_ = 0;
    long long free_cells_ = 0;
};

}  // namespace lbmcpu

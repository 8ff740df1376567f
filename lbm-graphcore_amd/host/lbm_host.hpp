// lbm_host.hpp -- host-side problem I/O kept from the reference so its gate
// (check/check.py) keeps working unchanged.
//
//   Params::fromFile        main/include/LbmParams.hpp:28-58
//   Obstacles::fromFile     main/include/LbmParams.hpp:92-123 (+ bounds check,
//                           as LastChance.cpp:476-478 does)
//   initialiseCells         main/include/LatticeBoltzmannUtils.hpp:137-157
//   reynoldsNumber          LatticeBoltzmannUtils.hpp:202-205
//   writeAverageVelocities  LatticeBoltzmannUtils.hpp:208-219
//   writeResults            LatticeBoltzmannUtils.hpp:221-281
//   averageVelocity         LastChance.cpp:290-339 (used by compare_lbm)
//   timedStep               main/include/GraphcoreUtils.hpp:130-138
#pragma once

#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <fstream>
#include <iomanip>
#include <iostream>
#include <optional>
#include <string>
#include <vector>

#include "lbm_hip.h"

namespace lbmhost {

constexpr unsigned NumSpeeds = 9;

struct Params {
    size_t nx = 0, ny = 0, maxIters = 0, reynolds_dim = 0;
    float density = 0.f, accel = 0.f, omega = 0.f;

    static std::optional<Params> fromFile(const std::string &filename) {
        std::ifstream file(filename);
        if (!file.is_open()) {
            std::cerr << "Could not read parameters from " << filename << std::endl;
            return std::nullopt;
        }
        try {
            std::string line;
            auto u = [&]() -> size_t { std::getline(file, line); return std::stoul(line); };
            auto f = [&]() -> float { std::getline(file, line); return std::stof(line); };
            Params p;
            p.nx = u();
            p.ny = u();
            p.maxIters = u();
            p.reynolds_dim = u();
            p.density = f();
            p.accel = f();
            p.omega = f();
            return p;
        } catch (const std::exception &) {
            std::cerr << "Could not read parameters from " << filename << std::endl;
            return std::nullopt;
        }
    }

    lbm_params abi() const {
        return lbm_params{(int32_t)nx, (int32_t)ny, (int32_t)maxIters, (int32_t)reynolds_dim, density, accel, omega};
    }
};

struct Obstacles {
    size_t nx = 0, ny = 0;
    std::vector<uint8_t> data;  // [ny][nx]

    bool at(size_t x, size_t y) const { return data[y * nx + x] != 0; }

    static std::optional<Obstacles> fromFile(size_t nx, size_t ny, const std::string &filename) {
        std::ifstream file(filename);
        if (!file.is_open()) {
            std::cerr << "Could not read parameters from " << filename << std::endl;
            return std::nullopt;
        }
        Obstacles o;
        o.nx = nx;
        o.ny = ny;
        o.data.assign(nx * ny, 0);
        std::string line;
        while (std::getline(file, line)) {
            int x = 0, y = 0, v = 0;
            const int n = sscanf(line.c_str(), "%d %d %d", &x, &y, &v);
            if (n <= 0) break;  // blank tail ends the list
            if (n != 3 || v != 1) {
                std::cerr << "Malformed line: obstacle must be 1" << std::endl;
                return std::nullopt;
            }
            if (x < 0 || y < 0 || (size_t)x >= nx || (size_t)y >= ny) {
                std::cerr << "obstacle (" << x << "," << y << ") outside the grid" << std::endl;
                return std::nullopt;
            }
            o.data[(size_t)y * nx + (size_t)x] = 1;
        }
        return o;
    }
};

inline std::vector<float> initialiseCells(const Params &p) {
    std::vector<float> c(p.nx * p.ny * NumSpeeds);
    const float w0 = p.density * 4.f / 9.f, w1 = p.density / 9.f, w2 = p.density / 36.f;
    for (size_t i = 0; i < p.nx * p.ny; ++i) {
        float *s = &c[i * NumSpeeds];
        s[0] = w0;
        s[1] = s[2] = s[3] = s[4] = w1;
        s[5] = s[6] = s[7] = s[8] = w2;
    }
    return c;
}

inline float reynoldsNumber(const Params &p, float average_velocity) {
    const float viscosity = 1.f / 6.f * (2.f / p.omega - 1.f);
    return average_velocity * p.reynolds_dim / viscosity;
}

struct Macro {
    float ux, uy, u, pressure;
};

inline Macro macroscopic(const Params &p, const Obstacles &o, const std::vector<float> &cells, size_t ii, size_t jj) {
    const float c_sq = 1.f / 3.f;
    if (o.at(ii, jj)) return Macro{0.f, 0.f, 0.f, p.density * c_sq};
    const float *c = &cells[(ii + jj * p.nx) * NumSpeeds];
    float rho = 0.f;
    for (unsigned k = 0; k < NumSpeeds; ++k) rho += c[k];
    const float ux = (c[1] + c[5] + c[8] - (c[3] + c[6] + c[7])) / rho;
    const float uy = (c[2] + c[5] + c[6] - (c[4] + c[7] + c[8])) / rho;
    return Macro{ux, uy, sqrtf((ux * ux) + (uy * uy)), rho * c_sq};
}

inline float averageVelocity(const Params &p, const Obstacles &o, const std::vector<float> &cells) {
    int tot_cells = 0;
    float tot_u = 0.f;
    for (size_t jj = 0; jj < p.ny; ++jj)
        for (size_t ii = 0; ii < p.nx; ++ii)
            if (!o.at(ii, jj)) {
                tot_u += macroscopic(p, o, cells, ii, jj).u;
                ++tot_cells;
            }
    return tot_u / (float)tot_cells;
}

inline bool writeAverageVelocities(const std::string &filename, const std::vector<float> &av_vels) {
    std::ofstream file(filename);
    if (!file.is_open()) return false;
    for (size_t i = 0; i < av_vels.size(); ++i)
        file << i << ":\t" << std::scientific << std::setprecision(12) << av_vels[i] << "\n";
    return true;
}

inline bool writeResults(const std::string &filename, const Params &p, const Obstacles &o,
                         const std::vector<float> &cells) {
    std::ofstream file(filename);
    if (!file.is_open()) return false;
    for (size_t jj = 0; jj < p.ny; ++jj)
        for (size_t ii = 0; ii < p.nx; ++ii) {
            const Macro m = macroscopic(p, o, cells, ii, jj);
            file << ii << " " << jj << " " << std::setprecision(12) << std::scientific << m.ux << " " << m.uy << " "
                 << m.u << " " << m.pressure << " " << (int)o.at(ii, jj) << "\n";
        }
    return true;
}

template <class F>
double timedStep(const std::string &description, F &&f) {
    std::cerr << std::setw(60) << description;
    const auto tic = std::chrono::high_resolution_clock::now();
    f();
    const auto toc = std::chrono::high_resolution_clock::now();
    const double s = std::chrono::duration<double>(toc - tic).count();
    std::cerr << " took " << std::right << std::setw(12) << std::setprecision(5) << s << "s" << std::endl;
    return s;
}

// Fail loudly on any C-ABI error.
inline void check(int rc, lbm_handle *h, const char *what) {
    if (rc != LBM_OK) {
        std::cerr << what << " failed (" << rc << "): " << lbm_last_error(h) << std::endl;
        std::exit(EXIT_FAILURE);
    }
}

}  // namespace lbmhost

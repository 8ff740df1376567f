// Host code under AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY §5
// "Race detection / sanitizers": host ASan/UBSan on the CPU path).  Built and
// run by tests/test_sanitizers.py with -fsanitize=address,undefined
// -fno-sanitize-recover=all, so any invalid access, leak or UB aborts.
//
// Exercises the host side the product keeps from the reference: the params /
// obstacles loaders (lbm-graphcore_amd/host/lbm_host.hpp, restating
// LbmParams.hpp:28-58, :92-123) on the reference's own files and on
// malformed ones, the equilibrium initialisation, the .dat writers
// (LatticeBoltzmannUtils.hpp:208-281), the Reynolds number, and the CPU
// oracle (oracle/lbm_oracle.c, lbm_oracle3d.c: test infrastructure) on small
// problems: full runs, ghosted sub-block steps, the unfused pipeline, the
// OpenMP restatement and the D3Q19 restatement.
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <string>
#include <vector>

#include "../../lbm-graphcore_amd/host/lbm_host.hpp"

extern "C" {
typedef struct {
    int32_t nx, ny, max_iters, reynolds_dim;
    float density, accel, omega;
} oracle_params;
typedef struct {
    int32_t nx, ny, nz, max_iters;
    float density, accel, omega;
} oracle3d_params;
void oracle_init_equilibrium(const oracle_params *p, float *cells);
int64_t oracle_free_cells(const oracle_params *p, const uint8_t *obst);
float oracle_step_ghosted(const oracle_params *p, int w, int h, const float *old, float *out, const uint8_t *obst,
                          int accel_row);
int oracle_run(const oracle_params *p, float *cells, const uint8_t *obst, int iters, float *av_vels);
int oracle_run_mt(const oracle_params *p, float *cells, const uint8_t *obst, int iters, float *av_vels, int threads);
int oracle_pipe_run(const oracle_params *p, float *cells, const uint8_t *obst, int iters, float *av_vels);
float oracle_av_velocity(const oracle_params *p, const float *cells, const uint8_t *obst);
void oracle3d_init_equilibrium(const oracle3d_params *p, float *cells);
int oracle3d_run(const oracle3d_params *p, float *cells, const uint8_t *obst, int iters, float *av_vels);
}

static int fails = 0;
#define EXPECT(c)                                                          \
    do {                                                                   \
        if (!(c)) {                                                        \
            std::fprintf(stderr, "host_check: %s:%d: %s\n", __FILE__, __LINE__, #c); \
            ++fails;                                                       \
        }                                                                  \
    } while (0)

static void write_file(const std::string &path, const std::string &text) {
    std::ofstream f(path);
    f << text;
}

int main(int argc, char **argv) {
    if (argc < 3) {
        std::fprintf(stderr, "usage: host_check GOLDEN_PARAMS_DIR TMP_DIR\n");
        return 2;
    }
    const std::string gold = argv[1], tmp = argv[2];
    const char *grids[] = {"128x128", "128x256", "256x256", "1024x1024"};
    for (const char *g : grids) {
        auto p = lbmhost::Params::fromFile(gold + "/input_" + g + ".params");
        EXPECT(p.has_value());
        if (!p) continue;
        auto o = lbmhost::Obstacles::fromFile(p->nx, p->ny, gold + "/obstacles_" + g + ".dat");
        EXPECT(o.has_value());
        if (!o) continue;
        EXPECT(o->data.size() == p->nx * p->ny);
    }
    // malformed inputs are rejected, never read out of bounds
    write_file(tmp + "/bad.params", "128\n128\nnot-a-number\n");
    EXPECT(!lbmhost::Params::fromFile(tmp + "/bad.params").has_value());
    write_file(tmp + "/empty.params", "");
    EXPECT(!lbmhost::Params::fromFile(tmp + "/empty.params").has_value());
    EXPECT(!lbmhost::Params::fromFile(tmp + "/missing.params").has_value());
    write_file(tmp + "/oob.dat", "3 4 1\n200 4 1\n");
    EXPECT(!lbmhost::Obstacles::fromFile(16, 8, tmp + "/oob.dat").has_value());
    write_file(tmp + "/neg.dat", "-1 2 1\n");
    EXPECT(!lbmhost::Obstacles::fromFile(16, 8, tmp + "/neg.dat").has_value());
    write_file(tmp + "/val.dat", "1 2 0\n");
    EXPECT(!lbmhost::Obstacles::fromFile(16, 8, tmp + "/val.dat").has_value());
    write_file(tmp + "/short.dat", "1 2\n");
    EXPECT(!lbmhost::Obstacles::fromFile(16, 8, tmp + "/short.dat").has_value());

    // the 128x128 reference problem, 50 steps, writers and Reynolds
    auto p = lbmhost::Params::fromFile(gold + "/input_128x128.params");
    auto o = lbmhost::Obstacles::fromFile(p->nx, p->ny, gold + "/obstacles_128x128.dat");
    std::vector<float> cells = lbmhost::initialiseCells(*p);
    const oracle_params op{(int32_t)p->nx, (int32_t)p->ny, 50, (int32_t)p->reynolds_dim, p->density, p->accel,
                           p->omega};
    std::vector<float> av(50, 0.f), av2(50, 0.f);
    std::vector<float> c2 = cells;
    EXPECT(oracle_run(&op, cells.data(), o->data.data(), 50, av.data()) == 0);
    EXPECT(oracle_run_mt(&op, c2.data(), o->data.data(), 50, av2.data(), 4) == 0);
    EXPECT(cells == c2);
    EXPECT(oracle_free_cells(&op, o->data.data()) == 15876);
    const float av_last = lbmhost::averageVelocity(*p, *o, cells);
    EXPECT(av_last > 0.f && av_last == oracle_av_velocity(&op, cells.data(), o->data.data()));
    EXPECT(lbmhost::reynoldsNumber(*p, av[49]) > 0.f);
    EXPECT(lbmhost::writeAverageVelocities(tmp + "/av_vels.dat", av));
    EXPECT(lbmhost::writeResults(tmp + "/final_state.dat", *p, *o, cells));
    std::vector<float> c3 = lbmhost::initialiseCells(*p);
    EXPECT(oracle_pipe_run(&op, c3.data(), o->data.data(), 20, av.data()) == 0);

    // a ghosted 5x4 sub-block step
    {
        const int w = 5, h = 4;
        std::vector<float> g((size_t)(w + 2) * (h + 2) * 9, 0.01f), out((size_t)w * h * 9);
        std::vector<uint8_t> ob((size_t)w * h, 0);
        ob[3] = 1;
        (void)oracle_step_ghosted(&op, w, h, g.data(), out.data(), ob.data(), 2);
    }
    // D3Q19 restatement, small channel
    {
        const oracle3d_params q{12, 7, 5, 6, 0.1f, 0.002f, 1.7f};
        std::vector<float> c((size_t)12 * 7 * 5 * 19);
        std::vector<uint8_t> ob((size_t)12 * 7 * 5, 0);
        for (int z = 0; z < 5; ++z)
            for (int x = 0; x < 12; ++x) ob[((size_t)z * 7 + 0) * 12 + x] = ob[((size_t)z * 7 + 6) * 12 + x] = 1;
        std::vector<float> a3(6);
        oracle3d_init_equilibrium(&q, c.data());
        EXPECT(oracle3d_run(&q, c.data(), ob.data(), 6, a3.data()) == 0);
    }
    if (fails) return 1;
    std::printf("host_check: ok\n");
    return 0;
}

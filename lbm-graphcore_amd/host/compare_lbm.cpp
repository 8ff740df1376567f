// compare_lbm -- the reference's compareLbm target (main/LastChance.cpp,
// main/CMakeLists.txt:38-40) with the same positional interface and output
// lines (LastChance.cpp:136-144, :279-284, :554-635), computed by the HIP
// engine through the C ABI:
//
//   compare_lbm <paramfile> <obstaclefile>
//
// Writes final_state.dat and av_vels.dat in the working directory with
// LastChance's printf formats, prints ==done==, the Reynolds number of the
// final state (calc_reynolds, LastChance.cpp:529-534) and elapsed times.
#include <sys/resource.h>
#include <sys/time.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "lbm_host.hpp"

int main(int argc, char *argv[]) {
    if (argc != 3) {
        fprintf(stderr, "Usage: %s <paramfile> <obstaclefile>\n", argv[0]);
        return EXIT_FAILURE;
    }
    auto params = lbmhost::Params::fromFile(argv[1]);
    if (!params) {
        fprintf(stderr, "could not read param file: %s\n", argv[1]);
        return EXIT_FAILURE;
    }
    auto obstacles = lbmhost::Obstacles::fromFile(params->nx, params->ny, argv[2]);
    if (!obstacles) {
        fprintf(stderr, "could not read obstacle file: %s\n", argv[2]);
        return EXIT_FAILURE;
    }
    auto cells = lbmhost::initialiseCells(*params);
    std::vector<float> av_vels(params->maxIters, 0.f);
    const lbm_params abi = params->abi();
    lbm_handle *h = nullptr;
    lbmhost::check(lbm_create(&abi, obstacles->data.data(), 1, &h), nullptr, "lbm_create");
    lbmhost::check(lbm_load_cells(h, cells.data()), h, "lbm_load_cells");

    timeval t;
    gettimeofday(&t, nullptr);
    const double tic = t.tv_sec + t.tv_usec / 1e6;
    lbmhost::check(lbm_run(h), h, "lbm_run");
    gettimeofday(&t, nullptr);
    const double toc = t.tv_sec + t.tv_usec / 1e6;
    rusage ru;
    getrusage(RUSAGE_SELF, &ru);
    const double usr = ru.ru_utime.tv_sec + ru.ru_utime.tv_usec / 1e6;
    const double sys = ru.ru_stime.tv_sec + ru.ru_stime.tv_usec / 1e6;

    lbmhost::check(lbm_store(h, cells.data(), av_vels.data(), (int32_t)av_vels.size()), h, "lbm_store");
    const float re = lbmhost::reynoldsNumber(*params, lbmhost::averageVelocity(*params, *obstacles, cells));
    printf("==done==\n");
    printf("Reynolds number:\t\t%.12E\n", re);
    printf("Elapsed time:\t\t\t%.6lf (s)\n", toc - tic);
    printf("Elapsed user CPU time:\t\t%.6lf (s)\n", usr);
    printf("Elapsed system CPU time:\t%.6lf (s)\n", sys);

    FILE *fp = fopen("final_state.dat", "w");
    if (!fp) {
        fprintf(stderr, "could not open file output file\n");
        return EXIT_FAILURE;
    }
    for (size_t jj = 0; jj < params->ny; ++jj)
        for (size_t ii = 0; ii < params->nx; ++ii) {
            const auto m = lbmhost::macroscopic(*params, *obstacles, cells, ii, jj);
            fprintf(fp, "%zu %zu %.12E %.12E %.12E %.12E %d\n", ii, jj, m.ux, m.uy, m.u, m.pressure,
                    (int)obstacles->at(ii, jj));
        }
    fclose(fp);
    fp = fopen("av_vels.dat", "w");
    if (!fp) {
        fprintf(stderr, "could not open file output file\n");
        return EXIT_FAILURE;
    }
    for (size_t i = 0; i < av_vels.size(); ++i) fprintf(fp, "%zu:\t%.12E\n", i, av_vels[i]);
    fclose(fp);
    lbm_destroy(h);
    return EXIT_SUCCESS;
}

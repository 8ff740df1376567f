// lbm_runner -- the reference's LbmRunner CLI (main/LbmRunner.cpp:11-147) on
// top of the HIP engine's C ABI instead of a Poplar Engine.
//
//   lbm_runner --params P --obstacles O [-n N] [--device gpu|loopback|cpu] [-d] [--exe ignored]
//              [--runs 5] [--kernel auto|resident|stream|step2|vec4|scalar|pipeline] [--spl S] [--out-dir DIR]
//              [--tolerance] [--json FILE]
//
// Flow (same program numbering as the reference):
//   load params/obstacles -> initialise cells on host -> create engine
//   run(0) ≙ lbm_load_cells -> run(1) ≙ lbm_run (accelerate + maxIters steps)
//   run(2) ≙ lbm_store -> write av_vels.dat / final_state.dat
//   print ==done==, compute time, Reynolds number (av_vels[maxIters-1])
//   then `runs` more lbm_run calls timed by device events (≙ readTimer),
//   reported as MLUPS, GB/s and % of the HBM roofline (and, with --json, as
//   one JSON record); -d creates the engine with LBM_FLAG_PROFILE and ends
//   with a per-launch-class device-time summary (≙ engine.printProfileSummary,
//   LbmRunner.cpp:115-122).
// --device loopback places all N sub-domains on GPU 0 (the emulator analogue
// of --device ipumodel: exercises the multi-GPU halo path on one device).
// --device cpu runs the same fused step on the host's cores (lbm_cpu.hpp:
// OpenMP rows, bitwise equal to the GPU engine's default numerics); the
// GPU-only options (-n, --tolerance, --kernel, --spl, --graph-steps) do not
// apply there and are refused with a message.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iomanip>
#include <iostream>
#include <memory>
#include <string>
#include <vector>

#include "lbm_cpu.hpp"
#include "lbm_host.hpp"

namespace {

void usage(const char *exe) {
    std::cerr << exe << " - Runs the Lattice Boltzmann D2Q9-BGK engine on MI355X GPUs\n"
              << "Usage:\n  " << exe << " [OPTION...]\n\n"
              << "  -d, --debug          Print per-phase detail\n"
              << "      --device arg     gpu, loopback or cpu (default: gpu)\n"
              << "  -n, --num-gpus arg   number of GPUs / sub-domains to use (default: 1)\n"
              << "      --exe arg        accepted for compatibility with the reference (ignored)\n"
              << "      --params arg     filename of parameters file\n"
              << "      --obstacles arg  filename of obstacles file\n"
              << "      --runs arg       timed re-runs after the first (default: 5)\n"
              << "      --kernel arg     auto, resident, stream, step2, vec4, scalar or pipeline (default: auto; vec4/scalar = one\n"
              << "                       step per launch; pipeline = unfused per-stage kernels)\n"
              << "      --spl arg        stream kernel: time steps per launch, 2..6, 2..10 with --tolerance (default:\n"
              << "                       library choice, 6; 10 with --tolerance)\n"
              << "      --tolerance      fp32 tolerance-mode collision (LBM_FLAG_TOLERANCE: one reciprocal of rho per\n"
              << "                       cell; not bit-identical to the reference, within the tolerance lbm_hip.h states)\n"
              << "      --out-dir arg    directory for av_vels.dat / final_state.dat (default: .)\n"
              << "      --graph-steps arg  replay the step loop as hipGraphs of 2*arg launches (0 = library default, <0 = off)\n"
              << "      --dump-partitioning arg  write the sub-domain decomposition as JSON\n"
              << "      --json arg       append one JSON results record (MLUPS, GB/s, roofline, profile) to this file\n";
}

constexpr double HBM_PEAK_GBS = 8000.0;  // MI355X HBM3E (MI355X_MICROARCH.md)
constexpr double BYTES_PER_UPDATE = 72.0;  // 9 fp32 loads + 9 fp32 stores per cell

std::string json_str(const std::string &v) {
    std::string o = "\"";
    for (char c : v) {
        if (c == '"' || c == '\\') o += '\\';
        if ((unsigned char)c < 0x20) continue;
        o += c;
    }
    return o + "\"";
}

// --device cpu: the reference's program sequence on the host backend
int run_cpu(const lbmhost::Params &params, const lbmhost::Obstacles &obstacles, const std::string &outDir, int runs) {
    std::cout << "Running on the host CPU (" << lbmcpu::Engine::threads()
              << " threads; bitwise numerics: the reference's LastChance.cpp arithmetic)" << std::endl;
    auto cells = lbmhost::initialiseCells(params);
    std::vector<float> av_vels;
    std::unique_ptr<lbmcpu::Engine> e;
    lbmhost::timedStep("Creating engine and loading obstacles", [&]() {
        e = std::make_unique<lbmcpu::Engine>((int)params.nx, (int)params.ny, params.density, params.accel,
                                             params.omega, obstacles.data);
    });
    lbmhost::timedStep("Running copy to device step", [&]() { e->load(cells); });
    double total_compute_time =
        lbmhost::timedStep("Running LBM", [&]() { e->run((int)params.maxIters, av_vels); });
    lbmhost::timedStep("Running copy to host step", [&]() { e->store(cells); });
    lbmhost::timedStep("Writing output files ", [&]() {
        lbmhost::writeAverageVelocities(outDir + "/av_vels.dat", av_vels);
        lbmhost::writeResults(outDir + "/final_state.dat", params, obstacles, cells);
    });
    std::cout << "==done==" << std::endl;
    std::cout << "Total compute time was \t" << std::right << std::setw(12) << std::setprecision(5)
              << total_compute_time << "s" << std::endl;
    const float lastAv = params.maxIters > 0 ? av_vels[params.maxIters - 1] : 0.f;
    std::cout << "Reynolds number:  \t" << std::right << std::setw(12) << std::setprecision(12) << std::scientific
              << lbmhost::reynoldsNumber(params, lastAv) << std::endl;
    if (runs > 0) {
        std::cout << "Now doing " << runs << " runs and averaging CPU timing:" << std::endl;
        double secs = 0.0;
        for (int r = 0; r < runs; ++r) {
            e->load(cells);
            secs += e->run((int)params.maxIters, av_vels);
        }
        const double avg = secs / runs;
        std::cout << "Average CPU timing for program is: " << std::fixed << std::setprecision(5) << std::setw(12)
                  << avg << "s" << std::endl;
        std::cout << "MLUPS: " << std::fixed << std::setprecision(1)
                  << (double)params.nx * params.ny * params.maxIters / avg / 1e6 << std::endl;
    }
    return EXIT_SUCCESS;
}

}  // namespace

int main(int argc, char *argv[]) {
    std::string paramsFile, obstaclesFile, device = "gpu", exeFile, kernel = "auto", outDir = ".", dumpFile, jsonFile;
    std::vector<std::string> gpuOnly;  // GPU-only options given on the command line
    int spl = 0;
    int numGpus = 1, runs = 5, graphSteps = 0;
    bool debug = false, tolerance = false;
    for (int i = 1; i < argc; ++i) {
        std::string a = argv[i];
        std::string val;
        const auto eq = a.find('=');
        if (a.rfind("--", 0) == 0 && eq != std::string::npos) {
            val = a.substr(eq + 1);
            a = a.substr(0, eq);
        }
        auto next = [&](std::string &dst) -> bool {
            if (!val.empty()) { dst = val; return true; }
            if (i + 1 >= argc) return false;
            dst = argv[++i];
            return true;
        };
        std::string v;
        if (a == "-d" || a == "--debug") {
            debug = true;
        } else if (a == "--device") {
            if (!next(device)) { usage(argv[0]); return EXIT_FAILURE; }
        } else if (a == "-n" || a == "--num-gpus" || a == "--num-ipus") {
            if (!next(v)) { usage(argv[0]); return EXIT_FAILURE; }
            numGpus = std::atoi(v.c_str());
            if (numGpus != 1) gpuOnly.push_back(a);
        } else if (a == "--exe") {
            if (!next(exeFile)) { usage(argv[0]); return EXIT_FAILURE; }
        } else if (a == "--params") {
            if (!next(paramsFile)) { usage(argv[0]); return EXIT_FAILURE; }
        } else if (a == "--obstacles") {
            if (!next(obstaclesFile)) { usage(argv[0]); return EXIT_FAILURE; }
        } else if (a == "--runs") {
            if (!next(v)) { usage(argv[0]); return EXIT_FAILURE; }
            runs = std::atoi(v.c_str());
        } else if (a == "--kernel") {
            if (!next(kernel)) { usage(argv[0]); return EXIT_FAILURE; }
            if (kernel != "auto" && kernel != "resident" && kernel != "pipeline" && kernel != "stream" && kernel != "step2" && kernel != "vec4" && kernel != "scalar") {
                usage(argv[0]);
                return EXIT_FAILURE;
            }
            gpuOnly.push_back(a);
        } else if (a == "--spl") {
            std::string v;
            if (!next(v)) { usage(argv[0]); return EXIT_FAILURE; }
            spl = std::atoi(v.c_str());
            gpuOnly.push_back(a);
        } else if (a == "--tolerance") {
            tolerance = true;
            gpuOnly.push_back(a);
        } else if (a == "--out-dir") {
            if (!next(outDir)) { usage(argv[0]); return EXIT_FAILURE; }
        } else if (a == "--graph-steps") {
            if (!next(v)) { usage(argv[0]); return EXIT_FAILURE; }
            graphSteps = std::atoi(v.c_str());
            gpuOnly.push_back(a);
        } else if (a == "--dump-partitioning") {
            if (!next(dumpFile)) { usage(argv[0]); return EXIT_FAILURE; }
        } else if (a == "--json") {
            if (!next(jsonFile)) { usage(argv[0]); return EXIT_FAILURE; }
        } else if (a == "-h" || a == "--help") {
            usage(argv[0]);
            return EXIT_SUCCESS;
        } else {
            usage(argv[0]);
            return EXIT_FAILURE;
        }
    }
    if (paramsFile.empty() || obstaclesFile.empty() || numGpus < 1 ||
        (device != "gpu" && device != "loopback" && device != "cpu")) {
        usage(argv[0]);
        return EXIT_FAILURE;
    }
    if (debug) std::cout << "Capturing profile information during this run." << std::endl;

    auto params = lbmhost::Params::fromFile(paramsFile);
    if (!params.has_value()) {
        std::cerr << "Could not parse parameters file. Aborting" << std::endl;
        return EXIT_FAILURE;
    }
    auto obstacles = lbmhost::Obstacles::fromFile(params->nx, params->ny, obstaclesFile);
    if (!obstacles.has_value()) {
        std::cerr << "Could not parse obstacles file" << std::endl;
        return EXIT_FAILURE;
    }
    if (!dumpFile.empty()) {
        // partitioning.json in the layout of grids::serializeToJson
        // (StructuredGridUtils.hpp:135-158), one entry per GPU sub-domain;
        // tile/worker are always 0 here.  Unlike the reference writer the
        // "slice" object is closed, so the file is valid JSON.
        std::vector<lbm_rect> rects(numGpus);
        int32_t R = 0, C = 0;
        if (lbm_partition((int32_t)params->nx, (int32_t)params->ny, numGpus, 0, 0, &R, &C, rects.data()) != LBM_OK) {
            std::cerr << "Cannot partition the grid into " << numGpus << " parts" << std::endl;
            return EXIT_FAILURE;
        }
        std::ofstream f(dumpFile);
        f << R"({"GridPartitioning" : [)" << "\n";
        for (int i = 0; i < numGpus; ++i) {
            if (i) f << ",\n";
            f << "  {\n";
            f << "    \"ipu\":" << i << ",\n";
            f << "    \"tile\":" << 0 << ",\n";
            f << "    \"worker\":" << 0 << ",\n";
            f << "    \"slice\": {\n";
            f << "       \"rows\" : { \"from\" : " << rects[i].y0 << ",\"to\" : " << rects[i].y0 + rects[i].h << "},\n";
            f << "       \"cols\" : { \"from\" : " << rects[i].x0 << ",\"to\" : " << rects[i].x0 + rects[i].w << "}\n";
            f << "    }\n  }";
        }
        f << "\n]}\n";
        std::cout << "Wrote " << R << "x" << C << " decomposition to " << dumpFile << std::endl;
    }
    if (device == "cpu") {
        if (!gpuOnly.empty()) {
            // the host backend has one numerics (bitwise) and one kernel: a
            // '--device cpu --tolerance' run must not silently write bitwise results
            std::cerr << "--device cpu does not take the GPU-only option(s):";
            for (auto &o : gpuOnly) std::cerr << " " << o;
            std::cerr << " (the host backend runs the reference arithmetic on one domain)" << std::endl;
            return EXIT_FAILURE;
        }
        return run_cpu(*params, *obstacles, outDir, runs);
    }
    const int ndev = lbm_device_count();
    if (ndev <= 0) {
        std::cerr << "No HIP device visible" << std::endl;
        return EXIT_FAILURE;
    }
    if (device == "gpu")
        std::cout << "Running on " << numGpus << " GPU(s)" << std::endl;
    else
        std::cout << "Running " << numGpus << " sub-domain(s) in loop-back on GPU 0" << std::endl;

    double total_compute_time = 0.0;
    auto cells = lbmhost::initialiseCells(*params);
    std::vector<float> av_vels(params->maxIters, 0.0f);

    lbm_handle *h = nullptr;
    const lbm_params abi = params->abi();
    std::vector<int32_t> devs;
    if (device == "loopback") devs.push_back(0);
    lbmhost::timedStep("Creating engine and loading obstacles", [&]() {
        lbm_config cfg{};
        cfg.parts = numGpus;
        cfg.transport = LBM_TRANSPORT_LOCAL;
        cfg.devices = devs.empty() ? nullptr : devs.data();
        cfg.num_devices = (int32_t)devs.size();
        cfg.kernel = kernel == "scalar" ? LBM_KERNEL_SCALAR
                   : kernel == "vec4"   ? LBM_KERNEL_VEC4
                   : kernel == "step2"  ? LBM_KERNEL_STEP2
                   : kernel == "stream" ? LBM_KERNEL_STREAM
                   : kernel == "resident" ? LBM_KERNEL_RESIDENT
                   : kernel == "pipeline" ? LBM_KERNEL_PIPELINE
                                        : LBM_KERNEL_AUTO;
        if (kernel == "scalar" || kernel == "vec4") cfg.flags |= LBM_FLAG_ONE_STEP;
        if (tolerance) cfg.flags |= LBM_FLAG_TOLERANCE;
        if (debug) cfg.flags |= LBM_FLAG_PROFILE;
        cfg.steps_per_launch = spl;
        cfg.graph_steps = graphSteps;
        lbmhost::check(lbm_create_ex(&abi, obstacles->data.data(), &cfg, &h), nullptr, "lbm_create_ex");
    });
    if (debug) {
        std::vector<lbm_rect> rects(numGpus);
        int32_t n = 0;
        lbm_local_rects(h, rects.data(), numGpus, &n);
        for (int i = 0; i < n; ++i)
            std::cout << "sub-domain " << i << ": " << rects[i].w << "x" << rects[i].h << " at (row:" << rects[i].y0
                      << ",col:" << rects[i].x0 << ")" << std::endl;
        const int32_t k = lbm_kernel_in_use(h);
        std::cout << "step kernel: "
                  << (k == LBM_KERNEL_RESIDENT ? "resident" : k == LBM_KERNEL_PIPELINE ? "pipeline" : k == LBM_KERNEL_STREAM ? "stream" : k == LBM_KERNEL_STEP2 ? "step2" : k == LBM_KERNEL_VEC4 ? "vec4" : "scalar")
                  << " (" << lbm_steps_per_launch(h) << " steps per launch)" << std::endl;
    }
    lbmhost::timedStep("Running copy to device step", [&]() {
        lbmhost::check(lbm_load_cells(h, cells.data()), h, "lbm_load_cells");
    });
    total_compute_time += lbmhost::timedStep("Running LBM", [&]() { lbmhost::check(lbm_run(h), h, "lbm_run"); });
    lbmhost::timedStep("Running copy to host step", [&]() {
        lbmhost::check(lbm_store(h, cells.data(), av_vels.data(), (int32_t)av_vels.size()), h, "lbm_store");
    });
    lbmhost::timedStep("Writing output files ", [&]() {
        lbmhost::writeAverageVelocities(outDir + "/av_vels.dat", av_vels);
        lbmhost::writeResults(outDir + "/final_state.dat", *params, *obstacles, cells);
    });

    std::cout << "==done==" << std::endl;
    std::cout << "Total compute time was \t" << std::right << std::setw(12) << std::setprecision(5)
              << total_compute_time << "s" << std::endl;
    const float lastAv = params->maxIters > 0 ? av_vels[params->maxIters - 1] : 0.f;
    std::cout << "Reynolds number:  \t" << std::right << std::setw(12) << std::setprecision(12) << std::scientific
              << lbmhost::reynoldsNumber(*params, lastAv) << std::endl;

    const int32_t kin = lbm_kernel_in_use(h);
    const char *kname = kin == LBM_KERNEL_RESIDENT ? "resident" : kin == LBM_KERNEL_PIPELINE ? "pipeline"
                      : kin == LBM_KERNEL_STREAM ? "stream" : kin == LBM_KERNEL_STEP2 ? "step2"
                      : kin == LBM_KERNEL_VEC4 ? "vec4" : "scalar";
    const double cells_total = (double)params->nx * params->ny;
    double avg = 0.0, mlups = 0.0, eff_gbs = 0.0, pass_gbs = 0.0;
    int32_t fused_l = 0, single_l = 0;
    if (runs > 0) {
        std::cout << "Now doing " << runs << " runs and averaging GPU-reported timing:" << std::endl;
        double secs = 0.0;
        for (int r = 0; r < runs; ++r) {
            lbmhost::check(lbm_run(h), h, "lbm_run");
            double s = 0.0;
            lbm_last_run_seconds(h, &s);
            secs += s;
        }
        avg = secs / runs;
        mlups = cells_total * params->maxIters / avg / 1e6;
        lbm_run_stats(h, &fused_l, &single_l);
        // 72 B per cell update; a launch that advances S steps
        // moves the lattice through HBM once, so the roofline is per pass
        eff_gbs = BYTES_PER_UPDATE * cells_total * params->maxIters / avg / 1e9;
        std::cout << "Average GPU timing for program is: " << std::fixed << std::setprecision(5) << std::setw(12)
                  << avg << "s" << std::endl;
        std::cout << "MLUPS: " << std::fixed << std::setprecision(1) << mlups << std::endl;
        std::cout << "GB/s (72 B per cell update): " << std::fixed << std::setprecision(1) << eff_gbs << std::endl;
        if (kin == LBM_KERNEL_RESIDENT) {
            std::cout << "HBM roofline: n/a (the resident kernel holds the lattice on chip for the whole run; "
                         "bound by the per-step hand-off between tiles)" << std::endl;
        } else {
            const int passes = fused_l + single_l;
            pass_gbs = BYTES_PER_UPDATE * cells_total * passes / avg / 1e9;
            std::cout << "HBM passes per run: " << passes << " (" << fused_l << " fused launches of up to "
                      << lbm_steps_per_launch(h) << " steps, " << single_l << " one-step)" << std::endl;
            std::cout << "HBM GB/s per lattice pass: " << std::fixed << std::setprecision(1) << pass_gbs << " = "
                      << std::setprecision(1) << 100.0 * pass_gbs / HBM_PEAK_GBS << " % of the "
                      << (int)HBM_PEAK_GBS << " GB/s HBM roofline" << std::endl;
        }
    }
    std::vector<lbm_kernel_time> prof;
    if (debug) {
        int32_t n = 0;
        if (lbm_profile_summary(h, nullptr, 0, &n) == LBM_OK && n > 0) {
            prof.resize(n);
            lbm_profile_summary(h, prof.data(), n, &n);
            std::cout << "Profile summary (device time per launch class over the " << (runs + 1)
                      << " runs; events around every launch):" << std::endl;
            std::cout << "  " << std::left << std::setw(52) << "launch class" << std::right << std::setw(10)
                      << "launches" << std::setw(14) << "total ms" << std::setw(12) << "mean ms" << std::setw(12)
                      << "min ms" << std::setw(12) << "max ms" << std::endl;
            for (const auto &k : prof)
                std::cout << "  " << std::left << std::setw(52) << k.name << std::right << std::setw(10) << k.launches
                          << std::fixed << std::setprecision(3) << std::setw(14) << k.total_ms << std::setw(12)
                          << (k.launches ? k.total_ms / k.launches : 0.0) << std::setw(12) << k.min_ms << std::setw(12)
                          << k.max_ms << std::endl;
        }
    }
    if (!jsonFile.empty()) {
        std::ofstream f(jsonFile, std::ios::app);
        f << "{\"tool\": \"lbm_runner\", \"params\": " << json_str(paramsFile) << ", \"grid\": \"" << params->nx << "x"
          << params->ny << "\", \"steps\": " << params->maxIters << ", \"device\": " << json_str(device)
          << ", \"sub_domains\": " << numGpus << ", \"kernel\": \"" << kname
          << "\", \"steps_per_launch\": " << lbm_steps_per_launch(h)
          << ", \"numerics\": \"" << (lbm_numerics(h) ? "tolerance" : "bitwise") << "\", \"runs\": " << runs
          << std::setprecision(9) << ", \"avg_seconds\": " << avg << std::setprecision(6) << ", \"mlups\": " << mlups
          << ", \"gbs_per_update\": " << eff_gbs << ", \"hbm_passes_per_run\": " << fused_l + single_l
          << ", \"gbs_per_pass\": " << pass_gbs << ", \"hbm_roofline_frac\": "
          << (kin == LBM_KERNEL_RESIDENT || runs <= 0 ? std::string("null") : std::to_string(pass_gbs / HBM_PEAK_GBS))
          << ", \"hbm_peak_gbs\": " << HBM_PEAK_GBS
          << ", \"reynolds\": " << std::scientific << std::setprecision(9) << lbmhost::reynoldsNumber(*params, lastAv)
          << std::defaultfloat << ", \"profile\": [";
        for (size_t i = 0; i < prof.size(); ++i)
            f << (i ? ", " : "") << "{\"name\": " << json_str(prof[i].name) << ", \"launches\": " << prof[i].launches
              << std::setprecision(6) << ", \"total_ms\": " << prof[i].total_ms << ", \"min_ms\": " << prof[i].min_ms
              << ", \"max_ms\": " << prof[i].max_ms << "}";
        f << "]}\n";
        std::cout << "Results record appended to " << jsonFile << std::endl;
    }
    lbm_destroy(h);
    return EXIT_SUCCESS;
}

// galac — the GALA compiler driver for MI355X.
//
//   galac <program.txt> <output dir> [--no-fuse] [--ir] [--quiet]
//
// Mirrors tests/gala_train.cpp (the reference's driver): parse the DSL program, print the
// model configuration, build the IR, run the middle-end passes in the reference's order
// and write the generated program.  The reference then builds gala.cu with CMake; galac
// writes <dir>/gala.cpp plus a Makefile that links the prebuilt libgala_torch.so /
// libgala_hip.so (`make -C <dir>` -> <dir>/gala_prog).
#include <chrono>
#include <fstream>
#include <iostream>
#include <sys/stat.h>
#include <unistd.h>

#include "ir.h"

namespace {

std::string self_pkg_dir(const char *argv0) {
    // galac lives in <pkg>/gala/; the Makefile points back at <pkg>
    char buf[4096];
    const ssize_t n = readlink("/proc/self/exe", buf, sizeof(buf) - 1);
    std::string p = n > 0 ? std::string(buf, (size_t)n) : std::string(argv0);
    for (int up = 0; up < 2; ++up) {
        const size_t k = p.find_last_of('/');
        p = k == std::string::npos ? "." : p.substr(0, k);
    }
    return p;
}

}  // namespace

int main(int argc, char **argv) {
    std::string in, out;
    bool fuse = true, show_ir = false, quiet = false;
    std::string json_path;
    for (int i = 1; i < argc; ++i) {
        const std::string a = argv[i];
        if (a == "--no-fuse") fuse = false;
        else if (a == "--ir") show_ir = true;
        else if (a == "--quiet") quiet = true;
        else if (a == "--ir-json" && i + 1 < argc) json_path = argv[++i];
        else if (in.empty()) in = a;
        else if (out.empty()) out = a;
        else {
            std::cerr << "galac: unexpected argument " << a << "\n";
            return 2;
        }
    }
    if (in.empty()) {
        std::cerr << "usage: galac <program.txt> [<output dir>] [--no-fuse] [--ir] [--ir-json FILE] [--quiet]\n";
        return 2;
    }
    const auto t0 = std::chrono::steady_clock::now();
    try {
        galac::Program prog = galac::parse_file(in);
        galac::Module m = galac::lower(prog);
        const galac::Schedule &s = m.sched;
        if (!quiet) {
            std::cout << " ---------------- printing model config ----------------------\n"
                      << "Dataset: " << s.dataset << "\nLayers: " << m.num_layers
                      << "\nIterations: " << s.iterations << "\nValidation step: "
                      << s.validation_step << "\nFeature size: " << s.feat_size
                      << "\nLabel size: " << s.label_size << "\nUndirected: " << s.undirected
                      << "\nUnweighted: " << s.unweighted << "\nSparse: " << s.sparse
                      << "\nCol tile: " << s.col_tile << "\nGraph sample: " << s.data_sample
                      << "\nKernel sample: " << s.kernel_sample
                      << (s.dynamic_sample ? " (dynamic)" : "") << "\nCoarsen: " << s.coarsen
                      << "\n---------------------------------------------------------------\n";
        }
        if (show_ir) std::cout << "IR (lowered):\n" << m.dump();
        const std::string pre_json = m.to_json();
        galac::run_passes(m, fuse);
        if (!json_path.empty())
            std::ofstream(json_path) << "{\"pre\": " << pre_json << ", \"post\": " << m.to_json() << "}\n";
        if (!quiet)
            for (const std::string &n : m.notes) std::cout << "pass: " << n << "\n";
        if (show_ir) std::cout << "IR (after passes):\n" << m.dump();
        if (!out.empty()) {
            ::mkdir(out.c_str(), 0755);
            std::ofstream(out + "/gala.cpp") << galac::emit_program(m);
            std::ofstream(out + "/Makefile") << galac::emit_makefile(m, self_pkg_dir(argv[0]));
        }
    } catch (const galac::DslError &e) {
        std::cerr << in << ":" << e.what() << "\n";
        return 1;
    } catch (const std::exception &e) {
        std::cerr << "galac: " << e.what() << "\n";
        return 1;
    }
    const double ms =
        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (!quiet) std::cout << "Time taken for GALA compilation: " << ms << std::endl;
    return 0;
}

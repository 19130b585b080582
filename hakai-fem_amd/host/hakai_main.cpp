// hakai -- command-line driver, the MI355X counterpart of `julia HAKAI_j.jl file.inp`
// (main() -> hakai(ARGS[1]), v2/HAKAI_j.jl:3729-3735). Writes <out_dir>/file%03d.vtk
// (the reference writes the Windows literal temp\\file%03d.vtk, v2/HAKAI_j.jl:3564).
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "../../include/hakai_hip.h"

int main(int argc, char** argv) {
    if (argc < 2) {
        std::fprintf(stderr, "usage: %s file.inp [out_dir=temp] [--device N] [--quiet]\n", argv[0]);
        return 2;
    }
    const char* out = "temp";
    int device = 0, verbose = 1;
    for (int i = 2; i < argc; ++i) {
        if (!std::strcmp(argv[i], "--device") && i + 1 < argc) device = std::atoi(argv[++i]);
        else if (!std::strcmp(argv[i], "--quiet")) verbose = 0;
        else out = argv[i];
    }
    const int r = hakai_run_inp(argv[1], out, device, verbose);
    if (r) {
        std::fprintf(stderr, "hakai: error %d: %s\n", r, hakai_last_error());
        return 1;
    }
    return 0;
}

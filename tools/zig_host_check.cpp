// Host-side check of the ziggurat attempt parser (gs_ziggurat.hpp) against
// NumPy: prints n normals for the PCG64 state given on the command line.
// Build: hipcc -O2 -ffp-contract=off tools/zig_host_check.cpp -o /tmp/zig_check
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include "../gnn-sparsification-research_amd/csrc/gs_ziggurat.hpp"
int main(int argc, char **argv) {
    using namespace gs;
    u128 s = ((u128)strtoull(argv[1], 0, 16) << 64) | strtoull(argv[2], 0, 16);
    u128 inc = ((u128)strtoull(argv[3], 0, 16) << 64) | strtoull(argv[4], 0, 16);
    long n = atol(argv[5]);
    Pcg64 g{s, inc};
    double *out = (double *)malloc(sizeof(double) * n);
    long i = 0;
    while (i < n) {
        bool p; double v;
        zig_attempt<false>(g, &p, &v);
        if (p) out[i++] = v;
    }
    fwrite(out, sizeof(double), n, stdout);
    return 0;
}

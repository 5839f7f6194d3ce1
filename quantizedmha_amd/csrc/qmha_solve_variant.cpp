// qmha_solve_variant.cpp -- per-variant `solve` shim.  Compiled once per kernel variant
// with -DQMHA_SOLVE_VARIANT=<id> -DQMHA_SOLVE_NAME=<name> into libqmha_<name>.so, which
// links libqmha.so.  Mirrors the reference's one-`solve`-per-binary build (Makefile:39-53):
// a caller that dlopen()s libqmha_fa_tc_v1a.so and binds `solve` gets the FP16 path.
#include <cstdio>

#include "../../include/launchers.h"

#ifndef QMHA_SOLVE_VARIANT
#error "QMHA_SOLVE_VARIANT must be defined"
#endif
#define QMHA_STR2(x) #x
#define QMHA_STR(x) QMHA_STR2(x)

extern "C" __attribute__((visibility("default"))) void solve(const float* Q, const float* K, const float* V,
                                                            float* output, int N, int d_model, int h) {
    int st = qmha_solve_variant(Q, K, V, output, N, d_model, h, QMHA_SOLVE_VARIANT);
    if (st != QMHA_OK)
        std::fprintf(stderr, "qmha solve(" QMHA_STR(QMHA_SOLVE_NAME) "): %s: %s\n", qmha_status_string(st),
                     qmha_last_error());
}

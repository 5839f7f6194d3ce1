// occupancy.cpp -- what the HIP runtime says about a kernel's occupancy on this GPU:
// usage: occupancy <code-object.co> <block-size> <kernel-name-substring>...
// (extract the .co from a built object with tools/isa.py-style unbundling, see tools/occ.sh)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>
#include <fstream>

int main(int argc, char** argv) {
    if (argc < 4) { std::fprintf(stderr, "usage: occupancy <co> <block> <name>...\n"); return 2; }
    hipModule_t m;
    if (hipModuleLoad(&m, argv[1]) != hipSuccess) { std::fprintf(stderr, "load failed\n"); return 1; }
    const int block = std::atoi(argv[2]);
    for (int i = 3; i < argc; ++i) {
        hipFunction_t f;
        if (hipModuleGetFunction(&f, m, argv[i]) != hipSuccess) { std::printf("%s: not found\n", argv[i]); continue; }
        int nb = 0;
        (void)hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&nb, f, block, 0);
        int regs = 0, lds = 0;
        (void)hipFuncGetAttribute(&regs, HIP_FUNC_ATTRIBUTE_NUM_REGS, f);
        (void)hipFuncGetAttribute(&lds, HIP_FUNC_ATTRIBUTE_SHARED_SIZE_BYTES, f);
        std::printf("%-60.60s block %d -> %d blocks/CU (%d waves/SIMD), regs %d, lds %d\n", argv[i], block, nb,
                    nb * block / 64 / 4, regs, lds);
    }
    return 0;
}

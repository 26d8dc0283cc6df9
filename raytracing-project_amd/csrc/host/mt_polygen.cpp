// mt_polygen.cpp — build tool: writes the mt19937 checkpoint-tree jump
// polynomials (mt_poly.hpp mt_tree_polys, K twist blocks per segment =
// mt_jump.hpp kTableK) to a file that librtamd.so reads at run time instead
// of recomputing them.  Usage: mt_polygen <out-file> [levels] [K]
#include <cstdio>
#include <cstdlib>

#include "mt_poly.hpp"

int main(int argc, char** argv) {
    if (argc < 2) {
        std::fprintf(stderr, "usage: %s <out-file> [levels]\n", argv[0]);
        return 2;
    }
    const int levels = argc > 2 ? std::atoi(argv[2]) : 4;
    const int K = argc > 3 ? std::atoi(argv[3]) : 16;
    if (levels < 1 || levels > 8 || K < 1) return 2;
    if (!rtamd::mt_save_tree_polys(argv[1], K, levels)) {
        std::fprintf(stderr, "mt_polygen: cannot write %s\n", argv[1]);
        return 1;
    }
    return 0;
}

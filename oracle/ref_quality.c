/*
 * oracle/ref_quality.c -- TEST INFRASTRUCTURE ONLY.
 * Q-sweep oracle: includes the UNMODIFIED reference utils/original.c (the
 * upstream encoder encoder.c was adapted from) and calls its own
 * set_quality() (original.c:504-509, commented out in its main at
 * :1157-1158) before running its main().  Usage: ref_quality <ppm> <Q>;
 * writes out.jpg into the working directory (which needs hisParts/).
 */
#define main orig_main
#include REF_ORIGINAL_C
#undef main
#include <stdlib.h>

int main(int argc, char **argv) {
    if (argc != 3) return 2;
    int q = atoi(argv[2]);
    set_quality(luma_quantizer, q);
    set_quality(chroma_quantizer, q);
    return orig_main(argc, argv);
}

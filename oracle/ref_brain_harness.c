/*
 * oracle/ref_brain_harness.c -- TEST INFRASTRUCTURE ONLY.
 * Thin C wrapper linked with the unmodified reference main/brain.c into
 * oracle/_ref/libref_brain.so.  It reproduces the caller contract of
 * main.c:136-163: subsample(raw) -> compare(sub, saved) -> store(sub, saved),
 * on caller-given frames of runtime size (see ref_brain_shim.h).
 */
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
#include "brain.h"

int ref_stride = 320;
int ref_height = 240;

/* brain.c:16-45; the PPM copy the reference writes goes to /dev/null */
int ref_subsample(const uint8_t *bgr, int w, int h, uint8_t *sub) {
    ref_stride = w;
    ref_height = h;
    FILE *f = fopen("/dev/null", "w");
    if (!f) return -1;
    subsample(f, (uint8_t *)bgr, sub);
    fclose(f);
    return 0;
}

/* brain.c:104-233 with main.c's 100-entry diffDims (main.c:34) and the
 * differences[2][WIDTH/8] scratch (main.c:35) */
int ref_compare(const uint8_t *sub, const uint8_t *saved, int w, int h, area_t outs[100]) {
    ref_stride = w;
    ref_height = h;
    pair_t *diff = malloc(sizeof(pair_t) * 2 * (size_t)(w / 8));
    if (!diff) return -1;
    int n = compare((uint8_t *)sub, (uint8_t *)saved, outs, (pair_t(*)[w / 8])diff);
    free(diff);
    return n;
}

void ref_enlarge_adjust(area_t *a, int w, int h) {
    ref_stride = w;
    ref_height = h;
    enlargeAdjust(a);
}

/*
 * oracle/ref_brain_shim.h -- pre-included (gcc -include) when compiling the
 * UNMODIFIED reference main/brain.c into oracle/_ref/libref_brain.so.  Like
 * ref_shim.h it pulls in the reference's own include/define.h (#pragma once)
 * and turns the compile-time frame size WIDTH x HEIGHT (define.h:3-4) into
 * runtime variables, so frames other than 320x240 can be fed to the
 * reference's change detector.  Nothing else in the reference is replaced.
 */
#pragma once
#include REF_DEFINE_H
#undef WIDTH
#undef HEIGHT
extern int ref_stride;
extern int ref_height;
#define WIDTH ref_stride
#define HEIGHT ref_height

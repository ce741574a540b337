/*
 * oracle/ref_shim.h -- pre-included (gcc -include) when compiling the
 * UNMODIFIED reference main/encoder.c into oracle/_ref/.  It pulls in the
 * reference's own include/define.h first (that header is `#pragma once`, so
 * encoder.h's later include of it is a no-op) and then turns the compile-time
 * input row stride WIDTH (define.h:3, used at encoder.c:132) into a runtime
 * variable, so frames wider than 320 px can be fed to the reference.  Nothing
 * else in the reference is replaced.
 */
#pragma once
#include REF_DEFINE_H
#undef WIDTH
extern int ref_stride;
#define WIDTH ref_stride

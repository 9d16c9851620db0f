/*
 * oracle.c -- TEST INFRASTRUCTURE ONLY.  CPU restatement of the AANet hot path
 * (see oracle_impl.h for the per-function reference citations).  Built into
 * oracle/liboracle.so by oracle/Makefile; loaded only by tests/, smoke() and the
 * cpu_baseline leg of bench.py.
 */
#include <math.h>
#include <stdlib.h>

#define REAL float
#define SUFFIX _f32
#include "oracle_impl.h"
#undef REAL
#undef SUFFIX

#define REAL double
#define SUFFIX _f64
#include "oracle_impl.h"
#undef REAL
#undef SUFFIX

int orc_version(void) { return 1; }

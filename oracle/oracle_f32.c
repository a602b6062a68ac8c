/*
 * oracle_f32.c — the oracle (mpcr_oracle.c) compiled with every double as
 * float, for bench.py's cpu_baseline "the same fp32 algorithm" figure
 * (the reference computes in fp32, JAX x64
 * off).  TEST / BASELINE INFRASTRUCTURE ONLY, never linked into libmpcr.
 *
 * <tgmath.h> makes sqrt / fabs / acos ... resolve to their float versions,
 * -fsingle-precision-constant (oracle/Makefile) keeps literals in float, and
 * the model struct is the same header with float fields
 * (oracle.Runner(precision="fp32") converts the fp64 struct).  The parity
 * checker stays the fp64 build.
 */
#include <tgmath.h>
#undef I /* complex.h (via tgmath.h) takes the name; the oracle uses it for inertias */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef double mpcr_hp; /* the line-search bookkeeping stays fp64 (mpcr_oracle.c lspt) */
#define MPCR_HP_DEFINED
#define double float
#define mpcr_model_t mpcr_model_f32_t
#include "../include/mpcr_model.h"
#include "mpcr_oracle.c"

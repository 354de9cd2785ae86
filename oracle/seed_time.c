/* Link-time wrapper for time(2) used ONLY by the oracle/_ref build of the
 * reference (test infrastructure, never shipped). The reference seeds its
 * RNG with ran_seed(time(0)) (C_implementations/src/decodeMinSum.cpp:187);
 * linking with -Wl,--wrap=time routes that call here so the run is
 * reproducible: REF_SEED (default 134159, the constant commented at :187). */
#include <stdlib.h>
#include <time.h>
time_t __wrap_time(time_t *t)
{
    const char *s = getenv("REF_SEED");
    time_t v = s ? (time_t)atol(s) : (time_t)134159;
    if (t) *t = v;
    return v;
}

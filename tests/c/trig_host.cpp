// Host build of drone_rl_amd/csrc/trig.h for tests/test_trig_host.py.
#include <cstdint>

#include "../../drone_rl_amd/csrc/trig.h"

extern "C" void trig_sincos(int64_t n, const double *x, double *s, double *c) {
    for (int64_t i = 0; i < n; ++i) {
        const dr::SinCos t = dr::sincos_medium(x[i]);
        s[i] = t.s;
        c[i] = t.c;
    }
}

extern "C" void trig_sincosf(int64_t n, const float *x, float *s, float *c) {
    for (int64_t i = 0; i < n; ++i) {
        const dr::SinCosF t = dr::sincosf_medium(x[i]);
        s[i] = t.s;
        c[i] = t.c;
    }
}

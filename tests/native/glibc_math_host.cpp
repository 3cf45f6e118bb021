// Host build of csrc/glibc_math.h for the bit-exactness test against the host libm.
// TEST INFRASTRUCTURE (tests/test_glibc_math.py).  Compiled with -ffp-contract=off.
#include <math.h>
#include <stdint.h>
#include <string.h>
#include "glibc_math.h"

extern "C" {
// mode 0 log, 1 exp, 2 pow.  Returns the number of results differing bit-wise from libm;
// the first mismatching input index is written to *first (or -1).
int64_t gm_check(int mode, const double* x, const double* y, int64_t n, int64_t* first) {
  int64_t bad = 0;
  *first = -1;
  for (int64_t i = 0; i < n; i++) {
    double a, b;
    if (mode == 0) { a = gm_log(x[i]); b = log(x[i]); }
    else if (mode == 1) { a = gm_exp(x[i]); b = exp(x[i]); }
    else { a = gm_pow(x[i], y[i]); b = pow(x[i], y[i]); }
    uint64_t ua, ub;
    memcpy(&ua, &a, 8);
    memcpy(&ub, &b, 8);
    if (ua != ub && !(a != a && b != b)) {
      if (*first < 0) *first = i;
      bad++;
    }
  }
  return bad;
}
void gm_eval(int mode, const double* x, const double* y, double* out, int64_t n) {
  for (int64_t i = 0; i < n; i++)
    out[i] = mode == 0 ? gm_log(x[i]) : mode == 1 ? gm_exp(x[i]) : gm_pow(x[i], y[i]);
}
}

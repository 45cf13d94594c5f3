/*
 * ref_reduction.c -- TEST INFRASTRUCTURE ONLY.
 * Restates the MPI_SUM cases of reduction() in src/mpi/ext_mpi_native_exec.c:207-239:
 * one scalar pass "p1[i] += p2[i]" per SREDUCE line. Compiled like the reference
 * (gcc -O3 -fPIC, no -ffast-math: Makefile:12) so IEEE round-to-nearest and denormals
 * are kept and the per-element order is exactly the schedule's.
 */
#include "ref_oracle.h"

int ref_type_size(int dtype) {
  switch (dtype) {
  case REF_DOUBLE: return (int)sizeof(double);
  case REF_LONG: return (int)sizeof(long int);
  case REF_FLOAT: return (int)sizeof(float);
  case REF_INT: return (int)sizeof(int);
  case REF_CHAR: return 1;
  }
  return -1;
}

void ref_reduction(int dtype, void *p1, const void *p2, long n) {
  long i;
  switch (dtype) {
  case REF_DOUBLE: /* ext_mpi_native_exec.c:211-216 */
    for (i = 0; i < n; i++) ((double *)p1)[i] += ((const double *)p2)[i];
    break;
  case REF_LONG: /* :217-222 */
    for (i = 0; i < n; i++) ((long int *)p1)[i] += ((const long int *)p2)[i];
    break;
  case REF_FLOAT: /* :223-228 */
    for (i = 0; i < n; i++) ((float *)p1)[i] += ((const float *)p2)[i];
    break;
  case REF_INT: /* :229-234 */
    for (i = 0; i < n; i++) ((int *)p1)[i] += ((const int *)p2)[i];
    break;
  case REF_CHAR: /* :235-239 */
    for (i = 0; i < n; i++) ((char *)p1)[i] += ((const char *)p2)[i];
    break;
  }
}

/*
 * ref_reduction.c -- TEST INFRASTRUCTURE ONLY.
 * Restates reduction() in src/mpi/ext_mpi_native_exec.c:207-318: the MPI_SUM cases (:207-239,
 * one scalar pass "p1[i] += p2[i]" per SREDUCE line) and the MPI_MIN / MPI_MAX cases (:240-318,
 * "if (p2[i] < p1[i]) p1[i] = p2[i]" / "if (p2[i] > p1[i]) p1[i] = p2[i]"). Compiled like the reference
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

#define REF_PICK(T, CMP)                                                                  \
  for (i = 0; i < n; i++)                                                                 \
    if (((const T *)p2)[i] CMP((T *)p1)[i]) ((T *)p1)[i] = ((const T *)p2)[i];

void ref_reduction_op(int op, int dtype, void *p1, const void *p2, long n) {
  long i;
  if (op == REF_RED_SUM) {
    ref_reduction(dtype, p1, p2, n);
  } else if (op == REF_RED_MIN) {
    switch (dtype) {
    case REF_DOUBLE: REF_PICK(double, <) break;  /* :240-247 */
    case REF_LONG: REF_PICK(long int, <) break;  /* :248-255 */
    case REF_FLOAT: REF_PICK(float, <) break;    /* :256-263 */
    case REF_INT: REF_PICK(int, <) break;        /* :264-271 */
    case REF_CHAR: REF_PICK(char, <) break;      /* :272-278 */
    }
  } else if (op == REF_RED_MAX) {
    switch (dtype) {
    case REF_DOUBLE: REF_PICK(double, >) break;  /* :279-286 */
    case REF_LONG: REF_PICK(long int, >) break;  /* :287-294 */
    case REF_FLOAT: REF_PICK(float, >) break;    /* :295-302 */
    case REF_INT: REF_PICK(int, >) break;        /* :303-310 */
    case REF_CHAR: REF_PICK(char, >) break;      /* :311-317 */
    }
  }
}

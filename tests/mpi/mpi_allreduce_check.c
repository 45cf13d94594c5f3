/* Drop-in check of libext_mpi_collectives.so, written like an application of the reference
 * (tests/benchmark.c shape): only MPI calls plus the MPI-4 prototype from ext_mpi_interface.h.
 * argv: count dtype(f|d|i|l) mem(dev|host) [inplace] [blocking] [min|max]. "blocking" drives MPI_Allreduce
 * (run with EXT_MPI_BLOCKING set) instead of MPI_Allreduce_init. Prints "RESULT ok" / "RESULT no-device"
 * / "RESULT pmpi" (no GPU; a blocking call handed to PMPI_Allreduce, exact) / "RESULT fail ...".
 * Integer inputs are checked exactly against PMPI_Allreduce; float inputs are integer-valued (exact in any order) so the same comparison applies. */
#include <mpi.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "ext_mpi_amd_gpu.h"
#include "ext_mpi_interface.h"

int main(int argc, char **argv) {
  int rank, size, count = argc > 1 ? atoi(argv[1]) : 1000, rc, i, bad = 0, flag;
  char t = argc > 2 ? argv[2][0] : 'f';
  int dev = argc > 3 ? !strcmp(argv[3], "dev") : 1, inplace = 0, blocking = 0;
  MPI_Datatype dt = t == 'd' ? MPI_DOUBLE : t == 'i' ? MPI_INT : t == 'l' ? MPI_LONG : MPI_FLOAT;
  int ts = (t == 'd' || t == 'l') ? 8 : 4;
  size_t bytes = (size_t)count * ts;
  void *hs, *hr, *ref, *s = NULL, *r = NULL;
  MPI_Request req, p2p[2];
  MPI_Op op = MPI_SUM;
  for (i = 4; i < argc; i++) {
    inplace |= !strcmp(argv[i], "inplace");
    blocking |= !strcmp(argv[i], "blocking");
    if (!strcmp(argv[i], "min")) op = MPI_MIN;
    if (!strcmp(argv[i], "max")) op = MPI_MAX;
  }
  MPI_Init(&argc, &argv);
  MPI_Comm_rank(MPI_COMM_WORLD, &rank);
  MPI_Comm_size(MPI_COMM_WORLD, &size);
  hs = malloc(bytes);
  hr = malloc(bytes);
  ref = malloc(bytes);
  for (i = 0; i < count; i++) {
    long v = (long)(rank + 1) * (i % 1000) - 7 * rank;
    if (t == 'f') ((float *)hs)[i] = (float)v;
    else if (t == 'd') ((double *)hs)[i] = (double)v;
    else if (t == 'i') ((int *)hs)[i] = (int)v;
    else ((long *)hs)[i] = v;
  }
  PMPI_Allreduce(hs, ref, count, dt, op, MPI_COMM_WORLD);
  /* requests we do not own fall through to PMPI (ext_mpi_interface.c:257-265) */
  {
    int a = rank, b = -1, peer = (rank + 1) % size, from = (rank + size - 1) % size;
    MPI_Send_init(&a, 1, MPI_INT, peer, 5, MPI_COMM_WORLD, &p2p[0]);
    MPI_Recv_init(&b, 1, MPI_INT, from, 5, MPI_COMM_WORLD, &p2p[1]);
    MPI_Startall(2, p2p);
    MPI_Waitall(2, p2p, MPI_STATUSES_IGNORE);
    MPI_Request_free(&p2p[0]);
    MPI_Request_free(&p2p[1]);
    if (b != from) bad |= 1;
  }
  if (ext_mpi_amd_gpu_device_count() <= 0) {
    if (blocking) rc = MPI_Allreduce(hs, hr, count, dt, op, MPI_COMM_WORLD) == MPI_SUCCESS ? 0 : -5;
    else rc = MPI_Allreduce_init(hs, hr, count, dt, op, MPI_COMM_WORLD, MPI_INFO_NULL, &req);
    /* a blocking call this path does not take goes to PMPI_Allreduce: "pmpi" when exact */
    if (blocking && rc == 0 && memcmp(hr, ref, bytes)) bad |= 2;
    MPI_Allreduce(MPI_IN_PLACE, &bad, 1, MPI_INT, MPI_BOR, MPI_COMM_WORLD);
    if (rank == 0)
      printf("RESULT %s rc=%d\n", bad ? "fail" : rc == -5 ? "no-device" : blocking && rc == 0 ? "pmpi" : "fail", rc);
    MPI_Finalize();
    return 0;
  }
  if (dev) {
    ext_mpi_amd_gpu_malloc(&r, bytes);
    if (!inplace) ext_mpi_amd_gpu_malloc(&s, bytes);
    ext_mpi_amd_gpu_memcpy_hd(inplace ? r : s, hs, bytes);
  } else {
    r = hr;
    s = hs;
    if (inplace) memcpy(hr, hs, bytes);
  }
  if (blocking) {
    /* repeated calls (handle cache hits), a second buffer pair (a miss), a derived communicator */
    void *s2 = NULL, *r2 = NULL;
    MPI_Comm dup;
    MPI_Comm_dup(MPI_COMM_WORLD, &dup);
    if (dev) {
      ext_mpi_amd_gpu_malloc(&r2, bytes);
      ext_mpi_amd_gpu_malloc(&s2, bytes);
      ext_mpi_amd_gpu_memcpy_hd(s2, hs, bytes);
    } else {
      r2 = malloc(bytes);
      s2 = malloc(bytes);
      memcpy(s2, hs, bytes);
    }
    for (int it = 0; it < 6; it++) {
      int second = it == 3 || it == 4;
      void *rr = second ? r2 : r, *ss = second ? s2 : s;
      MPI_Comm c = it == 5 ? dup : MPI_COMM_WORLD;
      if (inplace) {
        if (dev) ext_mpi_amd_gpu_memcpy_hd(rr, hs, bytes);
        else memcpy(rr, hs, bytes);
      }
      rc = MPI_Allreduce(inplace ? MPI_IN_PLACE : ss, rr, count, dt, op, c);
      if (rc != MPI_SUCCESS) {
        printf("RESULT fail blocking rc=%d\n", rc);
        MPI_Abort(MPI_COMM_WORLD, 1);
      }
      if (dev) ext_mpi_amd_gpu_memcpy_dh(hr, rr, bytes);
      else if (rr != hr) memcpy(hr, rr, bytes);
      if (memcmp(hr, ref, bytes)) bad |= 4 << it;
    }
    MPI_Comm_free(&dup);
    if (dev) {
      ext_mpi_amd_gpu_free(r2);
      ext_mpi_amd_gpu_free(s2);
    } else {
      free(r2);
      free(s2);
    }
    goto report;
  }
  rc = MPI_Allreduce_init(inplace ? MPI_IN_PLACE : s, r, count, dt, op, MPI_COMM_WORLD, MPI_INFO_NULL, &req);
  if (rc) {
    printf("RESULT fail init rc=%d\n", rc);
    MPI_Abort(MPI_COMM_WORLD, 1);
  }
  for (int it = 0; it < 3; it++) {
    if (inplace) { /* the persistent buffer is reused: refill it each round */
      if (dev) ext_mpi_amd_gpu_memcpy_hd(r, hs, bytes);
      else memcpy(hr, hs, bytes);
    }
    MPI_Start(&req);
    if (it == 1) {
      do { MPI_Test(&req, &flag, MPI_STATUS_IGNORE); } while (!flag);
    } else {
      MPI_Wait(&req, MPI_STATUS_IGNORE);
    }
    if (dev) ext_mpi_amd_gpu_memcpy_dh(hr, r, bytes);
    if (memcmp(hr, ref, bytes)) bad |= 2;
  }
  MPI_Request_free(&req);
report:
  MPI_Allreduce(MPI_IN_PLACE, &bad, 1, MPI_INT, MPI_BOR, MPI_COMM_WORLD);
  if (rank == 0) printf("RESULT %s (size=%d count=%d type=%c mem=%s%s%s%s) bad=%d\n", bad ? "fail" : "ok", size, count, t,
                        dev ? "dev" : "host", inplace ? " inplace" : "", blocking ? " blocking" : "",
                        op == MPI_MIN ? " min" : op == MPI_MAX ? " max" : "", bad);
  if (dev) {
    ext_mpi_amd_gpu_free(r);
    ext_mpi_amd_gpu_free(s);
  }
  MPI_Finalize();
  return 0;
}

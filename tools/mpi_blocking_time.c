/* Latency of the blocking MPI_Allreduce front end on device buffers (the staging of
 * device buffers through communicator scratch) against the persistent MPI_Allreduce_init path on
 * the same buffers, through libext_mpi_collectives.so. argv: count [iterations].
 * Prints "TIME blocking <us> persistent <us> bytes <n> ranks <p>" on rank 0 (max over ranks). */
#include <mpi.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "ext_mpi_amd_gpu.h"
#include "ext_mpi_interface.h"

static double timed(int n, void *s, void *r, int count, MPI_Request *req) {
  double t0, el;
  int i;
  for (i = 0; i < 5; i++) { /* warm-up: handle creation and its cache */
    if (req) {
      MPI_Start(req);
      MPI_Wait(req, MPI_STATUS_IGNORE);
    } else {
      MPI_Allreduce(s, r, count, MPI_FLOAT, MPI_SUM, MPI_COMM_WORLD);
    }
  }
  MPI_Barrier(MPI_COMM_WORLD);
  t0 = MPI_Wtime();
  for (i = 0; i < n; i++) {
    if (req) {
      MPI_Start(req);
      MPI_Wait(req, MPI_STATUS_IGNORE);
    } else {
      MPI_Allreduce(s, r, count, MPI_FLOAT, MPI_SUM, MPI_COMM_WORLD);
    }
  }
  el = (MPI_Wtime() - t0) / n;
  MPI_Allreduce(MPI_IN_PLACE, &el, 1, MPI_DOUBLE, MPI_MAX, MPI_COMM_WORLD);
  return el * 1e6;
}

int main(int argc, char **argv) {
  int rank, size, count = argc > 1 ? atoi(argv[1]) : 1024, n = argc > 2 ? atoi(argv[2]) : 200, i;
  size_t bytes = (size_t)count * 4;
  void *s, *r;
  float *h, *got;
  MPI_Request req;
  double tb, tp;
  int bad = 0;
  MPI_Init(&argc, &argv);
  MPI_Comm_rank(MPI_COMM_WORLD, &rank);
  MPI_Comm_size(MPI_COMM_WORLD, &size);
  h = (float *)malloc(bytes);
  got = (float *)malloc(bytes);
  for (i = 0; i < count; i++) h[i] = (float)((rank + 1) * (i % 100));
  ext_mpi_amd_gpu_malloc(&s, bytes);
  ext_mpi_amd_gpu_malloc(&r, bytes);
  ext_mpi_amd_gpu_memcpy_hd(s, h, bytes);
  tb = timed(n, s, r, count, NULL);
  ext_mpi_amd_gpu_memcpy_dh(got, r, bytes);
  for (i = 0; i < count; i++)
    if (got[i] != (float)(size * (size + 1) / 2 * (i % 100))) bad = 1;
  MPI_Allreduce_init(s, r, count, MPI_FLOAT, MPI_SUM, MPI_COMM_WORLD, MPI_INFO_NULL, &req);
  tp = timed(n, s, r, count, &req);
  MPI_Request_free(&req);
  MPI_Allreduce(MPI_IN_PLACE, &bad, 1, MPI_INT, MPI_BOR, MPI_COMM_WORLD);
  if (rank == 0) printf("TIME blocking %.2f persistent %.2f bytes %zu ranks %d %s\n", tb, tp, bytes, size, bad ? "BAD" : "ok");
  ext_mpi_amd_gpu_free(s);
  ext_mpi_amd_gpu_free(r);
  MPI_Finalize();
  return 0;
}

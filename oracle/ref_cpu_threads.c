/*
 * ref_cpu_threads.c -- TEST / BASELINE INFRASTRUCTURE ONLY (bench.py cpu_baseline leg).
 *
 * Times the reference's CPU execution shape: R host threads stand in for the R node ranks
 * (which the reference runs as processes sharing XPMEM-mapped buffers). Each thread runs
 * its own rank's copy-in + copy-out program: memcpy per SMEMCPY line, one scalar
 * "p1[i] += p2[i]" pass per SREDUCE line (ext_mpi_native_exec.c:207-234, :392-396,
 * :529-536), and a spin barrier where the schedule has a SET_NODE_BARRIER
 * (ext_mpi_native_exec.c:21-84 uses pairwise flags; a sense-reversing barrier is used here).
 */
#include <pthread.h>
#include <stdatomic.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include "ref_oracle.h"

typedef struct {
  ref_op *ops;
  int n;
  int pc;
} rank_prog;

int ref_build_programs_(int R, long count, int dtype, const char *copyin, int in_place, void *progs_out);

typedef struct {
  atomic_int count;
  atomic_int sense;
  int total;
} spin_barrier;

static void barrier_wait(spin_barrier *b, int *local_sense) {
  *local_sense = !*local_sense;
  if (atomic_fetch_add_explicit(&b->count, 1, memory_order_acq_rel) == b->total - 1) {
    atomic_store_explicit(&b->count, 0, memory_order_relaxed);
    atomic_store_explicit(&b->sense, *local_sense, memory_order_release);
  } else {
    while (atomic_load_explicit(&b->sense, memory_order_acquire) != *local_sense) {
    }
  }
}

typedef struct {
  int R, r, dtype, nsets;
  long iters;
  rank_prog *prog;
  void *const *send;
  void *const *recv;
  spin_barrier *bar;
  double *t_out;
} worker_arg;

static double now_s(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

static void *worker(void *varg) {
  worker_arg *a = (worker_arg *)varg;
  int sense = 0, tsize = ref_type_size(a->dtype);
  long it;
  double t0;
  barrier_wait(a->bar, &sense);
  t0 = now_s();
  for (it = 0; it < a->iters; it++) {
    int pc;
    /* buffer set of this iteration (sets rotate so the working set can exceed the host caches) */
    void *const *send = a->send + (size_t)(it % a->nsets) * (size_t)a->R;
    void *const *recv = a->recv + (size_t)(it % a->nsets) * (size_t)a->R;
    for (pc = 0; pc < a->prog->n; pc++) {
      const ref_op *o = &a->prog->ops[pc];
      if (o->op == REF_OP_PHASE) {
        barrier_wait(a->bar, &sense);
        continue;
      }
      {
        char *dst = (char *)(o->dbuf == REF_BUF_RECV ? recv : send)[(a->r + o->drel) % a->R] + o->doff;
        const char *src = (const char *)(o->sbuf == REF_BUF_RECV ? recv : send)[(a->r + o->srel) % a->R] + o->soff;
        if (o->op == REF_OP_COPY)
          memcpy(dst, src, (size_t)o->bytes);
        else
          ref_reduction(a->dtype, dst, src, o->bytes / tsize);
      }
    }
    barrier_wait(a->bar, &sense); /* next Start only after every rank finished */
  }
  if (a->r == 0) *a->t_out = now_s() - t0;
  return NULL;
}

/* nsets buffer sets of R send and R receive buffers (set k at [k * R, (k + 1) * R)); iteration i
   runs on set i % nsets. */
double ref_cpu_allreduce_threads_sets(int R, long count, int dtype, const char *copyin, int nsets,
                                      void *const *sendbufs, void *const *recvbufs, long iters) {
  rank_prog *progs;
  pthread_t *th;
  worker_arg *args;
  spin_barrier bar;
  double elapsed = -1.0;
  int r;
  if (R < 2 || nsets < 1) return -1.0;
  progs = (rank_prog *)calloc((size_t)R, sizeof(rank_prog));
  if (ref_build_programs_(R, count, dtype, copyin, 0, progs)) goto done;
  atomic_init(&bar.count, 0);
  atomic_init(&bar.sense, 0);
  bar.total = R;
  th = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)R);
  args = (worker_arg *)malloc(sizeof(worker_arg) * (size_t)R);
  for (r = 0; r < R; r++) {
    args[r].R = R;
    args[r].r = r;
    args[r].dtype = dtype;
    args[r].nsets = nsets;
    args[r].iters = iters;
    args[r].prog = &progs[r];
    args[r].send = sendbufs;
    args[r].recv = recvbufs;
    args[r].bar = &bar;
    args[r].t_out = &elapsed;
    pthread_create(&th[r], NULL, worker, &args[r]);
  }
  for (r = 0; r < R; r++) pthread_join(th[r], NULL);
  free(args);
  free(th);
done:
  for (r = 0; r < R; r++) free(progs[r].ops);
  free(progs);
  return elapsed;
}

double ref_cpu_allreduce_threads(int R, long count, int dtype, const char *copyin,
                                 void *const *sendbufs, void *const *recvbufs, long iters) {
  return ref_cpu_allreduce_threads_sets(R, count, dtype, copyin, 1, sendbufs, recvbufs, iters);
}

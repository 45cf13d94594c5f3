/*
 * ext_mpi.h -- native (handle-based) API of libext_mpi_collectives.so for the Allreduce path,
 * same prototypes as the reference's include/mpi/ext_mpi.h:69-89 (Allreduce subset) and
 * EXT_MPI_Init / EXT_MPI_Finalize (src/mpi/ext_mpi.c:1043-1061).
 */
#ifndef EXT_MPI_H_
#define EXT_MPI_H_

#include <mpi.h>

#ifdef __cplusplus
extern "C" {
#endif

int EXT_MPI_Init(void);
int EXT_MPI_Initialized(int *flag);
int EXT_MPI_Finalize(void);
int EXT_MPI_Allreduce_init(const void *sendbuf, void *recvbuf, int count, MPI_Datatype datatype, MPI_Op op,
                           MPI_Comm comm, MPI_Info info, int *handle);
int EXT_MPI_Start(int handle);
int EXT_MPI_Test(int handle);
int EXT_MPI_Wait(int handle);
int EXT_MPI_Done(int handle);

#ifdef __cplusplus
}
#endif

#endif

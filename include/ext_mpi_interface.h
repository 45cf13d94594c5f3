/*
 * ext_mpi_interface.h -- the drop-in MPI surface of libext_mpi_collectives.so (PMPI layer),
 * same prototypes as the reference's include/mpi/ext_mpi_interface.h:12 (MPI-4 persistent
 * collective, declared here because MPI-3 libraries such as MPICH 3.3 lack it).
 *
 * Link (or LD_PRELOAD) libext_mpi_collectives.so before the MPI library: its strong
 * MPI_Init, MPI_Init_thread, MPI_Finalize, MPI_Start, MPI_Startall, MPI_Wait, MPI_Waitall,
 * MPI_Waitany, MPI_Waitsome, MPI_Test, MPI_Testall, MPI_Testany, MPI_Testsome and
 * MPI_Request_free override the library's (reference src/mpi/ext_mpi_interface.c:71-426) and
 * forward every request they do not own to PMPI_*.
 */
#ifndef EXT_MPI_INTERFACE_H_
#define EXT_MPI_INTERFACE_H_

#include <mpi.h>

#ifdef __cplusplus
extern "C" {
#endif

int MPI_Allreduce_init(const void *sendbuf, void *recvbuf, int count, MPI_Datatype datatype, MPI_Op op, MPI_Comm comm,
                       MPI_Info info, MPI_Request *request);

#ifdef __cplusplus
}
#endif

#endif

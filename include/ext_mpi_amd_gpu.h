/*
 * ext_mpi_amd_gpu.h -- device C ABI of libext_mpi_amd.so, replacing the reference's
 * include/gpu/gpu_core.h:11-22 (implemented in src/gpu/cuda_core.cu:7-106):
 *
 *   ext_mpi_amd_gpu_malloc            <- ext_mpi_gpu_malloc(void **p, int size)
 *   ext_mpi_amd_gpu_free              <- ext_mpi_gpu_free(void *p)
 *   ext_mpi_amd_gpu_memcpy_hd / _dh   <- ext_mpi_gpu_memcpy_hd / _dh(void *dst, void *src, int n)
 *   ext_mpi_amd_gpu_is_device_pointer <- ext_mpi_gpu_is_device_pointer(const void *p)
 *   ext_mpi_amd_gpu_synchronize       <- ext_mpi_gpu_synchronize()
 *   ext_mpi_amd_gpu_copy_reduce       <- ext_mpi_gpu_copy_reduce(char op, void *desc, int count)
 *
 * Sizes are size_t (the reference's int limits buffers to 2 GiB) and errors are returned
 * (the reference exit(13)s). copy_reduce takes one owner chunk: `nsrc` leaves folded in the
 * given order (left fold: ((src[0] + src[1]) + src[2]) + ...) and the result stored to `ndst`
 * destinations, i.e. one fused SMEMCPY + (nsrc-1) x SREDUCE + fan-out stream of byte_code.c.
 */
#ifndef EXT_MPI_AMD_GPU_H_
#define EXT_MPI_AMD_GPU_H_

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

int ext_mpi_amd_gpu_malloc(void **p, size_t bytes);
int ext_mpi_amd_gpu_free(void *p);
int ext_mpi_amd_gpu_memcpy_hd(void *dst, const void *src, size_t bytes);
int ext_mpi_amd_gpu_memcpy_dh(void *dst, const void *src, size_t bytes);
int ext_mpi_amd_gpu_is_device_pointer(const void *p);
int ext_mpi_amd_gpu_synchronize(void);
int ext_mpi_amd_gpu_device_count(void);
int ext_mpi_amd_gpu_device_of(const void *p); /* device ordinal owning p, -1 for host memory */
int ext_mpi_amd_gpu_copy_reduce(int dtype, int op, int nsrc, const void *const *srcs, int ndst, void *const *dsts,
                                long count, void *hip_stream);
/* Stream-ordered helpers of the MPI layer's staging (no reference counterpart: its copies are
 * synchronous): a copy enqueued on hip_stream, and hip_stream made to wait (an event, no host
 * synchronisation) for the work enqueued so far on the legacy default stream -- which itself
 * waits for every blocking stream, where an application that does not synchronise before an MPI
 * call leaves the work producing its send buffer. */
int ext_mpi_amd_gpu_memcpy_async(void *dst, const void *src, size_t bytes, void *hip_stream);
int ext_mpi_amd_gpu_after_default_stream(void *hip_stream);

#ifdef __cplusplus
}
#endif
#endif

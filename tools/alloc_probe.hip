// Probe: does the runtime sub-allocate hipMalloc / uncached allocations out of shared chunks?
// Prints each allocation's address range (hipMemGetAddressRange), buffer id and IPC handle prefix.
#include <hip/hip_runtime.h>
#include <stdio.h>

static void show(const char *what, void *p) {
  void *base = nullptr;
  size_t size = 0;
  unsigned long long id = 0;
  hipIpcMemHandle_t h;
  hipMemGetAddressRange(&base, &size, p);
  hipPointerGetAttribute(&id, HIP_POINTER_ATTRIBUTE_BUFFER_ID, (hipDeviceptr_t)base);
  hipError_t e = hipIpcGetMemHandle(&h, base);
  const unsigned char *b = (const unsigned char *)&h;
  printf("%-22s p=%p base=%p size=%zu id=%llu ipc=%s ", what, p, base, size, id, hipGetErrorString(e));
  for (int i = 0; i < 24; i++) printf("%02x", b[i]);
  printf("\n");
}

int main() {
  size_t sizes[] = {4096, 1 << 20, 2 << 20, 4 << 20, 64 << 20};
  for (size_t s : sizes) {
    for (int k = 0; k < 2; k++) {
      void *p = nullptr, *q = nullptr;
      char w[64];
      hipMalloc(&p, s);
      snprintf(w, sizeof(w), "hipMalloc %zu #%d", s, k);
      show(w, p);
      hipExtMallocWithFlags(&q, s, hipDeviceMallocUncached);
      snprintf(w, sizeof(w), "uncached %zu #%d", s, k);
      show(w, q);
    }
  }
  return 0;
}

// where hipMallocSignalMemory lives (diagnostic): pointer attributes of an 8-byte signal word
#include <hip/hip_runtime.h>
#include <stdio.h>
int main() {
    void* p = nullptr;
    hipError_t e = hipExtMallocWithFlags(&p, 8, hipMallocSignalMemory);
    printf("alloc %s %p\n", hipGetErrorString(e), p);
    hipPointerAttribute_t a;
    e = hipPointerGetAttributes(&a, p);
    printf("attr %s type %d device %d hostPointer %p devicePointer %p isManaged %d allocationFlags %u\n",
           hipGetErrorString(e), (int)a.type, a.device, a.hostPointer, a.devicePointer, a.isManaged, a.allocationFlags);
    printf("hipMemoryTypeHost=%d hipMemoryTypeDevice=%d\n", (int)hipMemoryTypeHost, (int)hipMemoryTypeDevice);
    hipFree(p);
    return 0;
}

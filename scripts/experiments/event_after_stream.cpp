// Does HIP tolerate using an event after the stream it was recorded on is destroyed?  (Round 4: a
// workspace's part-lease events outlive the streams they were recorded on.)  Not product code.
#include <hip/hip_runtime.h>
#include <stdio.h>
__global__ void k_spin(int* p) { if (threadIdx.x == 0) atomicAdd(p, 1); }
int main() {
    int* d = nullptr;
    if (hipMalloc(&d, 4) != hipSuccess) return 2;
    for (int it = 0; it < 2000; ++it) {
        hipStream_t s, t;
        hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
        hipStreamCreateWithFlags(&t, hipStreamNonBlocking);
        hipEvent_t e;
        hipEventCreateWithFlags(&e, hipEventDisableTiming);
        hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s, d);
        hipEventRecord(e, s);
        if (it & 1) hipStreamSynchronize(s);
        hipStreamDestroy(s);
        const hipError_t q = hipEventQuery(e);
        const hipError_t y = hipEventSynchronize(e);
        const hipError_t w = hipStreamWaitEvent(t, e, 0);
        hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, t, d);
        const hipError_t z = hipStreamSynchronize(t);
        if (it < 4 || y != hipSuccess || w != hipSuccess || z != hipSuccess)
            printf("it %d: query %d sync %d wait %d stream %d\n", it, (int)q, (int)y, (int)w, (int)z);
        hipStreamDestroy(t);
        hipEventDestroy(e);
    }
    printf("done\n");
    return 0;
}

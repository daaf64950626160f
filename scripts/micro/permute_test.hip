// Micro-test: ds_permute_b32 semantics for unwritten destination lanes (exec-masked sources).
#include <hip/hip_runtime.h>
#include <stdio.h>
__global__ void k(int* out) {
    int lane = threadIdx.x;
    int v = 7;  // sentinel in every lane before the permute
    int r = v;
    if (lane % 3 == 0) {  // only some lanes push: lane i pushes (100+i) to lane (i/3)
        r = __builtin_amdgcn_ds_permute((lane / 3) * 4, 100 + lane);
    } else {
        r = __builtin_amdgcn_ds_permute(0, 0);  // placeholder (not executed for these lanes in SIMT? it is, separately)
    }
    out[lane] = r;
    // variant 2: single permute with exec mask from a branch around ONLY the permute
    int w = -1;
    if (lane % 3 == 0) w = __builtin_amdgcn_ds_permute((lane / 3) * 4, 200 + lane);
    out[64 + lane] = w;
    // variant 3: all lanes active, some push to distinct lanes, others push to a dump lane 63
    int dst = (lane % 3 == 0) ? (lane / 3) : 63;
    int z = __builtin_amdgcn_ds_permute(dst * 4, (lane % 3 == 0) ? 1 : 0);
    out[128 + lane] = z;
}
int main() {
    int* d; hipMalloc(&d, 192 * 4);
    hipLaunchKernelGGL(k, 1, 64, 0, 0, d);
    int h[192]; hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
    for (int v = 0; v < 3; ++v) { printf("variant %d:", v + 1); for (int i = 0; i < 64; ++i) printf(" %d", h[v * 64 + i]); printf("\n"); }
    return 0;
}

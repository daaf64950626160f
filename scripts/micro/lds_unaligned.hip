// Checks that unaligned ds_read_b128 / b64 / b32 (aligned(1) LDS pointers, which hipcc emits for
// gfx950) return the bytes at the unaligned address, and times them against aligned reads.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
typedef unsigned int v4 __attribute__((ext_vector_type(4)));
typedef v4 __attribute__((aligned(1))) v4u;
typedef unsigned long long u64u __attribute__((aligned(1)));
__global__ void k(unsigned* out, unsigned a) {
    __shared__ __attribute__((aligned(16))) unsigned char lds[4096 + 16];
    for (int i = threadIdx.x; i < 4096 + 16; i += 64) lds[i] = (unsigned char)(i * 7 + (i >> 8));
    __syncthreads();
    const unsigned p = (a + threadIdx.x * 13) & 4095;
    const v4 v = *(const v4u*)(lds + p);
    const unsigned long long w = *(const u64u*)(lds + p + 3);
    out[threadIdx.x * 6 + 0] = v.x;
    out[threadIdx.x * 6 + 1] = v.y;
    out[threadIdx.x * 6 + 2] = v.z;
    out[threadIdx.x * 6 + 3] = v.w;
    out[threadIdx.x * 6 + 4] = (unsigned)w;
    out[threadIdx.x * 6 + 5] = (unsigned)(w >> 32);
}
int timing();
int main() {
    unsigned* d;
    (void)hipMalloc(&d, 64 * 6 * 4);
    unsigned h[64 * 6];
    int bad = 0;
    for (unsigned a = 0; a < 64; ++a) {
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, a);
        (void)hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
        for (int t = 0; t < 64; ++t) {
            const unsigned p = (a + t * 13) & 4095;
            auto byte = [](unsigned i) { return (unsigned)(unsigned char)(i * 7 + (i >> 8)); };
            for (int j = 0; j < 16; ++j)
                if (((h[t * 6 + j / 4] >> (8 * (j % 4))) & 0xFF) != byte(p + j)) bad++;
            for (int j = 0; j < 8; ++j)
                if (((h[t * 6 + 4 + j / 4] >> (8 * (j % 4))) & 0xFF) != byte(p + 3 + j)) bad++;
        }
    }
    printf("unaligned LDS reads: %s (%d bad bytes)\n", bad ? "WRONG" : "ok", bad);
    if (bad) return 1;
    return timing();
}
// (timing) dependent chains of LDS reads: aligned b128, unaligned b128, unaligned b64, unaligned b32
template <int MODE>
__global__ void kt(unsigned* out, unsigned a, int iters) {
    __shared__ __attribute__((aligned(16))) unsigned char lds[8192 + 32];
    for (int i = threadIdx.x; i < 8192 + 32; i += blockDim.x) lds[i] = (unsigned char)(i * 7);
    __syncthreads();
    unsigned p = (a + threadIdx.x * 37) & 8191, acc = 0;
    for (int i = 0; i < iters; ++i) {
        unsigned q = MODE == 0 ? (p & ~15u) : p;
        if (MODE <= 1) {
            const v4 v = *(const v4u*)(lds + q);
            acc += v.x ^ v.y ^ v.z ^ v.w;
        } else if (MODE == 2) {
            acc += (unsigned)*(const u64u*)(lds + q);
        } else {
            typedef unsigned u32u __attribute__((aligned(1)));
            acc += *(const u32u*)(lds + q);
        }
        p = (p + acc * 13 + 29) & 8191;
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}
int timing() {
    unsigned* d;
    (void)hipMalloc(&d, 1024 * 1024 * 4);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    const char* names[4] = {"aligned b128", "unaligned b128", "unaligned b64", "unaligned b32"};
    for (int m = 0; m < 4; ++m) {
        for (int rep = 0; rep < 2; ++rep) {
            (void)hipEventRecord(a, 0);
            if (m == 0) hipLaunchKernelGGL(kt<0>, dim3(1024), dim3(1024), 0, 0, d, 5u, 4096);
            if (m == 1) hipLaunchKernelGGL(kt<1>, dim3(1024), dim3(1024), 0, 0, d, 5u, 4096);
            if (m == 2) hipLaunchKernelGGL(kt<2>, dim3(1024), dim3(1024), 0, 0, d, 5u, 4096);
            if (m == 3) hipLaunchKernelGGL(kt<3>, dim3(1024), dim3(1024), 0, 0, d, 5u, 4096);
            (void)hipEventRecord(b, 0);
            (void)hipEventSynchronize(b);
            float ms = 0;
            (void)hipEventElapsedTime(&ms, a, b);
            if (rep) printf("%-16s %.3f ms (1024 x 1024 lanes x 4096 dependent reads)\n", names[m], ms);
        }
    }
    return 0;
}

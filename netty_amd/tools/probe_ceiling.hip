// probe_ceiling.hip — measurement tool, not part of libnetty_amd: the random-access ceiling that
// bounds the Snappy encoder (bench.py reports the encoder's probe rate against it).
//
// Every lane runs a serial chain of `steps` probes into its own 128 KiB table (16 384 u64 entries,
// the encoder's wide entries), each an agent-scope atomic exchange whose result picks the next
// index, and — for load_permille / 1000 of the steps (bench.py: 258, the encoder's first reads of a
// candidate on the bench corpus: 4 275 matches of 7+ bytes per 16 546 probes per 64 KiB chunk) — a
// dependent 4-byte load at a random position of the lane's own 64 KiB input region, and — for
// insert_permille / 1000 of the steps (bench.py: 467, the 7 724 inserts after matches per 16 546
// probes) — an agent-scope store of a 64-bit entry to another random slot (the insert, :187-188).
// That is the encoder's memory-request pattern without its compute, stream reads or output.
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ void __launch_bounds__(256) k_probe_chain(uint64_t* __restrict__ tab, const uint32_t* __restrict__ inp, uint32_t lanes,
                                                     uint32_t steps, uint32_t load_permille, uint32_t insert_permille,
                                                     uint32_t* __restrict__ sink) {
    const uint32_t l = blockIdx.x * blockDim.x + threadIdx.x;
    if (l >= lanes) return;
    uint64_t* t = tab + (size_t)l * 16384u;
    const uint32_t* src = inp + (size_t)l * 16384u;
    uint32_t h = l * 0x9E3779B1u, acc = 0;
    for (uint32_t i = 0; i < steps; ++i) {
        uint32_t v = (uint32_t)__hip_atomic_exchange(&t[(h * 0x1e35a7bdu) >> 18], (uint64_t)i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (((h >> 7) % 1000u) < load_permille) v += src[(v * 0x27D4EB2Fu + i) >> 18];
        if (((h >> 17) % 1000u) < insert_permille)
            __hip_atomic_store(&t[(h * 0x2545F491u) >> 18], (uint64_t)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        acc += v;
        h = h * 0x85EBCA77u + v + i;
    }
    sink[l] = acc;
}

// tab: lanes x 128 KiB, inp: lanes x 64 KiB (contents arbitrary); sink: lanes u32.  Runs a short
// warm-up chain, then the timed one; *ms = the timed kernel's duration.  Returns 0 or -1 on a HIP error.
extern "C" int32_t nx_probe_ceiling(uint64_t* tab, const uint32_t* inp, uint32_t* sink, uint32_t lanes, uint32_t steps,
                                    uint32_t load_permille, uint32_t insert_permille, float* ms, void* stream) {
    const hipStream_t st = (hipStream_t)stream;
    const dim3 grid((lanes + 255u) / 256u), block(256);
    hipEvent_t a, b;
    if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) return -1;
    hipLaunchKernelGGL(k_probe_chain, grid, block, 0, st, tab, inp, lanes, 256u, load_permille, insert_permille, sink);
    int32_t rc = 0;
    if (hipEventRecord(a, st) != hipSuccess) rc = -1;
    hipLaunchKernelGGL(k_probe_chain, grid, block, 0, st, tab, inp, lanes, steps, load_permille, insert_permille, sink);
    if (hipGetLastError() != hipSuccess || hipEventRecord(b, st) != hipSuccess || hipEventSynchronize(b) != hipSuccess ||
        hipEventElapsedTime(ms, a, b) != hipSuccess)
        rc = -1;
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    return rc;
}

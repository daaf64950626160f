# Instrumented copy of snappy_decode.hip: per-frame pass / round counters (diagnostic build only).
import sys
s = open(sys.argv[1]).read()
def rep(a, b, n=1):
    global s
    assert s.count(a) == n, (a[:60], s.count(a))
    s = s.replace(a, b)
rep("struct Window {\n", "__device__ unsigned long long g_dec_stats[8];\nstruct Window {\n")
rep("uint32_t xv, int lane, uint32_t P0s = 0u, bool last = true, Window* nw = nullptr) {",
    "uint32_t xv, int lane, uint32_t P0s = 0u, bool last = true, Window* nw = nullptr, uint32_t* cnt = nullptr) {")
rep("        const uint32_t mk = incl_max_scan(L.scratch[lane]);\n        const uint32_t P = P0 + lane;\n        const bool valid = P < Ptot;\n",
    "        const uint32_t mk = incl_max_scan(L.scratch[lane]);\n        const uint32_t P = P0 + lane;\n        const bool valid = P < Ptot;\n"
    "        if (cnt) { cnt[1] += 1; cnt[7] += (uint32_t)__popcll(__ballot(valid)); }\n")
rep("        if (__ballot(dep)) {\n", "        if (__ballot(dep)) {\n            if (cnt) cnt[3] += 1;\n")
rep("        if (__ballot(valid && gl)) {\n", "        if (__ballot(valid && gl)) {\n            if (cnt) cnt[4] += 1;\n")
rep("        if (has_ov) {\n", "        if (has_ov) {\n            if (cnt) cnt[5] += 1;\n")
rep("            if (round > 64) return false;\n", "            if (round > 64) return false;\n            if (cnt) cnt[2] += 1;\n")
rep("        uint32_t pdone = 0;\n        bool primed = false;\n", "        uint32_t pdone = 0;\n        bool primed = false;\n        uint32_t cnt[8] = {0, 0, 0, 0, 0, 0, 0, 0};\n")
rep("lane, pdone, last, &nw)) {", "lane, pdone, last, &nw, cnt)) {")
rep("            const bool last = b + 64u >= N;\n", "            const bool last = b + 64u >= N;\n            cnt[0] += 1;\n")
rep("        if (st == kGuardTrip + 2) O = Ofin;  // unreachable on a consistent record stream\n",
    "        if (st == kGuardTrip + 2) O = Ofin;  // unreachable on a consistent record stream\n"
    "        if (lane == 0) for (int q = 0; q < 8; ++q) atomicAdd(&g_dec_stats[q], (unsigned long long)cnt[q]);\n")
s += '''
extern "C" int32_t nx_dec_stats_read(unsigned long long* out) {
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(nx::dec::g_dec_stats), sizeof(unsigned long long) * 8) != hipSuccess) return -1;
    unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    return hipMemcpyToSymbol(HIP_SYMBOL(nx::dec::g_dec_stats), z, sizeof z) == hipSuccess ? 0 : -1;
}
'''
open(sys.argv[2], "w").write(s)

# Instrumented copy of snappy_decode.hip: per-section shader-clock stamps of k_expand's passes
# (diagnostic build only; s_memtime, summed per wave and added to a device array per frame).
#   python scripts/mk_dec_stamps.py netty_amd/csrc/snappy_decode.hip /tmp/stamps.hip
#   scripts/build_dec_variant.sh stamps /tmp/stamps.hip && python scripts/dec_stats.py --stamps
# Each stamp waits for the wave's outstanding LDS and scalar loads (s_memtime shares lgkmcnt), so
# the sections are "issued and their LDS traffic complete"; the build runs slower than the product.
import sys
s = open(sys.argv[1]).read()


def rep(a, b, n=1):
    global s
    assert s.count(a) == n, (a[:60], s.count(a))
    s = s.replace(a, b)


T = "__builtin_amdgcn_s_memtime()"
rep("struct Window {\n", "__device__ unsigned long long g_dec_stats[16];\nstruct Window {\n")
rep("                            bool staged = true) {",
    "                            bool staged = true, unsigned long long* tm = nullptr) {")
# [9] expand_tags prologue (record table, piece bases)
rep("    WaveLds& L = io.L;\n    const uint8_t* ring8 = reinterpret_cast<const uint8_t*>(L.ring);\n    const uint32_t* lds32 = L.ring;",
    "    const unsigned long long te = %s;\n    WaveLds& L = io.L;\n    const uint8_t* ring8 = reinterpret_cast<const uint8_t*>(L.ring);\n    const uint32_t* lds32 = L.ring;" % T)
rep("    uint32_t P0 = P0s;\n    if (P0 >= Pend) {",
    "    tm[9] += %s - te;\n    uint32_t P0 = P0s;\n    if (P0 >= Pend) {" % T)
rep("    } else do {\n",
    "    } else do {\n        unsigned long long t0 = %s, tq;\n" % T)
# [0] piece -> record map, record reads, pass bounds
rep("        const uint32_t pe = uni((uint32_t)__builtin_amdgcn_readlane((int)x1, (int)last));\n",
    "        const uint32_t pe = uni((uint32_t)__builtin_amdgcn_readlane((int)x1, (int)last));\n"
    "        tq = %s; tm[0] += tq - t0; t0 = tq;\n" % T)
# [1] source addresses, far-load issue, producer map
rep("        const bool has_ov = __ballot(valid && overlap) != 0ull;\n",
    "        tq = %s; tm[1] += tq - t0; t0 = tq;\n        const bool has_ov = __ballot(valid && overlap) != 0ull;\n" % T)
# [2] overlap addresses
rep("        const uint32_t w = sp >> 2;\n",
    "        tq = %s; tm[2] += tq - t0; t0 = tq;\n        const uint32_t w = sp >> 2;\n" % T)
# [3] round 0 (includes the wait for far / unstaged loads), [4] dependent rounds
rep("            if (!pending) break;\n            if (round >= 64) return false;\n",
    "            if (round == 0) { tq = %s; tm[3] += tq - t0; t0 = tq; }\n"
    "            if (!pending) break;\n            if (round >= 64) return false;\n" % T)
# [5] flush (stores + CRC); [6] passes
rep("        io.flush_to(pe);\n    } while",
    "        tq = %s; tm[4] += tq - t0; t0 = tq;\n        io.flush_to(pe);\n"
    "        tq = %s; tm[5] += tq - t0; tm[6] += 1;\n    } while" % (T, T))
# [7] whole frame (window setup, finish and result included)
rep("        uint32_t pdone = 0;\n        bool primed = false;\n",
    "        uint32_t pdone = 0;\n        bool primed = false;\n"
    "        unsigned long long tm[16] = {};\n        const unsigned long long tf = %s;\n        unsigned long long tw, tw2;\n" % T)
# [8] window setup, [10] slide, [12] windows
rep("        for (uint32_t b = 0; b < N;) {\n            const bool valid = b + (uint32_t)lane < N;\n",
    "        for (uint32_t b = 0; b < N;) {\n            tw = %s; tm[12] += 1;\n            const bool valid = b + (uint32_t)lane < N;\n" % T)
rep("            Window nw{0u, 0u, 0u};\n            if (!expand_tags(",
    "            Window nw{0u, 0u, 0u};\n            tm[8] += %s - tw;\n            if (!expand_tags(" % T)
rep("lane, pdone, last, &nw, &rnext, kExpandStaged)) {", "lane, pdone, last, &nw, &rnext, kExpandStaged, tm)) {")
rep("            if (last) {\n                O = E;\n                break;\n            }\n",
    "            tw2 = %s;\n            if (last) {\n                O = E;\n                break;\n            }\n" % T)
rep("            O = nw.O;\n        }\n",
    "            O = nw.O;\n            tm[10] += %s - tw2;\n        }\n        const unsigned long long tfin = %s;\n" % (T, T))
rep("        write_result(lane, crc, st, expect != nullptr, expect ? expect[c] : 0u, O, 0u, &out_len[c], nullptr, &status[c],\n"
    "                     crc_out ? &crc_out[c] : nullptr);\n    }\n}\n",
    "        write_result(lane, crc, st, expect != nullptr, expect ? expect[c] : 0u, O, 0u, &out_len[c], nullptr, &status[c],\n"
    "                     crc_out ? &crc_out[c] : nullptr);\n"
    "        tm[7] = %s - tf;\n        tm[11] = tm[7] + tf - tfin;\n"
    "        if (lane == 0) for (int q = 0; q < 16; ++q) atomicAdd(&g_dec_stats[q], tm[q]);\n    }\n}\n" % T)
# k_parse: [13] burst-reload cycles, [14] tag-loop cycles, [15] whole-kernel cycles, per wave
_k0 = s.index("k_parse(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,")
_k1 = s.index("__global__", _k0)
_pre, s, _post = s[:_k0], s[_k0:_k1], s[_k1:]
rep("    uint32_t ip = 0, op = 0;\n    int32_t st = NX_OK;\n    bool run = false;\n",
    "    uint32_t ip = 0, op = 0;\n    int32_t st = NX_OK;\n    bool run = false;\n"
    "    const unsigned long long tp0 = %s;\n    unsigned long long tpr = 0, tpi = 0, tpa, tpb;\n" % T)
rep("        if (run && !win.has(ip)) win.load(ip);  // burst reload: one wait for the whole wave\n        while (run && win.has(ip)) {\n",
    "        tpa = %s;\n        if (run && !win.has(ip)) win.load(ip);  // burst reload: one wait for the whole wave\n"
    "        tpb = %s; tpr += tpb - tpa;\n        while (run && win.has(ip)) {\n" % (T, T))
rep("            run = ip < in_len;\n        }\n    }\n    if (st == kNeedFused) {\n",
    "            run = ip < in_len;\n        }\n        tpi += %s - tpb;\n    }\n"
    "    if ((threadIdx.x & 63) == 0) { atomicAdd(&g_dec_stats[13], tpr); atomicAdd(&g_dec_stats[14], tpi); atomicAdd(&g_dec_stats[15], %s - tp0); }\n"
    "    if (st == kNeedFused) {\n" % (T, T))
s = _pre + s + _post
s += '''
extern "C" int32_t nx_dec_stats_read(unsigned long long* out) {
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(nx::dec::g_dec_stats), sizeof(unsigned long long) * 16) != hipSuccess) return -1;
    unsigned long long z[16] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(nx::dec::g_dec_stats), z, sizeof z) == hipSuccess ? 0 : -1;
}
'''
open(sys.argv[2], "w").write(s)

/* enc_chain_model.c — CPU model of a two-phase Snappy encoder, counting the
 * memory requests it would issue per chunk so that it can be priced against the measured rates
 * before any kernel is written.  Not product code.
 *
 * Snappy.encode (Snappy.java:82-165) keeps a 16 384-slot short[] table that every probe reads and
 * writes and every match end writes (table[hash(ip-1)], :148-150).  Written positions only increase
 * (probe positions increase; the two inserts after a match are matchEnd-1 and matchEnd, which the
 * next probes pass), so table[h] at a probe of position p is the LAST WRITTEN position q < p with
 * hash(q) == h (or 0 when there is none — the zeroed table).
 *
 *   phase A (wave-parallel, no decisions): prev[q] = the previous position with the same hash as q.
 *   phase B (lane-serial walker): at a probe of p, follow prev[] from p over positions that were
 *            never written until the first written one; that is table[hash(p)].  Written positions
 *            are marked in the entry array as the walker writes them.
 *
 * The walker runs the reference's greedy loop exactly (the table replaced by the chain walk), and the
 * program checks that both produce the same tag stream for every chunk.  It counts, per chunk:
 *   probes, inserts, matches — the reference's table requests (one read-modify-write each);
 *   hops     — chain steps over unwritten positions (each a dependent random load in phase B);
 *   hops_pc  — the same with path compression (a walked unwritten position is re-pointed at the
 *              written one found, so no later walk repeats it: one store per compressed hop).
 *
 *   cc -O2 -o enc_chain_model scripts/experiments/enc_chain_model.c -I include
 *   ./enc_chain_model [chunks] [stride]   (chunk indices 0, stride, 2*stride, ... of the bench corpus)
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "netty_amd_textgen.h"

#define HT 16384
#define SHIFT 18 /* numberOfLeadingZeros(16384) + 1 */

static inline uint32_t be32(const uint8_t* p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | (uint32_t)p[3];
}
static inline uint32_t hsh(const uint8_t* in, int32_t i) { return (be32(in + i) * 0x1e35a7bdu) >> SHIFT; }

static int32_t fml(const uint8_t* in, int32_t minIndex, int32_t inIndex, int32_t maxIndex) {
    int32_t matched = 0;
    while (inIndex <= maxIndex - 4 && be32(in + inIndex) == be32(in + minIndex + matched)) {
        inIndex += 4;
        matched += 4;
    }
    while (inIndex < maxIndex && in[minIndex + matched] == in[inIndex]) {
        ++inIndex;
        ++matched;
    }
    return matched;
}

/* tag stream: (literal start, literal length) and (copy offset, copy length) events */
typedef struct {
    int32_t a, b, kind;
} Ev;

typedef struct {
    uint64_t probes, inserts, matches, m7, hops, hops_pc, pc_stores, ext_steps;
} Census;

/* table-based reference (Snappy.java:104-158); mode 1 = chain walker instead of the table */
static int encode(const uint8_t* in, int32_t length, int mode, Ev* ev, Census* C) {
    static uint16_t table[HT];
    static int32_t prev[65536 + 8], link[65536 + 8];
    static uint8_t written[65536 + 8];
    int ne = 0;
    memset(table, 0, sizeof table);
    if (mode) {  /* phase A: prev[q] = previous position with the same hash (-1: none) */
        static int32_t last[HT];
        for (int i = 0; i < HT; ++i) last[i] = -1;
        for (int32_t q = 0; q + 4 <= length; ++q) {
            const uint32_t h = hsh(in, q);
            prev[q] = last[h];
            last[h] = q;
        }
        memcpy(link, prev, sizeof(int32_t) * (size_t)(length > 0 ? length : 1));
        memset(written, 0, (size_t)length + 8);
    }
    /* table[h] read at p: the last written position before p with that hash */
    #define READ_TABLE(p, h, out)                                                   \
        do {                                                                        \
            if (!mode) {                                                            \
                out = table[h];                                                     \
            } else {                                                                \
                int32_t q = prev[p], steps = 0;                                     \
                while (q >= 0 && !written[q]) { ++steps; q = prev[q]; }             \
                C->hops += (uint64_t)steps;                                         \
                /* path compression: the same walk over `link` */                   \
                int32_t r = link[p], s2 = 0, first = r;                             \
                while (r >= 0 && !written[r]) { ++s2; r = link[r]; }                \
                C->hops_pc += (uint64_t)s2;                                         \
                for (int32_t u = first; u >= 0 && !written[u];) {                   \
                    const int32_t nx = link[u];                                     \
                    if (nx != r) { link[u] = r; C->pc_stores++; }                   \
                    u = nx;                                                         \
                }                                                                   \
                out = q >= 0 ? (uint32_t)q : 0u;                                    \
            }                                                                       \
        } while (0)
    #define WRITE_TABLE(h, pos)                                                     \
        do {                                                                        \
            if (!mode) table[h] = (uint16_t)(pos); else written[pos] = 1;           \
        } while (0)
    int32_t inIndex = 0, nextEmit = 0;
    if (length >= 15) {
        uint32_t nextHash = hsh(in, ++inIndex);
        for (;;) {
            int32_t skip = 32, candidate, nextIndex = inIndex;
            do {
                inIndex = nextIndex;
                const uint32_t hash = nextHash;
                const int32_t bbl = skip++ >> 5;
                nextIndex = inIndex + bbl;
                if (nextIndex > length - 4) goto done;
                nextHash = hsh(in, nextIndex);
                uint32_t t;
                READ_TABLE(inIndex, hash, t);
                candidate = (int32_t)t;
                WRITE_TABLE(hash, inIndex);
                C->probes++;
            } while (be32(in + inIndex) != be32(in + candidate));
            ev[ne++] = (Ev){nextEmit, inIndex - nextEmit, 0};
            int32_t insertTail;
            do {
                const int32_t base = inIndex;
                const int32_t matched = 4 + fml(in, candidate + 4, inIndex + 4, length);
                C->matches++;
                C->m7 += matched >= 7;
                C->ext_steps += (uint64_t)((matched - 4 + 7) / 8);
                inIndex += matched;
                ev[ne++] = (Ev){base - candidate, matched, 1};
                insertTail = inIndex - 1;
                nextEmit = inIndex;
                if (inIndex >= length - 4) goto done;
                const uint32_t prevHash = hsh(in, insertTail);
                WRITE_TABLE(prevHash, inIndex - 1);
                const uint32_t currentHash = hsh(in, insertTail + 1);
                uint32_t t;
                READ_TABLE(inIndex, currentHash, t);
                candidate = (int32_t)t;
                WRITE_TABLE(currentHash, inIndex);
                C->probes++;
                C->inserts++;
            } while (be32(in + insertTail + 1) == be32(in + candidate));
            nextHash = hsh(in, insertTail + 2);
            ++inIndex;
        }
    }
done:
    if (nextEmit < length) ev[ne++] = (Ev){nextEmit, length - nextEmit, 0};
    return ne;
}

/* the events as Snappy.encode writes them (encodeLiteral :268-281, encodeCopy :283-313), after the
 * preamble; for the byte-level check against the oracle (tests/test_encoder_chain_model.py) */
static size_t emit(const uint8_t* in, int32_t length, const Ev* ev, int ne, uint8_t* out) {
    size_t op = 0;
    for (int i = 0;; ++i) {
        const uint32_t b = (uint32_t)length >> (i * 7);
        if (b & 0xFFFFFF80u) out[op++] = (uint8_t)((b & 0x7f) | 0x80);
        else { out[op++] = (uint8_t)b; break; }
    }
    for (int k = 0; k < ne; ++k) {
        if (ev[k].kind == 0) {
            const int32_t len = ev[k].b;
            if (len <= 0) continue;
            if (len < 61) {
                out[op++] = (uint8_t)((len - 1) << 2);
            } else {
                int bl = 0;
                for (uint32_t v = (uint32_t)(len - 1); v > 1; v >>= 1) ++bl;  /* bitsToEncode */
                const int nb = 1 + bl / 8;
                out[op++] = (uint8_t)((59 + nb) << 2);
                for (int i = 0; i < nb; ++i) out[op++] = (uint8_t)(((len - 1) >> (i * 8)) & 0xff);
            }
            memcpy(out + op, in + ev[k].a, (size_t)len);
            op += (size_t)len;
        } else {
            const int32_t off = ev[k].a;
            int32_t len = ev[k].b;
            #define COPY1(L)                                                                               \
                do {                                                                                       \
                    if ((L) < 12 && off < 2048) {                                                          \
                        out[op++] = (uint8_t)(1 | (((L) - 4) << 2) | ((off >> 8) << 5));                   \
                        out[op++] = (uint8_t)(off & 0xff);                                                 \
                    } else {                                                                               \
                        out[op++] = (uint8_t)(2 | (((L) - 1) << 2));                                       \
                        out[op++] = (uint8_t)(off & 0xff);                                                 \
                        out[op++] = (uint8_t)((off >> 8) & 0xff);                                          \
                    }                                                                                      \
                } while (0)
            while (len >= 68) { COPY1(64); len -= 64; }
            if (len > 64) { COPY1(60); len -= 60; }
            COPY1(len);
        }
    }
    return op;
}

#ifdef WITH_ORACLE
#include "../../oracle/netty_oracle.h"
#endif

int main(int argc, char** argv) {
    const int chunks = argc > 1 ? atoi(argv[1]) : 48;
    const uint64_t stride = argc > 2 ? strtoull(argv[2], NULL, 10) : 34133; /* spread over 1 638 400 */
    static nx_textgen_tables tg;
    nx_textgen_build(&tg);
    static uint8_t buf[65536 + 16];
    static Ev e0[70000], e1[70000];
    Census T0 = {0}, T1 = {0};
    int bad = 0;
    for (int c = 0; c < chunks; ++c) {
        nx_tg_chunk(&tg, (uint64_t)c * stride, buf, 65536);
        Census C0 = {0}, C1 = {0};
        const int n0 = encode(buf, 65536, 0, e0, &C0);
        const int n1 = encode(buf, 65536, 1, e1, &C1);
        if (n0 != n1 || memcmp(e0, e1, sizeof(Ev) * (size_t)n0) != 0) ++bad;
#ifdef WITH_ORACLE
        {  /* byte-level: the chain walker's output equals the oracle's Snappy.encode */
            static uint8_t a[80000], o[80000];
            const size_t na = emit(buf, 65536, e1, n1, a);
            const size_t no = orc_snappy_encode(buf, 65536, o);
            if (na != no || memcmp(a, o, na) != 0) ++bad;
        }
#endif
        T0.probes += C0.probes; T0.inserts += C0.inserts; T0.matches += C0.matches; T0.m7 += C0.m7; T0.ext_steps += C0.ext_steps;
        T1.hops += C1.hops; T1.hops_pc += C1.hops_pc; T1.pc_stores += C1.pc_stores;
    }
    const double n = chunks;
    printf("{\"chunks\": %d, \"stride\": %llu, \"tag_streams_identical\": %s,\n", chunks, (unsigned long long)stride, bad ? "false" : "true");
    printf(" \"per_chunk\": {\"probes\": %.1f, \"inserts\": %.1f, \"matches\": %.1f, \"matches_7plus\": %.1f, \"extension_steps_8B\": %.1f,\n",
           T0.probes / n, T0.inserts / n, T0.matches / n, T0.m7 / n, T0.ext_steps / n);
    printf("  \"chain_hops\": %.1f, \"chain_hops_path_compressed\": %.1f, \"path_compression_stores\": %.1f,\n", T1.hops / n,
           T1.hops_pc / n, T1.pc_stores / n);
    printf("  \"hops_per_probe\": %.3f, \"hops_per_probe_pc\": %.3f}}\n", (double)T1.hops / T0.probes, (double)T1.hops_pc / T0.probes);
    return bad ? 1 : 0;
}

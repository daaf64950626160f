/*
 * netty_amd_textgen.h — the synthetic "text-like" chunk generator named by BASELINE.json
 * configs 2/3/5: a 4096-word pseudo-English vocabulary (2–10 letters drawn
 * from an English letter-frequency table), Zipf(s = 1.1) word ranks, separators ' ' (90 %)
 * and ". " (10 %), chunk i seeded with 0x5EED ^ i.
 *
 * Header-only so that the host (oracle, CPU baseline) and the device generator
 * (netty_amd/csrc/textgen.hip) produce byte-identical chunks.  All per-chunk arithmetic is
 * integer; the only floating point is the one-time Zipf CDF build on the host.
 */
#ifndef NETTY_AMD_TEXTGEN_H
#define NETTY_AMD_TEXTGEN_H
#include <stdint.h>
#include <stddef.h>

#if defined(__HIPCC__)
#define NX_TG_HD __host__ __device__ inline
#else
#define NX_TG_HD static inline
#endif

#define NX_TG_WORDS 4096u
#define NX_TG_MAX_WORD 10u
#define NX_TG_SEED_XOR 0x5EEDull

typedef struct {
    uint32_t cdf[NX_TG_WORDS];             /* cdf[k] = floor(2^32 * P(rank <= k)), last = 0xFFFFFFFF */
    uint32_t off[NX_TG_WORDS + 1];         /* word k = chars[off[k] .. off[k+1]) */
    uint8_t chars[NX_TG_WORDS * NX_TG_MAX_WORD];
} nx_textgen_tables;

NX_TG_HD uint64_t nx_tg_splitmix(uint64_t* s) {
    uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

/* Returns the number of bytes of the word+separator written (bounded by cap). */
NX_TG_HD uint32_t nx_tg_pick(const uint32_t* cdf, uint32_t u) {
    uint32_t lo = 0, hi = NX_TG_WORDS - 1; /* first k with cdf[k] > u (cdf[last] = ~0 > any u < ~0) */
    while (lo < hi) {
        uint32_t mid = (lo + hi) >> 1;
        if (cdf[mid] > u) hi = mid; else lo = mid + 1;
    }
    return lo;
}

/* Generate chunk `idx` of n bytes into out (byte-at-a-time reference form). */
NX_TG_HD void nx_tg_chunk(const nx_textgen_tables* t, uint64_t idx, uint8_t* out, size_t n) {
    uint64_t s = NX_TG_SEED_XOR ^ idx;
    size_t pos = 0;
    while (pos < n) {
        uint64_t r = nx_tg_splitmix(&s);
        uint32_t w = nx_tg_pick(t->cdf, (uint32_t)(r >> 32));
        for (uint32_t c = t->off[w]; c < t->off[w + 1] && pos < n; ++c) out[pos++] = t->chars[c];
        if (((uint32_t)(r & 0xFFFFu)) % 10u == 0u) {
            if (pos < n) out[pos++] = '.';
        }
        if (pos < n) out[pos++] = ' ';
    }
}

#include <math.h>
/* Build the vocabulary + Zipf CDF (host only, deterministic). */
static inline void nx_textgen_build(nx_textgen_tables* t) {
    /* English letter frequencies (per mille), a..z */
    static const uint16_t freq[26] = {82, 15, 28, 43, 127, 22, 20, 61, 70, 2, 8, 40, 24,
                                      67, 75, 19, 1, 60, 63, 91, 28, 10, 24, 2, 20, 1};
    uint32_t cum[26], tot = 0;
    for (int i = 0; i < 26; ++i) { tot += freq[i]; cum[i] = tot; }
    uint64_t s = 0x70CAB0ull;
    uint32_t o = 0;
    for (uint32_t k = 0; k < NX_TG_WORDS; ++k) {
        t->off[k] = o;
        uint32_t len = 2u + (uint32_t)(nx_tg_splitmix(&s) % 9u);
        for (uint32_t j = 0; j < len; ++j) {
            uint32_t r = (uint32_t)(nx_tg_splitmix(&s) % tot);
            int c = 0;
            while (cum[c] <= r) ++c;
            t->chars[o++] = (uint8_t)('a' + c);
        }
    }
    t->off[NX_TG_WORDS] = o;
    double total = 0.0;
    for (uint32_t k = 1; k <= NX_TG_WORDS; ++k) total += pow((double)k, -1.1);
    double acc = 0.0;
    for (uint32_t k = 1; k <= NX_TG_WORDS; ++k) {
        acc += pow((double)k, -1.1);
        double v = acc / total * 4294967296.0;
        t->cdf[k - 1] = v >= 4294967295.0 ? 0xFFFFFFFFu : (uint32_t)v;
    }
    t->cdf[NX_TG_WORDS - 1] = 0xFFFFFFFFu;
}

#endif

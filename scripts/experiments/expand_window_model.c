// C model of k_window (snappy_decode.hip) for ONE half-wave (32 lanes = one frame): lanes hold
// records (a cursor per lane), up to two aligned output qwords per lane per round; literal and far-copy
// bytes fetched at admission / after each step (usable the next round, aligned to the destination
// qwords); ring-reading copies wait on a done-bitmap (set when written, cleared when the block is
// flushed; sources below the frontier F are final).  Verifies bytes against a serial decode.
// Usage: FR=frames.bin ./model  (frames.bin: [u32 len][snappy block] records)
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <stdint.h>

typedef struct { uint32_t rec, ost; } Rin;
static int parse(const uint8_t* in, uint32_t n, uint32_t* rec, uint8_t* out, uint32_t* olen) {
    uint32_t ip = 0;
    while (1) { uint32_t c = in[ip++]; if (!(c & 0x80)) break; }
    uint32_t op = 0; int nr = 0;
    while (ip < n) {
        uint32_t tag = in[ip++], t = tag & 3;
        if (t == 0) {
            uint32_t l = tag >> 2;
            if (l >= 60) { uint32_t nb = l - 59; l = 0; for (uint32_t k = 0; k < nb; ++k) l |= in[ip + k] << (8 * k); ip += nb; }
            l += 1;
            for (uint32_t k = 0; k < l; k += 64) { uint32_t m = l - k < 64 ? l - k : 64; rec[nr++] = ((m - 1) << 25) | (ip + k); }
            memcpy(out + op, in + ip, l); ip += l; op += l;
        } else {
            uint32_t l, off;
            if (t == 1) { l = 4 + ((tag >> 2) & 7); off = ((tag & 0xe0) << 3) | in[ip]; ip += 1; }
            else if (t == 2) { l = 1 + (tag >> 2); off = in[ip] | (in[ip + 1] << 8); ip += 2; }
            else { l = 1 + (tag >> 2); off = in[ip] | (in[ip + 1] << 8) | (in[ip + 2] << 16) | ((uint32_t)in[ip + 3] << 24); ip += 4; }
            rec[nr++] = 0x80000000u | ((l - 1) << 25) | off;
            for (uint32_t k = 0; k < l; ++k) out[op + k] = out[op + k - off];
            op += l;
        }
    }
    *olen = op; return nr;
}

#define NL 32
#define R 4096u
#define H 2048u
#define MULTI 2
static long st_rounds, st_modular, st_slow;

static uint64_t ld_qw(const uint8_t* p) { uint64_t v; memcpy(&v, p, 8); return v; }

int expand(const uint8_t* in, uint32_t in_len, const uint32_t* recs, uint32_t N, uint32_t Ofin, uint8_t* gout) {
    uint64_t ring[R / 8]; static uint32_t holds[R]; for (uint32_t z = 0; z < R; ++z) holds[z] = 0xFFFFFFFF;
    uint32_t bits[R / 32];
    memset(ring, 0xCD, sizeof ring);
    memset(bits, 0, sizeof bits);
    // lane state
    int has[NL], mid[NL]; uint32_t s[NL], e[NL], x[NL], cp[NL], cur[NL], elig[NL]; uint64_t D0[NL], D1[NL];
    memset(has, 0, sizeof has);
    // batch registers: B0/B1 hold 32 records with ostart; next = index within B0 of the next unadmitted
    uint32_t B0r[NL], B0s[NL], B1r[NL], B1s[NL];
    uint32_t bbase = 0;  // record index of B0[0]
    uint32_t obase = 0;  // ostart after B1's last
    uint32_t next = 0;
    // load B0, B1
    for (int b = 0; b < 2; ++b) {
        uint32_t* Rr = b ? B1r : B0r; uint32_t* Rs = b ? B1s : B0s;
        uint32_t acc = obase;
        for (int t = 0; t < NL; ++t) {
            uint32_t i = b * NL + t;
            uint32_t r = i < N ? recs[i] : 0; uint32_t len = i < N ? ((r >> 25) & 63) + 1 : 0;
            Rr[t] = r; Rs[t] = acc; acc += len;
        }
        obase = acc;
    }
    uint32_t F = 0, flushed = 0;
    for (int guard = 0;; ++guard) {
        if (guard > 2000000) return -2;
        // ---- admission
        uint32_t rank = 0;
        for (int t = 0; t < NL; ++t) {
            if (has[t]) continue;
            uint32_t k = next + rank;
            uint32_t ri = bbase + k;
            if (ri >= N) continue;
            uint32_t r = k < NL ? B0r[k] : B1r[k - NL];
            uint32_t os = k < NL ? B0s[k] : B1s[k - NL];
            if (k >= 2 * NL) continue;  // beyond the loaded batches
            uint32_t len = ((r >> 25) & 63) + 1;
            if (os + len > F + H) continue;  // horizon (monotone in k)
            rank++;
            has[t] = 1; s[t] = os; e[t] = os + len; cur[t] = os; cp[t] = r >> 31; x[t] = r & 0x1FFFFFF;
            elig[t] = 1;
            int far = cp[t] && x[t] > R - H && (os - x[t]) + len <= flushed;
            mid[t] = cp[t] && x[t] > R - H && !far;
            if (!cp[t] || far) {
                cp[t] = cp[t] ? 2 : 0;
                // 16 bytes aligned to the destination qword of cur
                uint32_t d = os & 7;
                int64_t a = cp[t] ? (int64_t)(os - x[t]) - d : (int64_t)x[t] - d;
                const uint8_t* base = cp[t] ? gout : in;
                uint8_t tmp[16] = {0};
                for (int j = 0; j < 16; ++j) { int64_t p = a + j; if (p >= 0 && (cp[t] ? p < (int64_t)flushed : p < (int64_t)in_len)) tmp[j] = base[p]; }
                if (cp[t] && a + 16 > (int64_t)flushed && (int64_t)(os - x[t]) + (e[t] - os < 16 - d ? e[t] - os : 16 - d) > (int64_t)flushed) { fprintf(stderr, "far unflushed\n"); return -3; }
                memcpy(&D0[t], tmp, 8); memcpy(&D1[t], tmp + 8, 8);
                elig[t] = 0;
            }
        }
        next += rank;
        if (next >= NL) {  // B0 exhausted: shift, load the next batch
            memcpy(B0r, B1r, sizeof B0r); memcpy(B0s, B1s, sizeof B0s);
            bbase += NL; next -= NL;
            uint32_t acc = obase;
            for (int t = 0; t < NL; ++t) {
                uint32_t i = bbase + NL + t;
                uint32_t r = i < N ? recs[i] : 0; uint32_t len = i < N ? ((r >> 25) & 63) + 1 : 0;
                B1r[t] = r; B1s[t] = acc; acc += len;
            }
            obase = acc;
        }
        int any = 0; for (int t = 0; t < NL; ++t) any |= has[t];
        if (!any && bbase + next >= N) break;
        // ---- process (two-phase: all reads of a piece before its write, lanes in any order is fine
        //      because readiness excludes sources written this round by other lanes)
        uint64_t wval[NL][MULTI], wmask[NL][MULTI]; uint32_t wq[NL][MULTI]; int nw[NL];
        uint32_t ncur[NL];
        memset(nw, 0, sizeof nw);
        for (int t = 0; t < NL; ++t) {
            ncur[t] = cur[t];
            if (!has[t]) continue;
            if (!elig[t]) { elig[t] = 1; continue; }
            uint32_t c = cur[t];
            for (int m = 0; m < MULTI && c < e[t]; ++m) {
                uint32_t q = c >> 3, lo = c & 7, hi = (q * 8 + 8 < e[t] ? 8 : e[t] - q * 8);
                uint64_t mask = (hi == 8 ? ~0ull : ((1ull << (8 * hi)) - 1)) & ~((1ull << (8 * lo)) - 1);
                uint64_t v;
                if (cp[t] != 1) {  // literal / far: prefetched data (m-th qword of the 16 bytes loaded for cur's qword)
                    v = m == 0 ? D0[t] : D1[t];
                } else {
                    uint32_t off = x[t];
                    if (off < hi - lo) {  // modular: the piece reads its own output
                        // period [s - off, s) must be done
                        int ok = 1;
                        for (uint32_t b = s[t] - off; b < s[t]; ++b) if (b >= F && !((bits[(b % R) >> 5] >> (b & 31)) & 1)) ok = 0;
                        if (!ok) break;
                        uint8_t tmp[8] = {0};
                        for (uint32_t j = lo; j < hi; ++j) { uint32_t p = q * 8 + j; uint32_t sp = s[t] - off + ((p - s[t]) % off); tmp[j] = ((const uint8_t*)ring)[sp % R]; }
                        memcpy(&v, tmp, 8); st_modular++;
                    } else {
                        // source bytes [c - off, q*8+hi - off); those at or above cur (this round's own pieces) are fine
                        uint32_t a0 = c - off, a1 = q * 8 + hi - off;
                        if (a1 > cur[t]) a1 = cur[t];  // own earlier pieces this round
                        int ok = 1;
                        for (uint32_t b = a0 < F ? F : a0; b < a1; ++b) if (!((bits[(b % R) >> 5] >> (b & 31)) & 1)) ok = 0;
                        if (!ok) break;
                        // 8 bytes aligned to the destination qword: ring bytes at q*8 - off
                        uint8_t tmp[8];
                        for (int j = 0; j < 8; ++j) tmp[j] = ((const uint8_t*)ring)[(q * 8 - off + j) % R];
                        for (uint32_t j = lo; j < hi; ++j) { uint32_t p = q * 8 + j - off; if (p < cur[t] && holds[p % R] != p) { fprintf(stderr, "ring overwritten: pos %u holds %u\n", p, holds[p % R]); exit(3); } }
                        // own earlier piece written this round: model the in-order LDS (apply pending writes of this lane)
                        for (int w = 0; w < nw[t]; ++w)
                            for (int j = 0; j < 8; ++j) {
                                uint32_t p = (q * 8 - off + j);
                                if ((p >> 3) == wq[t][w] && ((wmask[t][w] >> (8 * (p & 7))) & 0xFF)) tmp[j] = (uint8_t)(wval[t][w] >> (8 * (p & 7)));
                            }
                        memcpy(&v, tmp, 8);
                    }
                }
                wval[t][nw[t]] = v; wmask[t][nw[t]] = mask; wq[t][nw[t]] = q; nw[t]++;
                c = q * 8 + hi;
            }
            ncur[t] = c;
        }
        // writes + done bits
        for (int t = 0; t < NL; ++t) {
            for (int w = 0; w < nw[t]; ++w) {
                uint32_t qi = wq[t][w] % (R / 8);
                ring[qi] = (ring[qi] & ~wmask[t][w]) | (wval[t][w] & wmask[t][w]);
                for (int j = 0; j < 8; ++j) if ((wmask[t][w] >> (8 * j)) & 0xFF) holds[(wq[t][w] * 8 + j) % R] = wq[t][w] * 8 + j;
                for (int j = 0; j < 8; ++j) if ((wmask[t][w] >> (8 * j)) & 0xFF) { uint32_t p = wq[t][w] * 8 + j; bits[(p % R) >> 5] |= 1u << (p & 31); }
            }
            if (!has[t]) continue;
            cur[t] = ncur[t];
            if (cur[t] >= e[t]) { has[t] = 0; continue; }
            if (nw[t] && cp[t] != 1) {  // literal / far: fetch the next 16 bytes (usable next round)
                uint32_t d = cur[t] & 7;
                int64_t a = cp[t] ? (int64_t)(cur[t] - x[t]) - d : (int64_t)x[t] + (cur[t] - s[t]) - d;
                const uint8_t* base = cp[t] ? gout : in;
                uint8_t tmp[16] = {0};
                for (int j = 0; j < 16; ++j) { int64_t p = a + j; if (p >= 0 && (cp[t] ? p < (int64_t)flushed : p < (int64_t)in_len)) tmp[j] = base[p]; }
                memcpy(&D0[t], tmp, 8); memcpy(&D1[t], tmp + 8, 8);
                elig[t] = 0;
            }
        }
        st_rounds++;
        // frontier
        F = bbase + next < N ? (next < NL ? B0s[next] : B1s[next - NL]) : Ofin;
        for (int t = 0; t < NL; ++t) if (has[t] && cur[t] < F) F = cur[t];
        for (int t = 0; t < NL; ++t) if (has[t] && mid[t] && cur[t] - x[t] + (R - H) < F) F = cur[t] - x[t] + (R - H);
        // flush whole blocks below F, clearing their done bits
        while (flushed + 512 <= F) {
            for (int j = 0; j < 512; ++j) gout[flushed + j] = ((const uint8_t*)ring)[(flushed + j) % R];
            for (int j = 0; j < 16; ++j) bits[((flushed % R) >> 5) + j] = 0;
            flushed += 512;
        }
    }
    for (uint32_t j = flushed; j < Ofin; ++j) gout[j] = ((const uint8_t*)ring)[j % R];
    return 0;
}

int main(void) {
    FILE* f = fopen(getenv("FR") ? getenv("FR") : "frames.bin", "rb");
    static uint8_t buf[1 << 17], ref[1 << 17], got[1 << 17];
    static uint32_t rec[70000];
    int nf = 0, bad = 0;
    for (;;) {
        uint32_t n;
        if (fread(&n, 4, 1, f) != 1) break;
        if (fread(buf, 1, n, f) != n) break;
        uint32_t olen; int nr = parse(buf, n, rec, ref, &olen);
        memset(got, 0, sizeof got);
        int rc = expand(buf, n, rec, nr, olen, got);
        if (rc != 0 || memcmp(got, ref, olen) != 0) { bad++; fprintf(stderr, "frame %d rc %d\n", nf, rc); }
        nf++;
    }
    // periodic inputs (overlapping copies) through the same path
    printf("frames %d bad %d rounds/frame %.0f modular %.1f\n", nf, bad, (double)st_rounds / nf, (double)st_modular / nf);
    return bad != 0;
}

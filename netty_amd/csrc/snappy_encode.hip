// snappy_encode.hip — Snappy block encoder, bit-exact with Netty's Snappy.encode (Snappy.java:82-313).
//
// Netty's greedy matcher is a serial state machine whose output depends on the exact probe order
// (the `skip++ >> 5` heuristic, :107-115) and on an evolving 16384-entry hash table (:97-100,
// 126-128, 148-152).  There is no safe intra-chunk speculation, so each chunk is one lane's serial
// state machine and the parallelism is the thousands of independent chunks of a batch (20 waves
// per CU → 327 680 chunks in flight on 256 CUs).  What the kernel optimises is the memory side of
// each lane's dependency chain:
//   * every 4-byte window is one unaligned dword load (Java's big-endian getInt = bswap), and the
//     bytes at the probe position are reused from the hash computation that loaded them;
//   * the next probe's table load is issued before the current candidate compare resolves
//     (a same-hash collision is forwarded in registers), so a probe costs one memory round trip;
//   * match extension compares 4 bytes per step and finds the first mismatch with ctz;
//   * output bytes are packed into dwords and written with aligned 4-byte stores; literal runs
//     are copied 4 bytes at a time with a funnel shift.
// Small batches take two latency forms of the same matcher (nx_snappy_encode_batch picks by batch
// size): up to one chunk per CU, a workgroup per chunk with the table and the chunk in LDS; up to
// kSpreadMaxChunks, one chunk per wave (lane 0), so no wave serialises 64 divergent matchers.
// Hash table: Java allocates a zeroed short[min(nextPow2(len),16384)] per call (:97-99,191).
// HBM forms (encode_chunk_w): each resident lane owns a 16384-entry uint64 slot in a device
// workspace; an entry is
//   stamp[63:58] | next3[57:34] | resid << pbits | position
// where resid (the low `shift` bits of the hash product) fixes the 4-byte word at `position` with
// the slot, and next3 holds the 3 bytes after it: the candidate compare and matches of 4-6 bytes
// need no read of the candidate's input bytes.  A stamp mismatch reads as position 0 — exactly a
// freshly zeroed table, without a clear per chunk.  The LDS form (encode_chunk) keeps 32-bit
// entries stamp[31:28] | check[27:16] | position[15:0] (its table must fit LDS with the chunk).
// The candidate position — and with it the emitted stream — is Java's in every form; only the
// memory traffic differs.
#include <stdlib.h>
#include <algorithm>
#include <mutex>
#include <vector>
#include "nx_common.hpp"
#include "workspace.hpp"

namespace nx {
namespace enc {

typedef uint32_t __attribute__((aligned(1))) u32u;

typedef uint64_t __attribute__((aligned(1))) u64u;

__device__ __forceinline__ uint32_t ld32(const uint8_t* p) { return *reinterpret_cast<const u32u*>(p); }  // LE, unaligned
__device__ __forceinline__ uint64_t ld64(const uint8_t* p) { return *reinterpret_cast<const u64u*>(p); }
__device__ __forceinline__ uint32_t hash_of(uint32_t le, int shift) {
    return (__builtin_bswap32(le) * 0x1e35a7bdu) >> shift;  // hash (:177-179) on the BIG-endian getInt
}

// Output writer: bytes are packed into `acc` and leave as aligned dword stores; with PAIR (8-byte
// aligned destination) two dwords leave as one 8-byte store.
template <bool PAIR>
struct WriterT {
    uint32_t* w;   // next aligned dword to store
    uint32_t acc;  // pending bytes (little-endian order)
    uint32_t na;   // number of pending bytes (0..3)
    uint32_t nw;   // dwords stored
    uint32_t s0;   // PAIR: the staged even dword
    __device__ __forceinline__ void emit(uint32_t v) {
        if (!PAIR) {
            w[nw] = v;
        } else if (nw & 1u) {
            *reinterpret_cast<uint2*>(w + nw - 1u) = make_uint2(s0, v);
        } else {
            s0 = v;
        }
        ++nw;
    }
    __device__ __forceinline__ void put(uint32_t b) {
        acc |= b << (8 * na);
        if (++na == 4) {
            emit(acc);
            acc = 0;
            na = 0;
        }
    }
    // append `n` bytes starting at p (unaligned source)
    __device__ __forceinline__ void copy(const uint8_t* p, int32_t n) {
        while (n >= 4) {
            const uint32_t v = ld32(p);
            if (na == 0) {
                emit(v);
            } else {
                emit(acc | (v << (8 * na)));
                acc = v >> (32 - 8 * na);
            }
            p += 4;
            n -= 4;
        }
        while (n-- > 0) put(*p++);
    }
    __device__ __forceinline__ uint32_t pos() const { return nw * 4 + na; }
    __device__ __forceinline__ void finish() {
        if (PAIR && (nw & 1u)) w[nw - 1u] = s0;
        uint8_t* t = reinterpret_cast<uint8_t*>(w + nw);
        for (uint32_t i = 0; i < na; ++i) t[i] = (uint8_t)(acc >> (8 * i));
    }
};

// LDS-staged writer (dense form): a lane's output dwords gather in its own LDS stage of SD dwords
// (SD*4-byte aligned units of the destination) and leave as whole units of 16-byte stores, so the L2
// receives full-line writes it needs no read-for-merge nor repeated partial write-backs for; the
// first unit (the destination need not be unit-aligned) and the tail are stored dword by dword.
template <int SD>
struct WriterL {
    uint32_t* st;   // this lane's LDS stage
    uint32_t* dst;  // output dword 0 (4-byte aligned)
    uint32_t acc;   // pending bytes (little-endian order)
    uint32_t na;    // number of pending bytes (0..3)
    uint32_t nw;    // dwords emitted
    uint32_t s;     // stage slot of the next dword = (dword address) mod SD
    uint32_t lo;    // first valid slot of the current unit (nonzero only for the first unit)
    __device__ __forceinline__ WriterL(uint32_t* stage, uint8_t* o)
        : st(stage), dst(reinterpret_cast<uint32_t*>(o)), acc(0), na(0), nw(0) {
        s = (uint32_t)(((uintptr_t)o >> 2) & (SD - 1));
        lo = s;
    }
    __device__ __forceinline__ void emit(uint32_t v) {
        st[s] = v;
        ++nw;
        if (s == SD - 1) {
            uint32_t* g = dst + nw - SD;  // the unit's slot 0
            if (lo == 0) {
#pragma unroll
                for (int q = 0; q < SD / 4; ++q)
                    reinterpret_cast<uint4*>(g)[q] = make_uint4(st[4 * q], st[4 * q + 1], st[4 * q + 2], st[4 * q + 3]);
            } else {
                for (uint32_t j = lo; j < SD; ++j) g[j] = st[j];
                lo = 0;
            }
            s = 0;
        } else {
            ++s;
        }
    }
    __device__ __forceinline__ void put(uint32_t b) {
        acc |= b << (8 * na);
        if (++na == 4) {
            emit(acc);
            acc = 0;
            na = 0;
        }
    }
    __device__ __forceinline__ void copy(const uint8_t* p, int32_t n) {
        while (n >= 4) {
            const uint32_t v = ld32(p);
            if (na == 0) {
                emit(v);
            } else {
                emit(acc | (v << (8 * na)));
                acc = v >> (32 - 8 * na);
            }
            p += 4;
            n -= 4;
        }
        while (n-- > 0) put(*p++);
    }
    __device__ __forceinline__ uint32_t pos() const { return nw * 4 + na; }
    __device__ __forceinline__ void finish() {
        uint32_t* g = dst + nw - s;  // slot 0 of the open unit
        for (uint32_t j = lo; j < s; ++j) g[j] = st[j];
        uint8_t* t = reinterpret_cast<uint8_t*>(dst + nw);
        for (uint32_t i = 0; i < na; ++i) t[i] = (uint8_t)(acc >> (8 * i));
    }
};

// Byte-store writer for unaligned destinations (same interface).
struct ByteWriter {
    uint8_t* o;
    uint32_t n;
    __device__ __forceinline__ void put(uint32_t b) { o[n++] = (uint8_t)b; }
    __device__ __forceinline__ void copy(const uint8_t* p, int32_t k) {
        for (int32_t i = 0; i < k; ++i) o[n + i] = p[i];
        n += (uint32_t)k;
    }
    __device__ __forceinline__ uint32_t pos() const { return n; }
    __device__ __forceinline__ void finish() {}
};

template <class Wr>
__device__ __forceinline__ void enc_literal(const uint8_t* in, Wr& w, int32_t length) {
    // encodeLiteral (:268-281)
    if (length < 61) {
        w.put((uint32_t)((length - 1) << 2));
    } else {
        const int32_t v = length - 1;
        const int bitLength = 31 - __clz((uint32_t)v);  // bitsToEncode (:249-257), v >= 60
        const int bytesToEncode = 1 + bitLength / 8;
        w.put((uint32_t)((59 + bytesToEncode) << 2));
        for (int i = 0; i < bytesToEncode; i++) w.put((uint32_t)((v >> (i * 8)) & 0xff));
    }
    w.copy(in, length);
}

template <class Wr>
__device__ __forceinline__ void enc_copy_off(Wr& w, int32_t offset, int32_t length) {
    // encodeCopyWithOffset (:283-292)
    if (length < 12 && offset < 2048) {
        w.put((uint32_t)(1 | ((length - 4) << 2) | ((offset >> 8) << 5)));
        w.put((uint32_t)(offset & 0xff));
    } else {
        w.put((uint32_t)(2 | ((length - 1) << 2)));
        w.put((uint32_t)(offset & 0xff));
        w.put((uint32_t)((offset >> 8) & 0xff));
    }
}

template <class Wr>
__device__ __forceinline__ void enc_copy(Wr& w, int32_t offset, int32_t length) {
    // encodeCopy (:301-313)
    while (length >= 68) {
        enc_copy_off(w, offset, 64);
        length -= 64;
    }
    if (length > 64) {
        enc_copy_off(w, offset, 60);
        length -= 60;
    }
    enc_copy_off(w, offset, length);
}

// Register window over the lane's own input stream: 32 bytes from a 16-byte-aligned address, plus
// the following 16-byte block prefetched one slide ahead.
// The scan front moves 1-2 bytes per probe, so one refill (two 16-byte loads) serves the next
// 10-25 stream reads that would otherwise each be a separate memory request; with 262 144 lanes
// streaming at once, L2 cannot keep a lane's current line between its probes.  Dword i of the
// window is picked by a 3-level select tree (dynamic register indexing would spill to scratch).
// A 16-byte block that holds at least one byte of the chunk never crosses a page, so the loads
// stay inside mapped memory; a second block wholly past the end is not loaded.
struct StreamWin {
    const uint8_t* origin;  // chunk start rounded down to 16 bytes
    uint32_t pad;           // chunk start - origin
    uint32_t end;           // chunk end, origin-relative
    uint32_t wb;            // window base, origin-relative, multiple of 16
    uint32_t w0, w1, w2, w3, w4, w5, w6, w7;
    uint32_t f0, f1, f2, f3;  // the block after the window (wb + 32), loaded one slide ahead
    __device__ __forceinline__ void init(const uint8_t* in, int32_t length) {
        pad = (uint32_t)((uintptr_t)in & 15u);
        origin = in - pad;  // pointer arithmetic, not an integer cast: keeps an LDS chunk's address space
        end = pad + (uint32_t)length;
        wb = 0x80000000u;  // empty: q - wb > 27 for every position
    }
    __device__ __forceinline__ static uint32_t sel(uint32_t i, uint32_t a0, uint32_t a1, uint32_t a2, uint32_t a3, uint32_t a4,
                                                   uint32_t a5, uint32_t a6, uint32_t a7) {
        const bool b0 = i & 1u, b1 = i & 2u, b2 = i & 4u;
        const uint32_t c0 = b0 ? a1 : a0, c1 = b0 ? a3 : a2, c2 = b0 ? a5 : a4, c3 = b0 ? a7 : a6;
        const uint32_t d0 = b1 ? c1 : c0, d1 = b1 ? c3 : c2;
        return b2 ? d1 : d0;
    }
    // the 4 bytes at chunk position p (p + 4 <= length), little-endian
    __device__ __forceinline__ uint32_t get(int32_t p) {
        const uint32_t q = (uint32_t)p + pad;
        uint32_t off = q - wb;
        if (off > 27u) {
            if (off < 44u) {
                // forward by less than 16 bytes past the window: slide it one block, keeping the
                // upper block, so each input block is loaded once on a forward scan; the new upper
                // block was prefetched at the previous slide (its load is off the dependent chain),
                // and the block after it is prefetched now
                wb += 16u;
                w0 = w4; w1 = w5; w2 = w6; w3 = w7;
                w4 = f0; w5 = f1; w6 = f2; w7 = f3;
                if (wb + 32u < end) {
                    const uint4 z = *reinterpret_cast<const uint4*>(origin + wb + 32u);
                    f0 = z.x; f1 = z.y; f2 = z.z; f3 = z.w;
                }
            } else {
                wb = q & ~15u;
                const uint4 x = *reinterpret_cast<const uint4*>(origin + wb);
                w0 = x.x; w1 = x.y; w2 = x.z; w3 = x.w;
                if (wb + 16u < end) {
                    const uint4 y = *reinterpret_cast<const uint4*>(origin + wb + 16u);
                    w4 = y.x; w5 = y.y; w6 = y.z; w7 = y.w;
                }
                if (wb + 32u < end) {
                    const uint4 z = *reinterpret_cast<const uint4*>(origin + wb + 32u);
                    f0 = z.x; f1 = z.y; f2 = z.z; f3 = z.w;
                }
            }
            off = q - wb;
        }
        const uint32_t i = off >> 2;
        const uint32_t lo = sel(i, w0, w1, w2, w3, w4, w5, w6, w7);
        const uint32_t hi = sel(i + 1u, w0, w1, w2, w3, w4, w5, w6, w7);
        return __builtin_amdgcn_alignbyte(hi, lo, off & 3u);
    }
};

// The 8 bytes at chunk position c, or its 4 when fewer than 8 remain: the candidate compare and the
// first step of the match extension share one memory request.
__device__ __forceinline__ uint64_t ld_cand(const uint8_t* in, int32_t c, int32_t length) {
    return c + 8 <= length ? ld64(in + c) : (uint64_t)ld32(in + c);
}

// 4 + findMatchingLength(in, candidate + 4, inIndex + 4, length)  (:224-239): the common-prefix
// length bounded by the bytes left, computed 4 bytes per step (the inIndex side from the window).
// `first` = the 4 bytes at a, already read with the candidate compare; b <= length - 4 implies
// a + 4 <= length (a < b), which is when ld_cand read them.
__device__ __forceinline__ int32_t match_len(const uint8_t* in, StreamWin& win, int32_t a, int32_t b, int32_t length,
                                             uint32_t first) {
    int32_t m = 0;
    if (b <= length - 4) {
        const uint32_t x0 = first ^ win.get(b);
        if (x0) return (int32_t)(__builtin_ctz(x0) >> 3);
        m = 4;
        while (b + m <= length - 4) {
            const uint32_t x = ld32(in + a + m) ^ win.get(b + m);
            if (x) return m + (int32_t)(__builtin_ctz(x) >> 3);
            m += 4;
        }
    }
    while (b + m < length && in[a + m] == in[b + m]) ++m;
    return m;
}

template <bool SWAP, class Wr>
__device__ uint32_t encode_chunk(const uint8_t* __restrict__ in, int32_t length, Wr& w, uint32_t* __restrict__ table, uint32_t stamp) {
    for (int i = 0;; i++) {  // preamble (:84-92)
        const uint32_t b = (uint32_t)length >> (i * 7);
        if ((b & 0xFFFFFF80u) != 0) {
            w.put((b & 0x7f) | 0x80);
        } else {
            w.put(b);
            break;
        }
    }
    uint32_t hts = length <= 1 ? 1u : (1u << (32 - __clz((uint32_t)(length - 1))));
    if (hts > 16384u) hts = 16384u;
    const int shift = __clz(hts) + 1;
    const uint32_t stag = stamp << 28;
    const uint32_t word0 = length >= 4 ? ld32(in) : 0u;  // getInt(base + 0): an empty slot's candidate
#define TST(ptr, v) (*(ptr) = (v))
    // read-and-insert of one table slot: a single atomic swap (one memory request instead of a
    // load and a store; same-address order keeps Java's read-then-write semantics).  SWAP = false,
    // load then store, is only instantiated by scripts/experiments/enc_var.cpp (8 % slower).
#define XCH(ptr, v) (SWAP ? __hip_atomic_exchange((ptr), (v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) \
                          : ({ const uint32_t o_ = *(ptr); *(ptr) = (v); o_; }))
#define CHK(wd) (((wd) ^ ((wd) >> 12) ^ ((wd) >> 24)) & 0xFFFu)
#define MK(pos, wd) (stag | (CHK(wd) << 16) | (uint32_t)(pos))
#define LIVE(e) (((e) & 0xF0000000u) == stag)
#define TBL_DEC(e) (LIVE(e) ? (int32_t)((e) & 0xFFFFu) : 0)
    // may getInt(ip) == getInt(candidate)?  false is exact, true needs the candidate bytes
#define MAYBE(e, wd) (LIVE(e) ? ((((e) >> 16) & 0xFFFu) == CHK(wd)) : ((wd) == word0))
    int32_t nextEmit = 0;
    if (length >= 15) {  // MIN_COMPRESSIBLE_BYTES (:34,104)
        StreamWin win;
        win.init(in, length);
        int32_t inIndex = 1;
        uint32_t nextWord = win.get(1);
        uint32_t nextHash = hash_of(nextWord, shift);
        for (;;) {  // outer: (:106)
            int32_t skip = 32;
            int32_t nextIndex = inIndex;
            int32_t candidate;
            uint32_t curWord;
            uint64_t cand8;  // the 8 bytes at candidate (4 near the chunk end), read once per compare
            // ---- probe run (:107-130), in Java's order: each probe's swap waits for the previous
            // compare (a speculative next swap, undone on a match, cost 7 % more time in requests);
            // only the next position's bytes and hash are computed ahead
            uint32_t entry;
            do {
                inIndex = nextIndex;
                const uint32_t hash = nextHash;
                curWord = nextWord;
                nextIndex = inIndex + (skip++ >> 5);
                if (nextIndex > length - 4) goto done;
                nextWord = win.get(nextIndex);
                nextHash = hash_of(nextWord, shift);
                entry = XCH(table + hash, MK(inIndex, curWord));
                candidate = TBL_DEC(entry);
            } while (!(MAYBE(entry, curWord) && curWord == (uint32_t)(cand8 = ld_cand(in, candidate, length))));

            enc_literal(in + nextEmit, w, inIndex - nextEmit);  // (:132)

            int32_t insertTail;
            for (;;) {  // (:135-154)
                const int32_t base = inIndex;
                const int32_t matched = 4 + match_len(in, win, candidate + 4, inIndex + 4, length, (uint32_t)(cand8 >> 32));
                inIndex += matched;
                enc_copy(w, base - candidate, matched);
                insertTail = inIndex - 1;
                nextEmit = inIndex;
                if (inIndex >= length - 4) goto done;
                const uint32_t wTail = win.get(insertTail);
                const uint32_t wCur = win.get(inIndex);
                const uint32_t prevHash = hash_of(wTail, shift);
                TST(table + prevHash, MK(inIndex - 1, wTail));
                const uint32_t currentHash = hash_of(wCur, shift);
                const uint32_t e = XCH(table + currentHash, MK(inIndex, wCur));
                candidate = TBL_DEC(e);
                if (!MAYBE(e, wCur) || wCur != (uint32_t)(cand8 = ld_cand(in, candidate, length))) break;
            }
            nextWord = win.get(insertTail + 2);
            nextHash = hash_of(nextWord, shift);  // (:156)
            ++inIndex;
        }
    }
done:
#undef TBL_DEC
#undef MAYBE
#undef LIVE
#undef MK
#undef CHK
#undef XCH
#undef TST
    if (nextEmit < length) enc_literal(in + nextEmit, w, length - nextEmit);  // (:162-164)
    w.finish();
    return w.pos();
}

// ---------------------------------------------------------------------------------------------
// Wide-entry form (the HBM-table kernels): each table entry carries enough of its position's bytes
// that most probes and most short matches need no read of the candidate's input bytes.
//   entry (64 bits) = stamp[63:58] | next3[57:34] | resid << pbits | position      (resid+position <= 34 bits)
//     resid  = the low `shift` bits of bswap(word) * 0x1e35a7bd: with the slot (= the high bits,
//              Snappy's hash) it determines the 4-byte word exactly, so getInt(ip) == getInt(candidate)
//              is decided from the entry alone (no 12-bit check, no false-positive loads);
//     next3  = the 3 bytes after the word (position + 4 .. + 6): a match of 4-6 bytes (45 % of this
//              corpus's matches) is measured without reading the candidate at all, longer ones read
//              from candidate + 7 on;
//     stamp  = 6 bits, as the narrow form's 4 (a mismatch reads as Java's zero: position 0, whose
//              word and next3 are held in registers).
// The emitted stream is unchanged: the same probes in the same order, the same table semantics.
__device__ __forceinline__ uint32_t bytes_at(const uint8_t* in, int32_t p, int32_t length) {  // up to 4 bytes at p (< length), LE, zero-padded
    if (p + 4 <= length) return ld32(in + p);
    uint32_t v = 0;
    for (int32_t i = 0; p + i < length && i < 4; ++i) v |= (uint32_t)in[p + i] << (8 * i);
    return v;
}

// 4 + findMatchingLength (:224-239) given the candidate's bytes 4..6 (cn3): bytes b.. against a..
// (a = candidate + 4 < b = ip + 4), bounded by length.
__device__ __forceinline__ int32_t match_len_w(const uint8_t* in, StreamWin& win, int32_t a, int32_t b, int32_t length, uint32_t cn3) {
    int32_t m = 0;
    if (b <= length - 4) {
        const uint32_t x0 = (cn3 ^ win.get(b)) & 0xFFFFFFu;
        if (x0) return (int32_t)(__builtin_ctz(x0) >> 3);
        m = 3;
        while (b + m <= length - 4) {
            const uint32_t x = ld32(in + a + m) ^ win.get(b + m);
            if (x) return m + (int32_t)(__builtin_ctz(x) >> 3);
            m += 4;
        }
    }
    while (b + m < length && in[a + m] == in[b + m]) ++m;
    return m;
}

template <class Wr>
__device__ uint32_t encode_chunk_w(const uint8_t* __restrict__ in, int32_t length, Wr& w, uint64_t* __restrict__ table, uint32_t stamp) {
    for (int i = 0;; i++) {  // preamble (:84-92)
        const uint32_t b = (uint32_t)length >> (i * 7);
        if ((b & 0xFFFFFF80u) != 0) {
            w.put((b & 0x7f) | 0x80);
        } else {
            w.put(b);
            break;
        }
    }
    uint32_t hts = length <= 1 ? 1u : (1u << (32 - __clz((uint32_t)(length - 1))));
    if (hts > 16384u) hts = 16384u;
    const int shift = __clz(hts) + 1;
    int32_t nextEmit = 0;
    if (length >= 15) {  // MIN_COMPRESSIBLE_BYTES (:34,104); hts >= 16, shift <= 28
        const uint32_t pbits = hts == 16384u ? 16u : (uint32_t)(32 - shift);  // positions < 2^pbits
        const uint32_t pmask = (1u << pbits) - 1u, rmask = (1u << shift) - 1u;
        const uint64_t stag = (uint64_t)stamp << 58;
        const uint32_t word0 = ld32(in);                            // getInt(base + 0): an empty slot's candidate
        const uint32_t n3_0 = bytes_at(in, 4, length) & 0xFFFFFFu;  // and the 3 bytes after it
#define RES(wd) ((__builtin_bswap32(wd) * 0x1e35a7bdu) & rmask)
#define MKW(pos, wd, n3) (stag | ((uint64_t)(n3) << 34) | ((uint64_t)RES(wd) << pbits) | (uint64_t)(uint32_t)(pos))
#define WLIVE(e) ((uint32_t)((e) >> 58) == stamp)
#define WMATCH(e, wd) (WLIVE(e) ? (((uint32_t)((e) >> pbits) & rmask) == RES(wd)) : ((wd) == word0))
#define WPOS(e) (WLIVE(e) ? (int32_t)((uint32_t)(e) & pmask) : 0)
#define WN3(e) (WLIVE(e) ? ((uint32_t)((e) >> 34) & 0xFFFFFFu) : n3_0)
#define XCH64(ptr, v) __hip_atomic_exchange((ptr), (v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
        StreamWin win;
        win.init(in, length);
        int32_t inIndex = 1;
        uint32_t nextWord = win.get(1);
        uint32_t nextHash = hash_of(nextWord, shift);
        for (;;) {  // outer: (:106)
            int32_t skip = 32;
            int32_t nextIndex = inIndex;
            uint64_t entry;
            uint32_t curWord;
            do {  // probe run (:107-130), in Java's order
                inIndex = nextIndex;
                const uint32_t hash = nextHash;
                curWord = nextWord;
                nextIndex = inIndex + (skip++ >> 5);
                if (nextIndex > length - 4) goto done;
                // the bytes after inIndex first (inIndex + 4 < length; bytes past the end are never
                // compared), then the next probe's word: the window only moves forward
                const uint32_t n3 = win.get(inIndex + 4) & 0xFFFFFFu;
                nextWord = win.get(nextIndex);
                nextHash = hash_of(nextWord, shift);
                entry = XCH64(table + hash, MKW(inIndex, curWord, n3));
            } while (!WMATCH(entry, curWord));
            int32_t candidate = WPOS(entry);
            uint32_t cn3 = WN3(entry);

            enc_literal(in + nextEmit, w, inIndex - nextEmit);  // (:132)

            int32_t insertTail;
            for (;;) {  // (:135-154)
                const int32_t base = inIndex;
                const int32_t matched = 4 + match_len_w(in, win, candidate + 4, inIndex + 4, length, cn3);
                inIndex += matched;
                enc_copy(w, base - candidate, matched);
                insertTail = inIndex - 1;
                nextEmit = inIndex;
                if (inIndex >= length - 4) goto done;
                const uint32_t wTail = win.get(insertTail);
                const uint32_t wCur = win.get(inIndex);
                const uint32_t n3c = win.get(inIndex + 4) & 0xFFFFFFu;
                const uint32_t n3t = ((wCur >> 24) | (n3c << 8)) & 0xFFFFFFu;  // bytes inIndex+3 .. +5
                const uint32_t prevHash = hash_of(wTail, shift);
                __hip_atomic_store(table + prevHash, MKW(inIndex - 1, wTail, n3t), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const uint32_t currentHash = hash_of(wCur, shift);
                const uint64_t e = XCH64(table + currentHash, MKW(inIndex, wCur, n3c));
                if (!WMATCH(e, wCur)) break;
                candidate = WPOS(e);
                cn3 = WN3(e);
            }
            nextWord = win.get(insertTail + 2);
            nextHash = hash_of(nextWord, shift);  // (:156)
            ++inIndex;
        }
#undef XCH64
#undef WN3
#undef WPOS
#undef WMATCH
#undef WLIVE
#undef MKW
#undef RES
    }
done:
    if (nextEmit < length) enc_literal(in + nextEmit, w, length - nextEmit);  // (:162-164)
    w.finish();
    return w.pos();
}

// __launch_bounds__(256, 5): at least 5 blocks of 256 (20 waves, 5 per SIMD) per CU, the residency
// the host launches for, so the kernel stays within 96 VGPRs per lane; with the 16-dword output stage
// (17 KiB of LDS per block) five blocks fit a CU.  Round 6 (profiles/r06/s1, placement-controlled,
// scripts/experiments/enc_curve.cpp): 313.6 ms per 327 680 chunks (0.957 us per chunk) against
// 261.6 ms per 262 144 (0.998) for the round-5 kernel at 4 blocks per CU with a 32-dword stage.
//
// SPREAD = false: lane t encodes chunks t, t + lanes, ... (throughput form, every lane of a wave busy).
// SPREAD = true: one chunk per WAVE, lane 0 only (small batches: lanes of different chunks never share
// a wave's divergent control flow, which otherwise serialises a wave's 64 matchers: 64 chunks in one
// wave take 6x as long as one).  Lane/wave w owns table slot w of the workspace in either form.
constexpr int kStageDw = 16;  // dense form: 64-byte output units staged in LDS (17 KiB per 256 lanes)
template <bool SWAP, bool SPREAD>
__global__ void __launch_bounds__(256, 5) k_snappy_encode(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
                                                       const uint32_t* __restrict__ in_len, uint8_t* __restrict__ out,
                                                       const uint64_t* __restrict__ out_off, uint32_t* __restrict__ out_len,
                                                       int32_t* __restrict__ status, uint32_t n, uint64_t* __restrict__ workspace,
                                                       uint32_t stamp_base) {
    const uint32_t gtid = blockIdx.x * blockDim.x + threadIdx.x;
    if (SPREAD && (gtid & 63u) != 0u) return;
    const uint32_t tid = SPREAD ? gtid >> 6 : gtid;
    const uint32_t nthreads = SPREAD ? (gridDim.x * blockDim.x) >> 6 : gridDim.x * blockDim.x;
    uint64_t* table = workspace + (size_t)tid * 16384u;
    uint32_t* stage = nullptr;
    if constexpr (!SPREAD) {
        __shared__ uint32_t stages[256 * (kStageDw + 1)];  // odd stride: lanes' slots on distinct banks
        stage = &stages[threadIdx.x * (kStageDw + 1)];
    }
    uint32_t iter = 0;
    for (uint32_t c = tid; c < n; c += nthreads, ++iter) {
        const uint32_t len = in_len[c];
        if (len > 65536u) {
            status[c] = NX_ERR_INVALID_ARG;
            out_len[c] = 0;
            continue;
        }
        const uint32_t stamp = stamp_base + iter + 1u;  // 1..63, host re-zeroes the workspace before wrap
        uint8_t* o = out + out_off[c];
        uint32_t olen;
        const uint8_t* src = in + in_off[c];
        if (!SPREAD && (((uintptr_t)o) & 3u) == 0) {
            WriterL<kStageDw> w(stage, o);
            olen = encode_chunk_w(src, (int32_t)len, w, table, stamp);
        } else if ((((uintptr_t)o) & 7u) == 0) {
            WriterT<true> w{reinterpret_cast<uint32_t*>(o), 0, 0, 0, 0};
            olen = encode_chunk_w(src, (int32_t)len, w, table, stamp);
        } else if ((((uintptr_t)o) & 3u) == 0) {
            WriterT<false> w{reinterpret_cast<uint32_t*>(o), 0, 0, 0, 0};
            olen = encode_chunk_w(src, (int32_t)len, w, table, stamp);
        } else {
            ByteWriter w{o, 0};
            olen = encode_chunk_w(src, (int32_t)len, w, table, stamp);
        }
        out_len[c] = olen;
        status[c] = NX_OK;
    }
}

// Latency form for batches of at most one chunk per CU: one workgroup per chunk clears a table in
// LDS and stages the chunk there, then one lane runs the matcher against LDS only (no stamps: the
// table is zeroed, an entry's stamp is 1).  128 KiB of LDS, one chunk per CU; 1.6x faster than the
// SPREAD form for a lone chunk (profiles/r02/notes/small_batches.md).
constexpr uint32_t kLdsTableBytes = 16384u * 4u;
constexpr uint32_t kLdsBytes = kLdsTableBytes + 65536u + 16u;
__global__ void __launch_bounds__(64) k_snappy_encode_lds(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
                                                         const uint32_t* __restrict__ in_len, uint8_t* __restrict__ out,
                                                         const uint64_t* __restrict__ out_off, uint32_t* __restrict__ out_len,
                                                         int32_t* __restrict__ status, uint32_t n) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint32_t* table = reinterpret_cast<uint32_t*>(smem);
    uint8_t* buf = smem + kLdsTableBytes;
    const uint32_t t = threadIdx.x;
    for (uint32_t c = blockIdx.x; c < n; c += gridDim.x) {
        const uint32_t len = in_len[c];
        if (len > 65536u) {
            if (t == 0) {
                status[c] = NX_ERR_INVALID_ARG;
                out_len[c] = 0;
            }
            continue;
        }
        const uint8_t* src = in + in_off[c];
        for (uint32_t i = t; i < 16384u / 4u; i += 64u) reinterpret_cast<uint4*>(table)[i] = make_uint4(0, 0, 0, 0);
        for (uint32_t i = 4u * t; i < len; i += 256u) {
            uint32_t v = 0;
            if (i + 4u <= len) {
                v = ld32(src + i);
            } else {
                for (uint32_t k = 0; i + k < len; ++k) v |= (uint32_t)src[i + k] << (8 * k);
            }
            *reinterpret_cast<uint32_t*>(buf + i) = v;
        }
        __syncthreads();
        if (t == 0) {
            uint8_t* o = out + out_off[c];
            uint32_t olen;
            if ((((uintptr_t)o) & 7u) == 0) {
                WriterT<true> w{reinterpret_cast<uint32_t*>(o), 0, 0, 0, 0};
                olen = encode_chunk<false>(buf, (int32_t)len, w, table, 1u);
            } else if ((((uintptr_t)o) & 3u) == 0) {
                WriterT<false> w{reinterpret_cast<uint32_t*>(o), 0, 0, 0, 0};
                olen = encode_chunk<false>(buf, (int32_t)len, w, table, 1u);
            } else {
                ByteWriter w{o, 0};
                olen = encode_chunk<false>(buf, (int32_t)len, w, table, 1u);
            }
            out_len[c] = olen;
            status[c] = NX_OK;
        }
        __syncthreads();  // the next chunk's staging overwrites the table and buffer
    }
}

}  // namespace enc
}  // namespace nx

namespace {
constexpr unsigned kEncBlock = 256;
constexpr uint32_t kMaxStamp = 63;  // 6-bit stamps 1..63
static_assert(nx::kWsSpec[(int)nx::WsKind::SnappyEnc].entry_bytes == sizeof(uint64_t) &&
                  nx::kWsSpec[(int)nx::WsKind::SnappyEnc].lg == 14 && nx::kWsSpec[(int)nx::WsKind::SnappyEnc].waves_per_cu == 20,
              "Snappy table geometry: 16384 64-bit entries, 20 waves per CU");
}  // namespace

namespace {
constexpr size_t kEncTableBytes = 16384u * sizeof(uint64_t);  // one lane's table (128 KiB)

// Launch sizes of the dense form for n chunks over `slots` resident lanes, one chunk per lane per
// launch (round 6).  A lane's chain runs faster the fewer waves share its SIMD,
// so a launch that does not fill the chip is not proportionally shorter: on 256 CUs the round-5
// kernel took 152 ms for 65 536 chunks and 261.6 for 262 144 (profiles/r06/s1/enc_curve.log), and
// the bench's 6.25 launches of 262 144 per 100 GiB paid ~90 ms for the quarter launch.  The plan
// therefore splits n into k = ceil(n / slots) launches as equal as possible in steps of half a block
// per CU (cus * 128 lanes), the remainder below one step going to the last launch: 1 638 400
// chunks -> 5 x 327 680; 819 200 -> 294 912 + 2 x 262 144; 409 600 -> 196 608 + 212 992.
size_t enc_plan(size_t n, size_t slots, int cus, uint32_t* sizes, size_t cap) {
    auto put = [&](size_t i, size_t v) {
        if (sizes && i < cap) sizes[i] = (uint32_t)v;
    };
    if (n == 0) return 0;
    if (n <= slots) {
        put(0, n);
        return 1;
    }
    const size_t k = (n + slots - 1) / slots;
    const size_t G = (size_t)cus * 128u;
    const size_t s = n / k / G * G;
    const size_t rem = n - k * s, plus = rem / G, last = rem - plus * G;  // plus < k
    if (s > 0 && (plus == 0 || s + G <= slots) && s + last <= slots) {
        for (size_t i = 0; i < k; ++i) put(i, s + (i < plus ? G : 0) + (i + 1 == k ? last : 0));
        return k;
    }
    const size_t e = (n + k - 1) / k;  // a capped workspace: plain equal launches
    for (size_t i = 0; i < k; ++i) put(i, std::min(e, n - i * e));
    return k;
}
}  // namespace

// Place and zero the device's encoder table workspace for batches of up to max_chunks chunks now, so
// a server sets it up at start-up, before its own buffers take the memory the placement choice draws
// candidates from.  Kept until nx_workspaces_trim.  Optional: the standalone batch
// API grows it on demand; batchers and handles hold their own share from creation.
//
// _ex (round 6): max_bytes caps the workspace for good (0: no cap; the tables of
// max_bytes / 128 KiB lanes, whole blocks of 256 above kSpreadMaxChunks lanes): later batches of any
// size run on those lanes (more launches, or one chunk per wave below kSpreadMaxChunks lanes) and the
// standalone calls never grow it past the cap until it is trimmed.  *bytes (nullable) = the
// workspace's bytes, *peak (nullable) = the most bytes its placement held at once
// (nx_workspace_placement_config bounds that).
extern "C" int32_t nx_snappy_encoder_reserve_ex(uint32_t max_chunks, uint64_t max_bytes, void* stream, uint64_t* bytes, uint64_t* peak) {
    int dev = 0, cus = 256;
    NX_HIP_CHECK(hipGetDevice(&dev));
    NX_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    if (bytes) *bytes = 0;
    if (peak) *peak = 0;
    nx::SharedWs& W = nx::shared_ws(nx::WsKind::SnappyEnc, dev);
    uint32_t units = max_chunks;
    if (max_bytes) {  // the cap holds for later batches even when this reservation needs no tables
        size_t lanes = (size_t)(max_bytes / kEncTableBytes);
        if (lanes > nx::kSpreadMaxChunks) lanes = lanes / 256 * 256;
        if (lanes == 0) return NX_ERR_INVALID_ARG;
        std::lock_guard<std::mutex> lk(W.mu);
        if (W.p && W.slots > lanes) return NX_ERR_INVALID_ARG;  // already larger than the cap: trim first
        W.cap = lanes;
        if (units > lanes) units = (uint32_t)lanes;
    }
    if (max_chunks <= (uint32_t)cus) return NX_OK;  // the LDS form needs no workspace
    const int32_t r = nx::ws_hold(nx::WsKind::SnappyEnc, dev, units, (hipStream_t)stream);
    if (r != NX_OK) return r;
    {
        std::lock_guard<std::mutex> lk(W.mu);
        W.kept = true;
        if (bytes) *bytes = (uint64_t)W.slots * kEncTableBytes;
        if (peak) *peak = W.place.peak;
    }
    nx::ws_unhold(nx::WsKind::SnappyEnc, dev);
    return NX_OK;
}

extern "C" int32_t nx_snappy_encoder_reserve(uint32_t max_chunks, void* stream) {
    return nx_snappy_encoder_reserve_ex(max_chunks, 0, stream, nullptr, nullptr);
}

// The plan itself for a given lane count and CU count (host arithmetic only: no device is touched),
// for callers that size their own work and for the CPU tests.  slots = resident lanes of the dense
// form (CUs x 20 x 64 for an uncapped workspace).
extern "C" int32_t nx_snappy_encode_plan_for(uint32_t n, uint32_t slots, int32_t cus, uint32_t* sizes, uint32_t cap, uint32_t* count) {
    if (!count || (cap && !sizes) || slots == 0 || cus <= 0) return NX_ERR_INVALID_ARG;
    *count = (uint32_t)enc_plan(n, slots, cus, sizes, cap);
    return NX_OK;
}

// The launches nx_snappy_encode_batch makes for n chunks on the current device with its present
// workspace (the one a batch of n would grow to when there is none yet): *count launches of
// sizes[0..] chunks (at most `cap` written).  A caller that cuts a large job into encode calls uses
// it so that each call is one full-occupancy launch (bench.py).
extern "C" int32_t nx_snappy_encode_plan(uint32_t n, uint32_t* sizes, uint32_t cap, uint32_t* count) {
    if (!count || (cap && !sizes)) return NX_ERR_INVALID_ARG;
    int dev = 0, cus = 256;
    NX_HIP_CHECK(hipGetDevice(&dev));
    NX_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    *count = 0;
    if (n == 0) return NX_OK;
    if (n <= (uint32_t)cus) {  // the LDS form: one launch
        if (cap) sizes[0] = n;
        *count = 1;
        return NX_OK;
    }
    nx::SharedWs& W = nx::shared_ws(nx::WsKind::SnappyEnc, dev);
    std::lock_guard<std::mutex> lk(W.mu);
    const size_t want = nx::ws_capped(W, nx::ws_want(nx::WsKind::SnappyEnc, n, cus));
    const size_t have = W.p && W.slots >= want ? W.slots : std::max(want, W.p ? W.slots : (size_t)0);
    const nx::LaneGrid g = nx::ws_grid(nx::WsKind::SnappyEnc, n, cus, have);
    if (g.spread) {
        if (cap) sizes[0] = n;
        *count = 1;
        return NX_OK;
    }
    *count = (uint32_t)enc_plan(n, g.slots, cus, sizes, cap);
    return NX_OK;
}

extern "C" int32_t nx_snappy_encode_batch(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len, uint8_t* out,
                                          const uint64_t* out_off, uint32_t* out_len, int32_t* status, uint32_t n, void* stream) {
    NX_CLEAR_STALE_ERROR();
    if (n == 0) return NX_OK;
    if (!in || !in_off || !in_len || !out || !out_off || !out_len || !status) return NX_ERR_INVALID_ARG;
    int dev = 0, cus = 256;
    NX_HIP_CHECK(hipGetDevice(&dev));
    NX_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    const hipStream_t st = (hipStream_t)stream;
    // Batch-size policy (profiles/r02/notes/small_batches.md): a chunk per CU with LDS tables, then a
    // chunk per wave, then the dense lane-per-chunk form once the batch fills the chip.
    if (n <= (uint32_t)cus) {
        static std::once_flag once;
        static hipError_t attr = hipSuccess;
        std::call_once(once, [] {
            attr = hipFuncSetAttribute((const void*)nx::enc::k_snappy_encode_lds, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)nx::enc::kLdsBytes);
        });
        NX_HIP_CHECK(attr);
        hipLaunchKernelGGL(nx::enc::k_snappy_encode_lds, dim3(n), dim3(64), nx::enc::kLdsBytes, st, in, in_off, in_len, out, out_off,
                           out_len, status, n);
        NX_HIP_CHECK(hipGetLastError());
        return NX_OK;
    }
    nx::WsLease lease(nx::WsKind::SnappyEnc, dev, st);
    NX_HIP_CHECK(lease.acquire(nx::ws_want(nx::WsKind::SnappyEnc, n, cus)));
    nx::SharedWs& W = lease.ws();
    const nx::LaneGrid g = nx::ws_grid(nx::WsKind::SnappyEnc, n, cus, W.slots);
    uint64_t* ws = static_cast<uint64_t*>(W.p);
    auto stamps = [&](uint32_t iters) -> hipError_t {  // 6-bit stamps: re-zero the tables before a wrap
        if (W.stamp + iters < kMaxStamp) return hipSuccess;
        W.stamp = 0;
        return hipMemsetAsync(ws, 0, W.slots * kEncTableBytes, st);
    };
    if (g.spread) {  // one chunk per wave; a wave takes at most kMaxStamp - 1 chunks per launch
        const size_t per_launch = g.slots * (kMaxStamp - 1);
        for (size_t base = 0; base < n; base += per_launch) {
            const uint32_t m = (uint32_t)std::min<size_t>(per_launch, n - base);
            const uint32_t iters = (uint32_t)((m + g.slots - 1) / g.slots);
            NX_HIP_CHECK(stamps(iters));
            const size_t waves = std::min<size_t>(g.slots, m);
            hipLaunchKernelGGL((nx::enc::k_snappy_encode<true, true>), dim3((unsigned)waves), dim3(64), 0, st, in, in_off + base,
                               in_len + base, out, out_off + base, out_len + base, status + base, m, ws, W.stamp);
            NX_HIP_CHECK(hipGetLastError());
            W.stamp += iters;
        }
        return NX_OK;
    }
    // the dense form: one chunk per lane per launch, launches planned by enc_plan
    const size_t k = enc_plan(n, g.slots, cus, nullptr, 0);
    std::vector<uint32_t> sizes(k);
    enc_plan(n, g.slots, cus, sizes.data(), k);
    size_t base = 0;
    for (size_t i = 0; i < k; ++i) {
        const uint32_t m = sizes[i];
        NX_HIP_CHECK(stamps(1));
        hipLaunchKernelGGL((nx::enc::k_snappy_encode<true, false>), dim3((m + kEncBlock - 1) / kEncBlock), dim3(kEncBlock), 0, st, in,
                           in_off + base, in_len + base, out, out_off + base, out_len + base, status + base, m, ws, W.stamp);
        NX_HIP_CHECK(hipGetLastError());
        W.stamp += 1;
        base += m;
    }
    return NX_OK;
}

// The probe times (ms) of the candidate placements the last large encoder workspace was chosen from
// and the index kept; *n = 0 when no workspace has been placed yet.  Diagnostics only.
extern "C" int32_t nx_snappy_encode_placement(float* probe_ms, int32_t cap, int32_t* n, int32_t* pick) {
    if (!n || !pick || (cap > 0 && !probe_ms)) return NX_ERR_INVALID_ARG;
    int dev = 0;
    NX_HIP_CHECK(hipGetDevice(&dev));
    nx::SharedWs& W = nx::shared_ws(nx::WsKind::SnappyEnc, dev);
    std::lock_guard<std::mutex> lk(W.mu);
    *n = W.place.n;
    *pick = W.place.pick;
    for (int32_t k = 0; k < W.place.n && k < cap; ++k) probe_ms[k] = W.place.ms[k];
    return NX_OK;
}

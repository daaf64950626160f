// e2e_capi.cpp — end-to-end rate of the Snappy frame handlers through the C-ABI a JNI caller uses
// (include/netty_amd.h section 3): C channels, each with its own SnappyFrameEncoder (jumbo frames) and
// SnappyFrameDecoder (validateChecksums), M messages of S bytes per channel from registered
// (page-locked) host memory, all submitted to one batcher, one flush per direction.  Times include
// the host framing and staging work of every submit, the H2D/D2H traffic and the kernels: host
// memory in, host memory out.  The framed bytes reach the decoders the way a socket delivers them,
// in a registered receive buffer (the copy into it is the network's and is not timed); decode is
// timed twice per round, through nx_snappy_frame_decoder_submit_registered (payloads gathered from
// the mapped pages at flush) and through nx_snappy_frame_decoder_submit (payloads copied at
// submit), each by its own set of decoders.  Prints one JSON object.
// flush_mib > 0 sets the batcher's auto-flush threshold (nx_batcher_set_flush_bytes): batches of that
// many MiB launch while later messages are still being submitted, rotating over the batcher's
// streams, so PCIe traffic and kernels of consecutive batches overlap.
// threads T > 1: T event-loop threads, each with its own batcher (Netty's model: a channel's handlers
// run on its event loop, and the loop's batcher is not shared), channel c on thread c % T; the phase
// times are the wall time of all threads.
// Usage: e2e_capi [C] [M] [S] [rounds] [flush_mib] [dec_flush_mib] [threads]
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <chrono>
#include <functional>
#include <thread>
#include <vector>
#include "../../include/netty_amd.h"
#include "../../include/netty_amd_textgen.h"

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

int main(int argc, char** argv) {
    const int C = argc > 1 ? atoi(argv[1]) : 256, M = argc > 2 ? atoi(argv[2]) : 256, S = argc > 3 ? atoi(argv[3]) : 65535;
    const int R = argc > 4 ? atoi(argv[4]) : 3;
    // auto-flush thresholds per direction (0 = one flush): decoding overlaps the next batch's gather
    // from the mapped receive pages with the previous batch's result writes over PCIe
    const size_t flush_mib = argc > 5 ? (size_t)atol(argv[5]) : 0;
    const size_t dec_flush_mib = argc > 6 ? (size_t)atol(argv[6]) : flush_mib;
    const int T = argc > 7 && atoi(argv[7]) > 0 ? atoi(argv[7]) : 1;
    const size_t N = (size_t)C * M, U = N * (size_t)S;
    uint8_t* in = (uint8_t*)aligned_alloc(4096, (U + 4095) / 4096 * 4096);
    static nx_textgen_tables tg;
    nx_textgen_build(&tg);
    const size_t distinct = N < 1024 ? N : 1024;
    for (size_t i = 0; i < distinct; ++i) nx_tg_chunk(&tg, i, in + i * S, S);
    for (size_t i = distinct; i < N; ++i) memcpy(in + i * S, in + (i % distinct) * S, S);
    if (nx_host_register(in, U) != NX_OK) {
        printf("{\"error\": \"nx_host_register failed\"}\n");
        return 1;
    }
    // one batcher per event-loop thread; the device workspaces and pinned arenas up front, as a server
    // would at start-up: no submit allocates
    std::vector<nx_batcher*> bs(T);
    const uint32_t nbatches = T > 1 ? 4 : 8;
    for (int t = 0; t < T; ++t) {
        nx_batcher* b = bs[t] = nx_batcher_new();
        if (!b || nx_batcher_reserve(b, (1u << NX_WS_SNAPPY_ENC) | (1u << NX_WS_DEC_RECORDS)) != NX_OK ||
            (dec_flush_mib && nx_batcher_reserve_arenas(b, nbatches, (dec_flush_mib + 64) << 20, (4 * dec_flush_mib + 64) << 20) != NX_OK)) {
            printf("{\"error\": \"batcher reservation failed\"}\n");
            return 1;
        }
    }
    std::vector<nx_snappy_frame_encoder*> enc(C);
    std::vector<nx_snappy_frame_decoder*> dec(C), dec2(C);
    for (int c = 0; c < C; ++c) {
        enc[c] = nx_snappy_frame_encoder_new(1);
        dec[c] = nx_snappy_frame_decoder_new(1);
        dec2[c] = nx_snappy_frame_decoder_new(1);
        if (!enc[c] || !dec[c] || !dec2[c]) {
            printf("{\"error\": \"handle creation failed\"}\n");
            return 1;
        }
    }
    // receive buffer: room for every framed message (stream id + jumbo chunk headers), registered once
    const size_t rx_cap = (U + N * 64 + 4095) / 4096 * 4096;
    uint8_t* rx = (uint8_t*)aligned_alloc(4096, rx_cap);
    if (nx_host_register(rx, rx_cap) != NX_OK) {
        printf("{\"error\": \"nx_host_register failed\"}\n");
        return 1;
    }
    std::vector<size_t> rx_off(N), rx_len(N);
    double best_e = 1e30, best_d = 1e30, best_dc = 1e30, comp_total = 0;
    double ph[6] = {0, 0, 0, 0, 0, 0};  // last round: encode submit, encode flush+wait, decode submit, decode flush+wait, copied
    std::vector<char> okt(T, 1);  // per thread: every call succeeded
    std::vector<int64_t> et(N), dt(N);
    // run f(t) on T threads (inline for T = 1) and return the wall time of the slowest submit part and
    // of the whole: each thread submits its channels, then flushes and waits for its last ticket
    auto run = [&](const std::function<void(int, double*)>& f, double* sub_s) {
        std::vector<double> ts(T, 0.0);
        const double t0 = now();
        if (T == 1) {
            f(0, &ts[0]);
        } else {
            std::vector<std::thread> th;
            for (int t = 0; t < T; ++t) th.emplace_back(f, t, &ts[t]);
            for (auto& x : th) x.join();
        }
        double mx = 0;
        for (double x : ts) mx = x > mx ? x : mx;
        *sub_s = mx - t0;
        return now() - t0;
    };
    auto last_ticket = [&](const std::vector<int64_t>& tk, int t) {
        int64_t last = -1;
        for (int c = t; c < C; c += T) last = tk[(size_t)c * M + (M - 1)] > last ? tk[(size_t)c * M + (M - 1)] : last;
        return last;
    };
    auto check_decoded = [&](const std::vector<int64_t>& tk) {
        for (size_t i = 0; i < N; ++i) {
            nx_batcher* b = bs[(i / M) % T];
            const nx_msg* ms;
            size_t nm;
            const char* err;
            const int32_t st = nx_batcher_result(b, tk[i], &ms, &nm, &err);
            size_t tot = 0;
            for (size_t k = 0; k < nm; ++k) tot += ms[k].len;
            if (st != NX_OK || tot != (size_t)S) okt[0] = 0;
            else if (i % 97 == 0) {  // spot-check the bytes
                size_t o = 0;
                for (size_t k = 0; k < nm; ++k) {
                    if (memcmp(ms[k].data, in + i * S + o, ms[k].len) != 0) okt[0] = 0;
                    o += ms[k].len;
                }
            }
            nx_batcher_release(b, tk[i]);
        }
    };
    uint64_t arena_allocs_round0 = 0;
    auto arena_allocs_now = [&] {
        uint64_t tot = 0;
        for (nx_batcher* b : bs) {
            uint64_t a = 0;
            nx_batcher_arena_stats(b, &a, nullptr, nullptr);
            tot += a;
        }
        return tot;
    };
    for (int r = 0; r < R; ++r) {
        if (r == 1) arena_allocs_round0 = arena_allocs_now();
        for (nx_batcher* b : bs) nx_batcher_set_flush_bytes(b, flush_mib << 20);
        double sub;
        const double te = run([&](int t, double* tsub) {
            nx_batcher* b = bs[t];
            for (int m = 0; m < M; ++m)
                for (int c = t; c < C; c += T) {
                    const size_t i = (size_t)c * M + m;
                    et[i] = nx_snappy_frame_encoder_submit(enc[c], b, in + i * S, S, 1);
                    if (et[i] <= 0) okt[t] = 0;
                }
            *tsub = now();
            nx_batcher_flush(b);
            if (nx_batcher_wait(b, last_ticket(et, t)) != NX_OK) okt[t] = 0;
        }, &sub);
        ph[0] = sub;
        ph[1] = te - sub;
        // the framed output of every encode() reaches the receive buffer (network delivery, not timed)
        double comp = 0;
        size_t at = 0;
        for (size_t i = 0; i < N; ++i) {
            nx_batcher* b = bs[(i / M) % T];
            const nx_msg* ms;
            size_t nm;
            const char* err;
            if (nx_batcher_result(b, et[i], &ms, &nm, &err) != NX_OK || nm != 1 || at + ms[0].len > rx_cap) {
                okt[0] = 0;
                rx_off[i] = at;
                rx_len[i] = 0;
                continue;
            }
            memcpy(rx + at, ms[0].data, ms[0].len);
            rx_off[i] = at;
            rx_len[i] = ms[0].len;
            at += (ms[0].len + 15) & ~(size_t)15;
            comp += (double)ms[0].len;
            nx_batcher_release(b, et[i]);
        }
        // decode: registered cumulations (no copy at submit), then copied cumulations (the payloads
        // are copied into the pinned staging at submit), each by its own set of decoders
        for (nx_batcher* b : bs) nx_batcher_set_flush_bytes(b, dec_flush_mib << 20);
        double tdec[2];
        for (int pass = 0; pass < 2; ++pass) {
            const bool reg = pass == 0;
            std::vector<nx_snappy_frame_decoder*>& dd = reg ? dec : dec2;
            tdec[pass] = run([&](int t, double* tsub) {
                nx_batcher* b = bs[t];
                for (int m = 0; m < M; ++m)
                    for (int c = t; c < C; c += T) {
                        const size_t i = (size_t)c * M + m;
                        size_t consumed = 0;
                        dt[i] = reg ? nx_snappy_frame_decoder_submit_registered(dd[c], b, rx + rx_off[i], rx_len[i], &consumed)
                                    : nx_snappy_frame_decoder_submit(dd[c], b, rx + rx_off[i], rx_len[i], &consumed);
                        if (dt[i] <= 0 || consumed != rx_len[i]) okt[t] = 0;
                    }
                *tsub = now();
                nx_batcher_flush(b);
                if (nx_batcher_wait(b, last_ticket(dt, t)) != NX_OK) okt[t] = 0;
            }, &sub);
            ph[2 + 2 * pass] = sub;
            ph[3 + 2 * pass] = tdec[pass] - sub;
            check_decoded(dt);
        }
        if ((r > 0 || R == 1) && tdec[1] < best_dc) best_dc = tdec[1];
        if (r > 0 || R == 1) {
            if (te < best_e) best_e = te;
            if (tdec[0] < best_d) best_d = tdec[0];
        }
        comp_total = comp;
    }
    bool ok = true;
    for (char x : okt) ok = ok && x;
    uint64_t fl = 0, la = 0, ch = 0, arena_bytes = 0, dma_fl = 0;
    for (nx_batcher* b : bs) {
        uint64_t f1 = 0, l1 = 0, c1 = 0, ab = 0, d1 = 0, db = 0;
        nx_batcher_stats(b, &f1, &l1, &c1);
        nx_batcher_arena_stats(b, nullptr, &ab, nullptr);
        nx_batcher_dma_stats(b, &d1, &db);
        fl += f1;
        la += l1;
        ch += c1;
        arena_bytes += ab;
        dma_fl += d1;
    }
    const uint64_t arena_allocs = arena_allocs_now();
    const double g = (double)U / (1 << 30);
    printf("{\"channels\": %d, \"messages_per_channel\": %d, \"message_bytes\": %d, \"threads\": %d, \"uncompressed_bytes\": %zu, "
           "\"compressed_bytes\": %.0f, \"encode_gib_s\": %.3f, \"decode_gib_s\": %.3f, \"round_trip_gib_s\": %.3f, "
           "\"decode_copied_gib_s\": %.3f, \"encode_s\": %.4f, \"decode_s\": %.4f, \"decode_copied_s\": %.4f, "
           "\"phases_s\": {\"encode_submit\": %.4f, \"encode_flush_wait\": %.4f, \"decode_submit\": %.4f, "
           "\"decode_flush_wait\": %.4f, \"decode_copied_submit\": %.4f, \"decode_copied_flush_wait\": %.4f}, "
           "\"flush_mib\": %zu, \"decode_flush_mib\": %zu, \"flushes\": %llu, \"launches\": %llu, "
           "\"dma_flushes\": %llu, \"arena_allocs_after_round0\": %llu, \"pinned_arena_mib\": %.0f, \"verified\": %s}\n",
           C, M, S, T, U, comp_total, g / best_e, g / best_d, g / (best_e + best_d), g / best_dc, best_e, best_d, best_dc, ph[0], ph[1],
           ph[2], ph[3], ph[4], ph[5], flush_mib, dec_flush_mib, (unsigned long long)fl, (unsigned long long)la, (unsigned long long)dma_fl,
           (unsigned long long)(R > 1 ? arena_allocs - arena_allocs_round0 : arena_allocs), arena_bytes / 1048576.0, ok ? "true" : "false");
    for (int c = 0; c < C; ++c) {
        nx_snappy_frame_encoder_free(enc[c]);
        nx_snappy_frame_decoder_free(dec[c]);
        nx_snappy_frame_decoder_free(dec2[c]);
    }
    for (nx_batcher* b : bs) nx_batcher_free(b);
    nx_host_unregister(in);
    nx_host_unregister(rx);
    free(in);
    free(rx);
    return ok ? 0 : 3;
}

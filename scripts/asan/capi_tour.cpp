// capi_tour.cpp — host-side AddressSanitizer driver (scripts/asan/build_asan.sh) for the handler and
// batcher C-ABI beyond what netty_amd/tools/e2e_capi.cpp covers: every codec's synchronous handlers
// (Snappy frames, FastLZ frames at both levels with and without checksums, LZF, LZ4 frames fast and
// high) over text, random and empty messages fed to the decoders in random slices (cumulation), the
// same jobs through one batcher (outputs compared with the synchronous ones), corrupted streams
// (any status, never a memory error), and handles freed while their jobs are in flight.
// Prints one JSON line; exit 0 when every round trip matched.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <functional>
#include <string>
#include <vector>
#include "../../include/netty_amd.h"
#include "../../include/netty_amd_textgen.h"

typedef std::vector<uint8_t> Bytes;
static uint64_t g_rng = 0x9E3779B97F4A7C15ull;
static uint32_t rnd() {
    g_rng ^= g_rng << 13;
    g_rng ^= g_rng >> 7;
    g_rng ^= g_rng << 17;
    return (uint32_t)g_rng;
}
static int g_fail = 0;
static std::string g_list;  // the first failures, '; '-separated
static void fail(const std::string& what) {
    if (g_fail < 24) g_list += (g_fail ? "; " : "") + what;
    ++g_fail;
}

// A codec's synchronous handler pair behind one interface.
struct Codec {
    const char* name;
    bool identity;  // decode(encode(m)) == m; false for FastLZ level 2, whose reference encoder corrupts
                    // messages of more than one chunk (its readU16 quirk): there the
                    // batched paths are compared with the synchronous decode instead
    std::function<void*()> new_enc, new_dec;
    std::function<void(void*)> free_enc, free_dec;
    std::function<bool(void*, const Bytes&, Bytes&)> encode;  // one message -> framed bytes (appended)
    std::function<bool(void*, Bytes&)> finish;                // end of stream (LZ4 close), may append
    std::function<int32_t(void*, const uint8_t*, size_t, size_t*, const nx_msg**, size_t*, const char**)> decode;
    std::function<int64_t(void*, nx_batcher*, const Bytes&)> submit_enc;
    std::function<int64_t(void*, nx_batcher*, const uint8_t*, size_t, size_t*)> submit_dec;
};

static Bytes make_msg(const nx_textgen_tables* tg, int kind, size_t n, uint64_t idx) {
    Bytes m(n);
    if (kind == 0 && n) {
        Bytes t(65536);
        for (size_t o = 0; o < n; o += 65536) {
            nx_tg_chunk(tg, idx * 97 + o / 65536, t.data(), 65536);
            memcpy(m.data() + o, t.data(), n - o < 65536 ? n - o : 65536);
        }
    } else {
        for (size_t i = 0; i < n; ++i) m[i] = (uint8_t)rnd();
    }
    return m;
}

// Feed `stream` to a fresh decoder in random slices, as a channel's reads arrive; returns the status
// of the last call and appends the decoded messages to out.
static int32_t feed(const Codec& c, void* d, const Bytes& stream, Bytes& out) {
    Bytes cum;
    size_t pos = 0;
    int32_t st = NX_OK;
    while (pos < stream.size() || !cum.empty()) {
        const size_t take = pos < stream.size() ? 1 + rnd() % (stream.size() - pos < 70000 ? stream.size() - pos : 70000) : 0;
        cum.insert(cum.end(), stream.begin() + pos, stream.begin() + pos + take);
        pos += take;
        size_t consumed = 0, nm = 0;
        const nx_msg* msgs = nullptr;
        const char* err = nullptr;
        st = c.decode(d, cum.data(), cum.size(), &consumed, &msgs, &nm, &err);
        for (size_t i = 0; i < nm; ++i) out.insert(out.end(), msgs[i].data, msgs[i].data + msgs[i].len);
        if (st != NX_OK) return st;
        if (consumed > cum.size()) {
            fail(std::string(c.name) + ": consumed past the cumulation");
            return -1;
        }
        cum.erase(cum.begin(), cum.begin() + consumed);
        if (take == 0 && consumed == 0) break;  // the rest is an incomplete frame
    }
    return st;
}

int main(int argc, char** argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 2;
    static nx_textgen_tables tg;
    nx_textgen_build(&tg);
    std::vector<Codec> codecs;
    codecs.push_back({"snappy_frame", true, [] { return (void*)nx_snappy_frame_encoder_new(0); },
                      [] { return (void*)nx_snappy_frame_decoder_new(1); },
                      [](void* e) { nx_snappy_frame_encoder_free((nx_snappy_frame_encoder*)e); },
                      [](void* d) { nx_snappy_frame_decoder_free((nx_snappy_frame_decoder*)d); },
                      [](void* e, const Bytes& m, Bytes& o) {
                          Bytes t(nx_snappy_frame_max_encoded_length(m.size()) + 64);
                          const int64_t r = nx_snappy_frame_encoder_encode((nx_snappy_frame_encoder*)e, m.data(), m.size(), t.data(), t.size());
                          if (r < 0) return false;
                          o.insert(o.end(), t.begin(), t.begin() + r);
                          return true;
                      },
                      [](void*, Bytes&) { return true; },
                      [](void* d, const uint8_t* in, size_t n, size_t* c, const nx_msg** m, size_t* k, const char** e) {
                          return nx_snappy_frame_decoder_decode((nx_snappy_frame_decoder*)d, in, n, c, m, k, e);
                      },
                      [](void* e, nx_batcher* b, const Bytes& m) {
                          return nx_snappy_frame_encoder_submit((nx_snappy_frame_encoder*)e, b, m.data(), m.size(), 0);
                      },
                      [](void* d, nx_batcher* b, const uint8_t* in, size_t n, size_t* c) {
                          return nx_snappy_frame_decoder_submit((nx_snappy_frame_decoder*)d, b, in, n, c);
                      }});
    for (int level = 1; level <= 2; ++level)
        for (int ck = 0; ck <= 1; ++ck) {
            static char names[4][24];
            char* nm = names[(level - 1) * 2 + ck];
            snprintf(nm, 24, "fastlz_l%d_ck%d", level, ck);
            codecs.push_back({nm, level == 1, [level, ck] { return (void*)nx_fastlz_frame_encoder_new(level, ck); },
                              [ck] { return (void*)nx_fastlz_frame_decoder_new(ck); },
                              [](void* e) { nx_fastlz_frame_encoder_free((nx_fastlz_frame_encoder*)e); },
                              [](void* d) { nx_fastlz_frame_decoder_free((nx_fastlz_frame_decoder*)d); },
                              [](void* e, const Bytes& m, Bytes& o) {
                                  Bytes t(nx_fastlz_frame_max_encoded_length(m.size()) + 64);
                                  const int64_t r = nx_fastlz_frame_encoder_encode((nx_fastlz_frame_encoder*)e, m.data(), 0, m.size(), t.data(), t.size());
                                  if (r < 0) return false;
                                  o.insert(o.end(), t.begin(), t.begin() + r);
                                  return true;
                              },
                              [](void*, Bytes&) { return true; },
                              [](void* d, const uint8_t* in, size_t n, size_t* c, const nx_msg** m, size_t* k, const char** e) {
                                  return nx_fastlz_frame_decoder_decode((nx_fastlz_frame_decoder*)d, in, n, c, m, k, e);
                              },
                              [](void* e, nx_batcher* b, const Bytes& m) {
                                  return nx_fastlz_frame_encoder_submit((nx_fastlz_frame_encoder*)e, b, m.data(), 0, m.size());
                              },
                              [](void* d, nx_batcher* b, const uint8_t* in, size_t n, size_t* c) {
                                  return nx_fastlz_frame_decoder_submit((nx_fastlz_frame_decoder*)d, b, in, n, c);
                              }});
        }
    codecs.push_back({"lzf", true, [] { return (void*)nx_lzf_encoder_new(16); }, [] { return (void*)nx_lzf_decoder_new(); },
                      [](void* e) { nx_lzf_encoder_free((nx_lzf_encoder*)e); },
                      [](void* d) { nx_lzf_decoder_free((nx_lzf_decoder*)d); },
                      [](void* e, const Bytes& m, Bytes& o) {
                          Bytes t(nx_lzf_frame_max_encoded_length(m.size()) + 64);
                          const int64_t r = nx_lzf_encoder_encode((nx_lzf_encoder*)e, m.data(), m.size(), t.data(), t.size());
                          if (r < 0) return false;
                          o.insert(o.end(), t.begin(), t.begin() + r);
                          return true;
                      },
                      [](void*, Bytes&) { return true; },
                      [](void* d, const uint8_t* in, size_t n, size_t* c, const nx_msg** m, size_t* k, const char** e) {
                          return nx_lzf_decoder_decode((nx_lzf_decoder*)d, in, n, c, m, k, e);
                      },
                      [](void* e, nx_batcher* b, const Bytes& m) { return nx_lzf_encoder_submit((nx_lzf_encoder*)e, b, m.data(), m.size()); },
                      [](void* d, nx_batcher* b, const uint8_t* in, size_t n, size_t* c) {
                          return nx_lzf_decoder_submit((nx_lzf_decoder*)d, b, in, n, c);
                      }});
    for (int high = 0; high <= 1; ++high)
        codecs.push_back({high ? "lz4_frame_high" : "lz4_frame", true,
                          [high] { return (void*)nx_lz4_frame_encoder_new_ex(65536, high, 0x7FFFFFFF); },
                          [] { return (void*)nx_lz4_frame_decoder_new(1); },
                          [](void* e) { nx_lz4_frame_encoder_free((nx_lz4_frame_encoder*)e); },
                          [](void* d) { nx_lz4_frame_decoder_free((nx_lz4_frame_decoder*)d); },
                          [](void* e, const Bytes& m, Bytes& o) {
                              Bytes t(nx_lz4_frame_max_encoded_length(m.size() + 65536, 65536) + 64);
                              int64_t r = nx_lz4_frame_encoder_encode((nx_lz4_frame_encoder*)e, m.data(), m.size(), t.data(), t.size());
                              if (r < 0) return false;
                              o.insert(o.end(), t.begin(), t.begin() + r);
                              r = nx_lz4_frame_encoder_flush((nx_lz4_frame_encoder*)e, t.data(), t.size());
                              if (r < 0) return false;
                              o.insert(o.end(), t.begin(), t.begin() + r);
                              return true;
                          },
                          [](void* e, Bytes& o) {
                              Bytes t(1024);
                              const int64_t r = nx_lz4_frame_encoder_close((nx_lz4_frame_encoder*)e, t.data(), t.size());
                              if (r < 0) return false;
                              o.insert(o.end(), t.begin(), t.begin() + r);
                              return true;
                          },
                          [](void* d, const uint8_t* in, size_t n, size_t* c, const nx_msg** m, size_t* k, const char** e) {
                              return nx_lz4_frame_decoder_decode((nx_lz4_frame_decoder*)d, in, n, c, m, k, e);
                          },
                          [](void* e, nx_batcher* b, const Bytes& m) {
                              return nx_lz4_frame_encoder_submit((nx_lz4_frame_encoder*)e, b, m.data(), m.size(), 1);
                          },
                          [](void* d, nx_batcher* b, const uint8_t* in, size_t n, size_t* c) {
                              return nx_lz4_frame_decoder_submit((nx_lz4_frame_decoder*)d, b, in, n, c);
                          }});

    const size_t sizes[] = {0, 1, 17, 100, 4096, 65535, 65536, 65537, 200000};
    size_t round_trips = 0, batch_jobs = 0, corrupt_runs = 0;
    for (int r = 0; r < rounds; ++r) {
        nx_batcher* b = nx_batcher_new();
        if (!b) {
            fail("nx_batcher_new");
            break;
        }
        for (const Codec& c : codecs) {
            // messages of every size and kind
            std::vector<Bytes> msgs;
            for (size_t s : sizes)
                for (int kind = 0; kind < 2; ++kind) msgs.push_back(make_msg(&tg, kind, s, r * 1000 + msgs.size()));
            // synchronous encode, then decode in slices
            void* e = c.new_enc();
            Bytes stream, want;
            for (const Bytes& m : msgs) {
                if (!c.encode(e, m, stream)) fail(std::string(c.name) + ": encode");
                want.insert(want.end(), m.begin(), m.end());
            }
            if (!c.finish(e, stream)) fail(std::string(c.name) + ": finish");
            c.free_enc(e);
            void* d = c.new_dec();
            Bytes got;
            const int32_t st = feed(c, d, stream, got);
            c.free_dec(d);
            if (c.identity && (st != NX_OK || got != want)) {
                size_t k = 0;
                while (k < got.size() && k < want.size() && got[k] == want[k]) ++k;
                fail(std::string(c.name) + ": sync round trip (status " + std::to_string(st) + ", " + std::to_string(got.size()) + " of " +
                     std::to_string(want.size()) + " bytes, first difference at " + std::to_string(k) + ")");
            }
            // the reference's own output and status are the expectation (with checksums, the corrupted
            // level-2 block fails validation: FastLzFrameDecoder.java:178-184)
            const int32_t want_st = c.identity ? NX_OK : st;
            if (!c.identity) want = got;
            ++round_trips;
            // the same messages as batcher jobs: each message's framed bytes must equal the synchronous ones
            void* eb = c.new_enc();
            void* es = c.new_enc();
            std::vector<int64_t> tickets;
            std::vector<Bytes> sync_out;
            for (const Bytes& m : msgs) {
                Bytes one;
                if (!c.encode(es, m, one)) fail(std::string(c.name) + ": encode (reference)");
                sync_out.push_back(one);
                tickets.push_back(c.submit_enc(eb, b, m));
            }
            c.free_enc(eb);  // freed with jobs in flight (allowed: each job holds a reference)
            c.free_enc(es);
            if (nx_batcher_flush(b) != NX_OK) fail(std::string(c.name) + ": flush");
            for (size_t i = 0; i < tickets.size(); ++i) {
                if (tickets[i] <= 0) {
                    fail(std::string(c.name) + ": submit encode");
                    continue;
                }
                if (nx_batcher_wait(b, tickets[i]) != NX_OK) fail(std::string(c.name) + ": wait");
                const nx_msg* ms = nullptr;
                size_t nm = 0;
                const char* err = nullptr;
                const int32_t rs = nx_batcher_result(b, tickets[i], &ms, &nm, &err);
                Bytes one;
                for (size_t k = 0; k < nm; ++k) one.insert(one.end(), ms[k].data, ms[k].data + ms[k].len);
                if (rs != NX_OK || one != sync_out[i]) fail(std::string(c.name) + ": batched encode differs");
                nx_batcher_release(b, tickets[i]);
                ++batch_jobs;
            }
            // the synchronous stream decoded as batcher jobs over a cumulation, decoder freed mid-flight
            void* db = c.new_dec();
            Bytes cum(stream.begin(), stream.end());
            std::vector<int64_t> dt;
            size_t pos = 0;
            while (pos < cum.size()) {
                const size_t n = 1 + rnd() % (cum.size() - pos < 150000 ? cum.size() - pos : 150000);
                size_t consumed = 0;
                const int64_t t = c.submit_dec(db, b, cum.data() + pos, n, &consumed);
                if (t <= 0) {
                    fail(std::string(c.name) + ": submit decode");
                    break;
                }
                dt.push_back(t);
                pos += consumed;
                if (consumed == 0 && pos + n >= cum.size()) break;
            }
            c.free_dec(db);
            if (nx_batcher_flush(b) != NX_OK) fail(std::string(c.name) + ": flush (decode)");
            Bytes gotb;
            int32_t seen_st = NX_OK;
            for (int64_t t : dt) {
                nx_batcher_wait(b, t);
                const nx_msg* ms = nullptr;
                size_t nm = 0;
                const char* err = nullptr;
                const int32_t rs = nx_batcher_result(b, t, &ms, &nm, &err);
                for (size_t k = 0; k < nm; ++k) gotb.insert(gotb.end(), ms[k].data, ms[k].data + ms[k].len);
                if (rs != NX_OK && rs != want_st) fail(std::string(c.name) + ": batched decode status " + std::to_string(rs));
                if (rs != NX_OK) seen_st = rs;
                nx_batcher_release(b, t);
                ++batch_jobs;
            }
            if (gotb != want || seen_st != want_st) fail(std::string(c.name) + ": batched decode differs");
            // corrupted streams: a flipped byte, a truncation; any status, never a memory error
            for (int k = 0; k < 6 && !stream.empty(); ++k) {
                Bytes bad = stream;
                if (k < 4) {
                    bad[rnd() % bad.size()] ^= (uint8_t)(1u << (rnd() % 8));
                } else {
                    bad.resize(rnd() % bad.size());
                }
                void* dc = c.new_dec();
                Bytes junk;
                (void)feed(c, dc, bad, junk);
                c.free_dec(dc);
                size_t consumed = 0;
                void* dj = c.new_dec();
                const int64_t t = c.submit_dec(dj, b, bad.data(), bad.size(), &consumed);
                c.free_dec(dj);
                if (t > 0) {
                    nx_batcher_wait(b, t);
                    const nx_msg* ms = nullptr;
                    size_t nm = 0;
                    const char* err = nullptr;
                    (void)nx_batcher_result(b, t, &ms, &nm, &err);
                    nx_batcher_release(b, t);
                }
                ++corrupt_runs;
            }
        }
        nx_batcher_free(b);
    }
    // Round 6 entry points: the LZ4 frame encoder after close (IllegalStateException for a message whose
    // blocks need fewer than blockSize bytes, pass-through for a larger one, sync and batcher), the
    // host-side launch plan, the placement bound and a byte-capped Snappy reservation.
    size_t r6_checks = 0;
    {
        nx_batcher* b = nx_batcher_new();
        for (int path = 0; path < 2 && b; ++path) {
            nx_lz4_frame_encoder* e = nx_lz4_frame_encoder_new_ex(4096, 0, 0x7FFFFFFF);
            Bytes t(nx_lz4_frame_max_encoded_length(8192, 4096) + 64);
            if (nx_lz4_frame_encoder_close(e, t.data(), t.size()) < 0) fail("r6: lz4 close");
            const Bytes small = make_msg(&tg, 0, 100, 7), big = make_msg(&tg, 1, 5000, 8);
            int64_t rs, rb;
            if (path == 0) {
                rs = nx_lz4_frame_encoder_encode(e, small.data(), small.size(), t.data(), t.size());
                rb = nx_lz4_frame_encoder_encode(e, big.data(), big.size(), t.data(), t.size());
                if (rb != (int64_t)big.size() || memcmp(t.data(), big.data(), big.size()) != 0) fail("r6: lz4 pass-through after close");
            } else {
                rs = nx_lz4_frame_encoder_submit(e, b, small.data(), small.size(), 0);
                rb = nx_lz4_frame_encoder_submit(e, b, big.data(), big.size(), 0);
                if (rb <= 0) fail("r6: lz4 pass-through job after close");
                else {
                    nx_batcher_flush(b);
                    nx_batcher_wait(b, rb);
                    const nx_msg* ms = nullptr;
                    size_t nm = 0;
                    const char* err = nullptr;
                    if (nx_batcher_result(b, rb, &ms, &nm, &err) != NX_OK || nm != 1 || ms[0].len != big.size() ||
                        memcmp(ms[0].data, big.data(), big.size()) != 0)
                        fail("r6: lz4 pass-through job bytes");
                    nx_batcher_release(b, rb);
                }
            }
            const char* msg = nx_lz4_frame_encoder_error(e);
            if (rs != NX_ERR_LZ4_ENCODE_FINISHED || !msg || strcmp(msg, "encode finished and not enough space to write remaining data") != 0)
                fail("r6: lz4 encode after close");
            nx_lz4_frame_encoder_free(e);
            ++r6_checks;
        }
        if (b) nx_batcher_free(b);
        uint32_t sizes[8] = {0}, cnt = 0;
        if (nx_snappy_encode_plan_for(1638400, 327680, 256, sizes, 8, &cnt) != NX_OK || cnt != 5 || sizes[4] != 327680) fail("r6: plan");
        if (nx_snappy_encode_plan_for(819200, 327680, 256, sizes, 2, &cnt) != NX_OK || cnt != 3) fail("r6: plan (cap)");
        if (nx_workspace_placement_config(0, 0) != NX_OK) fail("r6: placement config");
        if (nx_workspaces_trim() != NX_OK) fail("r6: trim");
        uint64_t bytes = 0, peak = 0;
        if (nx_snappy_encoder_reserve_ex(40000, 20480ull * 131072ull + 5, nullptr, &bytes, &peak) != NX_OK || bytes != 20480ull * 131072ull ||
            peak < bytes)
            fail("r6: capped reserve");
        if (nx_snappy_encoder_reserve_ex(40000, 1000ull * 131072ull, nullptr, nullptr, nullptr) == NX_OK) fail("r6: cap below a live workspace");
        r6_checks += 3;
    }
    const int32_t trim = nx_workspaces_trim();
    if (trim != NX_OK) fail("nx_workspaces_trim");
    printf("{\"codecs\": %zu, \"rounds\": %d, \"round_trips\": %zu, \"batch_jobs\": %zu, \"corrupt_runs\": %zu, \"round6_checks\": %zu, "
           "\"failures\": %d, \"failure_list\": \"%s\", \"verified\": %s}\n",
           codecs.size(), rounds, round_trips, batch_jobs, corrupt_runs, r6_checks, g_fail, g_list.c_str(), g_fail ? "false" : "true");
    fflush(stdout);
    return g_fail ? 1 : 0;
}

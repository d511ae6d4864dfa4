// host_sanitize.cpp — drives the host C++ cores under AddressSanitizer + UndefinedBehaviorSanitizer
// (SURVEY.md §5.2 "race detection / sanitizers": GPU ASan is not available on the MI355X pool, so the sanitizers run
// on the host code).  Built and run by tests/test_host_sanitizers.py via chronos.native.build_sanitize_harness().
//
// Deterministic pseudo-random inputs, biased toward the edges the reference's Python never checked: 255/256/300-byte
// paths, empty fields, invalid UTF-8, every filter prefix/suffix, chains past the caps, malformed automata.  Every
// check is an invariant, so a sanitizer report or a failed CHECK is the only way this program exits non-zero.
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include <vector>

#include "../constrain/token_dfa_core.h"
#include "../sensor_host/sensor_core.h"

#define CHECK(c)                                                                    \
    do {                                                                            \
        if (!(c)) {                                                                 \
            std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
            std::exit(2);                                                           \
        }                                                                           \
    } while (0)

using namespace chronos;

static std::mt19937_64 rng(20261016);

static std::string rand_bytes(size_t n, bool ascii) {
    std::string s(n, '\0');
    for (auto& c : s) c = ascii ? (char)(' ' + rng() % 95) : (char)(rng() % 256);
    return s;
}

static std::string rand_path() {
    static const char* heads[] = {"/lib/", "/usr/lib/", "/usr/share/", "/etc/ssl/", "/etc/fonts/", "/etc/host",
                                  "/dev/", "/proc/", "/tmp/", "/home/u/", "", "/"};
    static const char* tails[] = {".so", ".cache", ".mo", ".conf", ".crt", ".curlrc", ".bin", "", ".so.6", "x"};
    std::string s = heads[rng() % 12];
    const size_t body = rng() % 4 == 0 ? 240 + rng() % 80 : rng() % 40;  // around the 256-byte field
    s += rand_bytes(body, rng() % 8 != 0);
    s += tails[rng() % 10];
    return s;
}

static void test_filters_and_codec() {
    for (int i = 0; i < 20000; ++i) {
        const std::string p = rand_path();
        const bool a = open_is_noise(p, false), b = open_is_noise(p, true);
        CHECK(!a || b || true);  // both evaluate without touching memory past the field (ASan is the check)
        std::string field = p;
        field.resize(CHRONOS_PATH_LEN, '\0');
        (void)chronos_path_len(field.c_str());
        const uint32_t pid = (uint32_t)rng();
        const std::string comm = rand_bytes(rng() % 24, rng() % 2), type = rng() % 2 ? "OPEN" : "EXEC";
        const std::string rec = encode(pid, comm, p, type);
        CHECK(rec.size() == kRecordSize);
        const Event e = decode(reinterpret_cast<const uint8_t*>(rec.data()));
        CHECK(e.pid == pid && e.type == type);
        CHECK(e.comm.size() <= CHRONOS_COMM_LEN - 1 && e.argv.size() <= CHRONOS_PATH_LEN - 1);
        CHECK(comm.compare(0, e.comm.size(), e.comm) == 0);
        (void)valid_utf8(e.comm);
        (void)valid_utf8(rand_bytes(rng() % 16, false));
    }
}

static void test_tracker() {
    const std::vector<std::string> ignore = {"node", "code", "ollama", "python", "chrome", "vmtools", "git"};
    const std::vector<std::string> trig = {"curl", "chmod", "bash", "nc", "cat"};
    for (int cfg = 0; cfg < 4; ++cfg) {
        ChainTracker t(ignore, trig, 2, cfg & 1, cfg & 2 ? 8 : 0, cfg & 2 ? 64 : 0);
        std::string buf;
        for (int i = 0; i < 5000; ++i) {
            static const char* comms[] = {"bash", "curl", "python3", "attack_chain.sh", "sshd", "cat", "rsync"};
            const std::string comm = rng() % 10 ? comms[rng() % 7] : rand_bytes(rng() % 20, false);
            buf += encode((uint32_t)(rng() % 300), comm, rand_path(), rng() % 3 ? "OPEN" : "EXEC");
        }
        const auto fired = t.feed_records(buf, cfg & 1, cfg & 2);
        for (const auto& f : fired) {
            CHECK(f.history.size() >= 2);
            if (cfg & 2) CHECK(f.history.size() <= 8);
        }
        const auto st = t.stats();
        CHECK(st.fired == fired.size());
        CHECK(st.seen + st.dropped_kernel == buf.size() / kRecordSize);
        if (cfg & 2) CHECK(t.num_pids() <= 64);
        for (uint32_t pid = 0; pid < 300; pid += 7) {
            (void)t.chain(pid);
            t.evict(pid);
            CHECK(t.chain(pid).empty());
        }
        bool threw = false;
        try {
            t.feed_records(std::string(kRecordSize + 1, 'x'), false, false);
        } catch (const std::invalid_argument&) {
            threw = true;
        }
        CHECK(threw);
    }
}

static void test_token_dfa() {
    int compiled = 0;
    for (int round = 0; round < 6; ++round) {
        const int64_t S = 4 + rng() % 40;
        std::vector<int32_t> T(S * 256, -1);
        for (int64_t s = 0; s < S; ++s)
            for (int c = 0; c < 256; ++c)
                if (rng() % 4 == 0) T[s * 256 + c] = (int32_t)(rng() % S);
        std::vector<bool> accept(S);
        for (int64_t s = 0; s < S; ++s) accept[s] = rng() % 5 == 0;
        accept[round == 0 ? 0 : rng() % S] = true;  // round 0: the start state accepts, so it always compiles
        const int64_t V = 500 + rng() % 3000;
        std::vector<std::string> toks(V);
        for (auto& t : toks) t = rand_bytes(rng() % 9, false);
        const std::vector<int32_t> eos = {(int32_t)(V - 1), (int32_t)V + 5, -3};  // out-of-range ids are ignored
        std::vector<int16_t> nx((S + 1) * V), dist(S + 1);
        std::vector<int64_t> live;
        try {
            compile_token_dfa_core(T.data(), S, accept, toks, eos, 0, nx.data(), dist.data(), live);
        } catch (const std::runtime_error&) {
            continue;  // start cannot reach an accepting state: a valid refusal
        }
        ++compiled;
        CHECK(dist[S] == 0 && dist[0] < 32767 && (int64_t)live.size() == S + 1);
        for (int64_t s = 0; s <= S; ++s)
            for (int64_t v = 0; v < V; ++v) {
                const int16_t t = nx[s * V + v];
                CHECK(t >= -1 && t <= S);
                if (t >= 0) CHECK(dist[t] < 32767);
                if (t >= 0 && t < S && s < S && !toks[v].empty()) CHECK(walk_core(T.data(), (int32_t)s, toks[v]) == t);
            }
    }
    CHECK(compiled >= 1);
    std::vector<int32_t> bad(2 * 256, 7);  // transition target >= S
    std::vector<int16_t> nx(3 * 4), dist(3);
    std::vector<int64_t> live;
    bool threw = false;
    try {
        compile_token_dfa_core(bad.data(), 2, {true, false}, {"a", "b", "c", "d"}, {3}, 0, nx.data(), dist.data(), live);
    } catch (const std::invalid_argument&) {
        threw = true;
    }
    CHECK(threw);
}

int main() {
    test_filters_and_codec();
    test_tracker();
    test_token_dfa();
    std::printf("host_sanitize ok\n");
    return 0;
}

// token_dfa_core.h — the pybind-free core of the token-automaton compiler (token_dfa.cpp binds it to Python;
// csrc/tests/host_sanitize.cpp drives it under AddressSanitizer / UndefinedBehaviorSanitizer).
//
//   next[s][v] = state reached from byte-DFA state s by feeding token v's bytes, or -1 if any byte is illegal
//   next[accept][eos] = DONE (= S), dist[s] = fewest tokens from s to DONE (BFS on the reversed token graph)
#pragma once
#include <algorithm>
#include <cstdint>
#include <deque>
#include <stdexcept>
#include <string>
#include <unordered_set>
#include <utility>
#include <vector>

namespace chronos {

struct Trie {
    // children stored as a sorted edge list per node (vocab tries are sparse below depth 2)
    struct Node {
        std::vector<std::pair<uint8_t, int32_t>> kids;
        std::vector<int32_t> tokens;  // token ids whose byte string ends here
    };
    std::vector<Node> nodes{1};

    void insert(const std::string& s, int32_t id) {
        int32_t cur = 0;
        for (unsigned char c : s) {
            auto& k = nodes[cur].kids;
            auto it = std::lower_bound(k.begin(), k.end(), std::make_pair(c, (int32_t)-1),
                                       [](const auto& a, const auto& b) { return a.first < b.first; });
            if (it != k.end() && it->first == c) {
                cur = it->second;
            } else {
                const int32_t n = (int32_t)nodes.size();
                k.insert(it, {c, n});
                nodes.emplace_back();
                cur = n;
            }
        }
        nodes[cur].tokens.push_back(id);
    }
};

// T: [S, 256] byte-DFA transitions (-1 = illegal); nx: [S+1, V] out, dist: [S+1] out, live: [S+1] out.
// Throws std::invalid_argument / std::runtime_error on malformed input or an unreachable accepting state.
inline void compile_token_dfa_core(const int32_t* T, int64_t S, const std::vector<bool>& accept,
                                   const std::vector<std::string>& toks, const std::vector<int32_t>& eos_ids,
                                   int32_t start, int16_t* nx, int16_t* dist, std::vector<int64_t>& live_tokens) {
    if ((int64_t)accept.size() != S) throw std::invalid_argument("accept must have S entries");
    if (S + 1 > 32767) throw std::invalid_argument("too many states for an int16 table");
    if (start < 0 || start >= S) throw std::invalid_argument("start state out of range");
    const int64_t V = (int64_t)toks.size();
    const int32_t DONE = (int32_t)S;
    for (int64_t i = 0; i < S * 256; ++i)
        if (T[i] < -1 || T[i] >= S) throw std::invalid_argument("transition target out of range");
    Trie trie;
    for (int64_t v = 0; v < V; ++v)
        if (!toks[v].empty()) trie.insert(toks[v], (int32_t)v);
    live_tokens.assign(S + 1, 0);
    std::fill(nx, nx + (S + 1) * V, (int16_t)-1);
    // DFS over the trie from every state.
    std::vector<std::pair<int32_t, int32_t>> stack;  // (trie node, dfa state)
    for (int64_t s = 0; s < S; ++s) {
        int16_t* row = nx + s * V;
        stack.clear();
        stack.push_back({0, (int32_t)s});
        while (!stack.empty()) {
            auto [node, st] = stack.back();
            stack.pop_back();
            const auto& nd = trie.nodes[node];
            if (node != 0)
                for (int32_t id : nd.tokens) row[id] = (int16_t)st;
            for (const auto& [c, child] : nd.kids) {
                const int32_t ns = T[(int64_t)st * 256 + c];
                if (ns >= 0) stack.push_back({child, ns});
            }
        }
        if (accept[s])
            for (int32_t e : eos_ids)
                if (e >= 0 && e < V) row[e] = (int16_t)DONE;
    }
    // reverse edges (deduplicated) and BFS from DONE
    std::vector<std::unordered_set<int32_t>> rev(S + 1);
    for (int64_t s = 0; s < S; ++s) {
        const int16_t* row = nx + s * V;
        for (int64_t v = 0; v < V; ++v)
            if (row[v] >= 0) {
                rev[row[v]].insert((int32_t)s);
                ++live_tokens[s];
            }
    }
    std::fill(dist, dist + S + 1, (int16_t)32767);
    std::deque<int32_t> q;
    dist[DONE] = 0;
    q.push_back(DONE);
    while (!q.empty()) {
        const int32_t u = q.front();
        q.pop_front();
        for (int32_t p : rev[u])
            if (dist[p] == 32767) {
                dist[p] = (int16_t)(dist[u] + 1);
                q.push_back(p);
            }
    }
    // Tokens leading into a dead state (one that can never reach DONE) are removed, so the sampler can never
    // walk into a trap even with an unlimited budget.
    for (int64_t s = 0; s < S; ++s) {
        int16_t* row = nx + s * V;
        for (int64_t v = 0; v < V; ++v)
            if (row[v] >= 0 && dist[row[v]] == 32767) row[v] = -1;
    }
    if (dist[start] == 32767) throw std::runtime_error("grammar start state cannot reach an accepting state");
}

// Walk one byte string through a byte DFA (host-side validation of generated text).
inline int32_t walk_core(const int32_t* T, int32_t state, const std::string& data) {
    for (unsigned char c : data) {
        if (state < 0) return -1;
        state = T[(int64_t)state * 256 + c];
    }
    return state;
}

}  // namespace chronos

// token_dfa.cpp — host compiler from a byte-level DFA (JSON / verdict-schema grammar) to a token-level automaton
// over the model vocabulary (pybind11 module `_constrain_native`).
//
// Reference behaviour being replaced: Ollama's `format: "json"` (chronos_sensor.py:118) forces syntactically valid
// JSON through llama.cpp's grammar sampler, which walks the grammar per candidate token on the CPU at every step
// (SURVEY.md §2.1 X6).  Here the walk is done ONCE at start-up:
//
//   next[s][v] = state reached from byte-DFA state s by feeding token v's bytes, or -1 if any byte is illegal
//   next[accept][eos] = DONE, dist[s] = fewest tokens from s to DONE (BFS on the reversed token graph)
//
// and the result is uploaded to the GPU, where sampler.hip applies it inside the captured decode graph.  Token
// strings are walked over a byte trie of the vocabulary, so a state only explores token prefixes its grammar allows.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <cstdint>
#include <deque>
#include <stdexcept>
#include <string>
#include <unordered_set>
#include <vector>

namespace py = pybind11;

namespace {

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

py::tuple compile_token_dfa(py::array_t<int32_t, py::array::c_style | py::array::forcecast> trans,
                            std::vector<bool> accept, std::vector<py::bytes> tokens, std::vector<int32_t> eos_ids,
                            int32_t start) {
    if (trans.ndim() != 2 || trans.shape(1) != 256) throw std::invalid_argument("trans must be [S, 256] int32");
    const int64_t S = trans.shape(0);
    if ((int64_t)accept.size() != S) throw std::invalid_argument("accept must have S entries");
    if (S + 1 > 32767) throw std::invalid_argument("too many states for an int16 table");
    const int64_t V = (int64_t)tokens.size();
    const int32_t* T = trans.data();
    const int32_t DONE = (int32_t)S;

    Trie trie;
    {
        std::vector<std::string> toks(V);
        for (int64_t v = 0; v < V; ++v) toks[v] = std::string(tokens[v]);
        py::gil_scoped_release nogil;
        for (int64_t v = 0; v < V; ++v)
            if (!toks[v].empty()) trie.insert(toks[v], (int32_t)v);
    }

    py::array_t<int16_t> next_arr({S + 1, V});
    py::array_t<int16_t> dist_arr({S + 1});
    int16_t* nx = next_arr.mutable_data();
    int16_t* dist = dist_arr.mutable_data();
    std::vector<int64_t> live_tokens(S + 1, 0);
    {
        py::gil_scoped_release nogil;
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
    }
    if (dist[start] == 32767) throw std::runtime_error("grammar start state cannot reach an accepting state");
    return py::make_tuple(next_arr, dist_arr, py::cast(live_tokens));
}

// Walk one byte string through a byte DFA (tests / host-side validation of generated text).
int32_t walk(py::array_t<int32_t, py::array::c_style | py::array::forcecast> trans, int32_t state, py::bytes data) {
    const int32_t* T = trans.data();
    for (unsigned char c : std::string(data)) {
        if (state < 0) return -1;
        state = T[(int64_t)state * 256 + c];
    }
    return state;
}

}  // namespace

PYBIND11_MODULE(_constrain_native, m) {
    m.doc() = "CHRONOS token-level grammar automaton compiler (JSON / verdict schema -> device tables)";
    m.def("compile_token_dfa", &compile_token_dfa, py::arg("trans"), py::arg("accept"), py::arg("tokens"),
          py::arg("eos_ids"), py::arg("start") = 0,
          "Returns (next[S+1, V] int16, dist[S+1] int16, live_tokens[S+1]); state S is DONE.");
    m.def("walk", &walk);
}

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

#include "token_dfa_core.h"

namespace py = pybind11;

namespace {

py::tuple compile_token_dfa(py::array_t<int32_t, py::array::c_style | py::array::forcecast> trans,
                            std::vector<bool> accept, std::vector<py::bytes> tokens, std::vector<int32_t> eos_ids,
                            int32_t start) {
    if (trans.ndim() != 2 || trans.shape(1) != 256) throw std::invalid_argument("trans must be [S, 256] int32");
    const int64_t S = trans.shape(0), V = (int64_t)tokens.size();
    if (S + 1 > 32767) throw std::invalid_argument("too many states for an int16 table");
    std::vector<std::string> toks(V);
    for (int64_t v = 0; v < V; ++v) toks[v] = std::string(tokens[v]);
    py::array_t<int16_t> next_arr({S + 1, V});
    py::array_t<int16_t> dist_arr({S + 1});
    std::vector<int64_t> live_tokens;
    int16_t* nx = next_arr.mutable_data();
    int16_t* dist = dist_arr.mutable_data();
    const int32_t* T = trans.data();
    {
        py::gil_scoped_release nogil;
        chronos::compile_token_dfa_core(T, S, accept, toks, eos_ids, start, nx, dist, live_tokens);
    }
    return py::make_tuple(next_arr, dist_arr, py::cast(live_tokens));
}

int32_t walk(py::array_t<int32_t, py::array::c_style | py::array::forcecast> trans, int32_t state, py::bytes data) {
    return chronos::walk_core(trans.data(), state, std::string(data));
}

}  // namespace

PYBIND11_MODULE(_constrain_native, m) {
    m.doc() = "CHRONOS token-level grammar automaton compiler (JSON / verdict schema -> device tables)";
    m.def("compile_token_dfa", &compile_token_dfa, py::arg("trans"), py::arg("accept"), py::arg("tokens"),
          py::arg("eos_ids"), py::arg("start") = 0,
          "Returns (next[S+1, V] int16, dist[S+1] int16, live_tokens[S+1]); state S is DONE.");
    m.def("walk", &walk);
}

// sensor_host.cpp — native host half of the CHRONOS sensor (pybind11 module `_sensor_native`).
//
// What lives here (the reference's native component is the eBPF C; its host equivalent is C++):
//   * the in-kernel noise policy, compiled from the SAME header as the BPF program (chronos_filters.h),
//     for replaying raw/unfiltered traces and for table-driven tests;
//   * the 288-byte data_t codec (reference chronos_sensor.py:18-23; BCC's ctypes mirror at :125);
//   * a batched chain tracker with the reference's user-space semantics (chronos_sensor.py:124-157):
//       strict UTF-8 decode (drop on error, :127-131) -> comm ignore list (substring, :133-135)
//       -> "[TYPE] comm -> argv" (:137) -> append to per-TGID chain (:138)
//       -> trigger keyword (substring, :141) && len >= 2 (:142) -> emit chain, reset (:157)
//     plus opt-in fixes for SURVEY.md §2.8 Q4 (bounded chains / PID cap) and Q5 (word-boundary triggers).
// The Python tracker in sensor/chain.py is the readable oracle; tests check both agree event for event.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "sensor_core.h"

namespace py = pybind11;

PYBIND11_MODULE(_sensor_native, m) {
    using namespace chronos;
    m.doc() = "CHRONOS sensor host library: shared eBPF filter policy, data_t codec, batched chain tracker";
    m.attr("RECORD_SIZE") = kRecordSize;
    m.def("open_is_noise", &open_is_noise, py::arg("path"), py::arg("strict") = false);
    m.def("has_prefix", [](const std::string& s, const std::string& p) {
        std::string a = s; a.resize(CHRONOS_PATH_LEN, '\0');
        std::string b = p; b.resize(CHRONOS_PREFIX_SCAN + 1, '\0');
        return chronos_has_prefix(a.c_str(), b.c_str()) != 0;
    });
    m.def("has_suffix", [](const std::string& s, const std::string& p) {
        std::string a = s; a.resize(CHRONOS_PATH_LEN, '\0');
        std::string b = p; b.resize(CHRONOS_SUFFIX_SCAN + 1, '\0');
        return chronos_has_suffix(a.c_str(), chronos_path_len(a.c_str()), b.c_str()) != 0;
    });
    m.def("encode_record", [](uint32_t pid, const std::string& comm, const std::string& argv, const std::string& type) {
        return py::bytes(encode(pid, comm, argv, type));
    });
    m.def("decode_records", [](const std::string& buf) {
        if (buf.size() % kRecordSize != 0) throw std::invalid_argument("buffer is not a multiple of 288 bytes");
        py::list out;
        const auto* base = reinterpret_cast<const uint8_t*>(buf.data());
        for (size_t off = 0; off < buf.size(); off += kRecordSize) {
            Event e = decode(base + off);
            out.append(py::make_tuple(e.pid, py::bytes(e.comm), py::bytes(e.argv), py::bytes(e.type)));
        }
        return out;
    });
    m.def("valid_utf8", [](const std::string& s) { return valid_utf8(s); });
    py::class_<ChainTracker>(m, "ChainTracker")
        .def(py::init<std::vector<std::string>, std::vector<std::string>, size_t, bool, size_t, size_t>(),
             py::arg("ignore"), py::arg("triggers"), py::arg("min_len") = 2, py::arg("word_triggers") = false,
             py::arg("max_chain") = 0, py::arg("max_pids") = 0)
        .def("feed_event", [](ChainTracker& t, uint32_t pid, py::bytes comm, py::bytes argv, py::bytes type) -> py::object {
            Event e{pid, std::string(comm), std::string(argv), std::string(type)};
            Trigger tr;
            if (t.feed(e, &tr)) return py::make_tuple(tr.pid, tr.history);
            return py::none();
        })
        .def("feed_records", [](ChainTracker& t, py::bytes buf, bool kernel_filter, bool strict) {
            std::vector<Trigger> fired;
            std::string b(buf);
            {
                py::gil_scoped_release nogil;
                fired = t.feed_records(b, kernel_filter, strict);
            }
            py::list out;
            for (auto& f : fired) out.append(py::make_tuple(f.pid, f.history));
            return out;
        }, py::arg("buf"), py::arg("kernel_filter") = false, py::arg("strict") = false)
        .def("evict", &ChainTracker::evict)
        .def("chain", &ChainTracker::chain)
        .def("num_pids", &ChainTracker::num_pids)
        .def("stats", [](const ChainTracker& t) {
            const auto s = t.stats();
            py::dict d;
            d["seen"] = s.seen; d["dropped_kernel"] = s.dropped_kernel; d["dropped_decode"] = s.dropped_decode;
            d["dropped_ignored"] = s.dropped_ignored; d["fired"] = s.fired; d["evicted"] = s.evicted;
            d["pids"] = s.pids;
            return d;
        });
}

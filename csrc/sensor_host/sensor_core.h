// sensor_core.h — the pybind-free core of the CHRONOS sensor host library (sensor_host.cpp binds it to Python;
// csrc/tests/host_sanitize.cpp drives it under AddressSanitizer / UndefinedBehaviorSanitizer).
//
//   * the in-kernel noise policy, compiled from the SAME header as the BPF program (chronos_filters.h);
//   * the 288-byte data_t codec (reference chronos_sensor.py:18-23; BCC's ctypes mirror at :125);
//   * the chain tracker with the reference's user-space semantics (chronos_sensor.py:124-157) plus the opt-in
//     SURVEY.md §2.8 Q4 (bounded chains / PID cap) and Q5 (word-boundary triggers) fixes.
#pragma once
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <deque>
#include <iterator>
#include <list>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../project-chronos-distributed-behavioral-edr-ebpf-llm-_amd/sensor/bpf/chronos_filters.h"

namespace chronos {

constexpr size_t kRecordSize = 288;
constexpr size_t kOffPid = 0, kOffComm = 4, kOffArgv = 20, kOffType = 276;
static_assert(kOffType + CHRONOS_TYPE_LEN + 2 == kRecordSize, "data_t layout");

// C-string view of a fixed char array: bytes up to the first NUL (what ctypes c_char arrays return).
inline std::string cfield(const uint8_t* p, size_t cap) {
    size_t n = 0;
    while (n < cap && p[n] != 0) ++n;
    return std::string(reinterpret_cast<const char*>(p), n);
}

// Strict UTF-8 validation with Python's rules (no overlongs, no surrogates, <= U+10FFFF).
inline bool valid_utf8(const std::string& s) {
    const auto* p = reinterpret_cast<const unsigned char*>(s.data());
    size_t i = 0, n = s.size();
    while (i < n) {
        unsigned c = p[i];
        if (c < 0x80) { ++i; continue; }
        size_t len; unsigned cp;
        if ((c & 0xE0) == 0xC0) { len = 2; cp = c & 0x1F; }
        else if ((c & 0xF0) == 0xE0) { len = 3; cp = c & 0x0F; }
        else if ((c & 0xF8) == 0xF0) { len = 4; cp = c & 0x07; }
        else return false;
        if (i + len > n) return false;
        for (size_t k = 1; k < len; ++k) {
            if ((p[i + k] & 0xC0) != 0x80) return false;
            cp = (cp << 6) | (p[i + k] & 0x3F);
        }
        if ((len == 2 && cp < 0x80) || (len == 3 && cp < 0x800) || (len == 4 && cp < 0x10000)) return false;
        if (cp > 0x10FFFF || (cp >= 0xD800 && cp <= 0xDFFF)) return false;
        i += len;
    }
    return true;
}

inline bool is_word(char c) {
    return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9') || c == '_';
}

// Substring match (reference) or whole-word match (fix for Q5: `nc` no longer fires on `rsync`).
inline bool contains(const std::string& hay, const std::string& needle, bool word) {
    if (needle.empty()) return true;
    size_t pos = hay.find(needle);
    if (!word) return pos != std::string::npos;
    while (pos != std::string::npos) {
        bool left = pos == 0 || !is_word(hay[pos - 1]);
        size_t end = pos + needle.size();
        bool right = end >= hay.size() || !is_word(hay[end]);
        if (left && right) return true;
        pos = hay.find(needle, pos + 1);
    }
    return false;
}

struct Event {
    uint32_t pid;
    std::string comm, argv, type;
};

inline Event decode(const uint8_t* r) {
    Event e;
    std::memcpy(&e.pid, r + kOffPid, 4);
    e.comm = cfield(r + kOffComm, CHRONOS_COMM_LEN);
    e.argv = cfield(r + kOffArgv, CHRONOS_PATH_LEN);
    e.type = cfield(r + kOffType, CHRONOS_TYPE_LEN);
    return e;
}

inline std::string encode(uint32_t pid, const std::string& comm, const std::string& argv, const std::string& type) {
    std::string out(kRecordSize, '\0');
    std::memcpy(&out[kOffPid], &pid, 4);
    // Same truncation the kernel applies: comm keeps 15 chars + NUL, argv 255 + NUL, type 9 + NUL.
    std::memcpy(&out[kOffComm], comm.data(), std::min(comm.size(), size_t(CHRONOS_COMM_LEN - 1)));
    std::memcpy(&out[kOffArgv], argv.data(), std::min(argv.size(), size_t(CHRONOS_PATH_LEN - 1)));
    std::memcpy(&out[kOffType], type.data(), std::min(type.size(), size_t(CHRONOS_TYPE_LEN - 1)));
    return out;
}

inline bool open_is_noise(const std::string& path, bool strict) {
    char buf[CHRONOS_PATH_LEN + 1] = {0};
    std::memcpy(buf, path.data(), std::min(path.size(), size_t(CHRONOS_PATH_LEN - 1)));
    return strict ? chronos_open_is_noise_strict(buf) : chronos_open_is_noise(buf);
}

struct Trigger {
    uint32_t pid;
    std::vector<std::string> history;
};

class ChainTracker {
  public:
    ChainTracker(std::vector<std::string> ignore, std::vector<std::string> triggers, size_t min_len,
                 bool word_triggers, size_t max_chain, size_t max_pids)
        : ignore_(std::move(ignore)), triggers_(std::move(triggers)), min_len_(min_len),
          word_(word_triggers), max_chain_(max_chain), max_pids_(max_pids) {}

    // Feed one decoded event; returns true and fills `out` when the chain fires.
    bool feed(const Event& e, Trigger* out) {
        ++seen_;
        if (!valid_utf8(e.comm) || !valid_utf8(e.argv) || !valid_utf8(e.type)) { ++drop_decode_; return false; }
        for (const auto& x : ignore_)
            if (contains(e.comm, x, false)) { ++drop_ignored_; return false; }
        std::string s;
        s.reserve(e.type.size() + e.comm.size() + e.argv.size() + 6);
        s += '['; s += e.type; s += "] "; s += e.comm; s += " -> "; s += e.argv;
        auto& chain = touch(e.pid);
        chain.push_back(s);
        if (max_chain_ && chain.size() > max_chain_) chain.pop_front();
        bool hit = false;
        for (const auto& t : triggers_)
            if (contains(s, t, word_)) { hit = true; break; }
        if (hit && chain.size() >= min_len_) {
            ++fired_;
            out->pid = e.pid;
            out->history.assign(chain.begin(), chain.end());
            chain.clear();
            return true;
        }
        return false;
    }

    // Batched feed of raw data_t records.  `kernel_filter` re-applies the in-kernel OPEN policy (replay of
    // unfiltered traces); live BPF records were already filtered.
    std::vector<Trigger> feed_records(const std::string& buf, bool kernel_filter, bool strict) {
        if (buf.size() % kRecordSize != 0) throw std::invalid_argument("buffer is not a multiple of 288 bytes");
        std::vector<Trigger> fired;
        const auto* base = reinterpret_cast<const uint8_t*>(buf.data());
        for (size_t off = 0; off < buf.size(); off += kRecordSize) {
            Event e = decode(base + off);
            if (kernel_filter && e.type == "OPEN") {
                char path[CHRONOS_PATH_LEN + 1] = {0};
                std::memcpy(path, base + off + kOffArgv, CHRONOS_PATH_LEN);
                path[CHRONOS_PATH_LEN - 1] = 0;
                if (strict ? chronos_open_is_noise_strict(path) : chronos_open_is_noise(path)) { ++drop_kernel_; continue; }
            }
            Trigger t;
            if (feed(e, &t)) fired.push_back(std::move(t));
        }
        return fired;
    }

    void evict(uint32_t pid) {
        auto it = chains_.find(pid);
        if (it == chains_.end()) return;
        lru_.erase(it->second.lru);
        chains_.erase(it);
    }
    std::vector<std::string> chain(uint32_t pid) const {
        auto it = chains_.find(pid);
        if (it == chains_.end()) return {};
        return {it->second.events.begin(), it->second.events.end()};
    }
    size_t num_pids() const { return chains_.size(); }
    struct Stats {
        uint64_t seen, dropped_kernel, dropped_decode, dropped_ignored, fired, evicted, pids;
    };
    Stats stats() const {
        return {seen_, drop_kernel_, drop_decode_, drop_ignored_, fired_, evicted_, (uint64_t)chains_.size()};
    }

  private:
    struct Slot {
        std::deque<std::string> events;
        std::list<uint32_t>::iterator lru;
    };
    std::deque<std::string>& touch(uint32_t pid) {
        auto it = chains_.find(pid);
        if (it != chains_.end()) {
            lru_.splice(lru_.end(), lru_, it->second.lru);
            return it->second.events;
        }
        if (max_pids_ && chains_.size() >= max_pids_) {  // Q4 fix: bounded memory, evict least-recently-seen
            uint32_t victim = lru_.front();
            lru_.pop_front();
            chains_.erase(victim);
            ++evicted_;
        }
        lru_.push_back(pid);
        Slot s;
        s.lru = std::prev(lru_.end());
        return chains_.emplace(pid, std::move(s)).first->second.events;
    }

    std::vector<std::string> ignore_, triggers_;
    size_t min_len_;
    bool word_;
    size_t max_chain_, max_pids_;
    std::unordered_map<uint32_t, Slot> chains_;
    std::list<uint32_t> lru_;
    uint64_t seen_ = 0, drop_kernel_ = 0, drop_decode_ = 0, drop_ignored_ = 0, fired_ = 0, evicted_ = 0;
};

}  // namespace chronos

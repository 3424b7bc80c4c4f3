// dccl_amd/csrc/bootstrap.cpp — see bootstrap.hpp.
#include "bootstrap.hpp"

#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <map>
#include <mutex>
#include <sstream>
#include <thread>

namespace dccl_amd {
namespace {

constexpr const char* kMagic = "DCCLRDV2";

// A publisher's stamp: pid, that process's start time, and the generation (how many times this process
// has published to the path).  A reader remembers the last stamp it consumed per (path, reader), so a
// second group formed under the same tag by the same live rank 0 is never joined with the previous id.
struct Stamp {
    long pid = 0;
    unsigned long long start = 0, gen = 0;
    bool operator==(const Stamp& o) const { return pid == o.pid && start == o.start && gen == o.gen; }
};
std::mutex g_mu;
std::map<std::string, unsigned long long> g_published;  // path -> generations published by this process
std::map<std::string, Stamp> g_consumed;                 // path#reader -> last stamp consumed

}  // namespace

unsigned long long proc_start_time(long pid) {
    std::ifstream f("/proc/" + std::to_string(pid) + "/stat");
    std::string line;
    if (!std::getline(f, line)) return 0;
    const size_t rp = line.rfind(')');  // the command name may contain spaces and parentheses
    if (rp == std::string::npos) return 0;
    std::istringstream rest(line.substr(rp + 1));
    std::string tok;
    for (int field = 3; field <= 22; ++field) {  // fields after ')' start at 3 (state)
        if (!(rest >> tok)) return 0;
        if (field == 3 && (tok == "Z" || tok == "X" || tok == "x")) return 0;  // exited, not yet reaped: gone
        if (field == 22) return std::strtoull(tok.c_str(), nullptr, 10);
    }
    return 0;
}

namespace {

std::string to_hex(const std::string& s) {
    static const char* d = "0123456789abcdef";
    std::string h;
    h.reserve(2 * s.size());
    for (unsigned char c : s) {
        h.push_back(d[c >> 4]);
        h.push_back(d[c & 15]);
    }
    return h;
}

bool from_hex(const std::string& h, std::string* out) {
    if (h.size() % 2) return false;
    out->clear();
    for (size_t i = 0; i < h.size(); i += 2) {
        char* end = nullptr;
        const std::string byte = h.substr(i, 2);
        const long v = std::strtol(byte.c_str(), &end, 16);
        if (end != byte.c_str() + 2) return false;
        out->push_back(static_cast<char>(v));
    }
    return true;
}

// The payload and stamp of a file published by a live process for `world` ranks, or false.
bool try_read(const std::string& path, uint32_t world, std::string* payload, Stamp* st) {
    std::ifstream f(path);
    std::string magic, hex;
    uint32_t w = 0;
    if (!(f >> magic >> st->pid >> st->start >> st->gen >> w >> hex) || magic != kMagic) return false;
    if (w != world || st->pid <= 0 || st->start == 0 || proc_start_time(st->pid) != st->start) return false;  // stale
    return from_hex(hex, payload);
}

}  // namespace

std::string rdv_path(const char* prefix) {
    const char* dir = std::getenv("DCCL_BOOTSTRAP_DIR");
    const char* tag = std::getenv("DCCL_BOOTSTRAP_TAG");
    if (!tag) tag = std::getenv("MASTER_PORT");
    return std::string(dir ? dir : "/tmp") + "/" + prefix + (tag ? tag : "default");
}

double rdv_timeout_s() {
    const char* t = std::getenv("DCCL_BOOTSTRAP_TIMEOUT_S");
    const double v = t ? std::strtod(t, nullptr) : 120.0;
    return v > 0 ? v : 120.0;
}

dccl::ncclResult_t rdv_publish(const std::string& path, uint32_t world, const std::string& payload) {
    const long pid = static_cast<long>(::getpid());
    const unsigned long long start = proc_start_time(pid);
    if (start == 0) return dccl::ncclSystemError;
    unsigned long long gen = 0;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        gen = ++g_published[path];
    }
    const std::string tmp = path + ".tmp." + std::to_string(pid);
    {
        std::ofstream f(tmp, std::ios::trunc);
        f << kMagic << ' ' << pid << ' ' << start << ' ' << gen << ' ' << world << ' ' << to_hex(payload) << '\n';
        if (!f) return dccl::ncclSystemError;
    }
    if (std::rename(tmp.c_str(), path.c_str()) != 0) {
        std::remove(tmp.c_str());
        return dccl::ncclSystemError;
    }
    return dccl::ncclSuccess;
}

namespace {

std::string took_marker(const std::string& path, const Stamp& st, uint32_t reader) {
    return path + ".took." + std::to_string(st.pid) + "." + std::to_string(st.start) + "." + std::to_string(st.gen) +
           "." + std::to_string(reader);
}

// Reader `reader` took publication `st`: leave a marker, and the reader that completes the set (every rank
// but the publisher, rank 0) removes the publication and the markers.  A process that starts afterwards finds
// no file and waits for the next publication, so it can never join a group that already formed, whether or
// not rank 0 ever calls dccl_bootstrap_done.
void mark_taken(const std::string& path, const Stamp& st, uint32_t world, uint32_t reader) {
    { std::ofstream(took_marker(path, st, reader)) << '\n'; }
    for (uint32_t r = 1; r < world; ++r)
        if (!std::ifstream(took_marker(path, st, r)).good()) return;
    std::string payload;
    Stamp now;
    if (try_read(path, world, &payload, &now) && now == st) std::remove(path.c_str());
    for (uint32_t r = 1; r < world; ++r) std::remove(took_marker(path, st, r).c_str());
}

}  // namespace

dccl::ncclResult_t rdv_read(const std::string& path, uint32_t world, uint32_t reader, double timeout_s,
                            std::string* payload) {
    const auto deadline = std::chrono::steady_clock::now() + std::chrono::duration<double>(timeout_s);
    const std::string key = path + "#" + std::to_string(reader);
    for (;;) {
        Stamp st;
        if (try_read(path, world, payload, &st)) {
            bool fresh = false;
            {
                std::lock_guard<std::mutex> lk(g_mu);
                auto it = g_consumed.find(key);
                fresh = it == g_consumed.end() || !(it->second == st);  // not the publication this reader took
                if (fresh) g_consumed[key] = st;
            }
            if (fresh) {
                mark_taken(path, st, world, reader);
                return dccl::ncclSuccess;
            }
        }
        if (std::chrono::steady_clock::now() >= deadline) return dccl::ncclSystemError;
        std::this_thread::sleep_for(std::chrono::milliseconds(10));
    }
}

void rdv_remove(const std::string& path) { std::remove(path.c_str()); }

}  // namespace dccl_amd

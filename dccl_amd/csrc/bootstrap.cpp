// dccl_amd/csrc/bootstrap.cpp — see bootstrap.hpp.
#include "bootstrap.hpp"

#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <sstream>
#include <thread>

namespace dccl_amd {
namespace {

constexpr const char* kMagic = "DCCLRDV1";

// Start time of process `pid` in clock ticks since boot (/proc/<pid>/stat field 22), 0 if it is gone.
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
        if (field == 22) return std::strtoull(tok.c_str(), nullptr, 10);
    }
    return 0;
}

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

// The payload of a file published by a live process for `world` ranks, or false.
bool try_read(const std::string& path, uint32_t world, std::string* payload) {
    std::ifstream f(path);
    std::string magic, hex;
    long pid = 0;
    unsigned long long start = 0;
    uint32_t w = 0;
    if (!(f >> magic >> pid >> start >> w >> hex) || magic != kMagic) return false;
    if (w != world || pid <= 0 || start == 0 || proc_start_time(pid) != start) return false;  // stale
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
    const std::string tmp = path + ".tmp." + std::to_string(pid);
    {
        std::ofstream f(tmp, std::ios::trunc);
        f << kMagic << ' ' << pid << ' ' << start << ' ' << world << ' ' << to_hex(payload) << '\n';
        if (!f) return dccl::ncclSystemError;
    }
    if (std::rename(tmp.c_str(), path.c_str()) != 0) {
        std::remove(tmp.c_str());
        return dccl::ncclSystemError;
    }
    return dccl::ncclSuccess;
}

dccl::ncclResult_t rdv_read(const std::string& path, uint32_t world, double timeout_s, std::string* payload) {
    const auto deadline = std::chrono::steady_clock::now() + std::chrono::duration<double>(timeout_s);
    for (;;) {
        if (try_read(path, world, payload)) return dccl::ncclSuccess;
        if (std::chrono::steady_clock::now() >= deadline) return dccl::ncclSystemError;
        std::this_thread::sleep_for(std::chrono::milliseconds(10));
    }
}

void rdv_remove(const std::string& path) { std::remove(path.c_str()); }

}  // namespace dccl_amd

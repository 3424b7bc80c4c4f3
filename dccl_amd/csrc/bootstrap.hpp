// dccl_amd/csrc/bootstrap.hpp — single-node rendezvous files for the cross-process transports.
//
// The reference forms its group through Derecho's membership service (ncclCommInit,
// /root/reference/src/core/dccl.cpp:287-332).  One node of MI355X GPUs needs much less: rank 0
// publishes a small payload (the RCCL unique id, or the name of the IPC shared-memory segment) in a
// file of DCCL_BOOTSTRAP_DIR (default /tmp) named by DCCL_BOOTSTRAP_TAG or MASTER_PORT, and the other
// ranks poll for it.
//
// A file left behind by an earlier job with the same tag (a crash between publish and clean-up) must
// never be taken: a rank that joined with a stale RCCL id would block in ncclCommInitRank until RCCL
// gives up.  The publisher therefore stamps the file with its pid, that process's start time (field
// 22 of /proc/<pid>/stat) and the world size; a reader accepts a file only while that very process is
// alive and the world size matches.  Writes are atomic (temporary file + rename).
// The same live rank 0 may form a second group under the same tag: the stamp also carries a generation
// (the publisher's count of publications to that path), and a reader never takes the publication it
// already consumed (per path and reader rank), so it waits for the republished id instead of joining a
// finished bootstrap.
#pragma once

#include <cstdint>
#include <string>

#include "dccl/dccl.hpp"

namespace dccl_amd {

// <dir>/<prefix><tag>
std::string rdv_path(const char* prefix);
// Poll limit of rdv_read: DCCL_BOOTSTRAP_TIMEOUT_S, default 120 s.
double rdv_timeout_s();
dccl::ncclResult_t rdv_publish(const std::string& path, uint32_t world, const std::string& payload);
// Waits up to timeout_s for a file published by a live process for `world` ranks that `reader` (a rank) has
// not consumed before; ncclSystemError on timeout.
dccl::ncclResult_t rdv_read(const std::string& path, uint32_t world, uint32_t reader, double timeout_s,
                            std::string* payload);
void rdv_remove(const std::string& path);
// Start time of process `pid` in clock ticks since boot (/proc/<pid>/stat field 22), 0 if it is gone (a
// zombie that exited but was not reaped yet counts as gone): (pid, start time) names one process, also
// after the pid is reused.
unsigned long long proc_start_time(long pid);

}  // namespace dccl_amd
